"""ORACLE (test infrastructure only) — the alternating solver in the reference formulation.

Re-enacts qmc/qmc.ipynb cell 1, loop :559-634 (C-step :562-579, S-step :622-634) with S as
the free Adam variable (backup/notebooks/onebit_lowrank.ipynb:1230-1236): reference-style
get_tensor (slice-assignment loop + autograd), prob_probit, the masked -sum(Wx log P),
lambda_c ||C||_F + lambda_s ||S||_F, torch.optim.Adam and C[C<0] = 0.  This is also the CPU
baseline bench.py times ("port"): the same op sequence, hence the same O(R K^2 I J) autograd
cost as the reference.
"""
import time

import torch

from . import reference_ops as ro


def free_s_solve(S0, C0, Y, Wx, b, sigma, offset=0.0, log_model=False, n_iter=10,
                 lambda_c=100.0, lambda_s=100.0, lr_c=5e-3, lr_s=1e-2, snapshots=(), timer=None,
                 loss="probit", project_s=False):
    """loss="squared": the Euclidean criterion of qmc/qmc_dowjons.ipynb :138-162 in place of
    the probit likelihood (Obs = mid_bin(Y, b), computed once as at :114).
    project_s: S[S<0] = 0 after each S-step (the C-step's projection form, :579), the build's
    S >= 0 option for free S under the log model (not a reference setting)."""
    if loss == "squared":
        Obs = ro.mid_bin(Y, b)

        def data_term(S_, C_):
            return ro.dowjons_cost(S_, C_, Obs, Wx, offset, log_model)
    else:
        def data_term(S_, C_):
            return ro.masked_nll(S_, C_, Y, Wx, b, sigma, offset, log_model)
    S = S0.clone().requires_grad_(True)
    C = C0.clone().requires_grad_(True)
    optC = torch.optim.Adam([C], lr=lr_c)
    optS = torch.optim.Adam([S], lr=lr_s)
    costs_c, costs_s, snaps, step_times = [], [], {}, []
    for i in range(n_iter):
        t0 = time.perf_counter()
        Sc = S.detach().clone()
        optC.zero_grad()
        nll = data_term(Sc, C)
        cost = nll + lambda_c * torch.norm(C, "fro") + lambda_s * torch.norm(Sc, "fro")
        cost.backward()
        optC.step()
        with torch.no_grad():
            C[C < 0] = 0
        costs_c.append(cost.item())
        t1 = time.perf_counter()
        optS.zero_grad()
        nll = data_term(S, C)
        cost = nll + lambda_c * torch.norm(C, "fro") + lambda_s * torch.norm(S, "fro")
        cost.backward()
        optS.step()
        if project_s:
            with torch.no_grad():
                S[S < 0] = 0
        costs_s.append(cost.item())
        t2 = time.perf_counter()
        step_times.append((t1 - t0, t2 - t1))
        if i + 1 in snapshots:
            snaps[i + 1] = (S.detach().clone(), C.detach().clone())
        if timer is not None and timer(i + 1, t2 - t0):
            break
    return dict(S=S.detach(), C=C.detach(), costs_c=costs_c, costs_s=costs_s, snaps=snaps,
                step_times=step_times)


def dip_solve(decoder, Z, C0, Y, Wx, b, sigma, offset=0.0, log_model=True, n_iter=4,
              lambda_c=100.0, lambda_s=100.0, lr_c=5e-3, lr_s=1e-2, optimize="weights"):
    """The DIP variant of the loop (quantized_spectrum_cartography_amd.dip.solve: the
    reference's empty qmc/dip.py defined on the GAN loop of qmc/qmc.ipynb :541-634 with
    S = decoder(Z); optimize="weights": Adam on the decoder weights, Z fixed; "z": Adam on Z,
    the weights fixed, as the GAN loop) in the reference formulation: torch CPU autograd
    through masked_nll and the decoder, torch.optim.Adam.  The S-step cost keeps the
    notebook's lambda_s ||Z||_F term.  Costs as the GAN loop's (cost.item() before each
    step)."""
    R = Z.shape[0]
    I, J = Y.shape[-2], Y.shape[-1]
    C = C0.clone().requires_grad_(True)
    Zc = Z.clone().requires_grad_(optimize == "z")
    optC = torch.optim.Adam([C], lr=lr_c)
    for p in decoder.parameters():
        p.requires_grad_(optimize == "weights")
    optS = torch.optim.Adam([Zc] if optimize == "z" else list(decoder.parameters()), lr=lr_s)
    with torch.no_grad():
        S = decoder(Zc).reshape(R, 1, I, J)
    costs_c, costs_s = [], []
    for _ in range(n_iter):
        Sc = S.detach().clone()
        optC.zero_grad()
        nll = ro.masked_nll(Sc, C, Y, Wx, b, sigma, offset, log_model)
        cost = nll + lambda_c * torch.norm(C, "fro") + lambda_s * torch.norm(Zc, "fro")
        cost.backward()
        optC.step()
        with torch.no_grad():
            C[C < 0] = 0
        costs_c.append(cost.item())
        optS.zero_grad()
        S = decoder(Zc).reshape(R, 1, I, J)
        nll = ro.masked_nll(S, C, Y, Wx, b, sigma, offset, log_model)
        cost = nll + lambda_c * torch.norm(C, "fro") + lambda_s * torch.norm(Zc, "fro")
        cost.backward()
        optS.step()
        costs_s.append(cost.item())
    return dict(S=S.detach(), C=C.detach(), costs_c=costs_c, costs_s=costs_s)


def generator_solve(generator, Z0, C0, Y, Wx, b, sigma, offset=0.0, log_model=False, n_iter=5,
                    lambda_c=100.0, lambda_s=100.0, lr_c=5e-3, lr_s=1e-2, restart=False,
                    restart_samples=(200, 200)):
    """qmc/qmc.ipynb :541-634 verbatim in structure: S = generator(Z) (network frozen, Adam on Z),
    the C-step uses the S of the previous S-step, one random restart of Z at i == 1 whose
    second round re-evaluates the last first-round sample (temp_out, :611)."""
    R = Z0.shape[0]
    I, J = Y.shape[-2], Y.shape[-1]
    C = C0.clone().requires_grad_(True)
    Z = Z0.clone().requires_grad_(True)
    optC = torch.optim.Adam([C], lr=lr_c)
    optZ = torch.optim.Adam([Z], lr=lr_s)
    with torch.no_grad():
        S = generator(Z).reshape(R, 1, I, J)
    costs_c, costs_s = [], []
    for i in range(n_iter):
        Sc = S.detach().clone()
        optC.zero_grad()
        nll = ro.masked_nll(Sc, C, Y, Wx, b, sigma, offset, log_model)
        cost = nll + lambda_c * torch.norm(C, "fro") + lambda_s * torch.norm(Z, "fro")
        cost.backward()
        optC.step()
        with torch.no_grad():
            C[C < 0] = 0
        costs_c.append(cost.item())
        if restart and i == 1:
            best = 9999999
            n1, n2 = restart_samples
            with torch.no_grad():
                for _ in range(n1):
                    temp = torch.randn((R, Z.shape[1]), dtype=torch.float32)
                    temp_out = generator(temp).reshape(R, 1, I, J)
                    crit = (ro.masked_nll(temp_out, C, Y, Wx, b, sigma, offset, log_model)
                            + lambda_c * torch.norm(C, "fro") + lambda_s * torch.norm(S, "fro"))
                    if crit < best:
                        Z.data = temp.clone()
                        best = crit
                for _ in range(n2):
                    temp = 0.2 * torch.randn((R, Z.shape[1]), dtype=torch.float32) + Z
                    crit = (ro.masked_nll(temp_out, C, Y, Wx, b, sigma, offset, log_model)
                            + lambda_c * torch.norm(C, "fro") + lambda_s * torch.norm(S, "fro"))
                    if crit < best:
                        Z.data = temp.clone()
                        best = crit
        optZ.zero_grad()
        S = generator(Z).reshape(R, 1, I, J)
        nll = ro.masked_nll(S, C, Y, Wx, b, sigma, offset, log_model)
        cost = nll + lambda_c * torch.norm(C, "fro") + lambda_s * torch.norm(Z, "fro")
        cost.backward()
        optZ.step()
        costs_s.append(cost.item())
    return dict(S=S.detach(), C=C.detach(), Z=Z.detach(), costs_c=costs_c, costs_s=costs_s)
