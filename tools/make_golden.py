"""Generate golden input/output vectors from the REFERENCE implementation.

Runs only in the authoring container, where the read-only reference tree is mounted
at /root/reference.  It imports the reference's own modules at run time (nothing is
copied) and records inputs + outputs as small .npz fixtures under tests/golden/.
The GPU box never runs this script; tests there read the committed fixtures.

Reference modules used (paths relative to /root/reference):
  qmc/quantization_model.py      (linear probit model)       -> ops_linear, pass_*, solve_*
  qmc/quantization_model_log.py  (log-domain probit model)   -> ops_log, pass_log, solve_log
  qmc/utils.py                   (bin-edge / offset constants)
  qmc/nlls.py                    (Gauss-Newton offset fit; executed as a script)
  qmc/onebitdata1.mat            (shipped fixture, config 1)

The solver goldens re-enact the alternating C-step / S-step of qmc/qmc.ipynb cell 1
(source lines :559-634 of the raw notebook JSON) with S as the free Adam variable
(the free-S form of backup/notebooks/onebit_lowrank.ipynb:1230-1236), using the
reference's get_tensor / prob_probit and torch.optim.Adam verbatim.

The "DowJons" squared-criterion golden (solve_sq_32) re-enacts qmc/qmc_dowjons.ipynb :114-162
the same way (free S), with the reference's get_quantized_obs_from_ordinal / get_tensor.

Usage:  PYTHONDONTWRITEBYTECODE=1 python tools/make_golden.py [solve_sq_32]
"""
import io
import os
import runpy
import sys
import contextlib

import numpy as np
import scipy.io as sio
import torch

REF = "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden")

sys.dont_write_bytecode = True
sys.path += [os.path.join(REF, "qmc"), os.path.join(REF, "deep_prior")]
import quantization_model as qm  # noqa: E402
import quantization_model_log as qml  # noqa: E402
import utils as qutils  # noqa: E402

torch.set_num_threads(1)  # deterministic CPU reductions for the fixtures


def f32(t):
    return t.detach().cpu().numpy().astype(np.float32)


def save(name, **arrays):
    path = os.path.join(OUT, name + ".npz")
    np.savez_compressed(path, torch_version=np.array(torch.__version__), **arrays)
    print("wrote", path, sum(np.asarray(a).nbytes for a in arrays.values()), "bytes")


# ----------------------------------------------------------------------------------
# elementwise / small ops
# ----------------------------------------------------------------------------------
def gen_ops():
    g = {}
    torch.manual_seed(101)
    K, I, J, R = 6, 10, 12, 3
    X = torch.rand(K, I, J)
    g["X"] = f32(X)
    # linear one-bit: b = [0, thr, max]; quantize draws torch.randn from the global RNG
    thr = float(X.median())
    b1 = torch.tensor([0.0, thr, float(X.max())])
    sigma1 = 0.1
    torch.manual_seed(7)
    Y1 = qm.quantize(X, sigma1, b1)
    torch.manual_seed(7)
    g["noise_lin"] = f32(torch.randn(X.shape))
    g["b_onebit"], g["sigma_onebit"], g["Y_onebit"] = f32(b1), np.float32(sigma1), Y1.numpy()
    # linear multi-bin
    b5 = torch.linspace(0.0, 1.0, 6)
    torch.manual_seed(8)
    Y5 = qm.quantize(X, 0.05, b5)
    torch.manual_seed(8)
    g["noise_lin5"] = f32(torch.randn(X.shape))
    g["b_5bins"], g["sigma_5bins"], g["Y_5bins"] = f32(b5), np.float32(0.05), Y5.numpy()
    # prob_probit (linear clamps b[0], b[-1] to -/+1e5: quantization_model.py:31-33)
    Xh = torch.rand(K, I, J)
    g["Xhat"] = f32(Xh)
    g["P_onebit"] = f32(qm.prob_probit(Y1, Xh, b1, sigma1))
    g["P_5bins"] = f32(qm.prob_probit(Y5, Xh, b5, 0.05))
    # F_probit
    y = torch.linspace(-3, 3, 257)
    g["Fy"], g["F_probit_0p7"] = f32(y), f32(qm.F_probit(y, 0.7))
    # get_tensor / outer / NMSE
    S = torch.rand(R, 1, I, J)
    C = torch.rand(R, K)
    T = qm.get_tensor(S, C)
    g["S"], g["C"], g["T"] = f32(S), f32(C), f32(T)
    g["nmse"] = np.float32(qm.NMSE(T, X).item())
    # NegLikelihood (BCE-probit) with a {0,1} target
    tgt = (X > thr).float()
    crit = qm.NegLikelihood(mean=thr, std=0.2, probit=True)
    g["bce_target"], g["bce_mean"], g["bce_std"] = f32(tgt), np.float32(thr), np.float32(0.2)
    g["negll_bce"] = np.float32(crit(T, tgt).item())
    save("ops_linear", **g)

    # ---- log model ----
    h = {}
    torch.manual_seed(202)
    Xp = torch.rand(K, I, J) ** 6 * 0.05  # positive map-like values spanning many decades
    bl = torch.tensor(qutils.QUANTIZATION_BOUNDARIES_4_BINS_LOG)
    off = qutils.LOG_OFFSET_4
    torch.manual_seed(9)
    Yl = qml.quantize(Xp, 1.287, bl, offset=off)
    torch.manual_seed(9)
    h["noise_log"] = f32(torch.randn(Xp.shape))
    h["X"], h["b"], h["sigma"], h["offset"], h["Y"] = f32(Xp), f32(bl), np.float32(1.287), np.float64(off), Yl.numpy()
    Xh = torch.log(torch.rand(K, I, J) * 0.01 + off)
    h["Xhat"], h["P"] = f32(Xh), f32(qml.prob_probit(Yl, Xh, bl, 1.287))
    h["obs_mid"] = f32(qml.get_quantized_obs_from_ordinal(Yl, bl, 1.287))
    T2 = torch.rand(K, I, J) * 0.05
    h["T2"] = f32(T2)
    h["nmse_log"] = np.float32(qml.NMSE_LOG(T2, Xp, off).item())
    # default offset of the log module (LOG_OFFSET_7_ADJUSTED, quantization_model_log.py:7)
    b7 = torch.tensor(qutils.QUANTIZATION_BOUNDARIES_7_ADJUSTED)
    torch.manual_seed(10)
    Y7 = qml.quantize(Xp, 0.5, b7)
    torch.manual_seed(10)
    h["noise_log7"] = f32(torch.randn(Xp.shape))
    h["b7"], h["Y7"] = f32(b7), Y7.numpy()
    save("ops_log", **h)


# ----------------------------------------------------------------------------------
# one fused pass: NLL, cost, dS, dC through the reference autograd path
# ----------------------------------------------------------------------------------
def synth_onebit(seed, R, I, J, K, f=0.1):
    """BASELINE.md section 3 recipe (linear one-bit probit synthetic map)."""
    torch.manual_seed(seed)
    S_true = torch.rand(R, 1, I, J)
    C_true = torch.rand(R, K)
    T_true = qm.get_tensor(S_true, C_true)
    thr = float(T_true.median())
    tmax, tmin = float(T_true.max()), float(T_true.min())
    sigma = (tmax - tmin) / 4
    b = torch.tensor([0.0, thr, tmax])
    Y = qm.quantize(T_true, sigma, b).unsqueeze(1)
    Wx = torch.bernoulli(torch.full((K, 1, I, J), f))
    S0 = 0.5 * torch.rand(R, 1, I, J)
    C0 = 0.5 * torch.rand(R, K)
    return dict(S_true=S_true, C_true=C_true, T_true=T_true, b=b, sigma=sigma, Y=Y, Wx=Wx, S0=S0, C0=C0)


def synth_log(seed, R, I, J, K, f=0.1):
    """Log-model analogue (qmc.ipynb :510-537 with the _4_BINS_LOG edges and LOG_OFFSET_4)."""
    torch.manual_seed(seed)
    S_true = torch.rand(R, 1, I, J) ** 4 * 0.2
    C_true = torch.rand(R, K)
    T_true = qm.get_tensor(S_true, C_true)
    b = torch.tensor(qutils.QUANTIZATION_BOUNDARIES_4_BINS_LOG)
    off = qutils.LOG_OFFSET_4
    sigma = 5.0
    Y = qml.quantize(T_true, sigma, b, offset=off).unsqueeze(1)
    Wx = torch.bernoulli(torch.full((K, 1, I, J), f))
    # S0 kept >= 0.25 so that ten Adam steps (|step| <= lr) cannot drive T_hat + offset below 0,
    # where log() would return NaN
    S0 = 0.25 + 0.5 * torch.rand(R, 1, I, J)
    C0 = 0.5 * torch.rand(R, K)
    return dict(S_true=S_true, C_true=C_true, T_true=T_true, b=b, sigma=sigma, Y=Y, Wx=Wx, S0=S0, C0=C0,
                offset=off)


def ref_cost(mod, S, C, d, log_model, lam_c, lam_s):
    T_hat = mod.get_tensor(S, C).unsqueeze(1)
    if log_model:
        T_hat = torch.log(T_hat + d["offset"])
    nll = -torch.sum(d["Wx"] * torch.log(mod.prob_probit(d["Y"], T_hat, d["b"], d["sigma"])))
    return nll, nll + lam_c * torch.norm(C, "fro") + lam_s * torch.norm(S, "fro")


def gen_pass(name, d, log_model, lam_c=100.0, lam_s=100.0):
    mod = qml if log_model else qm
    S = d["S0"].clone().requires_grad_(True)
    C = d["C0"].clone().requires_grad_(True)
    nll, cost = ref_cost(mod, S, C, d, log_model, lam_c, lam_s)
    cost.backward()
    out = dict(S=f32(d["S0"]), C=f32(d["C0"]), Y=d["Y"].numpy().astype(np.int64), Wx=f32(d["Wx"]),
               b=f32(d["b"]), sigma=np.float32(d["sigma"]), offset=np.float64(d.get("offset", 0.0)),
               log_model=np.int32(log_model), lam_c=np.float32(lam_c), lam_s=np.float32(lam_s),
               nll=np.float64(nll.item()), cost=np.float64(cost.item()),
               dS=f32(S.grad), dC=f32(C.grad), T_true=f32(d["T_true"]))
    save(name, **out)


# ----------------------------------------------------------------------------------
# alternating solver (free S): qmc.ipynb :559-634 with S as the Adam variable
# ----------------------------------------------------------------------------------
def gen_solve(name, d, log_model, n_iter, lam_c=100.0, lam_s=100.0, lr_c=5e-3, lr_s=1e-2):
    mod = qml if log_model else qm
    S = d["S0"].clone().requires_grad_(True)
    C = d["C0"].clone().requires_grad_(True)
    optC = torch.optim.Adam([C], lr=lr_c)
    optS = torch.optim.Adam([S], lr=lr_s)
    costs_c, costs_s, nmses = [], [], []
    snaps = {}
    for i in range(n_iter):
        Sc = S.detach().clone()
        optC.zero_grad()
        T_hat = mod.get_tensor(Sc, C).unsqueeze(1)
        if log_model:
            T_hat = torch.log(T_hat + d["offset"])
        nll = -torch.sum(d["Wx"] * torch.log(mod.prob_probit(d["Y"], T_hat, d["b"], d["sigma"])))
        cost = nll + lam_c * torch.norm(C, "fro") + lam_s * torch.norm(Sc, "fro")
        cost.backward()
        optC.step()
        with torch.no_grad():
            C[C < 0] = 0
        costs_c.append(cost.item())
        optS.zero_grad()
        T_hat = mod.get_tensor(S, C).unsqueeze(1)
        if log_model:
            T_hat = torch.log(T_hat + d["offset"])
        nll = -torch.sum(d["Wx"] * torch.log(mod.prob_probit(d["Y"], T_hat, d["b"], d["sigma"])))
        cost = nll + lam_c * torch.norm(C, "fro") + lam_s * torch.norm(S, "fro")
        cost.backward()
        optS.step()
        costs_s.append(cost.item())
        with torch.no_grad():
            nmses.append(mod.NMSE(mod.get_tensor(S, C), d["T_true"]).item())
        if i + 1 in (1, n_iter):
            snaps["S_it%d" % (i + 1)] = f32(S)
            snaps["C_it%d" % (i + 1)] = f32(C)
    out = dict(S0=f32(d["S0"]), C0=f32(d["C0"]), Y=d["Y"].numpy().astype(np.uint8), Wx=f32(d["Wx"]).astype(np.uint8),
               b=f32(d["b"]), sigma=np.float32(d["sigma"]), offset=np.float64(d.get("offset", 0.0)),
               log_model=np.int32(log_model), lam_c=np.float32(lam_c), lam_s=np.float32(lam_s),
               lr_c=np.float32(lr_c), lr_s=np.float32(lr_s), n_iter=np.int32(n_iter),
               T_true=f32(d["T_true"]), costs_c=np.array(costs_c), costs_s=np.array(costs_s),
               nmse=np.array(nmses), **snaps)
    save(name, **out)


# ----------------------------------------------------------------------------------
# Euclidean ("DowJons") criterion: qmc/qmc_dowjons.ipynb :114-162 with S as the free Adam
# variable: Obs = get_quantized_obs_from_ordinal(Y, b, std) once, then per C- and S-step
#   cost = torch.norm(Wx*(log(get_tensor(S, C)+offset) - Obs))**2 + lam_c||C|| + lam_s||S||
# ----------------------------------------------------------------------------------
def gen_solve_sq(name, d, n_iter, lam_c=100.0, lam_s=100.0, lr_c=5e-3, lr_s=1e-2):
    Obs = qml.get_quantized_obs_from_ordinal(d["Y"], d["b"], d["sigma"])
    S = d["S0"].clone().requires_grad_(True)
    C = d["C0"].clone().requires_grad_(True)
    optC = torch.optim.Adam([C], lr=lr_c)
    optS = torch.optim.Adam([S], lr=lr_s)
    costs_c, costs_s, snaps = [], [], {}
    for i in range(n_iter):
        Sc = S.detach().clone()
        optC.zero_grad()
        T_hat = torch.log(qml.get_tensor(Sc, C).unsqueeze(1) + d["offset"])
        cost = (torch.norm(d["Wx"] * (T_hat - Obs)) ** 2 + lam_c * torch.norm(C, "fro")
                + lam_s * torch.norm(Sc, "fro"))
        cost.backward()
        optC.step()
        with torch.no_grad():
            C[C < 0] = 0
        costs_c.append(cost.item())
        optS.zero_grad()
        T_hat = torch.log(qml.get_tensor(S, C).unsqueeze(1) + d["offset"])
        cost = (torch.norm(d["Wx"] * (T_hat - Obs)) ** 2 + lam_c * torch.norm(C, "fro")
                + lam_s * torch.norm(S, "fro"))
        cost.backward()
        optS.step()
        costs_s.append(cost.item())
        if i + 1 in (1, n_iter):
            snaps["S_it%d" % (i + 1)] = f32(S)
            snaps["C_it%d" % (i + 1)] = f32(C)
    out = dict(S0=f32(d["S0"]), C0=f32(d["C0"]), Y=d["Y"].numpy().astype(np.uint8),
               Wx=f32(d["Wx"]).astype(np.uint8), b=f32(d["b"]), sigma=np.float32(d["sigma"]),
               offset=np.float64(d["offset"]), log_model=np.int32(1), lam_c=np.float32(lam_c),
               lam_s=np.float32(lam_s), lr_c=np.float32(lr_c), lr_s=np.float32(lr_s),
               n_iter=np.int32(n_iter), Obs=f32(Obs), costs_c=np.array(costs_c),
               costs_s=np.array(costs_s), **snaps)
    save(name, **out)


# ----------------------------------------------------------------------------------
# shipped fixture (config 1) and nlls known answers
# ----------------------------------------------------------------------------------
def gen_mat():
    m = sio.loadmat(os.path.join(REF, "qmc", "onebitdata1.mat"))
    # qmc_utils.load_data (qmc/qmc_utils.py:12-20) casts to float32; the notebook permutes
    # T(K,I,J), S(R,I,J), C(R,K) (qmc/qmc.ipynb :498-503)
    S_true = torch.from_numpy(m["S_true"]).float().permute(2, 0, 1)
    C_true = torch.from_numpy(m["C_true"]).float().permute(1, 0)
    T_true = torch.from_numpy(m["T_true"]).float().permute(2, 0, 1)
    T = torch.from_numpy(m["T"].astype(np.float32)).permute(2, 0, 1)
    T_rec = qm.get_tensor(S_true.unsqueeze(1), C_true)
    save("mat_c1", S_true=f32(S_true), C_true=f32(C_true), T_true=f32(T_true), T=T.numpy().astype(np.int8),
         Om=m["Om"].astype(np.uint8), T_rec=f32(T_rec), nmse_rec=np.float64(qm.NMSE(T_rec, T_true).item()))


def gen_nlls():
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        ns = runpy.run_path(os.path.join(REF, "qmc", "nlls.py"), run_name="__main__")
    theta = ns["theta_ls"]
    x = ns["x"]
    edges = (np.log(theta[0, 0] + x) + theta[1, 0] - theta[1, 0]).squeeze()
    save("nlls", raw=np.asarray(x).squeeze(), theta=np.asarray(theta).squeeze(), edges=edges,
         util_edges16=np.array(qutils.QUANTIZATION_BOUNDARIES_16_ADJUSTED),
         util_offset16=np.float64(qutils.LOG_OFFSET_16_ADJUSTED),
         util_edges7=np.array(qutils.QUANTIZATION_BOUNDARIES_7_ADJUSTED),
         util_offset7=np.float64(qutils.LOG_OFFSET_7_ADJUSTED))


def main():
    os.makedirs(OUT, exist_ok=True)
    if sys.argv[1:] == ["solve_sq_32"]:  # add only this fixture
        gen_solve_sq("solve_sq_32", synth_log(20267, 3, 32, 32, 16), n_iter=10)
        return
    gen_ops()
    gen_pass("pass_onebit_small", synth_onebit(20260, 3, 16, 16, 12), log_model=False)
    gen_pass("pass_onebit_64", synth_onebit(20261, 4, 64, 64, 32), log_model=False)
    gen_pass("pass_log_small", synth_log(20265, 3, 16, 16, 12), log_model=True)
    gen_solve("solve_onebit_64", synth_onebit(20262, 4, 64, 64, 32), log_model=False, n_iter=10)
    gen_solve("solve_log_32", synth_log(20266, 3, 32, 32, 16), log_model=True, n_iter=10)
    gen_solve_sq("solve_sq_32", synth_log(20267, 3, 32, 32, 16), n_iter=10)
    gen_mat()
    gen_nlls()


if __name__ == "__main__":
    main()
