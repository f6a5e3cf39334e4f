"""GPU parity at the BASELINE.json workloads themselves (configs C2-C5), not just small shapes.

Each config runs through the fused HIP path and is checked against the fp64 closed-form oracle
(oracle/explicit.py, evaluated at the observed entries only so that C3/C4 finish in seconds;
itself pinned to the reference's autograd and goldens, tests/test_oracle_*.py):
  * one pass: NLL, dS, dC at (S0, C0) vs explicit.nll_grad_obs             rel 1e-5
  * 3 outer iterations of the alternating solver vs explicit.explicit_solve  rel Frobenius 1e-5
    (the north_star tolerance on recovered S, C), costs rel 1e-5
Reference anchors: qmc/qmc.ipynb :559-645 (loop, per-entry mask :493, likelihood :568-575),
backup/notebooks/onebit_lowrank.ipynb :1230-1291 (free S).
Configs: C2 256x256x64 R=4; C3 512x512x256 R=8 (the metric's config, fused scpass path);
C4 one K-slab shard 512x512x128 R=16 of the 8-GPU 512x512x1024 problem through KSlabSolver
(world 1, RCCL); C5 256x256x64 R=4 log model, 4 log bins, sigma 5, offset 1e-10, generated
map, + the DIP path's fused dS at S = decoder(Z).
"""
import os
import socket

import numpy as np
import pytest
import torch

from conftest import rel_fro
from oracle import explicit

pytestmark = pytest.mark.gpu

TOL = 1e-5  # north_star: within 1e-5 relative (fp32)


def _onebit(cfg, seed):
    from quantized_spectrum_cartography_amd import synthetic
    I, J, K, R = synthetic.CONFIGS[cfg]
    return synthetic.onebit_problem(I, J, K, R, f=0.1, seed=seed), (I, J, K, R)


def _np(t, shape=None):
    a = t.detach().cpu().numpy()
    return a.reshape(shape) if shape is not None else a


def _pass_check(prob, dims, log_model=False, offset=0.0):
    from quantized_spectrum_cartography_amd import fused
    from quantized_spectrum_cartography_amd.obs import Observations
    I, J, K, R = dims
    P = I * J
    obs = Observations(prob["Y"], prob["Wx"], prob["b"], prob["sigma"], offset=offset,
                       log_model=log_model, R_hint=R)
    S = prob["S0"].cuda().requires_grad_(True)
    C = prob["C0"].cuda().requires_grad_(True)
    nll = fused.ProbitNLL.apply(S, C, obs)
    nll.backward()
    ob = explicit.observed(_np(prob["Y"], (K, P)), _np(prob["Wx"], (K, P)))
    assert ob[0].shape[0] == obs.nnz
    rn, rdS, rdC = explicit.nll_grad_obs(_np(prob["S0"], (R, P)), _np(prob["C0"]), ob,
                                         _np(prob["b"]), prob["sigma"], offset, log_model)
    assert np.isfinite(rn)
    assert abs(nll.item() - rn) / abs(rn) < TOL
    assert rel_fro(_np(S.grad, (R, P)), rdS) < TOL
    assert rel_fro(_np(C.grad), rdC) < TOL
    return ob


def _solver_check(prob, dims, ob, iters=3, log_model=False, offset=0.0, expect_fused=None,
                  lr_c=5e-3, lr_s=1e-2):
    from quantized_spectrum_cartography_amd import qmc
    I, J, K, R = dims
    P = I * J
    res = qmc.solve(prob["Y"], prob["Wx"], prob["b"], prob["sigma"], S_init=prob["S0"],
                    C_init=prob["C0"], max_iter=iters, log_model=log_model,
                    offset=offset if log_model else None, use_graph=True, lr_c=lr_c, lr_s=lr_s,
                    project_s=False)  # (the oracle's explicit solve does not project S)
    if expect_fused is not None:
        assert res.fused == expect_fused
    S, C, cc, cs = explicit.explicit_solve(_np(prob["S0"], (R, P)), _np(prob["C0"]), ob,
                                           _np(prob["b"]), prob["sigma"], offset, log_model,
                                           n_iter=iters, lr_c=lr_c, lr_s=lr_s)
    assert rel_fro(_np(res.S, (R, P)), S) < TOL
    assert rel_fro(_np(res.C), C) < TOL
    assert np.allclose(res.costs_c, cc, rtol=TOL) and np.allclose(res.costs_s, cs, rtol=TOL)


@pytest.mark.parametrize("cfg,seed,fused", [("c2", 20262, True), ("c3", 20263, True)])
def test_onebit_config_pass_and_solver(cfg, seed, fused):
    """C2 / C3 (BASELINE.md section 3 recipe, the bench's own inputs for C3)."""
    prob, dims = _onebit(cfg, seed)
    ob = _pass_check(prob, dims)
    _solver_check(prob, dims, ob, expect_fused=fused)


def test_c3_long_run_properties():
    """C3 at full size over 120 iterations (past what the oracle can follow): size-independent
    properties of the alternating solver (qmc/qmc.ipynb :559-634).
      * two solvers on the same inputs agree bit for bit (graph replay of chained chunks vs one
        eager run): the pass reductions are in a fixed order, no atomics;
      * both costs fall: the C-step cost after the run is below the first one, and so is the
        S-step cost;
      * C >= 0 after every C-step projection (:579), everything finite."""
    from quantized_spectrum_cartography_amd import qmc
    prob, (I, J, K, R) = _onebit("c3", 20263)
    kw = dict(S_init=prob["S0"], C_init=prob["C0"], max_iter=120)
    a = qmc.solve(prob["Y"], prob["Wx"], prob["b"], prob["sigma"], use_graph=True, **kw)
    b = qmc.solve(prob["Y"], prob["Wx"], prob["b"], prob["sigma"], use_graph=False, **kw)
    assert a.fused and b.fused
    assert np.array_equal(_np(a.S), _np(b.S)) and np.array_equal(_np(a.C), _np(b.C))
    assert a.costs_c == b.costs_c and a.costs_s == b.costs_s
    assert np.isfinite(_np(a.S)).all() and np.isfinite(_np(a.C)).all()
    assert (_np(a.C) >= 0).all()
    assert len(a.costs_c) == 120 and a.costs_c[-1] < a.costs_c[0] and a.costs_s[-1] < a.costs_s[0]


def _c5_problem(seed=5):
    from quantized_spectrum_cartography_amd import synthetic
    prob = synthetic.c5_problem(seed=seed)
    return prob, (256, 256, 64, 4), prob["offset"]


def test_c5_log_model_pass_and_solver():
    """C5: log model, 4 log bins, sigma = 5, offset LOG_OFFSET_4 (qmc/qmc.ipynb :510-537)."""
    prob, dims, off = _c5_problem()
    assert len(torch.unique(prob["Y"])) >= 3  # the generated map spans the log bins
    ob = _pass_check(prob, dims, log_model=True, offset=off)
    # free S in the log model: the step must keep T_hat = S C > 0 (S0 ~ 1e-3; the reference's
    # S = G(Z) is a sigmoid output and cannot go negative), so lr_s is scaled to S
    _solver_check(prob, dims, ob, log_model=True, offset=off, lr_s=1e-5)
    assert np.isfinite(ob[0]).all()


def test_c5_free_s_log_model_default_stays_finite():
    """free S under the log model with the DEFAULT arguments (lr_s 1e-2, the
    solver's own default S >= 0 projection) stays finite over 200 iterations at C5 -- without the
    projection T_hat + offset reached <= 0 within 200 steps and the cost went non-finite
    (gpurun_out/r05b/bench_c5.log)."""
    from quantized_spectrum_cartography_amd import qmc
    prob, dims, off = _c5_problem()
    res = qmc.solve(prob["Y"], prob["Wx"], prob["b"], prob["sigma"], S_init=prob["S0"],
                    C_init=prob["C0"], max_iter=200, log_model=True, offset=off, use_graph=True)
    S, C = _np(res.S), _np(res.C)
    assert np.isfinite(S).all() and np.isfinite(C).all()
    assert (S >= 0).all() and (C >= 0).all()
    assert np.isfinite(res.costs_c).all() and np.isfinite(res.costs_s).all()
    # (finite, not convergent: the notebook's lr_s = 1e-2 is ~10x the C5 fields' scale, so Adam's
    # sign steps overshoot -- the quality runs scale lr_s to S, tools/quality.py)


def test_c5_dip_fused_dS_isolated():
    """The HIP part of the DIP path at C5: the fused S-pass dS at S = decoder(Z) (the gradient
    dip.solve back-propagates through the decoder) vs the fp64 oracle, 1e-5."""
    from quantized_spectrum_cartography_amd import dip, fused
    from quantized_spectrum_cartography_amd.obs import Observations
    prob, (I, J, K, R), off = _c5_problem(seed=6)
    P = I * J
    dec = dip.make_decoder(I, J, seed=3).cuda().eval()
    Z = torch.randn((R, 256), generator=torch.Generator().manual_seed(4)).cuda()
    with torch.no_grad():
        S_dec = dec(Z).reshape(R, 1, I, J) * (1.0 / I)
    obs = Observations(prob["Y"], prob["Wx"], prob["b"], 5.0, offset=off, log_model=True,
                       R_hint=R)
    S = S_dec.clone().requires_grad_(True)
    C = prob["C0"].cuda()
    nll = fused.ProbitNLL.apply(S, C, obs)
    nll.backward()
    ob = explicit.observed(_np(prob["Y"], (K, P)), _np(prob["Wx"], (K, P)))
    rn, rdS, _ = explicit.nll_grad_obs(_np(S_dec, (R, P)), _np(C), ob, _np(prob["b"]), 5.0, off,
                                       True)
    assert abs(nll.item() - rn) / abs(rn) < TOL
    assert rel_fro(_np(S.grad, (R, P)), rdS) < TOL


def test_gan_fused_dS_isolated(golden):
    """The HIP part of the GAN path (qmc/qmc.ipynb :622-634, S = Generator256(Z),
    deep_prior/networks/gan.py:83-126) isolated at the north_star tolerance: the fused S-pass
    dS (and C-pass dC, NLL) at S = G(Z) on the generator's 51x51 output, with the notebook's
    log model, 4 log bins, sigma = 5, offset LOG_OFFSET_4 and f = 0.1 on the shipped map
    (onebitdata1.mat, tests/golden/mat_c1.npz), vs the fp64 oracle at 1e-5.  (Only the torch
    generator's own backward, MIOpen vs CPU conv numerics, is held to 1e-4 end to end in
    tests/test_gpu_fused.py::test_generator_solver_vs_oracle.)"""
    from quantized_spectrum_cartography_amd import fused, nets
    from quantized_spectrum_cartography_amd import quantization_model_log as qml
    from quantized_spectrum_cartography_amd.obs import Observations
    from quantized_spectrum_cartography_amd.utils import (LOG_OFFSET_4,
                                                          QUANTIZATION_BOUNDARIES_4_BINS_LOG)
    m = golden("mat_c1")
    T = torch.from_numpy(m["T_true"].astype(np.float32))  # (64, 51, 51)
    K, I, J = T.shape
    R, P = 2, I * J
    g = torch.Generator().manual_seed(31)
    b = torch.tensor(QUANTIZATION_BOUNDARIES_4_BINS_LOG)
    Y = qml.quantize(T, 5.0, b, offset=LOG_OFFSET_4, noise=torch.randn(T.shape, generator=g))
    Y = Y.cpu().unsqueeze(1)
    Wx = torch.bernoulli(torch.full((K, 1, I, J), 0.1), generator=g)
    assert len(torch.unique(Y)) >= 3
    torch.manual_seed(3)
    gen = nets.Generator256().cuda().eval()
    Z = torch.randn((R, 256), generator=torch.Generator().manual_seed(4)).cuda()
    with torch.no_grad():
        S_gen = gen(Z).reshape(R, 1, I, J)
    C0 = torch.from_numpy(m["C_true"].astype(np.float32)) * (0.5 + torch.rand(R, K, generator=g))
    obs = Observations(Y, Wx, b, 5.0, offset=LOG_OFFSET_4, log_model=True, R_hint=R)
    S = S_gen.clone().requires_grad_(True)
    C = C0.cuda().requires_grad_(True)
    nll = fused.ProbitNLL.apply(S, C, obs)
    nll.backward()
    ob = explicit.observed(_np(Y, (K, P)), _np(Wx, (K, P)))
    rn, rdS, rdC = explicit.nll_grad_obs(_np(S_gen, (R, P)), _np(C0), ob, _np(b), 5.0,
                                         LOG_OFFSET_4, True)
    assert np.isfinite(rn)
    assert abs(nll.item() - rn) / abs(rn) < TOL
    assert rel_fro(_np(S.grad, (R, P)), rdS) < TOL
    assert rel_fro(_np(C.grad), rdC) < TOL


def test_c5_dip_solve_defaults_finite():
    """dip.solve with its defaults (offset = the reference log model's LOG_OFFSET, zero C
    init): the first C-pass sees T_hat = 0 and must stay finite."""
    from quantized_spectrum_cartography_amd import dip
    from quantized_spectrum_cartography_amd.utils import QUANTIZATION_BOUNDARIES_4_BINS_LOG
    prob, (I, J, K, R), _ = _c5_problem(seed=7)
    b = torch.tensor(QUANTIZATION_BOUNDARIES_4_BINS_LOG)
    res = dip.solve(prob["Y"][:, :, :64, :64].contiguous(), prob["Wx"][:, :, :64, :64].contiguous(),
                    b, 5.0, R, max_iter=3)
    assert np.all(np.isfinite(res.costs_c)) and np.all(np.isfinite(res.costs_s))
    with pytest.raises(ValueError):
        dip.solve(prob["Y"][:, :, :64, :64], prob["Wx"][:, :, :64, :64], b, 5.0, R, offset=0.0,
                  max_iter=1)


@pytest.fixture(scope="module")
def pg():
    import torch.distributed as dist
    if dist.is_initialized():
        yield dist
        return
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % port, rank=0,
                            world_size=1, device_id=torch.device("cuda", 0))
    yield dist
    dist.destroy_process_group()


def test_c4_kslab_shard_pass_and_solver(pg):
    """C4 per-GPU shard: 512x512 pixels x K_loc = 128 of the 1024 bins, R = 16, through the
    north-star K-slab solver (RCCL world 1, hipGraph) -- pass and 3 iterations vs the oracle."""
    from quantized_spectrum_cartography_amd import fused, synthetic
    from quantized_spectrum_cartography_amd.distributed import KSlabSolver, kslab_observations
    I, J, K, R = 512, 512, 128, 16
    P = I * J
    prob = synthetic.kslab_onebit_problem(I, J, K, R, 0, 1, dist=None, f=0.1, seed=20264)
    obs = kslab_observations(prob["Y"], prob["Wx"], prob["b"], prob["sigma"], pg, R_hint=R)
    S = prob["S0"].cuda().requires_grad_(True)
    C = prob["C0"].cuda().requires_grad_(True)
    nll = fused.ProbitNLL.apply(S, C, obs)
    nll.backward()
    ob = explicit.observed(_np(prob["Y"], (K, P)), _np(prob["Wx"], (K, P)))
    bb = _np(prob["b"])
    rn, rdS, rdC = explicit.nll_grad_obs(_np(prob["S0"], (R, P)), _np(prob["C0"]), ob, bb,
                                         prob["sigma"])
    assert abs(nll.item() - rn) / abs(rn) < TOL
    assert rel_fro(_np(S.grad, (R, P)), rdS) < TOL
    assert rel_fro(_np(C.grad), rdC) < TOL
    sol = KSlabSolver(obs, prob["S0"], prob["C0"], dist=pg, hist_cap=8)
    sol.run(3, use_graph=True)
    torch.cuda.synchronize()
    assert sol.graph_error is None
    Sx, Cx, cc, cs = explicit.explicit_solve(_np(prob["S0"], (R, P)), _np(prob["C0"]), ob, bb,
                                             prob["sigma"], n_iter=3)
    assert rel_fro(_np(sol.S_pixels(), (R, P)), Sx) < TOL
    assert rel_fro(_np(sol.C), Cx) < TOL
    hc, hs = sol.history()
    assert np.allclose(hc, cc, rtol=TOL) and np.allclose(hs, cs, rtol=TOL)


def test_c2_holdout_early_stopping_beats_the_fixed_run():
    """qmc.solve(holdout=...) on C2 (BASELINE recipe): the unregularised free-S MLE over-fits
    with ~6 one-bit samples per pixel (map NMSE best near iteration 50, then growing); stopping
    on the held-out NLL returns an earlier, better map than the fixed 600-iteration run."""
    from quantized_spectrum_cartography_amd import metrics, qmc
    prob, (I, J, K, R) = _onebit("c2", 20262)
    kw = dict(S_init=prob["S0"], C_init=prob["C0"], max_iter=600, use_graph=True)
    full = qmc.solve(prob["Y"], prob["Wx"], prob["b"], prob["sigma"], **kw)
    es = qmc.solve(prob["Y"], prob["Wx"], prob["b"], prob["sigma"], holdout=0.1, check_every=10,
                   patience=5, **kw)
    assert es.iters < 600 and es.best_iter <= es.iters
    assert np.isfinite(_np(es.S)).all() and np.isfinite(_np(es.C)).all()
    m_full = metrics.map_nmse(full.S, full.C, prob["T_true"])
    m_es = metrics.map_nmse(es.S, es.C, prob["T_true"])
    assert m_es < m_full, (m_es, m_full)
