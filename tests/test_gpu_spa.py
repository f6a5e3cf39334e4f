"""GPU parity of the SPA warm start (qsc_syrk, qsc_spa) and the NNLS C-update (qsc_nnls) vs the
numpy fp64 oracle (oracle/spa.py, NMF_SPA.m / joint_opt_ae.m:404-417 restated).

Tolerances: picked bins identical; the K x K Gram (f32 MFMA products, f32 accumulation over
P pixels) 1e-5 relative Frobenius; C and S 1e-4 relative (the C fit inverts an R x R block of
the f32 Gram); NNLS solutions 1e-4 relative and exact zero patterns away from degenerate ties.
"""
import numpy as np
import pytest
import torch

from conftest import rel_fro
from oracle import spa as ospa

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def spa():
    from quantized_spectrum_cartography_amd import spa
    return spa


@pytest.mark.parametrize("K,P", [(1, 7), (37, 1001), (64, 4096), (130, 3000), (256, 65536)])
def test_syrk_matches_fp64(spa, K, P):
    g = torch.Generator().manual_seed(K * 7 + P)
    T = torch.rand((K, P), generator=g)
    w = (torch.rand(P, generator=g) < 0.5).float()
    G = spa.syrk(T.cuda(), w.cuda()).cpu().numpy()
    Tn = T.double().numpy()
    Go = (Tn * w.double().numpy()[None, :]) @ Tn.T
    assert rel_fro(G, Go) < 1e-5
    assert np.array_equal(G, G.T)
    G2 = spa.syrk(T.cuda()).cpu().numpy()
    assert rel_fro(G2, Tn @ Tn.T) < 1e-5


@pytest.mark.parametrize("K,P,R,seed,masked", [(32, 400, 3, 0, False), (64, 1000, 6, 1, True),
                                               (128, 2048, 8, 2, False),
                                               (256, 16384, 16, 3, True)])
def test_spa_matches_oracle(spa, K, P, R, seed, masked):
    C, S, T, pure = ospa.separable_problem(K, P, R, seed)
    mask = (np.random.default_rng(seed).random(P) < 0.4) if masked else None
    Co, So, idx_o = ospa.nmf_spa(T, R, mask)
    Tt = torch.from_numpy(T).float().cuda()
    wt = torch.from_numpy(mask.astype(np.float32)).cuda() if masked else None
    Cg, Sg, idx = spa.spa_init(Tt, R, wt)
    assert idx == idx_o and sorted(idx) == sorted(pure)
    assert rel_fro(Cg.cpu().numpy(), Co.T) < 1e-4
    assert rel_fro(Sg.cpu().numpy(), So) < 1e-4
    Cm, Sm = spa.NMF_SPA(Tt, R) if not masked else (None, None)
    if Cm is not None:
        assert Cm.shape == (K, R) and Sm.shape == (R, P)


def test_spa_stops_on_vanishing_residual(spa):
    C, S, T, pure = ospa.separable_problem(48, 500, 2, 7)
    Cg, Sg, idx = spa.spa_init(torch.from_numpy(T).float().cuda(), 5)
    assert sorted(idx) == sorted(pure)
    assert torch.all(Cg[2:] == 0) and torch.all(Sg[2:] == 0)


@pytest.mark.parametrize("R,P,K,lam", [(1, 50, 9, 0.0), (4, 300, 64, 0.1), (8, 2000, 256, 0.5),
                                       (16, 4096, 100, 1.0)])
def test_nnls_matches_lsqnonneg(R, P, K, lam):
    from quantized_spectrum_cartography_amd import gram
    rng = np.random.default_rng(R * 100 + K)
    Q = rng.standard_normal((R, P)).astype(np.float32)
    Y = rng.standard_normal((K, P)).astype(np.float32)
    Co = ospa.nnls_c_update(Q, Y, lam)  # (K, R)
    Cg = gram.nnls_spectra(torch.from_numpy(Q).cuda(), torch.from_numpy(Y).cuda(), lam)
    Cg = Cg.cpu().numpy().T
    assert np.all(Cg >= 0)
    assert rel_fro(Cg, Co) < 1e-4
    # active sets agree wherever the oracle's coordinate is clearly away from the bound
    clear = (Co > 1e-3 * np.abs(Co).max()) | (Co == 0)
    assert np.array_equal((Cg > 0)[clear & (Co > 0)], np.ones(int((clear & (Co > 0)).sum()), bool))
