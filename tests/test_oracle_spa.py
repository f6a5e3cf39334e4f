"""CPU: the SPA / NNLS oracle (oracle/spa.py) by known-answer tests.

The reference's SPA warm start and NNLS C-update are MATLAB (backup/algorithms/NMF_SPA.m,
joint_opt_ae.m:404-417), which cannot run here; the restatement is pinned by construction:
on noiseless separable data SPA must pick exactly the planted pure bins and NMF_SPA must
return the planted spectra up to scale; the NNLS restatement must satisfy the KKT conditions
of its problem.
"""
import numpy as np
import pytest

from oracle import spa as ospa


@pytest.mark.parametrize("K,P,R,seed", [(32, 400, 3, 0), (64, 1000, 6, 1), (128, 2048, 8, 2)])
def test_spa_picks_planted_pure_bins(K, P, R, seed):
    C, S, T, pure = ospa.separable_problem(K, P, R, seed)
    Cs, Sm, idx = ospa.nmf_spa(T, R)
    assert sorted(idx) == sorted(pure)
    # recovered spectra = planted ones up to scale and permutation
    Ct = C / np.linalg.norm(C, axis=1, keepdims=True)
    for r, k in enumerate(idx):
        owner = pure.index(k)
        np.testing.assert_allclose(Cs[:, r], Ct[owner], rtol=1e-9, atol=1e-12)
    # and the reconstruction is exact
    np.testing.assert_allclose(Cs @ Sm, T, rtol=1e-9, atol=1e-9)


def test_spa_masked_pixels_zero_and_stops_on_zero_residual():
    C, S, T, pure = ospa.separable_problem(32, 300, 2, 5)
    mask = np.random.default_rng(0).random(300) < 0.3
    Cs, Sm, idx = ospa.nmf_spa(T, 4, mask)  # rank 2 data: residual vanishes after 2 picks
    assert len(idx) == 2 and sorted(idx) == sorted(pure)
    assert np.all(Sm[:, ~mask] == 0)


def test_nnls_kkt():
    rng = np.random.default_rng(3)
    R, P, K, lam = 6, 200, 40, 0.3
    Q = rng.standard_normal((R, P))
    Y = rng.standard_normal((K, P))
    C = ospa.nnls_c_update(Q, Y, lam)
    G = Q @ Q.T + lam ** 2 * np.eye(R)
    B = Q @ Y.T
    assert np.all(C >= 0)
    grad = G @ C.T - B  # (R, K): >= 0 where c = 0, = 0 where c > 0
    assert np.all(grad[C.T == 0] >= -1e-9)
    np.testing.assert_allclose(grad[C.T > 0], 0.0, atol=1e-8)
