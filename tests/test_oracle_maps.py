"""CPU: the synthetic-map oracle (oracle/maps.py) and the host-side pieces of maps.py.

No run of the MATLAB reference is possible here; the shadowing generators are pinned by the
covariance the reference specifies (Shadowing_data.m:6-7: E[z(x) z(x')] = var^2 exp(-|x-x'|/Xc)).
"""
import numpy as np
import torch

from oracle import maps as omaps
from quantized_spectrum_cartography_amd import maps


def test_cholesky_shadowing_covariance():
    rng = np.random.default_rng(0)
    I = J = 6
    var, Xc = 2.0, 5.0
    Z = np.stack([omaps.shadowing_chol(I, J, var, Xc, rng) for _ in range(3000)])
    emp = np.mean(Z[:, 2, 2] * Z[:, 2, 3])
    assert abs(np.mean(Z ** 2) - var ** 2) < 0.15 * var ** 2
    assert abs(emp - omaps.exp_cov(1.0, var, Xc)) < 0.2 * var ** 2


def test_circulant_embedding_reproduces_exponential_covariance():
    # the covariance the embedding actually realises = inverse FFT of the clipped eigenvalues
    for I, J, Xc in [(51, 51, 50.0), (64, 48, 10.0), (256, 256, 50.0)]:
        lam, M, N, neg = maps._embedding(I, J, Xc, 1.0, torch.device("cpu"))
        c = torch.fft.ifft2(lam.to(torch.complex128)).real.numpy()
        d = np.sqrt(np.arange(I)[:, None] ** 2 + np.arange(J)[None, :] ** 2)
        err = np.abs(c[:I, :J] - np.exp(-d / Xc)).max()
        assert err < 0.03, (I, J, Xc, err, neg)


def test_psd_basis_shapes_and_peaks():
    rng = np.random.default_rng(1)
    C = maps.psd_basis(64, 4, rng)
    assert C.shape == (64, 4) and np.all(C >= 0)
    np.testing.assert_allclose(np.linalg.norm(C, axis=0), 1.0, rtol=1e-12)
    Cs = maps.psd_basis(64, 3, np.random.default_rng(2), basis="s", separable=False)
    assert Cs.shape == (64, 3) and np.all(Cs >= 0)


def test_compose_oracle_properties():
    rng = np.random.default_rng(3)
    sh = rng.standard_normal((2, 20, 30))
    loc = np.array([[3.0, 4.0], [19.5, 10.0]])
    S = omaps.compose(sh, loc, [2.2, 2.4])
    np.testing.assert_allclose(np.linalg.norm(S.reshape(2, -1), axis=1), 1.0)
    Sd = omaps.compose(sh, loc, [2.2, 2.4], dB=True)
    np.testing.assert_allclose(Sd, 10 * np.log10(S))
