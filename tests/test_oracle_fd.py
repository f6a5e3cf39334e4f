"""CPU: the closed-form gradient of the oracle (oracle/explicit.py, the math the fused HIP
passes implement) against central finite differences of its own NLL in fp64 (SURVEY.md §4
build test plan: "gradient vs finite differences in fp64 on CPU"), for the linear one-bit,
multi-bin, log and squared criteria."""
import numpy as np
import pytest

from oracle import explicit


def _case(seed, R=3, K=7, P=11, nbins=2, log_model=False):
    rng = np.random.default_rng(seed)
    S = rng.uniform(0.2, 1.0, (R, P))
    C = rng.uniform(0.2, 1.0, (R, K))
    T = C.T @ S
    if log_model:
        x = np.log(T + 1e-3)
        b = np.quantile(x, np.linspace(0, 1, nbins + 1))
        b[0], b[-1] = -23.0, 3.0
        sigma = 0.7
        Y = np.clip(np.searchsorted(b, x + 0.3 * rng.standard_normal(x.shape)) - 1, 0, nbins - 1)
    else:
        b = np.quantile(T, np.linspace(0, 1, nbins + 1))
        sigma = (T.max() - T.min()) / 4
        Y = np.clip(np.searchsorted(b, T + 0.2 * sigma * rng.standard_normal(T.shape)) - 1, 0,
                    nbins - 1)
    Wx = (rng.random((K, P)) < 0.6).astype(np.float64)
    return S, C, Y, Wx, b, sigma


@pytest.mark.parametrize("nbins,log_model,loss", [(2, False, "probit"), (5, False, "probit"),
                                                  (4, True, "probit"), (4, True, "squared"),
                                                  (4, False, "squared")])
def test_gradient_matches_finite_differences(nbins, log_model, loss):
    S, C, Y, Wx, b, sigma = _case(3 + nbins, nbins=nbins, log_model=log_model)
    off = 1e-3 if log_model else 0.0
    if loss == "probit":
        f = lambda S_, C_: explicit.nll_grad(S_, C_, Y, Wx, b, sigma, off, log_model)
    else:
        f = lambda S_, C_: explicit.sq_loss_grad(S_, C_, Y, Wx, b, off, log_model)
    _, dS, dC = f(S, C)
    h = 1e-6
    for X, D, which in ((S, dS, 0), (C, dC, 1)):
        num = np.zeros_like(X)
        for idx in np.ndindex(X.shape):
            Xp, Xm = X.copy(), X.copy()
            Xp[idx] += h
            Xm[idx] -= h
            args_p = (Xp, C) if which == 0 else (S, Xp)
            args_m = (Xm, C) if which == 0 else (S, Xm)
            num[idx] = (f(*args_p)[0] - f(*args_m)[0]) / (2 * h)
        np.testing.assert_allclose(D, num, rtol=2e-5, atol=1e-6 * np.abs(num).max())
