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


def test_observed_form_equals_dense_form():
    """nll_grad_obs (observed entries only, chunked) == nll_grad (dense, masked), both models."""
    rng = np.random.default_rng(3)
    for log_model in (False, True):
        R, K, P = 4, 9, 57
        S = rng.random((R, P)) + 0.1
        C = rng.random((R, K)) + 0.1
        T = C.T @ S
        b = np.quantile(np.log(T) if log_model else T, [0, 0.3, 0.6, 1.0])
        b[0] -= 1.0
        Y = np.clip(np.digitize(np.log(T) if log_model else T, b[1:-1]), 0, 2)
        Wx = (rng.random((K, P)) < 0.4).astype(np.float64)
        ref = explicit.nll_grad(S, C, Y, Wx, b, 0.3, 1e-3, log_model)
        obs = explicit.observed(Y, Wx)
        got = explicit.nll_grad_obs(S, C, obs, b, 0.3, 1e-3, log_model, chunk=50)
        assert abs(got[0] - ref[0]) <= 1e-12 * abs(ref[0])
        assert np.allclose(got[1], ref[1], rtol=1e-12, atol=1e-14)
        assert np.allclose(got[2], ref[2], rtol=1e-12, atol=1e-14)


def test_explicit_solve_follows_reference_solver():
    """The fp64 explicit-gradient loop tracks the reference formulation (oracle/solver.py,
    pinned to the reference goldens) within the fp32-vs-fp64 tolerance."""
    import torch
    from oracle import reference_ops as ro, solver as osolver
    g = torch.Generator().manual_seed(4)
    R, I, J, K = 3, 10, 9, 12
    S_t, C_t = torch.rand(R, 1, I, J, generator=g), torch.rand(R, K, generator=g)
    T = ro.get_tensor(S_t, C_t)
    b = torch.tensor([0.0, float(T.median()), float(T.max())])
    sigma = (float(T.max()) - float(T.min())) / 4
    Y = ro.quantize(T, sigma, b, noise=torch.randn(T.shape, generator=g)).unsqueeze(1)
    Wx = torch.bernoulli(torch.full((K, 1, I, J), 0.4), generator=g)
    S0, C0 = 0.5 * torch.rand(R, 1, I, J, generator=g), 0.5 * torch.rand(R, K, generator=g)
    ref = osolver.free_s_solve(S0, C0, Y, Wx, b, sigma, n_iter=4)
    obs = explicit.observed(Y.reshape(K, -1).numpy(), Wx.reshape(K, -1).numpy())
    S, C, cc, cs = explicit.explicit_solve(S0.reshape(R, -1).numpy(), C0.numpy(), obs, b.numpy(),
                                           sigma, n_iter=4)
    rel = lambda a, b_: np.linalg.norm(a - b_) / np.linalg.norm(b_)
    assert rel(S, ref["S"].reshape(R, -1).double().numpy()) < 1e-5
    assert rel(C, ref["C"].double().numpy()) < 1e-5
    assert np.allclose(cc, ref["costs_c"], rtol=1e-5) and np.allclose(cs, ref["costs_s"], rtol=1e-5)
