"""ORACLE (test infrastructure only) — Gauss-Newton fit of y = log(theta0 + x) + theta1.

Restates qmc/nlls.py:19-41: x = raw bin edges, y = 0..n-1, H = [1/(theta0 + x), 1], forty
updates theta += (H^T H)^-1 H^T (y - h(theta)) starting from theta = (1e-7, 0).  Pinned against
the reference's own outputs (tests/golden/nlls.npz) and qmc/utils.py:43-51.
"""
import numpy as np


def gauss_newton(raw, theta0=1e-7, iters=40):
    x = np.asarray(raw, np.float64).reshape(-1, 1)
    y = np.arange(x.shape[0], dtype=np.float64).reshape(-1, 1)
    th = np.array([[theta0], [0.0]])
    for _ in range(iters):
        H = np.concatenate((1.0 / (th[0, 0] + x), np.ones_like(x)), axis=1)
        r = y - (np.log(th[0, 0] + x) + th[1, 0])
        th = th + np.linalg.inv(H.T @ H) @ H.T @ r
    edges = np.log(th[0, 0] + x).ravel()
    return th.ravel(), edges
