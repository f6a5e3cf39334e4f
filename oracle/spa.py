"""ORACLE (test infrastructure only) — SPA warm start and NNLS C-update in numpy fp64.

Restates, statement for statement, the MATLAB reference (text only; MATLAB is not in this
image, so these restatements are "parity unpinned" against a run of the reference and are
pinned instead by known-answer tests: on separable data SPA must return the planted pure bins
and NMF_SPA the planted factors up to scale):
  backup/algorithms/NMF_SPA.m:1-29   NMF_SPA(T, R)
  backup/algorithms/NMF_SPA.m:31-56  SPA(X, r)  (explicit residual, max column norm, first index)
  backup/algorithms/NMF_SPA.m:58-75  ColumnNormalization
  backup/algorithms/joint_opt_ae.m:404-417  per-bin lsqnonneg([Q'; lambda I], [y; 0])
ColumnSumNormalization and ColumnPositive are called but not defined in the reference tree;
they are taken as "divide each column by its sum" and "negate a column whose sum is negative".
lsqnonneg is MATLAB's Lawson-Hanson NNLS; scipy.optimize.nnls implements the same algorithm.
"""
import numpy as np
from scipy.optimize import nnls as _nnls


def spa(X, r):
    """NMF_SPA.m:31-56 (0-based indices)."""
    Rm = np.array(X, np.float64, copy=True)
    normR = np.sum(Rm ** 2, axis=0)
    K = []
    i = 0
    while i < r and normR.max() > 1e-12:
        j = int(np.argmax(np.sum(Rm ** 2, axis=0)))  # first index of the max, like MATLAB
        K.append(j)
        u = Rm[:, j] / np.linalg.norm(Rm[:, j])
        Rm = Rm - np.outer(u, u @ Rm)
        normR = np.sum(Rm ** 2, axis=0)
        i += 1
    return K


def column_sum_normalization(X):
    Nz = np.broadcast_to(X.sum(axis=0, keepdims=True), X.shape)
    return X / Nz, Nz


def column_positive(C):
    s = np.where(C.sum(axis=0) < 0, -1.0, 1.0)
    return C * s[None, :]


def column_normalization(X):
    d = np.linalg.norm(X, axis=0)
    Y = np.where(d[None, :] == 0, X, X / np.where(d == 0, 1.0, d)[None, :])
    return Y, d


def nmf_spa(T, R, mask=None):
    """NMF_SPA.m:1-29; T (K, N) [optionally restricted to the pixels where mask != 0, as
    joint_opt_ae.m:185-247 does with Tm(:, Ov)].  Returns C (K, R), Sm (R, N) with zero
    columns at unsampled pixels, and the picked bins."""
    T = np.asarray(T, np.float64)
    N = T.shape[1]
    keep = np.ones(N, bool) if mask is None else (np.asarray(mask) != 0)
    Tm = T[:, keep].T
    Tm_norm, Nz = column_sum_normalization(Tm)
    idx = spa(Tm_norm, R)
    Sm = Tm_norm[:, idx] * Nz[:, idx]
    Tm = Tm_norm * Nz
    C = (np.linalg.inv(Sm.T @ Sm) @ Sm.T) @ Tm
    C = C.T
    Cp = column_positive(C)
    Cp[Cp < 0] = 0
    C, d = column_normalization(Cp)
    Sm = (Sm * d[None, :]).T
    S_full = np.zeros((len(idx), N))
    S_full[:, keep] = Sm
    return C, S_full, idx


def nnls_c_update(Q, Y, lam):
    """joint_opt_ae.m:409-417: for each bin, c = lsqnonneg([Q'; lam I], [Y(k,:)'; 0]);
    returns C (K, R)."""
    Q = np.asarray(Q, np.float64)
    Y = np.asarray(Y, np.float64)
    R = Q.shape[0]
    A = np.vstack([Q.T, lam * np.eye(R)])
    C = np.zeros((Y.shape[0], R))
    for k in range(Y.shape[0]):
        b = np.concatenate([Y[k], np.zeros(R)])
        C[k] = _nnls(A, b)[0]
    return C


def separable_problem(K, P, R, seed=0, pure=None):
    """Planted separable data: C_true (R, K) >= 0 with one pure bin per emitter (only that
    emitter is active there), S_true (R, P) >= 0, T = C_true^T S_true (K, P)."""
    rng = np.random.default_rng(seed)
    C = rng.uniform(0.05, 1.0, (R, K))
    if pure is None:
        pure = rng.choice(K, R, replace=False)
    for r, k in enumerate(pure):
        C[:, k] = 0.0
        C[r, k] = rng.uniform(0.8, 1.2)
    S = rng.uniform(0.0, 1.0, (R, P)) ** 2
    return C, S, C.T @ S, [int(k) for k in pure]
