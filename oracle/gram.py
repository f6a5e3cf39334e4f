"""ORACLE (test infrastructure only) — R x R normal equations in numpy fp64.

backup/algorithms/NMF_SPA.m:18-19: C = (inv(Sm'*Sm) * Sm') * Tm, i.e. the R x R Gram of the
selected columns followed by a solve; backup/algorithms/joint_opt_ae.m:404-416: the C-update
as least squares with the [Q'; lambda I] augmentation (non-negativity dropped here).
"""
import numpy as np


def gram(S, w=None):
    S = np.asarray(S, np.float64)
    Sw = S * (np.asarray(w, np.float64)[None, :] if w is not None else 1.0)
    return Sw @ S.T


def rhs(S, T, w=None):
    S = np.asarray(S, np.float64)
    Sw = S * (np.asarray(w, np.float64)[None, :] if w is not None else 1.0)
    return Sw @ np.asarray(T, np.float64).T


def solve(G, B, lam=0.0):
    R = G.shape[0]
    return np.linalg.solve(G + lam * np.eye(R), B)
