"""R x R normal equations on the MFMA (libqsc_hip.so: qsc_gram, qsc_gram_rhs, qsc_chol_solve).

Reference semantics (MATLAB, backup/algorithms):
  NMF_SPA.m:18-19        C = (inv(Sm'*Sm)*Sm') * Tm         (pseudo-inverse C-fit)
  joint_opt_ae.m:404-416 C-update as ridge least squares with [Q'; lambda I] rows
Here S is (R, P) and T is (K, P); the contractions over the P = I*J pixels run as f32 MFMA
(v_mfma_f32_16x16x4_f32) and the R x R system is solved by a Cholesky factorisation on the GPU.
"""
import torch

from . import _lib
from ._model import _dev, _ws


def gram(S, w=None):
    """G = (S * w) S^T, (R, R)."""
    R = S.shape[0]
    Sd = _dev(S.detach().to(torch.float32)).reshape(R, -1)
    P = Sd.shape[1]
    wd = _dev(w.detach().to(torch.float32)).reshape(P) if w is not None else None
    G = torch.empty((R, R), dtype=torch.float32, device=Sd.device)
    ws = _ws(_lib.lib().qsc_gram_workspace_bytes(R, P, R), Sd.device)
    _lib.call("qsc_gram", _lib.ptr(Sd), _lib.ptr(wd), R, P, _lib.ptr(G), _lib.ptr(ws), ws.numel(),
              _lib.stream())
    return G


def cross(S, T, w=None):
    """B = (S * w) T^T, (R, K): S (R, P), T (K, P)."""
    R = S.shape[0]
    Sd = _dev(S.detach().to(torch.float32)).reshape(R, -1)
    P = Sd.shape[1]
    Td = _dev(T.detach().to(torch.float32)).reshape(-1, P)
    K = Td.shape[0]
    wd = _dev(w.detach().to(torch.float32)).reshape(P) if w is not None else None
    B = torch.empty((R, K), dtype=torch.float32, device=Sd.device)
    ws = _ws(_lib.lib().qsc_gram_workspace_bytes(R, P, K), Sd.device)
    _lib.call("qsc_gram_rhs", _lib.ptr(Sd), _lib.ptr(Td), _lib.ptr(wd), R, P, K, _lib.ptr(B),
              _lib.ptr(ws), ws.numel(), _lib.stream())
    return B


def chol_solve(G, B, lam=0.0):
    """X = (G + lam I)^-1 B (Cholesky; NaN output if G + lam I is not positive definite)."""
    R, K = B.shape
    Gd = _dev(G.to(torch.float32))
    Bd = _dev(B.to(torch.float32))
    X = torch.empty_like(Bd)
    _lib.call("qsc_chol_solve", _lib.ptr(Gd), _lib.ptr(Bd), R, K, float(lam), _lib.ptr(X),
              _lib.stream())
    return X


def ls_spectra(S, T, w=None, lam=0.0):
    """Least-squares power spectra C (R, K) for fixed S: argmin ||T - C^T S||^2 + lam ||C||^2."""
    return chol_solve(gram(S, w), cross(S, T, w), lam)


def nnls(G, B, lam=0.0):
    """X (R, K) with X[:, k] = argmin_{x >= 0} x^T (G + lam I) x / 2 - B[:, k]^T x (HIP)."""
    R, K = B.shape
    Gd = _dev(G.to(torch.float32))
    Bd = _dev(B.to(torch.float32))
    X = torch.empty_like(Bd)
    _lib.call("qsc_nnls", _lib.ptr(Gd), _lib.ptr(Bd), R, K, float(lam), _lib.ptr(X),
              _lib.stream())
    return X


def nnls_spectra(Q, Y, lam=0.0, w=None):
    """Non-negative C-update of backup/algorithms/joint_opt_ae.m:404-417.

    Q (R, P): spatial factors at the sampled pixels (Sm*W); Y (K, P): the data there (Tm*W).
    For every bin k, c_k = lsqnonneg([Q'; lam I], [Y(k,:)'; 0]); returns C (R, K) (the
    reference stacks the c_k' as rows of a K x R matrix).  Normal equations on the MFMA Gram,
    Lawson-Hanson active set per bin on the GPU."""
    return nnls(gram(Q, w), cross(Q, Y, w), float(lam) ** 2)
