"""SPA warm start: backup/algorithms/NMF_SPA.m on the GPU (libqsc_hip.so: qsc_syrk, qsc_spa).

Reference semantics (MATLAB, text only):
  NMF_SPA.m:1-29   [C, Sm] = NMF_SPA(T, R): Tm = T' (pixels x bins) is column-sum normalised,
                   SPA (NMF_SPA.m:31-56) picks R columns = frequency bins where one emitter
                   dominates, C = (inv(Sm'Sm) Sm' Tm)' on the un-normalised data, then
                   ColumnPositive, C(C<0) = 0, unit-norm columns (ColumnNormalization) with
                   the removed norms d moved onto Sm.
  joint_opt_ae.m:211-247  the same on the sampled pixels Tm(:, Ov) (here: the pixel mask w).
The two helpers ColumnSumNormalization / ColumnPositive are not in the reference tree; they are
taken as "divide each column by its sum" and "negate a column whose sum is negative".

The data term is the K x K Gram (T w) T^T on the f32 MFMA; SPA then runs in Gram form (no
residual matrix), and the C fit reads G[sel, sel] and G[sel, :] of the same Gram.
"""
import torch

from . import _lib
from ._model import _dev, _ws


def syrk(T, w=None):
    """G = (T w) T^T for T (K, P): the K x K Gram over the (masked) pixels."""
    Td = _dev(T.detach().to(torch.float32)).reshape(T.shape[0], -1)
    K, P = Td.shape
    wd = _dev(w.detach().to(torch.float32)).reshape(P) if w is not None else None
    G = torch.empty((K, K), dtype=torch.float32, device=Td.device)
    ws = _ws(_lib.lib().qsc_syrk_workspace_bytes(K, P), Td.device)
    _lib.call("qsc_syrk", _lib.ptr(Td), _lib.ptr(wd), K, P, _lib.ptr(G), _lib.ptr(ws),
              ws.numel(), _lib.stream())
    return G


def spa_init(T, R, w=None, return_gram=False):
    """SPA factors of T (K, P) [or (K, I, J)] restricted to the pixel mask w (P,) (nonzero =
    sampled).  Returns (C (R, K), S (R, P), sel (list of picked bins)); C has unit-norm
    non-negative rows, S = mask * T[sel] * d.  Fewer than R bins are picked when the residual
    vanishes (the extra rows of C and S are zero)."""
    K = T.shape[0]
    Td = _dev(T.detach().to(torch.float32)).reshape(K, -1)
    P = Td.shape[1]
    if not 1 <= R <= min(K, _lib.QSC_MAX_R):
        raise ValueError("R must be in 1..%d" % min(K, _lib.QSC_MAX_R))
    wd = _dev(w.detach().to(torch.float32)).reshape(P) if w is not None else None
    dev = Td.device
    sel = torch.empty(R, dtype=torch.int32, device=dev)
    cnt = torch.empty(1, dtype=torch.int32, device=dev)
    C = torch.empty((R, K), dtype=torch.float32, device=dev)
    S = torch.empty((R, P), dtype=torch.float32, device=dev)
    G = torch.empty((K, K), dtype=torch.float32, device=dev) if return_gram else None
    ws = _ws(_lib.lib().qsc_spa_workspace_bytes(K, P, R), dev)
    _lib.call("qsc_spa", _lib.ptr(Td), _lib.ptr(wd), K, P, R, _lib.ptr(sel), _lib.ptr(cnt),
              _lib.ptr(C), _lib.ptr(S), _lib.ptr(G), _lib.ptr(ws), ws.numel(), _lib.stream())
    n = int(cnt.item())
    out = (C, S, sel[:n].tolist())
    return out + (G,) if return_gram else out


def NMF_SPA(T, R):
    """MATLAB-shaped NMF_SPA(T, R) (backup/algorithms/NMF_SPA.m:1): T (K, N) -> (C (K, R),
    Sm (R, N))."""
    C, S, _ = spa_init(T, R)
    return C.t().contiguous(), S
