"""ORACLE (test infrastructure only) — closed-form likelihood gradients in numpy fp64.

Documents the math the fused HIP passes implement (include/qsc.h) and checks it against the
reference's autograd (reference_ops.masked_nll + backward) to 1e-6.  For every observed entry
e = (k, p) (Wx = 1; qmc/qmc.ipynb :493, :572):
    t = sum_r S[r,p] C[r,k];  x = t  or  log(t + offset)
    a = std * 1.414213;  u = (b[y+1] - x)/a;  w = (b[y] - x)/a       (linear: b[0]=-1e5, b[-1]=1e5)
    P = 0.5 (1 + erf u) - 0.5 (1 + erf w);  nll = -sum log P
    g = (exp(-u^2) - exp(-w^2)) / (a sqrt(pi) P) * (1/(t + offset) if log else 1)
    dS[r,p] = sum_k g C[r,k];  dC[r,k] = sum_p g S[r,p]
Squared ("DowJons") criterion, qmc/qmc_dowjons.ipynb :142: Obs = (b[y] + b[y+1])/2 (raw edges,
qmc/quantization_model_log.py:43-51), r = x - Obs, loss = sum r^2, g = 2 r (1/(t + offset) if log).
"""
import math

import numpy as np
from scipy.special import erf


def edges_of(b, log_model):
    e = np.asarray(b, dtype=np.float64).copy()
    if not log_model:
        e[0], e[-1] = -1e5, 1e5
    return e


def nll_grad(S, C, Y, Wx, b, sigma, offset=0.0, log_model=False):
    """S (R,P), C (R,K), Y (K,P) int, Wx (K,P) 0/1 -> (nll, dS (R,P), dC (R,K)) in fp64."""
    S = np.asarray(S, np.float64)
    C = np.asarray(C, np.float64)
    Y = np.asarray(Y).astype(np.int64)
    Wx = np.asarray(Wx, np.float64)
    e = edges_of(b, log_model)
    T = C.T @ S  # (K, P)
    x = np.log(T + offset) if log_model else T
    a = sigma * 1.414213
    u = (e[Y + 1] - x) / a
    w = (e[Y] - x) / a
    P = 0.5 * (1 + erf(u)) - 0.5 * (1 + erf(w))
    obs = Wx != 0
    with np.errstate(divide="ignore", invalid="ignore"):
        nll = -np.sum(np.log(P[obs]))
        gx = (np.exp(-u * u) - np.exp(-w * w)) / (a * math.sqrt(math.pi) * P)
    g = np.where(obs, gx * (1.0 / (T + offset) if log_model else 1.0), 0.0)
    dS = C @ g          # (R,K)@(K,P)
    dC = S @ g.T        # (R,P)@(P,K)
    return nll, dS, dC


def sq_loss_grad(S, C, Y, Wx, b, offset=0.0, log_model=True):
    """Squared criterion -> (loss, dS (R,P), dC (R,K)) in fp64."""
    S = np.asarray(S, np.float64)
    C = np.asarray(C, np.float64)
    Y = np.asarray(Y).astype(np.int64)
    Wx = np.asarray(Wx, np.float64)
    e = np.asarray(b, dtype=np.float32)
    obs_val = ((e[Y] + e[Y + 1]) / np.float32(2.0)).astype(np.float64)  # fp32 midpoints
    T = C.T @ S
    x = np.log(T + offset) if log_model else T
    r = x - obs_val
    obs = Wx != 0
    loss = float(np.sum(r[obs] ** 2))
    g = np.where(obs, 2.0 * r * (1.0 / (T + offset) if log_model else 1.0), 0.0)
    return loss, C @ g, S @ g.T


def adam_step(p, m, v, g, step, lr, beta1=0.9, beta2=0.999, eps=1e-8):
    """torch.optim.Adam single-tensor update in fp64 (reference for the fused epilogues)."""
    m = beta1 * m + (1 - beta1) * g
    v = beta2 * v + (1 - beta2) * g * g
    bc1 = 1 - beta1 ** step
    bc2 = 1 - beta2 ** step
    p = p - (lr / bc1) * m / (np.sqrt(v) / math.sqrt(bc2) + eps)
    return p, m, v


# ---------------------------------------------------------------------------------------
# Observed-entries-only form (for the full-size parity tests: the same closed form evaluated
# at the nnz observed (k, p) only, so C3 / C4 passes take seconds, not minutes).
# ---------------------------------------------------------------------------------------
def observed(Y, Wx):
    """(kk, pp, yy) of the observed entries of Y (K,P) under the 0/1 mask Wx (K,P)."""
    Y = np.asarray(Y).reshape(np.asarray(Y).shape[0], -1)
    Wx = np.asarray(Wx).reshape(Y.shape)
    kk, pp = np.nonzero(Wx)
    return kk.astype(np.int64), pp.astype(np.int64), Y[kk, pp].astype(np.int64)


def _scatter(kk, pp, g, K, P):
    from scipy.sparse import csr_matrix
    return csr_matrix((g, (kk, pp)), shape=(K, P))


def _threads():
    import os
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, min(n, 16))


def nll_grad_obs(S, C, obs, b, sigma, offset=0.0, log_model=False, chunk=1 << 20, threads=None):
    """nll_grad restricted to observed entries obs = (kk, pp, yy): identical math (fp64),
    evaluated in chunks of `chunk` entries on a thread pool (numpy releases the GIL in its
    loops), so C4's 27 M entries take seconds.  Each chunk returns its NLL and its per-factor
    bincounts of the gradient (R x P and R x K), summed in chunk order: the result does not
    depend on the thread count, and host memory stays bounded by chunk-sized temporaries plus
    one R x (P + K) partial per chunk (per-factor tasks over all entries held two
    nnz-sized fp64 arrays each, ~7 GB at C4 with 16 threads)."""
    from concurrent.futures import ThreadPoolExecutor
    S = np.asarray(S, np.float64)
    C = np.asarray(C, np.float64)
    kk, pp, yy = obs
    R, P = S.shape
    K = C.shape[1]
    ST, CT = np.ascontiguousarray(S.T), np.ascontiguousarray(C.T)  # row gathers
    e = edges_of(b, log_model)
    a = sigma * 1.414213

    def one(i0):
        k, p, y = kk[i0:i0 + chunk], pp[i0:i0 + chunk], yy[i0:i0 + chunk]
        t = np.einsum("nr,nr->n", ST[p], CT[k])
        x = np.log(t + offset) if log_model else t
        u = (e[y + 1] - x) / a
        w = (e[y] - x) / a
        Pr = 0.5 * (1 + erf(u)) - 0.5 * (1 + erf(w))
        with np.errstate(divide="ignore", invalid="ignore"):
            part = -float(np.sum(np.log(Pr)))
            gx = (np.exp(-u * u) - np.exp(-w * w)) / (a * math.sqrt(math.pi) * Pr)
        g = gx * (1.0 / (t + offset) if log_model else 1.0)
        # dS[r, p] = sum_k g C[r, k];  dC[r, k] = sum_p g S[r, p]  (this chunk's terms)
        dSc = np.stack([np.bincount(p, weights=g * CT[k, r], minlength=P) for r in range(R)])
        dCc = np.stack([np.bincount(k, weights=g * ST[p, r], minlength=K) for r in range(R)])
        return part, dSc, dCc

    nth = threads or _threads()
    nll, dS, dC = 0.0, np.zeros((R, P)), np.zeros((R, K))
    with ThreadPoolExecutor(nth) as ex:
        for part, dSc, dCc in ex.map(one, range(0, kk.shape[0], chunk)):
            nll += part
            dS += dSc
            dC += dCc
    return nll, dS, dC


def explicit_solve(S0, C0, obs, b, sigma, offset=0.0, log_model=False, n_iter=3,
                   lambda_c=100.0, lambda_s=100.0, lr_c=5e-3, lr_s=1e-2):
    """The free-S alternating loop (qmc/qmc.ipynb :559-634 with S as the Adam variable,
    backup/notebooks/onebit_lowrank.ipynb:1230-1236) with closed-form fp64 gradients:
      C-step: g = dC_nll + lambda_c C/||C|| (0 at C = 0, torch's norm backward); Adam(lr_c);
              C[C < 0] = 0
      S-step (at the new C): g = dS_nll + lambda_s S/||S||; Adam(lr_s).
    Returns (S, C, costs_c, costs_s), costs evaluated before each update as the reference's
    cost.item()."""
    S = np.asarray(S0, np.float64).copy()
    C = np.asarray(C0, np.float64).copy()
    mS, vS, mC, vC = (np.zeros_like(S), np.zeros_like(S), np.zeros_like(C), np.zeros_like(C))
    costs_c, costs_s = [], []

    def reg(X, lam):
        n = float(np.linalg.norm(X))
        return lam * n, (lam * X / n if n > 0 else np.zeros_like(X))

    for it in range(1, n_iter + 1):
        nll, _, dC = nll_grad_obs(S, C, obs, b, sigma, offset, log_model)
        rc, gc = reg(C, lambda_c)
        rs, _ = reg(S, lambda_s)
        costs_c.append(nll + rc + rs)
        C, mC, vC = adam_step(C, mC, vC, dC + gc, it, lr_c)
        C = np.maximum(C, 0.0)
        nll, dS, _ = nll_grad_obs(S, C, obs, b, sigma, offset, log_model)
        rc, _ = reg(C, lambda_c)
        rs, gs = reg(S, lambda_s)
        costs_s.append(nll + rc + rs)
        S, mS, vS = adam_step(S, mS, vS, dS + gs, it, lr_s)
    return S, C, costs_c, costs_s
