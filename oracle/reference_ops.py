"""ORACLE (test infrastructure only) — torch-CPU restatement of the reference functions.

Op-for-op with the reference so that results are bit-identical on the same torch build
(pinned in tests/test_oracle_golden.py).  CPU tensors only.

  quantize      qmc/quantization_model.py:8-20        qmc/quantization_model_log.py:9-21
  prob_probit   qmc/quantization_model.py:22-39       qmc/quantization_model_log.py:23-41
  F_probit      qmc/quantization_model.py:57-61       qmc/quantization_model_log.py:67-71
  outer         qmc/quantization_model.py:70-77
  get_tensor    qmc/quantization_model.py:79-86
  NMSE          qmc/quantization_model.py:88-92
  NMSE_LOG      qmc/quantization_model_log.py:104-111
  mid_bin       qmc/quantization_model_log.py:43-51
  bce_probit    qmc/quantization_model.py:97-113
  masked_nll    qmc/qmc.ipynb :571-572 (log(T_hat + offset), -sum(Wx * log P))
  dowjons_cost  qmc/qmc_dowjons.ipynb :138-142 (torch.norm(Wx*(log(T_hat+offset)-Obs))**2)
"""
import numpy as np
import torch

SQRT2_REF = 1.414213  # the reference's truncated constant, kept verbatim


def F_probit(y, std):
    return 0.5 * (1 + torch.erf(y / (std * SQRT2_REF)))


def quantize(X, noise_std, b, offset=None, log_model=False, noise=None):
    """Bin index of the noisy observation; later bins overwrite earlier ones."""
    if noise is None:
        noise = torch.randn(X.shape)
    base = torch.log(X + offset) if log_model else X
    x = base + noise * noise_std
    edges = torch.as_tensor(b, dtype=torch.float32).clone()
    edges[-1] = np.inf
    Y = torch.zeros(X.shape)
    for i in range(1, len(edges) - 1):
        Y[(edges[i] < x) & (x <= edges[i + 1])] = i
    return Y.long()


def prob_probit(Y, X_hat, b, noise_std, log_model=False):
    edges = torch.as_tensor(b, dtype=torch.float32).clone()
    if not log_model:
        edges[0] = -100000
        edges[-1] = 100000
    lo, hi = edges[Y], edges[Y + 1]
    return F_probit(hi - X_hat, noise_std) - F_probit(lo - X_hat, noise_std)


def outer(mat, vec):
    out = torch.zeros((*vec.shape, *mat.shape), dtype=torch.float32)
    for k in range(len(vec)):
        out[k, :, :] = mat * vec[k]
    return out


def get_tensor(S, C):
    """sum_r outer(S[r,0], C[r]) with the reference's accumulation (0 + first term, then +=)."""
    acc = 0
    for r in range(C.shape[0]):
        acc += outer(S[r, 0, :, :], C[r, :])
    return acc


def NMSE(T, T_target):
    return torch.norm(T - T_target, "fro") / torch.norm(T_target, "fro")


def NMSE_LOG(T, T_target, offset):
    a, b = torch.log(T + offset), torch.log(T_target + offset)
    return torch.norm(a - b, "fro") / torch.norm(b, "fro")


def mid_bin(Y, b):
    edges = torch.as_tensor(b, dtype=torch.float32).clone()
    return (edges[Y] + edges[Y + 1]) / 2.0


def bce_probit(T_sample, T_target, mean, std):
    return torch.nn.BCELoss()(F_probit(T_sample - mean, std), T_target)


def masked_nll(S, C, Y, Wx, b, noise_std, offset=0.0, log_model=False):
    """-sum(Wx * log(prob_probit(Y, T_hat, b, std))) with T_hat = get_tensor(S, C)."""
    T_hat = get_tensor(S, C).unsqueeze(1)
    if log_model:
        T_hat = torch.log(T_hat + offset)
    return -torch.sum(Wx * torch.log(prob_probit(Y, T_hat, b, noise_std, log_model)))


def dowjons_cost(S, C, Obs, Wx, offset=0.0, log_model=True):
    """torch.norm(Wx*(T_hat-Obs))**2 with T_hat = log(get_tensor(S, C) + offset)
    (qmc/qmc_dowjons.ipynb :138-142; Obs = mid_bin(Y, b), :114)."""
    T_hat = get_tensor(S, C).unsqueeze(1)
    if log_model:
        T_hat = torch.log(T_hat + offset)
    return torch.norm(Wx * (T_hat - Obs)) ** 2
