"""Reconstruction-quality metrics.

map NMSE  ||T_hat - T||_F / ||T||_F (qmc/quantization_model.py:88-92), fused on the GPU
          without materialising T_hat (see _model.map_nmse).
SLF NMSE  not defined by the reference (hard parts): S is recovered only
          up to per-emitter scale and emitter permutation, so each component is normalised to
          unit Frobenius norm (as qmc/generate_map.m:118 normalises the shadowing fields) and
          matched to the truth by the best permutation (Hungarian assignment on the R x R
          cross-Gram, computed with the MFMA kernels of gram.py):
              SLF-NMSE = sum_r ||s_hat_pi(r) - s_r||^2 / sum_r ||s_r||^2   (unit-norm s, s_hat)
"""
import numpy as np
import torch
from scipy.optimize import linear_sum_assignment

from . import gram
from ._model import map_nmse  # noqa: F401


def slf_nmse(S_hat, S_true):
    R = S_true.shape[0]
    Sh = S_hat.detach().reshape(R, -1).to(torch.float32)
    St = S_true.detach().reshape(S_true.shape[0], -1).to(torch.float32)
    Gh = gram.gram(Sh).double().cpu().numpy()
    Gt = gram.gram(St).double().cpu().numpy()
    X = gram.cross(Sh, St).double().cpu().numpy()  # <s_hat_i, s_j>
    nh = np.sqrt(np.maximum(np.diag(Gh), 1e-300))
    nt = np.sqrt(np.maximum(np.diag(Gt), 1e-300))
    cos = X / nh[:, None] / nt[None, :]
    cost = 2.0 - 2.0 * cos  # ||a/|a| - b/|b|||^2
    ri, ci = linear_sum_assignment(cost)
    return float(cost[ri, ci].sum() / R)
