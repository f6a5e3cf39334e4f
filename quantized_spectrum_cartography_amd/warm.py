"""Warm start of the alternating MLE from the quantized samples (SPA on a de-quantized map).

The reference notebook offers a warm start from "the solution of the NMF completion"
(qmc/qmc.ipynb :513-516, commented out; the NMF completion itself is MATLAB, not shipped) and
otherwise starts from zero S, C (:518-520).  This builds the warm start from the data the solver
sees -- quantized, sampled entries -- in two steps:

  1. de-quantize: per frequency bin, the fraction of the nearby sampled entries at or above each
     interior bin edge b_j estimates P(x >= b_j) = Phi((x_hat - b_j) / sigma) of the probit model
     (qmc/quantization_model*.py: x = T (linear) or log(T + offset) (log model) plus N(0, sigma^2)
     noise); inverting it, x_hat = b_j + sigma Phi^-1(p_j), averaged over the edges, is a
     dense estimate of the noiseless x.  "Nearby" = a Gaussian spatial window of `width`
     pixels (sampled-entry weighted), the only prior used.
  2. SPA (backup/algorithms/NMF_SPA.m, spa.spa_init on the MFMA Gram) of T_hat = x_hat
     (linear) or exp(x_hat) - offset (log model) gives C (unit-norm rows) and S.

Host-orchestrated torch ops on the device + the HIP SPA; run once per solve.
"""
import math

import torch
import torch.nn.functional as F

from . import spa


def _blur(x, width):
    """Separable Gaussian blur of (K, I, J) maps, sigma = width pixels, zero padding."""
    r = max(1, int(math.ceil(3 * width)))
    t = torch.arange(-r, r + 1, dtype=x.dtype, device=x.device)
    k = torch.exp(-0.5 * (t / width) ** 2)
    k = k / k.sum()
    y = x.unsqueeze(1)  # (K, 1, I, J)
    y = F.conv2d(y, k.view(1, 1, 1, -1), padding=(0, r))
    y = F.conv2d(y, k.view(1, 1, -1, 1), padding=(r, 0))
    return y.squeeze(1)


def dequantize(Y, Wx, bin_boundaries, noise_std, width=8.0, p_clip=0.02):
    """Dense estimate x_hat (K, I, J) of the noiseless model-domain map from the sampled bin
    indices (see module docstring).  Y, Wx: (K, 1, I, J) or (K, I, J)."""
    K = Y.shape[0]
    I, J = Y.shape[-2], Y.shape[-1]
    dev = Y.device
    Yd = Y.reshape(K, I, J).to(torch.float32)
    Wd = (Wx.reshape(K, I, J) != 0).to(torch.float32) if Wx is not None else torch.ones_like(Yd)
    b = [float(x) for x in (bin_boundaries.tolist() if isinstance(bin_boundaries, torch.Tensor)
                            else bin_boundaries)]
    den = _blur(Wd, width).clamp_min(1e-9)
    est = []
    for j in range(1, len(b) - 1):  # interior edges
        p = _blur(((Yd >= j).to(torch.float32) * Wd), width) / den
        p = p.clamp(p_clip, 1.0 - p_clip)
        est.append(b[j] + float(noise_std) * torch.special.ndtri(p))
    return torch.stack(est).mean(0).to(dev)


def warm_start(Y, Wx, bin_boundaries, noise_std, R, offset=0.0, log_model=False, width=8.0):
    """(S0 (R, 1, I, J), C0 (R, K)) for qmc.solve / dip.solve from the quantized samples."""
    K = Y.shape[0]
    I, J = Y.shape[-2], Y.shape[-1]
    xh = dequantize(Y, Wx, bin_boundaries, noise_std, width)
    T = (torch.exp(xh) - float(offset)).clamp_min(0.0) if log_model else xh.clamp_min(0.0)
    C, S, sel = spa.spa_init(T.reshape(K, I * J), R)
    return S.reshape(R, 1, I, J), C
