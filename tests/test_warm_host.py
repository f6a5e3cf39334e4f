"""CPU: the de-quantization step of the warm start (warm.dequantize; pure torch, device
agnostic) recovers the noiseless model-domain map from quantized, sampled entries.

Setting: the notebook's log model (qmc/qmc.ipynb :510-537: 4 log bins, sigma = 5, offset
LOG_OFFSET_4, per-entry Bernoulli(0.1) sampling :493) on a smooth synthetic log-map, and the
one-bit linear model of BASELINE.md section 3 (threshold at the median, sigma = range / 4)."""
import numpy as np
import torch

from quantized_spectrum_cartography_amd import warm
from quantized_spectrum_cartography_amd.utils import LOG_OFFSET_4, QUANTIZATION_BOUNDARIES_4_BINS_LOG


def _smooth_field(g, K, N, width):
    x = torch.randn((K, N, N), generator=g)
    return warm._blur(x, width) * width  # smooth, O(1) amplitude


def _quantize(x, b, sigma, g):
    xn = x + sigma * torch.randn(x.shape, generator=g)
    Y = torch.zeros(x.shape, dtype=torch.int64)
    for i in range(1, len(b) - 1):
        Y[xn > b[i]] = i
    return Y


def test_dequantize_log_model():
    g = torch.Generator().manual_seed(3)
    K, N = 8, 96
    x = -8.0 + 6.0 * _smooth_field(g, K, N, 10.0)       # log T across the bin edges
    b = QUANTIZATION_BOUNDARIES_4_BINS_LOG
    Y = _quantize(x, b, 5.0, g)
    Wx = (torch.rand(x.shape, generator=g) < 0.1).float()
    xh = warm.dequantize(Y, Wx, b, 5.0, width=8.0)
    assert xh.shape == x.shape and torch.isfinite(xh).all()
    err = float(torch.linalg.norm(xh - x) / torch.linalg.norm(x))
    assert err < 0.15, err                                # NMSE_LOG of the estimate
    c = np.corrcoef(xh.flatten().numpy(), x.flatten().numpy())[0, 1]
    assert c > 0.75, c


def test_dequantize_onebit_model():
    g = torch.Generator().manual_seed(4)
    K, N = 6, 80
    x = 1.0 + 0.3 * _smooth_field(g, K, N, 10.0)
    thr = float(x.median())
    sigma = float(x.max() - x.min()) / 4
    b = [0.0, thr, float(x.max())]
    Y = _quantize(x, b, sigma, g)
    Wx = (torch.rand(x.shape, generator=g) < 0.1).float()
    xh = warm.dequantize(Y, Wx, b, sigma, width=6.0)
    c = np.corrcoef(xh.flatten().numpy(), x.flatten().numpy())[0, 1]
    assert c > 0.6, c
    # no sampled entry at all -> the estimate stays finite (clipped probabilities)
    xz = warm.dequantize(Y, torch.zeros_like(Wx), b, sigma)
    assert torch.isfinite(xz).all()
