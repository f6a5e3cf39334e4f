"""Bin-edge design on the host: the Gauss-Newton log-offset fit of qmc/nlls.py and the
equal-count edges of qmc/utils.py:57-74.

qmc/nlls.py fits y = log(f + x) + c to raw bin edges x against y = 0..n-1 (equally spaced
log-domain edges): H = [1/(f + x), 1], forty updates theta += (H^T H)^-1 H^T (y - h(theta))
from theta = (1e-7, 0) (nlls.py:25-37).  Its outputs are the `*_ADJUSTED` edges and offsets of
qmc/utils.py:43-51.  Two parameters and <= 256 edges: microseconds of float64 work, so it stays
on the host (numpy), exactly as in the reference.
"""
import numpy as np

from .utils import find_boundaries


def fit_log_offset(raw_edges, theta0=1e-7, iters=40):
    """Return (offset f, shift c, log-domain edges log(f + x)) for raw edges x (qmc/nlls.py)."""
    x = np.asarray(raw_edges, np.float64).reshape(-1, 1)
    if x.shape[0] < 2:
        raise ValueError("need at least two bin edges")
    y = np.arange(x.shape[0], dtype=np.float64).reshape(-1, 1)
    th = np.array([[float(theta0)], [0.0]])
    H = np.concatenate((1.0 / (th[0, 0] + x), np.ones_like(x)), axis=1)
    for _ in range(iters):
        r = y - (np.log(th[0, 0] + x) + th[1, 0])
        th = th + np.linalg.inv(H.T @ H) @ H.T @ r
        H = np.concatenate((1.0 / (th[0, 0] + x), np.ones_like(x)), axis=1)
    # the reference prints h(theta) - theta_1 = log(f + x) as the adjusted edges (nlls.py:41)
    return float(th[0, 0]), float(th[1, 0]), np.log(th[0, 0] + x).ravel()


def design_log_bins(samples, num_bins=8, theta0=1e-7, iters=40):
    """Equal-count raw edges of `samples` (qmc/utils.py:57-74), then their log-offset fit.

    Returns (log_edges, offset, raw_edges, raw_sd): use log_edges / offset as the
    bin_boundaries / offset of the log model (quantization_model_log)."""
    raw, sd = find_boundaries(samples, num_bins=num_bins)
    f, _, edges = fit_log_offset(raw, theta0, iters)
    return edges.tolist(), f, raw, sd
