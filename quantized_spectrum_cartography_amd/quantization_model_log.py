"""Log-domain probit quantization model — drop-in for qmc/quantization_model_log.py.

Observations are quantized in the log domain, log(X + offset) + noise; prob_probit uses the
raw (unclamped) edges.  The default offset is LOG_OFFSET_7_ADJUSTED as in the reference
(qmc/quantization_model_log.py:7).
"""
from ._model import (DeterministicCost, F_probit, F_sigmoid, NMSE, NMSE_LOG,  # noqa: F401
                     NegLikelihood, dither_probit, dither_sigmoid,
                     get_quantized_obs_from_ordinal, get_tensor, map_nmse, outer)
from ._model import prob_probit as _prob_probit
from ._model import quantize as _quantize
from .utils import LOG_OFFSET_7_ADJUSTED as LOG_OFFSET


def quantize(X, noise_std, bin_boundaries, offset=LOG_OFFSET, noise=None):
    """Y = Q(log(X + offset) + E) (qmc/quantization_model_log.py:9-21)."""
    return _quantize(X, noise_std, bin_boundaries, offset=offset, log_model=True, noise=noise)


def prob_probit(Y, X_hat, bin_boundaries, noise_std):
    """Phi(U - X) - Phi(W - X) on raw edges (qmc/quantization_model_log.py:23-41)."""
    return _prob_probit(Y, X_hat, bin_boundaries, noise_std, log_model=True)
