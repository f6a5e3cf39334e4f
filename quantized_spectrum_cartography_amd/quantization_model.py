"""Linear-domain probit quantization model — drop-in for qmc/quantization_model.py.

Same names, signatures and semantics as the reference module; the arithmetic runs in the HIP
kernels of libqsc_hip.so (see _model.py for the per-function reference citations).
"""
from ._model import (DeterministicCost, F_probit, F_sigmoid, NMSE, NegLikelihood,  # noqa: F401
                     dither_probit, dither_sigmoid, get_tensor, map_nmse, outer)
from ._model import prob_probit as _prob_probit
from ._model import quantize as _quantize


def quantize(X, noise_std, bin_boundaries, noise=None):
    """Y = Q(X + E), E ~ N(0, noise_std^2) (qmc/quantization_model.py:8-20)."""
    return _quantize(X, noise_std, bin_boundaries, log_model=False, noise=noise)


def prob_probit(Y, X_hat, bin_boundaries, noise_std):
    """Phi(U - X) - Phi(W - X) with b[0] = -1e5, b[-1] = 1e5 (qmc/quantization_model.py:22-39)."""
    return _prob_probit(Y, X_hat, bin_boundaries, noise_std, log_model=False)
