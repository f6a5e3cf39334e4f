"""quantized_spectrum_cartography_amd — MI355X-native one-bit / quantized MLE spectrum cartography.

A from-scratch gfx950 build of the hot path of shresthasagar/quantized_spectrum_cartography:
the probit likelihood of quantized, sparsely sampled radio maps T = sum_r S_r (x) c_r, its
gradients, and the alternating S/C Adam solver (qmc/qmc.ipynb cell 1), plus the qmc.py /
dip.py entry points.  Module map (reference file in parentheses):

  quantization_model      (qmc/quantization_model.py)      linear probit model
  quantization_model_log  (qmc/quantization_model_log.py)  log-domain probit model
  utils                   (qmc/utils.py)                   bin-edge / offset constants
  nlls                    (qmc/nlls.py)                    Gauss-Newton log-offset fit
  qmc                     (qmc/qmc.ipynb, qmc/qmc.py)      alternating solver
  dip                     (qmc/dip.py, empty upstream)     deep-image-prior solver
  obs, fused                                               packed observations, fused passes
  gram                    (backup/algorithms/NMF_SPA.m)    R x R normal equations (MFMA),
                          (joint_opt_ae.m:404-417)         non-negative C-update (NNLS)
  spa                     (backup/algorithms/NMF_SPA.m)    SPA warm start (MFMA K x K Gram)
  maps                    (qmc/generate_map.m,             scalable synthetic radio maps
                           qmc/Shadowing_data.m)
  metrics, synthetic                                       SLF/map NMSE, benchmark inputs
  distributed                                              IJ-/K-slab sharding over RCCL

All arithmetic on the path runs in libqsc_hip.so (HIP, gfx950); there is no CPU fallback.
"""
from . import _lib  # noqa: F401

__version__ = "0.1.0"


def build(force=False):
    from . import _build
    return _build.build(force=force)
