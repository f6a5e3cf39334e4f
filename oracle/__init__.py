"""ORACLE — test infrastructure only.

CPU restatement of the reference's hot path (shresthasagar/quantized_spectrum_cartography,
qmc/quantization_model{,_log}.py and the alternating solver of qmc/qmc.ipynb cell 1), used as
the checker for the HIP path and as the timed CPU baseline of bench.py.  Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg may import it; the product package
quantized_spectrum_cartography_amd never does, and has no CPU fallback.

Pinning: reference_ops.py / solver.py are pinned bit-for-bit against golden vectors generated
by importing the reference itself (tools/make_golden.py -> tests/golden/*.npz; checked by
tests/test_oracle_golden.py).  explicit.py (closed-form gradients, numpy fp64) is pinned
against reference_ops' autograd to 1e-6, and nlls.py against the reference's qmc/utils.py
constants.

Modules:
  reference_ops  torch-CPU, op-for-op restatement of the reference functions (+ autograd)
  solver         the alternating free-S / fixed-generator loop in the reference formulation
  explicit       numpy fp64 closed-form NLL, dS, dC over observed entries; Adam step
  nlls           Gauss-Newton log-offset fit (qmc/nlls.py)
  gram           R x R normal equations / regularised least squares (NMF_SPA.m, joint_opt_ae.m)
"""
