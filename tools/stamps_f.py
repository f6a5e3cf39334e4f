"""Phase timeline of the fused S-step + C-pass launch (qsc_scpass) from a QSC_DIAG_STAMPS build
(diagnostic only):

  python -c "from quantized_spectrum_cartography_amd import _build as b; \
      b.build(out='variants/libqsc_stamps.so', extra_flags=['-DQSC_DIAG_STAMPS=1'])"
  QSC_LIB_PATH=variants/libqsc_stamps.so python tools/stamps_f.py
"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from quantized_spectrum_cartography_amd import _lib, synthetic
    from quantized_spectrum_cartography_amd.obs import Observations
    from quantized_spectrum_cartography_amd.qmc import FreeSSolver
    I, J, K, R = synthetic.CONFIGS["c3"]
    prob = synthetic.onebit_problem(I, J, K, R, f=0.1, seed=20263, keep_T=False)
    obs = Observations(prob["Y"], prob["Wx"], prob["b"], prob["sigma"], R_hint=R)
    sol = FreeSSolver(obs, prob["S0"], prob["C0"], hist_cap=64)
    sol.run(10)
    e = sol.engine
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    e.scpass(sol.S, sol.C, sol.mS, sol.vS, sol.adam_s, sol.lambda_s)
    ev1.record()
    torch.cuda.synchronize()
    us = ev0.elapsed_time(ev1) * 1e3
    n = 4096 * 32
    buf = (ctypes.c_ulonglong * n)()
    assert _lib.lib().qsc_diag_stamps(buf, n) == 0
    st = np.frombuffer(buf, dtype=np.uint64).reshape(4096, 32).astype(np.int64)
    st = st[st[:, 0] > 0]
    r0 = st[:, 28].min()
    mt = (st[:, 31] - st[:, 0]).astype(np.float64)
    rt = (st[:, 29] - st[:, 28]).astype(np.float64)
    ghz = np.median(mt / rt) * 0.1
    pu = lambda x: "p0 %6.2f p10 %6.2f p50 %6.2f p90 %6.2f max %6.2f us" % tuple(
        np.percentile(x / 100.0, [0, 10, 50, 90, 100]))
    pc = lambda x: "p10 %6.2f p50 %6.2f p90 %6.2f max %6.2f us" % tuple(
        np.percentile(x / (ghz * 1e3), [10, 50, 90, 100]))
    print("scfused %.1f us (event), waves %d, span %.1f us (realtime), clock %.2f GHz" % (
        us, len(st), (st[:, 29].max() - r0) / 100.0, ghz))
    print("  start      ", pu(st[:, 28] - r0))
    print("  end        ", pu(st[:, 29] - r0))
    print("  staging    ", pc(st[:, 1] - st[:, 0]))
    w = np.arange(len(st)) % 16  # wave in workgroup (rows are wg-major: tile * 16 + wave)
    for nm, m in (("early", w < 4), ("late", w >= 4)):
        print("   %-5s C^T rows written" % nm, pc(st[m, 10] - st[m, 0]))
        print("   %-5s barrier passed  " % nm, pc(st[m, 1] - st[m, 10]))
    print("  tile start -> C^T reads issued", pc(st[:, 13] - st[:, 0]))
    print("  C^T reads issued -> staging starts", pc(st[:, 14] - st[:, 13]))
    print("  staging starts -> C^T rows written", pc(st[:, 10] - st[:, 14]))
    print("  start->C^T (realtime, vs grid start)", pu(st[:, 28] - r0 + (st[:, 10] - st[:, 0]) / ghz * 0.1))
    if (st[:, 12] > 0).any():
        m = st[:, 12] > 0
        print("  1st data   ", pc(st[m, 12] - st[m, 1]))
    print("  S-step     ", pc(st[:, 2] - st[:, 1]))
    print("  tile wait  ", pc(st[:, 3] - st[:, 2]))
    print("  C units    ", pc(st[:, 4] - st[:, 3]))
    print("  part sums  ", pc(st[:, 31] - st[:, 4]))


if __name__ == "__main__":
    main()
