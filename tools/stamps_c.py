"""Phase timeline of the C-pass from a QSC_DIAG_STAMPS build (diagnostic only).

  QSC_LIB_PATH=variants/libqsc_stamps.so python tools/stamps_c.py [--tile N]
"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tile", type=int, default=0)
    args = ap.parse_args()
    from quantized_spectrum_cartography_amd import _lib, synthetic
    from quantized_spectrum_cartography_amd.obs import Observations
    from quantized_spectrum_cartography_amd.qmc import FreeSSolver
    I, J, K, R = synthetic.CONFIGS["c3"]
    prob = synthetic.onebit_problem(I, J, K, R, f=0.1, seed=20263, keep_T=False)
    obs = Observations(prob["Y"], prob["Wx"], prob["b"], prob["sigma"], R_hint=R,
                       tile=args.tile or None)
    sol = FreeSSolver(obs, prob["S0"], prob["C0"], hist_cap=64)
    sol.run(10)
    e = sol.engine
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    e.cpass(sol.S, sol.C)
    ev1.record()
    torch.cuda.synchronize()
    us = ev0.elapsed_time(ev1) * 1e3
    n = 4096 * 32
    buf = (ctypes.c_ulonglong * n)()
    assert _lib.lib().qsc_diag_stamps(buf, n) == 0
    st = np.frombuffer(buf, dtype=np.uint64).reshape(4096, 32).astype(np.int64)
    st = st[st[:, 0] > 0]
    r0 = st[:, 28].min()
    pu = lambda x: "p0 %6.2f p10 %6.2f p50 %6.2f p90 %6.2f max %6.2f us" % tuple(
        np.percentile(x / 100.0, [0, 10, 50, 90, 100]))
    pc = lambda x: "p10 %7.0f p50 %7.0f p90 %7.0f max %7.0f cyc" % tuple(
        np.percentile(x, [10, 50, 90, 100]))
    print("C-pass %.1f us (event), waves %d, span %.1f us (realtime)" % (
        us, len(st), (st[:, 29].max() - r0) / 100.0))
    print("  start  ", pu(st[:, 28] - r0))
    print("  end    ", pu(st[:, 29] - r0))
    print("  staging", pc(st[:, 1] - st[:, 0]))
    print("  walk   ", pc(st[:, 2] - st[:, 1]))
    has3 = st[:, 3] > 0
    if has3.any():
        print("  sumwait", pc((st[:, 3] - st[:, 2])[has3]))
        print("  tail   ", pc((st[:, 31] - st[:, 3])[has3]))
    mt = (st[:, 31] - st[:, 0]).astype(np.float64)
    rt = (st[:, 29] - st[:, 28]).astype(np.float64)
    print("  clock p50 %.2f GHz; lifetime %s" % (np.median(mt / rt) * 0.1, pu(rt)))


if __name__ == "__main__":
    main()
