"""Phase timeline of the persistent S-pass from a QSC_DIAG_STAMPS build (diagnostic only).

  QSC_LIB_PATH=variants/libqsc_stamps.so python tools/stamps.py
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
    e.spass(sol.S, sol.C, 1, mS=sol.mS, vS=sol.vS, adam=sol.adam_s, lambda_s=sol.lambda_s)
    ev1.record()
    torch.cuda.synchronize()
    us = ev0.elapsed_time(ev1) * 1e3
    L = _lib.lib()
    n = 4096 * 32
    buf = (ctypes.c_ulonglong * n)()
    rc = L.qsc_diag_stamps(buf, n)
    assert rc == 0, rc
    st = np.frombuffer(buf, dtype=np.uint64).reshape(4096, 32).astype(np.int64)
    live = st[:, 0] > 0
    st = st[live]
    t0 = st[:, 0].min()
    end = st[:, 31].max()
    print("kernel %.1f us (event); waves %d; span %d cycles -> %.2f GHz" % (
        us, len(st), end - t0, (end - t0) / (us * 1e3)))
    rel = st - t0
    pct = lambda x: "p10 %7.0f p50 %7.0f p90 %7.0f max %7.0f" % tuple(np.percentile(x, [10, 50, 90, 100]))
    print("wave start     ", pct(rel[:, 0]))
    print("prologue (C/LDS)", pct(st[:, 1] - st[:, 0]))
    for i in range(9):
        a, b, c = 2 + 3 * i, 3 + 3 * i, 4 + 3 * i
        ok = st[:, c] > 0
        if not ok.any():
            break
        prev = st[ok, 1] if i == 0 else st[ok, 4 + 3 * (i - 1)]
        print("slice %d: n %4d wait-next %s" % (i, ok.sum(), pct(st[ok, a] - prev)))
        print("          walk      %s" % pct(st[ok, b] - st[ok, a]))
        print("          epilogue  %s" % pct(st[ok, c] - st[ok, b]))
    print("wave end       ", pct(rel[:, 31]))
    print("tail (end-last epilogue)", pct(st[:, 31] - st[np.arange(len(st)), 4 + 3 * ((st[:, 5:30:3] > 0).sum(1))]))


if __name__ == "__main__":
    main()
