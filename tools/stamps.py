"""Phase timeline of the persistent S-pass from a QSC_DIAG_STAMPS build (diagnostic only).

  QSC_LIB_PATH=variants/libqsc_stamps.so python tools/stamps.py
"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def cpass_timeline(sol, _lib, ctypes):
    e = sol.engine
    torch.cuda.synchronize()
    e.cpass(sol.S, sol.C)
    torch.cuda.synchronize()
    L = _lib.lib()
    n = 4096 * 32
    buf = (ctypes.c_ulonglong * n)()
    assert L.qsc_diag_stamps(buf, n) == 0
    st = np.frombuffer(buf, dtype=np.uint64).reshape(4096, 32).astype(np.int64)
    st = st[st[:, 0] > 0]
    r0 = st[:, 28].min()
    pct = lambda x: "p10 %7.0f p50 %7.0f p90 %7.0f max %7.0f" % tuple(np.percentile(x, [10, 50, 90, 100]))
    pct_us = lambda x: "p0 %6.2f p10 %6.2f p50 %6.2f p90 %6.2f max %6.2f us" % tuple(
        np.percentile(x / 100.0, [0, 10, 50, 90, 100]))
    print("C-pass: waves %d, span %.1f us" % (len(st), (st[:, 29].max() - r0) / 100.0))
    print("  start", pct_us(st[:, 28] - r0))
    print("  end  ", pct_us(st[:, 29] - r0))
    print("  staging+barrier", pct(st[:, 1] - st[:, 0]))
    print("  walk            ", pct(st[:, 2] - st[:, 1]))
    print("  partials+barrier", pct(st[:, 3] - st[:, 2]))
    print("  reduce+slab     ", pct(st[:, 31] - st[:, 3]))
    life = (st[:, 29] - st[:, 28]) / 100.0
    print("  wave lifetime   ", pct_us(st[:, 29] - st[:, 28]))
    print("  concurrency: sum(lifetimes)/span/waves-per-CU-capacity: %.2f waves resident on average per CU" % (
        life.sum() / ((st[:, 29].max() - r0) / 100.0) / 256))


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
    rt = (st[:, 29] - st[:, 28]).astype(np.float64)  # s_memrealtime, 100 MHz
    mt = (st[:, 31] - st[:, 0]).astype(np.float64)
    print("shader clock from memtime/memrealtime: p50 %.2f GHz (wave lifetime p50 %.1f us)" % (
        np.median(mt / rt) * 0.1, np.median(rt) / 100.0))
    print("kernel span by memrealtime: %.1f us" % ((st[:, 29].max() - st[:, 28].min()) / 100.0))
    r0 = st[:, 28].min()
    pct_us = lambda x: "p0 %6.2f p10 %6.2f p50 %6.2f p90 %6.2f max %6.2f us" % tuple(
        np.percentile(x / 100.0, [0, 10, 50, 90, 100]))
    print("start (realtime)", pct_us(st[:, 28] - r0))
    print("end   (realtime)", pct_us(st[:, 29] - r0))
    # per-wave work (sum of its slices' widths) under the static snake schedule
    W = 4096 if False else None
    W = int(live.sum())
    width = sol.obs.s_width.cpu().numpy().astype(np.int64)
    ns = len(width)
    work = np.zeros(W, np.int64)
    for w in range(W):
        t = 0
        while True:
            sidx = t * W + ((W - 1 - w) if (t & 1) else w)
            if sidx >= ns:
                break
            work[w] += width[sidx]
            t += 1
    end_us = (st[:, 29] - r0) / 100.0
    print("work per wave: min %d p50 %d max %d; corr(end, work) %.2f" % (
        work.min(), np.median(work), work.max(), np.corrcoef(end_us, work)[0, 1]))
    xcc = st[:, 27] & 0xF
    for x in np.unique(xcc):
        m = xcc == x
        print("  xcc %d: waves %4d end p50 %.2f max %.2f us, work p50 %d" % (
            x, m.sum(), np.median(end_us[m]), end_us[m].max(), np.median(work[m])))
    hw = st[:, 26]
    simd = (hw >> 4) & 3
    cu = (hw >> 8) & 0xF
    sh = (hw >> 12) & 1
    se = (hw >> 13) & 7
    key = ((xcc * 8 + se) * 2 + sh) * 16 + cu
    pairs = {}
    for idx in range(W):
        pairs.setdefault((key[idx], simd[idx]), []).append(idx)
    sw = np.array([work[v].sum() for v in pairs.values()])
    se_end = np.array([end_us[v].max() for v in pairs.values()])
    print("per-SIMD: waves/SIMD %s; work min %d p50 %d max %d; corr(SIMD end, SIMD work) %.2f" % (
        np.bincount([len(v) for v in pairs.values()]), sw.min(), np.median(sw), sw.max(),
        np.corrcoef(se_end, sw)[0, 1]))
    cpass_timeline(sol, _lib, ctypes)
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
