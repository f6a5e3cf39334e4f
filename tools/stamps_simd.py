"""Per-SIMD view of the fused launch's phase stamps (diagnostic build, QSC_DIAG_STAMPS):
for sample workgroups, each wave's slice ends, S-step end, C-pass start / end, grouped by the
SIMD it ran on (HW_ID), in microseconds from the workgroup's first stamp.

  QSC_LIB_PATH=variants/libqsc_stamps.so python tools/stamps_simd.py
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
    for _ in range(3):  # warm: the stamps of the last launch are kept
        e.scpass(sol.S, sol.C, sol.mS, sol.vS, sol.adam_s, sol.lambda_s)
    torch.cuda.synchronize()
    n = 4096 * 32
    buf = (ctypes.c_ulonglong * n)()
    assert _lib.lib().qsc_diag_stamps(buf, n) == 0
    st = np.frombuffer(buf, dtype=np.uint64).reshape(4096, 32).astype(np.int64)
    ghz = np.median((st[:, 31] - st[:, 0]) / np.maximum(st[:, 29] - st[:, 28], 1)) * 0.1
    us = lambda c: c / (ghz * 1e3)
    simd = (st[:, 26] >> 4) & 3  # HW_ID.SIMD_ID (bits 5:4)
    print("clock %.2f GHz" % ghz)
    agg = []
    for blk in range(256):
        w = np.arange(blk * 16, blk * 16 + 16)
        t0 = st[w, 0].min()
        s_end_blk = st[w, 2].max()
        for sm in range(4):
            ws = w[simd[w] == sm]
            agg.append([us(st[ws, 2].max() - st[ws, 1].min()), us(st[ws, 4].max() - st[ws, 3].min())])
        if blk in (0, 1, 100, 255):
            print("block %d: S end (block) %.2f, kernel-relative" % (blk, us(s_end_blk - t0)))
            for sm in range(4):
                ws = w[simd[w] == sm]
                for x in ws:
                    sl = [us(st[x, j] - t0) for j in range(5, 8) if 0 < st[x, j] - t0 < 10 ** 7]
                    fd = us(st[x, 12] - t0) if st[x, 12] > 0 else float("nan")
                    print("  simd %d wave %2d: staged %5.2f data %5.2f slices %s S-end %5.2f C %5.2f-%5.2f end %5.2f" % (
                        sm, x - blk * 16, us(st[x, 1] - t0), fd, " ".join("%5.2f" % v for v in sl),
                        us(st[x, 2] - t0), us(st[x, 3] - t0), us(st[x, 4] - t0), us(st[x, 31] - t0)))
    t0b = np.array([st[b * 16:(b + 1) * 16, 0].min() for b in range(256)]).repeat(16)
    for name, j in (("C^T written", 10), ("scalars set", 11), ("barrier", 1)):
        x = us(st[:, j] - t0b)
        print("%-12s from block start: p10 %.2f p50 %.2f p90 %.2f max %.2f" % (name, *np.percentile(x, [10, 50, 90, 100])))
    w0 = np.arange(0, 4096, 16)
    print("wave 0 scalars set - C^T written: p50 %.2f us" % np.median(us(st[w0, 11] - st[w0, 10])))
    a = np.array(agg)
    print("per-SIMD S phase span p10/p50/p90 %.2f %.2f %.2f; C phase span %.2f %.2f %.2f" % (
        *np.percentile(a[:, 0], [10, 50, 90]), *np.percentile(a[:, 1], [10, 50, 90])))


if __name__ == "__main__":
    main()
