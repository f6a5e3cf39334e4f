"""Per-wave phase stamps of the two-tile fused launch (scfused2_kernel, diagnostic build with
QSC_DIAG_STAMPS): S-step item ends, the arrival waits and C-pass unit spans of tile A and B.

  QSC_CTILE=512 QSC_LIB_PATH=variants/libqsc_stamps.so python tools/stamps_tt.py
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
    print("tile", obs.desc.PT, "ntiles", obs.desc.ntiles)
    sol = FreeSSolver(obs, prob["S0"], prob["C0"], hist_cap=64)
    sol.run(10)
    e = sol.engine
    for _ in range(3):
        e.scpass(sol.S, sol.C, sol.mS, sol.vS, sol.adam_s, sol.lambda_s)
    torch.cuda.synchronize()
    n = 4096 * 32
    buf = (ctypes.c_ulonglong * n)()
    assert _lib.lib().qsc_diag_stamps(buf, n) == 0
    st = np.frombuffer(buf, dtype=np.uint64).reshape(4096, 32).astype(np.int64)
    ghz = np.median((st[:, 31] - st[:, 0]) / np.maximum(st[:, 29] - st[:, 28], 1)) * 0.1
    us = lambda c: c / (ghz * 1e3)
    simd = (st[:, 26] >> 4) & 3
    print("clock %.2f GHz" % ghz)
    nb = 256
    for blk in (0, 1, 100, 255):
        w = np.arange(blk * 16, blk * 16 + 16)
        t0 = st[w, 0].min()
        print("block %d" % blk)
        for sm in range(4):
            for x in w[simd[w] == sm]:
                sl = [us(st[x, j] - t0) for j in range(5, 9) if 0 < st[x, j] - t0 < 10 ** 7]
                print("  simd %d wave %2d: staged %5.2f items %s | S-end %5.2f | A %5.2f-%5.2f | B %5.2f-%5.2f | end %5.2f" % (
                    sm, x - blk * 16, us(st[x, 1] - t0), " ".join("%5.2f" % v for v in sl),
                    us(st[x, 2] - t0), us(st[x, 3] - t0), us(st[x, 4] - t0), us(st[x, 14] - t0),
                    us(st[x, 15] - t0), us(st[x, 31] - t0)))
    ends = []
    for blk in range(nb):
        w = np.arange(blk * 16, blk * 16 + 16)
        t0 = st[w, 0].min()
        ends.append([us(st[w, 2].max() - t0), us(st[w, 3].min() - t0), us(st[w, 4].max() - t0),
                     us(st[w, 14].min() - t0), us(st[w, 15].max() - t0), us(st[w, 31].max() - t0)])
    a = np.array(ends)
    for i, name in enumerate(("S end (last wave)", "C(A) first start", "C(A) last end",
                              "C(B) first start", "C(B) last end", "block end")):
        print("%-18s p10 %.2f p50 %.2f p90 %.2f max %.2f" % (name, *np.percentile(a[:, i], [10, 50, 90, 100])))


if __name__ == "__main__":
    main()
