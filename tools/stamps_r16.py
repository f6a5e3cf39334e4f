"""Phase stamps of the rank-16 tile C-pass (c4k K-slab share; diagnostic build, QSC_DIAG_STAMPS):
per wave start, staged, walk end, part-sum barrier and end, in microseconds from the launch's
first stamp; block start times show the launch's rounds.

  QSC_LIB_PATH=variants/libqsc_stamps16.so python tools/stamps_r16.py
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
    I, J, K, R = synthetic.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "c4k"]
    prob = synthetic.onebit_problem(I, J, K, R, f=0.1, seed=20263, keep_T=False)
    obs = Observations(prob["Y"], prob["Wx"], prob["b"], prob["sigma"], R_hint=R)
    sol = FreeSSolver(obs, prob["S0"], prob["C0"], hist_cap=64)
    e = sol.engine
    print("PT %d ntiles %d nks %d" % (obs.desc.PT, obs.desc.ntiles, obs.desc.nks))
    for _ in range(4):  # the stamps of the last launch are kept
        e.cpass_nsq(sol.S, sol.C)
    torch.cuda.synchronize()
    n = 4096 * 32
    buf = (ctypes.c_ulonglong * n)()
    assert _lib.lib().qsc_diag_stamps(buf, n) == 0
    st = np.frombuffer(buf, dtype=np.uint64).reshape(4096, 32).astype(np.int64)
    live = st[:, 0] > 0
    st = st[live]
    ghz = np.median((st[:, 31] - st[:, 0]) / np.maximum(st[:, 29] - st[:, 28], 1)) * 0.1
    us = lambda c: c / (ghz * 1e3)
    t0 = st[:, 0].min()
    print("clock %.2f GHz, waves stamped %d, launch span %.2f us" % (
        ghz, len(st), us(st[:, 31].max() - t0)))
    for name, a, b in (("start (from launch)", None, 0), ("staging", 0, 1), ("walk", 1, 2),
                       ("to part barrier", 2, 3), ("part sums / end", 3, 31),
                       ("whole wave", 0, 31), ("end (from launch)", None, 31)):
        x = us(st[:, b] - (t0 if a is None else st[:, a]))
        print("%-20s p10 %6.2f p50 %6.2f p90 %6.2f max %6.2f" % (name, *np.percentile(x, [10, 50, 90, 100])))
    bs = np.sort(us(st[::8, 0] - t0))
    print("block starts (every 32nd):", " ".join("%.2f" % v for v in bs[::32]))


if __name__ == "__main__":
    main()
