"""Fused-finish tail timeline (diagnostic build, QSC_DIAG_STAMPS): for the last qsc_scpass_fin
launch, each workgroup's tile end, ticket time and arrival rank, and for the C-finish waiters
the end of the wait and of their C-finish item, in microseconds from the launch's first stamp.

  QSC_LIB_PATH=variants/libqsc_stamps.so python tools/stamps_fin.py
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
    sol = FreeSSolver(obs, prob["S0"], prob["C0"], hist_cap=64, fin=True)
    assert sol.fin
    sol.run(int(os.environ.get("FIN_ITERS", "30")))
    torch.cuda.synchronize()
    n = 4096 * 32
    buf = (ctypes.c_ulonglong * n)()
    assert _lib.lib().qsc_diag_stamps(buf, n) == 0
    st = np.frombuffer(buf, dtype=np.uint64).reshape(4096, 32).astype(np.int64)
    ghz = np.median((st[:, 31] - st[:, 0]) / np.maximum(st[:, 29] - st[:, 28], 1)) * 0.1
    us = lambda c: c / (ghz * 1e3)
    nt = obs.desc.ntiles
    w0 = np.arange(nt) * 16  # wave 0 of each workgroup
    t0 = st[w0, 0].min()
    rank = st[w0, 18]
    tile_end = np.array([st[b * 16:(b + 1) * 16, 31].max() for b in range(nt)])
    ticket = st[w0, 19]
    wait_end = st[w0, 20]
    fin_end = st[w0, 21]
    order = np.argsort(rank)
    print("clock %.2f GHz, tiles %d, state fused_fault %s" % (ghz, nt, sol.state()["fused_fault"]))
    print("first wave start to: tile ends p10 %.2f p50 %.2f p90 %.2f max %.2f" % tuple(
        us(np.percentile(tile_end - t0, [10, 50, 90, 100]))))
    print("ticket after own tile end: p50 %.2f max %.2f" % (us(np.median(ticket - tile_end)),
                                                             us((ticket - tile_end).max())))
    last = ticket.max()
    print("last ticket at %.2f" % us(last - t0))
    nvb = R * obs.desc.nks + 2
    for b in order[-nvb:][::4]:
        print("  rank %3d ticket %.2f wait-end %.2f (+%.2f after last) finish-end %.2f" % (
            rank[b], us(ticket[b] - t0), us(wait_end[b] - t0), us(wait_end[b] - last),
            us(fin_end[b] - t0)))
    we = wait_end[order[-nvb:]]
    fe = fin_end[order[-nvb:]]
    print("waiters: wait-end after last ticket p50 %.2f max %.2f; finish item p50 %.2f max %.2f; "
          "kernel end %.2f" % (us(np.median(we - last)), us((we - last).max()),
                               us(np.median(fe - we)), us((fe - we).max()), us(fe.max() - t0)))


if __name__ == "__main__":
    main()
