"""Timeline of one persistent-loop iteration (qsc_scpass_loop) from a QSC_DIAG_STAMPS build
(diagnostic only): the tail of body n-2 (drain, ticket, group record) and the head + body of
body n-1, per wave, on the 100 MHz realtime clock, relative to the first wave that ended body
n-2.

  python -c "from quantized_spectrum_cartography_amd import _build as b; \\
      b.build(out='variants/libqsc_stamps.so', extra_flags=['-DQSC_DIAG_STAMPS=1'])"
  QSC_LIB_PATH=variants/libqsc_stamps.so python tools/stamps_loop.py [n]
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
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    I, J, K, R = synthetic.CONFIGS["c3"]
    prob = synthetic.onebit_problem(I, J, K, R, f=0.1, seed=20263, keep_T=False)
    obs = Observations(prob["Y"], prob["Wx"], prob["b"], prob["sigma"], R_hint=R)
    sol = FreeSSolver(obs, prob["S0"], prob["C0"], hist_cap=64, loop=True)
    assert sol.loop
    sol.run(10)
    e = sol.engine
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    e.scpass_loop(sol.S, sol.C, sol.mS, sol.vS, sol.adam_s, sol.lambda_s, sol.mC, sol.vC,
                  sol.adam_c, sol.lambda_c, n, record=False)
    ev1.record()
    torch.cuda.synchronize()
    us = ev0.elapsed_time(ev1) * 1e3
    nw = 4096 * 32
    buf = (ctypes.c_ulonglong * nw)()
    assert _lib.lib().qsc_diag_stamps(buf, nw) == 0
    st = np.frombuffer(buf, dtype=np.uint64).reshape(4096, 32).astype(np.int64)
    st = st[st[:, 20] > 0]
    r0 = st[:, 20].min()
    q = lambda x: "p0 %6.2f p10 %6.2f p50 %6.2f p90 %6.2f max %6.2f us" % tuple(
        np.percentile(np.asarray(x, dtype=np.float64) / 100.0, [0, 10, 50, 90, 100]))
    print("loop of %d bodies: %.1f us (event) = %.2f us per body; waves %d" % (
        n, us, us / n, len(st)))
    print("tail of body n-2 (times from the first wave's body end):")
    print("  body end      ", q(st[:, 20] - r0))
    print("  stores drained", q(st[:, 21] - st[:, 20]))
    print("  ticket taken  ", q(st[:, 22] - st[:, 21]))
    last = st[:, 23] > 0
    if last.any():
        print("  group records ", q(st[last, 23] - st[last, 22]), "(%d waves)" % last.sum())
        print("  records at    ", q(st[last, 23] - r0))
    print("head of body n-1:")
    print("  entry         ", q(st[:, 17] - r0))
    print("  wait over     ", q(st[:, 18] - r0))
    print("  C-step done   ", q(st[:, 19] - st[:, 18]))
    print("body n-1:")
    print("  start         ", q(st[:, 28] - r0))
    print("  end           ", q(st[:, 29] - r0))
    print("  duration      ", q(st[:, 29] - st[:, 28]))
    print("period (last body end - last body n-2 end): %.2f us" % (
        (st[:, 29].max() - st[:, 20].max()) / 100.0))


if __name__ == "__main__":
    main()
