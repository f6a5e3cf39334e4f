"""Persistent fused loop (qsc_scpass_loop) against the launch pairs: bit-exactness of S, C,
moments and state after n iterations, the fault word, and the replay time per iteration of
both forms (hipGraph of the same run, HIP events).

  python tools/probe/loop_probe.py [I J K R n]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def timed(sol, n, reps=3):
    sol.prepare(n)
    best = None
    for _ in range(reps):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        sol.run(n, use_graph=True)
        e1.record()
        e1.synchronize()
        t = e0.elapsed_time(e1) * 1e3 / n
        best = t if best is None else min(best, t)
    return best


def main():
    from quantized_spectrum_cartography_amd import synthetic
    from quantized_spectrum_cartography_amd.obs import Observations
    from quantized_spectrum_cartography_amd.qmc import FreeSSolver
    I, J, K, R = (int(x) for x in (sys.argv[1:5] if len(sys.argv) > 4 else (512, 512, 256, 8)))
    n = int(sys.argv[5]) if len(sys.argv) > 5 else 5
    p = synthetic.onebit_problem(I, J, K, R, f=0.1, seed=5, keep_T=False)
    tile = int(os.environ.get("LOOP_TILE", "0")) or None
    o = Observations(p["Y"], p["Wx"], p["b"], p["sigma"], R_hint=R, tile=tile)
    a = FreeSSolver(o, p["S0"], p["C0"], hist_cap=4096, loop=False)
    b = FreeSSolver(o, p["S0"], p["C0"], hist_cap=4096, loop=True)
    print("tiles", o.desc.ntiles, "loop applies", b.loop, flush=True)
    if not b.loop:
        return 1
    a.run(n)
    b.run(n)
    torch.cuda.synchronize()
    sb = b.state()
    arr, grp = b.engine.loop_counters()
    print("fused_fault", sb["fused_fault"], "arrivals", arr, "expected", (n - 1) * o.desc.ntiles,
          "groups", grp, "expected", (n - 1) * min(o.desc.ntiles, 16), flush=True)
    same = all(torch.equal(x, y) for x, y in ((a.S, b.S), (a.C, b.C), (a.mS, b.mS), (a.vS, b.vS),
                                              (a.mC, b.mC), (a.vC, b.vC)))
    print("bitexact", same, "state equal", a.state() == sb,
          "hist equal", torch.equal(a.engine.hist[:4 * n], b.engine.hist[:4 * n]), flush=True)
    if not same or sb["fused_fault"]:
        return 1
    for m in (20, 200):
        ta = timed(a, m)
        tb = timed(b, m)
        print("iterations %d: launch pairs %.2f us/iter, persistent loop %.2f us/iter, fault %d" % (
            m, ta, tb, b.state()["fused_fault"]), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
