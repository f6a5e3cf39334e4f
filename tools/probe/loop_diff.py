"""Where the persistent loop departs from the launch pairs: after c_step + (n - 1) fused bodies
(the pairs: scpass / cfinish; the loop: one qsc_scpass_loop launch, whose end writes C, mC, vC and
qsc_state as the pairs leave them before their last cfinish), every tensor and state field is
compared, with the count and size of the differences.

  python tools/probe/loop_diff.py [R I J K tile n]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__)))), "tests"))


def diff(name, a, b):
    if torch.equal(a, b):
        print("  %-6s equal" % name, flush=True)
        return
    d = (a - b).abs()
    nz = (d > 0).nonzero()
    print("  %-6s DIFF: %d of %d entries, max %.3e; first at %s" % (
        name, int((d > 0).sum()), d.numel(), float(d.max()), nz[:4].tolist()), flush=True)


def main():
    from test_gpu_fused import _random_case
    from quantized_spectrum_cartography_amd.obs import Observations
    from quantized_spectrum_cartography_amd.qmc import FreeSSolver
    args = [int(x) for x in sys.argv[1:7]] if len(sys.argv) > 6 else [8, 192, 192, 256, 1024, 3]
    R, I, J, K, tile, n = args
    d = _random_case(58, R, I, J, K)
    o = Observations(d["Y"], d["Wx"], d["b"], d["sigma"], R_hint=R, tile=tile)
    print("tiles", o.desc.ntiles, "nks", o.desc.nks, flush=True)
    a = FreeSSolver(o, d["S0"], d["C0"], hist_cap=32, loop=False)
    b = FreeSSolver(o, d["S0"], d["C0"], hist_cap=32, loop=True)
    assert b.loop
    a.c_step()
    for _ in range(n - 1):
        a.fused_body()
    # the pairs' last fused_body ended with its cfinish; the loop leaves that one to the caller:
    # compare the loop against the pairs minus that last cfinish -- rerun the pairs to the
    # point before it
    a2 = FreeSSolver(o, d["S0"], d["C0"], hist_cap=32, loop=False)
    a2.c_step()
    for _ in range(n - 2):
        a2.fused_body()
    a2.engine.scpass(a2.S, a2.C, a2.mS, a2.vS, a2.adam_s, a2.lambda_s)
    b.c_step()
    b.engine.scpass_loop(b.S, b.C, b.mS, b.vS, b.adam_s, b.lambda_s, b.mC, b.vC, b.adam_c,
                         b.lambda_c, n - 1)
    torch.cuda.synchronize()
    print("after c_step + %d bodies (before the last cfinish):" % (n - 1), flush=True)
    for nm in ("S", "C", "mS", "vS", "mC", "vC"):
        diff(nm, getattr(a2, nm), getattr(b, nm))
    sa, sb = a2.state(), b.state()
    for k in sa:
        if sa[k] != sb[k]:
            print("  state %s: pairs %r loop %r" % (k, sa[k], sb[k]), flush=True)
    print("  loop counters", b.engine.loop_counters(), flush=True)
    ha, hb = a2.engine.hist[:4 * n].cpu(), b.engine.hist[:4 * n].cpu()
    print("  hist pairs", ha.tolist(), flush=True)
    print("  hist loop ", hb.tolist(), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
