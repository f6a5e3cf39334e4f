"""One small persistent-loop run (qsc_scloop) against the launch pairs: prints whether the
loop applied, its fault word and whether S, C and the state agree bit for bit."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    from quantized_spectrum_cartography_amd import synthetic
    from quantized_spectrum_cartography_amd.obs import Observations
    from quantized_spectrum_cartography_amd.qmc import FreeSSolver
    I, J, K, R = (int(x) for x in (sys.argv[1:5] if len(sys.argv) > 4 else (128, 128, 256, 8)))
    n = int(sys.argv[5]) if len(sys.argv) > 5 else 3
    p = synthetic.onebit_problem(I, J, K, R, f=0.1, seed=5, keep_T=False)
    o = Observations(p["Y"], p["Wx"], p["b"], p["sigma"], R_hint=R)
    a = FreeSSolver(o, p["S0"], p["C0"], hist_cap=64, loop=False)
    b = FreeSSolver(o, p["S0"], p["C0"], hist_cap=64, loop=True)
    print("tiles", o.desc.ntiles, "loop applies", b.loop, flush=True)
    a.run(n)
    b.run(n)
    torch.cuda.synchronize()
    sb = b.state()
    print("loop_fault", sb["loop_fault"], flush=True)
    same = all(torch.equal(x, y) for x, y in ((a.S, b.S), (a.C, b.C), (a.mS, b.mS), (a.vS, b.vS)))
    print("bitexact", same, "state equal", a.state() == sb, flush=True)
    return 0 if (same and sb["loop_fault"] == 0) else 1


if __name__ == "__main__":
    sys.exit(main())
