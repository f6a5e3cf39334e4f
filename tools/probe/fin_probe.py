"""One small fused-finish run (qsc_scpass_fin) against the launch pairs: prints whether it
applied, the state's fault word and whether S, C and the state agree bit for bit."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    from quantized_spectrum_cartography_amd import synthetic
    from quantized_spectrum_cartography_amd.obs import Observations
    from quantized_spectrum_cartography_amd.qmc import FreeSSolver
    I, J, K, R = (int(x) for x in (sys.argv[1:5] if len(sys.argv) > 4 else (192, 192, 256, 8)))
    n = int(sys.argv[5]) if len(sys.argv) > 5 else 3
    p = synthetic.onebit_problem(I, J, K, R, f=0.1, seed=5, keep_T=False)
    o = Observations(p["Y"], p["Wx"], p["b"], p["sigma"], R_hint=R, tile=1024)
    a = FreeSSolver(o, p["S0"], p["C0"], hist_cap=64, fin=False)
    b = FreeSSolver(o, p["S0"], p["C0"], hist_cap=64, fin=True)
    print("tiles", o.desc.ntiles, "fused finish applies", b.fin, flush=True)
    a.run(n)
    b.run(n)
    torch.cuda.synchronize()
    sb = b.state()
    print("fused_fault", sb["fused_fault"], flush=True)
    same = all(torch.equal(x, y) for x, y in ((a.S, b.S), (a.C, b.C), (a.mS, b.mS), (a.vS, b.vS)))
    print("bitexact", same, "state equal", a.state() == sb, flush=True)
    return 0 if (same and sb["fused_fault"] == 0 and b.fin) else 1


if __name__ == "__main__":
    sys.exit(main())
