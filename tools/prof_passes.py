"""Run the fused C3 kernels back to back (for rocprofv3 counter collection / kernel timing).

  rocprofv3 --kernel-trace --stats -d DIR -o run --output-format csv -- python3 tools/prof_passes.py
  rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "pass|cfinish" ... -- python3 tools/prof_passes.py
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    from quantized_spectrum_cartography_amd import synthetic
    from quantized_spectrum_cartography_amd.obs import Observations
    from quantized_spectrum_cartography_amd.qmc import FreeSSolver
    I, J, K, R = synthetic.CONFIGS[args.config]
    prob = synthetic.onebit_problem(I, J, K, R, seed=20263, keep_T=False)
    obs = Observations(prob["Y"], prob["Wx"], prob["b"], prob["sigma"], R_hint=R)
    print("obs", obs.stats(), flush=True)
    # the three-launch form (warm spass / cpass dispatches), then the fused form (scfused)
    for fuse in (False, True):
        sol = FreeSSolver(obs, prob["S0"], prob["C0"], hist_cap=args.iters + 4, fuse=fuse)
        sol.run(args.iters)
        torch.cuda.synchronize()
        print("done fuse=%s" % fuse, sol.state(), flush=True)


if __name__ == "__main__":
    main()
