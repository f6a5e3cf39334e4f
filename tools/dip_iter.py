"""Config 5's DIP iteration on its own (for a rocprofv3 kernel trace of just the solve):

  python tools/dip_iter.py [--iters 200] [--eager]

Builds the C5 problem and dip.solve's default solver (256^2 SizedDecoderDip, Adam on its weights,
lr_c sized to the data), runs `iters` iterations (captured hipGraph chunks after one eager
iteration, or all eager with --eager) and prints the per-iteration wall time.
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--eager", action="store_true")
    ap.add_argument("--benchmark", action="store_true",
                    help="torch.backends.cudnn.benchmark (MIOpen find mode) for the decoder")
    ap.add_argument("--optimize", default="weights", choices=["weights", "z"])
    a = ap.parse_args()
    if a.benchmark:
        torch.backends.cudnn.benchmark = True
    from quantized_spectrum_cartography_amd import dip, synthetic
    prob = synthetic.c5_problem(seed=5)
    sol = dip.solve(prob["Y"], prob["Wx"], prob["b"], prob["sigma"], 4, offset=prob["offset"],
                    log_model=True, lr_c="auto", build_only=True, hist_cap=a.iters + 8,
                    optimize=a.optimize)
    use_graph = not a.eager
    sol.run(2, use_graph=use_graph)
    if use_graph:
        sol.prepare(a.iters)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    sol.run(a.iters, use_graph=use_graph)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print("dip iterations: %d, %.1f us per iteration (%s, optimize %s, benchmark %s), "
          "graph_error %s" % (a.iters, dt / a.iters * 1e6, "graph" if use_graph else "eager",
                              a.optimize, a.benchmark, sol.graph_error))


if __name__ == "__main__":
    main()
