"""Quality runs on generated radio maps (SURVEY.md §8(d) metric 2).

A generate_map-style map (maps.generate_map: Gaussian PSD bumps, path loss x FFT-correlated
log-normal shadowing, unit-norm fields) of 256 x 256 pixels, K = 64 bins, R = 4 emitters is
quantized with the log model as the notebook does (qml.quantize(T, sigma, 4-bin log edges,
LOG_OFFSET_4), qmc/qmc.ipynb :537) and sampled per entry with f = 0.1 (:493).  The free-S solver
(fused launches, one-bit linear model on the same map, as onebit_lowrank.ipynb) and the DIP
solver (log model, the notebook's C5 setting) then run; reported:
SLF-NMSE (unit-norm, permutation-matched), map NMSE (qmc/quantization_model.py:88-92) and the
wall time.  Prints one JSON line.

  python tools/quality_c5.py [--iters 2000] [--dip-iters 200] [--sigma 0.5]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=2000)
    ap.add_argument("--dip-iters", type=int, default=200)
    ap.add_argument("--sigma", type=float, default=5.0)  # qmc/qmc.ipynb :537
    ap.add_argument("--seed", type=int, default=5)
    args = ap.parse_args()
    from quantized_spectrum_cartography_amd import dip, maps, metrics, qmc
    from quantized_spectrum_cartography_amd import quantization_model_log as qml
    from quantized_spectrum_cartography_amd.utils import LOG_OFFSET_4, QUANTIZATION_BOUNDARIES_4_BINS_LOG

    K, R, I = 64, 4, 256
    t0 = time.perf_counter()
    m = maps.generate_map(K, R, shadow_sigma=5.0, Xc=50.0, I=I, J=I, seed=args.seed)
    T, S_true = m["T"], m["S"]
    torch.manual_seed(args.seed)
    Y = qml.quantize(T.cpu(), args.sigma, QUANTIZATION_BOUNDARIES_4_BINS_LOG, LOG_OFFSET_4)
    Wx = torch.bernoulli(torch.full((K, 1, I, I), 0.1))
    t_gen = time.perf_counter() - t0
    b = QUANTIZATION_BOUNDARIES_4_BINS_LOG
    out = {"map": {"K": K, "R": R, "grid": [I, I], "f": 0.1, "model": "log, 4 bins",
                   "sigma": args.sigma, "offset": LOG_OFFSET_4, "gen_s": t_gen,
                   "bins_used": torch.bincount(Y.reshape(-1), minlength=4).tolist()}}

    # free S (onebit_lowrank.ipynb:1230-1291): one-bit linear model on the same map, threshold
    # at the median, sigma = (max - min)/4 (BASELINE.md recipe: keeps P away from 0, so the
    # reference's log P stays finite); S0, C0 = 0.5 rand (zero init is stationary)
    Tc = T.cpu()
    thr = float(Tc.median())
    s1 = (float(Tc.max()) - float(Tc.min())) / 4
    b1 = torch.tensor([0.0, thr, float(Tc.max())])
    torch.manual_seed(args.seed + 2)
    Y1 = qml._quantize(Tc, s1, b1, offset=0.0, log_model=False)
    g = torch.Generator().manual_seed(args.seed + 1)
    S0 = 0.5 * torch.rand(R, 1, I, I, generator=g) / I
    C0 = 0.5 * torch.rand(R, K, generator=g)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    res = qmc.solve(Y1.unsqueeze(1), Wx, b1, s1, S_init=S0, C_init=C0, max_iter=args.iters,
                    use_graph=True, lr_c=1e-3, lr_s=2e-6, lambda_c=0.0, lambda_s=0.0)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    out["free_s_onebit"] = {"iters": args.iters, "wall_s": dt, "sigma": s1, "thr": thr,
                            "slf_nmse": metrics.slf_nmse(res.S, S_true),
                            "map_nmse": metrics.map_nmse(res.S, res.C, T),
                            "cost_first": res.costs_s[0], "cost_last": res.costs_s[-1]}
    if args.dip_iters:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        rd = dip.solve(Y.unsqueeze(1), Wx, b, args.sigma, R, offset=LOG_OFFSET_4,
                       max_iter=args.dip_iters)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        out["dip"] = {"iters": args.dip_iters, "wall_s": dt,
                      "slf_nmse": metrics.slf_nmse(rd.S, S_true),
                      "map_nmse": metrics.map_nmse(rd.S, rd.C, T),
                      "cost_first": rd.costs_s[0], "cost_last": rd.costs_s[-1]}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
