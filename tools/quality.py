"""Reconstruction-quality runs (SURVEY.md section 8(d) metric 2).

Prints one JSON line of trajectories (map NMSE every few iterations, qmc/quantization_model.py
:88-92, and the final SLF-NMSE, metrics.slf_nmse):

  c2_free_s   BASELINE.md section 3 recipe at C2 (256 x 256 x 64, R = 4, one-bit probit, thr =
              median, sigma = range/4, f = 0.1, S0, C0 = 0.5 rand, lambda = 100, lr 5e-3 / 1e-2):
              the free-S solver of onebit_lowrank.ipynb :1230-1291 / qmc.ipynb :559-645 on the
              fused launches, the bench's workload at C2 size; map NMSE at log-spaced iterations
              and the best along the path (free S at ~6 one-bit samples per pixel over-fits);
  c2_free_s_f05  the same map sampled at f = 0.5 (onebit_lowrank.ipynb's f).
  c2_*_holdout_stop  the same runs stopped on the NLL of 10 % held-out observations
              (qmc.solve(holdout=0.1)): the stopping rule, without T_true.
  c5_*        a generate_map-style radio map (maps.generate_map: Gaussian PSD bumps, path loss x
              FFT-correlated log-normal shadowing, 256 x 256, K = 64, R = 4) quantized with the log
              model as qmc/qmc.ipynb :537 does (4 log bins, LOG_OFFSET_4, sigma = 5), f = 0.1:
                c5_warm_start  the de-quantized SPA warm start (warm.warm_start);
                c5_dip       the DIP solver from it (dip.solve warm="relative": S = S0
                             exp(D(Z) - D(Z0)), decoder weights optimised at lr 1e-3, C from
                             C0), one run per decoder seed, with the medians
                             (tools/c5_dip_sweep.py, profiles/r05/c5_dip_sweep_*.log);
                c5_dip_cold  the DIP solver from zero C (BN-calibrated decoder), the notebook's
                             cold setting, with the C-step sized to the data (lr_c="auto");
                c5_free_warm_projS_*  free S >= 0 (project_s) from the warm start.

  python tools/quality.py [--c2-iters 4000] [--dip-iters 600]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def traj(res, every):
    return [[every * (i + 1), round(float(v), 5)] for i, v in enumerate(res.nmse)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--c2-iters", type=int, default=4000)
    ap.add_argument("--dip-iters", type=int, default=600)
    ap.add_argument("--seed", type=int, default=5)
    ap.add_argument("--warm-iters", type=int, default=1000)
    ap.add_argument("--warm-width", type=float, default=8.0)
    ap.add_argument("--warm-lr-s", type=float, default=1e-3)
    ap.add_argument("--dip-warm-iters", type=int, default=3000)
    ap.add_argument("--dip-lr-s", type=float, default=1e-3)
    ap.add_argument("--dip-form", default="relative", choices=["residual", "relative"])
    ap.add_argument("--dip-seeds", type=int, nargs="*", default=[5, 6, 7, 8, 9, 10])
    ap.add_argument("--dip-cold-lr-c", default="auto")
    ap.add_argument("--dip-lr-c-scale", type=float, default=1e-2)
    ap.add_argument("--free-lr-scales", type=float, nargs="*", default=[1e-2, 1e-3])
    ap.add_argument("--skip-c2", action="store_true")
    args = ap.parse_args()
    from quantized_spectrum_cartography_amd import dip, maps, metrics, qmc, synthetic
    from quantized_spectrum_cartography_amd import quantization_model_log as qml
    from quantized_spectrum_cartography_amd.utils import LOG_OFFSET_4, QUANTIZATION_BOUNDARIES_4_BINS_LOG
    out = {}

    # ---- C2 free S, BASELINE recipe (f = 0.1) and the same map sampled at f = 0.5 ----
    I, J, K, R = synthetic.CONFIGS["c2"]
    for name, f in (() if args.skip_c2 else (("c2_free_s", 0.1), ("c2_free_s_f05", 0.5))):
        p = synthetic.onebit_problem(I, J, K, R, f=f, seed=20262)
        marks = sorted({int(round(x / 10.0)) * 10 for x in np.geomspace(10, args.c2_iters, 14)})
        t0 = time.perf_counter()
        res = qmc.solve(p["Y"], p["Wx"], p["b"], p["sigma"], S_init=p["S0"], C_init=p["C0"],
                        max_iter=args.c2_iters, use_graph=True, T_true=p["T_true"], nmse_every=10)
        torch.cuda.synchronize()
        tr = [[10 * (i + 1), round(float(v), 5)] for i, v in enumerate(res.nmse)]
        best = min(tr, key=lambda x: x[1])
        init = float(metrics.map_nmse(p["S0"].cuda(), p["C0"].cuda(), p["T_true"]))
        out[name] = {"iters": args.c2_iters, "f": f, "wall_s": time.perf_counter() - t0,
                     "map_nmse_init": init,
                     "map_nmse": [x for x in tr if x[0] in marks],
                     "map_nmse_best": best,
                     "slf_nmse": metrics.slf_nmse(res.S, p["S_true"]),
                     "cost_first": res.costs_s[0], "cost_last": res.costs_s[-1]}
        print(json.dumps({name: [tr[-1], best]}), file=sys.stderr, flush=True)
        # the same run stopped on 10 % held-out observations (qmc.solve(holdout=...)): no
        # knowledge of T_true, the stopping rule the free-S MLE needs at these sample counts
        t0 = time.perf_counter()
        es = qmc.solve(p["Y"], p["Wx"], p["b"], p["sigma"], S_init=p["S0"], C_init=p["C0"],
                       max_iter=args.c2_iters, use_graph=True, holdout=0.1, check_every=10,
                       patience=5)
        torch.cuda.synchronize()
        out[name + "_holdout_stop"] = {
            "holdout": 0.1, "check_every": 10, "patience": 5, "stopped_at": es.iters,
            "best_iter": es.best_iter, "wall_s": time.perf_counter() - t0,
            "map_nmse": float(metrics.map_nmse(es.S, es.C, p["T_true"])),
            "slf_nmse": metrics.slf_nmse(es.S, p["S_true"])}
        print(json.dumps({name + "_holdout_stop": out[name + "_holdout_stop"]}), file=sys.stderr,
              flush=True)
        del p, res, es

    # ---- C5: generated map, log model ----
    K, R, N = 64, 4, 256
    m = maps.generate_map(K, R, shadow_sigma=5.0, Xc=50.0, I=N, J=N, seed=args.seed)
    T, S_true = m["T"], m["S"]
    torch.manual_seed(args.seed)
    Y = qml.quantize(T.cpu(), 5.0, QUANTIZATION_BOUNDARIES_4_BINS_LOG, LOG_OFFSET_4).unsqueeze(1)
    Wx = torch.bernoulli(torch.full((K, 1, N, N), 0.1))
    b = QUANTIZATION_BOUNDARIES_4_BINS_LOG
    out["c5_map"] = {"K": K, "R": R, "grid": [N, N], "f": 0.1, "model": "log, 4 bins",
                     "sigma": 5.0, "offset": LOG_OFFSET_4,
                     "bins_used": torch.bincount(Y.reshape(-1), minlength=4).tolist()}
    if args.dip_iters:
        # the DIP solver from a cold start (zero C, BN-calibrated decoder): the notebook's setting
        every = max(1, args.dip_iters // 12)
        t0 = time.perf_counter()
        rd = dip.solve(Y, Wx, b, 5.0, R, offset=LOG_OFFSET_4, max_iter=args.dip_iters,
                       T_true=T, nmse_every=every,
                       lr_c=(args.dip_cold_lr_c if args.dip_cold_lr_c == "auto"
                             else float(args.dip_cold_lr_c)))
        torch.cuda.synchronize()
        zero = float(metrics.map_nmse(torch.zeros_like(rd.S), rd.C, T, log_offset=LOG_OFFSET_4))
        out["c5_dip_cold"] = {"iters": args.dip_iters, "wall_s": time.perf_counter() - t0,
                              "lr_c": rd.lr_c, "finite": bool(torch.isfinite(rd.S).all()),
                              "map_nmse": traj(rd, every), "slf_nmse": metrics.slf_nmse(rd.S, S_true),
                              # NMSE_LOG (qmc/quantization_model_log.py:104-111): the log-domain
                              # error the log model is fitted in, vs the all-zero map's
                              "map_nmse_log": float(metrics.map_nmse(rd.S, rd.C, T,
                                                                     log_offset=LOG_OFFSET_4)),
                              "map_nmse_log_zero_map": zero,
                              "cost_first": rd.costs_s[0], "cost_last": rd.costs_s[-1]}
        print(json.dumps({"c5_dip_cold": out["c5_dip_cold"]["map_nmse"][-1]}), file=sys.stderr,
              flush=True)
    if args.warm_iters:
        out.update(c5_warm_runs(Y, Wx, b, T, S_true, R, args))
    print(json.dumps(out), flush=True)


def _nmse_pair(S, C, T, off):
    from quantized_spectrum_cartography_amd import metrics
    return (float(metrics.map_nmse(S, C, T)), float(metrics.map_nmse(S, C, T, log_offset=off)))


def c5_warm_runs(Y, Wx, b, T, S_true, R, args):
    """C5 from the de-quantized SPA warm start (warm.warm_start; the notebook's optional warm
    start, qmc/qmc.ipynb :513-516): the warm start itself, the DIP solver from it (relative
    form) and free S >= 0 from it."""
    from quantized_spectrum_cartography_amd import dip, metrics, warm
    from quantized_spectrum_cartography_amd.utils import LOG_OFFSET_4
    out = {}
    t0 = time.perf_counter()
    S0, C0 = warm.warm_start(Y.cuda(), Wx.cuda(), b, 5.0, R, offset=LOG_OFFSET_4, log_model=True,
                             width=args.warm_width)
    torch.cuda.synchronize()
    lin, lg = _nmse_pair(S0, C0, T, LOG_OFFSET_4)
    out["c5_warm_start"] = {"width": args.warm_width, "map_nmse": lin, "map_nmse_log": lg,
                            "slf_nmse": metrics.slf_nmse(S0, S_true),
                            "wall_s": time.perf_counter() - t0}
    print(json.dumps({"c5_warm_start": [lin, lg]}), file=sys.stderr, flush=True)
    s_mag, c_mag = float(S0.abs().mean()), float(C0.abs().mean())
    # c5_dip: the DIP solver from the warm start (dip.solve warm=args.dip_form, the decoder's
    # weights optimised; C from C0), Adam steps at the warm-start C's scale for C and lr_s for
    # the decoder weights; one run per decoder seed (the outcome depends on the decoder's
    # initialisation and on MIOpen's conv numerics run to run: profiles/r05/c5_dip_sweep_*.log),
    # reported per seed with the median
    every = 25
    runs = []
    for sd in args.dip_seeds:
        t0 = time.perf_counter()
        rd = dip.solve(Y, Wx, b, 5.0, R, offset=LOG_OFFSET_4, max_iter=args.dip_warm_iters,
                       S_init=S0.cpu(), C_init=C0.cpu(), lr_c=args.dip_lr_c_scale * c_mag,
                       lr_s=args.dip_lr_s, warm=args.dip_form, T_true=T, nmse_every=every,
                       seed=sd)
        torch.cuda.synchronize()
        lin_f, lg_f = _nmse_pair(rd.S, rd.C, T, LOG_OFFSET_4)
        tr = traj(rd, every)
        runs.append({"seed": sd, "map_nmse": tr[:: max(1, len(tr) // 6)],
                     "map_nmse_final": lin_f, "map_nmse_log_final": lg_f,
                     "finite": bool(torch.isfinite(rd.S).all() and torch.isfinite(rd.C).all()),
                     "slf_nmse": metrics.slf_nmse(rd.S, S_true),
                     "wall_s": time.perf_counter() - t0,
                     "cost_first": rd.costs_s[0], "cost_last": rd.costs_s[-1]})
        print(json.dumps({"c5_dip_seed%d" % sd: [lin_f, lg_f, runs[-1]["slf_nmse"]]}),
              file=sys.stderr, flush=True)
    med = lambda key: float(np.median([r[key] for r in runs]))
    out["c5_dip"] = {"iters": args.dip_warm_iters, "start": "warm (c5_warm_start)",
                     "form": ("relative: S = S0 exp(D(Z) - D(Z0))" if args.dip_form == "relative"
                              else "residual: S = max(S0 + a (D(Z) - D(Z0)), 0)"),
                     "lr_s": args.dip_lr_s, "lr_c": args.dip_lr_c_scale * c_mag,
                     "seeds": args.dip_seeds, "runs": runs,
                     "median_map_nmse_final": med("map_nmse_final"),
                     "median_slf_nmse": med("slf_nmse"),
                     "median_map_nmse_log_final": med("map_nmse_log_final"),
                     "all_finite": all(r["finite"] for r in runs)}
    # free S from the warm start (qmc.solve, log model) with S >= 0 (project_s), Adam steps
    # scaled to the warm-start fields (lr = scale x mean |S0| / mean |C0|), map NMSE every 10
    from quantized_spectrum_cartography_amd import qmc
    for scale in args.free_lr_scales:
        t0 = time.perf_counter()
        rf = qmc.solve(Y, Wx, b, 5.0, R, S_init=S0.cpu(), C_init=C0.cpu(), offset=LOG_OFFSET_4,
                       log_model=True, lr_s=scale * s_mag, lr_c=scale * c_mag, project_s=True,
                       max_iter=args.warm_iters, use_graph=True, T_true=T, nmse_every=10)
        torch.cuda.synchronize()
        tr = [[10 * (i + 1), round(float(v), 5)] for i, v in enumerate(rf.nmse)]
        lin_f, lg_f = _nmse_pair(rf.S, rf.C, T, LOG_OFFSET_4)
        out["c5_free_warm_projS_lr%g" % scale] = {
            "iters": args.warm_iters, "lr_s": scale * s_mag, "lr_c": scale * c_mag,
            "project_s": True,
            "map_nmse": tr[:: max(1, len(tr) // 12)], "map_nmse_best": min(tr, key=lambda x: x[1]),
            "map_nmse_final": lin_f, "map_nmse_log_final": lg_f,
            "finite": bool(torch.isfinite(rf.S).all()),
            "slf_nmse": metrics.slf_nmse(rf.S, S_true),
            "wall_s": time.perf_counter() - t0,
            "cost_first": rf.costs_s[0], "cost_last": rf.costs_s[-1]}
        print(json.dumps({"c5_free_warm_projS_lr%g" % scale: [lin_f, lg_f]}), file=sys.stderr,
              flush=True)
    return out


if __name__ == "__main__":
    main()
