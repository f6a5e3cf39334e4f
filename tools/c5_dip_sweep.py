"""Config-5 DIP sweep: the generated log-model map of tools/quality.py; the
DIP solver (a) from a cold start (zero C, the notebook's setting) at several C-step sizes and
(b) from the de-quantized SPA warm start at several decoder step sizes / forms, with map NMSE
and SLF-NMSE tracked along the path (every `--every` iterations).  One JSON line per run.

  python tools/c5_dip_sweep.py [--iters 1500] [--cold-lr-c 5e-3 5e-5] [--warm-lr-s 1e-2 3e-2]
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
    ap.add_argument("--iters", type=int, default=1500)
    ap.add_argument("--every", type=int, default=100)
    ap.add_argument("--seed", type=int, default=5)
    ap.add_argument("--cold-lr-c", nargs="*", default=["5e-3", "auto"])
    ap.add_argument("--cold-lr-s", type=float, nargs="*", default=[1e-2])
    ap.add_argument("--cold-lr-c-rel", type=float, nargs="*", default=[1e-2])
    ap.add_argument("--warm-forms", nargs="*", default=["relative"])
    ap.add_argument("--warm-lr-s", type=float, nargs="*", default=[3e-2])
    ap.add_argument("--warm-lr-c-scale", type=float, nargs="*", default=[1e-2])
    ap.add_argument("--lambda-s", type=float, default=100.0)
    ap.add_argument("--seeds", type=int, nargs="*", default=[None])
    ap.add_argument("--residual-scale-rel", type=float, nargs="*", default=[1.0],
                    help="dip.solve residual_scale as a multiple of its default")
    args = ap.parse_args()
    from quantized_spectrum_cartography_amd import dip, maps, metrics, warm
    from quantized_spectrum_cartography_amd import quantization_model_log as qml
    from quantized_spectrum_cartography_amd.utils import LOG_OFFSET_4, QUANTIZATION_BOUNDARIES_4_BINS_LOG
    K, R, N = 64, 4, 256
    m = maps.generate_map(K, R, shadow_sigma=5.0, Xc=50.0, I=N, J=N, seed=args.seed)
    T, S_true = m["T"], m["S"]
    torch.manual_seed(args.seed)
    Y = qml.quantize(T.cpu(), 5.0, QUANTIZATION_BOUNDARIES_4_BINS_LOG, LOG_OFFSET_4).unsqueeze(1)
    Wx = torch.bernoulli(torch.full((K, 1, N, N), 0.1))
    b = QUANTIZATION_BOUNDARIES_4_BINS_LOG
    off = LOG_OFFSET_4

    def metrics_of(S, C):
        return dict(map=round(float(metrics.map_nmse(S, C, T)), 5),
                    log=round(float(metrics.map_nmse(S, C, T, log_offset=off)), 5),
                    slf=round(metrics.slf_nmse(S, S_true), 5),
                    finite=bool(torch.isfinite(S).all() and torch.isfinite(C).all()))

    def run(name, seed=None, **kw):
        path = []

        def cb(i, d):
            if i % args.every == 0:
                path.append([i, metrics_of(d["S"].detach(), d["C"])])
        t0 = time.perf_counter()
        res = dip.solve(Y, Wx, b, 5.0, R, offset=off, max_iter=args.iters,
                        seed=args.seed if seed is None else seed, callback=cb,
                        lambda_s=args.lambda_s, **kw)
        torch.cuda.synchronize()
        out = {"kw": {k: (v if isinstance(v, (int, float, str)) else "tensor")
                      for k, v in kw.items()},
               "final": metrics_of(res.S, res.C), "path": path,
               "cost_first": res.costs_s[0], "cost_last": res.costs_s[-1],
               "nll_c_last": res.costs_c[-1],
               "lr_c_used": getattr(res, "lr_c", None),
               "wall_s": round(time.perf_counter() - t0, 2)}
        print(json.dumps({name: out}), flush=True)

    S0, C0 = warm.warm_start(Y.cuda(), Wx.cuda(), b, 5.0, R, offset=off, log_model=True, width=8.0)
    torch.cuda.synchronize()
    starts = {0: (S0, C0)}
    print(json.dumps({"warm_start": metrics_of(S0, C0)}), flush=True)
    c_mag = float(C0.abs().mean())
    for lr_c in args.cold_lr_c:
        for lr_s in args.cold_lr_s:
            for rel in (args.cold_lr_c_rel if lr_c == "auto" else [None]):
                kw = dict(lr_c=(lr_c if lr_c == "auto" else float(lr_c)), lr_s=lr_s)
                if rel is not None:
                    kw["lr_c_rel"] = rel
                run("cold_lrc%s%s_lrs%g" % (lr_c, "" if rel is None else "_rel%g" % rel, lr_s),
                    **kw)
    for rf, (S0, C0) in starts.items():
        c_mag = float(C0.abs().mean())
        for form in args.warm_forms:
            for lr_s in args.warm_lr_s:
                for cs in args.warm_lr_c_scale:
                    for sd in args.seeds:
                        for ar in args.residual_scale_rel:
                            a0 = float(S0.abs().mean()) if form == "residual" else 1.0
                            run("warm_rf%d_%s_lrs%g_lrc%g_a%g_seed%s" % (rf, form, lr_s, cs, ar,
                                                                        sd),
                                seed=sd, S_init=S0.cpu(), C_init=C0.cpu(), lr_c=cs * c_mag,
                                lr_s=lr_s, warm=form, residual_scale=ar * a0)


if __name__ == "__main__":
    main()
