"""Config-5 exploration: the generated log-model map of tools/quality.py,
the de-quantized SPA warm start, then (a) free S >= 0 (project_s) from the warm start at a few
Adam step scales and (b) the DIP solver from a decoder pre-fitted to the warm start, with map
NMSE trajectories.  One JSON line per run on stdout.

  python tools/c5_explore.py [--iters 500] [--prefit 2000]
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
    ap.add_argument("--iters", type=int, default=500)
    ap.add_argument("--prefit", type=int, default=2000)
    ap.add_argument("--prefit-marks", type=int, nargs="*", default=[250, 1000])
    ap.add_argument("--ndf", type=int, nargs="*", default=[16, 64])
    ap.add_argument("--prefit-lr", type=float, default=1e-2)
    ap.add_argument("--seed", type=int, default=5)
    ap.add_argument("--free-scales", type=float, nargs="*", default=[1e-2, 3e-2])
    ap.add_argument("--dip-lr-s", type=float, nargs="*", default=[1e-4, 1e-3, 1e-2])
    ap.add_argument("--dip-lr-c-scales", type=float, nargs="*", default=[1e-2])
    ap.add_argument("--dip-forms", nargs="*", default=["residual", "relative"])
    ap.add_argument("--dip-lr-c-scale", type=float, default=1e-3)
    args = ap.parse_args()
    from quantized_spectrum_cartography_amd import dip, maps, metrics, qmc, warm
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

    def pair(S, C):
        return (round(float(metrics.map_nmse(S, C, T)), 5),
                round(float(metrics.map_nmse(S, C, T, log_offset=off)), 5))

    def emit(name, d):
        print(json.dumps({name: d}), flush=True)

    S0, C0 = warm.warm_start(Y.cuda(), Wx.cuda(), b, 5.0, R, offset=off, log_model=True, width=8.0)
    torch.cuda.synchronize()
    emit("warm_start", {"map_nmse_lin_log": pair(S0, C0)})
    s_mag, c_mag = float(S0.abs().mean()), float(C0.abs().mean())
    every = 10
    for scale in args.free_scales:
        t0 = time.perf_counter()
        rf = qmc.solve(Y, Wx, b, 5.0, R, S_init=S0.cpu(), C_init=C0.cpu(), offset=off,
                       log_model=True, lr_s=scale * s_mag, lr_c=scale * c_mag, project_s=True,
                       max_iter=args.iters, use_graph=True, T_true=T, nmse_every=every)
        torch.cuda.synchronize()
        tr = [[every * (i + 1), round(float(v), 5)] for i, v in enumerate(rf.nmse)]
        emit("free_projS_lr%g" % scale, {
            "lr_s": scale * s_mag, "lr_c": scale * c_mag, "iters": args.iters,
            "traj": tr[:: max(1, len(tr) // 10)], "best": min(tr, key=lambda x: x[1]),
            "final_lin_log": pair(rf.S, rf.C), "finite": bool(torch.isfinite(rf.S).all()),
            "wall_s": round(time.perf_counter() - t0, 2)})
    # DIP from the warm start, residual form (dip.solve warm="residual"): S = max(S0 + a (D(Z) -
    # D(Z0)), 0), the decoder weights optimised, C from C0 (lr_c at the warm-start C's scale)
    for form, lr_s in [(f, l) for f in args.dip_forms for l in args.dip_lr_s]:
        for cs in args.dip_lr_c_scales:
            t0 = time.perf_counter()
            lr_c = cs * c_mag
            rd = dip.solve(Y, Wx, b, 5.0, R, offset=off, max_iter=args.iters, S_init=S0.cpu(),
                           C_init=C0.cpu(), lr_c=lr_c, lr_s=lr_s, T_true=T, nmse_every=25,
                           seed=args.seed, warm=form)
            torch.cuda.synchronize()
            tr = [[25 * (i + 1), round(float(v), 5)] for i, v in enumerate(rd.nmse)]
            emit("dip_%s_lr_s%g_c%g" % (form, lr_s, cs), {
                "lr_s": lr_s, "lr_c": lr_c, "iters": args.iters, "traj": tr[:: max(1, len(tr) // 10)],
                "best": min(tr, key=lambda x: x[1]) if tr else None,
                "final_lin_log": pair(rd.S, rd.C), "finite": bool(torch.isfinite(rd.S).all()),
                "wall_s": round(time.perf_counter() - t0, 2)})

if __name__ == "__main__":
    main()
