"""Time the SPA warm start / NNLS kernels at the C3 shape (K = 256 bins, 512 x 512 pixels,
R = 8) with HIP events on the launch stream; prints one JSON line.

  syrk_f32   qsc_syrk: K x K Gram, f32 MFMA (v_mfma_f32_16x16x4_f32), peak 157.3 TF
  spa        qsc_spa: f64-MFMA Gram (v_mfma_f64_16x16x4_f64) + selection + fit + rows
  nnls       qsc_nnls: K independent R-variable NNLS problems (Lawson-Hanson, one thread each)
Algorithmic flops of a Gram: K (K + 1) / 2 entries x 2 P (the upper triangle; the kernel
computes whole 64 x 64 tile pairs of the upper triangle).
CPU leg: the numpy fp64 oracle (oracle/spa.py, explicit residual as the MATLAB) on the same
data, single call.
"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from quantized_spectrum_cartography_amd import gram, spa  # noqa: E402


def timed(fn, reps=20, warm=3):
    for _ in range(warm):
        fn()
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record(s)
    for _ in range(reps):
        fn()
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3  # us


def main():
    from oracle import spa as ospa
    K, I, J, R = 256, 512, 512, 8
    P = I * J
    C, S, T, pure = ospa.separable_problem(K, P, R, seed=3)
    Tt = torch.from_numpy(T).float().cuda()
    flops = K * (K + 1) / 2 * 2 * P
    t_syrk = timed(lambda: spa.syrk(Tt))
    t_spa = timed(lambda: spa.spa_init(Tt, R), reps=5)
    Cg, Sg, idx = spa.spa_init(Tt, R)
    Q = Sg
    Gq, Bq = gram.gram(Q), gram.cross(Q, Tt)
    t_nnls = timed(lambda: gram.nnls(Gq, Bq, 0.25))
    # map compose (qsc_map_compose): R = 16 fields of 1024 x 1024, HBM-bound
    from quantized_spectrum_cartography_amd import maps
    Rm, Im, Jm = 16, 1024, 1024
    sh = torch.randn((Rm, Im, Jm), device="cuda")
    loc = np.stack([1023 * np.random.default_rng(0).random(Rm), 1023 * np.random.default_rng(1).random(Rm)], 1)
    al = 2 + 0.5 * np.random.default_rng(2).random(Rm)
    ld = torch.as_tensor(loc, dtype=torch.float32, device="cuda")
    ad = torch.as_tensor(al, dtype=torch.float32, device="cuda")
    t_map = timed(lambda: maps.compose(sh, ld, ad))
    map_bytes = Rm * Im * Jm * 4 * 4  # read shadow, write S, re-read + write in the normalisation
    t0 = time.perf_counter()
    Co, So, idx_o = ospa.nmf_spa(T, R)
    t_cpu = time.perf_counter() - t0
    out = {
        "shape": {"K": K, "P": P, "R": R},
        "syrk_f32_us": t_syrk, "syrk_f32_TFLOPs": flops / t_syrk / 1e6,
        "syrk_f32_frac_of_157.3TF": flops / t_syrk / 1e6 / 157.3,
        "spa_total_us": t_spa, "spa_gram_f64_TFLOPs_upper_bound": flops / t_spa / 1e6,
        "nnls_us": t_nnls,
        "map_compose_us": t_map, "map_compose_GBs": map_bytes / t_map / 1e3,
        "map_compose_frac_of_8TBs": map_bytes / t_map / 1e3 / 8000.0,
        "picked_bins_match_oracle": idx == idx_o,
        "cpu_oracle_nmf_spa_s": t_cpu, "cpu_threads": torch.get_num_threads(),
    }
    print(json.dumps(out))


if __name__ == "__main__":
    main()
