"""Synthetic one-bit / quantized radio-map problems for tests and benchmarks.

`onebit_problem` follows the recipe of BASELINE.md section 3, the inputs
the reference's CPU path is timed on: torch.manual_seed(seed) on the host CPU, then in order
S_true = rand(R,1,I,J); C_true = rand(R,K); T_true = get_tensor(S_true, C_true);
thr = median(T_true); sigma = (max - min)(T_true)/4; b = [0, thr, max]; Y = quantize(T_true,
sigma, b) (linear probit, noise torch.randn on the host); Wx = bernoulli(full((K,1,I,J), f));
S0 = 0.5*rand(R,1,I,J); C0 = 0.5*rand(R,K).  Generated on the host so that the CPU baseline
and the GPU path see byte-identical inputs; T_true is reconstructed on the GPU when asked.
"""
import torch

from . import _model


def onebit_problem(I, J, K, R, f=0.1, seed=20260, device="cuda", keep_T=True, device_rng=False):
    """device_rng=True draws the same recipe from a device generator (seeded with `seed`): the
    same problem on every rank of a job, without the host RNG's minutes for C4-sized maps
    (512 x 512 x 1024: 268 M noise and mask samples), but not the host draw's values."""
    if device_rng:
        g = torch.Generator(device=device).manual_seed(seed)
        S_true = torch.rand(R, 1, I, J, generator=g, device=device)
        C_true = torch.rand(R, K, generator=g, device=device)
        T_true = _model.get_tensor(S_true, C_true)
        thr = float(T_true.median())
        tmax, tmin = float(T_true.max()), float(T_true.min())
        sigma = (tmax - tmin) / 4
        b = torch.tensor([0.0, thr, tmax])
        noise = torch.randn(T_true.shape, generator=g, device=device)
        Y = _model.quantize(T_true, sigma, b, noise=noise).unsqueeze(1)
        del noise
        Wx = torch.bernoulli(torch.full((K, 1, I, J), f, device=device), generator=g)
        S0 = 0.5 * torch.rand(R, 1, I, J, generator=g, device=device)
        C0 = 0.5 * torch.rand(R, K, generator=g, device=device)
        S_true, C_true, S0, C0 = S_true.cpu(), C_true.cpu(), S0.cpu(), C0.cpu()
        out = dict(S_true=S_true, C_true=C_true, b=b, sigma=sigma, Y=Y, Wx=Wx, S0=S0, C0=C0,
                   log_model=False, offset=0.0, thr=thr)
        if keep_T:
            out["T_true"] = T_true
        return out
    g_state = torch.random.get_rng_state()
    try:
        torch.manual_seed(seed)
        S_true = torch.rand(R, 1, I, J)
        C_true = torch.rand(R, K)
        # T_true on the GPU (bit-identical to the reference get_tensor), back to the host
        T_true = _model.get_tensor(S_true.to(device), C_true.to(device))
        thr = float(T_true.median())
        tmax, tmin = float(T_true.max()), float(T_true.min())
        sigma = (tmax - tmin) / 4
        b = torch.tensor([0.0, thr, tmax])
        noise = torch.randn(T_true.shape)
        Y = _model.quantize(T_true, sigma, b, noise=noise).unsqueeze(1)
        del noise
        Wx = torch.bernoulli(torch.full((K, 1, I, J), f))
        S0 = 0.5 * torch.rand(R, 1, I, J)
        C0 = 0.5 * torch.rand(R, K)
    finally:
        torch.random.set_rng_state(g_state)
    out = dict(S_true=S_true, C_true=C_true, b=b, sigma=sigma, Y=Y, Wx=Wx, S0=S0, C0=C0,
               log_model=False, offset=0.0, thr=thr)
    if keep_T:
        out["T_true"] = T_true
    return out


def kslab_onebit_problem(I, J, K_local, R, rank, world, dist=None, f=0.1, seed=20260,
                         device="cuda"):
    """One rank's K-slab of a global one-bit problem with K_local * world frequency bins.

    S_true and S0 are common to all ranks (same seed); C_true / C0 columns, the noise and the
    mask are drawn per slab.  The quantizer (thr = mean of the slabs' medians, sigma from the
    global min/max) is agreed over `dist` so that all slabs share one probit model."""
    # drawn on the device: every rank builds its slab at once without the host's CPU share
    g = torch.Generator(device=device).manual_seed(seed)
    S_true = torch.rand(R, 1, I, J, generator=g, device=device)
    S0 = 0.5 * torch.rand(R, 1, I, J, generator=g, device=device)
    gl = torch.Generator(device=device).manual_seed(seed + 1000 + rank)
    C_true = torch.rand(R, K_local, generator=gl, device=device)
    C0 = 0.5 * torch.rand(R, K_local, generator=gl, device=device)
    T = _model.get_tensor(S_true.to(device), C_true.to(device))
    stats = torch.tensor([float(T.median()), -float(T.min()), float(T.max())], dtype=torch.float64,
                         device=device)
    if dist is not None and world > 1:
        med = stats[:1].clone()
        dist.all_reduce(med)
        mx = stats[1:].clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        stats = torch.cat([med / world, mx])
    thr, tmin, tmax = float(stats[0]), -float(stats[1]), float(stats[2])
    sigma = (tmax - tmin) / 4
    b = torch.tensor([0.0, thr, tmax])
    noise = torch.randn(T.shape, generator=gl, device=device)
    Y = _model.quantize(T, sigma, b, noise=noise).unsqueeze(1)
    del noise
    Wx = torch.bernoulli(torch.full((K_local, 1, I, J), f, device=device), generator=gl)
    return dict(S_true=S_true.cpu(), C_true=C_true.cpu(), b=b, sigma=sigma, Y=Y, Wx=Wx,
                S0=S0.cpu(), C0=C0.cpu(), log_model=False, offset=0.0, thr=thr, T_true=T)


def ijslab_onebit_problem(I, J, K, R, rank, world, dist=None, f=0.1, seed=20260,
                          device="cuda"):
    """One rank's pixel block of a global one-bit problem on an (I * world) x J grid.

    C_true and C0 are common to all ranks (same seed); S_true / S0, the noise and the mask are
    drawn per block.  The quantizer (thr = mean of the blocks' medians, sigma from the global
    min/max) is agreed over `dist` so that all blocks share one probit model."""
    g = torch.Generator(device=device).manual_seed(seed)  # (on the device, as kslab_*)
    C_true = torch.rand(R, K, generator=g, device=device)
    C0 = 0.5 * torch.rand(R, K, generator=g, device=device)
    gl = torch.Generator(device=device).manual_seed(seed + 2000 + rank)
    S_true = torch.rand(R, 1, I, J, generator=gl, device=device)
    S0 = 0.5 * torch.rand(R, 1, I, J, generator=gl, device=device)
    T = _model.get_tensor(S_true.to(device), C_true.to(device))
    stats = torch.tensor([float(T.median()), -float(T.min()), float(T.max())], dtype=torch.float64,
                         device=device)
    if dist is not None and world > 1:
        med = stats[:1].clone()
        dist.all_reduce(med)
        mx = stats[1:].clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        stats = torch.cat([med / world, mx])
    thr, tmin, tmax = float(stats[0]), -float(stats[1]), float(stats[2])
    sigma = (tmax - tmin) / 4
    b = torch.tensor([0.0, thr, tmax])
    noise = torch.randn(T.shape, generator=gl, device=device)
    Y = _model.quantize(T, sigma, b, noise=noise).unsqueeze(1)
    del noise
    Wx = torch.bernoulli(torch.full((K, 1, I, J), f, device=device), generator=gl)
    return dict(S_true=S_true.cpu(), C_true=C_true.cpu(), b=b, sigma=sigma, Y=Y, Wx=Wx,
                S0=S0.cpu(), C0=C0.cpu(), log_model=False, offset=0.0, thr=thr, T_true=T)


def _orderable_keys(x):
    """float32 -> int64 keys in [0, 2^32) whose integer order is the float order."""
    bits = x.reshape(-1).contiguous().view(torch.int32).to(torch.int64) & 0xFFFFFFFF
    return torch.where(bits >= 0x80000000, 0xFFFFFFFF - bits, bits + 0x80000000)


def _key_to_float(key):
    import numpy as np
    bits = key - 0x80000000 if key >= 0x80000000 else 0xFFFFFFFF - key
    return float(np.array([bits], dtype=np.uint32).view(np.float32)[0])


def global_kth(x, kth, dist=None):
    """The kth smallest (0-based) float32 value of the union of every rank's `x` -- exactly,
    without gathering the values: a two-digit (16 + 16 bit) radix select over the order-keyed
    float bits, the 65536-bin histograms summed with two all-reduces.  With dist None, x is the
    whole set; kth = (n - 1) // 2 is torch.median's lower median."""
    key = _orderable_keys(x)
    hi = key >> 16

    def summed(h):
        if dist is not None:
            dist.all_reduce(h)
        return h

    h = summed(torch.bincount(hi, minlength=1 << 16))
    cum = h.cumsum(0)
    b_hi = int(torch.searchsorted(cum, torch.tensor([kth], device=cum.device), right=True)[0])
    below = int(cum[b_hi - 1]) if b_hi > 0 else 0
    lo = key[hi == b_hi] & 0xFFFF
    h2 = summed(torch.bincount(lo, minlength=1 << 16))
    cum2 = h2.cumsum(0)
    b_lo = int(torch.searchsorted(cum2, torch.tensor([kth - below], device=cum2.device),
                                  right=True)[0])
    return _key_to_float((b_hi << 16) | b_lo)


def _bin_seed(seed, k):
    return int(seed) * 1000003 + 7919 * (int(k) + 1)


def onebit_block_problem(I, J, K, R, k_range=None, i_range=None, f=0.1, seed=20260,
                         device="cuda", dist=None, keep_T=True, reconstruct=None,
                         quantizer=None):
    """Bins [k0, k1) x image rows [i0, i1) of ONE global one-bit problem that is a function of
    (seed, k) only, so a rank draws just its own block and the union of any split of the bins
    (K-slab) or rows (IJ-slab) over any number of ranks is the same map -- with no rank ever
    holding the whole map (C4: 268 M entries).

    The BASELINE.md recipe, blocked: S_true = rand(R,1,I,J), C_true = rand(R,K), S0 = 0.5 rand,
    C0 = 0.5 rand from one device generator (every rank draws the same small factors); the
    noise and the Bernoulli(f) mask of bin k from a generator seeded by (seed, k);
    T = get_tensor(S_true, C_true) on the block; thr = the exact lower median of the WHOLE map
    (global_kth over the ranks' blocks, = torch.median of the union), sigma = (max - min)/4 of
    the whole map (all-reduced), b = [0, thr, max]; Y = quantize(T, sigma, b).  `dist` must be
    the process group whose blocks partition the map (None: this block is the whole map).
    (`reconstruct` / `quantizer` replace get_tensor / quantize, for CPU tests of the blocking.)
    Returns split_problem's keys: block C_true / C0 / Y / Wx / T_true, full S_true / S0 (row
    block for i_range), plus "bounds" (k0, k1) and "rows" (i0, i1)."""
    quantize = quantizer or _model.quantize
    k0, k1 = k_range if k_range is not None else (0, K)
    i0, i1 = i_range if i_range is not None else (0, I)
    get_T = reconstruct or _model.get_tensor
    g = torch.Generator(device=device).manual_seed(seed)
    S_true = torch.rand(R, 1, I, J, generator=g, device=device)
    C_true = torch.rand(R, K, generator=g, device=device)
    S0 = 0.5 * torch.rand(R, 1, I, J, generator=g, device=device)
    C0 = 0.5 * torch.rand(R, K, generator=g, device=device)
    S_b, S0_b = S_true[..., i0:i1, :].contiguous(), S0[..., i0:i1, :].contiguous()
    C_b, C0_b = C_true[:, k0:k1].contiguous(), C0[:, k0:k1].contiguous()
    T = get_T(S_b, C_b)
    ext = torch.stack([T.max(), -T.min()]).to(torch.float64)
    if dist is not None:
        dist.all_reduce(ext, op=dist.ReduceOp.MAX)
    tmax, tmin = float(ext[0]), -float(ext[1])
    thr = global_kth(T, (I * J * K - 1) // 2, dist)
    sigma = (tmax - tmin) / 4
    b = torch.tensor([0.0, thr, tmax])
    noise = torch.empty((k1 - k0, i1 - i0, J), device=device)
    Wx = torch.empty((k1 - k0, 1, i1 - i0, J), device=device)
    full = torch.full((I, J), f, device=device)
    for k in range(k0, k1):
        gk = torch.Generator(device=device).manual_seed(_bin_seed(seed, k))
        noise[k - k0] = torch.randn((I, J), generator=gk, device=device)[i0:i1]
        Wx[k - k0, 0] = torch.bernoulli(full, generator=gk)[i0:i1]
    Y = quantize(T, sigma, b, noise=noise).unsqueeze(1)
    del noise
    out = dict(S_true=S_b.cpu(), C_true=C_b.cpu(), b=b, sigma=sigma, Y=Y, Wx=Wx, S0=S0_b.cpu(),
               C0=C0_b.cpu(), log_model=False, offset=0.0, thr=thr, bounds=(k0, k1),
               rows=(i0, i1))
    if keep_T:
        out["T_true"] = T
    return out


def block_problem(cfg, rank, world, shard, seed, dist=None, device="cuda", **kw):
    """This rank's share of the blocked global problem of a config (onebit_block_problem):
    shard "kslab" = bins kslab_bounds(K, world, rank), "ijslab" = rows kslab_bounds(I, ...)."""
    from .distributed import kslab_bounds
    I, J, K, R = cfg
    if shard == "kslab":
        return onebit_block_problem(I, J, K, R, k_range=kslab_bounds(K, world, rank), seed=seed,
                                    device=device, dist=dist, **kw)
    if shard == "ijslab":
        return onebit_block_problem(I, J, K, R, i_range=kslab_bounds(I, world, rank), seed=seed,
                                    device=device, dist=dist, **kw)
    raise ValueError("shard must be 'ijslab' or 'kslab'")


def split_problem(prob, rank, world, shard):
    """This rank's shard of ONE global problem (strong scaling: the map is fixed, N ranks share
    it).  shard="ijslab": rows [i0, i1) of the I axis (pixels), C replicated; shard="kslab":
    frequency bins [k0, k1), S replicated.  Shards are views/slices of the global tensors, so
    the union over ranks is the global problem exactly (tests/test_distributed_gloo.py)."""
    from .distributed import kslab_bounds
    out = dict(prob)
    if shard == "ijslab":
        I = prob["Y"].shape[-2]
        i0, i1 = kslab_bounds(I, world, rank)
        for key in ("S_true", "S0", "Y", "Wx", "T_true"):
            if key in prob:
                out[key] = prob[key][..., i0:i1, :].contiguous()
        out["bounds"] = (i0, i1)
    elif shard == "kslab":
        K = prob["Y"].shape[0]
        k0, k1 = kslab_bounds(K, world, rank)
        for key in ("Y", "Wx", "T_true"):
            if key in prob:
                out[key] = prob[key][k0:k1].contiguous()
        for key in ("C_true", "C0"):
            out[key] = prob[key][:, k0:k1].contiguous()
        out["bounds"] = (k0, k1)
    else:
        raise ValueError("shard must be 'ijslab' or 'kslab'")
    return out


def c5_problem(seed=5, I=256, K=64, R=4, f=0.1, sigma=5.0, device="cuda"):
    """BASELINE configs[4]: a generated 256 x 256 x 64 map with R = 4
    emitters (maps.generate_map: Gaussian PSDs, path loss x FFT-correlated shadowing, unit-norm
    fields as generate_map.m:118), observed through the LOG model with the notebook's 4 log
    bins, LOG_OFFSET_4 and sigma = 5 (qmc/qmc.ipynb :510-537), per-entry Bernoulli(f) mask
    (:493).  S0 = (0.25 + 0.5 rand)/I (the fields' scale), C0 = 0.5 rand.  `lr_s` is the free-S
    Adam step scaled to S (1e-5) so that T_hat = S C stays positive under the log model."""
    from . import maps
    from . import quantization_model_log as qml
    from .utils import LOG_OFFSET_4, QUANTIZATION_BOUNDARIES_4_BINS_LOG
    m = maps.generate_map(K, R, shadow_sigma=5.0, Xc=50.0, I=I, J=I, seed=seed, device=device)
    g = torch.Generator().manual_seed(seed)
    noise = torch.randn((K, I, I), generator=g)
    b = torch.tensor(QUANTIZATION_BOUNDARIES_4_BINS_LOG)
    Y = qml.quantize(m["T"].cpu(), sigma, b, offset=LOG_OFFSET_4, noise=noise).unsqueeze(1)
    Wx = torch.bernoulli(torch.full((K, 1, I, I), f), generator=g)
    S0 = (0.25 + 0.5 * torch.rand(R, 1, I, I, generator=g)) / I
    C0 = 0.5 * torch.rand(R, K, generator=g)
    return dict(Y=Y, Wx=Wx, b=b, sigma=float(sigma), S0=S0, C0=C0,
                S_true=m["S"].reshape(R, 1, I, I), C_true=m["C"], T_true=m["T"],
                log_model=True, offset=LOG_OFFSET_4, lr_s=1e-5)


CONFIGS = {
    # name: (I, J, K, R)   BASELINE.json configs
    "c2": (256, 256, 64, 4),
    "c3": (512, 512, 256, 8),
    "c4": (512, 512, 1024, 16),
    # one GPU's K-slab share of c4 at N = 8 (K_loc = 1024 / 8): the per-GPU kernel of the
    # north-star 8-GPU layout, benchable on one GPU
    "c4k": (512, 512, 128, 16),
    # one GPU's K-slab share of c3 at N = 2, 4, 8 (K_loc = 256 / N): the per-GPU sequence of
    # the default strong K-slab bench line, for the 1 -> 8 projection of DESIGN.md section 5
    "c3k2": (512, 512, 128, 8),
    "c3k4": (512, 512, 64, 8),
    "c3k8": (512, 512, 32, 8),
    # log model (4 log bins, sigma 5) on a generated map, free S (c5_problem)
    "c5": (256, 256, 64, 4),
    "c5dip": (256, 256, 64, 4),
}
