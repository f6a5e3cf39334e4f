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


CONFIGS = {
    # name: (I, J, K, R)   BASELINE.json configs
    "c2": (256, 256, 64, 4),
    "c3": (512, 512, 256, 8),
    "c4": (512, 512, 1024, 16),
    # one GPU's K-slab share of c4 at N = 8 (K_loc = 1024 / 8): the per-GPU kernel of the
    # north-star 8-GPU layout, benchable on one GPU
    "c4k": (512, 512, 128, 16),
}
