"""CPU (gloo, world sizes 2 and 3): the blocked global problem (synthetic.onebit_block_problem)
is world-size independent -- the union of the K-slab or IJ-slab blocks that the ranks draw on
their own is the world-1 problem exactly, with the global threshold (exact lower median,
synthetic.global_kth) and sigma agreed over the process group.  This is what lets every rank of
the C4 (512x512x1024) bench draw only its own slab.  The blocks are reconstructed and quantized
with the oracle's reference ops on the CPU (the product path would use the HIP ones)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import reference_ops as ro

CFG = (11, 9, 13, 3)  # I, J, K, R: odd sizes so the splits are uneven


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _block(k_range=None, i_range=None, group=None):
    from quantized_spectrum_cartography_amd.synthetic import onebit_block_problem
    I, J, K, R = CFG
    return onebit_block_problem(I, J, K, R, k_range=k_range, i_range=i_range, f=0.3, seed=77,
                                device="cpu", dist=group, reconstruct=ro.get_tensor,
                                quantizer=ro.quantize)


@pytest.mark.parametrize("n", [1, 2, 5, 1000, 4097])
def test_global_kth_is_torch_lower_median(n):
    from quantized_spectrum_cartography_amd.synthetic import global_kth
    g = torch.Generator().manual_seed(n)
    x = torch.randn(n, generator=g) * 3
    x[: n // 3] = x[0]  # ties
    if n > 4:
        x[1], x[2] = 0.0, -0.0
    assert global_kth(x, (n - 1) // 2) == float(x.median())
    for k in {0, n - 1, n // 4}:
        assert global_kth(x, k) == float(torch.sort(x).values[k])


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from quantized_spectrum_cartography_amd.distributed import kslab_bounds
        from quantized_spectrum_cartography_amd.synthetic import global_kth
        I, J, K, R = CFG
        res = {}
        # distributed selection over uneven local sets
        def part(r):
            return torch.randn(50 + 17 * r, generator=torch.Generator().manual_seed(100 + r))
        x = part(rank)
        allx = torch.cat([part(r) for r in range(world)])
        n = allx.numel()
        res["kth"] = global_kth(x, (n - 1) // 2, dist) == float(allx.median())
        ref = _block()
        for shard, kw, ax in (("kslab", "k_range", 0), ("ijslab", "i_range", -2)):
            span = kslab_bounds(K if shard == "kslab" else I, world, rank)
            blk = _block(**{kw: span}, group=dist)
            res[shard + "_thr"] = blk["thr"] == ref["thr"] and blk["sigma"] == ref["sigma"]
            for key in ("Y", "Wx", "T_true"):
                mine = blk[key].contiguous()
                sizes = [kslab_bounds(K if shard == "kslab" else I, world, r) for r in range(world)]
                shp = list(mine.shape)
                # gloo all_gather needs equal sizes: pad to the largest block
                big = max(b_ - a for a, b_ in sizes)
                pad_shape = list(shp)
                pad_shape[ax] = big
                padded = torch.zeros(pad_shape, dtype=mine.dtype)
                padded.narrow(ax, 0, shp[ax]).copy_(mine)
                outs = [torch.zeros_like(padded) for _ in range(world)]
                dist.all_gather(outs, padded)
                whole = torch.cat([o.narrow(ax, 0, b_ - a) for o, (a, b_) in zip(outs, sizes)],
                                  dim=ax)
                res["%s_%s" % (shard, key)] = bool(torch.equal(whole, ref[key]))
            rep = ("S_true", "S0") if shard == "kslab" else ("C_true", "C0")
            for key in rep:
                res["%s_%s_rep" % (shard, key)] = bool(torch.equal(blk[key], ref[key]))
        np.savez(out + ".r%d" % rank, names=np.array(sorted(res)),
                 vals=np.array([bool(res[k]) for k in sorted(res)]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_blocks_union_is_the_world1_problem(tmp_path, world):
    out = str(tmp_path / "blk")
    mp.start_processes(_worker, args=(world, _free_port(), out), nprocs=world, join=True,
                       start_method="spawn")
    for r in range(world):
        d = np.load(out + ".r%d.npz" % r)
        bad = [str(n) for n, v in zip(d["names"], d["vals"]) if not v]
        assert not bad, (r, bad)


def test_block_problem_recipe_world1():
    """The world-1 block is the BASELINE recipe on the whole map: thr = torch.median(T),
    sigma = (max - min)/4, Y = quantize(T + sigma * noise), per-bin noise/mask streams."""
    p = _block()
    T = p["T_true"]
    assert p["thr"] == float(T.median())
    assert p["sigma"] == (float(T.max()) - float(T.min())) / 4
    assert p["Y"].shape == (13, 1, 11, 9) and set(torch.unique(p["Y"]).tolist()) <= {0, 1}
    frac = float(p["Wx"].mean())
    assert 0.15 < frac < 0.45
    # the mask / noise of a bin do not depend on which other bins are drawn
    q = _block(k_range=(4, 6))
    assert torch.equal(q["Wx"], p["Wx"][4:6]) and torch.equal(q["T_true"], T[4:6])
