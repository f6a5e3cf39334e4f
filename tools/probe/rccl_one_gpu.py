"""Probe: can two RCCL ranks share one GPU on this pool's one-GPU box?  Each rank runs the
K-slab exchange's collectives (reduce-scatter, all-gather, all-reduce) eagerly and inside a
captured graph and checks the sums.

  python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 \
      --master-port 29533 tools/probe/rccl_one_gpu.py
"""
import os

import torch
import torch.distributed as dist


def main():
    rank, ws = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    n = 1 << 20
    x = torch.full((ws * n,), float(rank + 1), device="cuda")
    out = torch.empty(n, device="cuda")
    dist.reduce_scatter_tensor(out, x)
    want = ws * (ws + 1) / 2
    ok_rs = bool((out == want).all())
    g = torch.empty(ws * n, device="cuda")
    dist.all_gather_into_tensor(g, out)
    ok_ag = bool((g == want).all())
    a = torch.ones(8, device="cuda") * (rank + 1)
    dist.all_reduce(a)
    ok_ar = bool((a == want).all())
    # captured
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(gr, stream=s):
            dist.reduce_scatter_tensor(out, x)
            dist.all_gather_into_tensor(g, out)
    torch.cuda.current_stream().wait_stream(s)
    out.zero_()
    g.zero_()
    gr.replay()
    torch.cuda.synchronize()
    ok_graph = bool((g == want).all())
    print("rank %d/%d: reduce_scatter %s all_gather %s all_reduce %s captured %s" % (
        rank, ws, ok_rs, ok_ag, ok_ar, ok_graph), flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
