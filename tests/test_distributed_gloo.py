"""CPU (gloo, world size 2): the sharding logic of distributed.KSlabSolver and IJSlabSolver.

The solver is written against a small engine interface (fused.PassEngine on the GPU).  Here it
runs over a CPU emulation of that interface whose gradients come from the oracle's closed-form
math (oracle/explicit.py, fp64), so the test checks the sharding itself: the per-slab C-passes,
the all-reduced ||C||^2 of the non-squared regulariser, and the reduce-scatter of the partial
S-gradient, the Adam update of each rank's shard of S and the all-gather that re-replicates it.  Two ranks, each holding half of the frequency bins, must reproduce
a single-process run over all bins, and both must follow the reference op sequence
(oracle/solver.py) within the parity tolerance.
"""
import math
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import explicit
from oracle import reference_ops as ro
from oracle import solver as osolver

from conftest import rel_fro

R, I, J, K, ITERS = 3, 12, 10, 16, 6


class _Obs:
    """Observations stand-in: natural pixel order is the position order (Pp = P)."""

    def __init__(self, Y, Wx):
        self.K = Y.shape[0]
        self.I, self.J = Y.shape[-2], Y.shape[-1]
        self.P = self.Pp = self.I * self.J
        self.Y = Y.reshape(self.K, -1).numpy()
        self.Wx = Wx.reshape(self.K, -1).numpy()

    def to_positions(self, X):
        """(R, P) -> position order (Pp, R): position-major rows, as the device layout"""
        return X.detach().reshape(X.shape[0], self.P).to(torch.float32).t().contiguous()

    def to_pixels(self, Xp, R):
        return Xp.t().contiguous()


class _CpuEngine:
    """The PassEngine calls KSlabSolver makes, evaluated with the oracle's fp64 gradients and
    torch.optim.Adam's update (state kept like the device qsc_state)."""

    def __init__(self, obs, b, sigma):
        self.obs, self.b, self.sigma = obs, b, sigma
        self.hist_cap = 0
        self.hist = torch.zeros(4)
        self.st = dict(step_c=0, step_s=0, iter=0, normsq_s=0.0, nll_c=0.0, nll_s=0.0)
        self.calls = []
        self._cnsq = torch.zeros(1)

    def _grad(self, S, C):
        """fp64 NLL, dS (position order, like S), dC"""
        nll, gS, gC = explicit.nll_grad(S.t().double().numpy(), C.double().numpy(), self.obs.Y,
                                        self.obs.Wx, self.b, self.sigma)
        return nll, np.ascontiguousarray(gS.T), gC

    @staticmethod
    def _adam(p, m, v, g, step, adam):
        b1, b2 = adam.beta1, adam.beta2
        m.mul_(b1).add_(g, alpha=1 - b1)
        v.mul_(b2).addcmul_(g, g, value=1 - b2)
        denom = (v.sqrt() / math.sqrt(1 - b2 ** step)).add_(adam.eps)
        p.addcdiv_(m, denom, value=-adam.lr / (1 - b1 ** step))
        if adam.project_nonneg:
            p.clamp_(min=0.0)

    def init_state(self, S):
        self.st["normsq_s"] = float((S.double() ** 2).sum())

    def cpass(self, S, C):
        nll, _, dC = self._grad(S, C)
        self._dC, self.st["nll_c"] = torch.from_numpy(dC).float(), float(nll)

    def cpass_nsq(self, S, C):
        """qsc_cpass_nsq: the C-pass + ||C_slab||^2 into the cnsq slot + the slices' ||S||^2"""
        self.calls.append("cpass_nsq")
        self.cpass(S, C)
        self._cnsq[0] = float((C.double() ** 2).sum())
        self.st["normsq_s"] = float((S.double() ** 2).sum())  # (as slice_nsq)

    def cnsq(self):
        return self._cnsq

    def sumsq(self, x, out):
        out[0] = float((x.double() ** 2).sum())

    def cfinish(self, C, mode, dC=None, mC=None, vC=None, adam=None, lambda_c=0.0,
                normsq_ext=None, **kw):
        if mode == 2:  # IJ-slab: local gradient + this shard's ||S||^2
            n = C.numel()
            dC[:n] = self._dC.reshape(-1)
            dC[n] = self.st["normsq_s"]
            return
        nrm = math.sqrt(float(normsq_ext[0]))
        g = self._dC + (lambda_c / nrm if nrm > 0 else 0.0) * C
        self.st["step_c"] += 1
        self._adam(C, mC, vC, g, self.st["step_c"], adam)

    def cupdate(self, C, mC, vC, g, adam, lambda_c, normsq_s_ext=None):
        nrm = math.sqrt(float((C.double() ** 2).sum()))
        gg = g[:C.numel()].reshape(C.shape) + (lambda_c / nrm if nrm > 0 else 0.0) * C
        self.st["step_c"] += 1
        self._adam(C, mC, vC, gg, self.st["step_c"], adam)
        if normsq_s_ext is not None:
            self.st["normsq_s"] = float(normsq_s_ext[0])

    def spass(self, S, C, mode, dS=None, mS=None, vS=None, adam=None, lambda_s=0.0):
        nll, gS, _ = self._grad(S, C)
        self.st["nll_s"] = float(nll)
        self.st["iter"] += 1
        if mode == 0:
            dS.copy_(torch.from_numpy(gS).float())
            return
        # fused S-step on this shard: lambda_s S / ||S|| with the (global) norm in the state
        nrm = math.sqrt(self.st["normsq_s"])
        gg = torch.from_numpy(gS).float() + (lambda_s / nrm if nrm > 0 else 0.0) * S
        self.st["step_s"] += 1
        self._adam(S, mS, vS, gg, self.st["step_s"], adam)
        self.st["normsq_s"] = float((S.double() ** 2).sum())  # this shard's, settled later

    def spass_kslab(self, S, C, dS_rs, chunk_rows, nranks):
        """qsc_spass_kslab: dS rows into the reduce-scatter layout (nranks chunks of chunk_rows
        rows, each followed by row_unit extra rows) + ||C_slab||^2 into every extra row's first
        element"""
        self.calls.append("spass_kslab")
        P = S.shape[0]
        g = torch.empty_like(S)
        self.spass(S, C, 0, dS=g)
        u, cn = self.row_unit, float((C.double() ** 2).sum())
        for c in range(nranks):
            a, b_ = c * chunk_rows, min((c + 1) * chunk_rows, P)
            base = c * (chunk_rows + u)
            if b_ > a:
                dS_rs[base:base + (b_ - a)] = g[a:b_]
            dS_rs[base + chunk_rows, 0] = cn

    def scpass_supported(self):
        return True

    def scpass(self, S, C, mS, vS, adam, lambda_s):
        """qsc_scpass: the S-step, then the next C-pass at the updated S."""
        self.calls.append("scpass")
        self.spass(S, C, 1, mS=mS, vS=vS, adam=adam, lambda_s=lambda_s)
        self.cpass(S, C)

    row_unit = 1

    def supdate_rows(self, S, mS, vS, g_own, adam, lambda_s, r0, r1):
        """qsc_supdate_slices: Adam on rows [r0, r1) from the shard's reduce-scattered gradient"""
        nrm = math.sqrt(self.st["normsq_s"])
        gg = g_own[: r1 - r0] + (lambda_s / nrm if nrm > 0 else 0.0) * S[r0:r1]
        self.st["step_s"] += 1
        self._adam(S[r0:r1], mS[r0:r1], vS[r0:r1], gg, self.st["step_s"], adam)
        self.calls.append("supdate_rows")

    def slice_nsq(self, S):
        """qsc_slice_nsq: ||S||^2 of the all-gathered S (every rank the same)"""
        self.calls.append("slice_nsq")
        self.st["normsq_s"] = float((S.double() ** 2).sum())

    def supdate(self, S, mS, vS, g, adam, lambda_s):
        nrm = math.sqrt(self.st["normsq_s"])
        gg = g + (lambda_s / nrm if nrm > 0 else 0.0) * S
        self.st["step_s"] += 1
        self._adam(S, mS, vS, gg, self.st["step_s"], adam)
        self.st["normsq_s"] = float((S.double() ** 2).sum())

    def flush(self, record=True):
        pass

    def read_state(self):
        return dict(self.st)


def _problem(K=K):
    g = torch.Generator().manual_seed(11)
    S_true = torch.rand(R, 1, I, J, generator=g)
    C_true = torch.rand(R, K, generator=g)
    T = ro.get_tensor(S_true, C_true)
    thr = float(T.median())
    sigma = (float(T.max()) - float(T.min())) / 4
    b = torch.tensor([0.0, thr, float(T.max())])
    Y = ro.quantize(T, sigma, b, noise=torch.randn(T.shape, generator=g)).unsqueeze(1)
    Wx = torch.bernoulli(torch.full((K, 1, I, J), 0.4), generator=g)
    S0 = 0.5 * torch.rand(R, 1, I, J, generator=g)
    C0 = 0.5 * torch.rand(R, K, generator=g)
    return S0, C0, Y, Wx, b, sigma


class _SoloDist:
    """torch.distributed stand-in for a one-process run (all-reduce = identity)."""

    @staticmethod
    def all_reduce(t, op=None):
        return t

    @staticmethod
    def get_world_size():
        return 1

    @staticmethod
    def all_gather(outs, t):
        outs[0].copy_(t)

    @staticmethod
    def reduce_scatter_tensor(out, t):
        out.copy_(t)

    @staticmethod
    def all_gather_into_tensor(out, t):
        out.copy_(t)


def _run(dist_mod, rank, world, K=K):
    from quantized_spectrum_cartography_amd.distributed import KSlabSolver, kslab_bounds
    S0, C0, Y, Wx, b, sigma = _problem(K)
    k0, k1 = kslab_bounds(K, world, rank)
    obs = _Obs(Y[k0:k1], Wx[k0:k1])
    eng = _CpuEngine(obs, b.numpy(), sigma)
    sol = KSlabSolver(obs, S0, C0[:, k0:k1], dist=dist_mod, engine=eng)
    sol.run(ITERS)
    # reduce-scatter -> Adam on the owned 1/N of S -> all-gather
    assert eng.calls.count("supdate_rows") == ITERS
    # 4 kernels per iteration: the slices' ||S||^2 ride on the C-pass (no slice_nsq launch)
    assert eng.calls.count("cpass_nsq") == ITERS and "slice_nsq" not in eng.calls[:-1]
    # the global ||C||^2 rides on the reduce-scatter of dS: one all-reduce per run (its first
    # C-step), not one per iteration
    assert eng.calls.count("spass_kslab") == ITERS
    assert sol.r1 - sol.r0 <= -(-I * J // world)
    st = eng.read_state()
    st["shard"] = (sol.r0, sol.r1)
    return sol.S_pixels().reshape(R, I * J), sol.C_global(), st


def _run_ij(dist_mod, rank, world):
    """IJ-slab: rank g owns image rows [i0, i1) (all bins), C replicated."""
    from quantized_spectrum_cartography_amd.distributed import IJSlabSolver, kslab_bounds
    S0, C0, Y, Wx, b, sigma = _problem()
    i0, i1 = kslab_bounds(I, world, rank)
    obs = _Obs(Y[:, :, i0:i1], Wx[:, :, i0:i1])
    eng = _CpuEngine(obs, b.numpy(), sigma)
    sol = IJSlabSolver(obs, S0[:, :, i0:i1], C0, dist=dist_mod, engine=eng)
    sol.run(ITERS)
    return sol.S_pixels().reshape(R, -1), sol.C.clone(), eng.read_state()


def _worker(rank, world, port, out_path, mode, K_=K):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        S, C, st = (_run(dist, rank, world, K_) if mode == "k" else _run_ij(dist, rank, world))
        np.savez(out_path + ".r%d" % rank, S=S.numpy(), C=C.numpy(), step_s=st["step_s"],
                 shard=np.array(st.get("shard", (0, 0))))
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_kslab_bounds_partition():
    from quantized_spectrum_cartography_amd.distributed import kslab_bounds
    for K_, W in [(16, 2), (17, 3), (256, 8), (5, 8)]:
        spans = [kslab_bounds(K_, W, r) for r in range(W)]
        assert spans[0][0] == 0 and spans[-1][1] == K_
        assert all(a[1] == b_[0] for a, b_ in zip(spans, spans[1:]))
        sizes = [e - s for s, e in spans]
        assert max(sizes) - min(sizes) <= 1


def test_kslab_two_ranks_match_single_process(tmp_path):
    out = str(tmp_path / "k")
    mp.start_processes(_worker, args=(2, _free_port(), out, "k"), nprocs=2, join=True,
                       start_method="spawn")
    two = np.load(out + ".r0.npz")
    r1 = np.load(out + ".r1.npz")
    S1, C1, _ = _run(_SoloDist, 0, 1)
    # S is replicated: both ranks hold the same S after the all-gather of the updated shards
    assert np.array_equal(two["S"], r1["S"])
    assert int(two["step_s"]) == ITERS
    # the two shards are disjoint and cover every position row
    (a0, a1), (b0, b1) = two["shard"], r1["shard"]
    assert a0 == 0 and a1 == b0 and b1 == I * J
    # sharded == single process up to the summation order of the partial S-gradients
    assert rel_fro(two["S"], S1.numpy()) < 1e-6
    assert rel_fro(two["C"], C1.numpy()) < 1e-6
    # and both follow the reference op sequence
    S0, C0, Y, Wx, b, sigma = _problem()
    ref = osolver.free_s_solve(S0, C0, Y, Wx, b, sigma, n_iter=ITERS)
    assert rel_fro(two["S"], ref["S"].reshape(R, -1).numpy()) < 1e-5
    assert rel_fro(two["C"], ref["C"].numpy()) < 1e-5


@pytest.mark.parametrize("world,K_", [(3, 17), (4, 18)])
def test_kslab_uneven_ranks_match_single_process(tmp_path, world, K_):
    """K-slab over 3 and 4 ranks with uneven bin splits (17 = 6 + 6 + 5, 18 = 5 + 5 + 4 + 4)
    and position shards of unequal content: the same S, C as one process over all bins, and
    the reference op sequence within the parity tolerance."""
    from quantized_spectrum_cartography_amd.distributed import kslab_bounds
    out = str(tmp_path / "ku")
    mp.start_processes(_worker, args=(world, _free_port(), out, "k", K_), nprocs=world,
                       join=True, start_method="spawn")
    res = [np.load(out + ".r%d.npz" % r) for r in range(world)]
    sizes = [b_ - a for a, b_ in (kslab_bounds(K_, world, r) for r in range(world))]
    assert len(set(sizes)) == 2  # uneven
    for r in res[1:]:
        assert np.array_equal(r["S"], res[0]["S"]) and np.array_equal(r["C"], res[0]["C"])
    shards = [tuple(r["shard"]) for r in res]
    assert shards[0][0] == 0 and shards[-1][1] == I * J
    assert all(a[1] == b_[0] for a, b_ in zip(shards, shards[1:]))
    S1, C1, _ = _run(_SoloDist, 0, 1, K_)
    assert rel_fro(res[0]["S"], S1.numpy()) < 1e-6
    assert rel_fro(res[0]["C"], C1.numpy()) < 1e-6
    S0, C0, Y, Wx, b, sigma = _problem(K_)
    ref = osolver.free_s_solve(S0, C0, Y, Wx, b, sigma, n_iter=ITERS)
    assert rel_fro(res[0]["S"], ref["S"].reshape(R, -1).numpy()) < 1e-5
    assert rel_fro(res[0]["C"], ref["C"].numpy()) < 1e-5


def test_ijslab_two_ranks_match_single_process(tmp_path):
    out = str(tmp_path / "ij")
    mp.start_processes(_worker, args=(2, _free_port(), out, "ij"), nprocs=2, join=True,
                       start_method="spawn")
    r0, r1 = np.load(out + ".r0.npz"), np.load(out + ".r1.npz")
    # C is replicated: both ranks hold the same (all-reduced gradient, same update)
    assert np.array_equal(r0["C"], r1["C"])
    assert int(r0["step_s"]) == ITERS
    # the pixel blocks reassemble the single-process S (rows [0, I/2) and [I/2, I))
    S_two = np.concatenate([r0["S"].reshape(R, -1, J), r1["S"].reshape(R, -1, J)], axis=1)
    S1, C1, _ = _run_ij(_SoloDist, 0, 1)
    assert rel_fro(S_two.reshape(R, -1), S1.numpy()) < 1e-6
    assert rel_fro(r0["C"], C1.numpy()) < 1e-6
    S0, C0, Y, Wx, b, sigma = _problem()
    ref = osolver.free_s_solve(S0, C0, Y, Wx, b, sigma, n_iter=ITERS)
    assert rel_fro(S_two.reshape(R, -1), ref["S"].reshape(R, -1).numpy()) < 1e-5
    assert rel_fro(r0["C"], ref["C"].numpy()) < 1e-5


def test_ijslab_fused_sequence_equals_plain():
    """IJ-slab with the fused launch (S-step i + C-pass i+1, qsc_scpass) runs the same kernel
    sequence as plain iterations: cpass, exchange, (scpass, exchange) x (n-1), spass."""
    from quantized_spectrum_cartography_amd.distributed import IJSlabSolver
    S0, C0, Y, Wx, b, sigma = _problem()
    out = []
    for fuse in (True, False):
        eng = _CpuEngine(_Obs(Y, Wx), b.numpy(), sigma)
        sol = IJSlabSolver(_Obs(Y, Wx), S0, C0, dist=_SoloDist, engine=eng, fuse=fuse)
        assert sol.fuse == fuse
        sol.run(ITERS)
        out.append((sol.S.clone(), sol.C.clone(), eng.calls.count("scpass")))
    assert out[0][2] == ITERS - 1 and out[1][2] == 0
    assert torch.equal(out[0][0], out[1][0]) and torch.equal(out[0][1], out[1][1])


def _global_problem_cpu(I_=12, J_=10, K_=16, R_=3, seed=5):
    """A global problem dict with the keys synthetic.onebit_problem returns (CPU tensors)."""
    g = torch.Generator().manual_seed(seed)
    S_true = torch.rand(R_, 1, I_, J_, generator=g)
    C_true = torch.rand(R_, K_, generator=g)
    T_true = ro.get_tensor(S_true, C_true)
    return dict(S_true=S_true, C_true=C_true, T_true=T_true,
                Y=(T_true > T_true.median()).long().unsqueeze(1),
                Wx=torch.bernoulli(torch.full((K_, 1, I_, J_), 0.3), generator=g),
                S0=0.5 * torch.rand(R_, 1, I_, J_, generator=g),
                C0=0.5 * torch.rand(R_, K_, generator=g),
                b=torch.tensor([0.0, float(T_true.median()), float(T_true.max())]),
                sigma=0.1, log_model=False, offset=0.0)


def _split_worker(rank, world, port, out_path):
    """Each rank takes its strong-scaling shard of the same global problem (bench.py
    --scaling strong); the shards are all-gathered over gloo and must reassemble it."""
    from quantized_spectrum_cartography_amd.synthetic import split_problem
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        glob = _global_problem_cpu()
        ok = {}
        for shard, axis_of in (("ijslab", dict(S_true=-2, S0=-2, Y=-2, Wx=-2, T_true=-2)),
                               ("kslab", dict(Y=0, Wx=0, T_true=0, C_true=1, C0=1))):
            sh = split_problem(glob, rank, world, shard)
            for key, ax in axis_of.items():
                parts = [torch.empty_like(sh[key]) for _ in range(world)]
                dist.all_gather(parts, sh[key].contiguous())
                ok["%s_%s" % (shard, key)] = bool(torch.equal(torch.cat(parts, dim=ax), glob[key]))
            # the replicated blocks are the global ones
            rep = ("C_true", "C0") if shard == "ijslab" else ("S_true", "S0")
            for key in rep:
                ok["%s_%s_replicated" % (shard, key)] = bool(torch.equal(sh[key], glob[key]))
        np.savez(out_path + ".r%d" % rank, names=np.array(sorted(ok)),
                 vals=np.array([ok[k] for k in sorted(ok)]))
    finally:
        dist.destroy_process_group()


def test_strong_split_union_is_global_problem(tmp_path):
    out = str(tmp_path / "split")
    mp.start_processes(_split_worker, args=(2, _free_port(), out), nprocs=2, join=True,
                       start_method="spawn")
    for r in range(2):
        d = np.load(out + ".r%d.npz" % r)
        bad = [str(n) for n, v in zip(d["names"], d["vals"]) if not v]
        assert not bad, bad
    # uneven splits (C4 at N = 3, say) cover every row / bin exactly once
    from quantized_spectrum_cartography_amd.synthetic import split_problem
    glob = _global_problem_cpu(I_=13, K_=17)
    for shard, ax in (("ijslab", -2), ("kslab", 0)):
        parts = [split_problem(glob, r, 3, shard)["Y"] for r in range(3)]
        assert torch.equal(torch.cat(parts, dim=ax), glob["Y"])
