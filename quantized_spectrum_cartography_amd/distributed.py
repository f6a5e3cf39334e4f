"""Multi-GPU sharding of the alternating solver over RCCL (torch.distributed, backend "nccl").

Two layouts, both one process per GPU:

IJ-slab (bench.py's default for N > 1): rank g owns a block of pixels — its observations
Y[:, pixels] and its rows of S — and a replica of C (R x K, 8 KB at C3).  Per outer iteration
  C-step: local C-pass and slab reduction (qsc_cfinish mode 2), one all-reduce of
          [dC_local | ||S_local||^2] (R*K + 1 floats), the replicated C update (qsc_cupdate);
  S-step: the fused local S-pass (likelihood, dS, Adam), whose lambda_s ||S||_F regulariser
          uses the all-reduced ||S||^2 delivered by the C-step's collective.
One small collective per iteration; S never crosses the fabric.

K-slab (the north-star layout): rank g owns the frequency bins [k0, k1) — its
slab of the observations Y[k0:k1] and of the spectra C[:, k0:k1] — and a replica of S.  Per
outer iteration
  C-step: local C-pass (qsc_cpass_nsq: it also leaves the slab's ||C||^2 in its workspace and
          rebuilds every slice's ||S||^2 partial from the S tile it stages); the non-squared
          regulariser lambda_c ||C||_F needs the GLOBAL ||C||^2, so the ranks all-reduce that
          one float in place before the fused cfinish (Adam + projection);
  S-step: local S-pass in gradient mode (qsc_spass_kslab: partial dS over the slab's bins,
          written in the reduce-scatter layout -- N chunks of whole position slices, each
          followed by one extra slice that carries this slab's ||C_new||^2, the norm of the C
          the pass read); a REDUCE-SCATTER of that buffer (Pp x RP fp32, 8.4 MB at 512x512,
          R = 8) leaves rank g the summed gradient of its 1/N of the position slices AND the
          global ||C||^2 the next C-step's regulariser needs; Adam on the owned rows only
          (qsc_supdate_slices: 1/N of the S/mS/vS traffic); an ALL-GATHER of the updated shards
          (in place in S) re-replicates S; the next C-pass rebuilds the per-slice ||S_new||^2
          partials from the gathered S (bit-identical to the ones the shard updates produced),
          so the regulariser norm of the next step is the same on all ranks without another
          collective (before a final flush, history() runs qsc_slice_nsq for the last iteration).
          Same bytes on the fabric as one all-reduce, 1/N of the Adam traffic per rank.
An iteration is 4 kernels (cpass_nsq, cfinish, spass_kslab, supdate_slices) and 2 collectives
(reduce-scatter and all-gather of S-sized buffers).  The ||C||^2 rides on the reduce-scatter:
only the first C-step of a run, whose C no S-pass has normed yet (C may have been changed by
the caller between runs), all-reduces the C-pass's ||C_slab||^2 itself.
The next C-pass reads every tile's new S rows, which exist only after the all-gather, so the
S update cannot be fused into it the way qsc_scpass fuses IJ-slab's.
The pixel order of S (positions) is derived from the GLOBAL per-pixel observation counts
(all-reduced once at setup) so that every rank lays S out identically.

The class is written against a small engine interface (fused.PassEngine on the GPU) so that the
sharding logic is exercised by world-size-2 gloo tests on the CPU with an emulated engine.
"""
import math

import torch

from . import _lib
from ._model import _dev
from .qmc import issue_iterations, prepare_iterations, run_iterations


def kslab_bounds(K, world, rank):
    """Contiguous, balanced split of K frequency bins over `world` ranks."""
    base, extra = divmod(K, world)
    k0 = rank * base + min(rank, extra)
    return k0, k0 + base + (1 if rank < extra else 0)


def kslab_observations(Y_local, Wx_local, bin_boundaries, noise_std, dist, offset=0.0,
                       log_model=False, tile=None, R_hint=8):
    """Observations of this rank's K-slab with the pixel order of the global counts."""
    from .obs import Observations

    def hook(cnt):
        dist.all_reduce(cnt)
        return cnt
    return Observations(Y_local, Wx_local, bin_boundaries, noise_std, offset=offset,
                        log_model=log_model, tile=tile, R_hint=R_hint, count_hook=hook)



def _capturable(dist):
    """hipGraph capture of the iteration includes its collectives: RCCL ("nccl") can be
    captured, gloo (CPU rehearsals of the sharded bench on one GPU) cannot, and a failed
    capture leaves the stream unusable, so such process groups run eagerly from the start."""
    try:
        return dist.get_backend() == "nccl"
    except (RuntimeError, ValueError, AttributeError):
        return True

class IJSlabSolver:
    """Free-S alternating solver on one pixel block per rank (see module docstring)."""

    def __init__(self, obs, S_init_local, C_init, dist, lambda_c=100.0, lambda_s=100.0,
                 lr_c=5e-3, lr_s=1e-2, betas=(0.9, 0.999), eps=1e-8, project_c=True,
                 hist_cap=1024, engine=None, fuse=True):
        self.obs, self.dist = obs, dist
        R = S_init_local.shape[0]
        self.R = R
        if engine is None:
            from .fused import PassEngine
            engine = PassEngine(obs, R, hist_cap=hist_cap)
        self.engine = engine
        self.S = obs.to_positions(S_init_local.reshape(R, -1))
        dev = self.S.device
        self.C = C_init.detach().to(dev, torch.float32).reshape(R, obs.K).clone()
        self.mS, self.vS = torch.zeros_like(self.S), torch.zeros_like(self.S)
        self.mC, self.vC = torch.zeros_like(self.C), torch.zeros_like(self.C)
        # [dC_local (R*K) | ||S_local||^2]: the one all-reduced buffer of an iteration
        self.red = torch.zeros(R * obs.K + 1, dtype=torch.float32, device=dev)
        self.adam_c = _lib.make_adam(lr_c, betas, eps, project_nonneg=project_c)
        self.adam_s = _lib.make_adam(lr_s, betas, eps, project_nonneg=False)
        self.lambda_c, self.lambda_s = float(lambda_c), float(lambda_s)
        self.engine.init_state(self.S)
        # S-step + next C-pass in one launch (qsc_scpass), as FreeSSolver
        sup = getattr(self.engine, "scpass_supported", None)
        self.fuse = bool(fuse) and sup is not None and bool(sup())
        self._graphs = {}
        self.graph_tolerant, self.graph_error = True, None  # see qmc._capture
        self.graph_capturable = _capturable(dist)
        if not self.graph_capturable:
            self.graph_error = "collectives over %s are not graph-capturable" % dist.get_backend()

    def fused_body(self):
        """S-step i + C-pass i+1 (one launch), then C-step i+1's exchange and update."""
        self.engine.scpass(self.S, self.C, self.mS, self.vS, self.adam_s, self.lambda_s)
        self._c_exchange()

    def _c_exchange(self):
        e = self.engine
        e.cfinish(self.C, 2, dC=self.red)
        self.dist.all_reduce(self.red)
        e.cupdate(self.C, self.mC, self.vC, self.red, self.adam_c, self.lambda_c,
                  normsq_s_ext=self.red[self.R * self.obs.K:])

    def c_step(self):
        self.engine.cpass(self.S, self.C)
        self._c_exchange()

    def s_step(self):
        self.engine.spass(self.S, self.C, 1, mS=self.mS, vS=self.vS, adam=self.adam_s,
                          lambda_s=self.lambda_s)

    def iteration(self):
        self.c_step()
        self.s_step()

    def issue(self, n):
        issue_iterations(self, n)

    def prepare(self, n):
        prepare_iterations(self, n)

    def run(self, n, use_graph=False):
        run_iterations(self, n, use_graph)

    def state(self):
        return self.engine.read_state()

    def S_pixels(self):
        """This rank's pixel block of S, (R, 1, I_local, J)."""
        return self.obs.to_pixels(self.S, self.R).reshape(self.R, 1, self.obs.I, self.obs.J)

    def history(self):
        """Global per-iteration costs (NLL columns summed over ranks; collective)."""
        e = self.engine
        e.flush()
        st = e.read_state()
        n = min(int(st["iter"]), e.hist_cap)
        h = e.hist[: 4 * n].view(n, 4).clone()
        nll = h[:, :2].contiguous()
        self.dist.all_reduce(nll)
        h = torch.cat([nll, h[:, 2:]], dim=1).double().cpu()
        nsq_c_final = float((self.C.double() ** 2).sum().item())
        costs_c, costs_s = [], []
        for i in range(n):
            nll_c, nll_s, nsq_c, nsq_s = h[i].tolist()
            nsq_c_next = h[i + 1][2].item() if i + 1 < n else nsq_c_final
            costs_c.append(nll_c + self.lambda_c * math.sqrt(nsq_c) + self.lambda_s * math.sqrt(nsq_s))
            costs_s.append(nll_s + self.lambda_c * math.sqrt(nsq_c_next) + self.lambda_s * math.sqrt(nsq_s))
        return costs_c, costs_s


class KSlabSolver:
    """Free-S alternating solver on one K-slab per rank (see module docstring)."""

    def __init__(self, obs, S_init, C_init_local, dist, lambda_c=100.0, lambda_s=100.0,
                 lr_c=5e-3, lr_s=1e-2, betas=(0.9, 0.999), eps=1e-8, project_c=True,
                 hist_cap=1024, engine=None):
        self.obs, self.dist = obs, dist
        R = S_init.shape[0]
        self.R = R
        if engine is None:
            from .fused import PassEngine
            engine = PassEngine(obs, R, hist_cap=hist_cap)
        self.engine = engine
        S_pos = obs.to_positions(S_init.reshape(R, -1))
        dev = S_pos.device
        # shards of whole position slices (the engine's row unit): rank g owns rows
        # [g*chunk, (g+1)*chunk) of S; S, dS are padded to N*chunk rows so that the
        # reduce-scatter / all-gather move equal contiguous chunks (padding rows stay zero)
        ws = dist.get_world_size()
        self.rank = dist.get_rank() if ws > 1 else 0
        unit = getattr(engine, "row_unit", 1)
        Pp = S_pos.shape[0]
        units = -(-Pp // unit)
        self.chunk = -(-units // ws) * unit
        self.r0 = min(self.rank * self.chunk, Pp)
        self.r1 = min(self.r0 + self.chunk, Pp)
        rows = ws * self.chunk
        self.S_buf = torch.zeros((rows,) + tuple(S_pos.shape[1:]), dtype=torch.float32, device=dev)
        self.S_buf[:Pp] = S_pos
        self.S = self.S_buf[:Pp]
        # the reduce-scatter buffer: ws chunks of `chunk` gradient rows, each followed by one
        # extra slice (`unit` rows) whose first element carries this slab's ||C||^2
        # (qsc_spass_kslab); the rest of the extra slices stays zero
        self.unit = unit
        self.nranks = ws
        self.dS_buf = torch.zeros((ws * (self.chunk + unit),) + tuple(S_pos.shape[1:]),
                                  dtype=torch.float32, device=dev)
        self.dS_own = torch.zeros((self.chunk + unit,) + tuple(S_pos.shape[1:]),
                                  dtype=torch.float32, device=dev)
        # the global ||C||^2 the reduce-scatter delivers (1-float view of this rank's extra slice)
        self.nsq_rs = self.dS_own[self.chunk].reshape(-1)[:1]
        self.C = C_init_local.detach().to(dev, torch.float32).reshape(R, obs.K).clone()
        self.mS, self.vS = torch.zeros_like(self.S), torch.zeros_like(self.S)
        self.mC, self.vC = torch.zeros_like(self.C), torch.zeros_like(self.C)
        # the C-pass's ||C_slab||^2 slot (all-reduced in place each C-step)
        cn = getattr(engine, "cnsq", None)
        self.nsq_c = cn() if cn is not None else torch.zeros(1, dtype=torch.float32, device=dev)
        self.adam_c = _lib.make_adam(lr_c, betas, eps, project_nonneg=project_c)
        self.adam_s = _lib.make_adam(lr_s, betas, eps, project_nonneg=False)
        self.lambda_c, self.lambda_s = float(lambda_c), float(lambda_s)
        self.engine.init_state(self.S)
        self._graphs = {}
        self.graph_tolerant, self.graph_error = True, None  # see qmc._capture
        self.graph_capturable = _capturable(dist)
        if not self.graph_capturable:
            self.graph_error = "collectives over %s are not graph-capturable" % dist.get_backend()

    def begin_run(self):
        """(issue_iterations, at the start of every run): the run's first C-step all-reduces
        the C-pass's ||C_slab||^2, later ones take the one the reduce-scatter delivered."""
        self._rs_norm = False

    def c_step(self):
        e = self.engine
        e.cpass_nsq(self.S, self.C)  # + ||C_slab||^2 into nsq_c, + the slices' ||S||^2
        if getattr(self, "_rs_norm", False):
            nsq = self.nsq_rs  # global ||C||^2 from the previous S-step's reduce-scatter
        else:
            self.dist.all_reduce(self.nsq_c)
            nsq = self.nsq_c
        e.cfinish(self.C, 1, mC=self.mC, vC=self.vC, adam=self.adam_c, lambda_c=self.lambda_c,
                  normsq_ext=nsq)

    def s_step(self):
        e = self.engine
        # partial dS (+ ||C_slab||^2 of the updated C) in the reduce-scatter layout
        e.spass_kslab(self.S, self.C, self.dS_buf, self.chunk, self.nranks)
        # reduce-scatter -> Adam on the owned rows -> all-gather (in place in S_buf)
        self.dist.reduce_scatter_tensor(self.dS_own, self.dS_buf)
        e.supdate_rows(self.S, self.mS, self.vS, self.dS_own, self.adam_s, self.lambda_s,
                       self.r0, self.r1)
        lo = self.rank * self.chunk
        self.dist.all_gather_into_tensor(self.S_buf, self.S_buf[lo:lo + self.chunk])
        # (the next cpass_nsq rebuilds every slice's ||S_new||^2 partial from the gathered S)
        self._rs_norm = True

    def iteration(self):
        self.c_step()
        self.s_step()

    def issue(self, n):
        issue_iterations(self, n)

    def prepare(self, n):
        prepare_iterations(self, n)

    def run(self, n, use_graph=False):
        run_iterations(self, n, use_graph)

    def state(self):
        return self.engine.read_state()

    def S_pixels(self):
        return self.obs.to_pixels(self.S, self.R).reshape(self.R, 1, self.obs.I, self.obs.J)

    def C_global(self):
        """All ranks' C slabs concatenated along K (collective)."""
        return torch.cat(self._all_gather_var(self.C), dim=1)

    def _all_gather_var(self, C):
        ws = self.dist.get_world_size()
        k = torch.tensor([C.shape[1]], device=C.device)
        ks = [torch.zeros_like(k) for _ in range(ws)]
        self.dist.all_gather(ks, k)
        kmax = max(int(x.item()) for x in ks)
        pad = torch.zeros((C.shape[0], kmax), dtype=C.dtype, device=C.device)
        pad[:, :C.shape[1]] = C
        outs = [torch.empty_like(pad) for _ in range(ws)]
        self.dist.all_gather(outs, pad)
        return [o[:, :int(kk.item())] for o, kk in zip(outs, ks)]

    def history(self):
        """Global per-iteration costs (NLL columns summed over ranks; collective)."""
        e = self.engine
        e.slice_nsq(self.S)  # the last S update's partials (no C-pass has run since)
        e.flush()
        st = e.read_state()
        n = min(int(st["iter"]), e.hist_cap)
        h = e.hist[: 4 * n].view(n, 4).clone()
        nll = h[:, :2].contiguous()
        self.dist.all_reduce(nll)
        h = torch.cat([nll, h[:, 2:]], dim=1).double().cpu()
        nsq = torch.zeros(1, dtype=torch.float32, device=self.C.device)
        e.sumsq(self.C, nsq)
        self.dist.all_reduce(nsq)
        nsq_c_final = float(nsq.item())
        costs_c, costs_s = [], []
        for i in range(n):
            nll_c, nll_s, nsq_c, nsq_s = h[i].tolist()
            nsq_c_next = h[i + 1][2].item() if i + 1 < n else nsq_c_final
            costs_c.append(nll_c + self.lambda_c * math.sqrt(nsq_c) + self.lambda_s * math.sqrt(nsq_s))
            costs_s.append(nll_s + self.lambda_c * math.sqrt(nsq_c_next) + self.lambda_s * math.sqrt(nsq_s))
        return costs_c, costs_s
