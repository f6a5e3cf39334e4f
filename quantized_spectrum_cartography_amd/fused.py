"""Fused likelihood + gradient passes over packed observations (the hot path).

One *grad-step*  is one pass plus the update of the block it
differentiates:
  C-step:  qsc_cpass (per-tile dC partials)  ->  qsc_cfinish (fixed-order reduction,
           + lambda_c C/||C||, Adam, C[C<0] = 0)               qmc/qmc.ipynb :562-579
  S-step:  qsc_spass (dS in registers, + lambda_s S/||S||, Adam fused in the epilogue)
                                                                qmc/qmc.ipynb :622-634
Scalars (step counters, ||S||^2, NLLs, the cost history) stay on the device and their
book-keeping rides on those same kernels (qsc_state protocol in include/qsc.h), so an outer
iteration is three launches with no host synchronisation and is captured in one hipGraph.
qsc_scpass runs an S-step and the following C-pass as one launch (the C-pass of iteration i+1
reads only its tile's S_i, handed over in LDS), so solvers issue two launches per iteration.
"""
import torch

from . import _lib
from ._model import _dev, _ws


class PassEngine:
    """Workspace + device state for running the fused passes on one Observations set."""

    def __init__(self, obs, R, hist_cap=0):
        if not 1 <= R <= _lib.QSC_MAX_R:
            raise ValueError("rank R must be in [1, %d]" % _lib.QSC_MAX_R)
        self.obs, self.R = obs, R
        # the packed entries at this rank (signed rows, or a code-field copy: obs.layout)
        self.desc, self.s_entries, self.c_entries = obs.layout(R)
        dev = obs.device
        nb = _lib.lib().qsc_pass_workspace_bytes(self.desc, R)
        if nb == 0:
            raise _lib.QscError("invalid observation descriptor")
        # zeroed once: the S-pass keeps its slice scheduler words in the workspace and leaves
        # them zero at exit (include/qsc.h, qsc_pass_workspace_bytes)
        self.ws = torch.zeros(max(int(nb), 1), dtype=torch.uint8, device=dev)
        self.state = torch.zeros(_lib.STATE_BYTES, dtype=torch.uint8, device=dev)
        self.hist_cap = int(hist_cap)
        self.hist = torch.zeros(max(4 * self.hist_cap, 4), dtype=torch.float32, device=dev)
        # workspace generation: bumped by every launch that writes the workspace's pass partials
        # (slab, NLL / norm partials, cnsq) or C, so a solver can tell that a C-pass it left
        # ahead in the workspace was overwritten since (qmc.FreeSSolver.ahead)
        self.gen = 0

    # ---- state --------------------------------------------------------------------------
    def init_state(self, S_pos):
        ws = _ws(256 * 8, S_pos.device)
        _lib.call("qsc_state_init", _lib.ptr(self.state), _lib.ptr(S_pos), self.R, self.obs.Pp,
                  _lib.ptr(ws), ws.numel(), _lib.stream())

    def read_state(self):
        return _lib.read_state(self.state)

    def field(self, name):
        return _lib.state_field(self.state, name)

    # ---- passes -------------------------------------------------------------------------
    def cpass(self, S_pos, C):
        self.gen += 1
        o = self.obs
        _lib.call("qsc_cpass", self.desc, _lib.ptr(self.c_entries), _lib.ptr(o.c_width), _lib.ptr(o.c_off),
                  _lib.ptr(o.c_kmap), o.model, self.R, _lib.ptr(S_pos), _lib.ptr(C),
                  _lib.ptr(self.ws), self.ws.numel(), _lib.stream())

    def cpass_nsq(self, S_pos, C):
        """cpass that also writes every slice's ||S||^2 partial (qsc_cpass_nsq: the K-slab
        C-pass after the all-gather of S, in place of a qsc_slice_nsq launch)."""
        self.gen += 1
        o = self.obs
        _lib.call("qsc_cpass_nsq", self.desc, _lib.ptr(self.c_entries), _lib.ptr(o.c_width),
                  _lib.ptr(o.c_off), _lib.ptr(o.c_kmap), o.model, self.R, _lib.ptr(S_pos),
                  _lib.ptr(C), _lib.ptr(self.ws), self.ws.numel(), _lib.stream())

    def cnsq(self):
        """A 1-float view of the workspace slot where the C-pass leaves ||C||^2 of the C it
        read (qsc_pass_cnsq_offset): all-reduced in place by the K-slab solver."""
        off = int(_lib.lib().qsc_pass_cnsq_offset(self.desc, self.R))
        if off < 0 or off % 4:
            raise _lib.QscError("qsc_pass_cnsq_offset failed")
        return self.ws[off:off + 4].view(torch.float32)

    def cfinish(self, C, mode, dC=None, mC=None, vC=None, adam=None, lambda_c=0.0,
                normsq_ext=None, record=True):
        self.gen += 1
        hist, cap = (self.hist, self.hist_cap) if (record and self.hist_cap) else (None, 0)
        _lib.call("qsc_cfinish", self.desc, self.R, _lib.ptr(C), int(mode), _lib.ptr(dC),
                  _lib.ptr(mC), _lib.ptr(vC), adam, float(lambda_c), _lib.ptr(normsq_ext),
                  _lib.ptr(self.state), _lib.ptr(hist), cap, _lib.ptr(self.ws), self.ws.numel(),
                  _lib.stream())

    def spass(self, S_pos, C, mode, dS=None, mS=None, vS=None, adam=None, lambda_s=0.0):
        self.gen += 1
        o = self.obs
        _lib.call("qsc_spass", self.desc, _lib.ptr(self.s_entries), _lib.ptr(o.s_width), _lib.ptr(o.s_off),
                  o.model, self.R, _lib.ptr(S_pos), _lib.ptr(C), int(mode), _lib.ptr(dS),
                  _lib.ptr(mS), _lib.ptr(vS), adam, float(lambda_s), _lib.ptr(self.state),
                  _lib.ptr(self.ws), self.ws.numel(), _lib.stream())

    def spass_kslab(self, S_pos, C, dS_rs, chunk_rows, nranks):
        """K-slab S-pass (qsc_spass_kslab): the partial dS into the reduce-scatter buffer dS_rs
        (nranks chunks of chunk_rows rows, each followed by one extra slice holding this slab's
        ||C||^2 in its first element)."""
        self.gen += 1
        o = self.obs
        u = _lib.QSC_SLICE
        if chunk_rows % u:
            raise ValueError("K-slab chunks must be whole position slices")
        _lib.call("qsc_spass_kslab", self.desc, _lib.ptr(self.s_entries), _lib.ptr(o.s_width),
                  _lib.ptr(o.s_off), o.model, self.R, _lib.ptr(S_pos), _lib.ptr(C),
                  _lib.ptr(dS_rs), chunk_rows // u, int(nranks), _lib.ptr(self.state),
                  _lib.ptr(self.ws), self.ws.numel(), _lib.stream())

    def scpass_supported(self):
        return bool(_lib.lib().qsc_scpass_supported(self.desc, self.R))

    def scpass(self, S_pos, C, mS, vS, adam, lambda_s):
        """spass (mode 1, Adam) fused with the next cpass at the updated S (qsc_scpass)."""
        self.gen += 1
        o = self.obs
        _lib.call("qsc_scpass", self.desc, _lib.ptr(self.s_entries), _lib.ptr(o.s_width),
                  _lib.ptr(o.s_off), _lib.ptr(self.c_entries), _lib.ptr(o.c_width),
                  _lib.ptr(o.c_off), _lib.ptr(o.c_kmap), o.model, self.R, _lib.ptr(S_pos),
                  _lib.ptr(C), _lib.ptr(mS),
                  _lib.ptr(vS), adam, float(lambda_s), _lib.ptr(self.state), _lib.ptr(self.ws),
                  self.ws.numel(), _lib.stream())

    def supdate(self, S_pos, mS, vS, g, adam, lambda_s):
        self.gen += 1
        _lib.call("qsc_supdate", self.desc, self.R, _lib.ptr(S_pos), _lib.ptr(mS), _lib.ptr(vS),
                  _lib.ptr(g), adam, float(lambda_s), _lib.ptr(self.state), _lib.ptr(self.ws),
                  self.ws.numel(), _lib.stream())

    # K-slab shards: rows are dealt in whole position slices
    row_unit = _lib.QSC_SLICE

    def supdate_rows(self, S_pos, mS, vS, g_own, adam, lambda_s, r0, r1):
        """Adam on position rows [r0, r1) (multiples of QSC_SLICE) from the shard's gradient
        g_own (its first row is row r0) -- qsc_supdate_slices."""
        self.gen += 1
        u = _lib.QSC_SLICE
        if r0 % u or (r1 % u and r1 != self.obs.Pp):
            raise ValueError("shard rows must be whole position slices")
        _lib.call("qsc_supdate_slices", self.desc, self.R, r0 // u, -(-r1 // u), _lib.ptr(S_pos),
                  _lib.ptr(mS), _lib.ptr(vS), _lib.ptr(g_own), adam, float(lambda_s),
                  _lib.ptr(self.state), _lib.ptr(self.ws), self.ws.numel(), _lib.stream())

    def slice_nsq(self, S_pos):
        """Every slice's ||S||^2 partial from the (all-gathered) S -- qsc_slice_nsq."""
        self.gen += 1
        _lib.call("qsc_slice_nsq", self.desc, self.R, _lib.ptr(S_pos), _lib.ptr(self.ws),
                  self.ws.numel(), _lib.stream())

    def cupdate(self, C, mC, vC, g, adam, lambda_c, normsq_s_ext=None):
        """C update from an all-reduced gradient g (R*K [+1]) (IJ-slab sharding)."""
        self.gen += 1
        _lib.call("qsc_cupdate", self.R, self.obs.K, _lib.ptr(C), _lib.ptr(mC), _lib.ptr(vC),
                  _lib.ptr(g), adam, float(lambda_c), _lib.ptr(normsq_s_ext),
                  _lib.ptr(self.state), _lib.stream())

    def sumsq(self, x, out):
        """out[0] = ||x||^2 (fixed order, one workgroup; for small vectors such as C)."""
        _lib.call("qsc_sumsq_small", _lib.ptr(x), x.numel(), _lib.ptr(out), _lib.stream())

    def flush(self, record=True):
        hist, cap = (self.hist, self.hist_cap) if (record and self.hist_cap) else (None, 0)
        _lib.call("qsc_state_flush", self.desc, self.R, _lib.ptr(self.state), _lib.ptr(hist),
                  cap, _lib.ptr(self.ws), self.ws.numel(), _lib.stream())

    # ---- composite ----------------------------------------------------------------------
    def nll_grad(self, S_pos, C, need_dS=True, need_dC=True):
        """NLL (device scalar) and its gradients dS (position order) and dC, no regularisers."""
        dS = torch.empty_like(S_pos) if need_dS else None
        dC = torch.empty_like(C) if need_dC else None
        if need_dC or not need_dS:
            self.cpass(S_pos, C)
            self.cfinish(C, 0, dC=dC if need_dC else torch.empty_like(C), record=False)
        if need_dS:
            self.spass(S_pos, C, 0, dS=dS)
            self.flush(record=False)
            nll = self.field("nll_s").clone()[0]
        else:
            nll = self.field("nll_c").clone()[0]
        return nll, dS, dC


class _ProbitNLLFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, S, C, obs):
        R = S.shape[0]
        eng = PassEngine(obs, R)
        Cd = _dev(C.detach().to(torch.float32)).contiguous()
        S_pos = obs.to_positions(S.detach().reshape(R, -1))
        nll, dS_pos, dC = eng.nll_grad(S_pos, Cd, ctx.needs_input_grad[0], ctx.needs_input_grad[1])
        dS = obs.to_pixels(dS_pos, R).reshape(S.shape) if dS_pos is not None else None
        ctx.save_for_backward(*(t for t in (dS, dC) if t is not None))
        ctx.has = (dS is not None, dC is not None)
        return nll

    @staticmethod
    def backward(ctx, g):
        saved = list(ctx.saved_tensors)
        dS = saved.pop(0) * g if ctx.has[0] else None
        dC = saved.pop(0) * g if ctx.has[1] else None
        return dS, dC, None


class ProbitNLL:
    """-sum(Wx * log(prob_probit(Y, T_hat, b, std))) with T_hat = get_tensor(S, C) (optionally
    log(T_hat + offset)), evaluated by the fused HIP passes over observed entries only.

    Replaces the reference's get_tensor -> log -> prob_probit -> log -> masked sum chain
    (qmc/qmc.ipynb :568-572) and its autograd backward.  Usage:
        nll = ProbitNLL.apply(S, C, obs); (nll + lam*torch.norm(C)).backward()
    """

    @staticmethod
    def apply(S, C, obs):
        if S.dim() == 3:
            S = S.unsqueeze(1)
        return _ProbitNLLFn.apply(S, C, obs)
