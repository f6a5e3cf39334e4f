"""Alternating S/C maximum-likelihood solver — the drop-in for the qmc.py / qmc.ipynb solver.

The reference's solver is the notebook cell qmc/qmc.ipynb cell 1 (raw-JSON lines :422-653,
loop at :559-645); qmc/qmc.py is only its import preamble.  Per outer iteration it runs
  C-step (cinnerIter = 1):  cost = -sum(Wx log P(Y | T_hat(S, C))) + lambda_c ||C||_F
                            + lambda_s ||Z||_F;  Adam(lr 5e-3) on C;  C[C<0] = 0      (:562-579)
  S-step (sinnerIter = 1):  same cost;  Adam(lr 1e-2) on Z with S = G(Z)            (:622-634)
`solve` reproduces that loop in two modes:
  * free S (generator=None): S itself is the Adam variable with lambda_s ||S||_F, the form of
    backup/notebooks/onebit_lowrank.ipynb:1230-1236 (needed for maps that are not 51x51);
    every grad-step is a fused HIP pass with the Adam update on the device, no host sync.
  * generator (S = generator(Z)): the C-step is the fused HIP C-step; the S-step gets dS from
    the fused HIP S-pass and back-propagates it through the torch generator to Z (the
    reference's GAN path, Z optimised, network frozen: :547-550).
"""
import math
import warnings
from dataclasses import dataclass, field
from typing import List, Optional

import torch

from . import _lib
from ._model import _dev, map_nmse
from .fused import PassEngine
from .obs import Observations
from .utils import LOG_OFFSET_7_ADJUSTED as LOG_OFFSET


@dataclass
class SolveResult:
    S: torch.Tensor                     # (R, 1, I, J), natural pixel order
    C: torch.Tensor                     # (R, K)
    costs_c: List[float]                # cost evaluated in each C-step (before the update)
    costs_s: List[float]                # cost evaluated in each S-step (before the update)
    nmse: List[float] = field(default_factory=list)  # map NMSE after each tracked iteration
    Z: Optional[torch.Tensor] = None
    iters: int = 0
    fused: bool = False                 # S-step + next C-pass ran as one launch (qsc_scpass)


# Longest run captured as one hipGraph; longer runs replay several (results are identical:
# run(a) then run(b) equals run(a + b) bit for bit, tests/test_gpu_fused.py).
GRAPH_MAX_ITERS = 1024


def issue_iterations(solver, n):
    """Kernel sequence of n outer iterations of a solver with c_step / s_step / iteration and,
    when `solver.fuse`, fused_body (S-step i + C-pass i+1 in one launch, then C-step i+1's
    finish): c_step, fused_body x (n-1), s_step -- two launches per iteration.

    A solver with `chain` (FreeSSolver) ends a run with the fused launch instead of the
    stand-alone S-step: its last S-step also runs the NEXT iteration's C-pass, whose partials
    wait in the workspace (`ahead()`), and a following run starts with that C-pass's finish
    instead of a C-pass of its own.  The op sequence of run(a) then run(b) is then exactly that
    of run(a + b) -- c_step, fused_body x (a + b - 1), then the last S-step -- and every run of
    n iterations issues n fused launches and n C-step finishes (the steady state), where the
    stand-alone ends cost a C-pass and an S-pass per run."""
    if hasattr(solver, "begin_run"):
        solver.begin_run()
    if getattr(solver, "fuse", False) and getattr(solver, "chain", False) and n >= 1:
        if solver.ahead():
            solver.c_finish()
        else:
            solver.c_step()
        for _ in range(n - 1):
            solver.fused_body()
        solver.fused_last()
    elif getattr(solver, "fuse", False) and n >= 2:
        solver.c_step()
        for _ in range(n - 1):
            solver.fused_body()
        solver.s_step()
    else:
        for _ in range(n):
            solver.iteration()


# RCCL's watchdog thread (torch ProcessGroupNCCL) polls the completion events of the eager
# collectives still on its list every ~100 ms.  Polled while the collectives' stream is being
# captured, such an event fails the query ("operation not permitted on an event last recorded in
# a capturing stream") and the watchdog aborts the process -- seen on MI355X when a capture
# followed an eager collective within milliseconds (profiles/r06/capture_watchdog_abort.log).
# Before capturing collectives: drain the device, then let the watchdog retire its list.
CAPTURE_QUIESCE_S = 0.3


def quiesce_collectives(dist):
    try:
        nccl = dist is not None and dist.is_initialized() and dist.get_backend() == "nccl"
    except (AttributeError, RuntimeError, ValueError):  # (a stand-in process group)
        nccl = False
    if not nccl:
        return
    import time
    torch.cuda.synchronize()
    time.sleep(CAPTURE_QUIESCE_S)


def _capture(solver, n, tolerant):
    """Capture run(n)'s kernel sequence into a hipGraph on a side stream.

    A capture that fails part-way (an engine error, an illegal synchronisation, a collective
    that cannot be captured) is abandoned cleanly: any capture still open on the side stream or
    the current stream is ended and its graph destroyed, and the device is synchronised, BEFORE
    anything else is issued -- work issued onto a stream that is still capturing would be
    recorded instead of run, and a collective there fails ("operation not permitted when stream
    is capturing").  Then, for a tolerant solver, the failure is recorded in `graph_error`, the
    solver is marked not capturable and runs eagerly from then on; otherwise the error is
    re-raised.  If the capture cannot be ended the error is always raised."""
    quiesce_collectives(getattr(solver, "dist", None))
    g = torch.cuda.CUDAGraph()
    s = capture_stream()
    caller = torch.cuda.current_stream()
    s.wait_stream(caller)
    mark = solver.chain_mark() if hasattr(solver, "chain_mark") else None
    try:
        with torch.cuda.stream(s):
            # thread-local capture mode: other threads' HIP calls (RCCL's watchdog queries the
            # events of collectives issued before the capture) must neither fail nor invalidate
            # it -- in the default global mode the watchdog's query errors and aborts the process
            with torch.cuda.graph(g, stream=s, capture_error_mode="thread_local"):
                issue_iterations(solver, n)
    except Exception as e:  # noqa: BLE001 - every failure takes the same clean-up path
        if mark is not None:
            solver.chain_restore(mark)
        err = "%s: %s" % (type(e).__name__, e)
        del g
        abandon_capture(s, caller)  # raises if the caller's stream is left capturing
        if not tolerant:
            raise
        solver.graph_error = err
        solver.graph_capturable = False
        warnings.warn("hipGraph capture failed; running eagerly (%s)" % err, RuntimeWarning)
        return None
    if mark is not None:
        solver.chain_restore(mark)  # (capturing executes nothing: the device state is unchanged)
    torch.cuda.current_stream().wait_stream(s)
    _upload(g)
    return g


_hip = None


def _hip_lib():
    global _hip
    if _hip is None:
        import ctypes
        h = ctypes.CDLL("libamdhip64.so")
        h.hipGraphUpload.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        h.hipGraphUpload.restype = ctypes.c_int
        h.hipStreamIsCapturing.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)]
        h.hipStreamIsCapturing.restype = ctypes.c_int
        h.hipStreamEndCapture.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p)]
        h.hipStreamEndCapture.restype = ctypes.c_int
        h.hipGraphDestroy.argtypes = [ctypes.c_void_p]
        h.hipGraphDestroy.restype = ctypes.c_int
        h.hipGetLastError.argtypes = []
        h.hipGetLastError.restype = ctypes.c_int
        _hip = h
    return _hip


def capture_stream():
    """A side stream that is not in a capture: torch hands out streams from a fixed pool
    (round robin), and a stream whose capture was invalidated stays invalidated for good
    (abandon_capture), so after a failed capture the pool can return such a stream again;
    skip those."""
    for _ in range(4 * 32 + 1):  # torch's pool holds 32 streams per priority
        s = torch.cuda.Stream()
        if stream_capture_status(s) == 0:
            return s
    raise RuntimeError("no side stream out of capture for hipGraph capture")


def stream_capture_status(stream):
    """0 = not capturing, 1 = capture active, 2 = capture invalidated (hipStreamCaptureStatus)."""
    import ctypes
    st = ctypes.c_int(0)
    rc = _hip_lib().hipStreamIsCapturing(ctypes.c_void_p(stream.cuda_stream), ctypes.byref(st))
    return st.value if rc == 0 else -1  # -1: the query itself failed (treated as capturing)


def abandon_capture(side, caller):
    """Clean up after a capture on `side` failed: end (and discard) the capture still open on
    it, clear the HIP error state and synchronise the device.  HIP leaves a stream whose
    capture was invalidated in the invalidated state for good (measured, tools/probe/
    capture_fail.py: hipStreamEndCapture returns an error and the status stays 2), so the side
    stream is abandoned -- captures always use a fresh one -- and only the caller's stream,
    where eager work continues, must be out of capture.  Raises RuntimeError otherwise."""
    import ctypes
    h = _hip_lib()
    if stream_capture_status(side) != 0:
        graph = ctypes.c_void_p(None)
        h.hipStreamEndCapture(ctypes.c_void_p(side.cuda_stream), ctypes.byref(graph))
        if graph.value:
            h.hipGraphDestroy(graph)
    h.hipGetLastError()  # clear the (non-sticky) capture error
    if stream_capture_status(caller) != 0:
        raise RuntimeError("a failed hipGraph capture left the caller's stream capturing")
    torch.cuda.synchronize()
    h.hipGetLastError()


def _upload(g):
    """hipGraphUpload the instantiated graph now, so that its first replay does not pay the
    upload (a fixed ~tens of us that would otherwise land in a short timed run)."""
    try:
        ex = g.raw_cuda_graph_exec()
        rc = _hip_lib().hipGraphUpload(ex, torch.cuda.current_stream().cuda_stream)
        if rc != 0:
            raise RuntimeError("hipGraphUpload returned %d" % rc)
        torch.cuda.current_stream().synchronize()
    except (OSError, AttributeError, RuntimeError) as e:  # upload is an optimisation only
        warnings.warn("hipGraphUpload skipped (%s)" % e, RuntimeWarning)


def graph_for(solver, n):
    """The hipGraph of the exact kernel sequence of run(n) from the solver's current state
    (captured once per n and, for a chaining solver, per whether a C-pass is ahead)."""
    graphs = solver.__dict__.setdefault("_graphs", {})
    if getattr(solver, "graph_capturable", True) is False:
        return None  # eager (the reason is in solver.graph_error)
    key = (n, solver.ahead()) if hasattr(solver, "ahead") else n
    # a graph holds its tensors' addresses: a solver whose state tensors were swapped for others
    # (sol.C = ...) captures anew instead of replaying into the old storage
    ptrs = tuple(t.data_ptr() for t in (getattr(solver, a, None) for a in _STATE_TENSORS)
                 if isinstance(t, torch.Tensor))
    if solver.__dict__.get("_graph_ptrs") != ptrs:
        graphs.clear()
        solver._graph_ptrs = ptrs
    if key not in graphs:
        graphs[key] = _capture(solver, n, getattr(solver, "graph_tolerant", False))
    return graphs[key]


_STATE_TENSORS = ("S", "C", "mS", "vS", "mC", "vC", "S_buf", "dS_buf", "dS_own", "red")


def graph_chunks(n):
    """The graph lengths run(n) replays, in order: 1024-iteration chunks, then the remainder."""
    out = []
    while n > 0:
        m = min(n, GRAPH_MAX_ITERS)
        out.append(m)
        n -= m
    return out


def prepare_iterations(solver, n):
    """Capture (without executing) every graph that run(n, use_graph=True) will replay, so a
    later timed run(n) captures, instantiates and uploads nothing."""
    if not hasattr(solver, "chain_mark"):
        for m in sorted(set(graph_chunks(n))):
            graph_for(solver, m)
        return
    # A chaining solver's graphs are keyed by whether a C-pass is ahead: run(n) from the current
    # state replays (m, ahead()) for its first chunk and (m, True) for the later ones, and a later
    # run(n) starts with a C-pass ahead.  Capture both entry forms of every chunk size, so no
    # later run(n) captures anything whatever state it starts from.
    mark = solver.chain_mark()
    for m in sorted(set(graph_chunks(n))):
        for a in (False, True):
            if solver.chain_force(a):
                graph_for(solver, m)
    solver.chain_restore(mark)


def run_iterations(solver, n, use_graph):
    """run(n): eager, or as replays of whole-run hipGraphs (one replay when n <= 1024), so the
    device work of a timed run(n) does not depend on how earlier runs were split."""
    if not (use_graph and torch.cuda.is_available() and solver.S.is_cuda):
        issue_iterations(solver, n)
        return
    for m in graph_chunks(n):
        g = graph_for(solver, m)
        if g is None:
            issue_iterations(solver, m)
        else:
            g.replay()
            if hasattr(solver, "chain_replayed"):
                solver.chain_replayed()


class FreeSSolver:
    """Device-resident free-S alternating solver over one Observations set.

    State (position-ordered S, Adam moments, step counters, ||S||^2, NLLs) lives on the GPU.
    An iteration is cpass, cfinish (C-step) then spass (S-step).  With `fuse` (default where
    qsc_scpass_supported) `run(n)` issues the same kernel sequence with each S-step and the
    following C-pass in one launch: cpass, cfinish, (scpass, cfinish) x (n-1), spass -- two
    launches per iteration.  With `use_graph` the whole sequence of run(n) is captured once per
    n in a hipGraph (torch.cuda.CUDAGraph) and replayed; `prepare(n)` captures it ahead.
    """

    def __init__(self, obs, S_init, C_init, lambda_c=100.0, lambda_s=100.0, lr_c=5e-3, lr_s=1e-2,
                 betas=(0.9, 0.999), eps=1e-8, project_c=True, hist_cap=1024, fuse=True,
                 T_true=None, nmse_every=0, project_s=None, chain=True):
        self.obs = obs
        R = S_init.shape[0]
        self.R = R
        self.engine = PassEngine(obs, R, hist_cap=hist_cap)
        self.S = obs.to_positions(S_init.reshape(R, -1))
        self.C = _dev(C_init.detach().to(torch.float32)).reshape(R, obs.K).clone()
        self.mS, self.vS = torch.zeros_like(self.S), torch.zeros_like(self.S)
        self.mC, self.vC = torch.zeros_like(self.C), torch.zeros_like(self.C)
        self.adam_c = _lib.make_adam(lr_c, betas, eps, project_nonneg=project_c)
        # project_s: S >= 0 after every S-step (S[S<0] = 0, fused into the S-side Adam), the
        # domain of the reference's generator / decoder S (sigmoid outputs, deep_prior/networks/
        # dip.py:80).  Default (None): on under the log model, where T_hat + offset must stay > 0
        # -- unprojected free S drives T_hat + offset <= 0 within ~200 iterations at C5
        # (log of a non-positive value: a non-finite cost and S); off otherwise
        if project_s is None:
            project_s = bool(getattr(obs, "log_model", False))
        self.project_s = bool(project_s)
        self.adam_s = _lib.make_adam(lr_s, betas, eps, project_nonneg=self.project_s)
        self.lambda_c, self.lambda_s = float(lambda_c), float(lambda_s)
        self.engine.init_state(self.S)
        self.fuse = bool(fuse) and self.engine.scpass_supported()
        # chain: runs end with the fused launch (issue_iterations); `_ahead` says that the
        # workspace holds the C-pass of the next iteration at the current S, C (valid while
        # neither tensor was modified by torch since: their version counters)
        self.chain = bool(chain)
        self._ahead, self._ahead_ver = False, None
        self._graphs = {}
        # map NMSE after every `nmse_every`-th S-step, on the device inside the iteration
        # sequence (qsc_map_nmse_track; the reference evaluates it every iteration, :582, :637)
        self.nmse_every = int(nmse_every) if T_true is not None else 0
        if self.nmse_every:
            K, P = obs.K, obs.P
            self._T = _dev(T_true.detach().to(torch.float32)).reshape(K, P).contiguous()
            self._iperm = obs.iperm()
            self._nmse_hist = torch.zeros((max(hist_cap // self.nmse_every, 1), 2),
                                          dtype=torch.float64, device=self.S.device)
            self._nmse_ws = torch.empty(_lib.lib().qsc_reduce_workspace_bytes(0),
                                        dtype=torch.uint8, device=self.S.device)
    # one outer iteration = C grad-step + S grad-step
    def c_step(self):
        e = self.engine
        self._ahead = False
        e.cpass(self.S, self.C)
        e.cfinish(self.C, 1, mC=self.mC, vC=self.vC, adam=self.adam_c, lambda_c=self.lambda_c)

    def s_step(self):
        e = self.engine
        self._ahead = False
        e.spass(self.S, self.C, 1, mS=self.mS, vS=self.vS, adam=self.adam_s, lambda_s=self.lambda_s)
        self._track()

    # ---- run chaining (issue_iterations) ----
    def _chain_key(self):
        """What a C-pass left ahead depends on: S and C (their storage and torch version
        counters: an in-place torch write, or a fresh tensor swapped in) and the workspace it
        sits in (the engine's launch generation: any pass or finish launched on the engine since,
        by this solver or by a caller such as bench.time_kernel, may have overwritten it)."""
        return (self.S.data_ptr(), self.S._version, self.C.data_ptr(), self.C._version,
                self.engine.gen)

    def ahead(self):
        """True when the workspace holds the next iteration's C-pass at the current S, C."""
        return self.chain and self._ahead and self._ahead_ver == self._chain_key()

    def c_finish(self):
        """The C-step on the C-pass a previous run left ahead (its finish only)."""
        self._ahead = False
        self.engine.cfinish(self.C, 1, mC=self.mC, vC=self.vC, adam=self.adam_c,
                            lambda_c=self.lambda_c)

    def fused_last(self):
        """The run's last S-step, fused with the next iteration's C-pass (left ahead)."""
        e = self.engine
        e.scpass(self.S, self.C, self.mS, self.vS, self.adam_s, self.lambda_s)
        self._track()
        self.chain_replayed()

    def chain_replayed(self):
        """(after a replayed or issued chaining run: its last fused launch left a C-pass ahead)"""
        if self.chain and self.fuse:
            self._ahead, self._ahead_ver = True, self._chain_key()

    def chain_mark(self):
        return (self._ahead, self._ahead_ver, self.engine.gen)

    def chain_restore(self, mark):
        # (a capture issues launches without executing them: the engine's generation returns to
        # its value before the capture, so the captured run does not invalidate the state)
        self._ahead, self._ahead_ver, self.engine.gen = mark

    def chain_force(self, ahead):
        """Set the chaining state run() starts from (prepare: capture both entry forms)."""
        if ahead:
            self.chain_replayed()
        else:
            self._ahead = False
        return self.ahead() == bool(ahead)

    def iteration(self):
        self.c_step()
        self.s_step()

    def fused_body(self):
        """S-step i fused with C-pass i+1, then C-step i+1's finish (needs a C-step before)."""
        e = self.engine
        self._ahead = False
        e.scpass(self.S, self.C, self.mS, self.vS, self.adam_s, self.lambda_s)
        self._track()  # (S_{i+1}, C_{i+1}): C is updated by the cfinish below
        e.cfinish(self.C, 1, mC=self.mC, vC=self.vC, adam=self.adam_c, lambda_c=self.lambda_c)

    def _track(self):
        if not self.nmse_every:
            return
        o = self.obs
        _lib.call("qsc_map_nmse_track", _lib.ptr(self.S), _lib.ptr(self._iperm), self.S.shape[1],
                  _lib.ptr(self.C), _lib.ptr(self._T), self.R, o.P, o.K, 0, 0.0,
                  _lib.ptr(self.engine.state), self.nmse_every, _lib.ptr(self._nmse_hist),
                  self._nmse_hist.shape[0], _lib.ptr(self._nmse_ws), self._nmse_ws.numel(),
                  _lib.stream())

    def nmse_history(self):
        """Map NMSE after S-steps nmse_every, 2 nmse_every, ... recorded so far."""
        if not self.nmse_every:
            return []
        n = min(int(self.state()["iter"]) // self.nmse_every, self._nmse_hist.shape[0])
        h = self._nmse_hist[:n].cpu()
        return [float((a / b) ** 0.5) if b > 0 else float("nan") for a, b in h.tolist()]

    def issue(self, n):
        """Enqueue the kernel sequence of n outer iterations (no host sync)."""
        issue_iterations(self, n)

    def prepare(self, n):
        """Capture the kernel sequence of run(n) in a hipGraph now (capture executes nothing),
        so that a later run(n, use_graph=True) is graph replays only (one when n <= 1024)."""
        prepare_iterations(self, n)

    def run(self, n, use_graph=False):
        """Enqueue n outer iterations (no host sync)."""
        run_iterations(self, n, use_graph)

    # ---- results --------------------------------------------------------------------------
    def state(self):
        return self.engine.read_state()

    def S_pixels(self):
        return self.obs.to_pixels(self.S, self.R).reshape(self.R, 1, self.obs.I, self.obs.J)

    def history(self):
        self.engine.flush()  # settle the last S-pass (its history row)
        st = self.state()
        n = min(int(st["iter"]), self.engine.hist_cap)
        h = self.engine.hist[: 4 * n].view(n, 4).double().cpu()
        nsq_c_final = float((self.C.double() ** 2).sum().item())
        costs_c, costs_s = [], []
        for i in range(n):
            nll_c, nll_s, nsq_c, nsq_s = h[i].tolist()
            nsq_c_next = h[i + 1][2].item() if i + 1 < n else nsq_c_final
            costs_c.append(nll_c + self.lambda_c * math.sqrt(nsq_c) + self.lambda_s * math.sqrt(nsq_s))
            costs_s.append(nll_s + self.lambda_c * math.sqrt(nsq_c_next) + self.lambda_s * math.sqrt(nsq_s))
        return costs_c, costs_s


def solve(Y, Wx, bin_boundaries, noise_std, R=None, S_init=None, C_init=None, offset=None,
          log_model=False, lambda_c=100.0, lambda_s=100.0, lr_c=5e-3, lr_s=1e-2, max_iter=500,
          betas=(0.9, 0.999), eps=1e-8, project_c=True, generator=None, Z_init=None,
          restart=False, restart_samples=(200, 200), T_true=None, nmse_every=0,
          use_graph=False, obs=None, tile=None, callback=None, loss="probit", fuse=True,
          project_s=None, holdout=0.0, check_every=10, patience=5, holdout_seed=0):
    """Alternating S/C probit-MLE (qmc/qmc.ipynb :559-645).

    Args mirror the notebook globals: Y (K,1,I,J) bin indices, Wx (K,1,I,J) 0/1 mask,
    bin_boundaries / noise_std / offset of the model, lambda_c = lambda_s = 100,
    lr_c = 5e-3, lr_s = 1e-2, max_iter = 500.  With `generator` the S-step optimises Z_init
    through S = generator(Z) (Adam on Z, the network frozen); otherwise S is free.
    loss="squared" replaces the probit likelihood by the Euclidean criterion
    ||Wx (T_hat - Obs)||_F^2 of qmc/qmc_dowjons.ipynb :142-162 (Obs = bin midpoints,
    get_quantized_obs_from_ordinal); the cost history then holds that criterion.
    project_s=True keeps free S >= 0 (S[S<0] = 0 after each S-step, as C at :579).  The
    default (None) is True for the log model: it needs T_hat + offset > 0 (log at
    qmc/quantization_model_log.py:14, qmc/qmc.ipynb:571), which unprojected free S leaves within
    a few hundred steps, and the reference's own S is a sigmoid output (>= 0); False otherwise.
    project_s=False under the log model is accepted (the caller's choice) and warns.
    holdout > 0 (free S only; not in the reference, which runs a fixed iteration count): that
    fraction of the observed entries (seeded by holdout_seed) is held out of the fit; every
    `check_every` iterations their NLL at the current S, C is evaluated (fused HIP S-pass on
    the held-out set, same pixel order), and the run stops once it has not improved for
    `patience` checks, returning the S, C of the best check (result.best_iter, .holdout_nll).
    With ~6 one-bit samples per pixel (C2) the unregularised free-S MLE over-fits: the map
    NMSE is best after ~50 iterations and grows after.
    Returns a SolveResult with S (R,1,I,J) and C (R,K) on the GPU.
    """
    if log_model and obs is None:
        # the reference log model's default offset (qmc/quantization_model_log.py:7, 9)
        offset = LOG_OFFSET if offset is None else float(offset)
        if not offset > 0.0:
            raise ValueError("the log model needs offset > 0 (log(T_hat + offset) at T_hat = 0)")
    K = Y.shape[0]
    I, J = Y.shape[-2], Y.shape[-1]
    if R is None:
        R = (S_init.shape[0] if S_init is not None else
             (C_init.shape[0] if C_init is not None else Z_init.shape[0]))
    obs_h = None
    if holdout and generator is None:
        if obs is not None:
            raise ValueError("holdout splits the observations itself: pass Y, Wx, not obs")
        Wx_fit, Wx_h = split_holdout(Y, Wx, float(holdout), holdout_seed)
        obs = Observations(Y, Wx_fit, bin_boundaries, noise_std, offset=offset or 0.0,
                           log_model=log_model, tile=tile, R_hint=R, loss=loss)
        # the held-out entries in the SAME position order (perm) and tiles, so the solver's
        # position-order S is evaluated on them as it is
        obs_h = Observations(Y, Wx_h, bin_boundaries, noise_std, offset=offset or 0.0,
                             log_model=log_model, tile=obs.desc.PT, R_hint=R, loss=loss,
                             perm=obs.perm)
    if obs is None:
        obs = Observations(Y, Wx, bin_boundaries, noise_std, offset=offset or 0.0,
                           log_model=log_model, tile=tile, R_hint=R, loss=loss)
    if C_init is None:
        C_init = torch.zeros(R, K)
    if generator is None and obs_h is not None:
        return _solve_holdout(obs, obs_h, S_init, C_init, R, lambda_c, lambda_s, lr_c, lr_s,
                              max_iter, betas, eps, project_c, fuse, project_s, use_graph,
                              int(check_every), int(patience))
    if generator is None:
        if S_init is None:
            S_init = torch.zeros(R, 1, I, J)
        if project_s is None:
            project_s = bool(obs.log_model)
        elif log_model and not project_s:
            warnings.warn("free S under the log model without project_s: T_hat + offset can "
                          "reach <= 0 (a non-finite cost)", RuntimeWarning)
        # the NMSE history is recorded on the device inside the run (no host round trips);
        # a callback still gets control every nmse_every iterations (or once at the end)
        sol = FreeSSolver(obs, S_init, C_init, lambda_c, lambda_s, lr_c, lr_s, betas, eps,
                          project_c, hist_cap=max_iter, fuse=fuse,
                          T_true=T_true if nmse_every else None, nmse_every=nmse_every,
                          project_s=project_s)
        done = 0
        chunk = nmse_every if (callback is not None and nmse_every) else max_iter
        while done < max_iter:
            n = min(chunk, max_iter - done)
            sol.run(n, use_graph=use_graph)
            done += n
            if callback is not None:
                callback(done, sol)
        nmse = sol.nmse_history()
        costs_c, costs_s = sol.history()
        return SolveResult(S=sol.S_pixels(), C=sol.C.clone(), costs_c=costs_c, costs_s=costs_s,
                           nmse=nmse, iters=max_iter, fused=sol.fuse)
    return _solve_generator(obs, generator, Z_init, C_init, R, lambda_c, lambda_s, lr_c, lr_s,
                            max_iter, betas, eps, project_c, restart, restart_samples, T_true,
                            nmse_every, callback, use_graph=use_graph)


# iterations per captured hipGraph of the generator / DIP solver (GeneratorSolver): every
# iteration is ~100 graph nodes (the torch decoder's forward and backward, its optimizer step and
# the HIP passes), so long runs replay a chunk graph instead of one graph of the whole run
GEN_GRAPH_ITERS = 32


class GeneratorSolver:
    """S = generator(Z) alternating solver (qmc/qmc.ipynb :541-634) as a device-resident op
    sequence that is captured in hipGraphs (the DIP solver of dip.solve, the GAN path of solve).

    One iteration, no host synchronisation anywhere:
      C-step  fused HIP C-pass at S_pos (the S of the previous S-step, :564) + qsc_cfinish (Adam on
              C, C >= 0, :576-579); the step's NLL / ||C||^2 stay in the engine's history rows;
      S-step  S = generator(Z) (torch, MIOpen convs), S -> position order (qsc_perm_gather into
              the persistent S_pos), fused HIP S-pass in gradient mode (dS), qsc_state_flush
              (the S-step NLL into the history row), dS -> pixel order, the surrogate
              <S, dS> + lambda_s ||Z||_F back-propagated through the generator (:626-633), the
              optimizer step (:634) -- qsc_adam_flat over the flat parameter buffer, its step
              the engine state's S-step count; lambda_s ||Z|| recorded on the device.
    run(n, use_graph=True) replays captured chunk graphs of GEN_GRAPH_ITERS iterations (sharing
    one memory pool) after WARMUP eager iterations, which create the autograd / MIOpen
    workspaces outside capture.  The optimised tensors live in one flat buffer and take their
    Adam step in one launch (qsc_adam_flat: torch.optim.Adam's update bit for bit, the step
    count from the engine state).  Graph replay and eager issue run the same
    kernels on the same buffers, so the results are bitwise equal
    (tests/test_gpu_fused.py::test_generator_solver_graph_equals_eager).  A capture that fails
    (a library call that cannot be captured) is recorded in `graph_error` and the solver runs
    eagerly from then on."""

    WARMUP = 1

    def __init__(self, obs, generator, Z_init, C_init, R, lambda_c=100.0, lambda_s=100.0,
                 lr_c=5e-3, lr_s=1e-2, betas=(0.9, 0.999), eps=1e-8, project_c=True,
                 params=None, optimize_z=True, hist_cap=1024):
        dev = obs.device
        self.obs, self.net, self.R = obs, generator, R
        self.I, self.J = obs.I, obs.J
        self.engine = PassEngine(obs, R, hist_cap=max(int(hist_cap), 1))
        self.C = _dev(C_init.detach().to(torch.float32)).reshape(R, obs.K).clone()
        self.mC, self.vC = torch.zeros_like(self.C), torch.zeros_like(self.C)
        self.adam_c = _lib.make_adam(lr_c, betas, eps, project_nonneg=project_c)
        self.lambda_c, self.lambda_s = float(lambda_c), float(lambda_s)
        # The optimised tensors (Z and / or the decoder's parameters) live in ONE flat buffer
        # (each a view into it), so the S-step's Adam is one qsc_adam_flat launch over all of
        # them -- torch.optim.Adam's update bit for bit, at the step the engine state counts --
        # instead of torch's per-tensor launches (its capturable foreach path divides every
        # tensor by its 0-dim bias corrections in a launch of its own: ~150 launches of a few us
        # per iteration for the 256^2 decoder, round 6's profile).
        Z = Z_init.detach().to(dev, torch.float32)
        plist = list(params or [])
        sizes = ([Z.numel()] if optimize_z else []) + [q.numel() for q in plist]
        self.flat = torch.empty(sum(sizes), dtype=torch.float32, device=dev)
        o = 0
        if optimize_z:
            self.flat[:Z.numel()] = Z.reshape(-1)
            self.Z = self.flat[:Z.numel()].view(Z.shape).detach().requires_grad_(True)
            o = Z.numel()
        else:
            self.Z = Z.clone()
        for q in plist:
            n = q.numel()
            with torch.no_grad():
                self.flat[o:o + n] = q.detach().reshape(-1).to(dev, torch.float32)
                q.data = self.flat[o:o + n].view(q.shape)
            o += n
        self.plist = ([self.Z] if optimize_z else []) + plist
        self.m_flat = torch.zeros_like(self.flat)
        self.v_flat = torch.zeros_like(self.flat)
        self.g_flat = torch.zeros_like(self.flat)
        self.adam_s = _lib.make_adam(lr_s, betas, eps, project_nonneg=False)
        with torch.no_grad():
            S0 = generator(self.Z).reshape(R, 1, self.I, self.J)
        self.S_pos = obs.to_positions(S0.reshape(R, -1))
        self.engine.init_state(self.S_pos)
        self.dS_pos = torch.zeros_like(self.S_pos)
        self.dS_pix = torch.zeros((R, obs.P), dtype=torch.float32, device=dev)
        self.hist_cap = self.engine.hist_cap
        self.zreg = torch.zeros(self.hist_cap, dtype=torch.float32, device=dev)
        self.ctr = torch.zeros(1, dtype=torch.int64, device=dev)
        self.S_last = S0.detach()
        self.done = 0
        self._eager_done = 0
        self._graphs = {}
        self._pool = None
        self.graph_error = None
        self.graph_capturable = True

    # ---- one iteration (capturable) -----------------------------------------------------
    def c_step(self):
        e = self.engine
        e.cpass(self.S_pos, self.C)
        e.cfinish(self.C, 1, mC=self.mC, vC=self.vC, adam=self.adam_c, lambda_c=self.lambda_c)

    def s_step(self):
        e, R = self.engine, self.R
        # gradients set to None: backward then writes each one instead of zeroing and adding to
        # it (two elementwise launches per parameter tensor); inside a capture the new gradients
        # live in the graph's pool
        for q in self.plist:
            q.grad = None
        S = self.net(self.Z).reshape(R, 1, self.I, self.J)
        self.obs.to_positions(S.detach().reshape(R, -1), out=self.S_pos)
        e.spass(self.S_pos, self.C, 0, dS=self.dS_pos)
        e.flush(record=True)  # the S-step NLL -> this iteration's history row
        self.obs.to_pixels(self.dS_pos, R, out=self.dS_pix)
        reg = self.lambda_s * torch.norm(self.Z, "fro")
        surrogate = (S * self.dS_pix.reshape(R, 1, self.I, self.J)).sum() + reg
        surrogate.backward()
        if self.plist:
            # the gradients into the flat buffer (one batched copy), then Adam on all of them
            torch.cat([q.grad.reshape(-1) for q in self.plist], out=self.g_flat)
            _lib.call("qsc_adam_flat", _lib.ptr(self.flat), _lib.ptr(self.m_flat),
                      _lib.ptr(self.v_flat), _lib.ptr(self.g_flat), self.flat.numel(),
                      self.adam_s, _lib.ptr(e.state), _lib.stream())
        with torch.no_grad():
            self.zreg.index_copy_(0, self.ctr.clamp(max=self.hist_cap - 1),
                                  reg.detach().reshape(1))
            self.ctr += 1
        self.S_last = S.detach()

    def iteration(self):
        self.c_step()
        self.s_step()

    # ---- runs ---------------------------------------------------------------------------
    def _capture(self, m):
        g = torch.cuda.CUDAGraph()
        s = capture_stream()
        caller = torch.cuda.current_stream()
        s.wait_stream(caller)
        if self._pool is None:
            self._pool = torch.cuda.graph_pool_handle()
        gen0 = self.engine.gen
        try:
            with torch.cuda.stream(s):
                with torch.cuda.graph(g, stream=s, pool=self._pool,
                                      capture_error_mode="thread_local"):
                    for _ in range(m):
                        self.iteration()
        except Exception as e:  # noqa: BLE001 - every failure takes the same clean-up path
            del g
            abandon_capture(s, caller)
            self.engine.gen = gen0
            self.graph_error = "%s: %s" % (type(e).__name__, e)
            self.graph_capturable = False
            warnings.warn("hipGraph capture of the generator iteration failed; running eagerly "
                          "(%s)" % self.graph_error, RuntimeWarning)
            return None
        self.engine.gen = gen0
        caller.wait_stream(s)
        _upload(g)
        return g

    def _graph(self, m):
        if not self.graph_capturable:
            return None
        if m not in self._graphs:
            self._graphs[m] = self._capture(m)
        return self._graphs[m]

    def prepare(self, n):
        """Capture (without executing) the chunk graphs run(n) will replay.  Needs the WARMUP
        eager iterations done (they create the optimizer state outside capture)."""
        if self._eager_done < self.WARMUP:
            raise RuntimeError("prepare() after %d eager iterations (run them first)" % self.WARMUP)
        for m in sorted(set(_gen_chunks(n))):
            self._graph(m)

    def run(self, n, use_graph=True):
        """Enqueue n iterations (no host sync)."""
        use_graph = use_graph and torch.cuda.is_available() and self.C.is_cuda
        while n > 0 and (self._eager_done < self.WARMUP or not use_graph):
            self.iteration()
            self._eager_done += 1
            self.done += 1
            n -= 1
        for m in _gen_chunks(n):
            g = self._graph(m)
            if g is None:
                for _ in range(m):
                    self.iteration()
            else:
                g.replay()
            self.done += m

    # ---- results --------------------------------------------------------------------------
    def S_pixels(self):
        """The last S-step's generator output S (R, 1, I, J)."""
        return self.S_last

    def state(self):
        return self.engine.read_state()

    def history(self):
        """Per-iteration costs (qmc/qmc.ipynb :573, :631): C-step cost at the C it
        differentiates, S-step cost at the updated C (both with lambda_s ||Z|| of the S-step's
        Z), from the device history rows (one synchronisation)."""
        n = min(self.done, self.hist_cap)
        h = self.engine.hist[: 4 * n].view(n, 4).double().cpu()
        z = self.zreg[:n].double().cpu()
        nsq_c_final = float((self.C.double() ** 2).sum().item())
        costs_c, costs_s = [], []
        for i in range(n):
            nll_c, nll_s, nsq_c = h[i][0].item(), h[i][1].item(), h[i][2].item()
            nsq_next = h[i + 1][2].item() if i + 1 < n else nsq_c_final
            costs_c.append(nll_c + self.lambda_c * math.sqrt(nsq_c) + z[i].item())
            costs_s.append(nll_s + self.lambda_c * math.sqrt(nsq_next) + z[i].item())
        return costs_c, costs_s


def _gen_chunks(n):
    out = []
    while n > 0:
        m = min(n, GEN_GRAPH_ITERS)
        out.append(m)
        n -= m
    return out


def split_holdout(Y, Wx, frac, seed=0):
    """(Wx_fit, Wx_holdout): a seeded random `frac` of the observed entries (Wx == 1, or all
    entries when Wx is None) moved to the held-out mask."""
    W = (Wx if Wx is not None else torch.ones(Y.shape)).to(torch.float32)
    g = torch.Generator().manual_seed(int(seed))
    u = torch.rand(W.shape, generator=g).to(W.device)
    hold = (W > 0) & (u < frac)
    return W * (~hold).to(W.dtype), W * hold.to(W.dtype)


def _solve_holdout(obs, obs_h, S_init, C_init, R, lambda_c, lambda_s, lr_c, lr_s, max_iter,
                   betas, eps, project_c, fuse, project_s, use_graph, check_every, patience):
    """Free-S solve with early stopping on the held-out NLL (solve(holdout=...))."""
    I, J = obs.I, obs.J
    if S_init is None:
        S_init = torch.zeros(R, 1, I, J)
    sol = FreeSSolver(obs, S_init, C_init, lambda_c, lambda_s, lr_c, lr_s, betas, eps, project_c,
                      hist_cap=max_iter, fuse=fuse, project_s=project_s)
    eng_h = PassEngine(obs_h, R)
    eng_h.init_state(sol.S)
    dS_h = torch.empty_like(sol.S)
    hist_h, best, best_iter, best_SC = [], float("inf"), 0, None
    done = 0
    while done < max_iter:
        n = min(check_every, max_iter - done)
        sol.run(n, use_graph=use_graph)
        done += n
        eng_h.spass(sol.S, sol.C, 0, dS=dS_h)
        eng_h.flush(record=False)
        v = float(eng_h.read_state()["nll_s"])
        hist_h.append((done, v))
        if v < best:
            best, best_iter = v, done
            best_SC = (sol.S.clone(), sol.C.clone())
        elif done - best_iter >= patience * check_every:
            break
    costs_c, costs_s = sol.history()
    S_pos, C = best_SC if best_SC is not None else (sol.S, sol.C)
    res = SolveResult(S=obs.to_pixels(S_pos, R).reshape(R, 1, I, J), C=C.clone(),
                      costs_c=costs_c, costs_s=costs_s, iters=done, fused=sol.fuse)
    res.best_iter = best_iter
    res.holdout_nll = hist_h
    return res


def _solve_generator(obs, generator, Z_init, C_init, R, lambda_c, lambda_s, lr_c, lr_s, max_iter,
                     betas, eps, project_c, restart, restart_samples, T_true, nmse_every,
                     callback, params=None, optimize_z=True, use_graph=True):
    """S = generator(Z) variant (qmc/qmc.ipynb :541-634) on a GeneratorSolver.  The S-step
    optimises Z (optimize_z) plus any extra `params` -- the DIP solver passes the decoder
    weights.  The one-time random restart of Z (:590-619, i == 1) runs eagerly between the
    C-step and the S-step of iteration 1; the rest runs as captured hipGraph chunks (use_graph).
    With `callback` or NMSE tracking the run is split into chunks of `nmse_every` iterations
    (callback(i, dict(S, C, Z)) after each, S the last S-step's generator output)."""
    sol = GeneratorSolver(obs, generator, Z_init, C_init, R, lambda_c, lambda_s, lr_c, lr_s,
                          betas, eps, project_c, params=params, optimize_z=optimize_z,
                          hist_cap=max_iter)
    return drive_generator(sol, max_iter, restart, restart_samples, T_true, nmse_every, callback,
                           use_graph)


def drive_generator(sol, max_iter, restart=False, restart_samples=(200, 200), T_true=None,
                    nmse_every=0, callback=None, use_graph=True):
    """Run a fresh GeneratorSolver for max_iter iterations (the loop of qmc/qmc.ipynb :559-645)
    and collect its SolveResult."""
    obs, generator, R = sol.obs, sol.net, sol.R
    lambda_c, lambda_s = sol.lambda_c, sol.lambda_s
    nmse = []
    chunk = max(int(nmse_every), 1) if (callback is not None or (T_true is not None and nmse_every)) \
        else max_iter
    done = 0

    def after(k):
        if T_true is not None and nmse_every and k % nmse_every == 0:
            nmse.append(map_nmse(sol.S_last, sol.C, T_true))
        if callback is not None:
            callback(k, dict(S=sol.S_last, C=sol.C, Z=sol.Z))

    if restart and max_iter >= 2:
        # iteration 0, then iteration 1's C-step, the restart, and its S-step (eager)
        sol.run(1, use_graph=False)
        after(1)
        sol.c_step()
        _restart_z(sol, obs, generator, R, lambda_c, lambda_s, restart_samples)
        sol.s_step()
        sol._eager_done += 1
        sol.done += 1
        after(2)
        done = 2
    while done < max_iter:
        n = min(chunk - (done % chunk), max_iter - done)
        sol.run(n, use_graph=use_graph)
        done += n
        if callback is not None or (T_true is not None and nmse_every):
            after(done)
    costs_c, costs_s = sol.history()
    res = SolveResult(S=sol.S_last, C=sol.C, costs_c=costs_c, costs_s=costs_s, nmse=nmse,
                      Z=sol.Z.detach(), iters=max_iter)
    res.graph_error = sol.graph_error
    res.solver = sol
    return res


def _restart_z(sol, obs, generator, R, lambda_c, lambda_s, restart_samples):
    """The notebook's one-time random restart of Z at i == 1 (:590-619): 200 random candidates,
    the best by its full cost, then 200 perturbations of it -- whose cost the reference
    evaluates at the LAST first-round sample (temp_out, :611: a reference quirk kept as is).
    Candidates are scored on a separate pass engine (its own state), so the solver's step
    counters and history rows are untouched."""
    dev = obs.device
    I, J = obs.I, obs.J
    eng = PassEngine(obs, R, hist_cap=0)
    Sp = torch.empty_like(sol.S_pos)
    dSp = torch.empty_like(sol.S_pos)
    eng.init_state(Sp.zero_())
    Z = sol.Z

    def nll_of(S_cand):
        obs.to_positions(S_cand.reshape(R, -1), out=Sp)
        eng.spass(Sp, sol.C, 0, dS=dSp)
        eng.flush(record=False)
        return eng.read_state()["nll_s"]

    S_now = sol.S_last
    best = float("inf")
    n1, n2 = restart_samples
    last = None
    for _ in range(n1):
        cand = torch.randn((R, Z.shape[1]), dtype=torch.float32)
        with torch.no_grad():
            out = generator(cand.to(dev)).reshape(R, 1, I, J)
        crit = nll_of(out) + lambda_c * float(torch.norm(sol.C)) + lambda_s * float(torch.norm(S_now))
        last = out
        if crit < best:
            with torch.no_grad():
                Z.copy_(cand.to(dev))
            best = crit
    for _ in range(n2):
        cand = 0.2 * torch.randn((R, Z.shape[1]), dtype=torch.float32) + Z.detach().cpu()
        crit = nll_of(last) + lambda_c * float(torch.norm(sol.C)) + lambda_s * float(torch.norm(S_now))
        if crit < best:
            with torch.no_grad():
                Z.copy_(cand.to(dev))
            best = crit
