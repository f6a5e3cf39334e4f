"""hipGraph capture of the solver loop: a capture that fails part-way is abandoned cleanly and
the solver falls back to eager execution with bit-identical results (or raises, for a solver
that is not capture-tolerant), and prepare(n) captures every graph run(n) replays.

Reference loop being captured: qmc/qmc.ipynb :559-645 (C-step :562-579, S-step :622-634)."""
import numpy as np
import pytest
import torch

from test_gpu_fused import _random_case

pytestmark = pytest.mark.gpu


def _solver(d, **kw):
    from quantized_spectrum_cartography_amd.obs import Observations
    from quantized_spectrum_cartography_amd.qmc import FreeSSolver
    obs = Observations(d["Y"], d["Wx"], d["b"], d["sigma"], R_hint=4, tile=512)
    return FreeSSolver(obs, d["S0"], d["C0"], hist_cap=64, **kw)


def _sabotage(sol, how):
    """Make the solver's C-step fail while (and only while) it is being captured."""
    orig = sol.c_step

    def bad():
        if torch.cuda.is_current_stream_capturing():
            if how == "sync":
                # synchronising a capturing stream is illegal: HIP invalidates the capture
                torch.cuda.current_stream().synchronize()
            orig()
            raise RuntimeError("forced failure inside the capture")
        orig()
    sol.c_step = bad


@pytest.mark.parametrize("how", ["raise", "sync"])
def test_failed_capture_falls_back_to_eager_bitexact(how):
    from quantized_spectrum_cartography_amd import qmc
    d = _random_case(71, 4, 64, 64, 64)
    ref = _solver(d)
    ref.run(7, use_graph=False)
    sol = _solver(d)
    sol.graph_tolerant = True
    _sabotage(sol, how)
    with pytest.warns(RuntimeWarning, match="capture failed"):
        sol.run(7, use_graph=True)
    assert sol.graph_error and sol.graph_capturable is False
    cur = torch.cuda.current_stream()
    assert qmc.stream_capture_status(cur) == 0
    torch.cuda.synchronize()
    assert np.array_equal(ref.S.cpu().numpy(), sol.S.cpu().numpy())
    assert np.array_equal(ref.C.cpu().numpy(), sol.C.cpu().numpy())
    # later runs stay eager and keep matching
    ref.run(3, use_graph=False)
    sol.run(3, use_graph=True)
    assert np.array_equal(ref.S.cpu().numpy(), sol.S.cpu().numpy())


def test_failed_capture_raises_for_intolerant_solver_and_stream_stays_usable():
    from quantized_spectrum_cartography_amd import qmc
    d = _random_case(72, 4, 64, 64, 64)
    ref = _solver(d)
    ref.run(5, use_graph=False)
    sol = _solver(d)
    _sabotage(sol, "sync")
    with pytest.raises(RuntimeError):
        sol.run(5, use_graph=True)
    assert qmc.stream_capture_status(torch.cuda.current_stream()) == 0
    # nothing ran during the failed capture: an eager run from here equals the reference
    del sol.c_step
    sol.run(5, use_graph=False)
    assert np.array_equal(ref.S.cpu().numpy(), sol.S.cpu().numpy())
    assert np.array_equal(ref.C.cpu().numpy(), sol.C.cpu().numpy())


def test_prepare_captures_every_chunk(monkeypatch):
    """run(n) after prepare(n) captures nothing new, also when n spans several graph chunks
    (bench's timed region must be replay only)."""
    from quantized_spectrum_cartography_amd import qmc
    monkeypatch.setattr(qmc, "GRAPH_MAX_ITERS", 4)
    d = _random_case(73, 4, 64, 64, 64)
    sol = _solver(d)
    sol.prepare(10)
    # chunks 4, 4, 2, each captured in both entry forms: without a C-pass ahead (a first run)
    # and with the C-pass the previous chunk's or run's last fused launch left ahead
    # (qmc.issue_iterations) -- so neither this run(10) nor a later one captures
    assert sorted(sol._graphs) == [(2, False), (2, True), (4, False), (4, True)]
    calls = []
    orig = qmc._capture
    monkeypatch.setattr(qmc, "_capture", lambda *a: calls.append(a) or orig(*a))
    sol.run(10, use_graph=True)
    sol.run(10, use_graph=True)
    assert calls == []
    ref = _solver(d)
    ref.run(10, use_graph=False)
    ref.run(10, use_graph=False)
    assert np.array_equal(ref.S.cpu().numpy(), sol.S.cpu().numpy())


def test_chained_run_redoes_a_c_pass_overwritten_in_between():
    """a run that chains on the C-pass the previous run left ahead must not
    use it when anything overwrote the workspace since -- here a direct engine C-pass at another
    S (as bench.time_kernel or a tool would issue), which leaves S and C and their torch version
    counters untouched.  The next run redoes its C-pass: the result equals an uninterrupted
    run bit for bit."""
    d = _random_case(74, 4, 64, 64, 64)
    a = _solver(d)
    a.run(3, use_graph=True)
    assert a.ahead()
    S_other = a.S * 2.0
    a.engine.cpass(S_other, a.C)  # overwrites the slab partials the chain would use
    assert not a.ahead()
    a.run(3, use_graph=True)
    ref = _solver(d)
    ref.run(6, use_graph=False)
    assert np.array_equal(ref.S.cpu().numpy(), a.S.cpu().numpy())
    assert np.array_equal(ref.C.cpu().numpy(), a.C.cpu().numpy())
    # a fresh tensor swapped in for C (version counter 0 again) also breaks the chain
    b = _solver(d)
    b.run(3, use_graph=True)
    b.C = b.C.clone()
    assert not b.ahead()
    # and its next graph run captures anew at the new tensor (not a replay into the old one)
    b.run(2, use_graph=True)
    ref2 = _solver(d)
    ref2.run(5, use_graph=False)
    assert np.array_equal(ref2.C.cpu().numpy(), b.C.cpu().numpy())
