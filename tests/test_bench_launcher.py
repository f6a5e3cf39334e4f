"""bench.py's multi-GPU launch logic (CPU): `python3 bench.py --gpus N` without WORLD_SIZE starts
N ranks itself as a child torch.distributed.run job; as a rank it runs the bench."""
import subprocess
import sys

import pytest

import bench


def _args(argv):
    old = sys.argv
    try:
        sys.argv = ["bench.py"] + argv
        return bench.parse()
    finally:
        sys.argv = old


def test_single_gpu_runs_in_process():
    assert bench.maybe_launch(_args([]), argv=[], env={}) is None
    assert bench.maybe_launch(_args(["--gpus", "1"]), argv=["--gpus", "1"], env={}) is None


def test_rank_process_does_not_relaunch():
    a = _args(["--gpus", "8"])
    assert bench.maybe_launch(a, argv=["--gpus", "8"], env={"WORLD_SIZE": "8"}) is None


def test_plain_multi_gpu_command_spawns_torchrun(monkeypatch):
    seen = {}

    def fake_call(cmd, env=None):
        seen["cmd"], seen["env"] = cmd, env
        return 7
    monkeypatch.setattr(subprocess, "call", fake_call)
    argv = ["--gpus", "4", "--steps", "20", "--warmup", "5"]
    rc = bench.maybe_launch(_args(argv), argv=argv, env={"HSA_ENABLE_IPC_MODE_LEGACY": "0"})
    assert rc == 7  # the child's exit code is the bench's
    cmd = seen["cmd"]
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--nnodes=1" in cmd
    assert "--master-addr=127.0.0.1" in cmd
    assert any(c.startswith("--master-port=") for c in cmd)
    i = cmd.index(bench.__file__.replace(".pyc", ".py")) if bench.__file__ in cmd else \
        [j for j, c in enumerate(cmd) if c.endswith("bench.py")][0]
    assert cmd[i + 1:] == argv  # the script's own arguments are forwarded unchanged
    assert seen["env"]["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"


def test_launcher_command_runs_this_script():
    cmd = bench.launcher_cmd(["--gpus", "2"], 2, port=29999)
    assert cmd[-3].endswith("bench.py") and cmd[-2:] == ["--gpus", "2"]
    assert "--master-port=29999" in cmd


def test_world_size_mismatch_exits_nonzero(monkeypatch):
    """A process group whose size differs from --gpus never prints a bench line."""
    monkeypatch.setattr(bench, "dist_init", lambda: (None, 0, 1))
    monkeypatch.setattr(bench, "maybe_launch", lambda a: None)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2"])
    assert bench.main() == 2


@pytest.mark.parametrize("steps", [20, 4096])
def test_graph_chunks_cover_the_run(steps):
    from quantized_spectrum_cartography_amd import qmc
    ch = qmc.graph_chunks(steps // 2)
    assert sum(ch) == steps // 2 and max(ch) <= qmc.GRAPH_MAX_ITERS


def test_ranks_share_the_cpu_threads(monkeypatch):
    monkeypatch.setattr(bench.os, "sched_getaffinity", lambda pid: set(range(64)), raising=False)
    assert bench.rank_env({"OMP_NUM_THREADS": "16"}, 8)["OMP_NUM_THREADS"] == "2"
    assert bench.rank_env({}, 8)["OMP_NUM_THREADS"] == "8"
    assert bench.rank_env({"OMP_NUM_THREADS": "4"}, 8)["OMP_NUM_THREADS"] == "1"
    assert bench.rank_env({"X": "y"}, 2)["X"] == "y"


def test_heartbeat_reports_long_phases(capsys):
    import time
    with bench.heartbeat(0, "phase", every=0.05):
        time.sleep(0.2)
    err = capsys.readouterr().err
    assert "[bench] phase:" in err
    with bench.heartbeat(1, "phase", every=0.05):  # other ranks stay quiet
        time.sleep(0.12)
    assert capsys.readouterr().err == ""


def test_multi_gpu_default_is_the_metric():
    """BASELINE.json's metric is the ONE fixed 512x512x256 R=8 map at 1/2/4/8 GPUs, split by the
    north-star K-slab layout: --gpus N defaults to strong scaling, K-slab, config c3; the other
    layout and weak scaling ride along as extra keys."""
    a = _args(["--gpus", "8"])
    assert a.scaling == "strong" and a.shard == "kslab" and a.config == "c3"
    assert not a.no_extra


def test_extra_measurement_plan(monkeypatch):
    """The extra keys of an N > 1 run: the other layout at the same scaling, plus weak IJ-slab;
    weak values count every rank's grad-steps, strong ones the fixed map's."""
    built = []

    class _Obs:
        nnz = 7

    def fake_build(cfg, scaling, shard, rank, world, dist, hist_cap, keep_inputs=False):
        built.append((scaling, shard))
        return {}, _Obs(), object()

    monkeypatch.setattr(bench, "build_solver", fake_build)
    monkeypatch.setattr(bench, "timed_run", lambda *a, **k: (2.0, 2.0, 1e-4))
    a = _args(["--gpus", "4", "--steps", "10"])
    out = bench.extra_measurements((8, 8, 8, 2), a, 1, 4, None, "strong", "kslab")
    assert built == [("strong", "ijslab"), ("weak", "ijslab")]
    assert out["layouts"]["ijslab"]["value"] == 5.0 and out["weak"]["ijslab"]["value"] == 20.0


def _kslab_breakdown():
    k = {"cpass_nsq": {"us": 15.0, "bytes": 30e6, "symbol": "cpass_tile_kernel", "what": "C"},
         "cfinish": {"us": 4.0, "bytes": 1e6, "symbol": "cfinish_kernel", "what": "F"},
         "spass_grad": {"us": 12.0, "bytes": 40e6, "symbol": "spass_kernel", "what": "S"},
         "supdate_rows": {"us": 2.0, "bytes": 3e6, "symbol": "supdate", "what": "A"}}
    return {"kernels": k, "collectives": {"allreduce_cnsq": {"us": 9.0}}}


def test_kslab_roofline_names_a_kernel_the_layout_runs():
    """under K-slab the line's roofline is the dominant kernel of the K-slab
    iteration (spass mode 0 / cpass_nsq / ...) with its own bytes, never the fused S-step."""
    r = bench.select_roofline(True, _kslab_breakdown(), 1e-5, 1.0, 2e-5, 2.0, 0)
    assert r["symbol"] == "cpass_tile_kernel" and r["bytes"] == 30e6 and abs(r["t"] - 15e-6) < 1e-12
    assert "scfused" not in r["kernel"] and "spass_kernel (fused" not in r["kernel"]


def test_fused_roofline_uses_the_longer_of_self_replay_and_in_sequence():
    """frac uses the lower of the two fractions."""
    r = bench.select_roofline(True, None, 1e-5, 1.0, 27.4e-6, 77.2e6, 2.2e6,
                              {"scfused_us": 29.3})
    assert r["symbol"] == "scfused_kernel" and abs(r["t"] - 29.3e-6) < 1e-12
    assert r["t_self_replay"] == 27.4e-6 and abs(r["t_in_sequence"] - 29.3e-6) < 1e-12
    r = bench.select_roofline(True, None, 1e-5, 1.0, 27.4e-6, 77.2e6, 2.2e6, {"error": "x"})
    assert r["t"] == 27.4e-6 and r["t_in_sequence"] is None
    r = bench.select_roofline(False, None, 1e-5, 1.0, None, None, 0)
    assert r["symbol"] == "spass_kernel"


@pytest.mark.parametrize("world", [2, 4, 8])
def test_kslab_projection_keys(world):
    """Every strong K-slab C3 line carries DESIGN section 5's projection; other runs none."""
    p = bench.projection("c3", world, "kslab", "strong")
    lo, hi = p["iteration_us"]
    assert 0 < lo <= hi and p["grad_steps_per_s"] == [2e6 / hi, 2e6 / lo]
    assert bench.projection("c3", world, "ijslab", "strong") is None
    assert bench.projection("c3", world, "kslab", "weak") is None
    assert bench.projection("c3", 1, "kslab", "strong") is None
