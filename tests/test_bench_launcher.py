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
    monkeypatch.setattr(bench, "timed_run", lambda *a, **k: (2.0, 2.0))
    a = _args(["--gpus", "4", "--steps", "10"])
    out = bench.extra_measurements((8, 8, 8, 2), a, 1, 4, None, "strong", "kslab")
    assert built == [("strong", "ijslab"), ("weak", "ijslab")]
    assert out["layouts"]["ijslab"]["value"] == 5.0 and out["weak"]["ijslab"]["value"] == 20.0
