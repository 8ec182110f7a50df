"""bench.py's launch contract on CPU (no GPU call is reached):

* under a launcher, WORLD_SIZE must equal --gpus (a scaling run must never measure one GPU and
  call it N): the mismatch exits non-zero before torch or libecc is imported;
* `--gpus N` without a launcher spawns `torch.distributed.run` as a child with N ranks.
"""
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def _env(**kv):
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    env.update(kv)
    return env


def test_world_size_gpus_mismatch_exits_nonzero():
    for world, gpus in (("2", "1"), ("1", "4"), ("8", "2")):
        r = subprocess.run([sys.executable, "bench.py", "--gpus", gpus, "--steps", "1"], cwd=ROOT,
                           env=_env(WORLD_SIZE=world, RANK="0", LOCAL_RANK="0"),
                           capture_output=True, text=True, timeout=120)
        assert r.returncode == 2, (world, gpus, r.stdout, r.stderr)
        assert "WORLD_SIZE" in r.stderr
        assert not r.stdout.strip().startswith("{")


def test_launch_ranks_builds_child_command(monkeypatch):
    sys.path.insert(0, str(ROOT))
    import bench
    calls = []

    class R:
        returncode = 7

    def fake_run(cmd, env):
        calls.append((cmd, env))
        return R()

    monkeypatch.setattr(subprocess, "run", fake_run)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4", "--steps", "3"])
    args = bench.parse()
    assert bench.launch_ranks(args) == 7  # the child's exit code propagates
    cmd, env = calls[0]
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "127.0.0.1" in cmd
    assert cmd[-4:] == ["--gpus", "4", "--steps", "3"]
    assert env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    # one GPU, or under a matching launcher: no child
    monkeypatch.setattr(sys, "argv", ["bench.py"])
    assert bench.launch_ranks(bench.parse()) is None
    monkeypatch.setenv("WORLD_SIZE", "4")
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4"])
    assert bench.launch_ranks(bench.parse()) is None
    assert len(calls) == 1


def test_default_sizes_per_gpu_count():
    """One GPU keeps the metric's C4 batch (1221 slices = 20 004 864 events); the multi-GPU line is
    BASELINE C5 by default: 50 M events per GPU (3052 slices), 400 M at N = 8."""
    sys.path.insert(0, str(ROOT))
    import bench
    assert bench.parse([]).events == 20_004_864
    assert bench.parse(["--gpus", "1"]).preset == "c4"
    a8 = bench.parse(["--gpus", "8"])
    assert a8.preset == "c5" and a8.events == 3052 * 16384 == 50_003_968
    assert 8 * a8.events >= 400_000_000
    assert bench.parse(["--gpus", "2"]).events == 50_003_968
    # explicit sizes win
    assert bench.parse(["--gpus", "8", "--preset", "c4"]).events == 20_004_864
    assert bench.parse(["--gpus", "8", "--events", "163840"]).events == 163840
    assert bench.parse(["--preset", "c5"]).events == 50_003_968
