"""CPU: `bench.py --gpus N` turns itself into N ranks (torchrun child process) when no outer launcher
set WORLD_SIZE, and refuses a WORLD_SIZE that disagrees with --gpus."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def _env():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["MASTER_ADDR"] = "127.0.0.1"
    return env


def test_launch_command_shape():
    cmd = bench.launch_command(["--gpus", "8", "--steps", "3"], 8, 29555, python="py", script="b.py")
    assert cmd[:3] == ["py", "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--master-addr=127.0.0.1" in cmd and "--master-port=29555" in cmd
    assert cmd[-4:] == ["--gpus", "8", "--steps", "3"] and cmd[-5] == "b.py"


def test_maybe_launch_no_spawn_cases():
    assert bench.maybe_launch(1, [], env={}) is None                 # N = 1: run in-process
    assert bench.maybe_launch(4, [], env={"WORLD_SIZE": "4"}) is None  # already a rank
    assert bench.maybe_launch(8, [], env={"WORLD_SIZE": "1"}) == 2     # mismatch: refuse


@pytest.mark.parametrize("n", [2, 3])
def test_gpus_flag_spawns_ranks(n):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--launch-dry-run"],
                       capture_output=True, text=True, timeout=240, env=_env(), cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == n and d["gpus_flag"] == n and d["rank_sum"] == n * (n - 1) // 2


def test_gpus_flag_mismatch_exits_nonzero():
    env = _env()
    env["WORLD_SIZE"] = "2"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8", "--launch-dry-run"],
                       capture_output=True, text=True, timeout=120, env=env, cwd=ROOT)
    assert r.returncode != 0 and "WORLD_SIZE=2" in r.stderr
