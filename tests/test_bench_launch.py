"""bench.py starts its own ranks.

`python bench.py --gpus N` -- the driver's command form -- must run N ranks,
one process per GPU, and report n_gpus N / parallelism dpN.  The CPU tests
check the launcher's command and its refusal of a --gpus / WORLD_SIZE
mismatch; the GPU test runs the whole bench at --gpus 2 as two ranks on one
device over gloo (RCCL refuses two ranks on one GPU).
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_launch_command_shape():
    cmd = bench.launch_command(["--gpus", "8", "--steps", "3"], 8, 29555)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd
    assert "--master-addr=127.0.0.1" in cmd and "--master-port=29555" in cmd
    i = cmd.index(os.path.join(ROOT, "bench.py"))
    assert cmd[i + 1:] == ["--gpus", "8", "--steps", "3"]


def test_launcher_noop_for_one_gpu_and_inside_a_rank(monkeypatch):
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    assert bench.maybe_launch_ranks([], 1) is None
    monkeypatch.setenv("WORLD_SIZE", "4")
    assert bench.maybe_launch_ranks(["--gpus", "4"], 4) is None      # a rank of a torchrun job


def test_launcher_refuses_world_mismatch(monkeypatch):
    monkeypatch.setenv("WORLD_SIZE", "2")
    assert bench.maybe_launch_ranks(["--gpus", "8"], 8) == 2


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_bench_gpus2_launches_two_ranks():
    env = dict(os.environ, DRO_DIST_BACKEND="gloo", DRO_BENCH_DEVICE="0")
    env.pop("WORLD_SIZE", None)
    env.pop("RANK", None)
    env.pop("LOCAL_RANK", None)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2",
                          "--warmup", "2", "--no-cpu-baseline", "--no-roofline"],
                         env=env, cwd=ROOT, capture_output=True, text=True, timeout=540)
    assert out.returncode == 0, out.stderr[-4000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]                         # rank 0 prints ONE line
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["config"]["parallelism"] == "dp2"
    assert res["config"]["global_batch"] == 2 * res["config"]["per_gpu_batch"]
    assert res["value"] > 0
