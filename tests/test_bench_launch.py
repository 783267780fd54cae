"""bench.py's multi-GPU plumbing on the CPU (gloo): `--gpus N` with no torch.distributed environment starts N
ranks itself, each rank reads RANK / WORLD_SIZE, and the timing reduction is max(elapsed) / sum(units) over ranks.
A WORLD_SIZE that disagrees with --gpus is an error (a driver `--gpus 8` run can never silently time one GPU)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                           "MASTER_PORT")}
    env.update(kw)
    return env


@pytest.mark.parametrize("gpus", [1, 2, 3])
def test_bench_launches_and_reduces_over_ranks(gpus):
    out = subprocess.run([sys.executable, BENCH, "--gpus", str(gpus), "--dist-selftest"], env=_env(),
                         capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout  # rank 0 prints one line
    d = json.loads(lines[0])
    assert d == {"world": gpus, "max_elapsed": float(gpus), "sum_units": float(sum(r + 10 for r in range(gpus)))}


def test_bench_refuses_world_size_mismatch():
    out = subprocess.run([sys.executable, BENCH, "--gpus", "4", "--dist-selftest"],
                         env=_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"), capture_output=True, text=True,
                         timeout=120)
    assert out.returncode != 0
    assert "WORLD_SIZE=2" in out.stderr
