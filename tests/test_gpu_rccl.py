"""GPU: the RCCL ("nccl") backend through bench.py's rank plumbing, one rank on the box's one device.

bench.py's multi-GPU line (`--gpus N`, N > 1) initialises `torch.distributed` with the nccl backend (RCCL on ROCm)
and reduces the timing and the work over ranks with two device all-reduces; the training line's gradient bucket
(`gncde.train.reduce_gradients`) is one fp64 all-reduce.  A box here has one GPU and RCCL refuses two ranks on one
device, so this runs the same calls as a world of one: process-group init with `device_id`, barrier, the MAX / SUM
reductions of `bench.reduce_over_ranks`, and an all-reduce of a training-sized fp64 bucket, each of which launches
RCCL's kernels on the device.  The N > 1 arithmetic is covered by the gloo tests (tests/test_dist_cpu.py,
tests/test_gpu_dist.py); the driver's 8-GPU run is the multi-rank RCCL measurement.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_RANK = r"""
import json, os, sys
import torch
import torch.distributed as dist
sys.path[:0] = [os.environ["GNCDE_ROOT"]]
import bench
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
out = {"backend": dist.get_backend(), "world": dist.get_world_size()}
dist.barrier()
mx, tot = bench.reduce_over_ranks(dist, "cuda", 1.25, 409600.0)
out.update(max_elapsed=mx, sum_units=tot)
g = torch.Generator(device="cuda").manual_seed(5)
bucket = torch.randn(1 << 16, generator=g, device="cuda", dtype=torch.float64)
ref = bucket.clone()
dist.all_reduce(bucket, op=dist.ReduceOp.SUM)
torch.cuda.synchronize()
out["bucket_equal"] = bool(torch.equal(bucket, ref))
dist.destroy_process_group()
print("RESULT " + json.dumps(out), flush=True)
"""


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_rccl_world_of_one_runs_bench_reductions():
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0", WORLD_SIZE="1",
               LOCAL_RANK="0", GNCDE_ROOT=ROOT,
               HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    r = subprocess.run([sys.executable, "-c", _RANK], cwd=ROOT, env=env, capture_output=True, text=True, timeout=180)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("RESULT ")]
    assert r.returncode == 0 and lines, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
    out = json.loads(lines[-1][len("RESULT "):])
    print(out)
    assert out["backend"] == "nccl" and out["world"] == 1
    assert out["max_elapsed"] == 1.25 and out["sum_units"] == 409600.0
    assert out["bucket_equal"]
