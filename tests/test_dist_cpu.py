"""CPU, world_size 2 over gloo: the data-parallel pieces of the training step —
contiguous sharding and the gradient/loss all-reduce that turns per-rank summed losses into the gradient
of the reference's full-batch mean (loss_configs.py:47).  The GPU solve itself is exercised in
tests/test_gpu_grad.py; here a torch surrogate loss stands in for it so the collective logic runs on CPU."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from gncde.train import reduce_gradients, shard_range


def test_shard_range_covers_everything():
    for total in (0, 1, 7, 1024, 8193):
        for world in (1, 2, 3, 8):
            spans = [shard_range(total, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == total
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        shard_range(4, 2, 2)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _surrogate(theta, X, Y):
    """Stand-in per-sample model: nonlinear regression with per-sample inputs X [b, n, d], targets Y [b, n]."""
    return torch.tanh(X @ theta[:-1] + theta[-1])


def _worker(rank, world, port, X, Y, theta0, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        a, b = shard_range(X.shape[0], rank, world)
        theta = theta0.clone().requires_grad_(True)
        pred = _surrogate(theta, X[a:b], Y[a:b])
        sse = ((pred - Y[a:b]) ** 2).sum()
        sse.backward()
        g, loss = reduce_gradients(theta.grad.clone(), sse, pred.numel())
        out[rank] = torch.cat([g, loss.reshape(1).to(g.dtype)])
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("B", [7, 8])
def test_reduce_gradients_equals_full_batch_mean(B):
    gen = torch.Generator().manual_seed(0)
    X = torch.randn(B, 5, 3, generator=gen, dtype=torch.float64)
    Y = torch.randn(B, 5, generator=gen, dtype=torch.float64)
    theta0 = torch.randn(4, generator=gen, dtype=torch.float64)
    world = 2
    out = torch.zeros(world, 5, dtype=torch.float64).share_memory_()
    mp.spawn(_worker, args=(world, _free_port(), X, Y, theta0, out), nprocs=world, join=True)
    theta = theta0.clone().requires_grad_(True)
    full = ((_surrogate(theta, X, Y) - Y) ** 2).mean()
    full.backward()
    for r in range(world):  # every rank holds the identical global gradient and loss
        assert torch.allclose(out[r, :4], theta.grad, rtol=1e-12, atol=1e-14)
        assert torch.allclose(out[r, 4], full.detach(), rtol=1e-12)


def test_reduce_gradients_single_process_is_mean():
    g = torch.tensor([2.0, 4.0])
    gm, loss = reduce_gradients(g, torch.tensor(6.0), 3)
    assert torch.equal(gm, torch.tensor([2.0 / 3, 4.0 / 3])) and float(loss) == 2.0


def test_balanced_partition_is_deterministic_and_balanced():
    """train.balanced_partition (ranks balanced by the adaptive solves' step counts): every sample on
    exactly one rank, same answer on every call, equal costs -> round robin, skewed costs -> loads within the
    largest single cost of each other (LPT bound)."""
    from gncde import train
    rng = np.random.default_rng(3)
    for world in (1, 2, 3, 4, 8):
        for B in (0, 1, 7, 64, 1000):
            costs = rng.integers(5, 400, size=B).tolist()
            parts = train.balanced_partition(costs, world)
            assert parts == train.balanced_partition(costs, world)
            assert sorted(i for p in parts for i in p) == list(range(B))
            loads = [sum(costs[i] for i in p) for p in parts]
            if B:
                assert max(loads) - min(loads) <= max(costs)
    assert train.balanced_partition([1.0] * 6, 3) == [[0, 3], [1, 4], [2, 5]]


def _dp_partition_rank(rank, world, port, out):
    import torch.distributed as dist
    from gncde import train
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        B = 11
        own = list(range(*train.shard_range(B, rank, world)))
        steps = [10.0 * (i + 1) for i in own]  # this rank's samples' step counts
        costs = train.global_costs(own, steps, B, "cpu")
        parts = train.balanced_partition(costs, world)
        s = train.all_reduce_sum([len(parts[rank]), sum(costs[i] for i in parts[rank])], "cpu")
        out[rank, :B] = torch.tensor(costs)
        out[rank, B] = s[0]
        out[rank, B + 1] = s[1]
    finally:
        dist.destroy_process_group()


def test_dp_cost_gather_and_rebalance_over_gloo():
    """Every rank rebuilds the full step-count vector from its own samples (global_costs) and computes the same
    balanced partition; all_reduce_sum of the per-rank sample counts / loads gives the totals."""
    import torch.multiprocessing as mp
    world, B = 3, 11
    out = torch.zeros(world, B + 2, dtype=torch.float64).share_memory_()
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_dp_partition_rank, args=(r, world, port, out)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    want = torch.tensor([10.0 * (i + 1) for i in range(B)], dtype=torch.float64)
    for r in range(world):
        assert torch.equal(out[r, :B], want)
        assert out[r, B] == B and out[r, B + 1] == float(want.sum())
