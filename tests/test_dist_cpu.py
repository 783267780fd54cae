"""CPU, world_size 2 over gloo: the data-parallel pieces of the training step —
contiguous sharding and the gradient/loss all-reduce that turns per-rank summed losses into the gradient
of the reference's full-batch mean (loss_configs.py:47).  The GPU solve itself is exercised in
tests/test_gpu_grad.py; here a torch surrogate loss stands in for it so the collective logic runs on CPU."""
import os
import socket

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
