"""Training step — replaces ``make_step`` (trainer.py:288-327, trainer_pgt.py:319-358) for data-parallel
ranks (SURVEY §8 a9 + e).

    loss, grads = filter_value_and_grad(mse_loss)(model, data_i)         trainer.py:315
    updates, opt_state = optimiser.update(grads, opt_state, model)       :321  (clip_by_global_norm(1) + adamw)
    model = apply_updates(model, updates)                                :322

Here one process owns one GPU and a contiguous shard of the samples (``shard_range``).  Each rank
back-propagates the SUM of its squared errors through the GPU solve (autograd.solve -> gncde_integrate_vjp);
``reduce_gradients`` all-reduces the flat gradient and the (sse, count) pair as one fp64 bucket (one RCCL call
per step), and divides by the global element count, which is exactly the gradient of the reference's full-batch
``jnp.mean`` (loss_configs.py:47).  The optimiser update runs on the GPU over one flat parameter buffer
(gncde_clip_adamw): every rank applies the same update to the same parameters, so replicas stay identical
without a parameter broadcast.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from . import engine


def shard_range(total: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous shard [start, stop) of ``total`` samples for ``rank`` of ``world`` (sizes differ by <= 1)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    base, extra = divmod(total, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def dist_world() -> tuple[int, int]:
    """(rank, world) of the initialised process group, (0, 1) without one."""
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def balanced_partition(costs, world: int) -> list[list[int]]:
    """Samples -> ranks so that the ranks' summed costs are balanced (adaptive solves have per-sample
    step counts).  Longest-processing-time greedy: samples by decreasing cost (ties by index) each go to the rank
    with the least cost so far (ties by rank).  Deterministic, so every rank computes the same partition; each
    rank's list is returned in increasing sample order."""
    costs = [float(c) for c in costs]
    load = [0.0] * world
    parts: list[list[int]] = [[] for _ in range(world)]
    for i in sorted(range(len(costs)), key=lambda k: (-costs[k], k)):
        r = min(range(world), key=lambda q: (load[q], q))
        parts[r].append(i)
        load[r] += costs[i]
    return [sorted(p) for p in parts]


def all_reduce_sum(values, device) -> list[float]:
    """Sum a few host scalars over the ranks (one fp64 collective); identity without a process group."""
    t = torch.tensor([float(v) for v in values], dtype=torch.float64, device=device)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t.tolist()


def global_costs(own, local_costs, total: int, device) -> list[float]:
    """Every rank's per-sample costs for its own samples -> the full cost vector on every rank."""
    c = torch.zeros(total, dtype=torch.float64, device=device)
    if len(own):
        c[torch.as_tensor(list(own), device=device)] = torch.as_tensor(local_costs, dtype=torch.float64,
                                                                       device=device)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(c, op=dist.ReduceOp.SUM)
    return c.tolist()


def reduce_gradients(flat_grad: torch.Tensor, sse: torch.Tensor, count: int):
    """All-reduce (SUM) the flat gradient of this rank's summed loss and (sse, count) across ranks, then
    normalise to the gradient of the global mean.  Returns (mean-loss gradient, global mean loss).
    Works for any backend (RCCL for GPU ranks, gloo for the CPU tests); a no-op reduction when the
    process group is absent or has one rank."""
    P = flat_grad.numel()
    # One fp64 bucket [grad..., sse, count]: a single collective per step, and the element count stays exact
    # past 2^24 (config 4: 8192 x 80 x 128 targets).
    bucket = torch.cat([flat_grad.detach().reshape(-1).to(torch.float64),
                        sse.detach().to(device=flat_grad.device, dtype=torch.float64).reshape(1),
                        torch.full((1,), float(count), dtype=torch.float64, device=flat_grad.device)])
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(bucket, op=dist.ReduceOp.SUM)
    total = bucket[P + 1]
    flat_grad.copy_((bucket[:P] / total).to(flat_grad.dtype).view_as(flat_grad))
    return flat_grad, bucket[P] / total


class ClipAdamW:
    """``optax.chain(optax.clip_by_global_norm(1.0), optax.adamw(lr, weight_decay=wd))`` as built by
    ``OptimiserCfg.build`` (optimiser_configs.py:70-88), on the GPU kernel gncde_clip_adamw.

    The module's trainable parameters are re-seated as views into one flat fp32 device buffer, so the
    update is a single launch; ``flat_grad()`` gathers the gradients in the same order.
    """

    def __init__(self, module: torch.nn.Module, learning_rate: float, weight_decay: float = 0.0, b1: float = 0.9,
                 b2: float = 0.999, eps: float = 1e-8, gradient_clipping: bool = True):
        self.params = [p for p in module.parameters() if p.requires_grad]
        if not self.params:
            raise ValueError("no trainable parameters")
        dev = self.params[0].device
        if dev.type != "cuda" or any(p.device != dev for p in self.params):
            raise ValueError("ClipAdamW: move the model to one GPU first (model.to('cuda'))")
        total = sum(p.numel() for p in self.params)
        self.flat = torch.empty(total, dtype=torch.float32, device=dev)
        off = 0
        for p in self.params:
            k = p.numel()
            self.flat[off:off + k].copy_(p.detach().reshape(-1))
            p.data = self.flat[off:off + k].view_as(p)
            off += k
        self.m = torch.zeros_like(self.flat)
        self.v = torch.zeros_like(self.flat)
        self.count = 0
        self.lr, self.wd, self.b1, self.b2, self.eps = learning_rate, weight_decay, b1, b2, eps
        self.max_norm = 1.0 if gradient_clipping else 0.0

    def zero_grad(self):
        for p in self.params:
            p.grad = None

    def flat_grad(self) -> torch.Tensor:
        return torch.cat([p.grad.reshape(-1).to(torch.float32) if p.grad is not None
                          else torch.zeros(p.numel(), dtype=torch.float32, device=self.flat.device)
                          for p in self.params])

    def step(self, flat_grad: torch.Tensor, learning_rate: float | None = None) -> torch.Tensor:
        """Apply one update; returns device stats (global grad norm, max|grad|, max|update|)."""
        self.count += 1
        lr = self.lr if learning_rate is None else learning_rate
        return engine.clip_adamw(self.flat, flat_grad.contiguous(), self.m, self.v, self.count, lr, self.b1, self.b2,
                                 self.eps, self.wd, self.max_norm)


def make_step(opt: ClipAdamW, loss_terms, *args, **kwargs):
    """One data-parallel training step.  ``loss_terms(*args, **kwargs)`` returns (sum of squared errors on
    this rank's shard, element count) — e.g. ``GraphNeuralCDE.loss_terms``.  Returns (loss, max|grad|,
    max|update|) like trainer.py:327 (device scalars)."""
    opt.zero_grad()
    sse, count = loss_terms(*args, **kwargs)
    sse.backward()
    g, loss = reduce_gradients(opt.flat_grad(), sse, count)
    stats = opt.step(g)
    return loss, stats[1], stats[2]
