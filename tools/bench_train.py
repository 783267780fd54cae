#!/usr/bin/env python3
"""Training-step benchmark — BASELINE.json configs[3] shape: gene-dynamics-shaped community
graph with exactly n=128 nodes, 1024 samples per GPU, h=16, L=2, fixed-step RK4 (100 steps), MSE on the t1
read-out, clip_by_global_norm(1) + AdamW, gradient all-reduce over RCCL when run under torch.distributed.

    python tools/bench_train.py [--steps K --warmup W --batch B]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 tools/bench_train.py ...

One step = encoder -> GPU solve (SAVE_STEPS checkpoints) -> read-out -> loss -> GPU discrete adjoint ->
all-reduce -> gncde_clip_adamw.  Prints one JSON line (rank 0) with samples/s and the forward / backward split.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "perm-equiv-graph-neural-cdes_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=1024, help="samples per GPU")
    ap.add_argument("--nodes", type=int, default=128)
    ap.add_argument("--rk4-steps", type=int, default=100)
    ap.add_argument("--knots", type=int, default=80)
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)

    import gncde
    from gncde import layout, synthetic, train
    from gncde.models import GraphNeuralCDE, vector_fields as V

    B, n, h, L = args.batch, args.nodes, 16, 2
    prob, _, _ = synthetic.heat_batch(B, num_nodes=n, hidden=h, num_layers=L, T=args.knots, seed=1234 + rank,
                                      graph="community")
    vf = V.PermEquivGraphVectorField(h, h, h, L, 16, n, key=0)
    model = GraphNeuralCDE({"hidden_dim": h}, vf, "cubic", 1, solver={"method": "rk4", "steps": args.rk4_steps})
    model.to("cuda")
    opt = train.ClipAdamW(model, learning_rate=1e-3, weight_decay=1e-4)
    g = torch.Generator().manual_seed(99 + rank)
    x0 = torch.randn(B, prob.n, 1, generator=g).cuda()
    labels = torch.randn(B, prob.n, generator=g).cuda()
    grid, ns = layout.stack_grids([layout.rk4_grid(0.0, 5.0, args.rk4_steps)] * B)
    spec = gncde.SolverSpec(method=gncde._lib.RK4, save_mode=gncde._lib.SAVE_T1, grid=grid, nsteps=ns)

    def loss_terms():
        pred = model.predict_packed(prob, x0, spec).squeeze(-1)
        return ((pred - labels) ** 2).sum(), pred.numel()

    for _ in range(args.warmup):
        train.make_step(opt, loss_terms)
    torch.cuda.synchronize()

    # split timing of one step (forward / backward+update) with events on the launch stream
    s = torch.cuda.current_stream()
    e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    opt.zero_grad()
    e[0].record(s)
    sse, cnt = loss_terms()
    e[1].record(s)
    sse.backward()
    gflat, _ = train.reduce_gradients(opt.flat_grad(), sse, cnt)
    opt.step(gflat)
    e[2].record(s)
    torch.cuda.synchronize()
    fwd_ms, bwd_ms = e[0].elapsed_time(e[1]), e[1].elapsed_time(e[2])

    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss, mg, mu = train.make_step(opt, loss_terms)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device="cuda")
    if dist:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    elapsed = float(el.item())
    if rank == 0:
        fwd_evals = 4 * args.rk4_steps
        out = {"metric": "GNCDE training step (forward + discrete adjoint + all-reduce + AdamW)",
               "value": round(B * world * args.steps / elapsed, 1), "unit": "samples/s",
               "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
               "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True, "scaling": "weak",
               "forward_ms": round(fwd_ms, 3), "backward_update_ms": round(bwd_ms, 3),
               "forward_sample_evals_per_s": round(B * fwd_evals / (fwd_ms * 1e-3), 1),
               "loss": float(loss), "max_grad": float(mg), "max_update": float(mu),
               "dtype": "fp32", "data": "synthetic community graph (4 blocks) with edge events, random labels",
               "config": {"workload": f"gene_n{prob.n}_b{B}_L{L}_h{h}_T{args.knots}_rk4x{args.rk4_steps}_train",
                          "global_batch": B * world, "per_gpu_batch": B, "parallelism": f"dp{world}",
                          "forward_path": gncde.integrate_path(prob, gncde.SolverSpec(
                              method=gncde._lib.RK4, save_mode=gncde._lib.SAVE_STEPS, grid=grid, nsteps=ns))}}
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
