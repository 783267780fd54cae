#!/usr/bin/env python3
"""bench.py — GNCDE vector-field evals/sec on BASELINE.json configs[1]:
Heat-Diffusion n=64, batch=1024 per GPU, L=3, hidden 16, fixed-step RK4 (100 steps) on MI355X.

One "step" = one gncde_integrate launch that solves the whole per-GPU batch (1024 samples x 100 RK4
steps x 4 vector-field evaluations = 409,600 sample-evals) with inputs already resident in HBM.

  python bench.py [--gpus N --steps K --warmup W]
  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

Multi-GPU: samples are independent, so each rank integrates its own 1024-sample shard
with no collective in the data path ("scaling": "weak"); the timed region is bracketed by barrier +
synchronize and the max over ranks is reported.  Rank 0 prints ONE JSON line.  `--gpus N` with N > 1 and no
torch.distributed environment starts the N ranks itself (a torch.distributed.run child, before any GPU call) and
exits with its status; a WORLD_SIZE that disagrees with --gpus is an error.

The line also carries "train": BASELINE config 4's data-parallel training step (community graph n = 128, 1024
samples per GPU, h = 16, L = 2, RK4 x 100: forward, discrete adjoint, ONE gradient all-reduce over RCCL, ClipAdamW),
timed the same way (barrier + synchronize, max over ranks), so the 1 -> N curve includes the collective.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "perm-equiv-graph-neural-cdes_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

METRIC = "GNCDE vector-field evals/sec (batch×n×n) at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0       # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
FP32_MFMA_PEAK_TFS = 157.3  # MI355X_MICROARCH.md: f32 MFMA dense (= f32 vector peak)


def algorithmic_flops_per_eval(n, dims):
    """19 n^2 (spline) + sum_l [22 n^2 + 2 n^2 d_l + 2 n d_{l-1} d_l + 6 n d_l]."""
    f = 19 * n * n
    for l in range(1, len(dims)):
        f += 22 * n * n + 2 * n * n * dims[l] + 2 * n * dims[l - 1] * dims[l] + 6 * n * dims[l]
    return f


def executed_flops_per_sample(n, dims, rk4_steps):
    """The §8(d) flops as the fused kernel executes them: the spline (19 n^2) and every layer's fusion build
    (22 n^2) once per DISTINCT stage time (2 S + 1 forms per RK4 solve), the layer products once per evaluation."""
    forms, evals = 2 * rk4_steps + 1, 4 * rk4_steps
    per_form = 19 * n * n + 22 * n * n * (len(dims) - 1)
    per_eval = sum(2 * n * n * dims[l] + 2 * n * dims[l - 1] * dims[l] + 6 * n * dims[l] for l in range(1, len(dims)))
    return forms * per_form + evals * per_eval


def algorithmic_bytes_per_sample(n, d0, dL, T, rk4_steps):
    """HBM bytes one RK4 solve of one sample must move.  SURVEY §8(d) charges the active interval's fp32
    (d, c, b, a) operator-channel coefficients (16 n^2 B) and the time-channel means (12 n B) per vector-field
    evaluation; an RK4 step has only two DISTINCT stage times (k2/k3 share t + h/2, k4 shares t + h with the next
    step's k1), so a solve needs them 2 S + 1 times, not 4 S.  Plus the state in / out and the knots."""
    forms = 2 * rk4_steps + 1
    return forms * (16 * n * n + 12 * n) + 4 * n * (d0 + dL) + 4 * T


def source_sha16(rel):
    import hashlib
    with open(os.path.join(ROOT, rel), "rb") as fh:
        return hashlib.sha256(fh.read()).hexdigest()[:16]


FUSED_SRC = "perm-equiv-graph-neural-cdes_amd/csrc/gncde_fused.hip"


def load_traffic(workload, kernel):
    """HBM bytes per launch from the committed rocprofv3 PMC summary (profiles/pmc_traffic.json), or None when
    the file was measured on another workload, another kernel instance, or another revision of the kernel
    source (keyed by the sha256 of gncde_fused.hip, so a stale measurement is refused)."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(p) as fh:
            d = json.load(fh)
        if (d.get("workload") == workload and d.get("kernel") == kernel
                and d.get("source_sha16") == source_sha16(FUSED_SRC)):
            return float(d["hbm_bytes_per_launch"])
    except (OSError, ValueError, KeyError):
        pass
    return None


def roofline(bytes_per_launch, flops_per_launch, kernel_ms, traffic):
    """Both bounds for the dominant kernel; the binding one is chosen by arithmetic intensity against the fp32
    ridge point (peak flops / peak bandwidth), not by whichever fraction is larger."""
    sec = kernel_ms * 1e-3
    gbs = bytes_per_launch / sec / 1e9
    tfs = flops_per_launch / sec / 1e12
    hbm = {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": round(gbs / HBM_PEAK_GBS, 4), "algorithmic_per_launch": bytes_per_launch}
    mfma = {"bound": "mfma", "achieved": round(tfs, 2), "peak": FP32_MFMA_PEAK_TFS, "unit": "TFLOP/s",
            "frac": round(tfs / FP32_MFMA_PEAK_TFS, 4), "algorithmic_per_launch": flops_per_launch}
    intensity = flops_per_launch / bytes_per_launch
    ridge = FP32_MFMA_PEAK_TFS * 1e12 / (HBM_PEAK_GBS * 1e9)
    roof, alt = (mfma, hbm) if intensity >= ridge else (hbm, mfma)
    for r in (roof, alt):
        if r["frac"] > 1.0:  # physically impossible: the work model, not the kernel, is wrong
            print(f"bench.py: roofline fraction {r['frac']} > 1 for bound {r['bound']}", file=sys.stderr)
            r["valid"] = False
    roof["traffic"] = traffic
    roof["kernel_ms"] = round(kernel_ms, 4)
    roof["intensity_flop_per_byte"] = round(intensity, 2)
    roof["ridge_flop_per_byte"] = round(ridge, 2)
    if traffic is not None:
        alt["measured_hbm_GBs"] = round(traffic / sec / 1e9, 1)
    return roof, alt


def cpu_baseline(prob, spec, y0, layers, target_s):
    """The C restatement (oracle/gncde_oracle.c, OpenMP) on a bounded sample of the same workload."""
    from oracle import c_oracle
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or len(os.sched_getaffinity(0))
    threads = max(1, min(threads, len(os.sched_getaffinity(0))))
    lay = [{k: v.numpy() for k, v in L.items()} for L in layers]

    def run(nb):
        ts = prob.ts[:nb].cpu().numpy()
        coef = prob.coef[:nb].cpu().numpy()
        tcoef = prob.tcoef[:nb].cpu().numpy()
        grid = spec.grid[:nb].cpu().numpy()
        ns = spec.nsteps[:nb].cpu().numpy()
        yy = y0[:nb].cpu().numpy()
        t0 = time.perf_counter()
        _, nev = c_oracle.rk4(ts, coef, tcoef, lay, grid, ns, yy, nthreads=threads)
        return nev, time.perf_counter() - t0

    model = "unknown"
    try:  # the host CPU the baseline ran on (/proc/cpuinfo "model name")
        with open("/proc/cpuinfo") as fh:
            model = next((ln.split(":", 1)[1].strip() for ln in fh if ln.startswith("model name")), model)
    except OSError:
        pass
    c_oracle.load()
    nev1, dt1 = run(1)  # calibration (1 sample, 1 thread busy)
    nb = int(max(threads, min(prob.B, math.ceil(target_s / max(dt1, 1e-6)) * threads)))
    nb = min(nb, prob.B)
    nev, dt = run(nb)
    return {"value": nev / dt, "unit": "sample-evals/s", "cores": threads, "cpu_model": model, "kind": "port",
            "sample": f"{nb} of the {prob.B} samples, full 100-step RK4 solve each ({nev} VF evals, "
                      f"{dt:.1f} s, oracle/gncde_oracle.c fp32, literal reference fusion, OpenMP)"}


def world_from_env(gpus: int):
    """(world, rank, local_rank) from the torch.distributed environment; the world size must equal --gpus."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != gpus:
        raise SystemExit(f"bench.py: --gpus {gpus} but WORLD_SIZE={world}")
    return world, rank, local


def launch_ranks(gpus: int, argv) -> int:
    """Run this script as `gpus` ranks (one process per GPU) under torch.distributed.run; returns its status.
    Called before anything touches the GPU (the parent only waits)."""
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    return subprocess.call(cmd, env=env)


def reduce_over_ranks(dist, device, elapsed: float, units: float):
    """(max elapsed over ranks, sum of units over ranks): the job's time and its whole work."""
    el = torch.tensor([elapsed], dtype=torch.float64, device=device)
    tot = torch.tensor([units], dtype=torch.float64, device=device)
    if dist is not None:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
    return float(el.item()), float(tot.item())


def train_line(dist, rank, world, steps, warmup, rk4_steps):
    """BASELINE config 4's training step per rank (tools/bench_train.py's workload), whole-job samples/s."""
    import gncde
    from gncde import layout, synthetic, train
    from gncde.models import GraphNeuralCDE, vector_fields as V
    B, n, h, L, T = 1024, 128, 16, 2, 80
    prob, _, _ = synthetic.heat_batch(B, num_nodes=n, hidden=h, num_layers=L, T=T, seed=4321 + rank,
                                      graph="community")
    vf = V.PermEquivGraphVectorField(h, h, h, L, 16, n, key=0)
    model = GraphNeuralCDE({"hidden_dim": h}, vf, "cubic", 1, solver={"method": "rk4", "steps": rk4_steps}).to("cuda")
    opt = train.ClipAdamW(model, learning_rate=1e-3, weight_decay=1e-4)
    g = torch.Generator().manual_seed(99 + rank)
    x0 = torch.randn(B, n, 1, generator=g).cuda()
    labels = torch.randn(B, n, generator=g).cuda()
    grid, ns = layout.stack_grids([layout.rk4_grid(0.0, 5.0, rk4_steps)] * B)
    spec = gncde.SolverSpec(method=gncde._lib.RK4, save_mode=gncde._lib.SAVE_T1, grid=grid, nsteps=ns)

    def loss_terms():
        pred = model.predict_packed(prob, x0, spec).squeeze(-1)
        return ((pred - labels) ** 2).sum(), pred.numel()

    for _ in range(warmup):
        train.make_step(opt, loss_terms)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        loss, _, _ = train.make_step(opt, loss_terms)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed, samples = reduce_over_ranks(dist, "cuda", time.perf_counter() - t0, B * steps)
    out = {"metric": "GNCDE training step (forward + discrete adjoint + gradient all-reduce + ClipAdamW)",
           "value": round(samples / elapsed, 1), "unit": "samples/s", "n_gpus": world, "steps": steps,
           "warmup": warmup, "ms_per_step": round(elapsed / steps * 1e3, 3), "scaling": "weak",
           "loss": float(loss),
           "config": {"workload": f"gene_community_n{n}_b{B}_L{L}_h{h}_T{T}_rk4x{rk4_steps}_train",
                      "global_batch": B * world, "per_gpu_batch": B, "parallelism": f"dp{world}",
                      "collective": "one fp64 all-reduce bucket per step (RCCL)" if world > 1 else "none"}}
    del prob, model, opt
    torch.cuda.empty_cache()
    return out if rank == 0 else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=1024, help="samples per GPU")
    ap.add_argument("--rk4-steps", type=int, default=100)
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--train-steps", type=int, default=5, help="config-4 training steps timed (0: no train line)")
    ap.add_argument("--dist-selftest", action="store_true",
                    help="CPU check of the rank plumbing: gloo ranks reduce (rank + 1, rank + 10), no GPU work")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    world, rank, local = world_from_env(args.gpus)
    if args.dist_selftest:
        import torch.distributed as tdist
        if world > 1:
            tdist.init_process_group("gloo")
        mx, tot = reduce_over_ranks(tdist if world > 1 else None, "cpu", rank + 1.0, rank + 10.0)
        if rank == 0:
            print(json.dumps({"world": world, "max_elapsed": mx, "sum_units": tot}), flush=True)
        if world > 1:
            tdist.destroy_process_group()
        return
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)

    import gncde
    from gncde import layout, synthetic

    n_nodes, hidden, L, T = 64, 16, 3, 120
    B = args.batch
    prob, y0, layers = synthetic.heat_batch(B, num_nodes=n_nodes, hidden=hidden, num_layers=L, T=T,
                                            seed=1234 + rank)
    grids = [layout.rk4_grid(0.0, 5.0, args.rk4_steps)] * B  # every sample spans [0, final_time]
    grid, ns = layout.stack_grids(grids)
    spec = gncde.SolverSpec(method=gncde._lib.RK4, save_mode=gncde._lib.SAVE_T1, grid=grid, nsteps=ns)
    path = gncde.integrate_path(prob, spec)
    workload = f"heat_n{prob.n}_b{B}_L{L}_h{hidden}_T{T}_rk4x{args.rk4_steps}"

    # BASELINE config 4's training line runs between building the headline problem and its launches: besides its
    # own measurement it keeps the GPU busy up to the headline region (launched after an idle host-side setup, the
    # first ~12 k_fused launches ramp 3.26 -> 2.66 ms as the clocks rise, profiles/r05_bench_notes.txt)
    tr = None
    if args.train_steps > 0:
        tr = train_line(dist, rank, world, args.train_steps, 1, args.rk4_steps)

    ys, st = gncde.integrate(prob, spec, y0, stats=True)
    evals_per_launch = int(st[:, gncde._lib.STAT_EVALS].sum().item())
    for _ in range(args.warmup):
        gncde.integrate(prob, spec, y0)
    torch.cuda.synchronize()

    stream = torch.cuda.current_stream()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        gncde.integrate(prob, spec, y0)
    ev1.record(stream)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kernel_ms = ev0.elapsed_time(ev1) / args.steps  # one fused launch per step, same stream

    elapsed, total_evals = reduce_over_ranks(dist, "cuda", elapsed, evals_per_launch * args.steps)
    value = total_evals / elapsed

    if rank == 0:
        n = prob.n
        bytes_launch = B * algorithmic_bytes_per_sample(n, hidden, hidden, T, args.rk4_steps)
        flops_launch = evals_per_launch * algorithmic_flops_per_eval(n, prob.dims)
        roof, alt = roofline(bytes_launch, flops_launch, kernel_ms, load_traffic(workload, path))
        if roof["bound"] == "mfma":  # beside the §8(d) model: the flops the kernel actually executes per launch
            ex = B * executed_flops_per_sample(n, prob.dims, args.rk4_steps)
            roof["executed_per_launch"] = ex
            roof["executed_frac"] = round(ex / (kernel_ms * 1e-3) / 1e12 / FP32_MFMA_PEAK_TFS, 4)
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(prob, spec, y0, layers, args.cpu_seconds)
        out = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "sample-evals/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32",
            "data": "synthetic: heat-diffusion-shaped 8x8 grid graph with edge events, normalized-Laplacian "
                    "operator path, backward-Hermite coefficients built on device; random reference-init params",
            "config": {"workload": workload, "global_batch": B * world, "per_gpu_batch": B, "n": n,
                       "hidden": hidden, "layers": L, "knots": T, "solver": "rk4",
                       "solver_steps": args.rk4_steps, "parallelism": f"dp{world}"},
            "edge_evals_per_s": round(value * n * n, 1),
            "kernel": path,
            "roofline": roof,
            "roofline_other": alt,
            "cpu_baseline": cpu,
            "train": tr,
        }
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
