#!/usr/bin/env python3
"""Throughput of the BASELINE configs outside bench.py's headline (configs 3 and 5, CDE-wrapper shapes) and of
config 4's forward, one GPU.  Prints one JSON line per config: sample-evals/s, ms per solve, the kernel path,
and the algorithmic TFLOP/s (SURVEY §8d flops/eval) against the fp32 MFMA peak.

    python tools/bench_configs.py [--configs 3,4,5] [--reps 3]
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

FP32_PEAK = 157.3


def flops_per_eval(n, dims, de=0):
    """the (I + Abar) m product of every layer charged at that layer's output width."""
    f = 19 * n * n
    for l in range(1, len(dims)):
        f += 22 * n * n + 2 * n * n * dims[l] + 2 * n * dims[l - 1] * dims[l] + 6 * n * dims[l]
    return f + (4 * n * dims[-1] if de else 0)


def executed_flops_per_eval(n, dims, de=0):
    """The same model as the generic path executes it: a widening layer (the CDE read-out, d_L = 16 h) runs the n x n
    product at its input width in the reassociated order ((I + Abar) diag(inv) Z) W'^T (gncde_generic.hip)."""
    f = 19 * n * n
    for l in range(1, len(dims)):
        w = min(dims[l], dims[l - 1])
        f += 22 * n * n + 2 * n * n * w + 2 * n * dims[l - 1] * dims[l] + 6 * n * dims[l]
    return f + (4 * n * dims[-1] if de else 0)


def run(name, prob, spec, y0, reps, ref=None, ref_steps=None):
    import gncde
    path = gncde.integrate_path(prob, spec)
    ys, st = gncde.integrate(prob, spec, y0, stats=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        ys, st = gncde.integrate(prob, spec, y0, stats=True)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    evals = int(st[:, 2].sum())
    fpe = flops_per_eval(prob.n, prob.dims, prob.cde_embed)
    out = {"config": name, "path": path, "B": prob.B, "n": prob.n, "dims": prob.dims, "ms_per_solve": round(dt * 1e3, 2),
           "sample_evals_per_s": round(evals / dt, 1), "evals_per_sample": evals / prob.B,
           "tflops_algorithmic": round(evals * fpe / dt / 1e12, 3),
           "mfma_frac": round(evals * fpe / dt / 1e12 / FP32_PEAK, 4),
           "executed_frac": round(evals * executed_flops_per_eval(prob.n, prob.dims, prob.cde_embed) / dt / 1e12
                                  / FP32_PEAK, 4),
           "finite": bool(torch.isfinite(ys).all()),
           "steps_mean": float(st[:, 0].float().mean()), "rejects_mean": float(st[:, 1].float().mean())}
    if ref is not None:  # deviation of this arithmetic from the fp32 solve of the same problem
        out["rel_dev_vs_fp32"] = float((ys - ref).abs().max() / ref.abs().max())
    if ref_steps is not None:  # accepted steps per sample against the fp32 solve's
        d = (st[:, 0].float() - ref_steps.float()).abs() / ref_steps.float()
        out["steps_max_rel_diff_vs_fp32"] = round(float(d.max()), 4)
    print(json.dumps(out), flush=True)
    dump = os.environ.get("GNCDE_BENCH_DUMP")  # A/B checks: the solve's output
    if dump:
        torch.save(ys.cpu(), f"{dump}_{name}.pt")
    return ys, st[:, 0].clone()


EXPERIMENT_BF16M = os.environ.get("GNCDE_EXPERIMENT_BF16_MFMA") == "1"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="3,4,5")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--batch5", type=int, default=16, help="config 5 windows per launch (the TGB trainer uses 1)")
    ap.add_argument("--quick", action="store_true", help="config 5: fp32 and bf16_storage only")
    args = ap.parse_args()
    torch.cuda.set_device(0)
    import gncde
    from gncde import layout, synthetic
    L = gncde._lib
    for c in args.configs.split(","):
        if c == "3":  # England-shaped: n=129, h=64, de=8, L=3, d_L=1024, Tsit5 dt0=0.1 on [0, 3], B=64
            prob, y0 = synthetic.cde_batch(64, 129, 4, 64, 8, 3, 3.0)
            grid, ns = layout.stack_grids([layout.constant_step_grid(0.0, 3.0, 0.1)] * prob.B)
            spec = gncde.SolverSpec(method=L.TSIT5, save_mode=L.SAVE_T1, grid=grid, nsteps=ns)
            ys, _ = run("3_england_n129_h64_de8_L3_tsit5c", prob, spec, y0, args.reps)
            if EXPERIMENT_BF16M:  # (the retired single-plane mode: experiment build only)
                run("3_england_n129_h64_de8_L3_tsit5c_bf16_mfma", prob.with_compute("bf16_mfma"), spec, y0, args.reps,
                    ref=ys)
        elif c == "4":  # gene community n=128, h=16, L=2, RK4 100 steps, B=1024 (forward)
            prob, y0, _ = synthetic.heat_batch(1024, num_nodes=128, hidden=16, num_layers=2, T=80, graph="community")
            grid, ns = layout.stack_grids([layout.rk4_grid(0.0, 5.0, 100)] * prob.B)
            spec = gncde.SolverSpec(method=L.RK4, save_mode=L.SAVE_T1, grid=grid, nsteps=ns)
            run("4_gene_n128_h16_L2_rk4x100", prob, spec, y0, args.reps)
        elif c == "5":  # TGB-trade-shaped: n=255, h=32, L=4, de=8, d_L=512, Tsit5 + PID on [0, 1], B=16
            prob, y0 = synthetic.cde_batch(args.batch5, 255, 3, 32, 8, 4, 1.0)
            B = prob.B
            spec = gncde.SolverSpec(method=L.TSIT5, controller=L.CTRL_PID, save_mode=L.SAVE_T1, rtol=1e-3, atol=1e-6,
                                    t0=torch.zeros(B, device="cuda"), t1=torch.ones(B, device="cuda"),
                                    dt0=torch.full((B,), 0.01, device="cuda"))
            ys, s32 = run("5_trade_n255_h32_de8_L4_tsit5pid", prob, spec, y0, args.reps)
            # BASELINE config 5's bf16 path: bf16 operator coefficients in the persistent solve, fp32 products
            run("5_trade_n255_h32_de8_L4_tsit5pid_bf16_storage", prob.with_compute("bf16_storage"), spec, y0,
                args.reps, ref=ys, ref_steps=s32)
            if not args.quick:  # the multi-kernel split-product mode
                run("5_trade_n255_h32_de8_L4_tsit5pid_bf16", prob.with_compute("bf16"), spec, y0, args.reps, ref=ys,
                    ref_steps=s32)
            # the reference's own fixed grid (100 Tsit5 steps), fp32 and bf16 storage (the retired single-plane mode
            # too, against an experiment build)
            grid, ns = layout.stack_grids([layout.constant_step_grid(0.0, 1.0, 0.01)] * B)
            fspec = gncde.SolverSpec(method=L.TSIT5, save_mode=L.SAVE_T1, grid=grid, nsteps=ns)
            yf, _ = run("5_trade_fixed100", prob, fspec, y0, args.reps)
            run("5_trade_fixed100_bf16_storage", prob.with_compute("bf16_storage"), fspec, y0, args.reps, ref=yf)
            if not args.quick and EXPERIMENT_BF16M:
                run("5_trade_fixed100_bf16_mfma", prob.with_compute("bf16_mfma"), fspec, y0, args.reps, ref=yf)


if __name__ == "__main__":
    main()
