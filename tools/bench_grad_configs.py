#!/usr/bin/env python3
"""Reverse-mode timing of BASELINE configs 3 and 5 (the PGT / TGB shapes, generic reverse sweep) with and without
the stage record (GncdeSolver.stage_rec, autograd.STAGE_RECORD_SHARE = 0 disables it).

    python tools/bench_grad_configs.py [--configs 3,5] [--reps 2]

Prints one JSON line per (config, record) with forward and backward milliseconds (HIP events on the stream)."""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "perm-equiv-graph-neural-cdes_amd"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="3,5")
    ap.add_argument("--reps", type=int, default=2)
    args = ap.parse_args()
    torch.cuda.set_device(0)
    import gncde
    from gncde import autograd, layout, synthetic
    L = gncde._lib
    for c in args.configs.split(","):
        if c == "3":
            prob, y0 = synthetic.cde_batch(64, 129, 4, 64, 8, 3, 3.0)
            grid, ns = layout.stack_grids([layout.constant_step_grid(0.0, 3.0, 0.1)] * prob.B)
            spec = gncde.SolverSpec(method=L.TSIT5, save_mode=L.SAVE_T1, grid=grid, nsteps=ns)
            name = "3_england_n129_h64_de8_L3_tsit5c"
        else:
            prob, y0 = synthetic.cde_batch(16, 255, 3, 32, 8, 4, 1.0)
            B = prob.B
            spec = gncde.SolverSpec(method=L.TSIT5, controller=L.CTRL_PID, save_mode=L.SAVE_T1, rtol=1e-3, atol=1e-6,
                                    t0=torch.zeros(B, device="cuda"), t1=torch.ones(B, device="cuda"),
                                    dt0=torch.full((B,), 0.01, device="cuda"))
            name = "5_trade_n255_h32_de8_L4_tsit5pid"
        # config 5 also in BASELINE's bf16 mode (reverse mode: the fp32 adjoint over the coefficients read)
        # (problem, record share, mode, replay the accepted grid instead of the PID solve's own record)
        runs = [(prob, 0.25, "fp32", False), (prob, 0.0, "fp32", False)]
        if c == "5":
            runs = [(prob, 0.25, "fp32", False), (prob, 0.25, "fp32", True), (prob, 0.0, "fp32", True),
                    (prob.with_compute("bf16_storage"), 0.25, "bf16_storage", False),
                    (prob.with_compute("bf16"), 0.25, "bf16", False)]
        for pr, share, mode, replay in runs:
            autograd.STAGE_RECORD_SHARE = share
            autograd.NO_PID_RECORD[0] = replay
            fw, bw = [], []
            for _ in range(args.reps + 1):
                params = pr.params.clone().requires_grad_(True)
                e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
                e[0].record()
                out = autograd.solve(pr, spec, y0, params)
                loss = out.square().sum()
                e[1].record()
                loss.backward()
                e[2].record()
                torch.cuda.synchronize()
                fw.append(e[0].elapsed_time(e[1]))
                bw.append(e[1].elapsed_time(e[2]))
            dump = os.environ.get("GNCDE_BENCH_DUMP")  # A/B checks: the last repetition's gradient
            if dump:
                torch.save(params.grad.cpu(), f"{dump}_{c}_{mode}_{int(share > 0)}_{int(replay)}.pt")
            print(json.dumps({"config": name, "compute": mode, "stage_record": share > 0,
                              "pid_backward": ("replay" if replay else "record") if c == "5" else None,
                              "grad_finite": bool(torch.isfinite(params.grad).all()), "forward_ms": round(min(fw[1:]), 3),
                              "backward_ms": round(min(bw[1:]), 3)}), flush=True)
    autograd.STAGE_RECORD_SHARE = 0.25
    autograd.NO_PID_RECORD[0] = False


if __name__ == "__main__":
    main()
