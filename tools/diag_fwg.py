#!/usr/bin/env python3
"""Diagnostic (GPU): the persistent solve with forms workgroups (GNCDE_SOLVE_FWG=1) against the in-line forms
(GNCDE_SOLVE_FWG=0) at config 5's shape: per case, FW repeatability and the FW vs in-line differences."""
import dataclasses
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "perm-equiv-graph-neural-cdes_amd")]

import torch  # noqa: E402

import gncde  # noqa: E402
from gncde import _lib, layout, synthetic  # noqa: E402


def main():
    B = int(os.environ.get("DIAG_B", "16"))
    prob, y0 = synthetic.cde_batch(B, 255, 3, 32, 8, 4, 1.0, seed=63)
    if os.environ.get("DIAG_COMPUTE"):
        prob = prob.with_compute(os.environ["DIAG_COMPUTE"])
    pid = gncde.SolverSpec(method=_lib.TSIT5, controller=_lib.CTRL_PID, save_mode=_lib.SAVE_T1, rtol=1e-3, atol=1e-6,
                           t0=prob.ts[:, 0].contiguous(), t1=prob.ts[:, -1].contiguous(),
                           dt0=torch.full((B,), 0.01, device="cuda"))
    grid, ns = layout.stack_grids([layout.constant_step_grid(0.0, 1.0, 0.05)] * B)
    rgrid, rns = layout.stack_grids([layout.constant_step_grid(0.0, 1.0, 0.1)] * B)
    cases = {"rk4_t1": gncde.SolverSpec(method=_lib.RK4, save_mode=_lib.SAVE_T1, grid=rgrid, nsteps=rns),
             "tsit5_steps": gncde.SolverSpec(method=_lib.TSIT5, save_mode=_lib.SAVE_STEPS, grid=grid, nsteps=ns),
             "pid": pid}
    for name, sp in cases.items():
        res = {}
        for v in ("1", "1b", "0"):
            os.environ["GNCDE_SOLVE_FWG"] = v[0]
            path = gncde.integrate_path(prob, sp)
            rec = torch.zeros(B, 256, device="cuda")
            sp2 = dataclasses.replace(sp, step_ts=rec) if sp.controller == _lib.CTRL_PID else sp
            ys, st = gncde.integrate(prob, sp2, y0, stats=True)
            torch.cuda.synchronize()
            res[v] = (path, ys, st, rec)
        a, b, c = res["1"], res["1b"], res["0"]
        print(f"{name}: paths {a[0]} / {c[0]}; FW repeat equal {torch.equal(a[1], b[1])}, "
              f"FW vs inline max|diff| {float((a[1] - c[1]).abs().max()):.3e} (rel "
              f"{float((a[1] - c[1]).abs().max() / c[1].abs().max()):.2e}); stats equal {torch.equal(a[2], c[2])}; "
              f"FW status {a[2][:, 3].tolist()}")
        if not torch.equal(a[2], c[2]):
            print("   FW stats", a[2][:, :3].tolist())
            print("   in stats", c[2][:, :3].tolist())
        if name == "pid":
            d = (a[3] - c[3]).abs().max(dim=1).values
            print("   per-sample step-record max|diff|", [f"{x:.1e}" for x in d.tolist()])
            for bb in range(min(B, 2)):
                k = int((a[3][bb] != c[3][bb]).nonzero()[0]) if not torch.equal(a[3][bb], c[3][bb]) else -1
                print(f"   sample {bb}: first differing accepted step {k}: FW {a[3][bb, max(k-1,0):k+2].tolist()} "
                      f"in {c[3][bb, max(k-1,0):k+2].tolist()}")


if __name__ == "__main__":
    main()
