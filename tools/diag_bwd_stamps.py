#!/usr/bin/env python3
"""Diagnostic (GPU, experiment build only): per-phase wall time of one k_bwd_layer launch (layer 1) in the reverse
sweep of BASELINE config 3's shape (B = 64, n = 129, h = 64, L = 3, de = 8) or config 5's (DIAG_CFG=5), from the
s_memrealtime stamps (100 MHz) that a -DGNCDE_BWD_STAMPS build of gncde_rows_vjp.hip writes (the last layer-1
launch).  Run with GNCDE_LIB pointing at that build (perm-equiv-graph-neural-cdes_amd/Makefile `make stamps`)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "perm-equiv-graph-neural-cdes_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import gncde  # noqa: E402
from gncde import _lib, autograd, layout, synthetic  # noqa: E402

PHASES = ["form (loads, Horner, node features)", "operand registers", "zhat / g_P staging", "RMSNorm factors",
          "node sums", "K loop + row terms", "partials + fusion sums", "P / g_zhat rows", "g_W' partials",
          "RMSNorm^T + next g_out", "g_P_next, g_q_next"]


def main():
    cfg = os.environ.get("DIAG_CFG", "3")
    if cfg == "3":
        prob, y0 = synthetic.cde_batch(64, 129, 4, 64, 8, 3, 3.0)
        grid, ns = layout.stack_grids([layout.constant_step_grid(0.0, 0.2, 0.1)] * prob.B)
    else:
        prob, y0 = synthetic.cde_batch(16, 255, 3, 32, 8, 4, 1.0)
        grid, ns = layout.stack_grids([layout.constant_step_grid(0.0, 0.2, 0.1)] * prob.B)
    spec = gncde.SolverSpec(method=_lib.TSIT5, save_mode=_lib.SAVE_T1, grid=grid, nsteps=ns)
    lib = ctypes.CDLL(_lib.LIB_PATH)
    fn = lib.gncde_debug_bwd_stamps
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
    for _ in range(3):
        params = prob.params.clone().requires_grad_(True)
        autograd.solve(prob, spec, y0, params).square().sum().backward()
        torch.cuda.synchronize()
    buf = np.zeros(1024 * 16, dtype=np.uint64)
    assert fn(buf.ctypes.data, buf.size) == 0
    full = buf.reshape(1024, 16).astype(np.float64)
    full = full[full[:, 0] > 0]
    st = full[:, :12]
    t0 = st[:, 0].min()
    print(f"config {cfg}: {len(st)} workgroups; launch span {(st[:, 11].max() - t0) * 0.01:.2f} us, last start "
          f"{(st[:, 0].max() - t0) * 0.01:.2f} us")
    for k in range(1, 12):
        d = (st[:, k] - st[:, k - 1]) * 0.01
        print(f"  {PHASES[k - 1]:>38}: median {np.median(d):6.2f} us  max {d.max():6.2f}")
    print(f"  {'workgroup total':>38}: median {np.median((st[:, 11] - st[:, 0]) * 0.01):6.2f} us")
    sub = full[:, 12:15]
    if (sub > 0).all():  # form sub-stamps (from the launch start of each workgroup)
        for k, name in enumerate(["interval found", "A, dA operands arrived", "coefficient sums arrived"]):
            d = (sub[:, k] - st[:, 0]) * 0.01
            print(f"  {'form: ' + name:>38}: median {np.median(d):6.2f} us  max {d.max():6.2f}")


if __name__ == "__main__":
    main()
