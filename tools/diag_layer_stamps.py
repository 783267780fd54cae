#!/usr/bin/env python3
"""Diagnostic (GPU, experiment build only): per-phase wall time of the fp32 CDE read-out k_layer launch (MODE 2) in
BASELINE config 3's forward (B = 64, n = 129, h = 64, L = 3, de = 8), from the s_memrealtime stamps (100 MHz) that a
-DGNCDE_LAYER_STAMPS build of gncde_layer.hip writes (the last read-out launch).  Run with GNCDE_LIB pointing at that
build (perm-equiv-graph-neural-cdes_amd/Makefile `make stamps`)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "perm-equiv-graph-neural-cdes_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import gncde  # noqa: E402
from gncde import _lib, layout, synthetic  # noqa: E402

PHASES = ["Z staging", "RMSNorm factors", "P product", "P partials", "read-out K loop", "bias, sums, stores"]


def main():
    prob, y0 = synthetic.cde_batch(64, 129, 4, 64, 8, 3, 3.0)
    grid, ns = layout.stack_grids([layout.constant_step_grid(0.0, 0.3, 0.1)] * prob.B)
    spec = gncde.SolverSpec(method=_lib.TSIT5, save_mode=_lib.SAVE_T1, grid=grid, nsteps=ns)
    lib = ctypes.CDLL(_lib.LIB_PATH)
    fn = lib.gncde_debug_layer_stamps
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
    for _ in range(3):
        gncde.engine.integrate(prob, spec, y0)
        torch.cuda.synchronize()
    buf = np.zeros(1024 * 8, dtype=np.uint64)
    assert fn(buf.ctypes.data, buf.size) == 0
    st = buf.reshape(1024, 8).astype(np.float64)
    st = st[st[:, 0] > 0]
    t0 = st[:, 0].min()
    print(f"config 3 read-out: {len(st)} workgroups; launch span {(st[:, 6].max() - t0) * 0.01:.2f} us, last start "
          f"{(st[:, 0].max() - t0) * 0.01:.2f} us")
    starts = np.sort((st[:, 0] - t0) * 0.01)
    print("  start times (us) at workgroup quantiles 0.25/0.5/0.75/0.9/1: "
          + ", ".join(f"{np.quantile(starts, q):.2f}" for q in (0.25, 0.5, 0.75, 0.9, 1.0)))
    for k in range(1, 7):
        d = (st[:, k] - st[:, k - 1]) * 0.01
        print(f"  {PHASES[k - 1]:>22}: median {np.median(d):6.2f} us  max {d.max():6.2f}")
    print(f"  {'workgroup total':>22}: median {np.median((st[:, 6] - st[:, 0]) * 0.01):6.2f} us")


if __name__ == "__main__":
    main()
