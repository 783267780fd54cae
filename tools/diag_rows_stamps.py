#!/usr/bin/env python3
"""Diagnostic (GPU, experiment build only): per-phase wall time of one k_rows evaluation at BASELINE config 5's
shape, from s_memrealtime stamps (100 MHz) that a -DGNCDE_ROWS_STAMPS build of gncde_rows.hip writes (the last
round of every workgroup; with DIAG_SOLVE=1 the persistent Tsit5 + PID solve's 20th evaluation of every workgroup,
slots by ticket).  Run with GNCDE_LIB pointing at that build."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "perm-equiv-graph-neural-cdes_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import gncde  # noqa: E402
from gncde import _lib, synthetic  # noqa: E402

NAMES = ["start", "form", "operands"] + [f"{p}{l}" for l in range(3) for p in ("z", "prod", "pub")] + \
        ["z_out", "prod_out", "readout"]


def main():
    B = int(os.environ.get("DIAG_B", "16"))
    compute = os.environ.get("DIAG_COMPUTE", "fp32")
    prob, y0 = synthetic.cde_batch(B, 255, 3, 32, 8, 4, 1.0)
    prob = prob.with_compute(compute)
    t = torch.full((B,), 0.37, dtype=torch.float32, device="cuda")
    solve = os.environ.get("DIAG_SOLVE") == "1"
    spec = gncde.SolverSpec(method=_lib.TSIT5, controller=_lib.CTRL_PID, save_mode=_lib.SAVE_T1, rtol=1e-3, atol=1e-6,
                            t0=prob.ts[:, 0].contiguous(), t1=prob.ts[:, -1].contiguous(),
                            dt0=torch.full((B,), 0.01, device="cuda"))
    lib = ctypes.CDLL(_lib.LIB_PATH)
    fn = lib.gncde_debug_rows_stamps
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
    nwg = B * 16
    for rep in range(3):
        if solve:
            gncde.integrate(prob, spec, y0)
        else:
            gncde.vf_eval(prob, t, y0)
        torch.cuda.synchronize()
    buf = np.zeros(nwg * 16, dtype=np.uint64)
    assert fn(buf.ctypes.data, buf.size) == 0
    full = buf.reshape(nwg, 16).astype(np.float64)
    st = full[:, :15]
    if solve:  # slot 15: the start of the next evaluation
        it = (full[:, 15] - full[:, 0]) * 0.01
        ctl = (full[:, 15] - full[:, 14]) * 0.01
        print(f"  solve iteration (evaluation start -> next evaluation start) median {np.median(it):.2f} us, of which "
              f"controller + stage publication (read-out end -> next start) median {np.median(ctl):.2f} us")
    else:
        print(f"  rows-block Horner done (coefficient loads landed) at median "
              f"{np.median((full[:, 15] - full[:, 0]) * 0.01):.2f} us")
    t0 = st[:, 0].min()
    rel = (st - t0) * 0.01  # us
    print(f"B={B} {compute}: launch span {rel[:, 14].max():.2f} us; first WG start {0:.2f}, last WG start "
          f"{rel[:, 0].max():.2f} us")
    # group barriers: a sample's 16 workgroups (blockIdx layout of rows_vf_eval: g = (x & 7) + 8 (x / 128) when
    # the group count is a multiple of 8, else x / 16)
    G = B
    x = np.arange(nwg)
    g = (x & 7) + 8 * (x // (8 * 16)) if G % 8 == 0 and not solve else x // 16
    for name, pub, z in ((("stage input", 0, 3),) if solve else ()) + (("barrier 1", 5, 6), ("barrier 2", 8, 9),
                                                                         ("barrier 3", 11, 12)):
        last = np.array([rel[g == q, pub].max() for q in range(G)])
        first_z = np.array([rel[g == q, z].min() for q in range(G)])
        skew = np.array([rel[g == q, pub].max() - rel[g == q, pub].min() for q in range(G)])
        print(f"  {name}: last arrival -> first Z loaded median {np.median(first_z - last):.2f} us; arrival skew "
              f"median {np.median(skew):.2f} us")
    for k in range(1, 15):
        d = (st[:, k] - st[:, k - 1]) * 0.01
        print(f"  {NAMES[k]:>9}: median {np.median(d):6.2f} us  max {d.max():6.2f}  (ends at median {np.median(rel[:, k]):6.2f})")


if __name__ == "__main__":
    main()
