#!/usr/bin/env python3
"""Diagnostic: fixed-grid solve reverse mode (the generic sweep) vs the fp64 oracle, for B = 1 / 2 and L = 3 / 4."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "perm-equiv-graph-neural-cdes_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import gncde as G  # noqa: E402
from oracle import gncde_oracle as O  # noqa: E402
from oracle import gncde_oracle_grad as OG  # noqa: E402
from tests.golden import make_golden as MG  # noqa: E402


def rel(a, r):
    return float(np.max(np.abs(np.asarray(a) - r)) / np.max(np.abs(r)))


for (n, H, L, B, same, scale) in [(40, 32, 4, 1, False, 3.0), (40, 32, 4, 2, False, 3.0), (64, 32, 4, 2, False, 3.0),
                                  (64, 32, 4, 2, False, 1.0), (64, 32, 3, 2, False, 3.0)]:
    rng = np.random.default_rng(7000 + n + H)
    T = 4
    ts, coeffs, P = MG.problem(rng, B, n, T, "undirected", [H] * (L + 1), irregular=False)
    for lay in P.layers:
        for nm in OG.FUSION_NAMES["undirected"]:
            lay[nm] = lay[nm] * scale
    if same:  # every sample the same control
        ts = np.repeat(ts[:1], B, 0)
        coeffs = tuple(np.repeat(c[:1], B, 0) for c in coeffs)
    prob = G.make_problem(ts, coeffs, P.kind, P.layers)
    grids = [O.rk4_grid(ts[b, 0], ts[b, -1], 3) for b in range(B)]
    y0 = rng.standard_normal((B, n, H))
    gfin = rng.standard_normal((B, n, H))
    grid, ns = G.layout.stack_grids(grids)
    spec = G.SolverSpec(method=G._lib.RK4, save_mode=G._lib.SAVE_STEPS, grid=grid, nsteps=ns)
    ys = G.integrate(prob, spec, torch.tensor(y0, dtype=torch.float32, device="cuda"))
    spec1 = G.SolverSpec(method=G._lib.RK4, save_mode=G._lib.SAVE_T1, grid=grid, nsteps=ns)
    gy0 = G.integrate_vjp(prob, spec1, ys, torch.tensor(gfin, dtype=torch.float32, device="cuda"))[0].cpu().numpy()
    errs = []
    for b in range(B):
        ctrl = O.CubicInterpolation(ts[b], tuple(c[b] for c in coeffs))
        f = lambda t, y, c=ctrl: O.vector_field(P, t, y, c)  # noqa: E731
        fv = lambda t, y, g, c=ctrl: OG.vector_field_vjp(P, t, y, c, g)  # noqa: E731
        g_or, _ = OG.solve_fixed_grid_vjp(f, fv, grids[b], y0[b], "rk4", g_final=gfin[b])
        errs.append(rel(gy0[b], g_or))
    print(f"n={n} H={H} L={L} B={B} scale={scale}: gy0 rel err per sample {[f'{e:.1e}' for e in errs]}", flush=True)
