"""Debug: B-sample stage-path VJP vs oracle per sample (GPU)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "perm-equiv-graph-neural-cdes_amd"))
import gncde as G  # noqa: E402
from oracle import gncde_oracle as O  # noqa: E402
from oracle import gncde_oracle_grad as OG  # noqa: E402

n, L, method, B = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], int(sys.argv[4])
rng = np.random.default_rng(100 + n)
T, h = 5, 16
tsl, col = [], []
for _ in range(B):
    ts, X = O.make_graph_control(rng, n, T, irregular=False)
    tsl.append(ts)
    col.append(O.backward_hermite_coefficients(ts, X))
ts = np.stack(tsl)
coeffs = tuple(np.stack([c[q] for c in col]) for q in range(4))
P = O.init_vf_params(rng, "undirected", [h] * (L + 1))
for lay in P.layers:
    for nm in O.UNDIRECTED_PARAMS:
        lay[nm] = lay[nm] * 3.0
grids = [O.rk4_grid(ts[b, 0], ts[b, -1], 6) if method == "rk4" else O.constant_grid(ts[b, 0], ts[b, -1], 0.8)
         for b in range(B)]
y0 = rng.standard_normal((B, n, h))
gfin = rng.standard_normal((B, n, h))
prob = G.make_problem(ts, coeffs, "undirected", P.layers)
gg, ns = G.layout.stack_grids(grids)
spec = G.SolverSpec(method=G._lib.RK4 if method == "rk4" else G._lib.TSIT5, save_mode=G._lib.SAVE_STEPS, grid=gg,
                    nsteps=ns)
ys = G.integrate(prob, spec, torch.tensor(y0, dtype=torch.float32, device="cuda"))
spec.save_mode = G._lib.SAVE_T1
gy0, gp, gf = G.integrate_vjp(prob, spec, ys, torch.tensor(gfin, dtype=torch.float32, device="cuda"))
for b in range(B):
    ctrl = O.CubicInterpolation(ts[b], tuple(c[b] for c in coeffs))
    f = lambda t, y: O.vector_field(P, t, y, ctrl)  # noqa: E731
    fv = lambda t, y, g: OG.vector_field_vjp(P, t, y, ctrl, g)  # noqa: E731
    traj, _ = O.solve_fixed_grid(f, grids[b], y0[b], method, save_every_step=True, time_dtype=np.float32)
    g0, gr = OG.solve_fixed_grid_vjp(f, fv, grids[b], y0[b], method, g_final=gfin[b])
    fe = np.max(np.abs(ys[b].cpu().numpy() - traj)) / np.max(np.abs(traj))
    ge = np.max(np.abs(gy0[b].cpu().numpy() - g0)) / np.max(np.abs(g0))
    print(f"b={b} grid {len(grids[b])} fwd {fe:.2e} gy0 {ge:.2e} |g0| {np.abs(g0).max():.3e} |gpu| {gy0[b].abs().max().item():.3e}")
