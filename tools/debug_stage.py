"""Debug: forward checkpoints and stage-path VJP vs oracle for one (n, L, method) case (GPU)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "perm-equiv-graph-neural-cdes_amd"))
import gncde as G  # noqa: E402
from oracle import gncde_oracle as O  # noqa: E402
from oracle import gncde_oracle_grad as OG  # noqa: E402

n, L, method = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
rng = np.random.default_rng(7)
T, h = 5, 16
ts, X = O.make_graph_control(rng, n, T, irregular=os.environ.get("IRR", "1") == "1")
coeffs = tuple(c[None] for c in O.backward_hermite_coefficients(ts, X))
ts = ts[None]
P = O.init_vf_params(rng, "undirected", [h] * (L + 1))
scale = float(sys.argv[4]) if len(sys.argv) > 4 else 1.0
dt = float(sys.argv[5]) if len(sys.argv) > 5 else 2.0
for lay in P.layers:
    for nm in O.UNDIRECTED_PARAMS:
        lay[nm] = lay[nm] * scale
grid = O.rk4_grid(ts[0, 0], ts[0, -1], 3) if method == "rk4" else O.constant_grid(ts[0, 0], ts[0, -1], dt)
y0 = rng.standard_normal((1, n, h))
gfin = rng.standard_normal((1, n, h))
ctrl = O.CubicInterpolation(ts[0], tuple(c[0] for c in coeffs))
f = lambda t, y: O.vector_field(P, t, y, ctrl)  # noqa: E731
fv = lambda t, y, g: OG.vector_field_vjp(P, t, y, ctrl, g)  # noqa: E731
traj, _ = O.solve_fixed_grid(f, grid, y0[0], method, save_every_step=True, time_dtype=np.float32)
g0, gr = OG.solve_fixed_grid_vjp(f, fv, grid, y0[0], method, g_final=gfin[0])
prob = G.make_problem(ts, coeffs, "undirected", P.layers)
gg, ns = G.layout.stack_grids([grid])
spec = G.SolverSpec(method=G._lib.RK4 if method == "rk4" else G._lib.TSIT5, save_mode=G._lib.SAVE_STEPS, grid=gg,
                    nsteps=ns)
print("forward path", G.integrate_path(prob, spec))
ys = G.integrate(prob, spec, torch.tensor(y0, dtype=torch.float32, device="cuda"))
print("max|traj|", np.abs(traj).max(), "forward rel err", np.max(np.abs(ys[0].cpu().numpy() - traj)) / np.max(np.abs(traj)))
# single VF eval / VJP at one stage via a 1-step grid from the checkpoint
spec.save_mode = G._lib.SAVE_T1
gy0, gp, gf = G.integrate_vjp(prob, spec, ys, torch.tensor(gfin, dtype=torch.float32, device="cuda"))
print("gy0 rel err", np.max(np.abs(gy0[0].cpu().numpy() - g0)) / np.max(np.abs(g0)))
gp = gp.cpu().numpy()
off = 0
for l in range(L):
    for k in ("rms_w", "rms_b", "W", "b"):
        sz = gr[l][k].size
        print(l, k, np.max(np.abs(gp[off:off + sz].reshape(gr[l][k].shape) - gr[l][k])) / np.max(np.abs(gr[l][k])))
        off += sz
