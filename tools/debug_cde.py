"""Debug: generic CDE solve vs oracle, step by step (GPU box)."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "perm-equiv-graph-neural-cdes_amd")]
import numpy as np, torch
from oracle import gncde_oracle as O
import gncde
from gncde import layout
rng = np.random.default_rng(5)
B, n, T, h, de = 1, 10, 4, 8, 2
ts = np.arange(T, dtype=np.float64)[None]
_, X = O.make_graph_control(rng, n, T, irregular=False, t1=3.0)
ca = tuple(c[None] for c in O.backward_hermite_coefficients(ts[0], X))
x = rng.standard_normal((T, n, de))
Xd = np.stack([np.broadcast_to(ts[0][:, None, None], x.shape), x], axis=-1)
cx = tuple(c[None] for c in O.backward_hermite_coefficients(ts[0], Xd))
P = O.init_vf_params(rng, "undirected", [h, h, h * de * 2])
prob = gncde.make_problem(ts, ca, "undirected", P.layers, data_coeffs=cx, cde_hidden=h, cde_embed=de)
y0 = rng.standard_normal((1, n, h))
c_a = O.CubicInterpolation(ts[0], tuple(c[0] for c in ca)); c_x = O.CubicInterpolation(ts[0], tuple(c[0] for c in cx))
f = lambda t, y: O.cde_wrapper(P, h, de, t, y, c_a, c_x)
for t in [0.0, 0.05, 0.5, 1.0, 1.7, 3.0]:
    dy = gncde.vf_eval(prob, torch.tensor([t], device="cuda"), torch.tensor(y0, dtype=torch.float32, device="cuda"))
    ref = f(t, y0[0])
    print("vf t=%.2f err %.2e" % (t, np.abs(dy[0].cpu().numpy() - ref).max() / np.abs(ref).max()))
for method, g in (("tsit5", O.constant_grid(0.0, 3.0, 0.1)), ("rk4", O.rk4_grid(0.0, 3.0, 30))):
    grid, ns = layout.stack_grids([g])
    spec = gncde.SolverSpec(method=gncde._lib.TSIT5 if method == "tsit5" else gncde._lib.RK4,
                            save_mode=gncde._lib.SAVE_STEPS, grid=grid, nsteps=ns)
    ys = gncde.integrate(prob, spec, torch.tensor(y0, dtype=torch.float32, device="cuda")).cpu().numpy()[0]
    traj, _ = O.solve_fixed_grid(f, g, y0[0], method, save_every_step=True, time_dtype=np.float32)
    print(method, gncde.integrate_path(prob, spec), ["%.1e" % (np.abs(ys[k] - traj[k]).max() / np.abs(traj[k]).max()) for k in range(0, len(g), 3)])
