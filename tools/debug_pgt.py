"""Debug PGT driver pieces vs oracle (GPU box)."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "perm-equiv-graph-neural-cdes_amd")]
import numpy as np, torch
from oracle import gncde_oracle as O
import gncde
from gncde.models import PGTGraphNeuralCDE, vector_fields as V
from gncde.interpolation import CubicInterpolation
from gncde import layout, engine, _lib
rng = np.random.default_rng(24)
B, n, T, h, de, data_dim = 2, 10, 4, 8, 2, 3
ts = np.tile(np.arange(T, dtype=np.float64), (B, 1))
co_a, co_x, x0s = [], [], []
for b in range(B):
    _, X = O.make_graph_control(rng, n, T, irregular=False, t1=3.0)
    co_a.append(O.backward_hermite_coefficients(ts[b], X))
    x = rng.standard_normal((T, n, de))
    Xd = np.stack([np.broadcast_to(ts[b][:, None, None], x.shape), x], axis=-1)
    co_x.append(O.backward_hermite_coefficients(ts[b], Xd))
    x0s.append(rng.standard_normal((n, data_dim)))
ca = tuple(np.stack([c[q] for c in co_a]) for q in range(4))
cx = tuple(np.stack([c[q] for c in co_x]) for q in range(4))
x0 = np.stack(x0s)
vf = V.PermEquivGraphVectorField(h, h, h * de * 2, 2, de, n, key=9)
model = PGTGraphNeuralCDE({"hidden_dim": h, "data_dim": data_dim, "feature_dim": 1}, vf, "cubic", 5)
P = O.VFParams(vf.kind, [{k: v.double().cpu().numpy() for k, v in d.items()} for d in vf.layer_dicts()])
def mlp(m, x):
    for i, lin in enumerate(m.layers):
        x = x @ lin.weight.double().detach().numpy().T + lin.bias.double().detach().numpy()
        x = np.maximum(x, 0) if i < len(m.layers) - 1 else x
    return x
y0g = model.encoder.run(torch.tensor(x0, dtype=torch.float32, device="cuda")).cpu().numpy()
y0r = np.stack([mlp(model.encoder, x0[b]) for b in range(B)])
print("encoder err", np.abs(y0g - y0r).max() / np.abs(y0r).max())
control_adj = CubicInterpolation(torch.tensor(ts), ca); control_data = CubicInterpolation(torch.tensor(ts), cx)
prob = model.wrapped_vector_field.problem(control_adj, control_data)
g = O.constant_grid(0.0, 3.0, 0.1)
grid, ns = layout.stack_grids([g, g])
spec = engine.SolverSpec(method=_lib.TSIT5, save_mode=_lib.SAVE_T1, grid=grid, nsteps=ns)
yT = engine.integrate(prob, spec, torch.tensor(y0g, device="cuda")).cpu().numpy()
for b in range(B):
    c_a = O.CubicInterpolation(ts[b], tuple(c[b] for c in ca)); c_x = O.CubicInterpolation(ts[b], tuple(c[b] for c in cx))
    f = lambda t, y: O.cde_wrapper(P, h, de, t, y, c_a, c_x)
    yr, _ = O.solve_fixed_grid(f, g, y0g[b].astype(np.float64), "tsit5", time_dtype=np.float32)
    print("solve err", b, np.abs(yT[b] - yr).max() / np.abs(yr).max(), "|yT|", np.abs(yr).max())
    dg = model.decoder.run(torch.tensor(yr, dtype=torch.float32, device="cuda")).cpu().numpy()
    dr = mlp(model.decoder, yr)
    print("decoder err", np.abs(dg - dr).max() / np.abs(dr).max())
# sensitivity + fp32 emulation on CPU for the same problem
P32 = O.VFParams(P.kind, [{k: np.asarray(v, np.float32) for k, v in l.items()} for l in P.layers])
for b in range(B):
    c_a = O.CubicInterpolation(ts[b], tuple(c[b] for c in ca)); c_x = O.CubicInterpolation(ts[b], tuple(c[b] for c in cx))
    f = lambda t, y: O.cde_wrapper(P, h, de, t, y, c_a, c_x)
    c_a32 = O.CubicInterpolation(ts[b].astype(np.float32), tuple(np.asarray(c[b], np.float32) for c in ca))
    c_x32 = O.CubicInterpolation(ts[b].astype(np.float32), tuple(np.asarray(c[b], np.float32) for c in cx))
    f32 = lambda t, y: O.cde_wrapper(P32, h, de, np.float32(t), np.asarray(y, np.float32), c_a32, c_x32).astype(np.float64)
    y0 = y0g[b].astype(np.float64)
    yr, _ = O.solve_fixed_grid(f, g, y0, "tsit5", time_dtype=np.float32)
    yp, _ = O.solve_fixed_grid(f, g, y0 * (1 + 1e-7 * rng.standard_normal(y0.shape)), "tsit5", time_dtype=np.float32)
    y32, _ = O.solve_fixed_grid(f32, g, y0, "tsit5", time_dtype=np.float32)
    print("b", b, "sensitivity", np.abs(yp - yr).max() / np.abs(yr).max(), "fp32-emulated err", np.abs(y32 - yr).max() / np.abs(yr).max())
