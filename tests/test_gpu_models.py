"""GPU: the reference-interface modules (gncde.models) against the oracle on the same parameters.

Covers the drivers of SURVEY §8(a) rows a1 (GraphNeuralCDE: Tsit5 + PID + SaveAt(ts)), a7 (CDE wrapper)
and a8 (encoders / read-outs) through the same C-ABI the solver uses.
"""
import numpy as np
import pytest
import torch

from oracle import gncde_oracle as O

pytestmark = pytest.mark.gpu


def rel_err(x, ref):
    x, ref = np.asarray(x, np.float64), np.asarray(ref, np.float64)
    return float(np.max(np.abs(x - ref)) / max(np.max(np.abs(ref)), 1e-30))


@pytest.fixture(scope="module")
def G():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a HIP device")
    import gncde
    gncde._lib.load()
    return gncde


def oracle_params(vf):
    layers = [{k: v.double().cpu().numpy() for k, v in d.items()} for d in vf.layer_dicts()]
    return O.VFParams(vf.kind, layers)


def graph_controls(rng, B, n, T):
    ts_l, co_l = [], []
    for _ in range(B):
        ts, X = O.make_graph_control(rng, n, T)
        ts_l.append(ts)
        co_l.append(O.backward_hermite_coefficients(ts, X))
    return np.stack(ts_l), tuple(np.stack([c[q] for c in co_l]) for q in range(4))


def test_vf_single_sample_call_signature(G):
    """vf(t, y, CubicInterpolation(ts, coeffs)) like perm_equiv_graph_vector_field.py:85."""
    from gncde.interpolation import CubicInterpolation
    from gncde.models import vector_fields as V
    rng = np.random.default_rng(21)
    ts, coeffs = graph_controls(rng, 1, 12, 7)
    for cls in (V.PermEquivGraphVectorField, V.PermEquivDirGraphVectorField, V.GraphVectorField):
        vf = getattr(V, cls.__name__)(16, 16, 16, 3, 4, 12, key=7)  # registry lookup by name
        ctrl = CubicInterpolation(ts[0], tuple(c[0] for c in coeffs))
        y = rng.standard_normal((12, 16))
        t = float(np.float32(rng.uniform(ts[0, 0], ts[0, -1])))
        dy = vf(t, torch.tensor(y, dtype=torch.float32), ctrl)
        ref = O.vector_field(oracle_params(vf), t, y, O.CubicInterpolation(ts[0], tuple(c[0] for c in coeffs)))
        assert rel_err(dy.cpu().numpy(), ref) <= 2e-5, cls.__name__


def test_graph_neural_cde_forward_matches_oracle(G):
    """GraphNeuralCDE(ts, coeffs, x0) with the reference solve (Tsit5 + PID, SaveAt(ts))."""
    from gncde.models import GraphNeuralCDE, vector_fields as V
    rng = np.random.default_rng(22)
    B, n, T, h = 3, 12, 8, 16
    ts, coeffs = graph_controls(rng, B, n, T)
    x0 = rng.standard_normal((B, n, 1))
    vf = V.PermEquivGraphVectorField(h, h, h, 2, 16, n, key=3)
    model = GraphNeuralCDE({"hidden_dim": h}, vf, "cubic", 4)
    out, st = model.batched(torch.tensor(ts), coeffs, torch.tensor(x0), evolving_out=True, return_stats=True)
    out = out.cpu().numpy()
    assert out.shape == (B, T, n, 1)
    P = oracle_params(vf)
    Wi, bi = model.initial_linear.weight.double().detach().numpy(), model.initial_linear.bias.double().detach().numpy()
    Wf, bf = model.final_linear.weight.double().detach().numpy(), model.final_linear.bias.double().detach().numpy()
    for b in range(B):
        ctrl = O.CubicInterpolation(ts[b], tuple(c[b] for c in coeffs))
        f = lambda t, y, ctrl=ctrl: O.vector_field(P, t, y, ctrl)  # noqa: E731
        y0 = x0[b] @ Wi.T + bi
        ys, _ = O.solve_tsit5_pid(f, ts[b, 0], ts[b, -1], y0, save_ts=ts[b])
        truth, _ = O.solve_tsit5_pid(f, ts[b, 0], ts[b, -1], y0, rtol=1e-10, atol=1e-12, save_ts=ts[b],
                                     max_steps=200000)
        ref, ex = ys @ Wf.T + bf, truth @ Wf.T + bf
        # the adaptive step sequence is chaotic in the last bits: bound by the oracle's own spread
        spread = max(rel_err(O.solve_tsit5_pid(f, ts[b, 0], ts[b, -1], y0, rtol=1e-3 * s, save_ts=ts[b])[0]
                             @ Wf.T + bf, ex) for s in (1 - 1e-4, 1.0, 1 + 1e-4))
        acc_gpu = rel_err(out[b], ex)
        print(f"sample {b}: gpu {acc_gpu:.2e} oracle spread {spread:.2e} steps {st[b].tolist()}")
        assert acc_gpu <= 2.0 * max(spread, 1e-5)
    # single-sample call (the reference signature) == batched row
    one = model(torch.tensor(ts[1]), tuple(c[1] for c in coeffs), torch.tensor(x0[1]))
    assert torch.allclose(one.cpu(), torch.tensor(out[1]), rtol=0, atol=0)


def test_graph_neural_cde_rk4_override_is_fused(G):
    from gncde.models import GraphNeuralCDE, vector_fields as V
    rng = np.random.default_rng(23)
    ts, coeffs = graph_controls(rng, 2, 16, 6)
    vf = V.PermEquivGraphVectorField(16, 16, 16, 2, 16, 16, key=1)
    model = GraphNeuralCDE({"hidden_dim": 16}, vf, "cubic", 2, solver={"method": "rk4", "steps": 20})
    out = model.batched(torch.tensor(ts), coeffs, torch.tensor(rng.standard_normal((2, 16, 1))),
                        evolving_out=False)
    assert out.shape == (2, 16, 1) and torch.isfinite(out).all()


def test_pgt_driver_matches_oracle(G):
    """PGTGraphNeuralCDE: MLP encoder, CDE wrapper, Tsit5 ConstantStepSize(0.1) on [0, 3], decoder, sum."""
    from gncde.models import PGTGraphNeuralCDE, vector_fields as V
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
    with torch.no_grad():  # batched() records a backward (GPU adjoint) when grad is enabled
        out = model.batched(torch.tensor(ts), ca, cx, torch.tensor(x0)).cpu().numpy()
        per_node = model.batched(torch.tensor(ts), ca, cx, torch.tensor(x0), global_readout=False).cpu().numpy()
    P = oracle_params(vf)

    def mlp(m, x):
        for i, lin in enumerate(m.layers):
            x = x @ lin.weight.double().detach().numpy().T + lin.bias.double().detach().numpy()
            x = np.maximum(x, 0) if i < len(m.layers) - 1 else x
        return x
    for b in range(B):
        c_a = O.CubicInterpolation(ts[b], tuple(c[b] for c in ca))
        c_x = O.CubicInterpolation(ts[b], tuple(c[b] for c in cx))
        f = lambda t, y, c_a=c_a, c_x=c_x: O.cde_wrapper(P, h, de, t, y, c_a, c_x)  # noqa: E731
        grid = O.constant_grid(0.0, 3.0, 0.1)
        assert len(grid) - 1 == 30
        yT, _ = O.solve_fixed_grid(f, grid, mlp(model.encoder, x0[b]), "tsit5", time_dtype=np.float32)
        ref_nodes = mlp(model.decoder, yT)
        # this random-init CDE amplifies perturbations ~240x over the 30 steps (a 1e-7 change of y0 moves
        # yT by 2.4e-5), so an fp32 solve - GPU or the oracle's own fp32 emulation (1.4e-4) - sits ~1e-4
        # from the fp64 oracle
        assert rel_err(per_node[b], ref_nodes) <= 1e-3
        # the global read-out sums node outputs of mixed sign: judge it against the summed magnitudes
        assert abs(float(out[b, 0]) - ref_nodes.sum()) <= 1e-3 * np.abs(ref_nodes).sum()


@pytest.mark.parametrize("method", ["tsit5", "rk4"])
def test_cde_solve_matches_oracle(G, method):
    """CDE-wrapper solve (generic path) step by step against the oracle (configs 3 / 5 structure)."""
    rng = np.random.default_rng(5)
    n, T, h, de = 10, 4, 8, 2
    ts = np.arange(T, dtype=np.float64)[None]
    _, X = O.make_graph_control(rng, n, T, irregular=False, t1=3.0)
    ca = tuple(c[None] for c in O.backward_hermite_coefficients(ts[0], X))
    x = rng.standard_normal((T, n, de))
    Xd = np.stack([np.broadcast_to(ts[0][:, None, None], x.shape), x], axis=-1)
    cx = tuple(c[None] for c in O.backward_hermite_coefficients(ts[0], Xd))
    P = O.init_vf_params(rng, "undirected", [h, h, h * de * 2])
    prob = G.make_problem(ts, ca, "undirected", P.layers, data_coeffs=cx, cde_hidden=h, cde_embed=de)
    y0 = rng.standard_normal((1, n, h))
    c_a = O.CubicInterpolation(ts[0], tuple(c[0] for c in ca))
    c_x = O.CubicInterpolation(ts[0], tuple(c[0] for c in cx))
    f = lambda t, y: O.cde_wrapper(P, h, de, t, y, c_a, c_x)  # noqa: E731
    g = O.constant_grid(0.0, 3.0, 0.1) if method == "tsit5" else O.rk4_grid(0.0, 3.0, 30)
    grid, ns = G.layout.stack_grids([g])
    spec = G.SolverSpec(method=G._lib.TSIT5 if method == "tsit5" else G._lib.RK4, save_mode=G._lib.SAVE_STEPS,
                        grid=grid, nsteps=ns)
    assert G.integrate_path(prob, spec) == "generic"
    ys = G.integrate(prob, spec, torch.tensor(y0, dtype=torch.float32, device="cuda")).cpu().numpy()[0]
    traj, _ = O.solve_fixed_grid(f, g, y0[0], method, save_every_step=True, time_dtype=np.float32)
    assert rel_err(ys, traj) <= 1e-5
