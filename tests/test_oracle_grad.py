"""CPU: pin the reverse-mode oracle (oracle/gncde_oracle_grad.py) by central finite differences of the
fp64 forward oracle — the gradient the reference's training step takes (trainer.py:315) cannot be run
here (no jax), so this is what anchors it."""
import numpy as np
import pytest

from oracle import gncde_oracle as O
from oracle import gncde_oracle_grad as OG


def _problem(rng, kind, dims, n=6, T=5):
    ts, X = O.make_graph_control(rng, n, T)
    ctrl = O.CubicInterpolation(ts, O.backward_hermite_coefficients(ts, X))
    P = O.init_vf_params(rng, kind, dims)
    for lay in P.layers:
        lay["rms_w"] = lay["rms_w"] + 0.2 * rng.standard_normal(lay["rms_w"].shape)
        lay["rms_b"] = lay["rms_b"] + 0.2 * rng.standard_normal(lay["rms_b"].shape)
        for nm in OG.FUSION_NAMES[kind]:
            lay[nm] = lay[nm] * 5.0  # make the fusion terms matter at this size
    return ts, ctrl, P


def _directional_fd(fun, x, v, eps=1e-6):
    return (fun(x + eps * v) - fun(x - eps * v)) / (2 * eps)


@pytest.mark.parametrize("kind,dims", [("undirected", [4, 5, 4]), ("directed", [4, 4, 4, 4]),
                                       ("plain", [3, 6, 3])])
def test_vector_field_vjp_matches_finite_differences(kind, dims):
    rng = np.random.default_rng(11)
    ts, ctrl, P = _problem(rng, kind, dims)
    n = 6
    y = rng.standard_normal((n, dims[0]))
    g = rng.standard_normal((n, dims[-1]))
    t = float(rng.uniform(ts[0], ts[-1]))
    gy, grads = OG.vector_field_vjp(P, t, y, ctrl, g)
    theta = OG.params_to_vector(P)
    gtheta = OG.grads_to_vector(grads, kind)
    for _ in range(3):
        vy = rng.standard_normal(y.shape)
        vt = rng.standard_normal(theta.shape)
        fd = _directional_fd(lambda s: float(np.sum(g * O.vector_field(
            OG.vector_to_params(theta + s * vt, P), t, y + s * vy, ctrl))), 0.0, 1.0)
        an = float(np.sum(gy * vy) + np.sum(gtheta * vt))
        assert abs(fd - an) <= 1e-7 * max(1.0, abs(an)), (fd, an)


def test_cde_wrapper_vjp_matches_finite_differences():
    rng = np.random.default_rng(12)
    n, T, h, de = 5, 4, 3, 2
    ts = np.arange(T, dtype=np.float64)
    _, X = O.make_graph_control(rng, n, T, irregular=False, t1=3.0)
    ca = O.CubicInterpolation(ts, O.backward_hermite_coefficients(ts, X))
    x = rng.standard_normal((T, n, de))
    Xd = np.stack([np.broadcast_to(ts[:, None, None], x.shape), x], axis=-1)
    cx = O.CubicInterpolation(ts, O.backward_hermite_coefficients(ts, Xd))
    P = O.init_vf_params(rng, "undirected", [h, 4, h * de * 2])
    y = rng.standard_normal((n, h))
    g = rng.standard_normal((n, h))
    t = 1.3
    gy, grads = OG.cde_wrapper_vjp(P, h, de, t, y, ca, cx, g)
    theta, gtheta = OG.params_to_vector(P), OG.grads_to_vector(grads, "undirected")
    vy, vt = rng.standard_normal(y.shape), rng.standard_normal(theta.shape)
    fd = _directional_fd(lambda s: float(np.sum(g * O.cde_wrapper(
        OG.vector_to_params(theta + s * vt, P), h, de, t, y + s * vy, ca, cx))), 0.0, 1.0)
    an = float(np.sum(gy * vy) + np.sum(gtheta * vt))
    assert abs(fd - an) <= 1e-7 * max(1.0, abs(an))


@pytest.mark.parametrize("method,steps_mode", [("rk4", False), ("rk4", True), ("tsit5", False)])
def test_solve_vjp_matches_finite_differences(method, steps_mode):
    rng = np.random.default_rng(13)
    kind, dims = "undirected", [4, 4, 4]
    ts, ctrl, P = _problem(rng, kind, dims)
    n = 6
    y0 = rng.standard_normal((n, dims[0]))
    grid = O.rk4_grid(ts[0], ts[-1], 6) if method == "rk4" else O.constant_grid(ts[0], ts[-1], 0.9)
    G = len(grid)
    gsteps = rng.standard_normal((G, n, dims[0])) if steps_mode else None
    gfin = None if steps_mode else rng.standard_normal((n, dims[0]))

    def f_of(theta):
        Pt = OG.vector_to_params(theta, P)
        return lambda t, y: O.vector_field(Pt, t, y, ctrl)

    f = f_of(OG.params_to_vector(P))
    fv = lambda t, y, g: OG.vector_field_vjp(P, t, y, ctrl, g)  # noqa: E731
    gy0, grads = OG.solve_fixed_grid_vjp(f, fv, grid, y0, method, g_final=gfin, g_steps=gsteps)
    theta, gtheta = OG.params_to_vector(P), OG.grads_to_vector(grads, kind)

    def loss(s, vy, vt):
        ys, _ = O.solve_fixed_grid(f_of(theta + s * vt), grid, y0 + s * vy, method, save_every_step=True,
                                   time_dtype=np.float32)
        return float(np.sum(gsteps * ys)) if steps_mode else float(np.sum(gfin * ys[-1]))

    for _ in range(2):
        vy, vt = rng.standard_normal(y0.shape), rng.standard_normal(theta.shape)
        fd = _directional_fd(lambda s: loss(s, vy, vt), 0.0, 1.0)
        an = float(np.sum(gy0 * vy) + np.sum(gtheta * vt))
        assert abs(fd - an) <= 1e-6 * max(1.0, abs(an)), (fd, an)


def test_data_spline_vjp_matches_finite_differences():
    """Cotangent of the CDE wrapper's data knots (TGBGraphNeuralCDE's in-forward spline of the embedded data,
    tgb_graph_neural_cde.py:118-130) through a whole RK4 solve: cde_wrapper_vjp(data_grad=True) + hermite_vjp."""
    rng = np.random.default_rng(13)
    n, T, h, de = 4, 4, 3, 2
    ts = np.arange(T, dtype=np.float64)
    _, X = O.make_graph_control(rng, n, T, irregular=False, t1=3.0)
    ca = O.CubicInterpolation(ts, O.backward_hermite_coefficients(ts, X))
    x = rng.standard_normal((T, n, de))
    P = O.init_vf_params(rng, "undirected", [h, 4, h * de * 2])
    y0 = rng.standard_normal((n, h))
    g = rng.standard_normal((n, h))
    grid = O.rk4_grid(ts[0], ts[-1], 5)

    def spline(xv):
        Xd = np.stack([np.broadcast_to(ts[:, None, None], xv.shape), xv], axis=-1)
        return O.CubicInterpolation(ts, O.backward_hermite_coefficients(ts, Xd))

    cx = spline(x)
    f = lambda t, y: O.cde_wrapper(P, h, de, t, y, ca, cx)  # noqa: E731
    fv = lambda t, y, gg: OG.cde_wrapper_vjp(P, h, de, t, y, ca, cx, gg, data_grad=True)  # noqa: E731
    _, total = OG.solve_fixed_grid_vjp(f, fv, grid, y0, "rk4", g_final=g, time_dtype=None)
    gX = OG.hermite_vjp(ts, total[-1]["data_coef"])[..., 1]  # channel 1 = data (channel 0 = time)

    def loss(xv):
        c = spline(xv)
        yT, _ = O.solve_fixed_grid(lambda t, y: O.cde_wrapper(P, h, de, t, y, ca, c), grid, y0, "rk4",
                                   time_dtype=None)
        return float(np.sum(g * yT))

    for _ in range(2):
        v = rng.standard_normal(x.shape)
        fd = _directional_fd(lambda s: loss(x + s * v), 0.0, 1.0)
        an = float(np.sum(gX * v))
        assert abs(fd - an) <= 1e-6 * max(1.0, abs(an)), (fd, an)


@pytest.mark.parametrize("kind,dims", [("undirected", [4, 4, 4]), ("directed", [3, 4, 3])])
def test_adaptive_solve_dense_vjp_matches_finite_differences(kind, dims):
    """Reverse mode of the reference's training solve, Tsit5 + PIDController(1e-3, 1e-6) with SaveAt(ts)
    (graph_neural_cde.py:53-54,89-104 under trainer.py:315), on its accepted step sequence with the step sizes held
    constant: solve_grid_dense_vjp against central differences of solve_grid_dense on that grid.  Save times include
    t0 (the initial state itself), knots inside steps and t1."""
    rng = np.random.default_rng(21)
    ts, ctrl, P = _problem(rng, kind, dims)
    n = 6
    y0 = rng.standard_normal((n, dims[0]))

    def f_of(theta):
        Pt = OG.vector_to_params(theta, P)
        return lambda t, y: O.vector_field(Pt, t, y, ctrl)

    f = f_of(OG.params_to_vector(P))
    ys, st = O.solve_tsit5_pid(f, ts[0], ts[-1], y0, save_ts=ts)
    grid = st["grid"]
    assert len(grid) == st["steps"] + 1 and st["rejects"] >= 0
    # the dense forward on the recorded grid reproduces the adaptive solve's output
    assert np.max(np.abs(OG.solve_grid_dense(f, grid, y0, ts, time_dtype=None) - ys)) <= 1e-12 * np.max(np.abs(ys))
    g = rng.standard_normal(ys.shape)
    fv = lambda t, y, gg: OG.vector_field_vjp(P, t, y, ctrl, gg)  # noqa: E731
    gy0, grads = OG.solve_grid_dense_vjp(f, fv, grid, y0, ts, g)
    theta, gtheta = OG.params_to_vector(P), OG.grads_to_vector(grads, kind)

    def loss(s, vy, vt):
        return float(np.sum(g * OG.solve_grid_dense(f_of(theta + s * vt), grid, y0 + s * vy, ts)))

    for _ in range(2):
        vy, vt = rng.standard_normal(y0.shape), rng.standard_normal(theta.shape)
        fd = _directional_fd(lambda s: loss(s, vy, vt), 0.0, 1.0)
        an = float(np.sum(gy0 * vy) + np.sum(gtheta * vt))
        assert abs(fd - an) <= 1e-6 * max(1.0, abs(an)), (fd, an)
