"""Known-answer and property tests of the CPU oracle.

The data-side known answers mirror the reference's own tests (test/dataset/test_misc.py:43-58);
everything else is analytic (the hot path has no reference fixtures: parity unpinned).
"""
import numpy as np
import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from oracle import gncde_oracle as O


# ---- reference known answers (test/dataset/test_misc.py) ------------------------------------------
def test_zipf_smoothing_two_nodes():
    """test_misc.py:26-33 (pinned: expected 0.5 everywhere)."""
    A = np.array([[0, 1], [1, 0]], dtype=float)
    np.testing.assert_allclose(O.zipf_smoothing(A), [[0.5, 0.5], [0.5, 0.5]], rtol=1e-5)


def test_normalized_plus_two_nodes():
    """test_misc.py:36-41 (pinned: expected ones)."""
    A = np.array([[0, 1], [1, 0]], dtype=float)
    np.testing.assert_allclose(O.normalized_plus(A), [[1, 1], [1, 1]], rtol=1e-5)


def test_normalized_laplacian_two_nodes_follows_code():
    """The reference's test_misc.py:43-50 expects I - A = [[1,-1],[-1,1]], but misc.py:83-99 adds
    self-loops before normalising, which gives I - 0.5*ones.  The hot path consumes the CODE's
    operator (get_graph_operator default), so the oracle follows the code; the reference test is stale.
    """
    A = np.array([[0, 1], [1, 0]], dtype=float)
    np.testing.assert_allclose(O.normalized_laplacian(A), [[0.5, -0.5], [-0.5, 0.5]], rtol=1e-5)


def test_normalized_adj_two_nodes_follows_code():
    """Same staleness as above for test_misc.py:52-58 (misc.py:102-113 adds self-loops)."""
    A = np.array([[0, 1], [1, 0]], dtype=float)
    np.testing.assert_allclose(O.normalized_adj(A), [[0.5, 0.5], [0.5, 0.5]], rtol=1e-5)


# ---- spline ---------------------------------------------------------------------------------------
def _spline(rng, T=9, shape=(3, 4)):
    ts = np.sort(rng.uniform(0, 5, T))
    ys = rng.standard_normal((T,) + shape)
    return ts, ys, O.backward_hermite_coefficients(ts, ys)


def test_hermite_reproduces_knots_and_backward_slopes():
    rng = np.random.default_rng(0)
    ts, ys, co = _spline(rng)
    for k in range(len(ts)):
        np.testing.assert_allclose(O.spline_evaluate(ts, co, ts[k]), ys[k], atol=1e-12)
    for k in range(1, len(ts)):
        slope = (ys[k] - ys[k - 1]) / (ts[k] - ts[k - 1])
        np.testing.assert_allclose(O.spline_derivative(ts, co, ts[k]), slope, rtol=1e-10, atol=1e-10)


def test_hermite_first_interval_linear_and_c1():
    rng = np.random.default_rng(1)
    ts, ys, (d, c, b, a) = _spline(rng)
    assert np.all(d[0] == 0) and np.all(c[0] == 0)
    for k in range(1, len(ts) - 1):  # C1 at interior knots
        h = ts[k] - ts[k - 1]
        left = b[k - 1] + h * (2 * c[k - 1] + 3 * h * d[k - 1])
        np.testing.assert_allclose(left, b[k], rtol=1e-9, atol=1e-9)


def test_time_channel_derivative_is_exactly_one():
    rng = np.random.default_rng(2)
    ts32 = np.sort(rng.uniform(0, 5, 20)).astype(np.float32)
    X = np.broadcast_to(ts32[:, None, None], (20, 5, 5)).astype(np.float32)
    d, c, b, a = O.backward_hermite_coefficients(ts32, X)
    assert np.all(b == 1.0) and np.all(c == 0.0) and np.all(d == 0.0)
    assert np.all(np.mean(b, axis=1) == 1.0)


@pytest.mark.parametrize("t,expect", [(0.0, 0), (1.0, 0), (1.5, 1), (2.0, 1), (2.0000001, 2), (4.0, 3),
                                      (9.0, 3), (-1.0, 0)])
def test_interval_index_rule(t, expect):
    ts = np.array([0.0, 1.0, 2.0, 3.0, 4.0])
    assert O.interval_index(ts, t) == expect


# ---- fusion ---------------------------------------------------------------------------------------
KINDS = ["undirected", "directed", "plain"]


@pytest.mark.parametrize("kind", KINDS)
def test_factored_table_reproduces_literal_fusion(kind):
    rng = np.random.default_rng(3)
    n = 7
    A, dA = rng.standard_normal((n, n)), rng.standard_normal((n, n))
    params = O.init_vf_params(rng, kind, [4, 4, 4], fusion_scale=1.0)
    tab = O.fusion_coefficient_table(params, n)
    for l in range(2):
        lit = O.fused_matrix(params, l, A, dA) + np.eye(n)
        np.testing.assert_allclose(O.factored_matrix(tab[l], A, dA), lit, rtol=1e-12, atol=1e-12)


def test_fusion_single_coefficient_basis():
    """Only param5[0] non-zero: Abar = A (+ dA) + p/n * tile(rowsum(A)) (term_5 broadcasts along rows)."""
    rng = np.random.default_rng(4)
    n = 5
    A, dA = rng.standard_normal((n, n)), rng.standard_normal((n, n))
    p = {nm: np.zeros(2) for nm in O.UNDIRECTED_PARAMS}
    p["param5"][0] = 0.7
    expect = A + dA + 0.7 / n * np.tile(A.sum(1), (n, 1))
    np.testing.assert_allclose(O.fusion_undirected(p, A, dA), expect, atol=1e-12)
    p = {nm: np.zeros(2) for nm in O.UNDIRECTED_PARAMS}
    p["param7"][1] = 0.3  # quirk: multiplies sum(A) (layers.py:147)
    np.testing.assert_allclose(O.fusion_undirected(p, A, dA), A + dA + 0.3 / n**2 * A.sum(), atol=1e-12)
    p = {nm: np.zeros(2) for nm in O.UNDIRECTED_PARAMS}
    p["param3"][1] = 2.0
    np.testing.assert_allclose(O.fusion_undirected(p, A, dA), A + dA + 2.0 * np.diag(np.diag(dA)), atol=1e-12)


@settings(max_examples=20, deadline=None)
@given(seed=st.integers(0, 2**31 - 1), kind=st.sampled_from(KINDS))
def test_vector_field_permutation_equivariant(seed, kind):
    rng = np.random.default_rng(seed)
    n, T = 6, 5
    ts, X = O.make_graph_control(rng, n, T)
    params = O.init_vf_params(rng, kind, [4, 4, 4], fusion_scale=1.0)
    y = rng.standard_normal((n, 4))
    t = rng.uniform(ts[0], ts[-1])
    P = rng.permutation(n)
    ctrl = O.CubicInterpolation(ts, O.backward_hermite_coefficients(ts, X))
    ctrlP = O.CubicInterpolation(ts, O.backward_hermite_coefficients(ts, X[:, P][:, :, P]))
    out = O.vector_field(params, t, y, ctrl)
    outP = O.vector_field(params, t, y[P], ctrlP)
    np.testing.assert_allclose(outP, out[P], rtol=1e-10, atol=1e-10)


def test_conv_layer_reductions():
    rng = np.random.default_rng(5)
    n, d = 5, 3
    Z = rng.standard_normal((n, d))
    lay = {"W": np.eye(d), "b": np.zeros(d), "rms_w": np.ones(d), "rms_b": np.zeros(d)}
    np.testing.assert_allclose(O.conv_layer(Z, np.zeros((n, n)), lay), O.rmsnorm(Z, 1.0, 0.0), atol=1e-12)
    np.testing.assert_allclose(O.conv_layer(Z, -np.eye(n), lay), 0.0, atol=1e-12)


# ---- solvers --------------------------------------------------------------------------------------
def test_rk4_fourth_order_on_linear_ode():
    f = lambda t, y: -1.3 * y  # noqa: E731
    errs = []
    for N in (10, 20):
        g = O.rk4_grid(0.0, 2.0, N, dtype=np.float64)
        y, nev = O.solve_fixed_grid(f, g, np.array([1.0]))
        assert nev == 4 * N
        errs.append(abs(y[0] - np.exp(-2.6)))
    assert 12 < errs[0] / errs[1] < 20


def test_tsit5_fifth_order_on_linear_ode():
    f = lambda t, y: -1.3 * y  # noqa: E731
    errs = []
    for dt in (0.2, 0.1):
        g = O.constant_grid(0.0, 2.0, dt, dtype=np.float64, tol=1e-10)
        y, _ = O.solve_fixed_grid(f, g, np.array([1.0]), method="tsit5")
        errs.append(abs(y[0] - np.exp(-2.6)))
    assert errs[0] / errs[1] > 25


def test_tsit5_dense_weights_at_one_equal_b():
    np.testing.assert_allclose(O.tsit5_dense_weights(1.0), O.TSIT5_B, atol=1e-12)
    np.testing.assert_allclose(O.tsit5_dense_weights(0.0), 0.0, atol=1e-15)


def test_constant_step_grid_counts():
    """PGT: dt0=0.1 on [0,3] and TGB: dt0=0.01 on [0,1] (pgt_graph_neural_cde.py:110, tgb_...:340)."""
    g = O.constant_grid(0.0, 3.0, 0.1)
    assert len(g) - 1 == 30 and g[-1] == np.float32(3.0)
    g = O.constant_grid(0.0, 1.0, 0.01)
    assert len(g) - 1 == 100 and g[-1] == np.float32(1.0)
    assert np.all(np.diff(g) > 0)


def test_pid_solver_accuracy_and_dense_output():
    f = lambda t, y: np.stack([y[1], -y[0]])  # noqa: E731  harmonic oscillator
    ts = np.linspace(0, 3, 7)
    ys, stats = O.solve_tsit5_pid(f, 0.0, 3.0, np.array([1.0, 0.0]), rtol=1e-6, atol=1e-9, save_ts=ts)
    np.testing.assert_allclose(ys[:, 0], np.cos(ts), atol=1e-5)
    assert stats["steps"] > 3 and stats["evals"] == 3 + 6 * (stats["steps"] + stats["rejects"])
