"""GPU: the input-side kernels — gncde_graph_operator against the oracle operators, which the
reference's own known-answer tests pin (test/dataset/test_misc.py, mirrored in tests/test_oracle.py), and
gncde_hermite_coefficients bit-exact against an fp32 restatement of diffrax.backward_hermite_coefficients."""
import numpy as np
import pytest
import torch

from oracle import gncde_oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def G():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a HIP device")
    import gncde
    gncde._lib.load()
    return gncde


def test_graph_operator_reference_known_answers(G):
    """test_misc.py:26-41: the 2-node graph, zipf smoothing -> 0.5 everywhere, normalized_plus -> ones."""
    A = torch.tensor([[[0.0, 1.0], [1.0, 0.0]]])
    np.testing.assert_allclose(G.engine.graph_operator(A, "kipf")[0].cpu().numpy(), np.full((2, 2), 0.5), rtol=1e-6)
    np.testing.assert_allclose(G.engine.graph_operator(A, "normalized_plus")[0].cpu().numpy(), np.ones((2, 2)),
                               rtol=1e-6)


@pytest.mark.parametrize("kind,ref", [("norm_lap", O.normalized_laplacian), ("norm_adj", O.normalized_adj),
                                      ("kipf", O.zipf_smoothing), ("normalized_plus", O.normalized_plus),
                                      ("lap_unknown_name_defaults", O.normalized_laplacian)])
def test_graph_operator_matches_oracle(G, kind, ref):
    rng = np.random.default_rng(3)
    B, n = 3, 37
    A = (rng.random((B, n, n)) < 0.2) * rng.lognormal(size=(B, n, n))
    A[0, 5, :] = 0.0  # an isolated row: exercises the zero-degree guard of normalized_plus
    A[0, :, 5] = 0.0
    out = G.engine.graph_operator(torch.tensor(A), kind).cpu().numpy()
    for b in range(B):
        np.testing.assert_allclose(out[b], ref(A[b]), rtol=2e-5, atol=2e-6)


def _hermite_f32(ts, X):
    """fp32 restatement with the kernel's operation order (diffrax backward_hermite_coefficients)."""
    f = np.float32
    ts = ts.astype(f)
    X = X.astype(f)
    T = ts.shape[0]
    dt = (ts[1:] - ts[:-1]).reshape((T - 1,) + (1,) * (X.ndim - 1))
    slope = (X[1:] - X[:-1]) / dt
    deriv = np.concatenate([slope[:1], slope[:-1]], axis=0)
    dd = slope - deriv
    return -dd / (dt * dt), f(2.0) * dd / dt, deriv, X[:-1]


@pytest.mark.parametrize("shape", [(9, 9), (7, 3, 2)])
def test_hermite_coefficients_bit_exact(G, shape):
    rng = np.random.default_rng(4)
    B, T = 3, 11
    ts = np.sort(rng.uniform(0, 5, (B, T)), axis=1).astype(np.float32)
    ts[:, 0] = 0.0
    X = rng.standard_normal((B, T) + shape).astype(np.float32)
    out = G.engine.hermite_coefficients(torch.tensor(ts), torch.tensor(X)).cpu().numpy()
    assert out.shape == (B, T - 1, 4) + shape
    for b in range(B):
        ref = _hermite_f32(ts[b], X[b])
        for q in range(4):
            np.testing.assert_array_equal(out[b, :, q], ref[q])
        ref64 = O.backward_hermite_coefficients(ts[b].astype(np.float64), X[b].astype(np.float64))
        for q in range(4):
            scale = np.abs(ref64[q]).max()
            assert np.max(np.abs(out[b, :, q] - ref64[q])) <= 1e-4 * scale


def test_control_from_knots_equals_reference_layout_packing(G):
    """layout.control_from_knots (kernel) == layout.pack_control of the reference-layout coefficient tuple."""
    rng = np.random.default_rng(5)
    B, T, n = 2, 8, 12
    ts_l, X_l, co_l = [], [], []
    for _ in range(B):
        ts, X = O.make_graph_control(rng, n, T)
        ts_l.append(ts)
        X_l.append(X)
        co_l.append(O.backward_hermite_coefficients(ts.astype(np.float32).astype(np.float64),
                                                    X.astype(np.float32).astype(np.float64)))
    ts = np.stack(ts_l).astype(np.float32)
    X = np.stack(X_l).astype(np.float32)  # [B, T, n, n, 2], channel 0 = time
    coef, tcoef = G.layout.control_from_knots(torch.tensor(ts), torch.tensor(X[..., 1]), torch.tensor(X[..., 0]))
    ref_coef, ref_tcoef = G.layout.pack_control(tuple(np.stack([c[q] for c in co_l]) for q in range(4)))
    scale = ref_coef.abs().max()
    assert torch.max(torch.abs(coef - ref_coef)) <= 1e-4 * scale
    assert torch.max(torch.abs(tcoef - ref_tcoef)) <= 1e-4 * ref_tcoef.abs().max()
