"""CPU tests of the host logic (no GPU): layout packing, fusion-table mapping, step grids, golden
fixtures regenerate from the oracle."""
import os

import numpy as np
import pytest
import torch

from gncde import layout
from oracle import gncde_oracle as O
from tests.golden import make_golden as MG


@pytest.mark.parametrize("kind", ["undirected", "directed", "plain"])
def test_product_fusion_table_matches_oracle_mapping(kind):
    rng = np.random.default_rng(11)
    n = 9
    params = O.init_vf_params(rng, kind, [5, 5, 5, 5], fusion_scale=1.0)
    ours = layout.fusion_table(kind, params.layers, n).numpy()
    ref = O.fusion_coefficient_table(params, n)
    np.testing.assert_allclose(ours, ref, rtol=0, atol=1e-15)
    A, dA = rng.standard_normal((n, n)), rng.standard_normal((n, n))
    for l in range(3):  # and the table reproduces the literal reference fusion
        np.testing.assert_allclose(O.factored_matrix(ours[l], A, dA),
                                   O.fused_matrix(params, l, A, dA) + np.eye(n), atol=1e-12)


def test_pack_control_layout():
    rng = np.random.default_rng(12)
    B, T, n = 2, 6, 5
    ts = np.sort(rng.uniform(0, 3, (B, T)), axis=1)
    Xs = rng.standard_normal((B, T, n, n, 2))
    Xs[..., 0] = ts[:, :, None, None]
    co = [O.backward_hermite_coefficients(ts[b], Xs[b]) for b in range(B)]
    coeffs = tuple(np.stack([c[q] for c in co]) for q in range(4))
    coef, tcoef = layout.pack_control(coeffs, device="cpu")
    assert coef.shape == (B, T - 1, 4, n, n) and tcoef.shape == (B, T - 1, 3, n)
    for q in range(4):
        np.testing.assert_allclose(coef[:, :, q].numpy(), coeffs[q][..., 1].astype(np.float32))
    # tcoef = column means of (d, c, b) time channel; time channel derivative == 1 exactly
    np.testing.assert_allclose(tcoef[:, :, 2].numpy(), 1.0, atol=1e-6)
    np.testing.assert_allclose(tcoef[:, :, 0].numpy(), 0.0, atol=1e-6)


def test_pack_params_order():
    rng = np.random.default_rng(13)
    params = O.init_vf_params(rng, "undirected", [3, 4, 2])
    flat = layout.pack_params(params.layers, device="cpu").numpy()
    lay0, lay1 = params.layers
    expect = np.concatenate([lay0["rms_w"], lay0["rms_b"], lay0["W"].ravel(), lay0["b"],
                             lay1["rms_w"], lay1["rms_b"], lay1["W"].ravel(), lay1["b"]]).astype(np.float32)
    np.testing.assert_array_equal(flat, expect)
    assert layout.layer_dims(params.layers) == [3, 4, 2]


@pytest.mark.parametrize("t0,t1,N", [(0.0, 5.0, 100), (0.013, 4.97, 37), (1.0, 1.5, 3)])
def test_rk4_grid_bitwise_equals_oracle(t0, t1, N):
    np.testing.assert_array_equal(layout.rk4_grid(t0, t1, N), O.rk4_grid(t0, t1, N))


@pytest.mark.parametrize("t0,t1,dt0", [(0.0, 3.0, 0.1), (0.0, 1.0, 0.01), (0.5, 2.25, 0.3)])
def test_constant_grid_bitwise_equals_oracle(t0, t1, dt0):
    np.testing.assert_array_equal(layout.constant_step_grid(t0, t1, dt0), O.constant_grid(t0, t1, dt0))


def test_stack_grids_pads_with_last_knot():
    g, ns = layout.stack_grids([np.array([0, 1, 2], np.float32), np.array([0, 0.5], np.float32)], device="cpu")
    assert g.tolist() == [[0, 1, 2], [0, 0.5, 0.5]] and ns.tolist() == [2, 1]


def test_golden_fixtures_regenerate_from_oracle(golden_dir):
    """Recompute every golden VF output from its stored inputs with the oracle (freezes the oracle)."""
    names = sorted(f for f in os.listdir(golden_dir) if f.startswith("vf_") and f.endswith(".npz"))
    assert names
    for nm in names:
        z = np.load(os.path.join(golden_dir, nm))
        params = MG.load_layers(z)
        for b in range(z["ts"].shape[0]):
            ctrl = O.CubicInterpolation(z["ts"][b], (z["d"][b], z["c"][b], z["b"][b], z["a"][b]))
            dy = O.vector_field(params, float(z["t"][b]), z["y"][b], ctrl)
            np.testing.assert_allclose(dy, z["dy"][b], rtol=1e-12, atol=1e-12)


def test_golden_solve_fixture_regenerates(golden_dir):
    z = np.load(os.path.join(golden_dir, "rk4_undirected_n10_L3.npz"))
    params = MG.load_layers(z)
    b = 1
    ctrl = O.CubicInterpolation(z["ts"][b], (z["d"][b], z["c"][b], z["b"][b], z["a"][b]))
    f = lambda t, y: O.vector_field(params, t, y, ctrl)  # noqa: E731
    g = z["grid"][b][: int(z["nsteps"][b]) + 1]
    traj, nev = O.solve_fixed_grid(f, g, z["y0"][b], "rk4", save_every_step=True, time_dtype=np.float32)
    np.testing.assert_allclose(traj, z["ys"][b][: len(g)], rtol=1e-12, atol=1e-12)
    assert nev == 4 * (len(g) - 1)


def test_engine_refuses_without_gpu():
    """The product path has no CPU fallback: calling it without a HIP device raises."""
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    import gncde
    with pytest.raises(gncde.GncdeError):
        gncde.node_affine(torch.zeros(2, 3), torch.zeros(4, 3), None)
