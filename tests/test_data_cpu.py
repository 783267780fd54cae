"""CPU: the dataset restatement's host logic — config parsing, event indices, split,
padding by events — against the reference rules (ode_dataset.py, data_tools.py, dataset_configs.py)."""
import os

import numpy as np

from gncde import data


def test_cfg_from_reference_yaml_block_ignores_unknown_keys():
    cfg = data.DynDataCfg.from_dict({"name": "heat", "batch_size": 4, "num_nodes": 400, "cache_dir": ".cache",
                                     "layout": "community", "split_ratio": [0.8, 0.2]})
    assert cfg.name == "heat" and cfg.batch_size == 4 and cfg.num_nodes == 400
    assert list(cfg.split_ratio) == [0.8, 0.2]


def test_grid_graph_degrees():
    """data_tools.py grid: corners have 3 neighbours, edges 5, interior 8 (test_data_tools.py:18-35)."""
    A = data.grid_8_neighbor_graph(4)
    deg = A.sum(1).reshape(4, 4)
    assert deg[0, 0] == 3 and deg[0, 1] == 5 and deg[1, 1] == 8
    assert np.array_equal(A, A.T) and np.all(np.diag(A) == 0)


def test_split_irregular_follows_reference_rules():
    rng = np.random.default_rng(0)
    tr, extra, inter = data.split_indices(rng, "irregular", 100, (0.8, 0.2))
    assert extra == list(range(100, 120))
    assert len(inter) == 20 and 0 not in inter and sorted(inter) == inter
    assert sorted(set(tr) | set(inter)) == list(range(100)) and not set(tr) & set(inter)
    tr, extra, inter = data.split_indices(rng, "equal", 100, (0.8, 0.2))
    assert tr == list(range(80)) and extra == list(range(80, 100)) and inter is None


def test_events_and_padding():
    rng = np.random.default_rng(1)
    t = np.sort(rng.uniform(0, 5, (3, 120)), axis=1)
    ev_t, idx = data.events_happen_time(rng, t, 12, (0.8, 0.2), True)
    assert ev_t.shape == (3, 12) and np.all(np.diff(idx) > 0)
    assert np.sum(idx < 96) == 10 and np.all(idx >= 2)  # ceil(12 * 0.8) training events from index 2
    epoch = data.padding_by_time(100, idx)
    assert epoch[0] == 0 and epoch[-1] == np.sum(idx < 100) and np.all(np.diff(epoch) >= 0)
    A = np.zeros((2, 5, 5))
    stack = data.events_happen_graph(rng, A, 3, 0.5)
    assert stack.shape == (2, 4, 5, 5)


def test_split_sizes_match_reference_test():
    """test_ode_dataset.py:54-60 (irregular sampling, time_tick 100, split 0.8 / 0.2)."""
    rng = np.random.default_rng(1234)
    tr, extra, inter = data.split_indices(rng, "irregular", 100, (0.8, 0.2))
    assert len(tr) == int(100 * 0.8)
    assert len(extra) == 100 - len(tr)
    assert inter is not None


def test_ground_truth_solver_linear_known_answer():
    """diffeqsolve(ODETerm, Tsit5 | Dopri5, ConstantStepSize(dt0), SaveAt(ts)) restated (ode_dataset.py:279-293):
    dy/dt = lam y against exp(lam t) at irregular save times that fall between steps (dense output), per-sample
    time grids of different lengths, and ts[0] returning y0 itself."""
    import torch
    lam = torch.tensor([-1.3, 0.4], dtype=torch.float64)
    f = lambda y: lam[:, None, None] * y  # noqa: E731
    ts = np.array([[0.0, 0.013, 0.4, 0.777, 1.0], [0.0, 0.25, 0.5, 1.31, 2.0]])
    y0 = torch.tensor([[[1.0]], [[2.0]]], dtype=torch.float64)
    for method in ("Tsit5", "Dopri5"):
        ys = data.diffeqsolve_constant(f, ts, y0, method, dt0=0.05)
        ref = y0[:, None] * torch.exp(lam[:, None, None, None] * torch.tensor(ts)[:, :, None, None])
        err = float((ys - ref).abs().max() / ref.abs().max())
        assert ys.shape == (2, 5, 1, 1) and torch.equal(ys[:, 0], y0)
        assert err < 1e-7, (method, err)


def test_dynamic_ground_truth_hands_over_between_event_segments():
    """gen_all_data (ode_dataset.py:420-465): each event segment is its own solve started from the previous
    segment's last saved state, so the state at a segment's first time equals the state at the previous segment's
    last time (no evolution across that gap) -- the reference's hand-over, restated."""
    cfg = data.DynDataCfg(name="heat", batch_size=2, num_nodes=9, time_tick=20, dynamic_graph=True,
                          all_dynamic=True, sampling_type="irregular", method="Tsit5", seed=3)
    ds = data.DynDataset(cfg, device="cpu")
    y = ds.true_y.numpy()
    ev = np.sort(ds.events_indices)
    assert len(ev) > 0
    for e in ev:
        assert np.array_equal(y[:, e], y[:, e - 1])
    inside = [j for j in range(1, y.shape[1]) if j not in set(ev)]
    assert any(not np.array_equal(y[:, j], y[:, j - 1]) for j in inside)


def test_community_graph_matches_reference_generator():
    """data.community_graph restates ODEDataset._gen_community_graph (ode_dataset.py:189-202) + the layout
    reordering (data_tools.py:32-72): pinned against tests/golden/community_graphs.npz, which
    tests/golden/make_community.py wrote from networkx directly (the reference's own call sequence)."""
    import networkx as nx
    from gncde import data
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "community_graphs.npz"))
    assert str(z["networkx_version"]) == nx.__version__
    for key in z.files:
        if not key.startswith("A_"):
            continue
        _, n, seed, lay = key.split("_")
        n, seed = int(n[1:]), int(seed[1:])
        want = np.unpackbits(z[key])[:n * n].reshape(n, n).astype(float)
        got = data.community_graph(n, seed, None if lay == "None" else lay)
        assert np.array_equal(got, want), key
        assert np.array_equal(got, got.T) and not np.any(np.diag(got))
