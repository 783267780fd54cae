"""CPU: the dataset restatement's host logic — config parsing, event indices, split,
padding by events — against the reference rules (ode_dataset.py, data_tools.py, dataset_configs.py)."""
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
