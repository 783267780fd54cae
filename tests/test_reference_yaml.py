"""The reference's own perm_equiv_gncde_config.yaml files drive this engine's trainers unchanged (CPU, no GPU).

``north_star`` keeps the reference's ``configs/`` YAML and ``src/run/*/single_run.py`` entry points.  These tests
read the three perm-equiv configs from /root/reference (skipped where it is absent, e.g. on the GPU box) with
yaml.safe_load exactly as the reference's single_run.py does, construct the trainer the shim would run, and check
what it derives: nodes, widths, layers, data embedding, optimiser numbers (the YAMLs' ``1e-4`` / ``10e-2`` are
YAML-1.1 strings) and the solve.  The shims' default paths are the reference's (src/run/*/single_run.py:23-29).
"""
import importlib.util
import os

import pytest
import yaml

from gncde import run

REF = "/root/reference"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CASES = {
    "dyn": ("configs/dynamical_systems/perm_equiv_gncde_config.yaml",
            dict(model="graph_neural_cde", n=400, h=16, L=2, data_embed_dim=1, learning_rate=0.1, weight_decay=1e-4,
                 batch=4, solve={"method": "tsit5", "controller": "pid", "rtol": 1e-3, "atol": 1e-6, "dt0": None})),
    "pgt": ("configs/pgt/england/perm_equiv_gncde_config.yaml",
            dict(model="pgt_graph_neural_cde", n=129, h=64, L=3, data_embed_dim=8, learning_rate=1e-2,
                 weight_decay=1e-4, window_size=5, solve={"method": "tsit5", "controller": "constant", "dt0": 0.1})),
    "tgb": ("configs/tgb/trade/perm_equiv_gncde_config.yaml",
            dict(model="tgb_graph_neural_cde", n=255, h=32, L=4, data_embed_dim=8, learning_rate=1e-2,
                 weight_decay=1e-4, window_size=3, solve={"method": "tsit5", "controller": "constant", "dt0": 0.01})),
}


def _shim(kind):
    spec = importlib.util.spec_from_file_location(f"single_run_{kind}", os.path.join(ROOT, "src", "run", kind,
                                                                                    "single_run.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)  # (the shim runs only under __main__)
    return mod


@pytest.mark.parametrize("kind", sorted(CASES))
def test_shim_defaults_to_the_reference_path(kind):
    assert _shim(kind).CONFIG == CASES[kind][0]


@pytest.mark.parametrize("kind", sorted(CASES))
def test_reference_yaml_drives_the_trainer(kind):
    path = os.path.join(REF, CASES[kind][0])
    if not os.path.exists(path):
        pytest.skip("the reference checkout is not present (it never travels to the GPU box)")
    with open(path) as fh:
        cfg = yaml.safe_load(fh)
    # what the reference hands its trainers: optimiser numbers as YAML-1.1 strings
    assert isinstance(cfg["optimiser"]["weight_decay"], str)
    trainer = run.Trainer(cfg) if kind == "dyn" else run.WindowTrainer(cfg)
    got = trainer.describe()
    want = CASES[kind][1]
    for k, v in want.items():
        assert got[k] == pytest.approx(v) if isinstance(v, float) else got[k] == v, (k, got[k], v)


def test_single_run_refuses_a_missing_default(tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    with pytest.raises(SystemExit, match="not found"):
        run.single_run(CASES["dyn"][0], [])
