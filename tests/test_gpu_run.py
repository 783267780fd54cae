"""GPU: the single_run-style workflow end to end (SURVEY §8 f2 + f4): dataset generation on the GPU, graph
paths through the engine's input kernels, training steps through the GPU adjoint, PID evaluation, early
stopping bookkeeping and the safetensors checkpoint."""
import os

import pytest
import torch
import yaml

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("spi", [None, 1])
def test_dyn_single_run_small(tmp_path, spi):
    """trainer.py flow on the dyn config: spi None trains on the reference's adaptive Tsit5 + PID solve (reverse mode
    on the accepted steps), spi = 1 on the fixed RK4 grid override."""
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a HIP device")
    from gncde import data, run
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with open(os.path.join(root, "configs", "heat_grid_small.yaml")) as fh:
        cfg = yaml.safe_load(fh)
    cfg["dataset"].update(num_nodes=16, time_tick=16, batch_size=3)
    cfg["checkpoint_dir"] = str(tmp_path)
    ds = data.DynDataset(data.DynDataCfg.from_dict(cfg["dataset"]))
    assert ds.true_y.shape == (3, int(16 * 1.2), 16) and torch.isfinite(ds.true_y).all()
    # heat diffusion conserves nothing special but must decay towards the mean: bounded by the initial max
    assert float(ds.true_y.abs().max()) <= float(ds.x0.abs().max()) * 1.0001
    out = tmp_path / "metrics.jsonl"
    res = run.Trainer(cfg, epochs=12, steps_per_interval=spi, out=str(out)).run()
    assert res["best_epoch"] > 0 and res["best_validation_loss"] == res["best_validation_loss"]
    assert os.path.exists(res["checkpoint"])
    lines = out.read_text().splitlines()
    losses = [yaml.safe_load(l)["train_loss"] for l in lines if "train_loss" in l]
    assert losses[-1] < losses[0]


# config 5's bf16 path: bfloat16 operator coefficients in the persistent adaptive solve (fp32 products), which needs
# its shapes (h = 16 = the hidden width, de = 8); trained through the solve's accepted-step record
BF16S_TGB = {"compute": "bf16_storage", "solver": "pid", "hidden_dim": 16,
             "vector_field": {"name": "PermEquivGraphVectorField", "hidden_dim": 16, "num_layers": 2, "data_embed_dim": 8}}


@pytest.mark.parametrize("config,metric,model", [("pgt_england_small.yaml", "best_validation_loss", None),
                                                 ("tgb_trade_small.yaml", "best_validation_ndcg@10", None),
                                                 ("tgb_trade_small.yaml", "best_validation_ndcg@10", {"solver": "pid"}),
                                                 ("tgb_trade_small.yaml", "best_validation_ndcg@10", BF16S_TGB)])
def test_window_single_run_small(tmp_path, config, metric, model):
    """trainer_pgt / trainer_tgb flow: windows -> one optimiser step per window -> validation (MSE / NDCG@10)
    -> checkpoint -> test metrics of the best model.  solver "pid": the TGB model on BASELINE config 5's adaptive
    Tsit5 + PIDController (build-only `model.solver: pid`), trained through the reverse mode on the accepted steps;
    with `model.compute: bf16_storage`, the adaptive solve reads bfloat16 operator coefficients."""
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a HIP device")
    from gncde import data, run
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with open(os.path.join(root, "configs", config)) as fh:
        cfg = yaml.safe_load(fh)
    cfg["dataset"]["num_snapshots"] = 26 if "pgt" in config else 16
    cfg["checkpoint_dir"] = str(tmp_path)
    cfg["eval_freq"] = 2
    if model:
        cfg["model"].update(model)
    ds = data.WindowDataset(data.WindowDataCfg.from_dict(cfg["dataset"]))
    assert len(ds.train) >= 1 and len(ds.val) >= 1 and len(ds.test) >= 1
    out = tmp_path / "metrics.jsonl"
    res = run.WindowTrainer(cfg, epochs=4, out=str(out)).run()
    assert res[metric] == res[metric] and res["best_epoch"] >= 0
    assert os.path.exists(res["checkpoint"])
    recs = [yaml.safe_load(l) for l in out.read_text().splitlines()]
    assert all(r["train_loss"] == r["train_loss"] for r in recs if "train_loss" in r)
    if "tgb" in config:
        assert 0.0 <= res[metric] <= 1.0
