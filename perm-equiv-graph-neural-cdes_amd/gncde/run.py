"""``single_run``-style entry point for the dynamical-systems workflow (the reference's
``src/run/dyn/single_run.py`` -> ``engine.trainer.Trainer(**yaml).run()``), reading the same YAML schema
(configs/dynamical_systems/*.yaml) and running it on this engine:

    python -m gncde.run --config <reference>/configs/dynamical_systems/perm_equiv_gncde_config.yaml \\
                        [--epochs N] [--steps-per-interval M] [--out metrics.jsonl]

Flow (trainer.py:88-285): build the dataset (gncde.data, f2), the vector field by registry name
(vector_field_configs.py:52) and GraphNeuralCDE (model_configs.py:46-59); full-batch training steps
(make_step, trainer.py:288-327) with clip_by_global_norm(1) + AdamW on the GPU; every ``eval_freq`` epochs the
interpolation / extrapolation MSE with the model's own solve (Tsit5 + PIDController, SaveAt(ts)); early
stopping with ``patience`` / ``min_epochs``; the best model saved under ``checkpoint_dir`` (safetensors).

One deliberate difference: training differentiates a fixed-grid solve (``--steps-per-interval`` RK4 steps
between consecutive training knots, so every knot is a step state) instead of the adaptive Tsit5+PID
solve — the engine's reverse mode covers fixed grids.  Evaluation uses the reference
solve.  wandb is not used; metrics are printed (and appended to ``--out``) as JSON lines with the
reference's names (train_loss, max_grad, max_update, validation_loss, test_loss_extra ...).
"""
from __future__ import annotations

import argparse
import json
import os
import time

import numpy as np
import torch
import yaml

from . import _lib, data, engine, train
from .models import GraphNeuralCDE, vector_fields


def _mse(pred, y, idx):
    if not idx:
        return float("nan")
    sel = torch.as_tensor(idx, device=pred.device)
    return float(((pred[:, sel] - y[:, sel]) ** 2).mean())


class Trainer:
    """Mirror of the reference's dyn Trainer for GraphNeuralCDE models."""

    def __init__(self, cfg: dict, epochs: int | None = None, steps_per_interval: int = 2, out: str | None = None):
        self.cfg = cfg
        self.epochs = int(epochs if epochs is not None else cfg.get("epochs", 100))
        self.patience = int(cfg.get("patience", 10 ** 9))
        self.min_epochs = int(cfg.get("min_epochs", 0))
        self.log_freq = int(cfg.get("log_freq", 25))
        self.eval_freq = int(cfg.get("eval_freq", 25))
        self.seed = int(cfg.get("seed", 1234))
        self.steps_per_interval = steps_per_interval
        self.out = out
        m = cfg.get("model", {})
        if m.get("name", "graph_neural_cde") != "graph_neural_cde":
            raise NotImplementedError(f"model {m.get('name')}: this runner drives graph_neural_cde")
        self.model_cfg = m

    def _log(self, rec: dict):
        line = json.dumps(rec)
        print(line, flush=True)
        if self.out:
            with open(self.out, "a") as fh:
                fh.write(line + "\n")

    def build(self):
        torch.manual_seed(self.seed)
        ds = data.DynDataset(data.DynDataCfg.from_dict(self.cfg.get("dataset", {})))
        m, vfc = self.model_cfg, self.model_cfg.get("vector_field", {})
        h = int(m.get("hidden_dim", 16))
        cls = getattr(vector_fields, vfc.get("name", "PermEquivGraphVectorField"))
        vf = cls(input_dim=h, hidden_dim=int(vfc.get("hidden_dim", h)), output_dim=h,
                 num_layers=int(vfc.get("num_layers", 2)), data_embed_dim=1, num_nodes=ds.n, key=self.seed)
        model = GraphNeuralCDE(m, vf, m.get("interpolation", "cubic"), self.seed,
                               solver={"method": "rk4", "steps_per_interval": self.steps_per_interval})
        return ds, model.to("cuda")

    def run(self) -> dict:
        ds, model = self.build()
        opt_cfg = self.cfg.get("optimiser", {})
        sched = opt_cfg.get("schedule", {"name": "constant_schedule", "value": 1e-3})
        if sched.get("name", "constant_schedule") != "constant_schedule":
            raise NotImplementedError("only constant_schedule is wired (optimiser_configs.py)")
        opt = train.ClipAdamW(model, learning_rate=float(sched.get("value", 1e-3)),
                              weight_decay=float(opt_cfg.get("weight_decay", 0.0)),
                              gradient_clipping=bool(opt_cfg.get("gradient_clipping", True)))
        # training control over the training knots (the reference's train_graph_path_coeffs), validation over all
        ts_tr, coef_tr, tcoef_tr = ds.graph_path(ds.id_train)
        ts_all, coef_all, tcoef_all = ds.graph_path(list(range(ds.t.shape[1])))
        y_tr = ds.true_y[:, torch.as_tensor(ds.id_train, device=ds.true_y.device)]
        prob_tr = model.vector_field.problem_from_layout(ts_tr, coef_tr, tcoef_tr)
        spec_tr = model._spec(ts_tr, evolving_out=True)
        x0 = ds.x0

        def loss_terms():
            pred = model.predict_packed(prob_tr, x0, spec_tr).squeeze(-1)
            return ((pred - y_tr) ** 2).sum(), pred.numel()

        best, best_epoch, corr_test, bad = float("inf"), -1, float("nan"), 0
        ckpt_dir = self.cfg.get("checkpoint_dir", ".checkpoints/")
        ckpt = os.path.join(ckpt_dir, self.cfg.get("checkpoint_name", "gncde") + ".safetensors")
        for epoch in range(self.epochs):
            t0 = time.time()
            loss, mg, mu = train.make_step(opt, loss_terms)
            torch.cuda.synchronize()
            step_time = time.time() - t0
            if epoch % self.log_freq == 0:
                self._log({"epoch": epoch + 1, "train_loss": float(loss), "train_step_time": step_time,
                           "max_grad": float(mg), "max_update": float(mu)})
            if (epoch + 1) % self.eval_freq == 0 or epoch + 1 == self.epochs:
                with torch.no_grad():
                    prob_all = model.vector_field.problem_from_layout(ts_all, coef_all, tcoef_all)
                    pred = model.forward_packed(prob_all, x0, ts_all).squeeze(-1)  # PID, SaveAt(ts)
                val = _mse(pred, ds.true_y, ds.id_test_inter or ds.id_test_extra)
                extra = _mse(pred, ds.true_y, ds.id_test_extra)
                self._log({"epoch": epoch + 1, "validation_loss": val, "test_loss_extra": extra})
                if val < best:
                    best, best_epoch, corr_test, bad = val, epoch + 1, extra, 0
                    os.makedirs(ckpt_dir, exist_ok=True)
                    from safetensors.torch import save_file
                    save_file({k: v.detach().cpu().contiguous() for k, v in model.state_dict().items()}, ckpt)
                else:
                    bad += self.eval_freq
                    if epoch + 1 >= self.min_epochs and bad >= self.patience:
                        break
        res = {"best_validation_loss": best, "corr_test_loss": corr_test, "best_epoch": best_epoch,
               "checkpoint": ckpt}
        self._log(res)
        return res


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--config", required=True)
    ap.add_argument("--epochs", type=int, default=None)
    ap.add_argument("--steps-per-interval", type=int, default=2)
    ap.add_argument("--out", default=None)
    args = ap.parse_args(argv)
    with open(args.config) as fh:
        cfg = yaml.safe_load(fh)
    Trainer(cfg, args.epochs, args.steps_per_interval, args.out).run()


if __name__ == "__main__":
    main()
