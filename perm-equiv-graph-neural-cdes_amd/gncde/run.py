"""``single_run``-style entry points: the reference's ``src/run/{dyn,pgt,tgb}/single_run.py`` ->
``engine.trainer[_pgt|_tgb].Trainer(**yaml).run()``, reading the same YAML schema (configs/dynamical_systems,
configs/pgt, configs/tgb) and running it on this engine.  ``Trainer`` drives graph_neural_cde (dynamical
systems); ``WindowTrainer`` drives pgt_graph_neural_cde / tgb_graph_neural_cde over snapshot windows.

    python -m gncde.run --config <reference>/configs/dynamical_systems/perm_equiv_gncde_config.yaml \\
                        [--epochs N] [--steps-per-interval M] [--out metrics.jsonl]
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 -m gncde.run --config ...

Under torch.distributed.run every rank owns one GPU and a share of the samples (dyn: balanced by the adaptive
solves' step counts; pgt/tgb: the windows of each optimiser step), with one gradient all-reduce per step.

Flow (trainer.py:88-285): build the dataset (gncde.data, f2), the vector field by registry name
(vector_field_configs.py:52) and GraphNeuralCDE (model_configs.py:46-59); full-batch training steps
(make_step, trainer.py:288-327) with clip_by_global_norm(1) + AdamW on the GPU; every ``eval_freq`` epochs the
interpolation / extrapolation MSE with the model's own solve (Tsit5 + PIDController, SaveAt(ts)); early
stopping with ``patience`` / ``min_epochs``; the best model saved under ``checkpoint_dir`` (safetensors).

Training differentiates the reference's own solve (Tsit5 + PIDController, SaveAt(ts)) on each sample's
accepted step sequence (autograd.solve).  ``--steps-per-interval M`` optionally replaces it with
a fixed RK4 grid of M steps between consecutive knots (a build extension).  wandb is not used; metrics are printed (and appended to ``--out``) as JSON lines with the
reference's names (train_loss, max_grad, max_update, validation_loss, test_loss_extra ...).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import time

import numpy as np
import torch
import yaml

from . import _lib, data, engine, metrics, train
from .models import GraphNeuralCDE, vector_fields


def _mse(pred, y, idx):
    if not idx:
        return float("nan")
    sel = torch.as_tensor(idx, device=pred.device)
    return float(((pred[:, sel] - y[:, sel]) ** 2).mean())


def _optimiser(cfg: dict) -> dict:
    """The ``optimiser:`` block (optimiser_configs.py:53-88) as numbers.  The reference YAMLs write ``1e-4`` and
    ``10e-2``, which YAML 1.1 (yaml.safe_load) reads as strings; optax receives them through pydantic's float
    coercion, so they are floats here too."""
    opt_cfg = cfg.get("optimiser", {})
    sched = opt_cfg.get("schedule", {"name": "constant_schedule", "value": 1e-3})
    if sched.get("name", "constant_schedule") != "constant_schedule":
        raise NotImplementedError("only constant_schedule is wired (optimiser_configs.py)")
    return {"learning_rate": float(sched.get("value", 1e-3)), "weight_decay": float(opt_cfg.get("weight_decay", 0.0)),
            "gradient_clipping": bool(opt_cfg.get("gradient_clipping", True))}


class Trainer:
    """Mirror of the reference's dyn Trainer for GraphNeuralCDE models."""

    def __init__(self, cfg: dict, epochs: int | None = None, steps_per_interval: int | None = None,
                 out: str | None = None):
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
        if train.dist_world()[0] != 0:  # rank 0 speaks for the job
            return
        line = json.dumps(rec)
        print(line, flush=True)
        if self.out:
            with open(self.out, "a") as fh:
                fh.write(line + "\n")

    def describe(self) -> dict:
        """What ``run`` would build from this config, derived from the YAML alone (no GPU, no data): nodes n
        (grid: ceil(sqrt(num_nodes))^2, ode_dataset.py:56), hidden width h, layers L, data_embed_dim, the
        optimiser numbers and the solve (graph_neural_cde.py:53-54,86,94-104)."""
        m, vfc = self.model_cfg, self.model_cfg.get("vector_field", {})
        dc = data.DynDataCfg.from_dict(self.cfg.get("dataset", {}))
        n = int(math.ceil(math.sqrt(dc.num_nodes))) ** 2 if dc.graph_type == "grid" else int(dc.num_nodes)
        h = int(m.get("hidden_dim", 16))
        solve = ({"method": "tsit5", "controller": "pid", "rtol": 1e-3, "atol": 1e-6, "dt0": None}
                 if self.steps_per_interval is None else
                 {"method": "rk4", "controller": "grid", "steps_per_interval": self.steps_per_interval})
        return {"model": "graph_neural_cde", "vector_field": vfc.get("name", "PermEquivGraphVectorField"), "n": n,
                "h": h, "L": int(vfc.get("num_layers", 2)), "data_embed_dim": 1, "batch": int(dc.batch_size),
                **_optimiser(self.cfg), "solve": solve}

    def build(self):
        torch.manual_seed(self.seed)
        ds = data.DynDataset(data.DynDataCfg.from_dict(self.cfg.get("dataset", {})))
        m, vfc = self.model_cfg, self.model_cfg.get("vector_field", {})
        h = int(m.get("hidden_dim", 16))
        cls = getattr(vector_fields, vfc.get("name", "PermEquivGraphVectorField"))
        vf = cls(input_dim=h, hidden_dim=int(vfc.get("hidden_dim", h)), output_dim=h,
                 num_layers=int(vfc.get("num_layers", 2)), data_embed_dim=1, num_nodes=ds.n, key=self.seed)
        model = GraphNeuralCDE(m, vf, m.get("interpolation", "cubic"), self.seed,
                               solver=None if self.steps_per_interval is None else
                               {"method": "rk4", "steps_per_interval": self.steps_per_interval})
        return ds, model.to("cuda")

    def run(self) -> dict:
        ds, model = self.build()
        rank, world = train.dist_world()
        opt = train.ClipAdamW(model, **_optimiser(self.cfg))
        # training control over the training knots (the reference's train_graph_path_coeffs), validation over all
        ts_tr, coef_tr, tcoef_tr = ds.graph_path(ds.id_train)
        ts_all, coef_all, tcoef_all = ds.graph_path(list(range(ds.t.shape[1])))
        y_tr_all = ds.true_y[:, torch.as_tensor(ds.id_train, device=ds.true_y.device)]
        prob_tr_all = model.vector_field.problem_from_layout(ts_tr, coef_tr, tcoef_tr)
        prob_all_full = model.vector_field.problem_from_layout(ts_all, coef_all, tcoef_all)
        B = prob_tr_all.B
        adaptive = model.solver is None  # the reference's Tsit5 + PID solve: per-sample step counts differ

        # Data parallelism: each rank owns a set of samples; the step all-reduces the gradient of the
        # summed loss once (train.make_step), so the update equals the reference's full-batch step
        # (trainer.py:288-327, loss_configs.py:44-47).  Adaptive solves rebalance the sets by the previous epoch's
        # accepted step counts (balanced_partition) when the ranks' work differs by more than 10 %.
        def shard(own):
            st = dict(own=list(own))
            if not own:  # more ranks than samples: this rank contributes a zero gradient and zero sums
                return st
            st["prob"] = prob_tr_all.take(own) if world > 1 else prob_tr_all
            st["x0"] = ds.x0[torch.as_tensor(own, device=ds.x0.device)] if world > 1 else ds.x0
            st["y"] = y_tr_all[torch.as_tensor(own, device=y_tr_all.device)] if world > 1 else y_tr_all
            st["spec"] = model._spec(st["prob"].ts, evolving_out=True)
            if adaptive:
                st["spec"].stats_out = torch.zeros(len(own), 4, dtype=torch.int32, device=ds.x0.device)
            return st

        parts = [list(range(*train.shard_range(B, r, world))) for r in range(world)]  # every rank's samples
        sh = shard(parts[rank])

        def loss_terms():
            if not sh["own"]:
                return sum(p.sum() * 0.0 for p in model.parameters()), 0
            pred = model.predict_packed(sh["prob"], sh["x0"], sh["spec"]).squeeze(-1)
            return ((pred - sh["y"]) ** 2).sum(), pred.numel()

        def validate():
            """interpolation / extrapolation MSE over all samples (each rank its own, summed over ranks)."""
            own = sh["own"]
            if not own:
                v_s, v_c, e_s, e_c = train.all_reduce_sum([0.0, 0.0, 0.0, 0.0], ds.x0.device)
                return (v_s / v_c if v_c else float("nan")), (e_s / e_c if e_c else float("nan"))
            with torch.no_grad():
                pa = prob_all_full.take(own) if world > 1 else prob_all_full
                pred = model.forward_packed(pa, sh["x0"], pa.ts).squeeze(-1)  # PID, SaveAt(ts)
            yt = ds.true_y[torch.as_tensor(own, device=ds.true_y.device)] if world > 1 else ds.true_y
            sums = []
            for ids in (ds.id_test_inter or ds.id_test_extra, ds.id_test_extra):
                if ids:
                    sel = torch.as_tensor(ids, device=pred.device)
                    sums += [float(((pred[:, sel] - yt[:, sel]) ** 2).sum()), pred[:, sel].numel()]
                else:
                    sums += [0.0, 0.0]
            v_s, v_c, e_s, e_c = train.all_reduce_sum(sums, pred.device)
            return (v_s / v_c if v_c else float("nan")), (e_s / e_c if e_c else float("nan"))

        best, best_epoch, corr_test, bad = float("inf"), -1, float("nan"), 0
        ckpt_dir = self.cfg.get("checkpoint_dir", ".checkpoints/")
        ckpt = os.path.join(ckpt_dir, self.cfg.get("checkpoint_name", "gncde") + ".safetensors")
        for epoch in range(self.epochs):
            t0 = time.time()
            loss, mg, mu = train.make_step(opt, loss_terms)
            torch.cuda.synchronize()
            step_time = time.time() - t0
            if adaptive and world > 1:
                steps = sh["spec"].stats_out[:, _lib.STAT_STEPS].tolist() if sh["own"] else []
                costs = train.global_costs(sh["own"], steps, B, ds.x0.device)
                loads = [sum(costs[i] for i in p) for p in parts]
                if max(loads) > 1.1 * max(min(loads), 1.0):
                    parts = train.balanced_partition(costs, world)
                    sh = shard(parts[rank])
            if epoch % self.log_freq == 0:
                self._log({"epoch": epoch + 1, "train_loss": float(loss), "train_step_time": step_time,
                           "max_grad": float(mg), "max_update": float(mu)})
            if (epoch + 1) % self.eval_freq == 0 or epoch + 1 == self.epochs:
                val, extra = validate()
                self._log({"epoch": epoch + 1, "validation_loss": val, "test_loss_extra": extra})
                if val < best:
                    best, best_epoch, corr_test, bad = val, epoch + 1, extra, 0
                    if rank == 0:
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

class WindowTrainer:
    """Mirror of trainer_pgt.Trainer (trainer_pgt.py:140-316) and trainer_tgb.Trainer (trainer_tgb.py:150-307)
    for PGTGraphNeuralCDE / TGBGraphNeuralCDE over snapshot windows (gncde.data.WindowDataset).

    As in the reference, every training window is one optimiser step (SlidingWindowTemporalLoader, batch_size
    1); ``window_batch`` > 1 batches that many windows per step instead (one launch per step, gradients of the
    summed per-window losses).  PGT: MSE of the global read-out against the window's node labels, best model by
    validation loss.  TGB: masked cross-entropy, NDCG@10 on the masked rows (gncde.metrics), best model by
    validation NDCG@10.  The solve is the reference's fixed-step Tsit5 (dt0 0.1 / 0.01) in both directions."""

    def __init__(self, cfg: dict, epochs: int | None = None, out: str | None = None, window_batch: int = 1):
        self.cfg = cfg
        self.epochs = int(epochs if epochs is not None else cfg.get("epochs", 2000))
        self.patience = int(cfg.get("patience", -1))
        self.min_epochs = int(cfg.get("min_epochs", 100))
        self.log_freq = int(cfg.get("log_freq", 10))
        self.eval_freq = int(cfg.get("eval_freq", 10))
        self.seed = int(cfg.get("seed", 1234))
        self.out = out
        self.window_batch = max(1, int(window_batch))
        self.model_cfg = cfg.get("model", {})
        name = self.model_cfg.get("name")
        if name not in ("pgt_graph_neural_cde", "tgb_graph_neural_cde"):
            raise NotImplementedError(f"model {name}: this runner drives pgt/tgb_graph_neural_cde")
        self.tgb = name == "tgb_graph_neural_cde"

    _log = Trainer._log

    def describe(self) -> dict:
        """As Trainer.describe for the PGT / TGB drivers (pgt_graph_neural_cde.py:119-129: ConstantStepSize 0.1;
        tgb_graph_neural_cde.py:152-162: 0.01, or the build-only ``solver: pid``)."""
        from .models import PGTGraphNeuralCDE, TGBGraphNeuralCDE
        import inspect
        m, vfc = self.model_cfg, self.model_cfg.get("vector_field", {})
        dc = data.WindowDataCfg.from_dict(self.cfg.get("dataset", {}))
        n = data.window_nodes(dc.name)
        if "num_nodes" in vfc and int(vfc["num_nodes"]) != n:
            raise ValueError(f"vector_field.num_nodes {vfc['num_nodes']} != the {dc.name} graph's {n} nodes")
        h = int(m.get("hidden_dim", 32))
        cls = TGBGraphNeuralCDE if self.tgb else PGTGraphNeuralCDE
        dt0 = inspect.signature(cls.__init__).parameters["dt0"].default
        solve = {"method": "tsit5", "controller": "constant", "dt0": dt0}
        if self.tgb and m.get("solver") == "pid":
            solve = {"method": "tsit5", "controller": "pid", "rtol": 1e-3, "atol": 1e-6, "dt0": None}
        return {"model": self.model_cfg.get("name"), "vector_field": vfc.get("name", "PermEquivGraphVectorField"),
                "n": n, "h": h, "L": int(vfc.get("num_layers", 2)), "data_embed_dim": int(vfc.get("data_embed_dim", 8)),
                "window_size": int(dc.window_size), "windows_per_step": self.window_batch, **_optimiser(self.cfg),
                "solve": solve, "compute": m.get("compute", "fp32")}

    def build(self):
        from .models import PGTGraphNeuralCDE, TGBGraphNeuralCDE
        torch.manual_seed(self.seed)
        np.random.seed(self.seed)
        ds = data.WindowDataset(data.WindowDataCfg.from_dict(self.cfg.get("dataset", {})))
        m, vfc = self.model_cfg, self.model_cfg.get("vector_field", {})
        h = int(m.get("hidden_dim", 32))
        de = int(vfc.get("data_embed_dim", 8))
        cls = getattr(vector_fields, vfc.get("name", "PermEquivGraphVectorField"))
        vf = cls(input_dim=h, hidden_dim=int(vfc.get("hidden_dim", h)), output_dim=h * de * 2,
                 num_layers=int(vfc.get("num_layers", 2)), data_embed_dim=de, num_nodes=ds.n, key=self.seed)
        if self.tgb:
            # build-only model key `solver: pid` (BASELINE config 5's adaptive Tsit5); absent: the reference's
            # ConstantStepSize(0.01)
            # build-only key `compute` ("fp32" | "bf16" | "bf16_storage"): the solve's arithmetic
            model = TGBGraphNeuralCDE({k: v for k, v in m.items() if k not in ("solver", "compute")}, vf,
                                      m.get("interpolation", "cubic"), self.seed, solver=m.get("solver"),
                                      compute=m.get("compute", "fp32"))
        else:
            model = PGTGraphNeuralCDE(m, vf, m.get("interpolation", "cubic"), self.seed)
        return ds, model.to("cuda")

    def _chunks(self, starts, size):
        return [starts[i:i + size] for i in range(0, len(starts), size)]

    def _evaluate(self, model, ds, starts):
        """(mean loss, mean NDCG@10 or nan) over windows, one window at a time like the reference loader; with
        data parallelism each rank evaluates every world-th window and the sums are all-reduced."""
        if len(starts) == 0:
            return float("nan"), float("nan")
        rank, world = train.dist_world()
        loss, ndcg = 0.0, 0.0
        with torch.no_grad():
            for s in list(starts)[rank::world]:
                b = ds.batch([s])
                if self.tgb:
                    ce, cnt = model.loss_terms(*b)
                    loss += float(ce) / max(float(cnt), 1.0)
                    pred = model.batched(*b[:4])[0]
                    mask = b[5][0]
                    ndcg += metrics.ndcg_at_k(b[4][0][mask], pred[mask], k=10)
                else:
                    sse, cnt = model.loss_terms(*b)
                    loss += float(sse) / cnt
        loss, ndcg = train.all_reduce_sum([loss, ndcg], "cuda")
        return loss / len(starts), (ndcg / len(starts) if self.tgb else float("nan"))

    def run(self) -> dict:
        from safetensors.torch import save_file
        ds, model = self.build()
        opt = train.ClipAdamW(model, **_optimiser(self.cfg))
        # Data parallelism: each optimiser step takes `window_batch` windows (at least one per rank),
        # split over the ranks (balanced_partition by the windows' costs: the adaptive TGB solve's accepted step
        # counts from the previous epoch, else equal), with one gradient all-reduce per step (train.make_step
        # normalises by the global element count).
        rank, world = train.dist_world()
        # the global window batch stays --window-batch (the same training as one GPU): with fewer windows per step
        # than ranks the surplus ranks contribute zero gradients every step
        wb = self.window_batch
        if wb < world and rank == 0:
            import warnings
            warnings.warn(f"--window-batch {wb} < world size {world}: {world - wb} of {world} ranks idle every "
                          "optimiser step (pass --window-batch >= world to use them)", stacklevel=2)
        chunks = self._chunks(list(ds.train), wb)
        cost = {w: 1.0 for w in ds.train}

        def rank_batches():
            out = []
            for c in chunks:
                part = train.balanced_partition([cost[w] for w in c], world)[rank]
                out.append(([c[i] for i in part], ds.batch([c[i] for i in part]) if part else None))
            return out

        batches = rank_batches()
        best_val = -float("inf") if self.tgb else float("inf")
        best_epoch, test_loss, test_ndcg, bad = -1, float("nan"), float("nan"), 0
        ckpt_dir = self.cfg.get("checkpoint_dir", ".checkpoints/")
        ckpt = os.path.join(ckpt_dir, self.cfg.get("checkpoint_name", "gncde") + ".safetensors")
        for epoch in range(self.epochs):
            t0 = time.time()
            tot, mg, mu = 0.0, 0.0, 0.0
            steps_seen = {}
            for wins, b in batches:
                if b is None:  # more ranks than windows in this step: contribute a zero gradient
                    loss, g, u = train.make_step(opt, lambda: (sum(p.sum() * 0.0 for p in model.parameters()), 0))
                else:
                    loss, g, u = train.make_step(opt, model.loss_terms, *b)
                    if getattr(model, "last_steps", None) is not None:
                        steps_seen.update(zip(wins, model.last_steps.tolist()))
                tot += float(loss)
                mg, mu = max(mg, float(g)), max(mu, float(u))
            torch.cuda.synchronize()
            if world > 1 and getattr(model, "adaptive", False):
                pos = {w: i for i, w in enumerate(ds.train)}
                costs = train.global_costs([pos[w] for w in steps_seen], list(steps_seen.values()), len(ds.train),
                                           "cuda")
                new = {w: max(c, 1.0) for w, c in zip(ds.train, costs)}
                if new != cost:
                    cost = new
                    batches = rank_batches()
            rec = {"epoch": epoch + 1, "train_loss": tot / max(len(batches), 1), "train_step_time": time.time() - t0,
                   "max_grad": mg, "max_update": mu}
            if epoch == 0 or (epoch + 1) % self.log_freq == 0:
                self._log(rec)
            if (epoch + 1) % self.eval_freq == 0:
                t0 = time.time()
                vl, vn = self._evaluate(model, ds, ds.val)
                rec = {"epoch": epoch + 1, "validation_loss": vl, "validation_step_time": time.time() - t0}
                if self.tgb:
                    rec["validation_ndcg@10"] = vn
                self._log(rec)
                better = vn > best_val if self.tgb else vl < best_val
                if better:
                    best_val, best_epoch, bad = (vn if self.tgb else vl), epoch, 0
                    os.makedirs(ckpt_dir, exist_ok=True)
                    save_file({k: v.detach().cpu().contiguous() for k, v in model.state_dict().items()}, ckpt)
                    test_loss, test_ndcg = self._evaluate(model, ds, ds.test)
                else:
                    bad += 1
                    if self.patience > 0 and bad * self.eval_freq >= self.patience and epoch > self.min_epochs:
                        break
        key = "best_validation_ndcg@10" if self.tgb else "best_validation_loss"
        res = {key: best_val, "corr_test_loss": test_loss, "best_epoch": best_epoch, "checkpoint": ckpt,
               "windows_per_step": wb}
        if self.tgb:
            res["corr_test_ndcg"] = test_ndcg
        self._log(res)
        return res


def init_distributed():
    """One process per GPU under torch.distributed.run (WORLD_SIZE > 1): bind LOCAL_RANK's GPU and join the
    process group (RCCL; GNCDE_DIST_BACKEND=gloo for CPU-transport tests).  The trainers then shard their samples /
    windows and all-reduce one gradient bucket per step."""
    import torch.distributed as dist
    if int(os.environ.get("WORLD_SIZE", "1")) <= 1 or dist.is_initialized():
        return
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    backend = os.environ.get("GNCDE_DIST_BACKEND", "nccl")
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        dist.init_process_group(backend)


def single_run(default_config: str, argv=None):
    """The body of the ``src/run/{dyn,pgt,tgb}/single_run.py`` shims: the reference's hard-coded YAML path (relative
    to the working directory, as in the reference, e.g. src/run/dyn/single_run.py:23-24) unless ``--config`` is
    given; every other flag of ``main`` passes through."""
    import sys
    argv = list(sys.argv[1:] if argv is None else argv)
    if not any(a == "--config" or a.startswith("--config=") for a in argv):
        if not os.path.exists(default_config):
            raise SystemExit(f"{default_config} not found (run from the directory holding configs/, as the "
                             "reference's single_run.py expects, or pass --config <yaml>)")
        argv = ["--config", default_config] + argv
    return main(argv)


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--config", required=True)
    ap.add_argument("--epochs", type=int, default=None)
    ap.add_argument("--steps-per-interval", type=int, default=None,
                    help="dyn models: train on a fixed RK4 grid of M steps between knots instead of the reference's "
                         "adaptive Tsit5 + PID solve")
    ap.add_argument("--window-batch", type=int, default=1, help="pgt/tgb models: windows per optimiser step")
    ap.add_argument("--out", default=None)
    args = ap.parse_args(argv)
    init_distributed()
    with open(args.config) as fh:
        cfg = yaml.safe_load(fh)
    name = cfg.get("model", {}).get("name", "graph_neural_cde")
    if name in ("pgt_graph_neural_cde", "tgb_graph_neural_cde"):
        WindowTrainer(cfg, args.epochs, args.out, args.window_batch).run()
    else:
        Trainer(cfg, args.epochs, args.steps_per_interval, args.out).run()


if __name__ == "__main__":
    main()
