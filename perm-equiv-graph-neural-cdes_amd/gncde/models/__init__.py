"""Solve drivers mirroring ``src/models/{graph,pgt,tgb}_graph_neural_cde.py``.

Same constructor arguments ``(cfg, vector_field, interpolation, model_key)`` and single-sample
``__call__`` signatures as the reference; every call is a batch-of-one instance of ``batched(...)``,
which replaces ``jax.vmap(model)`` (``loss_configs.py:44``) with one ``gncde_integrate`` launch over
the whole batch.  Encoders / read-outs run on ``gncde_node_affine`` (+ ReLU for the MLPs).
"""
from __future__ import annotations

from types import SimpleNamespace

import numpy as np
import torch
from torch import nn

from .. import _lib, autograd, engine, layout
from ..interpolation import CubicInterpolation
from . import vector_fields
from .vector_fields.layers import _gen

__all__ = ["GraphNeuralCDE", "PGTGraphNeuralCDE", "TGBGraphNeuralCDE", "MLP", "vector_fields"]


def _linear(din, dout, g):
    lin = nn.Linear(din, dout)
    lim = 1.0 / din ** 0.5
    with torch.no_grad():
        lin.weight.copy_((2 * torch.rand(dout, din, generator=g) - 1) * lim)
        lin.bias.copy_((2 * torch.rand(dout, generator=g) - 1) * lim)
    return lin


def _affine(lin: nn.Linear, x: torch.Tensor) -> torch.Tensor:
    """Per-node Linear on gncde_node_affine; differentiable (gncde_node_affine_grad) when grad is enabled."""
    return autograd.node_affine(x, lin.weight, lin.bias)


class MLP(nn.Module):
    """``eqx.nn.MLP(in, out, width_size, depth)``: Linear -> ReLU -> ... -> Linear."""

    def __init__(self, in_size, out_size, width_size=16, depth=2, key=None):
        super().__init__()
        g = _gen(key)
        dims = [in_size] + [width_size] * depth + [out_size]
        self.layers = nn.ModuleList(_linear(dims[i], dims[i + 1], g) for i in range(len(dims) - 1))

    def run(self, x):
        for i, lin in enumerate(self.layers):
            x = _affine(lin, x)
            if i < len(self.layers) - 1:
                x = torch.relu(x)
        return x


def _cfg(cfg, **defaults):
    if cfg is None:
        return SimpleNamespace(**defaults)
    if isinstance(cfg, dict):
        d = dict(defaults)
        d.update(cfg)
        return SimpleNamespace(**d)
    return cfg


def _as_batched_coeffs(coeffs, batched):
    return coeffs if batched else tuple(torch.as_tensor(np.asarray(c) if not torch.is_tensor(c) else c)
                                        .unsqueeze(0) for c in coeffs)


def _control(ts, coeffs):
    """A reference-layout (d, c, b, a) tuple, or a control already packed (CubicInterpolation.from_layout)."""
    return coeffs if isinstance(coeffs, CubicInterpolation) else CubicInterpolation(ts, coeffs)


class GraphNeuralCDE(nn.Module):
    """``graph_neural_cde.py:12-113``: Linear(1->h) encoder, Tsit5 + PIDController(1e-3, 1e-6),
    dt0=None, SaveAt(ts) (evolving_out) or SaveAt(t1), Linear(h->1) read-out per node.

    ``solver`` (build extension, BASELINE configs 2/4) may override the reference solve with a fixed grid:
    {"method": "rk4"|"tsit5", "steps": N} — N equal steps on [ts[0], ts[-1]] (saves t1 only), or
    {"method": ..., "steps_per_interval": m} — m steps between consecutive knots, so the step states at the
    knots are the SaveAt(ts) outputs (evolving_out, differentiable: ``loss_terms``).
    """

    def __init__(self, cfg, vector_field, interpolation="cubic", model_key=None, solver=None, **kwargs):
        super().__init__()
        self.cfg = _cfg(cfg, hidden_dim=16, method="Tsit5", return_sequence=True)
        if interpolation != "cubic":
            raise NotImplementedError("only cubic (backward-Hermite) controls are on the hot path")
        if getattr(self.cfg, "method", "Tsit5") != "Tsit5":
            raise NotImplementedError(f"method {self.cfg.method}: only Tsit5 (explicit) is implemented")
        self.vector_field = vector_field
        self.interpolation = interpolation
        g = _gen(model_key)
        self.initial_linear = _linear(1, self.cfg.hidden_dim, g)
        self.final_linear = _linear(self.cfg.hidden_dim, 1, g)
        self.rtol, self.atol = 1e-3, 1e-6
        self.solver = solver

    def _spec(self, ts: torch.Tensor, evolving_out: bool) -> engine.SolverSpec:
        if self.solver is None:
            return engine.SolverSpec(method=_lib.TSIT5, controller=_lib.CTRL_PID,
                                     save_mode=_lib.SAVE_TS if evolving_out else _lib.SAVE_T1,
                                     rtol=self.rtol, atol=self.atol, t0=ts[:, 0].contiguous(),
                                     t1=ts[:, -1].contiguous(), save_ts=ts.contiguous() if evolving_out else None)
        method = _lib.RK4 if self.solver.get("method", "rk4") == "rk4" else _lib.TSIT5
        tsn = ts.cpu().numpy()
        if "steps_per_interval" in self.solver:
            grids = [layout.knot_grid(t, int(self.solver["steps_per_interval"])) for t in tsn]
            save = _lib.SAVE_STEPS if evolving_out else _lib.SAVE_T1
        else:
            if evolving_out:
                raise NotImplementedError("a uniform fixed grid saves at t1 only: use steps_per_interval")
            grids = [layout.rk4_grid(t[0], t[-1], int(self.solver["steps"])) for t in tsn]
            save = _lib.SAVE_T1
        grid, ns = layout.stack_grids(grids, device=ts.device)
        return engine.SolverSpec(method=method, controller=_lib.CTRL_GRID, save_mode=save, grid=grid, nsteps=ns)

    def _knot_states(self, ys: torch.Tensor, T: int) -> torch.Tensor:
        m = int(self.solver["steps_per_interval"])
        return ys[:, torch.arange(T, device=ys.device) * m]

    def batched(self, ts, coeffs_adj, x0, evolving_out=True, return_stats=False):
        """ts [B, T], coeffs_adj (d, c, b, a) each [B, T-1, n, n, 2], x0 [B, n, 1] -> [B, T, n, 1]
        (evolving_out & return_sequence) or [B, n, 1]."""
        control = CubicInterpolation(ts, coeffs_adj)
        ts_d = control.graph_layout()[0]
        x0 = torch.as_tensor(x0, dtype=torch.float32, device=ts_d.device)
        with torch.no_grad():
            y0 = _affine(self.initial_linear, x0)
            prob = self.vector_field.problem(control)
            spec = self._spec(ts_d, evolving_out)
            ys, st = engine.integrate(prob, spec, y0, stats=True)
            if torch.any(st[:, _lib.STAT_STATUS] != 0):
                raise RuntimeError("diffrax-equivalent failure: max_steps reached or non-finite state")
            if spec.controller == _lib.CTRL_GRID and spec.save_mode == _lib.SAVE_STEPS:
                ys = self._knot_states(ys, ts_d.shape[1])
            out = _affine(self.final_linear, ys)
        return (out, st) if return_stats else out

    def predict(self, ts, coeffs_adj, x0, evolving_out=True):
        """Differentiable batched forward: the prediction of ``batched`` with an autograd graph through the
        read-out, the GPU solve and the encoder.  The reference solve (Tsit5 + PIDController, SaveAt(ts)) is
        differentiated on its accepted step sequence (autograd.solve); a fixed-grid ``solver`` override by its
        discrete adjoint."""
        control = CubicInterpolation(ts, coeffs_adj)
        ts_d = control.graph_layout()[0]
        x0 = torch.as_tensor(x0, dtype=torch.float32, device=ts_d.device)
        return self.predict_packed(self.vector_field.problem(control), x0, self._spec(ts_d, evolving_out))

    def forward_packed(self, prob: engine.Problem, x0: torch.Tensor, ts: torch.Tensor,
                       evolving_out: bool = True) -> torch.Tensor:
        """The reference solve (Tsit5 + PIDController(1e-3, 1e-6), dt0=None, SaveAt(ts) or t1) on an already
        packed Problem: encoder -> gncde_integrate -> read-out.  No autograd graph."""
        with torch.no_grad():
            y0 = _affine(self.initial_linear, x0)
            ts = ts.to(y0.device, torch.float32)
            spec = engine.SolverSpec(method=_lib.TSIT5, controller=_lib.CTRL_PID,
                                     save_mode=_lib.SAVE_TS if evolving_out else _lib.SAVE_T1,
                                     rtol=self.rtol, atol=self.atol, t0=ts[:, 0].contiguous(),
                                     t1=ts[:, -1].contiguous(), save_ts=ts.contiguous() if evolving_out else None)
            ys, st = engine.integrate(prob, spec, y0, stats=True)
            if torch.any(st[:, _lib.STAT_STATUS] != 0):
                raise RuntimeError("diffrax-equivalent failure: max_steps reached or non-finite state")
            return _affine(self.final_linear, ys)

    def predict_packed(self, prob: engine.Problem, x0: torch.Tensor, spec: engine.SolverSpec) -> torch.Tensor:
        """``predict`` on an already packed device Problem (coefficients resident in HBM): encoder ->
        differentiable GPU solve (this module's parameters) -> read-out."""
        y0 = _affine(self.initial_linear, x0)
        params, fusion = self.vector_field.diff_tensors(prob.n, x0.device)
        ys = autograd.solve(prob, spec, y0, params, fusion)
        if spec.controller == _lib.CTRL_GRID and spec.save_mode == _lib.SAVE_STEPS:
            ys = self._knot_states(ys, prob.T)
        return _affine(self.final_linear, ys)

    def loss_terms(self, ts, coeffs_adj, x0, labels, evolving_out=True):
        """(sum of squared errors, element count) of ``MSECfg.mse_loss`` (loss_configs.py:22-47:
        mean((squeeze(pred, -1) - label)^2)) on this shard — summed, so data-parallel ranks can all-reduce
        before dividing by the global count."""
        pred = self.predict(ts, coeffs_adj, x0, evolving_out).squeeze(-1)
        labels = torch.as_tensor(labels, dtype=torch.float32, device=pred.device)
        if labels.shape != pred.shape:
            raise ValueError(f"labels {tuple(labels.shape)} != predictions {tuple(pred.shape)}")
        return ((pred - labels) ** 2).sum(), pred.numel()

    def __call__(self, ts, coeffs_adj, x0, evolving_out=True):
        ts = torch.as_tensor(np.asarray(ts) if not torch.is_tensor(ts) else ts, dtype=torch.float32)
        out = self.batched(ts.unsqueeze(0), _as_batched_coeffs(coeffs_adj, False),
                           torch.as_tensor(x0).unsqueeze(0), evolving_out)
        return out[0]


class PGTGraphNeuralCDE(nn.Module):
    """``pgt_graph_neural_cde.py:13-136``: MLP encoder (data_dim -> h), CDEWrapper(vf) against the
    node-data spline, Tsit5 + ConstantStepSize(dt0 = 0.1), SaveAt(t1), MLP decoder, global sum read-out."""

    def __init__(self, cfg, vector_field, interpolation="cubic", model_key=None, dt0=0.1, **kwargs):
        super().__init__()
        self.cfg = _cfg(cfg, hidden_dim=64, data_dim=8, feature_dim=1, method="Tsit5")
        self.vector_field = vector_field
        self.interpolation = interpolation
        g = _gen(model_key)
        enc_state = g.get_state()
        self.encoder = MLP(self.cfg.data_dim, self.cfg.hidden_dim, 16, 2, key=g)
        g.set_state(enc_state)  # pgt_graph_neural_cde.py:62: the decoder is built with encoder_key
        self.decoder = MLP(self.cfg.hidden_dim, self.cfg.feature_dim, 16, 2, key=g)
        self.wrapped_vector_field = vector_fields.CDEWrapperVectorField(vector_field, self.cfg.hidden_dim)
        self.dt0 = dt0

    def batched(self, ts, coeffs_adj, x_coeffs, x0, evolving_out=False, global_readout=True):
        if evolving_out:
            raise NotImplementedError("PGT drivers save at t1 (pgt_graph_neural_cde.py:116-117)")
        control_adj = _control(ts, coeffs_adj)
        control_data = _control(ts, x_coeffs)
        ts_d = control_adj.graph_layout()[0]
        y0 = self.encoder.run(torch.as_tensor(x0, dtype=torch.float32, device=ts_d.device))
        prob = self.wrapped_vector_field.problem(control_adj, control_data)
        grids = [layout.constant_step_grid(t[0], t[-1], self.dt0) for t in ts_d.cpu().numpy()]
        grid, ns = layout.stack_grids(grids, device=ts_d.device)
        spec = engine.SolverSpec(method=_lib.TSIT5, controller=_lib.CTRL_GRID, save_mode=_lib.SAVE_T1, grid=grid,
                                 nsteps=ns)
        if torch.is_grad_enabled():  # differentiable: GPU discrete adjoint through the CDE solve
            params, fusion = self.vector_field.diff_tensors(prob.n, ts_d.device)
            yT = autograd.solve(prob, spec, y0, params, fusion)
        else:
            yT = engine.integrate(prob, spec, y0)
        out = self.decoder.run(yT)
        return out.sum(dim=1) if global_readout else out

    def loss_terms(self, ts, coeffs_adj, x_coeffs, x0, labels):
        """(sum of squared errors, count) of trainer_pgt.mse_loss (trainer_pgt.py:45-66) over the windows of
        this shard.  The reference reshapes the global read-out to (feature_dim, 1) and subtracts the window's
        label (last_snapshot.y, one value per node): broadcasting compares the read-out with every node's
        label, and jnp.mean averages those feature_dim x n squares.  Same here, per window."""
        pred = self.batched(ts, coeffs_adj, x_coeffs, x0)  # [B, feature_dim]
        B = pred.shape[0]
        labels = torch.as_tensor(labels, dtype=torch.float32, device=pred.device).reshape(B, 1, -1)
        diff = pred.reshape(B, -1, 1) - labels
        return (diff ** 2).sum(), diff[0].numel() * B

    def __call__(self, ts, coeffs_adj, x_coeffs, x0, evolving_out=False, global_readout=True):
        ts = torch.as_tensor(np.asarray(ts) if not torch.is_tensor(ts) else ts, dtype=torch.float32)
        return self.batched(ts.unsqueeze(0), _as_batched_coeffs(coeffs_adj, False),
                            _as_batched_coeffs(x_coeffs, False), torch.as_tensor(x0).unsqueeze(0),
                            evolving_out, global_readout)[0]


class TGBGraphNeuralCDE(nn.Module):
    """``tgb_graph_neural_cde.py:13-171``: data spline built inside forward from Linear(n -> de) embeddings
    of the adjacency rows, Linear(n -> h) encoder, CDEWrapper(vf), Tsit5 + ConstantStepSize(dt0 = 0.01),
    Linear(h -> n) decoder per node.

    ``solver="pid"`` (build extension, BASELINE config 5's "adaptive Tsit5 solver") replaces ConstantStepSize with
    the dyn model's controller, PIDController(rtol 1e-3, atol 1e-6) with dt0 = None (graph_neural_cde.py:53-54,
    94-104), differentiated on each window's accepted steps; ``last_steps`` then holds every window's accepted
    step count of the latest forward (the data-parallel trainer balances ranks by it).

    ``compute`` (build extension): the solve's arithmetic, "fp32" | "bf16" | "bf16_storage" (include/gncde.h
    GNCDE_COMPUTE_*).  "bf16_storage" is config 5's bf16 path: bfloat16 operator coefficients (half the form's
    coefficient stream) read by the persistent adaptive solve with fp32 products, so the PID controller sees no
    rounding noise.  The single-plane "bf16_mfma" mode is not offered here: it deviates 8-24 % from
    fp32 at no speed-up (round-4 measurements) and the PID controller refuses it."""

    def __init__(self, cfg, vector_field, interpolation="cubic", model_key=None, dt0=0.01, solver=None,
                 compute="fp32", **kwargs):
        super().__init__()
        self.cfg = _cfg(cfg, hidden_dim=32, method="Tsit5", return_sequence=False, use_mlps=False)
        if getattr(self.cfg, "use_mlps", False):
            raise NotImplementedError("use_mlps=True variant not on the hot path")
        self.vector_field = vector_field
        n, de = vector_field.num_nodes, vector_field.data_embed_dim
        g = _gen(model_key)
        enc_state = g.get_state()
        self.encoder = _linear(n, self.cfg.hidden_dim, g)
        self.decoder = _linear(self.cfg.hidden_dim, n, g)
        g.set_state(enc_state)  # tgb_graph_neural_cde.py:86-89: data_encoder reuses encoder_key
        self.data_encoder = _linear(n, de, g)
        self.wrapped_vector_field = vector_fields.CDEWrapperVectorField(vector_field, self.cfg.hidden_dim)
        self.dt0 = dt0
        if solver not in (None, "constant", "pid"):
            raise ValueError(f"solver {solver!r}: None / 'constant' (ConstantStepSize) or 'pid'")
        self.adaptive = solver == "pid"
        if compute not in ("fp32", "bf16", "bf16_storage"):
            raise ValueError(f"compute {compute!r}: 'fp32', 'bf16' or 'bf16_storage' (the single-plane 'bf16_mfma' "
                             "mode is retired from the TGB model: 8-24 % from fp32 at no speed-up, DESIGN.md §3.5)")
        self.compute = compute
        self.last_steps = None

    def batched(self, ts, coeffs_adj, x_data, x0, start_time=None, evolving_out=False):
        if evolving_out:
            raise NotImplementedError("SaveAt(ts) with ConstantStepSize (dense output) is not implemented")
        control_adj = _control(ts, coeffs_adj)
        ts_d = control_adj.graph_layout()[0]
        xd = _affine(self.data_encoder, torch.as_tensor(x_data, dtype=torch.float32, device=ts_d.device))
        X = torch.stack([ts_d[:, :, None, None].expand_as(xd), xd], dim=-1)  # [B, T, n, de, 2]
        # the data spline rebuilt inside every forward (tgb_graph_neural_cde.py:118-130), on the GPU and
        # directly in the engine layout [B, T-1, 4, n, de, 2]
        grad = torch.is_grad_enabled()
        data_coef = autograd.hermite_coefficients(ts_d, X) if grad else engine.hermite_coefficients(ts_d, X)
        y0 = _affine(self.encoder, torch.as_tensor(x0, dtype=torch.float32, device=ts_d.device))
        prob = self.wrapped_vector_field.problem(control_adj, None, data_coef=data_coef.detach())
        if self.compute != "fp32":
            prob = prob.with_compute(self.compute)
        if self.adaptive:
            spec = engine.SolverSpec(method=_lib.TSIT5, controller=_lib.CTRL_PID, save_mode=_lib.SAVE_T1, rtol=1e-3,
                                     atol=1e-6, t0=ts_d[:, 0].contiguous(), t1=ts_d[:, -1].contiguous(),
                                     stats_out=torch.zeros(ts_d.shape[0], 4, dtype=torch.int32, device=ts_d.device))
        else:
            grids = [layout.constant_step_grid(t[0], t[-1], self.dt0) for t in ts_d.cpu().numpy()]
            grid, ns = layout.stack_grids(grids, device=ts_d.device)
            spec = engine.SolverSpec(method=_lib.TSIT5, controller=_lib.CTRL_GRID, save_mode=_lib.SAVE_T1, grid=grid,
                                     nsteps=ns)
        if grad:  # differentiable: discrete adjoint incl. the data spline -> data_encoder
            params, fusion = self.vector_field.diff_tensors(prob.n, ts_d.device)
            ys = autograd.solve(prob, spec, y0, params, fusion, data_coef=data_coef)
        elif self.adaptive:
            ys, st = engine.integrate(prob, spec, y0, stats=True)
            if torch.any(st[:, _lib.STAT_STATUS] != 0):
                raise RuntimeError("diffrax-equivalent failure: max_steps reached or non-finite state")
            spec.stats_out.copy_(st)
        else:
            ys = engine.integrate(prob, spec, y0)
        if self.adaptive:
            self.last_steps = spec.stats_out[:, _lib.STAT_STEPS]
        return _affine(self.decoder, ys)

    def loss_terms(self, ts, coeffs_adj, x_data, x0, labels, source_mask):
        """(sum of masked cross-entropies, number of unmasked rows) of trainer_tgb.cross_entropy_loss
        (trainer_tgb.py:42-60): -sum(label * log_softmax(pred)) per node, rows where source_mask is True."""
        pred = self.batched(ts, coeffs_adj, x_data, x0)
        labels = torch.as_tensor(labels, dtype=torch.float32, device=pred.device).reshape(pred.shape)
        mask = torch.as_tensor(source_mask, device=pred.device).reshape(pred.shape[:-1]).to(pred.dtype)
        ce = -(labels * torch.log_softmax(pred, dim=-1)).sum(dim=-1)
        return (ce * mask).sum(), mask.sum()

    def __call__(self, ts, coeffs_adj, x_data, x0, start_time=None, evolving_out=False):
        ts = torch.as_tensor(np.asarray(ts) if not torch.is_tensor(ts) else ts, dtype=torch.float32)
        return self.batched(ts.unsqueeze(0), _as_batched_coeffs(coeffs_adj, False),
                            torch.as_tensor(x_data).unsqueeze(0), torch.as_tensor(x0).unsqueeze(0),
                            start_time, evolving_out)[0]
