"""Differentiable fixed-grid solve: ``torch.autograd`` over ``gncde_integrate`` / ``gncde_integrate_vjp``.

Replaces ``equinox.filter_value_and_grad`` through ``diffrax.diffeqsolve`` (trainer.py:315 over
graph_neural_cde.py:94-104): the forward keeps every step state (SAVE_STEPS) as the checkpoints, and the
backward is the discrete adjoint computed on the GPU (gncde_vjp.hip).  Parameters enter as the packed
buffer ``params`` (include/gncde.h layout) and the factored fusion table ``fusion`` [L, 24]; both are
ordinary differentiable torch tensors, so gradients flow on to the reference-named module parameters
through ``layout.fusion_table_torch`` (the linear map whose transpose turns table gradients into
``param1..param8`` gradients) and ``torch.cat`` of the ConvLayer weights.
"""
from __future__ import annotations

import dataclasses

import torch

from . import _lib, engine


class _FixedGridSolve(torch.autograd.Function):
    @staticmethod
    def forward(ctx, y0, params, fusion, data_coef, prob, spec):
        p = dataclasses.replace(prob, params=params.detach().to(torch.float32).contiguous(),
                                fusion=fusion.detach().to(torch.float32).contiguous())
        if data_coef is not None:
            p = dataclasses.replace(p, data_coef=data_coef.detach().to(torch.float32).contiguous())
        steps = dataclasses.replace(spec, save_mode=_lib.SAVE_STEPS)
        ys = engine.integrate(p, steps, y0.detach())
        ctx.prob, ctx.spec = p, spec
        ctx.dtypes = (y0.dtype, params.dtype, fusion.dtype)
        ctx.save_for_backward(ys)
        if spec.save_mode == _lib.SAVE_STEPS:
            return ys
        return ys[:, -1].contiguous()  # padded steps of short samples repeat the final state

    @staticmethod
    def backward(ctx, g):
        (ys,) = ctx.saved_tensors
        gdata = None
        if ctx.needs_input_grad[3]:
            gy0, gp, gf, gdata = engine.integrate_vjp(ctx.prob, ctx.spec, ys, g, data_grad=True)
        else:
            gy0, gp, gf = engine.integrate_vjp(ctx.prob, ctx.spec, ys, g)
        d0, dp, df = ctx.dtypes
        return gy0.to(d0), gp.to(dp), gf.to(df), gdata, None, None


def solve(prob: engine.Problem, spec: engine.SolverSpec, y0: torch.Tensor, params: torch.Tensor | None = None,
          fusion: torch.Tensor | None = None, data_coef: torch.Tensor | None = None) -> torch.Tensor:
    """Fixed-grid solve that records a backward.  ``spec.save_mode`` SAVE_T1 returns [B, n, d] (final
    state), SAVE_STEPS returns [B, G, n, d].  ``params`` / ``fusion`` default to the problem's own
    (then only ``y0`` can carry gradients).  ``data_coef`` (CDE problems) replaces the problem's data
    spline with a differentiable one (TGBGraphNeuralCDE's in-forward spline of the embedded data)."""
    if spec.controller != _lib.CTRL_GRID:
        raise _lib.GncdeError("the differentiable solve needs a fixed grid (GRID controller); "
                              "adaptive PID solves are forward-only in this build")
    if spec.save_mode not in (_lib.SAVE_T1, _lib.SAVE_STEPS):
        raise _lib.GncdeError("differentiable solve: save_mode must be SAVE_T1 or SAVE_STEPS")
    params = prob.params if params is None else params
    fusion = prob.fusion if fusion is None else fusion
    return _FixedGridSolve.apply(y0, params, fusion, data_coef, prob, spec)


class _Hermite(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ts, X, ncoef):
        ctx.save_for_backward(ts)
        ctx.ncoef = ncoef
        return engine.hermite_coefficients(ts, X.detach(), ncoef)

    @staticmethod
    def backward(ctx, g):
        (ts,) = ctx.saved_tensors
        return None, engine.hermite_coefficients_vjp(ts, g, ctx.ncoef), None


def hermite_coefficients(ts: torch.Tensor, X: torch.Tensor, ncoef: int = 4) -> torch.Tensor:
    """Differentiable (w.r.t. X) backward-Hermite coefficients on gncde_hermite_coefficients(_vjp)."""
    return _Hermite.apply(ts, X, ncoef)


class _NodeAffine(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, W, b):
        ctx.save_for_backward(x, W)
        ctx.has_b = b is not None
        return engine.node_affine(x, W, b)

    @staticmethod
    def backward(ctx, g):
        x, W = ctx.saved_tensors
        gx, gW, gb = engine.node_affine_grad(x, W, g, ctx.needs_input_grad[0], ctx.needs_input_grad[1],
                                             ctx.has_b and ctx.needs_input_grad[2])
        return gx, gW, gb


def node_affine(x: torch.Tensor, W: torch.Tensor, b: torch.Tensor | None) -> torch.Tensor:
    """Differentiable per-node affine map (eqx.nn.Linear under vmap) on gncde_node_affine(_grad)."""
    return _NodeAffine.apply(x.to(torch.float32), W.to(device=x.device, dtype=torch.float32),
                             None if b is None else b.to(device=x.device, dtype=torch.float32))
