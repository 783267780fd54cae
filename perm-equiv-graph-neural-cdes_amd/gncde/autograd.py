"""Differentiable solves: ``torch.autograd`` over ``gncde_integrate`` / ``gncde_integrate_vjp_ex``.

Replaces ``equinox.filter_value_and_grad`` through ``diffrax.diffeqsolve`` (trainer.py:315 over
graph_neural_cde.py:94-104).  Fixed grids: the forward keeps every step state (SAVE_STEPS) as the checkpoints,
and the backward is the discrete adjoint computed on the GPU (gncde_stage.hip / gncde_vjp.hip).  Adaptive
Tsit5 + PIDController: the forward records each sample's accepted step sequence (GncdeSolver.step_ts); the
backward replays that grid for the checkpoints and runs the same discrete adjoint over it, with the step sizes
held constant (what RecursiveCheckpointAdjoint differentiates through diffrax's while_loop: rejected attempts
leave no trace in the accepted solution) and SaveAt(ts)'s Tsit5 dense interpolant differentiated through
its stage values.  Parameters enter as the packed
buffer ``params`` (include/gncde.h layout) and the factored fusion table ``fusion`` [L, 24]; both are
ordinary differentiable torch tensors, so gradients flow on to the reference-named module parameters
through ``layout.fusion_table_torch`` (the linear map whose transpose turns table gradients into
``param1..param8`` gradients) and ``torch.cat`` of the ConvLayer weights.
"""
from __future__ import annotations

import dataclasses

import torch

from . import _lib, engine


# Tests / A-B runs set NO_PID_RECORD[0] = True to take the replay backward of adaptive solves instead of their record
NO_PID_RECORD = [False]

# Share of the free device memory a stage record may take (GncdeSolver.stage_rec: the forward stores every step's
# stage inputs so the reverse sweep recomputes none; config 4 needs 2.5 GB of the 288 GB).
STAGE_RECORD_SHARE = 0.25


def with_stage_record(prob: engine.Problem, spec: engine.SolverSpec, want: bool = True) -> engine.SolverSpec:
    """``spec`` with a freshly allocated stage record (and, where the reverse sweep reads one, an activation
    record) when it fits in STAGE_RECORD_SHARE of the free device memory."""
    if not want:
        return spec
    floats = engine.stage_record_floats(prob, spec)
    if floats == 0 or prob.B == 0:
        return spec
    free, _ = torch.cuda.mem_get_info(prob.params.device)
    if prob.B * floats * 4 > STAGE_RECORD_SHARE * free:
        return spec
    dev = prob.params.device
    spec = dataclasses.replace(spec, stage_rec=torch.empty(prob.B, floats, dtype=torch.float32, device=dev))
    act = engine.activation_record_floats(prob, spec)
    if act and (prob.B * floats + act) * 4 <= STAGE_RECORD_SHARE * free:
        spec = dataclasses.replace(spec, act_rec=torch.empty(act, dtype=torch.float32, device=dev))
    return spec


class _FixedGridSolve(torch.autograd.Function):
    @staticmethod
    def forward(ctx, y0, params, fusion, data_coef, prob, spec, record):
        p = dataclasses.replace(prob, params=params.detach().to(torch.float32).contiguous(),
                                fusion=fusion.detach().to(torch.float32).contiguous())
        if data_coef is not None:
            p = dataclasses.replace(p, data_coef=data_coef.detach().to(torch.float32).contiguous())
        steps = with_stage_record(p, dataclasses.replace(spec, save_mode=_lib.SAVE_STEPS, stage_rec=None), record)
        ys = engine.integrate(p, steps, y0.detach())
        ctx.prob, ctx.spec = p, dataclasses.replace(spec, stage_rec=steps.stage_rec, act_rec=steps.act_rec)
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
        return gy0.to(d0), gp.to(dp), gf.to(df), gdata, None, None, None


def tsit5_dense_weights(theta: torch.Tensor) -> torch.Tensor:
    """Tsit5 free interpolant b_j(theta), j = 0..6, in fp32 with the kernels' formula (gncde_pid.hip
    tsit5_dense_w; oracle/gncde_oracle.py tsit5_dense_weights): y(t + th h) = y + h sum_j b_j(th) K_j."""
    th = theta.to(torch.float32)
    t2 = th * th
    return torch.stack([
        -1.0530884977290216 * th * (th - 1.3299890189751412) * (t2 - 1.4364028541716351 * th + 0.7139816917074209),
        0.1017 * t2 * (t2 - 2.1966568338249754 * th + 1.2949852507374631),
        2.490627285651252793 * t2 * (t2 - 2.38535645472061657 * th + 1.57803468208092486),
        -16.54810288924490272 * (th - 1.21712927295533244) * (th - 0.61620406037800089) * t2,
        47.37952196281928122 * (th - 1.203071208372362603) * (th - 0.658047292653547382) * t2,
        -34.87065786149660974 * (th - 1.2) * (th - 0.666666666666666667) * t2,
        2.5 * (th - 1.0) * (th - 0.6) * t2], dim=-1)


def pid_replay_grid(step_ts: torch.Tensor, nsteps: torch.Tensor, pad: int = 1):
    """The accepted step sequences of a recorded PID solve as a fixed grid [B, max(nsteps) + 1 + pad]: sample b's
    times step_ts[b, :nsteps[b] + 1], then its last time repeated (zero-length padded steps, identities)."""
    G = int(nsteps.max().item()) + 1 + pad
    cols = torch.arange(G, device=step_ts.device)
    idx = torch.minimum(cols[None, :], nsteps.to(torch.long)[:, None])
    return step_ts.gather(1, idx).contiguous(), nsteps.to(torch.int32).contiguous()


def dense_output_cotangents(grid: torch.Tensor, nsteps: torch.Tensor, save_ts: torch.Tensor, g: torch.Tensor):
    """Reverse mode of SaveAt(ts) through the Tsit5 dense interpolant on a (replayed) grid.

    The save point s of sample b lies in step k (t_k < ts <= t_{k+1}; ts <= t0 returns y0), th = (ts - t_k) / h_k,
    and y(ts) = y_k + h_k sum_j b_j(th) K_j with K_6 = f(t_{k+1}, y_{k+1}) = stage 0 of step k + 1 (FSAL).  Its
    cotangent g_s therefore goes to y_k (returned as per-step cotangents gys [B, G, n, d]) and to the stage values
    (gstage [B, G-1, 6, n, d]: h_k b_j(th) g_s on stage j < 6 of step k, h_k b_6(th) g_s on stage 0 of step k+1;
    the grid carries a padded step after every sample's last one, so k + 1 is always a step index)."""
    B, G = grid.shape
    S = save_ts.shape[1]
    E = g[0, 0].numel()
    ns = nsteps.to(torch.long)
    gf = g.reshape(B, S, E).to(torch.float32)
    t0 = grid[:, :1]
    # k: last grid index with t_k < ts among the sample's real knots (searchsorted 'left' - 1), clamped to a step
    kk = torch.searchsorted(grid.contiguous(), save_ts.to(torch.float32).contiguous(), right=False) - 1
    kk = torch.minimum(torch.clamp(kk, min=0), (ns - 1).clamp(min=0)[:, None])
    direct = save_ts <= t0  # y0 itself
    tk = grid.gather(1, kk)
    hk = grid.gather(1, kk + 1) - tk
    th = torch.where(direct | (hk == 0), torch.zeros_like(hk), (save_ts - tk) / torch.where(hk == 0, 1.0, hk))
    w = tsit5_dense_weights(th) * hk[..., None]  # [B, S, 7] = h_k b_j(th)
    w = torch.where(direct[..., None], torch.zeros_like(w), w)
    gys = torch.zeros(B, G, E, dtype=torch.float32, device=g.device)
    gys.scatter_add_(1, torch.where(direct, 0, kk)[..., None].expand(B, S, E), gf)
    gst = torch.zeros(B, G - 1, 6, E, dtype=torch.float32, device=g.device)
    flat = gst.view(B, (G - 1) * 6, E)
    for j in range(6):
        flat.scatter_add_(1, (kk * 6 + j)[..., None].expand(B, S, E), w[..., j, None] * gf)
    flat.scatter_add_(1, ((kk + 1) * 6)[..., None].expand(B, S, E), w[..., 6, None] * gf)
    shp = tuple(g.shape[2:])
    return gys.view((B, G) + shp), gst.view((B, G - 1, 6) + shp)


# The accepted-step record's slot count is sized from the largest step count seen so far (records that turn out too
# short fall back to the replay); at most STAGE_RECORD_SHARE of the free device memory.
_PID_STEPS_SEEN = [0]


def pid_records(prob: engine.Problem, spec: engine.SolverSpec) -> engine.SolverSpec:
    """``spec`` with the persistent adaptive solve's accepted-step record allocated (GncdeSolver.pid_ckpt, ABI 8:
    checkpoints, stage inputs and the stage evaluations' hidden outputs, so that the reverse mode need not re-run
    the forward over the accepted grid), or unchanged when the solve's path keeps none or it does not fit."""
    if prob.B == 0:
        return spec
    R = min(spec.max_steps + 1, max(64, 2 * _PID_STEPS_SEEN[0] + 8))
    trial = dataclasses.replace(spec, rec_steps=R, stage_rec=None, act_rec=None, pid_ckpt=None)
    sf, af = engine.stage_record_floats(prob, trial), engine.activation_record_floats(prob, trial)
    if not sf or not af:
        return spec
    E = prob.n * prob.dims[0]
    per_slot = (prob.B * sf + af) // R + prob.B * E  # floats per record slot (stage inputs, activations, checkpoint)
    free, _ = torch.cuda.mem_get_info(prob.params.device)
    fit = int(STAGE_RECORD_SHARE * free) // (4 * per_slot)
    if fit < R:
        if fit < 8:
            return spec
        R = fit
        trial = dataclasses.replace(trial, rec_steps=R)
        sf, af = engine.stage_record_floats(prob, trial), engine.activation_record_floats(prob, trial)
    dev = prob.params.device
    return dataclasses.replace(trial, stage_rec=torch.empty(prob.B, sf, dtype=torch.float32, device=dev),
                               act_rec=torch.empty(af, dtype=torch.float32, device=dev),
                               pid_ckpt=torch.empty(prob.B, R, prob.n, prob.dims[0], dtype=torch.float32, device=dev))


def pid_record_grid_inputs(spec: engine.SolverSpec, ns: torch.Tensor, G: int, L: int):
    """The fixed-grid reverse sweep's inputs on the replayed accepted grid (G columns) from the adaptive solve's
    record: checkpoints ys [B, G, n, d], the stage record [B, (G-1) 5 n d] and the activation record's first G-1
    slots.  Past a sample's ns accepted steps the grid has zero-length padded steps: their checkpoints and stage
    inputs are the final state, and every stage evaluation is f(t_ns, y_ns) = the recorded FSAL evaluation of the
    last step (slot (ns, 0)), which is copied into the padded slots."""
    ck = spec.pid_ckpt
    B, R = ck.shape[0], ck.shape[1]
    E = ck[0, 0].numel()
    cols = torch.arange(G, device=ck.device)
    nsl = ns.to(torch.long)
    idx = torch.minimum(cols[None, :], nsl[:, None])  # [B, G]
    ckf = ck.view(B, R, E)
    ys = ckf.gather(1, idx[..., None].expand(B, G, E)).view((B, G) + tuple(ck.shape[2:]))
    final = ckf.gather(1, nsl[:, None, None].expand(B, 1, E))  # [B, 1, E]
    src = spec.stage_rec.view(B, R, 5, E)[:, :G - 1]
    pad = (cols[:G - 1][None, :] >= nsl[:, None])[..., None, None]  # [B, G-1, 1, 1]
    srec = torch.where(pad, final[:, :, None, :], src).reshape(B, -1).contiguous()
    ar = spec.act_rec.view(R, 6, L - 1, B, E)
    kk, bb = torch.nonzero(cols[:G - 1][:, None] >= nsl[None, :], as_tuple=True)  # padded (step, sample) pairs
    if kk.numel():
        ar[kk, :, :, bb] = ar[nsl[bb], 0, :, bb][:, None].expand(-1, 6, -1, -1).clone()
    return ys.contiguous(), srec, ar[:G - 1].reshape(-1)


class _PidSolve(torch.autograd.Function):
    @staticmethod
    def forward(ctx, y0, params, fusion, data_coef, prob, spec, record):
        p = dataclasses.replace(prob, params=params.detach().to(torch.float32).contiguous(),
                                fusion=fusion.detach().to(torch.float32).contiguous())
        if data_coef is not None:
            p = dataclasses.replace(p, data_coef=data_coef.detach().to(torch.float32).contiguous())
        rec = torch.empty(prob.B, spec.max_steps + 1, dtype=torch.float32, device=y0.device)
        fwd = dataclasses.replace(spec, step_ts=rec)
        if record:  # the backward reads the solve's own record of its accepted steps instead of replaying them
            fwd = pid_records(p, fwd)
        ys, st = engine.integrate(p, fwd, y0.detach(), stats=True)
        if torch.any(st[:, _lib.STAT_STATUS] != 0):
            raise _lib.GncdeError("adaptive solve failed (max_steps reached or non-finite error estimate)")
        if spec.stats_out is not None:
            spec.stats_out.copy_(st)
        ctx.prob, ctx.spec, ctx.fwd = p, spec, fwd
        ctx.dtypes = (y0.dtype, params.dtype, fusion.dtype)
        ctx.save_for_backward(y0.detach().to(torch.float32).contiguous(), rec, st[:, _lib.STAT_STEPS].contiguous())
        return ys

    @staticmethod
    def backward(ctx, g):
        y0, rec, ns = ctx.saved_tensors
        spec, fwd = ctx.spec, ctx.fwd
        ctx.fwd = None
        dense = spec.save_mode == _lib.SAVE_TS
        grid, nst = pid_replay_grid(rec, ns, pad=1 if dense else 0)
        steps = engine.SolverSpec(method=_lib.TSIT5, controller=_lib.CTRL_GRID, save_mode=_lib.SAVE_STEPS, grid=grid,
                                  nsteps=nst, flags=spec.flags)
        want_data = ctx.needs_input_grad[3]
        max_ns = int(ns.max().item()) if ns.numel() else 0
        _PID_STEPS_SEEN[0] = max(_PID_STEPS_SEEN[0], max_ns)
        if fwd.pid_ckpt is not None and max_ns + 1 <= fwd.rec_steps:
            # the forward's own record: the reverse sweep of the accepted grid on the fp32 view of the problem
            # (bf16 coefficient storage: its values widened, which is what that forward read)
            p32 = ctx.prob if ctx.prob.compute == _lib.COMPUTE_FP32 else ctx.prob.with_compute("fp32")
            ys, srec, arec = pid_record_grid_inputs(fwd, ns, grid.shape[1], p32.L)
            rsteps = dataclasses.replace(steps, flags=steps.flags | _lib.FLAG_GENERIC, stage_rec=srec, act_rec=arec)
            if dense:
                gys, gst = dense_output_cotangents(grid, nst, spec.save_ts, g)
                res = engine.integrate_vjp(p32, rsteps, ys, gys, data_grad=want_data, gstage=gst)
            else:
                res = engine.integrate_vjp(p32, dataclasses.replace(rsteps, save_mode=_lib.SAVE_T1), ys, g,
                                           data_grad=want_data)
            gy0, gp, gf = res[:3]
            d0, dp, df = ctx.dtypes
            return gy0.to(d0), gp.to(dp), gf.to(df), (res[3] if want_data else None), None, None, None
        # The replay's forward keeps every stage's hidden outputs when the reverse sweep can read them (the
        # host-paced replay, not the one-launch persistent one: config 5's shape spends 35 us per stage re-running
        # the forward otherwise, against ~10 us the host-paced replay costs over the persistent one per evaluation)
        # (only when the activation record is actually allocated: under memory pressure the replay keeps the
        # one-launch persistent forward, since the reverse recomputes every stage either way)
        recorded = None
        if engine.integrate_path(ctx.prob, steps).startswith("rows_grid"):
            gen = dataclasses.replace(steps, flags=steps.flags | _lib.FLAG_GENERIC)
            if engine.activation_record_floats(ctx.prob, gen):
                gen = with_stage_record(ctx.prob, gen)
                if gen.act_rec is not None:
                    recorded = gen
        steps = recorded if recorded is not None else with_stage_record(ctx.prob, steps)
        ys = engine.integrate(ctx.prob, steps, y0)  # the checkpoints (and stage inputs): the accepted steps replayed
        if dense:
            gys, gst = dense_output_cotangents(grid, nst, spec.save_ts, g)
            res = engine.integrate_vjp(ctx.prob, steps, ys, gys, data_grad=want_data, gstage=gst)
        else:
            t1 = dataclasses.replace(steps, save_mode=_lib.SAVE_T1)
            res = engine.integrate_vjp(ctx.prob, t1, ys, g, data_grad=want_data)
        gy0, gp, gf = res[:3]
        d0, dp, df = ctx.dtypes
        return gy0.to(d0), gp.to(dp), gf.to(df), (res[3] if want_data else None), None, None, None


def solve(prob: engine.Problem, spec: engine.SolverSpec, y0: torch.Tensor, params: torch.Tensor | None = None,
          fusion: torch.Tensor | None = None, data_coef: torch.Tensor | None = None) -> torch.Tensor:
    """A solve that records a backward.  Fixed grid (GRID controller): SAVE_T1 returns [B, n, d] (final state),
    SAVE_STEPS [B, G, n, d].  Tsit5 + PIDController: SAVE_T1 [B, n, d] or SAVE_TS [B, S, n, d] (the dense output at
    spec.save_ts).  ``params`` / ``fusion`` default to the problem's own (then only ``y0`` can carry gradients).
    ``data_coef`` (CDE problems) replaces the problem's data spline with a differentiable one (TGBGraphNeuralCDE's
    in-forward spline of the embedded data)."""
    params = prob.params if params is None else params
    fusion = prob.fusion if fusion is None else fusion
    # the forward's stage record only pays when a backward will read it
    record = torch.is_grad_enabled() and any(t is not None and t.requires_grad for t in (y0, params, fusion, data_coef))
    if spec.controller == _lib.CTRL_PID:
        if spec.method != _lib.TSIT5 or spec.save_mode not in (_lib.SAVE_T1, _lib.SAVE_TS):
            raise _lib.GncdeError("differentiable adaptive solve: Tsit5 with SAVE_T1 or SAVE_TS")
        return _PidSolve.apply(y0, params, fusion, data_coef, prob, spec, record and not NO_PID_RECORD[0])
    if spec.save_mode not in (_lib.SAVE_T1, _lib.SAVE_STEPS):
        raise _lib.GncdeError("differentiable fixed-grid solve: save_mode must be SAVE_T1 or SAVE_STEPS")
    return _FixedGridSolve.apply(y0, params, fusion, data_coef, prob, spec, record)


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
