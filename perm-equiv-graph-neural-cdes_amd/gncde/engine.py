"""Batched entry points over torch device tensors -> libgncde_hip.so.

``vf_eval`` replaces ``jax.vmap(PermEquivGraphVectorField.__call__)`` (perm_equiv_graph_vector_field.py:85-129)
and ``integrate`` replaces ``jax.vmap`` of ``diffrax.diffeqsolve`` (graph_neural_cde.py:94-104 and the
PGT/TGB drivers).  All tensors must already live on the current CUDA(HIP) device; work is enqueued on
torch's current stream.  Errors from the library raise ``GncdeError``.
"""
from __future__ import annotations

import ctypes
import dataclasses
from dataclasses import dataclass, field

import torch

from . import _lib
from . import layout


def _require_gpu():
    if not torch.cuda.is_available():
        raise _lib.GncdeError("no HIP device visible: the GNCDE engine runs only on the GPU (no CPU path)")


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


@dataclass
class Problem:
    """Device-resident problem description (mirrors ``GncdeProblem``)."""

    ts: torch.Tensor            # [B, T]
    coef: torch.Tensor          # [B, T-1, 4, n, n]
    tcoef: torch.Tensor         # [B, T-1, 3, n]
    fusion: torch.Tensor        # [L, 24] fp32
    params: torch.Tensor        # packed fp32
    dims: list
    data_coef: torch.Tensor | None = None  # [B, T-1, 4, n, de, 2]
    cde_hidden: int = 0
    cde_embed: int = 0
    compute: int = _lib.COMPUTE_FP32  # COMPUTE_BF16(_STORAGE): the generic bf16 MFMA path (reverse mode: fp32 adjoint)
    _keep: list = field(default_factory=list)

    @property
    def B(self):
        return int(self.ts.shape[0])

    @property
    def n(self):
        return int(self.coef.shape[-1])

    @property
    def T(self):
        return int(self.ts.shape[1])

    @property
    def L(self):
        return len(self.dims) - 1

    def c_struct(self) -> _lib.GncdeProblem:
        for name in ("ts", "coef", "tcoef", "fusion", "params"):
            t = getattr(self, name)
            want = torch.bfloat16 if (name == "coef" and self.compute in _lib.BF16_COEF_MODES) else torch.float32
            if not (t.is_cuda and t.dtype == want and t.is_contiguous()):
                raise _lib.GncdeError(f"Problem.{name} must be a contiguous {want} CUDA tensor")
        if len(self.dims) - 1 > _lib.MAX_LAYERS:
            raise _lib.GncdeError("too many layers")
        s = _lib.GncdeProblem()
        s.B, s.n, s.T, s.L = self.B, self.n, self.T, self.L
        for i, d in enumerate(self.dims):
            s.dims[i] = int(d)
        s.cde_hidden, s.cde_embed = int(self.cde_hidden), int(self.cde_embed)
        s.ts, s.coef, s.tcoef = _ptr(self.ts).value, _ptr(self.coef).value, _ptr(self.tcoef).value
        s.data_coef = _ptr(self.data_coef).value if self.data_coef is not None else None
        s.fusion, s.params = _ptr(self.fusion).value, _ptr(self.params).value
        s.compute = int(self.compute)
        return s

    def shard(self, start: int, stop: int) -> "Problem":
        """Contiguous batch shard (data-parallel ranks own [start, stop))."""
        return Problem(ts=self.ts[start:stop], coef=self.coef[start:stop], tcoef=self.tcoef[start:stop],
                       fusion=self.fusion, params=self.params, dims=list(self.dims),
                       data_coef=None if self.data_coef is None else self.data_coef[start:stop],
                       cde_hidden=self.cde_hidden, cde_embed=self.cde_embed, compute=self.compute)

    def take(self, idx) -> "Problem":
        """The samples ``idx`` (any order) as their own Problem (a data-parallel rank's balanced shard)."""
        ix = torch.as_tensor(idx, dtype=torch.long, device=self.ts.device)
        return Problem(ts=self.ts[ix].contiguous(), coef=self.coef[ix].contiguous(), tcoef=self.tcoef[ix].contiguous(),
                       fusion=self.fusion, params=self.params, dims=list(self.dims),
                       data_coef=None if self.data_coef is None else self.data_coef[ix].contiguous(),
                       cde_hidden=self.cde_hidden, cde_embed=self.cde_embed, compute=self.compute)

    def with_compute(self, compute: str) -> "Problem":
        """The same problem in another arithmetic ("fp32" | "bf16" | "bf16_storage" | "bf16_mfma": coefficients cast
        here)."""
        mode = COMPUTE_MODES[compute]
        dt = torch.bfloat16 if mode in _lib.BF16_COEF_MODES else torch.float32
        return Problem(ts=self.ts, coef=self.coef.to(dt).contiguous(), tcoef=self.tcoef, fusion=self.fusion,
                       params=self.params, dims=list(self.dims), data_coef=self.data_coef,
                       cde_hidden=self.cde_hidden, cde_embed=self.cde_embed, compute=mode)


COMPUTE_MODES = {"fp32": _lib.COMPUTE_FP32, "bf16": _lib.COMPUTE_BF16, "bf16_storage": _lib.COMPUTE_BF16_STORAGE,
                 "bf16_mfma": _lib.COMPUTE_BF16_MFMA}


def make_problem(ts, coeffs, kind, layers, data_coeffs=None, cde_hidden=0, cde_embed=0, device="cuda",
                 compute="fp32"):
    """Build a Problem from reference-layout inputs (ts [B,T], coeffs (d,c,b,a) [B,T-1,n,n,2], layer dicts).

    compute="bf16" runs the n x n products on bf16 MFMA (split pairs, fp32-class results); "bf16_storage" also
    stores the operator coefficients in bfloat16; "bf16_mfma" (retired: the product library refuses it, an experiment
    build — `make experiment` — still has it) stores them in bfloat16 and runs every product on
    single-plane bf16 MFMA operands (BASELINE config 5's throughput mode; one-launch evaluation shapes only).  Reverse
    mode = the fp32 adjoint over the coefficients read, see gncde.h GNCDE_COMPUTE_*."""
    coef, tcoef = layout.pack_control(coeffs, device=device)
    mode = COMPUTE_MODES[compute]
    if mode in _lib.BF16_COEF_MODES:
        coef = coef.to(torch.bfloat16).contiguous()
    ts = torch.as_tensor(ts, dtype=torch.float32)
    if ts.dim() == 1:
        ts = ts.unsqueeze(0)
    n = coef.shape[-1]
    fusion = layout.fusion_table(kind, layers, n).to(torch.float32).to(device).contiguous()
    params = layout.pack_params(layers, device=device)
    dc = layout.pack_data_control(data_coeffs, device=device) if data_coeffs is not None else None
    return Problem(ts=ts.to(device).contiguous(), coef=coef, tcoef=tcoef, fusion=fusion, params=params,
                   dims=layout.layer_dims(layers), data_coef=dc, cde_hidden=cde_hidden, cde_embed=cde_embed,
                   compute=mode)


class _Workspace:
    """Grow-only device scratch buffer (one per device)."""

    _bufs: dict = {}

    @classmethod
    def get(cls, nbytes: int):
        dev = torch.cuda.current_device()
        buf = cls._bufs.get(dev)
        if buf is None or buf.numel() < nbytes:
            buf = torch.empty(max(nbytes, 1), dtype=torch.uint8, device="cuda")
            cls._bufs[dev] = buf
        return buf


def vf_eval(prob: Problem, t: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    """dy[b] = VF(t[b], y[b]) for every sample.  t [B], y [B, n, d_0] -> [B, n, d_out]."""
    _require_gpu()
    lib = _lib.load()
    ps = prob.c_struct()
    t = t.to(device=y.device, dtype=torch.float32).contiguous()
    y = y.contiguous()
    if y.shape != (prob.B, prob.n, prob.dims[0]) or t.shape != (prob.B,):
        raise _lib.GncdeError(f"vf_eval: bad shapes t{tuple(t.shape)} y{tuple(y.shape)}")
    dout = prob.cde_hidden if prob.cde_hidden > 0 else prob.dims[-1]
    dy = torch.empty(prob.B, prob.n, dout, dtype=torch.float32, device=y.device)
    nbytes = lib.gncde_workspace_bytes(ctypes.byref(ps), None)
    ws = _Workspace.get(nbytes)
    _lib.check(lib.gncde_vf_eval(ctypes.byref(ps), _ptr(t), _ptr(y), _ptr(dy), _ptr(ws), nbytes, _stream()))
    return dy


@dataclass
class SolverSpec:
    """Mirrors ``GncdeSolver``.  For fixed grids, ``grid`` [B, G] and ``nsteps`` [B] (layout.stack_grids)."""

    method: int = _lib.RK4
    controller: int = _lib.CTRL_GRID
    save_mode: int = _lib.SAVE_T1
    grid: torch.Tensor | None = None
    nsteps: torch.Tensor | None = None
    rtol: float = 1e-3
    atol: float = 1e-6
    max_steps: int = 4096
    t0: torch.Tensor | None = None
    t1: torch.Tensor | None = None
    dt0: torch.Tensor | None = None
    save_ts: torch.Tensor | None = None
    step_ts: torch.Tensor | None = None  # PID: OUTPUT [B, cap] accepted step times (t0 first), filled by integrate
    # GRID: stage record [B, stage_record_floats(prob, solver)] written by integrate, read by integrate_vjp
    stage_rec: torch.Tensor | None = None
    flags: int = 0  # GNCDE_FLAG_* (FLAG_GENERIC: the generic forward and reverse sweep even where fused kernels fit)
    # host side only (not in GncdeSolver): autograd.solve copies the forward's stats [B, 4] here when given (the
    # trainers balance data-parallel shards by the adaptive solves' accepted step counts)
    stats_out: torch.Tensor | None = None
    # GRID: activation record [activation_record_floats(prob, solver)] (the whole batch, [G-1, S, L-1, B, n, H]),
    # written by integrate, read by integrate_vjp (ABI 7)
    act_rec: torch.Tensor | None = None
    # PID (ABI 8): the persistent solve's record of its accepted steps — checkpoints [B, rec_steps, n, d] here,
    # stage_rec [B, rec_steps * 5 * n * d], act_rec [rec_steps * 6 * (L-1) * B * n * H] (autograd.pid_records)
    pid_ckpt: torch.Tensor | None = None
    rec_steps: int = 0

    def c_struct(self) -> _lib.GncdeSolver:
        s = _lib.GncdeSolver()
        s.method, s.controller, s.save_mode, s.max_steps = self.method, self.controller, self.save_mode, \
            self.max_steps
        s.grid_len = int(self.grid.shape[1]) if self.grid is not None else 0
        s.n_save = int(self.save_ts.shape[1]) if self.save_ts is not None else 0
        s.rtol, s.atol = self.rtol, self.atol
        s.grid = _ptr(self.grid).value if self.grid is not None else None
        s.nsteps = _ptr(self.nsteps).value if self.nsteps is not None else None
        s.t0 = _ptr(self.t0).value if self.t0 is not None else None
        s.t1 = _ptr(self.t1).value if self.t1 is not None else None
        s.dt0 = _ptr(self.dt0).value if self.dt0 is not None else None
        s.save_ts = _ptr(self.save_ts).value if self.save_ts is not None else None
        if self.step_ts is not None:
            if not (self.step_ts.is_cuda and self.step_ts.dtype == torch.float32 and self.step_ts.is_contiguous()):
                raise _lib.GncdeError("SolverSpec.step_ts must be a contiguous fp32 CUDA tensor [B, cap]")
            s.step_ts = _ptr(self.step_ts).value
            s.step_ts_len = int(self.step_ts.shape[1])
        if self.stage_rec is not None:
            if not (self.stage_rec.is_cuda and self.stage_rec.dtype == torch.float32
                    and self.stage_rec.is_contiguous() and self.stage_rec.dim() == 2):
                raise _lib.GncdeError("SolverSpec.stage_rec must be a contiguous fp32 CUDA tensor [B, floats]")
            s.stage_rec = _ptr(self.stage_rec).value
            s.stage_rec_len = int(self.stage_rec.shape[1])
        if self.act_rec is not None:
            if not (self.act_rec.is_cuda and self.act_rec.dtype == torch.float32 and self.act_rec.is_contiguous()):
                raise _lib.GncdeError("SolverSpec.act_rec must be a contiguous fp32 CUDA tensor")
            s.act_rec = _ptr(self.act_rec).value
            s.act_rec_len = int(self.act_rec.numel())
        if self.pid_ckpt is not None:
            if not (self.pid_ckpt.is_cuda and self.pid_ckpt.dtype == torch.float32 and self.pid_ckpt.is_contiguous()):
                raise _lib.GncdeError("SolverSpec.pid_ckpt must be a contiguous fp32 CUDA tensor [B, rec_steps, n, d]")
            s.pid_ckpt = _ptr(self.pid_ckpt).value
        s.rec_steps = int(self.rec_steps)
        s.flags = int(self.flags)
        return s

    def shard(self, start, stop):
        """The spec of samples [start, stop) (the activation record is batch-major and is not carried over: a
        shard records its own)."""
        cut = lambda x: None if x is None else x[start:stop]  # noqa: E731
        return SolverSpec(self.method, self.controller, self.save_mode, cut(self.grid), cut(self.nsteps),
                          self.rtol, self.atol, self.max_steps, cut(self.t0), cut(self.t1), cut(self.dt0),
                          cut(self.save_ts), cut(self.step_ts), cut(self.stage_rec), self.flags)


def stage_record_floats(prob: Problem, solver: SolverSpec) -> int:
    """Floats per sample of the stage record the reverse sweep would read (0: it would ignore one)."""
    lib = _lib.load()
    ss = dataclasses.replace(solver, stage_rec=None).c_struct()
    return int(lib.gncde_stage_record_floats(ctypes.byref(prob.c_struct()), ctypes.byref(ss)))


def activation_record_floats(prob: Problem, solver: SolverSpec) -> int:
    """Floats of the activation record (the whole batch) the reverse sweep would read (0: none is kept)."""
    lib = _lib.load()
    ss = dataclasses.replace(solver, stage_rec=None, act_rec=None).c_struct()
    return int(lib.gncde_activation_record_floats(ctypes.byref(prob.c_struct()), ctypes.byref(ss)))


def integrate_path(prob: Problem, solver: SolverSpec) -> str:
    lib = _lib.load()
    ps, ss = prob.c_struct(), solver.c_struct()
    buf = ctypes.create_string_buffer(128)
    _lib.check(lib.gncde_integrate_path(ctypes.byref(ps), ctypes.byref(ss), buf, 128))
    return buf.value.decode()


def integrate(prob: Problem, solver: SolverSpec, y0: torch.Tensor, stats: bool = False):
    """Solve every sample.  Returns ys (and stats [B, 4] int32 if requested)."""
    _require_gpu()
    lib = _lib.load()
    ps, ss = prob.c_struct(), solver.c_struct()
    y0 = y0.to(torch.float32).contiguous()
    ds = prob.dims[0]
    if y0.shape != (prob.B, prob.n, ds):
        raise _lib.GncdeError(f"integrate: y0 shape {tuple(y0.shape)} != {(prob.B, prob.n, ds)}")
    if solver.save_mode == _lib.SAVE_T1:
        ys = torch.empty(prob.B, prob.n, ds, dtype=torch.float32, device=y0.device)
    elif solver.save_mode == _lib.SAVE_STEPS:
        ys = torch.empty(prob.B, ss.grid_len, prob.n, ds, dtype=torch.float32, device=y0.device)
    else:
        ys = torch.empty(prob.B, ss.n_save, prob.n, ds, dtype=torch.float32, device=y0.device)
    st = torch.zeros(prob.B, 4, dtype=torch.int32, device=y0.device)
    nbytes = lib.gncde_workspace_bytes(ctypes.byref(ps), ctypes.byref(ss))
    ws = _Workspace.get(nbytes) if nbytes else None
    _lib.check(lib.gncde_integrate(ctypes.byref(ps), ctypes.byref(ss), _ptr(y0), _ptr(ys), _ptr(st),
                                   _ptr(ws), nbytes, _stream()))
    return (ys, st) if stats else ys


def integrate_vjp(prob: Problem, solver: SolverSpec, ys_steps: torch.Tensor, gys: torch.Tensor,
                  data_grad: bool = False, gstage: torch.Tensor | None = None):
    """Reverse mode of ``integrate`` for a fixed grid (the discrete adjoint ``jax.grad`` takes through
    diffrax's RecursiveCheckpointAdjoint, trainer.py:315).

    ys_steps: [B, G, n, d] the forward's SAVE_STEPS states; gys: cotangent of the forward output in
    ``solver.save_mode`` layout (SAVE_T1 [B, n, d] or SAVE_STEPS [B, G, n, d]); gstage (optional):
    [B, G-1, S, n, d] extra cotangents of the stage values (S = 4 RK4 / 6 Tsit5; gncde_integrate_vjp_ex).
    Returns (gy0 [B, n, d], gparams [P] summed over samples, gfusion [L, 24] summed over samples), plus the
    cotangent of ``prob.data_coef`` (layout of data_coef) when ``data_grad`` (CDE problems only).
    """
    _require_gpu()
    lib = _lib.load()
    ps, ss = prob.c_struct(), solver.c_struct()
    ys_steps = ys_steps.to(torch.float32).contiguous()
    gys = gys.to(torch.float32).contiguous()
    B, n, ds = prob.B, prob.n, prob.dims[0]
    if ys_steps.shape != (B, ss.grid_len, n, ds):
        raise _lib.GncdeError(f"integrate_vjp: ys_steps shape {tuple(ys_steps.shape)}")
    want = (B, n, ds) if solver.save_mode == _lib.SAVE_T1 else (B, ss.grid_len, n, ds)
    if gys.shape != want:
        raise _lib.GncdeError(f"integrate_vjp: gys shape {tuple(gys.shape)} != {want}")
    if gstage is not None:
        S = 4 if solver.method == _lib.RK4 else 6
        gstage = gstage.to(torch.float32).contiguous()
        if gstage.shape != (B, ss.grid_len - 1, S, n, ds):
            raise _lib.GncdeError(f"integrate_vjp: gstage shape {tuple(gstage.shape)} != "
                                  f"{(B, ss.grid_len - 1, S, n, ds)}")
    if data_grad and prob.data_coef is None:
        raise _lib.GncdeError("integrate_vjp(data_grad=True) needs a CDE problem")
    dev = prob.params.device
    gy0 = torch.empty(B, n, ds, dtype=torch.float32, device=dev)
    gparams = torch.empty_like(prob.params)
    gfusion = torch.empty_like(prob.fusion)
    gdata = torch.empty_like(prob.data_coef) if data_grad else None
    nbytes = lib.gncde_vjp_workspace_bytes(ctypes.byref(ps), ctypes.byref(ss))
    ws = _Workspace.get(nbytes) if nbytes else None
    _lib.check(lib.gncde_integrate_vjp_ex(ctypes.byref(ps), ctypes.byref(ss), _ptr(ys_steps), _ptr(gys),
                                          _ptr(gstage), _ptr(gy0), _ptr(gparams), _ptr(gfusion), _ptr(gdata),
                                          _ptr(ws), nbytes, _stream()))
    return (gy0, gparams, gfusion, gdata) if data_grad else (gy0, gparams, gfusion)


def node_affine(x: torch.Tensor, W: torch.Tensor, b: torch.Tensor | None) -> torch.Tensor:
    """out[..., :] = W @ x[..., :] + b per row (eqx.nn.Linear under vmap)."""
    _require_gpu()
    lib = _lib.load()
    x = x.to(torch.float32).contiguous()
    W = W.to(device=x.device, dtype=torch.float32).contiguous()
    bb = b.to(device=x.device, dtype=torch.float32).contiguous() if b is not None else None
    din, dout = int(W.shape[1]), int(W.shape[0])
    rows = x.numel() // din
    out = torch.empty(*x.shape[:-1], dout, dtype=torch.float32, device=x.device)
    _lib.check(lib.gncde_node_affine(rows, din, dout, _ptr(x), _ptr(W), _ptr(bb), _ptr(out), _stream()))
    return out


def node_affine_grad(x: torch.Tensor, W: torch.Tensor, g: torch.Tensor, need_x=True, need_w=True, need_b=True):
    """Reverse mode of ``node_affine``: (gx, gW, gb) for cotangent g [..., dout] (None where not needed)."""
    _require_gpu()
    lib = _lib.load()
    x = x.to(torch.float32).contiguous()
    W = W.to(device=x.device, dtype=torch.float32).contiguous()
    g = g.to(device=x.device, dtype=torch.float32).contiguous()
    din, dout = int(W.shape[1]), int(W.shape[0])
    rows = x.numel() // din
    gx = torch.empty_like(x) if need_x else None
    gW = torch.empty_like(W) if need_w else None
    gb = torch.empty(dout, dtype=torch.float32, device=x.device) if need_b else None
    _lib.check(lib.gncde_node_affine_grad(rows, din, dout, _ptr(x), _ptr(W), _ptr(g), _ptr(gx), _ptr(gW), _ptr(gb),
                                          _stream()))
    return gx, gW, gb


def clip_adamw(params: torch.Tensor, grads: torch.Tensor, m: torch.Tensor, v: torch.Tensor, step: int, lr: float,
               b1: float, b2: float, eps: float, weight_decay: float, max_norm: float) -> torch.Tensor:
    """In-place optax.chain(clip_by_global_norm, adamw) update of a flat fp32 buffer.  Returns the device
    stats [3] = (global grad norm, max|grad|, max|update|)."""
    _require_gpu()
    lib = _lib.load()
    for t in (params, grads, m, v):
        if not (t.is_cuda and t.dtype == torch.float32 and t.is_contiguous() and t.numel() == params.numel()):
            raise _lib.GncdeError("clip_adamw: params/grads/m/v must be contiguous fp32 CUDA buffers of one size")
    P = params.numel()
    stats = torch.zeros(3, dtype=torch.float32, device=params.device)
    nbytes = lib.gncde_adamw_workspace_bytes(P)
    ws = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=params.device)
    _lib.check(lib.gncde_clip_adamw(P, _ptr(params), _ptr(grads), _ptr(m), _ptr(v), int(step), lr, b1, b2, eps,
                                    weight_decay, max_norm, _ptr(stats), _ptr(ws), nbytes, _stream()))
    return stats


_OPERATORS = {"norm_lap": _lib.OP_NORM_LAP, "norm_adj": _lib.OP_NORM_ADJ, "kipf": _lib.OP_KIPF,
              "normalized_plus": _lib.OP_NORMALIZED_PLUS}


def graph_operator(A: torch.Tensor, operator_type: str = "norm_lap") -> torch.Tensor:
    """``get_graph_operator(operator_type, A, L)`` (misc.py:104-113) on the GPU for a stack of graphs
    A [..., n, n].  Unknown names fall back to norm_lap exactly like the reference's ``else`` branch."""
    _require_gpu()
    lib = _lib.load()
    kind = _OPERATORS.get(operator_type.lower(), _lib.OP_NORM_LAP)
    A = A.to(device="cuda", dtype=torch.float32).contiguous()
    n = int(A.shape[-1])
    graphs = A.numel() // (n * n)
    out = torch.empty_like(A)
    ws = torch.empty(2 * max(graphs, 1) * n, dtype=torch.float32, device=A.device)
    _lib.check(lib.gncde_graph_operator(kind, graphs, n, _ptr(A), _ptr(out), _ptr(ws), _stream()))
    return out


def hermite_coefficients(ts: torch.Tensor, X: torch.Tensor, ncoef: int = 4) -> torch.Tensor:
    """Backward-Hermite coefficients of X [B, T, ...] over ts [B, T] in the engine layout
    [B, T-1, ncoef, ...] ((d, c, b, a) order; ncoef=3 drops a)."""
    _require_gpu()
    lib = _lib.load()
    X = X.to(device="cuda", dtype=torch.float32).contiguous()
    ts = ts.to(device=X.device, dtype=torch.float32).contiguous()
    B, T = int(X.shape[0]), int(X.shape[1])
    C = X.numel() // max(B * T, 1)
    out = torch.empty((B, T - 1, ncoef) + tuple(X.shape[2:]), dtype=torch.float32, device=X.device)
    _lib.check(lib.gncde_hermite_coefficients(B, T, C, ncoef, _ptr(ts), _ptr(X), _ptr(out), _stream()))
    return out


def hermite_coefficients_vjp(ts: torch.Tensor, gout: torch.Tensor, ncoef: int = 4) -> torch.Tensor:
    """Reverse mode of ``hermite_coefficients`` w.r.t. X: gout [B, T-1, ncoef, ...] -> gX [B, T, ...]."""
    _require_gpu()
    lib = _lib.load()
    gout = gout.to(device="cuda", dtype=torch.float32).contiguous()
    ts = ts.to(device=gout.device, dtype=torch.float32).contiguous()
    B, T = int(ts.shape[0]), int(ts.shape[1])
    C = gout.numel() // max(B * (T - 1) * ncoef, 1)
    gX = torch.empty((B, T) + tuple(gout.shape[3:]), dtype=torch.float32, device=gout.device)
    _lib.check(lib.gncde_hermite_coefficients_vjp(B, T, C, ncoef, _ptr(ts), _ptr(gout), _ptr(gX), _stream()))
    return gX


def interval_index(ts: torch.Tensor, t: torch.Tensor, sample: torch.Tensor) -> torch.Tensor:
    _require_gpu()
    lib = _lib.load()
    ts = ts.to(torch.float32).contiguous()
    t = t.to(device=ts.device, dtype=torch.float32).contiguous()
    sample = sample.to(device=ts.device, dtype=torch.int32).contiguous()
    idx = torch.empty(t.numel(), dtype=torch.int32, device=ts.device)
    _lib.check(lib.gncde_interval_index(_ptr(ts), int(ts.shape[0]), int(ts.shape[1]), _ptr(t), _ptr(sample),
                                        _ptr(idx), int(t.numel()), _stream()))
    return idx
