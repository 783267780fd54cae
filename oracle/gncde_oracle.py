"""CPU oracle for the GNCDE hot path — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import this
module, and only as the checker.  The product path (``gncde`` package + ``libgncde_hip.so``) never
calls into it and has no CPU fallback.

What it is
    A plain numpy (float64 by default, float32 on request) restatement of the reference's hot path:

    * ``diffrax.backward_hermite_coefficients`` / ``CubicInterpolation.evaluate|derivative`` as called at
      ``src/configs/dataset_configs.py:147-173`` and ``src/models/vector_fields/perm_equiv_graph_vector_field.py:98-102``
    * ``ConvEquivFusionLayer._fusion``          ``src/models/vector_fields/layers.py:102-160``
    * ``ConvEquivFusionDirectedLayer._fusion``  ``src/models/vector_fields/layers.py:256-337``
    * ``ConvLayer.__call__``                    ``src/models/vector_fields/layers.py:36-48`` (equinox RMSNorm/Linear)
    * ``PermEquivGraphVectorField.__call__``    ``src/models/vector_fields/perm_equiv_graph_vector_field.py:85-129``
    * ``GraphVectorField.__call__``             ``src/models/vector_fields/graph_vector_field.py:80-115``
    * ``CDEWrapperVectorField.__call__``        ``src/models/vector_fields/cde_wrapper_vector_field.py:19-26``
    * the diffrax solves driven from ``src/models/graph_neural_cde.py:94-104`` (Tsit5 + PIDController,
      dt0=None, SaveAt), ``pgt_graph_neural_cde.py:119-129`` and ``tgb_graph_neural_cde.py:152-162``
      (Tsit5 + ConstantStepSize), plus the build's fixed-step RK4 extension (BASELINE config 2).
    * graph operators ``src/dataset/misc.py:58-113``.

PARITY UNPINNED for the hot path: the reference's arithmetic lives in jax/diffrax/equinox, none of
which is installed in this image (ordinary ModuleNotFoundError), and the reference's own
tests (``test/``) hold no golden vectors for models, layers or solvers.  The diffrax/equinox semantics
below are restated from their published algorithms (diffrax and equinox are
unpinned in ``environment.yaml:5-31``).  The data-side operators ARE pinned by the reference's
known-answer tests (``test/dataset/test_misc.py:43-58``), mirrored in ``tests/test_oracle.py``.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np

# ----------------------------------------------------------------------------------------------
# Spline (diffrax CubicInterpolation / backward_hermite_coefficients), SURVEY App. A.1-A.2
# ----------------------------------------------------------------------------------------------


def backward_hermite_coefficients(ts, ys):
    """Restates ``diffrax.backward_hermite_coefficients(ts, ys)`` (call site dataset_configs.py:170).

    ys: [T, ...].  Returns (d, c, b, a), each [T-1, ...].  First knot derivative = forward difference,
    later knot derivatives = backward differences, so interval 0 is linear.
    """
    ts = np.asarray(ts)
    ys = np.asarray(ys)
    T = ts.shape[0]
    dt = (ts[1:] - ts[:-1]).reshape((T - 1,) + (1,) * (ys.ndim - 1))
    slope = (ys[1:] - ys[:-1]) / dt
    deriv = np.concatenate([slope[:1], slope[:-1]], axis=0)  # derivative at the left knot
    dd = slope - deriv
    a = ys[:-1]
    b = deriv
    c = 2.0 * dd / dt
    d = -dd / (dt * dt)
    return d, c, b, a


def interval_index(ts, t):
    """``clip(searchsorted(ts, t, side='left') - 1, 0, T-2)`` — the diffrax CubicInterpolation rule."""
    T = len(ts)
    i = int(np.searchsorted(np.asarray(ts), t, side="left")) - 1
    return min(max(i, 0), T - 2)


def spline_evaluate(ts, coeffs, t):
    d, c, b, a = coeffs
    i = interval_index(ts, t)
    f = t - ts[i]
    return a[i] + f * (b[i] + f * (c[i] + f * d[i]))


def spline_derivative(ts, coeffs, t):
    d, c, b, a = coeffs
    i = interval_index(ts, t)
    f = t - ts[i]
    return b[i] + f * (2.0 * c[i] + f * 3.0 * d[i])


@dataclass
class CubicInterpolation:
    """Minimal stand-in for ``diffrax.CubicInterpolation(ts, coeffs)``: ``.evaluate`` / ``.derivative``."""

    ts: np.ndarray
    coeffs: tuple

    def evaluate(self, t):
        return spline_evaluate(self.ts, self.coeffs, t)

    def derivative(self, t):
        return spline_derivative(self.ts, self.coeffs, t)


# ----------------------------------------------------------------------------------------------
# Fusion layers — literal restatements of the reference term sets (quirks included)
# ----------------------------------------------------------------------------------------------

UNDIRECTED_PARAMS = ("param1", "param2", "param3", "param4", "param5", "param6", "param7", "param8")
DIRECTED_PARAMS = ("param1", "param2", "param3", "param4", "param4_prime", "param5", "param5_prime",
                   "param6", "param6_prime", "param7", "param8")


def fusion_undirected(p, A, dA):
    """``ConvEquivFusionLayer._fusion`` (layers.py:102-160). p: dict name -> array(2)."""
    n = A.shape[0]
    rA, rdA = A.sum(axis=1), dA.sum(axis=1)
    sA, sdA = A.sum(), dA.sum()
    one = np.ones((n, 1), dtype=A.dtype)
    t1 = (1.0 + p["param1"][0]) * A + (1.0 + p["param1"][1]) * dA
    t2 = p["param2"][0] * A.T + p["param2"][1] * dA.T
    t3 = p["param3"][0] * np.diag(np.diag(A)) + p["param3"][1] * np.diag(np.diag(dA))
    t4 = p["param4"][0] / n * np.tile(rA, (n, 1)).T + p["param4"][1] / n * np.tile(rdA, (n, 1)).T
    t5 = p["param5"][0] / n * np.tile(rA, (n, 1)) + p["param5"][1] / n * np.tile(rdA, (n, 1))
    t6 = p["param6"][0] / n * np.diag(rA) + p["param6"][1] / n * np.diag(rdA)
    # layers.py:144-148 — the second half multiplies sum(adjacency), not sum(control_gradient)
    t7 = p["param7"][0] / n**2 * np.full(A.shape, sA) + p["param7"][1] / n**2 * np.full(dA.shape, sA)
    t8 = (p["param8"][0] * sA + p["param8"][1] * sdA) / n**2 * np.eye(n, dtype=A.dtype)
    del one
    return t1 + t2 + t3 + t4 + t5 + t6 + t7 + t8


def fusion_directed(p, A, dA):
    """``ConvEquivFusionDirectedLayer._fusion`` (layers.py:256-337), quirks of :281-293 kept."""
    n = A.shape[0]
    rA, rdA = A.sum(axis=1), dA.sum(axis=1)
    cA, cdA = A.sum(axis=0), dA.sum(axis=0)
    sA, sdA = A.sum(), dA.sum()
    t1 = (1.0 + p["param1"][0]) * A + (1.0 + p["param1"][1]) * dA
    t2 = p["param2"][0] * A.T + p["param2"][1] * dA.T
    t3 = p["param3"][0] * np.diag(np.diag(A)) + p["param3"][1] * np.diag(np.diag(dA))
    t4 = p["param4"][0] / n * np.tile(cA, (n, 1)).T + p["param4"][1] / n * np.tile(cdA, (n, 1)).T
    t4p = p["param4_prime"][0] / n * np.tile(rA, (n, 1)) + p["param4_prime"][1] / n * np.tile(cdA, (n, 1))
    t5 = p["param5"][0] / n * np.tile(cA, (n, 1)) + p["param5"][1] / n * np.tile(cdA, (n, 1))
    t5p = p["param5_prime"][0] / n * np.tile(rA, (n, 1)) + p["param5_prime"][1] / n * np.tile(rdA, (n, 1))
    t6 = p["param6"][0] / n * np.diag(cA) + p["param6"][1] / n * np.diag(cdA)
    t6p = p["param6_prime"][0] / n * np.diag(rA) + p["param6_prime"][1] / n * np.diag(rdA)
    t7 = p["param7"][0] / n**2 * np.full(A.shape, sA) + p["param7"][1] / n**2 * np.full(dA.shape, sA)
    t8 = (p["param8"][0] * sA + p["param8"][1] * sdA) / n**2 * np.eye(n, dtype=A.dtype)
    return t1 + t2 + t3 + t4 + t4p + t5 + t5p + t6 + t6p + t7 + t8


def fusion_plain(A, dA):
    """``GraphVectorField`` message matrix ``A + dA`` (graph_vector_field.py:94)."""
    return A + dA


# ----------------------------------------------------------------------------------------------
# ConvLayer / vector fields
# ----------------------------------------------------------------------------------------------


def rmsnorm(x, w, b, eps=1e-5):
    """equinox ``nn.RMSNorm(shape)`` over the feature axis: x * rsqrt(mean(x^2) + eps) * w + b."""
    inv = 1.0 / np.sqrt(np.mean(x * x, axis=-1, keepdims=True) + eps)
    return x * inv * w + b


def conv_layer(Z, Abar, layer):
    """``ConvLayer.__call__`` (layers.py:36-48): m = Linear(RMSNorm(Z)); return m + Abar @ m."""
    Zn = rmsnorm(Z, layer["rms_w"], layer["rms_b"])
    m = Zn @ layer["W"].T + layer["b"]
    return m + Abar @ m


@dataclass
class VFParams:
    """Parameters of PermEquivGraphVectorField / PermEquivDirGraphVectorField / GraphVectorField.

    kind: "undirected" | "directed" | "plain".  layers[l] is a dict with the fusion params
    (param1..param8[, *_prime], each shape (2,)) and rms_w, rms_b [d_in], W [d_out, d_in], b [d_out].
    """

    kind: str
    layers: list = field(default_factory=list)

    @property
    def dims(self):
        return [self.layers[0]["W"].shape[1]] + [lay["W"].shape[0] for lay in self.layers]


def fused_matrix(params: VFParams, l, A, dA):
    lay = params.layers[l]
    if params.kind == "undirected":
        return fusion_undirected(lay, A, dA)
    if params.kind == "directed":
        return fusion_directed(lay, A, dA)
    if params.kind == "plain":
        return fusion_plain(A, dA)
    raise ValueError(params.kind)


def vector_field(params: VFParams, t, y, control):
    """``PermEquivGraphVectorField.__call__`` (perm_equiv_graph_vector_field.py:85-129) and siblings.

    control: CubicInterpolation over [T, n, n, 2] knots (channel 0 = time, channel 1 = operator).
    """
    X = control.evaluate(t)
    dX = control.derivative(t)
    A, dA, tg = X[..., -1], dX[..., -1], dX[..., 0]
    Z = y
    L = len(params.layers)
    for l in range(L):
        Abar = fused_matrix(params, l, A, dA)
        Z = conv_layer(Z, Abar, params.layers[l])
        if l < L - 1:
            Z = np.maximum(Z, 0.0)
    tgm = np.mean(tg, axis=0)  # [n]
    return tgm[:, None] * Z


def cde_wrapper(params: VFParams, hidden_dim, data_embed_dim, t, y, control_adj, control_data):
    """``CDEWrapperVectorField.__call__`` (cde_wrapper_vector_field.py:19-26)."""
    F = vector_field(params, t, y, control_adj).reshape(-1, hidden_dim, data_embed_dim, 2)
    dX = control_data.derivative(t)  # [n, de, 2]
    return np.einsum("nmlk,nlk->nm", F, dX)


# ----------------------------------------------------------------------------------------------
# Parameter init (equinox / reference conventions; NOT bit-identical to JAX threefry — params are
# injected for parity)
# ----------------------------------------------------------------------------------------------


def init_vf_params(rng, kind, dims, fusion_scale=1.0 / 15):
    """dims = [d_0, ..., d_L].  Fusion params U(-1,1)/15 (layers.py:86-95); Linear W,b ~ U(±1/sqrt(d_in));
    RMSNorm weight ones, bias zeros (equinox defaults).  ``rng``: np.random.Generator."""
    names = {"undirected": UNDIRECTED_PARAMS, "directed": DIRECTED_PARAMS, "plain": ()}[kind]
    layers = []
    for l in range(len(dims) - 1):
        din, dout = dims[l], dims[l + 1]
        lay = {nm: fusion_scale * rng.uniform(-1, 1, size=2) for nm in names}
        lim = 1.0 / math.sqrt(din)
        lay["W"] = rng.uniform(-lim, lim, size=(dout, din))
        lay["b"] = rng.uniform(-lim, lim, size=(dout,))
        lay["rms_w"] = np.ones(din)
        lay["rms_b"] = np.zeros(din)
        layers.append(lay)
    return VFParams(kind=kind, layers=layers)


def fusion_coefficient_table(params: VFParams, n):
    """Maps reference fusion params onto the build's factored form, 24 floats/layer:

        Abar + I = eA*A + edA*dA + eTA*A^T + eTdA*dA^T + diag(u) + w 1^T + 1 v^T
        u_i = idc + uDA*A_ii + uDdA*dA_ii + uRA*r_i + uRdA*rd_i + uCA*c_i + uCdA*cd_i + uSA*s + uSdA*sd
        w_i = wRA*r_i + wRdA*rd_i + wCA*c_i + wCdA*cd_i + wSA*s + wSdA*sd
        v_k = vRA*r_k + vRdA*rd_k + vCA*c_k + vCdA*cd_k
    with r/c = row/col sums, s = total sum of A (d-suffix: of dA).  Index order = FC_* constants of
    include/gncde.h.  idc = 1 is ConvLayer's residual ``m + Abar@m`` (layers.py:47).
    """
    L = len(params.layers)
    tab = np.zeros((L, 24), dtype=np.float64)
    for l, p in enumerate(params.layers):
        t = tab[l]
        t[22] = 1.0
        if params.kind == "plain":
            t[0] = t[1] = 1.0
            continue
        t[0], t[1] = 1.0 + p["param1"][0], 1.0 + p["param1"][1]
        t[2], t[3] = p["param2"][0], p["param2"][1]
        t[4], t[5] = p["param3"][0], p["param3"][1]
        t[16] = p["param7"][0] / n**2 + p["param7"][1] / n**2
        t[10], t[11] = p["param8"][0] / n**2, p["param8"][1] / n**2
        if params.kind == "undirected":
            t[12], t[13] = p["param4"][0] / n, p["param4"][1] / n
            t[18], t[19] = p["param5"][0] / n, p["param5"][1] / n
            t[6], t[7] = p["param6"][0] / n, p["param6"][1] / n
        else:
            t[14], t[15] = p["param4"][0] / n, p["param4"][1] / n
            t[18] += p["param4_prime"][0] / n
            t[21] += p["param4_prime"][1] / n
            t[20] += p["param5"][0] / n
            t[21] += p["param5"][1] / n
            t[18] += p["param5_prime"][0] / n
            t[19] += p["param5_prime"][1] / n
            t[8], t[9] = p["param6"][0] / n, p["param6"][1] / n
            t[6], t[7] = p["param6_prime"][0] / n, p["param6_prime"][1] / n
    return tab


def factored_matrix(tab_row, A, dA):
    """Materialise Abar + I from one row of the coefficient table (used to check the mapping)."""
    t = tab_row
    r, rd, c, cd = A.sum(1), dA.sum(1), A.sum(0), dA.sum(0)
    s, sd = A.sum(), dA.sum()
    u = (t[22] + t[4] * np.diag(A) + t[5] * np.diag(dA) + t[6] * r + t[7] * rd + t[8] * c + t[9] * cd
         + t[10] * s + t[11] * sd)
    w = t[12] * r + t[13] * rd + t[14] * c + t[15] * cd + t[16] * s + t[17] * sd
    v = t[18] * r + t[19] * rd + t[20] * c + t[21] * cd
    return (t[0] * A + t[1] * dA + t[2] * A.T + t[3] * dA.T + np.diag(u) + w[:, None] + v[None, :])


# ----------------------------------------------------------------------------------------------
# Solvers (diffrax restated; RK4 = build extension for BASELINE config 2)
# ----------------------------------------------------------------------------------------------

TSIT5_C = np.array([0.0, 0.161, 0.327, 0.9, 0.9800255409045097, 1.0, 1.0])
TSIT5_A = [
    [],
    [0.161],
    [-0.008480655492356989, 0.335480655492357],
    [2.897153057105493, -6.359448489975075, 4.3622954328695815],
    [5.325864828439257, -11.748883564062828, 7.4955393428898365, -0.09249506636175525],
    [5.86145544294642, -12.92096931784711, 8.159367898576159, -0.071584973281401, -0.028269050394068383],
    [0.09646076681806523, 0.01, 0.4798896504144996, 1.379008574103742, -3.290069515436081, 2.324710524099774],
]
TSIT5_B = np.array(TSIT5_A[6] + [0.0])
# b - b_hat (Tsitouras 2011; global sign irrelevant under the RMS norm)
TSIT5_BERR = np.array([0.001780011052226, 0.000816434459657, -0.007880878010262, 0.144711007173263,
                       -0.582357165452555, 0.458082105929187, -1.0 / 66.0])


def tsit5_dense_weights(theta):
    """Tsit5 free interpolant b_i(theta): y(t0 + theta*dt) = y0 + sum_i b_i(theta) k_i (k_i increments)."""
    th = theta
    b1 = -1.0530884977290216 * th * (th - 1.3299890189751412) * (th * th - 1.4364028541716351 * th
                                                                   + 0.7139816917074209)
    b2 = 0.1017 * th * th * (th * th - 2.1966568338249754 * th + 1.2949852507374631)
    b3 = 2.490627285651252793 * th * th * (th * th - 2.38535645472061657 * th + 1.57803468208092486)
    b4 = -16.54810288924490272 * (th - 1.21712927295533244) * (th - 0.61620406037800089) * th * th
    b5 = 47.37952196281928122 * (th - 1.203071208372362603) * (th - 0.658047292653547382) * th * th
    b6 = -34.87065786149660974 * (th - 1.2) * (th - 0.666666666666666667) * th * th
    b7 = 2.5 * (th - 1.0) * (th - 0.6) * th * th
    return np.array([b1, b2, b3, b4, b5, b6, b7])


def rms(x):
    x = np.asarray(x)
    return float(np.sqrt(np.mean(x * x)))


def rk4_grid(t0, t1, nsteps, dtype=np.float32):
    """Build extension: t_k = t0 + k*(t1-t0)/nsteps in fp32, last knot exactly t1."""
    t0, t1 = dtype(t0), dtype(t1)
    h = dtype((t1 - t0) / dtype(nsteps))
    g = np.array([dtype(t0 + dtype(k) * h) for k in range(nsteps + 1)], dtype=dtype)
    g[-1] = t1
    return g


def constant_grid(t0, t1, dt0, dtype=np.float32, tol=1e-6):
    """diffrax ConstantStepSize grid: t_{k+1} = t_k + dt0 (fp32), clipped to t1; a step ending within
    ``tol`` of t1 snaps to t1 (diffrax ``_clip_to_end``)."""
    t0, t1, dt0 = dtype(t0), dtype(t1), dtype(dt0)
    g = [t0]
    t = t0
    while t < t1:
        tn = dtype(t + dt0)
        if tn > dtype(t1 - dtype(tol)):
            tn = t1
        g.append(tn)
        t = tn
    return np.array(g, dtype=dtype)


def _stage_times(t, h, cs, time_dtype):
    """Stage times t + c*h.  With time_dtype=np.float32 they are formed exactly as the GPU kernels do
    (fl(t + fl(c*h)), c=1 -> fl(t + h)) so both sides evaluate the spline at bit-identical times."""
    if time_dtype is None:
        return [t + c * h for c in cs]
    f32 = np.float32
    t32, h32 = f32(t), f32(h)
    out = []
    for c in cs:
        if c == 0.0:
            out.append(float(t32))
        elif c == 1.0:
            out.append(float(f32(t32 + h32)))
        else:
            out.append(float(f32(t32 + f32(f32(c) * h32))))
    return out


def rk4_step(f, t, y, h, time_dtype=None):
    t1, tm, _, te = _stage_times(t, h, [0.0, 0.5, 0.5, 1.0], time_dtype)
    k1 = f(t1, y)
    k2 = f(tm, y + (0.5 * h) * k1)
    k3 = f(tm, y + (0.5 * h) * k2)
    k4 = f(te, y + h * k3)
    return y + (h / 6.0) * (k1 + 2.0 * k2 + 2.0 * k3 + k4)


def solve_fixed_grid(f, grid, y0, method="rk4", save_every_step=False, time_dtype=None):
    """Fixed-grid solve (RK4 or Tsit5 with ConstantStepSize, FSAL).  Returns (final state or all step
    states, number of vector-field evaluations)."""
    y = np.array(y0, dtype=np.float64)
    ys = [y.copy()]
    nevals = 0
    fk = None
    for k in range(len(grid) - 1):
        if time_dtype is None:
            t, h = float(grid[k]), float(grid[k + 1]) - float(grid[k])
        else:
            t = float(time_dtype(grid[k]))
            h = float(time_dtype(time_dtype(grid[k + 1]) - time_dtype(grid[k])))
        if method == "rk4":
            y = rk4_step(f, t, y, h, time_dtype)
            nevals += 4
        elif method == "tsit5":
            if fk is None:
                fk = f(t, y)
                nevals += 1
            t_end = float(grid[k + 1]) if time_dtype is None else float(time_dtype(grid[k + 1]))
            y, _, ks = tsit5_step(f, t, y, h, k1=h * fk, time_dtype=time_dtype, t_end=t_end)
            fk = ks[6] / h if h != 0 else f(t + h, y)
            nevals += 6
        else:
            raise ValueError(method)
        ys.append(y.copy())
    return (np.stack(ys) if save_every_step else y), nevals


def tsit5_step(f, t, y, h, k1=None, time_dtype=None, t_end=None):
    """One Tsit5 step.  Returns (y1, y_err, ks) with ks the 7 increments (dt * f); ks[6] = h f(t_end, y1): the FSAL
    stage is evaluated at the step's end time t_end (the grid knot / the controller's t + dt; t + h if not given),
    where it is reused as the next step's first stage."""
    tst = _stage_times(t, h, list(TSIT5_C), time_dtype)
    if t_end is not None:
        tst[6] = float(t_end)
    ks = []
    if k1 is None:
        k1 = h * f(tst[0], y)
    ks.append(k1)
    for i in range(1, 7):
        yi = y + sum(TSIT5_A[i][j] * ks[j] for j in range(i))
        ks.append(h * f(tst[i], yi))
    y1 = y + sum(TSIT5_B[j] * ks[j] for j in range(6))
    yerr = sum(TSIT5_BERR[j] * ks[j] for j in range(7))
    return y1, yerr, ks


def select_initial_step(f, t0, y0, rtol, atol, error_order=5.0):
    """diffrax ``_select_initial_step`` (Hairer): 2 vector-field evaluations."""
    f0 = f(t0, y0)
    scale = atol + np.abs(y0) * rtol
    d0 = rms(y0 / scale)
    d1 = rms(f0 / scale)
    if d0 < 1e-5 or d1 < 1e-5:
        h0 = 1e-6
    else:
        h0 = 0.01 * (d0 / d1)
    y1 = y0 + h0 * f0
    f1 = f(t0 + h0, y1)
    d2 = rms((f1 - f0) / scale) / h0
    max_d = max(d1, d2)
    if max_d <= 1e-15:
        h1 = max(1e-6, h0 * 1e-3)
    else:
        h1 = (0.01 / max_d) ** (1.0 / error_order)
    return min(100.0 * h0, h1)


def solve_tsit5_pid(f, t0, t1, y0, rtol=1e-3, atol=1e-6, dt0=None, save_ts=None, max_steps=4096,
                    safety=0.9, factormin=0.2, factormax=10.0, error_order=5.0):
    """Tsit5 + PIDController(rtol, atol) with diffrax defaults (pcoeff=0, icoeff=1, dcoeff=0), FSAL,
    SaveAt(ts) via the Tsit5 dense interpolant (SaveAt(t1) if save_ts is None).

    Returns (ys, stats) with stats = dict(steps, rejects, evals, grid): grid = the accepted step times
    (t0 first), the sequence the reverse mode differentiates on.
    """
    evals = 0
    y = np.array(y0, dtype=np.float64)
    t = float(t0)
    if dt0 is None:
        dt = select_initial_step(f, t, y, rtol, atol, error_order)
        evals += 2
    else:
        dt = float(dt0)
    out = []
    si = 0
    if save_ts is not None:
        save_ts = np.asarray(save_ts, dtype=np.float64)
        while si < len(save_ts) and save_ts[si] <= t:
            out.append(y.copy())
            si += 1
    fk = f(t, y)
    evals += 1
    steps = rejects = 0
    grid = [t]
    while t < t1:
        if steps + rejects >= max_steps:
            raise RuntimeError("max_steps exceeded")
        tn = t + dt
        if tn > t1 - 1e-6:
            tn = float(t1)
        h = tn - t
        y1, yerr, ks = tsit5_step(f, t, y, h, k1=h * fk, t_end=tn)
        evals += 6
        scale = atol + rtol * np.maximum(np.abs(y), np.abs(y1))
        err = rms(yerr / scale)
        keep = err < 1.0 and np.isfinite(err)
        if not np.isfinite(err):
            factor = factormin
        else:
            inv = np.inf if err == 0 else 1.0 / err
            fmin = 1.0 if keep else factormin
            factor = min(max(safety * inv ** (1.0 / error_order), fmin), factormax)
        if keep:
            if save_ts is not None:
                while si < len(save_ts) and save_ts[si] <= tn:
                    theta = (save_ts[si] - t) / h
                    bw = tsit5_dense_weights(theta)
                    out.append(y + sum(bw[j] * ks[j] for j in range(7)))
                    si += 1
            y = y1
            fk = ks[6] / h  # FSAL: stage 7 is f(t1, y1)
            t = tn
            grid.append(t)
            steps += 1
        else:
            rejects += 1
        dt = factor * h
    stats = dict(steps=steps, rejects=rejects, evals=evals, grid=np.array(grid))
    if save_ts is None:
        return y, stats
    return np.stack(out), stats


# ----------------------------------------------------------------------------------------------
# Graph operators (src/dataset/misc.py:58-113) — pinned by test/dataset/test_misc.py:43-58
# ----------------------------------------------------------------------------------------------


def normalized_laplacian(A):
    A = np.asarray(A, dtype=np.float64) + np.eye(A.shape[0])
    dout = A.sum(1).astype(np.float32)
    din = A.sum(0).astype(np.float32)
    return np.eye(A.shape[0]) - np.diag(np.power(dout, -0.5)) @ A @ np.diag(np.power(din, -0.5))


def normalized_adj(A):
    A = np.asarray(A, dtype=np.float64) + np.eye(A.shape[0])
    dout = A.sum(1).astype(np.float32)
    din = A.sum(0).astype(np.float32)
    return np.diag(np.power(dout, -0.5)) @ A @ np.diag(np.power(din, -0.5))


def zipf_smoothing(A):
    """misc.py:16-33: D^-1/2 (A+I) D^-1/2 with degrees of A+I."""
    return normalized_adj(A)


def normalized_plus(A):
    """misc.py:36-57: D^-1/2 (A+I) D^-1/2 with degrees of A (no self-loop in the degrees)."""
    A = np.asarray(A, dtype=np.float64)
    dout = A.sum(1).astype(np.float32)
    din = A.sum(0).astype(np.float32)
    with np.errstate(divide="ignore"):
        so = np.where(dout != 0, np.power(dout, -0.5), 0.0)
        si = np.where(din != 0, np.power(din, -0.5), 0.0)
    return np.diag(so) @ (A + np.eye(A.shape[0])) @ np.diag(si)


# ----------------------------------------------------------------------------------------------
# Synthetic problem builder (same layout as the reference's coeffs: (d,c,b,a) each [T-1, n, n, 2])
# ----------------------------------------------------------------------------------------------


def make_graph_control(rng, n, T, t0=0.0, t1=5.0, irregular=True, dynamic=True):
    """Knots X[T,n,n,2] = stack([t broadcast, operator(t)]) like ``get_graph_interpolation_coeffs``
    (dataset_configs.py:147-173), with a randomly perturbed norm-Laplacian operator path."""
    if irregular:
        inner = np.sort(rng.uniform(t0, t1, size=T - 2))
        ts = np.concatenate([[t0], inner, [t1]])
    else:
        ts = np.linspace(t0, t1, T)
    ts = ts.astype(np.float32).astype(np.float64)
    base = (rng.uniform(size=(n, n)) < 0.15).astype(np.float64)
    ops = []
    for k in range(T):
        Ak = base.copy()
        if dynamic:
            flip = rng.uniform(size=(n, n)) < 0.02
            Ak = np.where(flip, 1.0 - Ak, Ak)
        ops.append(normalized_laplacian(Ak))
    ops = np.stack(ops)
    X = np.stack([np.broadcast_to(ts[:, None, None], ops.shape), ops], axis=-1)
    return ts, X
