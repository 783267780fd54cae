"""CPU oracle for the reverse mode of the GNCDE hot path — TEST INFRASTRUCTURE ONLY.

Only ``tests/`` (and the golden-fixture generator) may import this module, as the checker.

What it is
    A hand-written numpy (float64) reverse mode of ``oracle.gncde_oracle``'s forward, i.e. of what
    ``jax.value_and_grad`` computes for the reference's training step (``src/train/trainer.py:315``):

    * the vector field's VJP — ConvLayer (layers.py:36-48: RMSNorm -> Linear -> m + Abar m), the ReLU
      between layers (perm_equiv_graph_vector_field.py:117-121), the time-channel scaling (:127) and the
      CDE wrapper contraction (cde_wrapper_vector_field.py:19-26).  The fusion matrices are used in their
      LITERAL reference form (oracle.fusion_undirected/directed/plain, quirks included): each fusion
      parameter's gradient is <dL/dAbar, dAbar/dparam>, with dAbar/dparam obtained by evaluating the
      literal fusion with a unit parameter (the fusion is affine in its parameters).
    * the discrete adjoint of the fixed-grid RK4 / Tsit5 solve — what diffrax's default
      RecursiveCheckpointAdjoint differentiates (graph_neural_cde.py:94-104, pgt_graph_neural_cde.py:119-129).
    * the adaptive Tsit5 + PIDController solve with SaveAt(ts) (graph_neural_cde.py:53-54,89-104) differentiated
      on its accepted step sequence with the step sizes held constant (solve_grid_dense_vjp): the Tsit5 steps
      of that grid plus the reverse mode of the dense interpolant at the save times.

PARITY: jax is not installed, so this cannot be compared with jax.grad itself.  It is pinned instead by
central finite differences of the fp64 forward oracle (tests/test_oracle_grad.py), which checks the
restatement independently of how it was derived.
"""
from __future__ import annotations

import numpy as np

from . import gncde_oracle as O

FUSION_NAMES = {"undirected": O.UNDIRECTED_PARAMS, "directed": O.DIRECTED_PARAMS, "plain": ()}


def _fusion_basis(kind, lay, A, dA):
    """{(name, j): dAbar/dparam[name][j]} for the literal fusion of ``kind`` (affine in the params)."""
    names = FUSION_NAMES[kind]
    if not names:
        return {}
    zero = {nm: np.zeros(2) for nm in names}
    f = O.fusion_undirected if kind == "undirected" else O.fusion_directed
    base = f(zero, A, dA)
    out = {}
    for nm in names:
        for j in range(2):
            p = {k: v.copy() for k, v in zero.items()}
            p[nm][j] = 1.0
            out[(nm, j)] = f(p, A, dA) - base
    return out


def _control(control, t):
    X = control.evaluate(t)
    dX = control.derivative(t)
    return X[..., -1], dX[..., -1], dX[..., 0]


def vector_field_vjp(params: O.VFParams, t, y, control, g):
    """(g_y, grads) for out = vector_field(params, t, y, control) and cotangent g [n, d_L].

    grads[l] is a dict with the same keys as params.layers[l] (fusion params, W, b, rms_w, rms_b).
    """
    A, dA, tg = _control(control, t)
    tgm = np.mean(tg, axis=0)
    L = len(params.layers)
    # forward tape
    tape = []
    Z = np.asarray(y, np.float64)
    for l in range(L):
        lay = params.layers[l]
        Abar = O.fused_matrix(params, l, A, dA)
        inv = 1.0 / np.sqrt(np.mean(Z * Z, axis=-1, keepdims=True) + 1e-5)
        xh = Z * inv
        zn = xh * lay["rms_w"] + lay["rms_b"]
        m = zn @ lay["W"].T + lay["b"]
        pre = m + Abar @ m
        tape.append((Z, inv, xh, zn, m, Abar, pre))
        Z = np.maximum(pre, 0.0) if l < L - 1 else pre
    # backward
    gZ = tgm[:, None] * np.asarray(g, np.float64)
    grads = [None] * L
    for l in range(L - 1, -1, -1):
        lay = params.layers[l]
        Zin, inv, xh, zn, m, Abar, pre = tape[l]
        gpre = gZ * (pre > 0) if l < L - 1 else gZ
        gAbar = gpre @ m.T
        gm = gpre + Abar.T @ gpre
        gr = {"b": gm.sum(axis=0), "W": gm.T @ zn}
        gzn = gm @ lay["W"]
        gr["rms_w"] = (gzn * xh).sum(axis=0)
        gr["rms_b"] = gzn.sum(axis=0)
        gxh = gzn * lay["rms_w"]
        d = Zin.shape[-1]
        gZ = inv * (gxh - xh * np.sum(gxh * xh, axis=-1, keepdims=True) / d)
        for (nm, j), basis in _fusion_basis(params.kind, lay, A, dA).items():
            gr.setdefault(nm, np.zeros(2))[j] = float(np.sum(gAbar * basis))
        grads[l] = gr
    return gZ, grads


def cde_wrapper_vjp(params: O.VFParams, hidden_dim, data_embed_dim, t, y, control_adj, control_data, g,
                    data_grad=False):
    """VJP of oracle.cde_wrapper: out[n,m] = sum_lk F[n,m,l,k] dX[n,l,k].

    With ``data_grad`` the per-layer grads list gets one more entry, {"data_coef": [4, T-1, n, de, 2]}: the
    cotangent of the data spline's (d, c, b, a) coefficients (dX = b + f (2c + 3f d) at the stage interval,
    so the 'a' row stays zero).  It accumulates over stages like the parameter gradients."""
    dX = control_data.derivative(t)
    g = np.asarray(g, np.float64)
    gF = np.einsum("nm,nlk->nmlk", g, dX).reshape(g.shape[0], -1)
    gy, grads = vector_field_vjp(params, t, y, control_adj, gF)
    if not data_grad:
        return gy, grads
    F = O.vector_field(params, t, y, control_adj).reshape(-1, hidden_dim, data_embed_dim, 2)
    gdX = np.einsum("nm,nmlk->nlk", g, F)
    ts = np.asarray(control_data.ts)
    i = O.interval_index(ts, t)
    f = t - ts[i]
    gco = np.zeros((4, len(ts) - 1) + gdX.shape)
    gco[0, i] = 3.0 * f * f * gdX
    gco[1, i] = 2.0 * f * gdX
    gco[2, i] = gdX
    return gy, list(grads) + [{"data_coef": gco}]


def hermite_jacobian(ts):
    """J[q, i, j] = d coef_q(interval i) / d X[j] of backward_hermite_coefficients over knots ts (the map is
    linear in X and acts on every channel alike), evaluated column by column on unit knot vectors."""
    T = len(ts)
    J = np.zeros((4, T - 1, T))
    for j in range(T):
        e = np.zeros((T, 1))
        e[j, 0] = 1.0
        co = O.backward_hermite_coefficients(np.asarray(ts, np.float64), e)
        for q in range(4):
            J[q, :, j] = co[q][:, 0]
    return J


def hermite_vjp(ts, gco):
    """Cotangent of the knot values X [T, ...] from the coefficients' cotangent gco [4, T-1, ...]."""
    J = hermite_jacobian(ts)
    return np.einsum("qij,qi...->j...", J, np.asarray(gco, np.float64))


def _tableau(method):
    if method == "rk4":
        return [0.0, 0.5, 0.5, 1.0], [[], [0.5], [0.0, 0.5], [0.0, 0.0, 1.0]], [1 / 6, 2 / 6, 2 / 6, 1 / 6]
    if method == "tsit5":
        return list(O.TSIT5_C[:6]), [list(r) for r in O.TSIT5_A[:6]], list(O.TSIT5_B[:6])
    raise ValueError(method)


def _acc(total, grads):
    if total is None:
        return [{k: np.array(v, np.float64) for k, v in g.items()} for g in grads]
    for tl, gl in zip(total, grads):
        for k, v in gl.items():
            tl[k] = tl[k] + v
    return total


def solve_fixed_grid_vjp(f, f_vjp, grid, y0, method="rk4", g_final=None, g_steps=None, time_dtype=np.float32,
                         y_lin=None):
    """Reverse mode of oracle.solve_fixed_grid (same stage times, same grid).

    f(t, y) -> dy; f_vjp(t, y, g) -> (g_y, grads).  Cotangent of the final state ``g_final`` [n, d] or of
    every saved step state ``g_steps`` [G, n, d].  Returns (g_y0, summed parameter grads).
    ``y_lin`` [G, n, d]: step states to linearise at instead of this function's own fp64 forward (e.g. the GPU's
    fp32 trajectory, so that both adjoints see the same side of every ReLU kink; the stage inputs are re-formed
    from them in fp64).
    """
    cs, a, b = _tableau(method)
    y = np.asarray(y0, np.float64)
    ys = [y]
    G = len(grid)
    geo = []
    for k in range(G - 1):
        if time_dtype is None:
            t, h = float(grid[k]), float(grid[k + 1]) - float(grid[k])
        else:
            t = float(time_dtype(grid[k]))
            h = float(time_dtype(time_dtype(grid[k + 1]) - time_dtype(grid[k])))
        geo.append((t, h))
        if method == "rk4":
            y = O.rk4_step(f, t, y, h, time_dtype)
        else:
            y, _, _ = O.tsit5_step(f, t, y, h, time_dtype=time_dtype)
        ys.append(y)
    if y_lin is not None:
        ys = [np.asarray(v, np.float64) for v in y_lin]
    lam = np.array(g_steps[-1] if g_steps is not None else g_final, np.float64)
    total = None
    S = len(cs)
    for k in range(G - 2, -1, -1):
        t, h = geo[k]
        tst = O._stage_times(t, h, cs, time_dtype)
        yk = ys[k]
        U, K = [], []
        for i in range(S):
            u = yk + h * sum((a[i][j] * K[j] for j in range(i)), np.zeros_like(yk))
            U.append(u)
            K.append(f(tst[i], u))
        gK = [h * b[i] * lam for i in range(S)]
        gy = lam.copy()
        for i in range(S - 1, -1, -1):
            gu, gr = f_vjp(tst[i], U[i], gK[i])
            total = _acc(total, gr)
            gy = gy + gu
            for j in range(i):
                if a[i][j] != 0.0:
                    gK[j] = gK[j] + h * a[i][j] * gu
        lam = gy + (g_steps[k] if g_steps is not None else 0.0)
    return lam, total


def _locate(grid, ts):
    """(k, theta) of a save time: t_k < ts <= t_{k+1} (k = -1: ts <= t0, the initial state)."""
    if ts <= grid[0]:
        return -1, 0.0
    k = int(np.searchsorted(grid, ts, side="left")) - 1
    k = min(max(k, 0), len(grid) - 2)
    return k, (ts - grid[k]) / (grid[k + 1] - grid[k])


def _grid_geometry(grid, time_dtype):
    geo = []
    for k in range(len(grid) - 1):
        if time_dtype is None:
            geo.append((float(grid[k]), float(grid[k + 1]) - float(grid[k])))
        else:
            t = float(time_dtype(grid[k]))
            geo.append((t, float(time_dtype(time_dtype(grid[k + 1]) - time_dtype(grid[k])))))
    return geo


def _tsit5_stages(f, t, h, y, time_dtype, t_end=None):
    """The 7 stage inputs / values of a Tsit5 step (stage 7: f(t_end, y1), the step's end knot) and y1."""
    tst = O._stage_times(t, h, list(O.TSIT5_C), time_dtype)
    if t_end is not None:
        tst[6] = float(t_end)
    U, K = [], []
    for i in range(7):
        if i < 6:
            u = y + h * sum((O.TSIT5_A[i][j] * K[j] for j in range(i)), np.zeros_like(y))
        else:
            u = y + h * sum(O.TSIT5_B[j] * K[j] for j in range(6))
        U.append(u)
        K.append(f(tst[i], u))
    return tst, U, K


def _end_knots(grid, time_dtype):
    """Each step's end knot as the kernels see it (the FSAL stage's time)."""
    return [float(grid[k + 1]) if time_dtype is None else float(time_dtype(grid[k + 1])) for k in range(len(grid) - 1)]


def solve_grid_dense(f, grid, y0, save_ts, time_dtype=np.float32):
    """Tsit5 on the accepted step sequence ``grid`` with SaveAt(ts) through the dense interpolant: what an adaptive
    solve outputs once its steps are fixed.  Returns [S, n, d]."""
    y = np.asarray(y0, np.float64)
    geo = _grid_geometry(grid, time_dtype)
    ys, stages = [y], []
    for (t, h), te in zip(geo, _end_knots(grid, time_dtype)):
        _, _, K = _tsit5_stages(f, t, h, ys[-1], time_dtype, te)
        stages.append(K)
        ys.append(ys[-1] + h * sum(O.TSIT5_B[j] * K[j] for j in range(6)))
    out = []
    for ts in save_ts:
        k, th = _locate(np.asarray(grid, np.float64), float(ts))
        if k < 0:
            out.append(ys[0])
            continue
        w = O.tsit5_dense_weights(th)
        out.append(ys[k] + geo[k][1] * sum(w[j] * stages[k][j] for j in range(7)))
    return np.stack(out)


def solve_grid_dense_vjp(f, f_vjp, grid, y0, save_ts, g_saves, time_dtype=np.float32):
    """Reverse mode of solve_grid_dense for cotangents g_saves [S, n, d]: (g_y0, summed parameter grads).

    Per save point s in step k: y(ts) = y_k + h_k sum_j b_j(th) K_j, j = 0..6, K_6 = f(t_{k+1}, y_{k+1}).  Going
    backwards over the steps, the cotangent of K_6 of step k is pulled back through f onto y_{k+1} first; then the
    usual Tsit5 adjoint of step k runs with stage seeds h_k (b_j lambda_{k+1} + sum_s b_j(th_s) g_s)."""
    y = np.asarray(y0, np.float64)
    geo = _grid_geometry(grid, time_dtype)
    gridd = np.asarray(grid, np.float64)
    ys = [y]
    tend = _end_knots(grid, time_dtype)
    for (t, h), te in zip(geo, tend):
        _, _, K = _tsit5_stages(f, t, h, ys[-1], time_dtype, te)
        ys.append(ys[-1] + h * sum(O.TSIT5_B[j] * K[j] for j in range(6)))
    N = len(geo)
    dense = [np.zeros((7,) + y.shape) for _ in range(N)]   # sum_s b_j(th_s) g_s per step
    direct = [np.zeros_like(y) for _ in range(N + 1)]      # cotangent straight onto y_k
    for ts, g in zip(save_ts, g_saves):
        k, th = _locate(gridd, float(ts))
        if k < 0:
            direct[0] = direct[0] + g
            continue
        direct[k] = direct[k] + g
        dense[k] = dense[k] + O.tsit5_dense_weights(th)[:, None, None] * g
    lam = direct[N].copy()
    total = None
    b = list(O.TSIT5_B[:6])
    for k in range(N - 1, -1, -1):
        t, h = geo[k]
        tst, U, _ = _tsit5_stages(f, t, h, ys[k], time_dtype, tend[k])
        if np.any(dense[k][6]):  # K_6 = f(t_{k+1}, y_{k+1})
            gu, gr = f_vjp(tst[6], U[6], h * dense[k][6])
            total = _acc(total, gr)
            lam = lam + gu
        gK = [h * (b[i] * lam + dense[k][i]) for i in range(6)]
        gy = lam + direct[k]
        for i in range(5, -1, -1):
            gu, gr = f_vjp(tst[i], U[i], gK[i])
            total = _acc(total, gr)
            gy = gy + gu
            for j in range(i):
                if O.TSIT5_A[i][j] != 0.0:
                    gK[j] = gK[j] + h * O.TSIT5_A[i][j] * gu
        lam = gy
    return lam, total


def grads_to_vector(grads, kind):
    """Flatten per-layer grads in a fixed order (for comparisons): fusion params then rms_w, rms_b, W, b."""
    out = []
    for g in grads:
        for nm in FUSION_NAMES[kind]:
            out.append(np.asarray(g[nm]).ravel())
        for nm in ("rms_w", "rms_b", "W", "b"):
            out.append(np.asarray(g[nm]).ravel())
    return np.concatenate(out)


def params_to_vector(params: O.VFParams):
    return grads_to_vector(params.layers, params.kind)


def vector_to_params(vec, like: O.VFParams) -> O.VFParams:
    layers, off = [], 0
    for lay in like.layers:
        new = {}
        for nm in list(FUSION_NAMES[like.kind]) + ["rms_w", "rms_b", "W", "b"]:
            shape = np.asarray(lay[nm]).shape
            size = int(np.prod(shape))
            new[nm] = np.asarray(vec[off:off + size]).reshape(shape)
            off += size
        layers.append(new)
    return O.VFParams(kind=like.kind, layers=layers)
