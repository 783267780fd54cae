"""Host-side packing into the engine's HBM layout (include/gncde.h).

* control path:  the reference's ``diffrax.backward_hermite_coefficients`` tuple (d, c, b, a), each
  ``[B, T-1, n, n, 2]`` (channel 0 = time, 1 = operator; dataset_configs.py:147-173) becomes
  ``coef [B, T-1, 4, n, n]`` (operator channel, same (d,c,b,a) order) and ``tcoef [B, T-1, 3, n]``
  (column means of the time channel's d, c, b — the VF's ``jnp.mean(derivative(t)[..., 0], axis=0)``,
  perm_equiv_graph_vector_field.py:101,127, is linear in the coefficients).
* parameters:    per layer ``rms_w[d_l], rms_b[d_l], W[d_{l+1}, d_l], b[d_{l+1}]`` back to back.
* fusion table:  the reference's ``param1..param8`` (+ ``*_prime``) mapped to the factored form
  ``(I + Abar) = eA A + edA dA + eTA A^T + eTdA dA^T + diag(u) + w 1^T + 1 v^T`` (24 columns, gncde.h).
* step grids:    fp32 grids for fixed-step solvers, computed with exactly the fp32 arithmetic the
  reference's ConstantStepSize loop performs (diffrax ``_clip_to_end`` 1e-6 snap).
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib

FC = _lib.FC

# column indices (gncde.h GNCDE_FC_*)
E_A, E_DA, ET_A, ET_DA = 0, 1, 2, 3
UD_A, UD_DA, UR_A, UR_DA, UC_A, UC_DA, US_A, US_DA = 4, 5, 6, 7, 8, 9, 10, 11
WR_A, WR_DA, WC_A, WC_DA, WS_A, WS_DA = 12, 13, 14, 15, 16, 17
VR_A, VR_DA, VC_A, VC_DA = 18, 19, 20, 21
IDC = 22


def pack_control(coeffs, ts=None, device="cuda"):
    """(d, c, b, a) each [B, T-1, n, n, 2] (torch or numpy) -> (coef [B,T-1,4,n,n], tcoef [B,T-1,3,n]).

    A single-sample tuple ([T-1, n, n, 2]) is promoted to B = 1.
    """
    parts = [torch.as_tensor(np.asarray(x) if not torch.is_tensor(x) else x) for x in coeffs]
    if parts[0].dim() == 4:
        parts = [p.unsqueeze(0) for p in parts]
    parts = [p.to(device=device, dtype=torch.float32) for p in parts]
    d, c, b, a = parts
    coef = torch.stack([d[..., 1], c[..., 1], b[..., 1], a[..., 1]], dim=2).contiguous()
    # column means over rows (axis 0 of each [n, n] time-channel matrix)
    tcoef = torch.stack([d[..., 0].mean(dim=-2), c[..., 0].mean(dim=-2), b[..., 0].mean(dim=-2)],
                        dim=2).contiguous()
    return coef, tcoef


def control_from_knots(ts, X_op, X_time=None):
    """Engine control layout straight from knot values on the GPU (gncde_hermite_coefficients):
    X_op [B, T, n, n] operator path -> coef [B, T-1, 4, n, n]; the time channel X_time [B, T, n, n] (default:
    ts broadcast, the reference's stacking at dataset_configs.py:168-170) -> tcoef [B, T-1, 3, n] (coefficients
    of its column means; for X_time = ts that is d = c = 0, b = 1)."""
    from . import engine
    ts = torch.as_tensor(ts, dtype=torch.float32, device="cuda")
    if ts.dim() == 1:
        ts = ts.unsqueeze(0)
    coef = engine.hermite_coefficients(ts, X_op, 4)
    B, T, n = int(X_op.shape[0]), int(X_op.shape[1]), int(X_op.shape[-1])
    if X_time is None:
        tcoef = torch.zeros(B, T - 1, 3, n, device=coef.device)
        tcoef[:, :, 2] = 1.0
    else:
        # coefficients first, column means second (as the reference's VF does): the mean of the knots first
        # would round and the cubic term of a short interval would amplify that (d ~ 1/dt^2)
        tcoef = engine.hermite_coefficients(ts, torch.as_tensor(X_time, device="cuda"), 3).mean(dim=-2)
    return coef, tcoef


def pack_data_control(coeffs, device="cuda"):
    """CDE data spline (d, c, b, a) each [B, T-1, n, de, 2] -> [B, T-1, 4, n, de, 2]."""
    parts = [torch.as_tensor(np.asarray(x) if not torch.is_tensor(x) else x) for x in coeffs]
    if parts[0].dim() == 4:
        parts = [p.unsqueeze(0) for p in parts]
    return torch.stack([p.to(device=device, dtype=torch.float32) for p in parts], dim=2).contiguous()


FUSION_PARAM_NAMES = {
    "undirected": ("param1", "param2", "param3", "param4", "param5", "param6", "param7", "param8"),
    "directed": ("param1", "param2", "param3", "param4", "param4_prime", "param5", "param5_prime", "param6",
                 "param6_prime", "param7", "param8"),
    "plain": (),
}


def fusion_map(kind: str, n: int):
    """The (linear) map from one layer's reference fusion parameters to its factored-table row:

        row = base + concat(param_a, param_b, ...) @ M        (names in FUSION_PARAM_NAMES[kind] order)

    kind "undirected": ConvEquivFusionLayer._fusion (layers.py:102-160)
    kind "directed":   ConvEquivFusionDirectedLayer._fusion (layers.py:256-337)
    kind "plain":      GraphVectorField message matrix A + dA (graph_vector_field.py:94)
    Returns (names, base [24] float64, M [2*len(names), 24] float64).
    """
    if kind not in FUSION_PARAM_NAMES:
        raise ValueError(kind)
    names = FUSION_PARAM_NAMES[kind]
    base = torch.zeros(FC, dtype=torch.float64)
    base[IDC] = 1.0  # ConvLayer residual: m + Abar @ m (layers.py:47)
    base[E_A] = base[E_DA] = 1.0  # plain: A + dA; fusion kinds: term_1 = (1 + param1) * (A, dA)
    M = torch.zeros(2 * len(names), FC, dtype=torch.float64)

    def put(name, j, col, coef):
        M[2 * names.index(name) + j, col] += coef

    if kind == "plain":
        return names, base, M
    put("param1", 0, E_A, 1.0), put("param1", 1, E_DA, 1.0)  # term_1
    put("param2", 0, ET_A, 1.0), put("param2", 1, ET_DA, 1.0)  # term_2 transpose
    put("param3", 0, UD_A, 1.0), put("param3", 1, UD_DA, 1.0)  # term_3 diag(diag)
    # term_7: both halves multiply sum(adjacency) (layers.py:144-148)
    put("param7", 0, WS_A, 1.0 / n**2), put("param7", 1, WS_A, 1.0 / n**2)
    put("param8", 0, US_A, 1.0 / n**2), put("param8", 1, US_DA, 1.0 / n**2)  # term_8
    if kind == "undirected":
        put("param4", 0, WR_A, 1.0 / n), put("param4", 1, WR_DA, 1.0 / n)  # row sums -> rows
        put("param5", 0, VR_A, 1.0 / n), put("param5", 1, VR_DA, 1.0 / n)  # row sums -> cols
        put("param6", 0, UR_A, 1.0 / n), put("param6", 1, UR_DA, 1.0 / n)  # diag(row sums)
    else:
        put("param4", 0, WC_A, 1.0 / n), put("param4", 1, WC_DA, 1.0 / n)  # col sums -> rows
        put("param4_prime", 0, VR_A, 1.0 / n)  # tile(rowsum A)
        put("param4_prime", 1, VC_DA, 1.0 / n)  # tile(colsum dA)  (quirk :288-293)
        put("param5", 0, VC_A, 1.0 / n), put("param5", 1, VC_DA, 1.0 / n)
        put("param5_prime", 0, VR_A, 1.0 / n), put("param5_prime", 1, VR_DA, 1.0 / n)
        put("param6", 0, UC_A, 1.0 / n), put("param6", 1, UC_DA, 1.0 / n)
        put("param6_prime", 0, UR_A, 1.0 / n), put("param6_prime", 1, UR_DA, 1.0 / n)
    return names, base, M


def fusion_table(kind: str, layers, n: int) -> torch.Tensor:
    """Map the reference's fusion parameters (layer dicts) to the factored table [L, 24] (float64, host)."""
    names, base, M = fusion_map(kind, n)
    rows = []
    for lay in layers:
        flat = [torch.as_tensor(lay[nm]).detach().double().cpu().reshape(2) for nm in names]
        rows.append(base + (torch.cat(flat) @ M if names else 0.0))
    return torch.stack(rows)


def fusion_table_torch(kind: str, layer_params, n: int) -> torch.Tensor:
    """Differentiable ``fusion_table``: layer_params[l] = list of (2,) tensors in FUSION_PARAM_NAMES order.
    The backward of the table is M^T (gfusion rows -> parameter gradients)."""
    names, base, M = fusion_map(kind, n)
    dev = layer_params[0][0].device if names else "cpu"
    base, M = base.to(dev), M.to(dev)
    rows = [base + (torch.cat([p.double().reshape(2) for p in ps]) @ M if names else 0.0) for ps in layer_params]
    return torch.stack(rows)


def pack_params(layers, device="cuda") -> torch.Tensor:
    chunks = []
    for lay in layers:
        for name in ("rms_w", "rms_b", "W", "b"):
            chunks.append(torch.as_tensor(np.asarray(lay[name]) if not torch.is_tensor(lay[name])
                                          else lay[name]).reshape(-1).to(torch.float32).cpu())
    return torch.cat(chunks).to(device).contiguous()


def layer_dims(layers):
    W0 = layers[0]["W"]
    dims = [int(W0.shape[1])] + [int(lay["W"].shape[0]) for lay in layers]
    return dims


# ---- step grids ---------------------------------------------------------------------------------------


def rk4_grid(t0: float, t1: float, nsteps: int) -> np.ndarray:
    """Fixed-step RK4 (build extension, BASELINE config 2): t_k = fl(t0 + fl(k * fl((t1-t0)/N)))."""
    f32 = np.float32
    t0, t1 = f32(t0), f32(t1)
    h = f32(f32(t1 - t0) / f32(nsteps))
    g = np.empty(nsteps + 1, dtype=f32)
    for k in range(nsteps + 1):
        g[k] = f32(t0 + f32(f32(k) * h))
    g[-1] = t1
    return g


def knot_grid(ts, steps_per_interval: int) -> np.ndarray:
    """Fixed grid that contains every knot: each [ts_i, ts_{i+1}] split into m equal fp32 steps (the knot
    itself exact).  Step states at indices i*m are then exactly the SaveAt(ts) outputs of the solve, so a
    fixed-step solve can be trained on trajectories like graph_neural_cde.py:89-92 (evolving_out)."""
    f32 = np.float32
    ts = np.asarray(ts, dtype=f32)
    m = int(steps_per_interval)
    if m < 1 or ts.ndim != 1 or ts.shape[0] < 2:
        raise ValueError("knot_grid: need ts [T>=2] and steps_per_interval >= 1")
    out = [ts[0]]
    for i in range(ts.shape[0] - 1):
        a, b = ts[i], ts[i + 1]
        h = f32(f32(b - a) / f32(m))
        out.extend(f32(a + f32(f32(k) * h)) for k in range(1, m))
        out.append(b)
    return np.asarray(out, dtype=f32)


def constant_step_grid(t0: float, t1: float, dt0: float, tol: float = 1e-6) -> np.ndarray:
    """diffrax ConstantStepSize: t_{k+1} = fl(t_k + dt0), snapped to t1 when within tol (fp32)."""
    f32 = np.float32
    t0, t1, dt0 = f32(t0), f32(t1), f32(dt0)
    out = [t0]
    t = t0
    thr = f32(t1 - f32(tol))
    while t < t1:
        tn = f32(t + dt0)
        if tn > thr:
            tn = t1
        out.append(tn)
        t = tn
    return np.asarray(out, dtype=f32)


def stack_grids(grids, device="cuda"):
    """List of per-sample grids -> (grid [B, G] padded with the last knot, nsteps [B] int32)."""
    G = max(len(g) for g in grids)
    out = np.empty((len(grids), G), dtype=np.float32)
    ns = np.empty(len(grids), dtype=np.int32)
    for b, g in enumerate(grids):
        out[b, :len(g)] = g
        out[b, len(g):] = g[-1]
        ns[b] = len(g) - 1
    return torch.from_numpy(out).to(device), torch.from_numpy(ns).to(device)
