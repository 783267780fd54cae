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


def pack_data_control(coeffs, device="cuda"):
    """CDE data spline (d, c, b, a) each [B, T-1, n, de, 2] -> [B, T-1, 4, n, de, 2]."""
    parts = [torch.as_tensor(np.asarray(x) if not torch.is_tensor(x) else x) for x in coeffs]
    if parts[0].dim() == 4:
        parts = [p.unsqueeze(0) for p in parts]
    return torch.stack([p.to(device=device, dtype=torch.float32) for p in parts], dim=2).contiguous()


def fusion_table(kind: str, layers, n: int) -> torch.Tensor:
    """Map the reference's fusion parameters to the factored table [L, 24] (float64 on host).

    kind "undirected": ConvEquivFusionLayer._fusion (layers.py:102-160)
    kind "directed":   ConvEquivFusionDirectedLayer._fusion (layers.py:256-337)
    kind "plain":      GraphVectorField message matrix A + dA (graph_vector_field.py:94)
    """
    L = len(layers)
    tab = torch.zeros(L, FC, dtype=torch.float64)

    def p(lay, name, j):
        return float(torch.as_tensor(lay[name]).double().reshape(-1)[j])

    for l, lay in enumerate(layers):
        t = tab[l]
        t[IDC] = 1.0  # ConvLayer residual: m + Abar @ m (layers.py:47)
        if kind == "plain":
            t[E_A] = t[E_DA] = 1.0
            continue
        t[E_A], t[E_DA] = 1.0 + p(lay, "param1", 0), 1.0 + p(lay, "param1", 1)  # term_1
        t[ET_A], t[ET_DA] = p(lay, "param2", 0), p(lay, "param2", 1)  # term_2 transpose
        t[UD_A], t[UD_DA] = p(lay, "param3", 0), p(lay, "param3", 1)  # term_3 diag(diag)
        # term_7: both halves multiply sum(adjacency) (layers.py:144-148)
        t[WS_A] = p(lay, "param7", 0) / n**2 + p(lay, "param7", 1) / n**2
        t[US_A], t[US_DA] = p(lay, "param8", 0) / n**2, p(lay, "param8", 1) / n**2  # term_8
        if kind == "undirected":
            t[WR_A], t[WR_DA] = p(lay, "param4", 0) / n, p(lay, "param4", 1) / n  # row sums -> rows
            t[VR_A], t[VR_DA] = p(lay, "param5", 0) / n, p(lay, "param5", 1) / n  # row sums -> cols
            t[UR_A], t[UR_DA] = p(lay, "param6", 0) / n, p(lay, "param6", 1) / n  # diag(row sums)
        elif kind == "directed":
            t[WC_A], t[WC_DA] = p(lay, "param4", 0) / n, p(lay, "param4", 1) / n  # col sums -> rows
            t[VR_A] += p(lay, "param4_prime", 0) / n  # tile(rowsum A)
            t[VC_DA] += p(lay, "param4_prime", 1) / n  # tile(colsum dA)  (quirk :288-293)
            t[VC_A] += p(lay, "param5", 0) / n
            t[VC_DA] += p(lay, "param5", 1) / n
            t[VR_A] += p(lay, "param5_prime", 0) / n
            t[VR_DA] += p(lay, "param5_prime", 1) / n
            t[UC_A], t[UC_DA] = p(lay, "param6", 0) / n, p(lay, "param6", 1) / n
            t[UR_A], t[UR_DA] = p(lay, "param6_prime", 0) / n, p(lay, "param6_prime", 1) / n
        else:
            raise ValueError(kind)
    return tab


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
