"""fp64 model of the bf16 MFMA mode's rounding points — TEST INFRASTRUCTURE ONLY.

Only ``tests/`` may import this module, and only as the checker.

``GNCDE_COMPUTE_BF16_MFMA`` (include/gncde.h; csrc/gncde_rows.hip, ``k_rows<H, MODE, true>``) is this engine's own
throughput arithmetic for BASELINE config 5 ("bf16 MFMA path"): the reference computes in fp32 only, so there is no
reference counterpart to restate.  What the mode defines is WHERE values are rounded to bfloat16; everything else is
fp32 accumulation.  This module states those points in fp64 on top of ``gncde_oracle`` (which restates the reference
vector field, perm_equiv_graph_vector_field.py:85-129, layers.py:36-48, cde_wrapper_vector_field.py:19-26), so a
GPU test can tell rounding the mode defines (large, ~2^-8 per operand) from an indexing or accumulation error:

* the operator coefficients ``(d, c, b, a)[..., 1]`` are stored as bf16 (the caller rounds them: ``coef_bf16``);
* layer l with input Z (RMSNorm folded: W' = W diag(rms_w), b' = b + W rms_b, inv = rsqrt(mean(Z^2) + eps)):
    P  = bf16((I + Abar_l) diag(inv)) @ bf16(Z)                  (the n x n product, fp32 accumulate)
    out = bf16(P) @ bf16(W')^T + q_l b'^T,  q_l = (I + Abar_l) 1   (the Linear, bias term in fp32)
  hidden layers take relu(out) (kept fp32 between layers); the ODE output is tg * out;
* the de = 8 CDE read-out contracts the widening layer without forming it:
    dy[i, m] = tg_i (sum_{c, j} bf16(P[i, c] dX[i, j]) bf16(W')[16 m + j, c] + q_i sum_j b'[16 m + j] dX[i, j]).
"""
from __future__ import annotations

import numpy as np

from oracle import gncde_oracle as O


def bf16(x):
    """x -> fp32 -> bfloat16 (round to nearest even) -> fp64."""
    u = np.asarray(x, dtype=np.float32).view(np.uint32).astype(np.uint64)
    u = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) << 16
    return u.astype(np.uint32).view(np.float32).astype(np.float64)


def coef_bf16(coeffs):
    """(d, c, b, a) [.., n, n, 2] with the operator channel rounded to bf16 (the time channel stays fp32)."""
    out = []
    for c in coeffs:
        q = np.array(c, dtype=np.float64)
        q[..., 1] = bf16(c[..., 1])
        out.append(q)
    return tuple(out)


def _layer(params: O.VFParams, l, A, dA, Z):
    """(P unrounded, bf16 W', b', q) of layer l."""
    lay = params.layers[l]
    M = np.eye(A.shape[0]) + O.fused_matrix(params, l, A, dA)
    inv = 1.0 / np.sqrt(np.mean(Z * Z, axis=-1) + 1e-5)
    P = bf16(M * inv[None, :]) @ bf16(Z)
    Wp = bf16(lay["W"] * lay["rms_w"][None, :])
    bp = lay["b"] + lay["W"] @ lay["rms_b"]
    return P, Wp, bp, M.sum(axis=1)


def _hidden(params, A, dA, y):
    Z = y
    for l in range(len(params.layers) - 1):
        P, Wp, bp, q = _layer(params, l, A, dA, Z)
        Z = np.maximum(bf16(P) @ Wp.T + q[:, None] * bp[None, :], 0.0)
    return Z


def vector_field(params: O.VFParams, t, y, control):
    """The ODE vector field as the bf16 mode computes it (control: bf16-rounded coefficients)."""
    X, dX = control.evaluate(t), control.derivative(t)
    A, dA, tg = X[..., -1], dX[..., -1], dX[..., 0]
    Z = _hidden(params, A, dA, y)
    P, Wp, bp, q = _layer(params, len(params.layers) - 1, A, dA, Z)
    return np.mean(tg, axis=0)[:, None] * (bf16(P) @ Wp.T + q[:, None] * bp[None, :])


def cde_wrapper(params: O.VFParams, hidden_dim, data_embed_dim, t, y, control_adj, control_data):
    """The de = 8 CDE wrapper's vector field as the bf16 mode computes it (read-out contracted, see above)."""
    assert data_embed_dim == 8
    H = hidden_dim
    X, dXa = control_adj.evaluate(t), control_adj.derivative(t)
    A, dA, tg = X[..., -1], dXa[..., -1], dXa[..., 0]
    Z = _hidden(params, A, dA, y)
    P, Wp, bp, q = _layer(params, len(params.layers) - 1, A, dA, Z)
    dX = control_data.derivative(t).reshape(A.shape[0], 16)  # [n, (de, 2)] -> j = 2 l + k
    Q = bf16(P[:, None, :] * dX[:, :, None])                  # [n, j, c]
    acc = np.einsum("njc,mjc->nm", Q, Wp.reshape(H, 16, H))
    bias = dX @ bp.reshape(H, 16).T                           # [n, m]
    return np.mean(tg, axis=0)[:, None] * (acc + q[:, None] * bias)
