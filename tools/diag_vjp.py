#!/usr/bin/env python3
"""Diagnostic: the reverse mode of ONE evaluation (gncde_rows_vjp.hip) against oracle vector_field_vjp."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "perm-equiv-graph-neural-cdes_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import gncde  # noqa: E402
from gncde import _lib  # noqa: E402
from oracle import gncde_oracle as O  # noqa: E402
from oracle import gncde_oracle_grad as OG  # noqa: E402
from tests.golden import make_golden as MG  # noqa: E402

lib = _lib.load()
lib.gncde_diag_vf_vjp_bytes.restype = ctypes.c_size_t
P_ = ctypes.c_void_p
for (n, H, L) in [(40, 32, 2), (40, 32, 3), (40, 32, 4), (40, 16, 4), (40, 32, 5)]:
    rng = np.random.default_rng(n + L)
    B, T = 2, 4
    ts, coeffs, P = MG.problem(rng, B, n, T, "undirected", [H] * (L + 1), irregular=False)
    prob = gncde.make_problem(ts, coeffs, P.kind, P.layers)
    y = rng.standard_normal((B, n, H))
    g = rng.standard_normal((B, n, H))
    t = np.array([0.5 * (ts[b, 0] + ts[b, -1]) for b in range(B)], dtype=np.float32)
    ps = prob.c_struct()
    nbytes = lib.gncde_diag_vf_vjp_bytes(ctypes.byref(ps))
    ws = torch.zeros(nbytes, dtype=torch.uint8, device="cuda")
    gy = torch.zeros(B, n, H, device="cuda")
    gp = torch.zeros(prob.params.numel(), device="cuda")
    gf = torch.zeros(L, 24, device="cuda")
    yt = torch.tensor(y, dtype=torch.float32, device="cuda")
    gt = torch.tensor(g, dtype=torch.float32, device="cuda")
    tt = torch.tensor(t, device="cuda")
    rc = lib.gncde_diag_vf_vjp(ctypes.byref(ps), P_(tt.data_ptr()), P_(yt.data_ptr()), P_(gt.data_ptr()),
                               P_(gy.data_ptr()), P_(gp.data_ptr()), P_(gf.data_ptr()), P_(ws.data_ptr()),
                               ctypes.c_size_t(nbytes), None)
    torch.cuda.synchronize()
    gys, total = [], None
    for b in range(B):
        ctrl = O.CubicInterpolation(ts[b], tuple(c[b] for c in coeffs))
        gyb, gr = OG.vector_field_vjp(P, float(t[b]), y[b], ctrl, g[b])
        gys.append(gyb)
        total = OG._acc(total, gr)
    def rel(a, r):
        return float(np.max(np.abs(np.asarray(a) - r)) / np.max(np.abs(r)))
    errs = {"gy": rel(gy.cpu().numpy(), np.stack(gys))}
    gpn = gp.cpu().numpy()
    off = 0
    for l in range(L):
        for k in ("rms_w", "rms_b", "W", "b"):
            sz = total[l][k].size
            errs[f"{k}{l}"] = rel(gpn[off:off + sz].reshape(total[l][k].shape), total[l][k])
            off += sz
    names, base, M = gncde.layout.fusion_map("undirected", n)
    ref = np.stack([np.concatenate([total[l][nm] for nm in names]) for l in range(L)])
    errs["fusion"] = rel(gf.double().cpu().numpy() @ M.numpy().T, ref)
    print(f"n={n} H={H} L={L} rc={rc}: " + " ".join(f"{k} {v:.1e}" for k, v in errs.items()), flush=True)
