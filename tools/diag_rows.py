#!/usr/bin/env python3
"""Diagnostic: one-launch evaluation (gncde_rows.hip) vs the fp64 oracle over a sweep of shapes (n, widths, CDE),
fp32 and bf16_mfma.  Prints one line per case.  Test infrastructure (imports oracle/)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "perm-equiv-graph-neural-cdes_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import gncde  # noqa: E402
from oracle import bf16_model as BM  # noqa: E402
from oracle import gncde_oracle as O  # noqa: E402
from tests.golden import make_golden as MG  # noqa: E402


def case(n, H, L, cde, kind="undirected", B=2, T=4, seed=0, compute="fp32"):
    rng = np.random.default_rng(seed if seed else n)
    dims = [H] * L + [16 * H if cde else H]
    ts, coeffs, params = MG.problem(rng, B, n, T, kind, dims)
    kw, xc = {}, None
    if cde:
        xs = [O.backward_hermite_coefficients(ts[b], rng.standard_normal((T, n, 8, 2))) for b in range(B)]
        xc = tuple(np.stack([x[q] for x in xs]) for q in range(4))
        kw = dict(data_coeffs=xc, cde_hidden=H, cde_embed=8)
    prob = gncde.make_problem(ts, coeffs, params.kind, params.layers, compute=compute, **kw)
    y = rng.standard_normal((B, n, H))
    t = np.array([rng.uniform(ts[b, 0], ts[b, -1]) for b in range(B)], dtype=np.float32).astype(np.float64)
    dy = gncde.vf_eval(prob, torch.tensor(t, dtype=torch.float32, device="cuda"),
                       torch.tensor(y, dtype=torch.float32, device="cuda")).cpu().numpy()
    errs = []
    bf = compute == "bf16_mfma"
    M = BM if bf else O
    cq = BM.coef_bf16(coeffs) if bf else coeffs
    for b in range(B):
        ctrl = O.CubicInterpolation(ts[b], tuple(c[b] for c in cq))
        if cde:
            ref = M.cde_wrapper(params, H, 8, t[b], y[b], ctrl, O.CubicInterpolation(ts[b], tuple(c[b] for c in xc)))
        else:
            ref = M.vector_field(params, t[b], y[b], ctrl)
        d = np.abs(dy[b] - ref)
        rows = np.where(d.max(axis=1) > 1e-4 * np.abs(ref).max())[0]
        if len(rows):
            cols = np.where(d.max(axis=0) > 1e-4 * np.abs(ref).max())[0]
            print(f"   sample {b}: bad cols {cols[:16].tolist()} ({len(cols)}), rows {rows[:32].tolist()}")
        errs.append((float(d.max() / np.abs(ref).max()), rows[:8].tolist(), len(rows)))
        if len(rows):
            print(f"   sample {b}: max|dy| {np.abs(dy[b]).max():.3e} max|ref| {np.abs(ref).max():.3e}; dy[0,:4] {dy[b][0, :4]}, "
                  f"ref[0,:4] {ref[0, :4]}; dy[n-1,:4] {dy[b][-1, :4]} ref {ref[-1, :4]}")
            ratio = dy[b] / np.where(np.abs(ref) > 1e-12, ref, np.nan)
            print(f"   ratio dy/ref median {np.nanmedian(ratio):.4f}, spread {np.nanpercentile(ratio, 10):.4f}..{np.nanpercentile(ratio, 90):.4f}")
    print(f"{compute} n={n} H={H} L={L} cde={cde} {kind}: " + " | ".join(f"err {e:.2e} bad rows {r} ({c})" for e, r, c in errs),
          flush=True)


if __name__ == "__main__":
    torch.cuda.set_device(0)
    if len(sys.argv) > 1:
        gncde._lib.load(sys.argv[1])
        print("library", sys.argv[1])
    for compute in os.environ.get("DIAG_MODES", "fp32,bf16_mfma").split(","):
        for (n, H, L, cde, T, seed) in [(255, 32, 3, True, 5, 1287), (255, 32, 3, True, 4, 0), (255, 32, 3, True, 5, 0),
                                        (200, 32, 3, True, 5, 0), (255, 32, 2, True, 5, 0), (255, 32, 3, False, 5, 0),
                                        (129, 32, 3, True, 5, 0), (64, 32, 3, True, 5, 0)]:
            case(n, H, L, cde, T=T, seed=seed, compute=compute)
