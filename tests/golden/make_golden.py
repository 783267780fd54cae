"""Generate the golden fixtures in tests/golden/*.npz from the fp64 CPU oracle (oracle/gncde_oracle.py).

    python tests/golden/make_golden.py

PARITY UNPINNED: the reference (JAX/diffrax/equinox) cannot be executed in this image, so these
vectors come from the build's restatement of the reference algorithm, not from the reference itself.
They freeze the oracle (tests/test_golden.py re-derives them) and are the GPU parity targets
(tests/test_gpu_parity.py).  Parameters are injected (drawn from the reference's init distributions
with numpy), so no JAX PRNG is involved.
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
from oracle import gncde_oracle as O  # noqa: E402
from oracle import gncde_oracle_grad as OG  # noqa: E402


def flat_layers(prefix, params: O.VFParams, out: dict):
    out[prefix + "kind"] = np.array(params.kind)
    out[prefix + "L"] = np.array(len(params.layers))
    for l, lay in enumerate(params.layers):
        for k, v in lay.items():
            out[f"{prefix}l{l}_{k}"] = np.asarray(v, dtype=np.float64)


def load_layers(z, prefix=""):
    kind = str(z[prefix + "kind"])
    L = int(z[prefix + "L"])
    layers = []
    for l in range(L):
        pre = f"{prefix}l{l}_"
        lay = {k[len(pre):]: np.asarray(z[k]) for k in z.files if k.startswith(pre)}
        layers.append(lay)
    return O.VFParams(kind=kind, layers=layers)


def problem(rng, B, n, T, kind, dims, irregular=True):
    ts_all, coeffs_all = [], []
    for _ in range(B):
        ts, X = O.make_graph_control(rng, n, T, irregular=irregular)
        ts_all.append(ts)
        coeffs_all.append(O.backward_hermite_coefficients(ts, X))
    params = O.init_vf_params(rng, kind, dims)
    # perturb RMSNorm affine so its weight/bias paths are exercised
    for lay in params.layers:
        lay["rms_w"] = lay["rms_w"] + 0.1 * rng.standard_normal(lay["rms_w"].shape)
        lay["rms_b"] = lay["rms_b"] + 0.1 * rng.standard_normal(lay["rms_b"].shape)
    ts = np.stack(ts_all)
    coeffs = tuple(np.stack([c[q] for c in coeffs_all]) for q in range(4))
    return ts, coeffs, params


def vf_case(rng, name, B, n, T, kind, dims):
    ts, coeffs, params = problem(rng, B, n, T, kind, dims)
    y = rng.standard_normal((B, n, dims[0]))
    # times: interior points, an exact knot, t0 and t1 (index-rule edges)
    t = np.array([rng.uniform(ts[b, 0], ts[b, -1]) for b in range(B)], dtype=np.float32).astype(np.float64)
    t[0] = ts[0, 0]
    if B > 1:
        t[1] = ts[1, -1]
    if B > 2:
        t[2] = ts[2, T // 2]
    dy = np.stack([O.vector_field(params, t[b], y[b], O.CubicInterpolation(ts[b], tuple(c[b] for c in coeffs)))
                   for b in range(B)])
    out = dict(ts=ts, d=coeffs[0], c=coeffs[1], b=coeffs[2], a=coeffs[3], y=y, t=t, dy=dy)
    flat_layers("", params, out)
    np.savez_compressed(os.path.join(HERE, name), **out)


def solve_case(rng, name, B, n, T, kind, dims, method, nsteps=None, dt0=None, irregular=True):
    ts, coeffs, params = problem(rng, B, n, T, kind, dims, irregular=irregular)
    y0 = rng.standard_normal((B, n, dims[0]))
    grids, ys = [], []
    for b in range(B):
        ctrl = O.CubicInterpolation(ts[b], tuple(c[b] for c in coeffs))
        f = lambda t, y, ctrl=ctrl: O.vector_field(params, t, y, ctrl)  # noqa: E731
        if method == "rk4":
            g = O.rk4_grid(ts[b, 0], ts[b, -1], nsteps)
        else:
            g = O.constant_grid(ts[b, 0], ts[b, -1], dt0)
        grids.append(g)
        traj, _ = O.solve_fixed_grid(f, g, y0[b], method=method, save_every_step=True,
                                     time_dtype=np.float32)
        ys.append(traj)
    G = max(len(g) for g in grids)
    grid = np.stack([np.concatenate([g, np.full(G - len(g), g[-1], np.float32)]) for g in grids])
    nst = np.array([len(g) - 1 for g in grids], dtype=np.int32)
    traj = np.stack([np.concatenate([y, np.repeat(y[-1:], G - len(y), axis=0)]) for y in ys])
    out = dict(ts=ts, d=coeffs[0], c=coeffs[1], b=coeffs[2], a=coeffs[3], y0=y0, grid=grid, nsteps=nst,
               ys=traj, method=np.array(method))
    flat_layers("", params, out)
    np.savez_compressed(os.path.join(HERE, name), **out)


def pid_case(rng, name, B, n, T, kind, dims, rtol=1e-3, atol=1e-6, dt0=None, cde=None):
    """Tsit5 + PIDController, SaveAt(ts=ts) — the GraphNeuralCDE solve (graph_neural_cde.py:94-104); with
    cde=(h, de) the CDE-wrapper vector field of the PGT/TGB drivers (BASELINE config 5's adaptive solve)."""
    if cde is not None:
        h, de = cde
        dims = [h] + list(dims[1:-1]) + [h * de * 2]
    ts, coeffs, params = problem(rng, B, n, T, kind, dims, irregular=cde is None)
    y0 = rng.standard_normal((B, n, dims[0]))
    ys, st, truth, ens, dco = [], [], [], [], []
    for b in range(B):
        ctrl = O.CubicInterpolation(ts[b], tuple(c[b] for c in coeffs))
        f = lambda t, y, ctrl=ctrl: O.vector_field(params, t, y, ctrl)  # noqa: E731
        if cde is not None:
            x = rng.standard_normal((T, n, de))
            X = np.stack([np.broadcast_to(ts[b][:, None, None], x.shape), x], axis=-1)
            dc = O.backward_hermite_coefficients(ts[b], X)
            dco.append(dc)
            cx = O.CubicInterpolation(ts[b], dc)
            f = lambda t, y, ctrl=ctrl, cx=cx: O.cde_wrapper(params, h, de, t, y, ctrl, cx)  # noqa: E731
        out, stats = O.solve_tsit5_pid(f, ts[b, 0], ts[b, -1], y0[b], rtol=rtol, atol=atol, dt0=dt0,
                                       save_ts=ts[b])
        ys.append(out)
        st.append([stats["steps"], stats["rejects"], stats["evals"]])
        # near-exact solution: the adaptive step sequence is chaotic in the last bits (a 1e-4 relative
        # change of rtol moves the output by ~1e-2), so parity is judged by accuracy against this
        tr, _ = O.solve_tsit5_pid(f, ts[b, 0], ts[b, -1], y0[b], rtol=1e-10, atol=1e-12, save_ts=ts[b],
                                  max_steps=200000)
        truth.append(tr)
        # accuracy spread of the reference algorithm itself: rtol perturbed by +-1e-4 .. 1e-2 relative (the
        # step sequence is chaotic, so a handful of perturbations samples the spread of equally valid solves)
        for scale in (1 - 1e-2, 1 - 1e-3, 1 - 1e-4, 1 + 1e-4, 1 + 1e-3, 1 + 1e-2):
            pe, _ = O.solve_tsit5_pid(f, ts[b, 0], ts[b, -1], y0[b], rtol=rtol * scale, atol=atol, dt0=dt0,
                                      save_ts=ts[b])
            ens.append(np.max(np.abs(pe - tr)) / np.max(np.abs(tr)))
        ens.append(np.max(np.abs(out - tr)) / np.max(np.abs(tr)))
    out = dict(ts=ts, d=coeffs[0], c=coeffs[1], b=coeffs[2], a=coeffs[3], y0=y0, ys=np.stack(ys),
               truth=np.stack(truth), ens_err=np.array(max(ens)),
               stats=np.array(st), rtol=np.array(rtol), atol=np.array(atol),
               dt0=np.array(np.nan if dt0 is None else dt0))
    if cde is not None:
        out.update(xd=np.stack([c[0] for c in dco]), xc=np.stack([c[1] for c in dco]),
                   xb=np.stack([c[2] for c in dco]), xa=np.stack([c[3] for c in dco]), h=np.array(h),
                   de=np.array(de))
    flat_layers("", params, out)
    np.savez_compressed(os.path.join(HERE, name), **out)


def cde_case(rng, name, B, n, T, h, de, L):
    dims = [h] + [h] * (L - 1) + [h * de * 2]
    ts, coeffs, params = problem(rng, B, n, T, "undirected", dims)
    # data spline: x [T, n, de] stacked with time (tgb_graph_neural_cde.py:115-130)
    dcoef = []
    for b in range(B):
        x = rng.standard_normal((T, n, de))
        X = np.stack([np.broadcast_to(ts[b][:, None, None], x.shape), x], axis=-1)
        dcoef.append(O.backward_hermite_coefficients(ts[b], X))
    dcoeffs = tuple(np.stack([c[q] for c in dcoef]) for q in range(4))
    y = rng.standard_normal((B, n, h))
    t = np.array([rng.uniform(ts[b, 0], ts[b, -1]) for b in range(B)], dtype=np.float32).astype(np.float64)
    dy = []
    for b in range(B):
        ca = O.CubicInterpolation(ts[b], tuple(c[b] for c in coeffs))
        cd = O.CubicInterpolation(ts[b], tuple(c[b] for c in dcoeffs))
        dy.append(O.cde_wrapper(params, h, de, t[b], y[b], ca, cd))
    out = dict(ts=ts, d=coeffs[0], c=coeffs[1], b=coeffs[2], a=coeffs[3], xd=dcoeffs[0], xc=dcoeffs[1],
               xb=dcoeffs[2], xa=dcoeffs[3], y=y, t=t, dy=np.stack(dy), h=np.array(h), de=np.array(de))
    flat_layers("", params, out)
    np.savez_compressed(os.path.join(HERE, name), **out)


def grad_case(rng, name, B, n, T, kind, dims, method, nsteps=None, dt0=None, cotangent="final", cde=None,
              data_grad=False):
    """Reverse mode of a fixed-grid solve (oracle/gncde_oracle_grad.py): expected dL/dy0 per sample and
    dL/dparams summed over samples for L = sum(g * y) with a random cotangent g."""
    if cde is not None:
        h, de = cde
        dims = [h] + list(dims[1:-1]) + [h * de * 2]
    ts, coeffs, params = problem(rng, B, n, T, kind, dims, irregular=cde is None)
    if cde is not None:
        ts = np.tile(np.linspace(0.0, 3.0, T), (B, 1))
        co = []
        for b in range(B):
            _, X = O.make_graph_control(rng, n, T, irregular=False, t1=3.0)
            co.append(O.backward_hermite_coefficients(ts[b], X))
        coeffs = tuple(np.stack([c[q] for c in co]) for q in range(4))
    for lay in params.layers:  # fusion params large enough that their gradients are well conditioned
        for nm in OG.FUSION_NAMES[kind]:
            lay[nm] = lay[nm] * 3.0
    ds = dims[0]
    y0 = rng.standard_normal((B, n, ds))
    grids, gys, gy0s, total, dco, gxs, xs = [], [], [], None, [], [], []
    for b in range(B):
        ctrl = O.CubicInterpolation(ts[b], tuple(c[b] for c in coeffs))
        if cde is None:
            f = lambda t, y, ctrl=ctrl: O.vector_field(params, t, y, ctrl)  # noqa: E731
            fv = lambda t, y, g, ctrl=ctrl: OG.vector_field_vjp(params, t, y, ctrl, g)  # noqa: E731
        else:
            x = rng.standard_normal((T, n, de))
            xs.append(x)
            Xd = np.stack([np.broadcast_to(ts[b][:, None, None], x.shape), x], axis=-1)
            dc = O.backward_hermite_coefficients(ts[b], Xd)
            dco.append(dc)
            cx = O.CubicInterpolation(ts[b], dc)
            f = lambda t, y, ctrl=ctrl, cx=cx: O.cde_wrapper(params, h, de, t, y, ctrl, cx)  # noqa: E731
            fv = lambda t, y, g, ctrl=ctrl, cx=cx: OG.cde_wrapper_vjp(params, h, de, t, y, ctrl, cx, g,  # noqa
                                                                      data_grad=data_grad)
        g = O.rk4_grid(ts[b, 0], ts[b, -1], nsteps) if method == "rk4" else O.constant_grid(ts[b, 0], ts[b, -1],
                                                                                             dt0)
        grids.append(g)
        gy = rng.standard_normal((n, ds) if cotangent == "final" else (len(g), n, ds))
        kw = dict(g_final=gy) if cotangent == "final" else dict(g_steps=gy)
        # ReLU networks have gradients that jump where a pre-activation crosses 0: an fp32 solve (GPU or
        # reference) lands on the other side of a nearby kink and legitimately differs by ~1%.  Keep only
        # samples whose gradient is stable under a 1e-6 relative perturbation of y0 (redraw y0 otherwise).
        for _ in range(20):
            gy0, gr = OG.solve_fixed_grid_vjp(f, fv, g, y0[b], method, **kw)
            gy0p, grp = OG.solve_fixed_grid_vjp(f, fv, g, y0[b] * (1 + 1e-6), method, **kw)
            if data_grad:  # the data spline's cotangent -> the data knots' (channel 1; channel 0 is time)
                gx, gr, grp = OG.hermite_vjp(ts[b], gr[-1]["data_coef"])[..., 1], gr[:-1], grp[:-1]
            va, vb = OG.grads_to_vector(gr, kind), OG.grads_to_vector(grp, kind)
            spread = max(np.max(np.abs(gy0p - gy0)) / np.max(np.abs(gy0)),
                         np.max(np.abs(vb - va)) / np.max(np.abs(va)))
            if spread < 1e-5:
                break
            y0[b] = rng.standard_normal((n, ds))
        else:
            raise RuntimeError(f"{name}: no gradient-stable sample found")
        gys.append(gy)
        gy0s.append(gy0)
        if data_grad:
            gxs.append(gx)
        total = OG._acc(total, gr)
    G = max(len(g) for g in grids)
    grid = np.stack([np.concatenate([g, np.full(G - len(g), g[-1], np.float32)]) for g in grids])
    nst = np.array([len(g) - 1 for g in grids], dtype=np.int32)
    if cotangent == "steps":  # padded steps repeat the final state: their cotangent is zero
        gys = [np.concatenate([gy, np.zeros((G - len(gy),) + gy.shape[1:])]) for gy in gys]
    out = dict(ts=ts, d=coeffs[0], c=coeffs[1], b=coeffs[2], a=coeffs[3], y0=y0, grid=grid, nsteps=nst,
               gys=np.stack(gys), gy0=np.stack(gy0s), method=np.array(method), cotangent=np.array(cotangent))
    if cde is not None:
        if data_grad:
            out.update(x=np.stack(xs), grad_x=np.stack(gxs))
        out.update(xd=np.stack([c[0] for c in dco]), xc=np.stack([c[1] for c in dco]),
                   xb=np.stack([c[2] for c in dco]), xa=np.stack([c[3] for c in dco]), h=np.array(h),
                   de=np.array(de))
    flat_layers("", params, out)
    for l, gl in enumerate(total):
        for k, v in gl.items():
            out[f"grad_l{l}_{k}"] = np.asarray(v, np.float64)
    np.savez_compressed(os.path.join(HERE, name), **out)


def main():
    rng = np.random.default_rng(1234)
    vf_case(rng, "vf_undirected_n16_L3.npz", 4, 16, 12, "undirected", [16, 16, 16, 16])
    vf_case(rng, "vf_directed_n16_L2.npz", 4, 16, 12, "directed", [16, 16, 16])
    vf_case(rng, "vf_plain_n16_L2.npz", 4, 16, 12, "plain", [16, 16, 16])
    vf_case(rng, "vf_undirected_n10_mixed.npz", 3, 10, 9, "undirected", [8, 24, 12])
    vf_case(rng, "vf_undirected_n4_L2.npz", 3, 4, 6, "undirected", [16, 16, 16])
    solve_case(rng, "rk4_undirected_n16_L2.npz", 4, 16, 12, "undirected", [16, 16, 16], "rk4", nsteps=20)
    solve_case(rng, "rk4_undirected_n10_L3.npz", 3, 10, 10, "undirected", [16, 16, 16, 16], "rk4", nsteps=15)
    solve_case(rng, "tsit5c_undirected_n16_L2.npz", 3, 16, 8, "undirected", [16, 16, 16], "tsit5", dt0=0.5)
    solve_case(rng, "rk4_directed_n32_h32_L2.npz", 2, 32, 8, "directed", [32, 32, 32], "rk4", nsteps=10)
    cde_case(rng, "cde_n12_h8_de3.npz", 3, 12, 5, 8, 3, 2)
    # widths differ between layers -> not covered by the fused kernel, exercises the generic solver
    solve_case(rng, "rk4_undirected_n12_mixed.npz", 2, 12, 7, "undirected", [16, 24, 16], "rk4", nsteps=8)
    # regular knots: with irregular knots 0.04 apart the cubic's d coefficients reach ~4e3 and any fp32
    # Horner evaluation (the reference's too) loses ~1e-4 relative over the solve (ill-conditioned)
    solve_case(rng, "tsit5c_plain_n20_mixed.npz", 2, 20, 6, "plain", [8, 12, 8], "tsit5", dt0=0.7,
               irregular=False)
    pid_case(rng, "pid_undirected_n16_L2.npz", 3, 16, 10, "undirected", [16, 16, 16])
    pid_case(rng, "pid_directed_n12_L3_dt0.npz", 2, 12, 8, "directed", [16, 16, 16, 16], dt0=0.05)
    # reverse mode (training step); a fresh stream so earlier fixtures stay byte-identical
    rng = np.random.default_rng(4321)
    grad_case(rng, "grad_rk4_undirected_n16_L2.npz", 3, 16, 8, "undirected", [16, 16, 16], "rk4", nsteps=10)
    grad_case(rng, "grad_tsit5c_directed_n12_L3.npz", 2, 12, 6, "directed", [16, 16, 16, 16], "tsit5",
              dt0=0.7, cotangent="steps")
    grad_case(rng, "grad_rk4_plain_n10_mixed.npz", 2, 10, 6, "plain", [8, 12, 8], "rk4", nsteps=7)
    grad_case(rng, "grad_rk4_cde_n10_h8_de2.npz", 2, 10, 4, "undirected", [8, 8, 0], "rk4", nsteps=9,
              cde=(8, 2))
    # adaptive solves outside the fused kernel's coverage (generic PID path): mixed widths, CDE wrapper
    rng = np.random.default_rng(2468)
    pid_case(rng, "pid_undirected_n20_mixed.npz", 3, 20, 8, "undirected", [16, 24, 16])
    pid_case(rng, "pid_cde_n10_h8_de2.npz", 2, 10, 5, "undirected", [8, 8, 0], dt0=0.05, cde=(8, 2))
    # de = 8 (configs 3 / 5): the CDE contraction runs in the last GEMM's epilogue; n = 70 and h = 5 leave partial
    # row and channel tiles
    cde_case(np.random.default_rng(9753), "cde_n70_h5_de8.npz", 3, 70, 6, 5, 8, 3)
    # the CDE data spline's cotangent (TGBGraphNeuralCDE trains its data encoder through it)
    rng = np.random.default_rng(8642)
    grad_case(rng, "grad_rk4_cde_data_n9_h4_de3.npz", 2, 9, 5, "undirected", [4, 6, 0], "rk4", nsteps=8,
              cde=(4, 3), data_grad=True)
    layer_cases()


def layer_cases():
    """Shapes of the fused generic layer kernel (csrc/gncde_layer.hip): widths 16 / 32 / 64, the CDE read-out with
    de = 8 (one or two channel groups per row block), widening ODE layers, and n with a partial or single-row last
    32-row block."""
    rng = np.random.default_rng(1357)
    cde_case(rng, "cde_n40_h16_de8.npz", 2, 40, 5, 16, 8, 2)
    cde_case(rng, "cde_n33_h32_de8.npz", 2, 33, 5, 32, 8, 3)
    cde_case(rng, "cde_n20_h64_de8.npz", 2, 20, 4, 64, 8, 2)
    vf_case(rng, "vf_undirected_n65_w16_32_64.npz", 2, 65, 4, "undirected", [16, 32, 64])
    vf_case(rng, "vf_directed_n48_h64_L2.npz", 2, 48, 4, "directed", [64, 64, 64])


def pid_cde8_cases():
    """Tsit5 + PIDController through the de = 8 read-out k_layer (BASELINE config 5's adaptive CDE solve, the
    contraction inside the read-out's MFMA K loop): h = 16 (L = 2) and h = 32 (L = 3) at n = 40."""
    rng = np.random.default_rng(5151)
    pid_case(rng, "pid_cde8_n40_h16_L2.npz", 2, 40, 3, "undirected", [16, 16, 0], cde=(16, 8))
    pid_case(rng, "pid_cde8_n40_h32_L3.npz", 2, 40, 3, "undirected", [32, 32, 32, 0], cde=(32, 8))


if __name__ == "__main__":
    if sys.argv[1:] == ["pid_cde8"]:  # the fixtures added in round 2 (earlier files stay byte-identical)
        pid_cde8_cases()
    else:
        main()
        pid_cde8_cases()
