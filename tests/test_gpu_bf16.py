"""GPU: the bf16 paths (GNCDE_COMPUTE_BF16 / _BF16_STORAGE, BASELINE config 5; the retired _BF16_MFMA against an
experiment build only).

COMPUTE_BF16 runs the n x n products on v_mfma_f32_16x16x32_bf16 with both operands split into bf16 (hi, lo) pairs:
three products, fp32 accumulation, ~2^-16 relative per product, so it is held to fp32-class tolerances (5x the fp32
path's).  COMPUTE_BF16_STORAGE also quantises the operator coefficients to bf16; it is compared with the fp64 oracle
evaluated on the same bf16-rounded coefficients (the quantisation is an input change, not an arithmetic error).
Tolerances (relative to the max magnitude of the reference tensor):
  * one vector-field evaluation:   RTOL_BF16_VF    = 1e-4
  * a fixed-grid solve trajectory: RTOL_BF16_SOLVE = 5e-4
"""
import os

import numpy as np
import pytest
import torch

from oracle import gncde_oracle as O
from tests.golden import make_golden as MG
from tests.test_gpu_parity import ACC_PID_FACTOR, problem_from, rel_err

pytestmark = pytest.mark.gpu

RTOL_BF16_VF = 1e-4
RTOL_BF16_SOLVE = 5e-4
VF_CASES = [("vf_undirected_n16_L3.npz", False), ("vf_directed_n16_L2.npz", False),
            ("vf_undirected_n10_mixed.npz", False), ("vf_plain_n16_L2.npz", False),
            ("cde_n70_h5_de8.npz", True), ("cde_n12_h8_de3.npz", True),
            # the bf16 product inside k_layer (csrc/gncde_layer.hip): K chunks of 32 with n = 65 / 48 / 40 / 33
            ("vf_undirected_n65_w16_32_64.npz", False), ("vf_directed_n48_h64_L2.npz", False),
            ("cde_n40_h16_de8.npz", True), ("cde_n33_h32_de8.npz", True)]


@pytest.fixture(scope="module")
def gncde():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a HIP device")
    import gncde as G
    G._lib.load()
    return G


def bf16_round(x):
    """fp32 -> bf16 (round to nearest even) -> fp64, as torch's .to(torch.bfloat16) does."""
    u = np.asarray(x, dtype=np.float32).view(np.uint32).astype(np.uint64)
    u = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) << 16
    return u.astype(np.uint32).view(np.float32).astype(np.float64)


def vf_reference_on_bf16_coefficients(z, params, data):
    """fp64 oracle VF with the operator channel of (d, c, b, a) rounded to bf16 (the time channel stays fp32)."""
    q = []
    for key in ("d", "c", "b", "a"):
        c = np.array(z[key], dtype=np.float64)
        c[..., 1] = bf16_round(z[key][..., 1])
        q.append(c)
    ts, t, y = z["ts"], z["t"], z["y"]
    out = []
    for b in range(ts.shape[0]):
        ctrl = O.CubicInterpolation(ts[b], tuple(c[b] for c in q))
        if data:
            cx = O.CubicInterpolation(ts[b], tuple(z[k][b] for k in ("xd", "xc", "xb", "xa")))
            out.append(O.cde_wrapper(params, int(z["h"]), int(z["de"]), t[b], y[b], ctrl, cx))
        else:
            out.append(O.vector_field(params, t[b], y[b], ctrl))
    return np.stack(out)


@pytest.mark.parametrize("name,data", VF_CASES)
def test_bf16_vf_eval_vs_oracle(gncde, golden_dir, name, data):
    z = np.load(os.path.join(golden_dir, name))
    params = MG.load_layers(z)
    prob = problem_from(gncde, z, params, data=data).with_compute("bf16")
    dy = gncde.vf_eval(prob, torch.tensor(z["t"], dtype=torch.float32, device="cuda"),
                       torch.tensor(z["y"], dtype=torch.float32, device="cuda"))
    err = rel_err(dy.cpu().numpy(), z["dy"])
    print(f"{name} bf16: rel err {err:.3e}")
    assert err <= RTOL_BF16_VF


@pytest.mark.parametrize("name,data", VF_CASES)
def test_bf16_storage_vf_eval_vs_oracle_on_quantised_input(gncde, golden_dir, name, data):
    z = np.load(os.path.join(golden_dir, name))
    params = MG.load_layers(z)
    prob = problem_from(gncde, z, params, data=data).with_compute("bf16_storage")
    assert prob.coef.dtype == torch.bfloat16
    dy = gncde.vf_eval(prob, torch.tensor(z["t"], dtype=torch.float32, device="cuda"),
                       torch.tensor(z["y"], dtype=torch.float32, device="cuda")).cpu().numpy()
    ref = vf_reference_on_bf16_coefficients(z, params, data)
    err, quant = rel_err(dy, ref), rel_err(z["dy"], ref)
    print(f"{name} bf16_storage: rel err {err:.3e} (input quantisation moves the fp32 result by {quant:.3e})")
    assert err <= RTOL_BF16_VF


@pytest.mark.parametrize("name", ["rk4_undirected_n12_mixed.npz", "tsit5c_plain_n20_mixed.npz",
                                  "rk4_undirected_n16_L2.npz", "rk4_directed_n32_h32_L2.npz"])
def test_bf16_solve_vs_oracle(gncde, golden_dir, name):
    z = np.load(os.path.join(golden_dir, name))
    params = MG.load_layers(z)
    prob = problem_from(gncde, z, params).with_compute("bf16")
    method = gncde._lib.RK4 if str(z["method"]) == "rk4" else gncde._lib.TSIT5
    spec = gncde.SolverSpec(method=method, save_mode=gncde._lib.SAVE_STEPS,
                            grid=torch.tensor(z["grid"], device="cuda"), nsteps=torch.tensor(z["nsteps"], device="cuda"))
    assert gncde.integrate_path(prob, spec) == "generic_bf16"
    ys = gncde.integrate(prob, spec, torch.tensor(z["y0"], dtype=torch.float32, device="cuda"))
    err = rel_err(ys.cpu().numpy(), z["ys"])
    print(f"{name} bf16 solve: rel err {err:.3e}")
    assert err <= RTOL_BF16_SOLVE


def test_bf16_pid_cde(gncde, golden_dir):
    """Adaptive Tsit5 + PID on the bf16 path: the split products leave no rounding noise for the error
    estimate, so the controller takes the fp32 path's steps and reaches the oracle's accuracy."""
    z = np.load(os.path.join(golden_dir, "pid_cde_n10_h8_de2.npz"))
    params = MG.load_layers(z)
    prob = problem_from(gncde, z, params, data=True).with_compute("bf16")
    ts = torch.tensor(z["ts"], dtype=torch.float32, device="cuda")
    dt0 = float(z["dt0"])
    spec = gncde.SolverSpec(method=gncde._lib.TSIT5, controller=gncde._lib.CTRL_PID, save_mode=gncde._lib.SAVE_T1,
                            rtol=float(z["rtol"]), atol=float(z["atol"]), t0=ts[:, 0].contiguous(),
                            t1=ts[:, -1].contiguous(),
                            dt0=None if np.isnan(dt0) else torch.full((ts.shape[0],), dt0, device="cuda"))
    ys, st = gncde.integrate(prob, spec, torch.tensor(z["y0"], dtype=torch.float32, device="cuda"), stats=True)
    st = st.cpu().numpy()
    assert np.all(st[:, 3] == 0)
    acc = rel_err(ys.cpu().numpy(), z["truth"][:, -1])
    print(f"pid cde bf16: rel err vs near-exact {acc:.3e}, steps {st[:, :2].tolist()} oracle {z['stats'][:, :2].tolist()}")
    assert acc <= ACC_PID_FACTOR * float(z["ens_err"])
    assert np.all(np.abs(st[:, 0] - z["stats"][:, 0]) <= 0.25 * z["stats"][:, 0])


RTOL_BF16_SPLIT_CFG5_VF = 1e-3


@pytest.mark.parametrize("n", [255, 64])
def test_bf16_config5_shape_vs_fp32(gncde, n):
    """TGB-trade-shaped CDE (de = 8, the widening read-out layer reassociated) at n = 255 (unaligned rows: the
    scalar load path) and n = 64 (16-byte rows).  One evaluation: the bf16 path against the fp32 path on the same
    inputs.  This data (normalised Laplacians of log-normal weights) cancels heavily in (I + Abar) m, which scales
    the split products' 2^-16 up, hence RTOL_BF16_SPLIT_CFG5_VF.  A 20-step Tsit5 solve: finite; its deviation from the
    fp32 solve (and the bf16-storage solve's, i.e. the model's sensitivity to bf16 inputs) is printed."""
    from gncde import layout, synthetic
    prob, y0 = synthetic.cde_batch(4, n, 3, 32, 8, 4, 1.0)
    t = torch.full((prob.B,), 0.37, device="cuda")
    ref = gncde.vf_eval(prob, t, y0).cpu().numpy()
    got = gncde.vf_eval(prob.with_compute("bf16"), t, y0).cpu().numpy()
    err = rel_err(got, ref)
    grid, ns = layout.stack_grids([layout.constant_step_grid(0.0, 1.0, 0.05)] * prob.B)
    spec = gncde.SolverSpec(method=gncde._lib.TSIT5, save_mode=gncde._lib.SAVE_T1, grid=grid, nsteps=ns)
    yr = gncde.integrate(prob, spec, y0).cpu().numpy()
    yb = gncde.integrate(prob.with_compute("bf16"), spec, y0).cpu().numpy()
    yq = gncde.integrate(prob.with_compute("bf16_storage"), spec, y0).cpu().numpy()
    print(f"config-5 shape n={n}: one eval bf16 vs fp32 {err:.3e}; 20-step solve: bf16 {rel_err(yb, yr):.3e}, "
          f"bf16_storage {rel_err(yq, yr):.3e}")
    assert err <= RTOL_BF16_SPLIT_CFG5_VF
    assert np.isfinite(yb).all() and np.isfinite(yq).all()


# Reverse mode of the bf16 modes (gncde_abi.hip fp32_view): the fp32 discrete adjoint over the coefficients the
# bf16 forward read.  It must equal, bit for bit, the fp32 adjoint called on those coefficients (BF16: the fp32
# planes; BF16_STORAGE: the planes rounded to bf16 and widened) with the same checkpoints; fixtures cover the fused
# stage sweep (n = 16, h = 16), the generic sweep (mixed widths) and the CDE wrapper with the data-spline cotangent.
BF16_GRAD_CASES = [("rk4_undirected_n16_L2.npz", False), ("rk4_undirected_n12_mixed.npz", False),
                   ("grad_rk4_cde_data_n9_h4_de3.npz", True)]
RTOL_BF16_GRAD = 5e-4  # bf16 (split products) vs the fp32 solve's gradient: the forward's product rounding only


@pytest.mark.parametrize("mode", ["bf16", "bf16_storage"])
@pytest.mark.parametrize("name,data", BF16_GRAD_CASES)
def test_bf16_reverse_mode_is_fp32_adjoint_of_read_coefficients(gncde, golden_dir, name, data, mode):
    import dataclasses
    z = np.load(os.path.join(golden_dir, name))
    params = MG.load_layers(z)
    p32 = problem_from(gncde, z, params, data=data)
    pb = p32.with_compute(mode)
    spec = gncde.SolverSpec(method=gncde._lib.RK4 if str(z["method"]) == "rk4" else gncde._lib.TSIT5,
                            save_mode=gncde._lib.SAVE_STEPS,
                            grid=torch.tensor(z["grid"], device="cuda"), nsteps=torch.tensor(z["nsteps"], device="cuda"))
    y0 = torch.tensor(z["y0"], dtype=torch.float32, device="cuda")
    ys = gncde.integrate(pb, spec, y0)
    gys = torch.randn(ys.shape, generator=torch.Generator().manual_seed(7)).to("cuda")
    got = gncde.integrate_vjp(pb, spec, ys, gys, data_grad=data)
    ref_prob = p32 if mode == "bf16" else dataclasses.replace(p32, coef=p32.coef.to(torch.bfloat16).float().contiguous())
    ref = gncde.integrate_vjp(ref_prob, spec, ys, gys, data_grad=data)
    assert len(got) == len(ref) == (4 if data else 3)
    for g, r in zip(got, ref):
        assert torch.isfinite(g).all()
        assert torch.equal(g, r)
    if mode == "bf16":  # against the fp32 solve's own gradient (its own checkpoints)
        ys32 = gncde.integrate(p32, spec, y0)
        full = gncde.integrate_vjp(p32, spec, ys32, gys, data_grad=data)
        for g, r in zip(got, full):
            assert rel_err(g.cpu().numpy(), r.cpu().numpy()) <= RTOL_BF16_GRAD


# ---- GNCDE_COMPUTE_BF16_MFMA: single-plane bf16 products (the one-launch evaluation, csrc/gncde_rows.hip) ---------
# The mode rounds every matrix-product operand to bf16 (oracle/bf16_model.py states where).  Two bars, relative to
# the max magnitude of the reference tensor:
#   * against the fp64 MODEL of those rounding points on the same bf16 coefficients.  The GPU rounds fp32 values, the
#     model fp64 ones, so now and then an operand lands on the other side of a bf16 rounding boundary (a 2^-8 step),
#     and through the dense (I + Abar) of the next layer such a flip reaches every row.  How far that moves the output
#     is measured on the model itself: the same evaluation with every pre-rounding value perturbed by 2^-22 relative
#     (fp32-class noise) gives the model's own SPREAD, and the GPU must agree with the model within
#     max(AGREE_BF16M, 10 x spread).  Shallow cases measure ~1e-7 (no flip lands); an indexing or accumulation error
#     is O(1);
#   * against the fp64 ORACLE (exact products) on the same bf16 coefficients: RTOL_BF16M_EXACT (max) — the accuracy
#     the mode gives up for its throughput (~2^-8 per operand, grown by the cancellation in (I + Abar) Z).
AGREE_BF16M = 1e-4
RTOL_BF16M_EXACT = 5e-2
# The mode is retired from the product library (round 6, include/gncde.h): these checks run only against the
# experiment build (`make -C perm-equiv-graph-neural-cdes_amd experiment`, then GNCDE_LIB=build_exp/libgncde_hip.so
# GNCDE_LIB_UNVERIFIED=1 GNCDE_EXPERIMENT_BF16_MFMA=1); the product suite checks the refusal.
experiment_bf16m = pytest.mark.skipif(os.environ.get("GNCDE_EXPERIMENT_BF16_MFMA") != "1",
                                      reason="single-plane bf16 mode: experiment build only")


def test_bf16_mfma_refused_by_product_library(gncde, golden_dir):
    """The product library refuses the retired single-plane mode loudly (GNCDE_ERR_UNSUPPORTED), for an evaluation,
    a fixed-grid solve and path selection alike: never a silent fallback to another arithmetic."""
    if os.environ.get("GNCDE_EXPERIMENT_BF16_MFMA") == "1":
        pytest.skip("experiment build loaded")
    z = np.load(os.path.join(golden_dir, "cde_n33_h32_de8.npz"))
    params = MG.load_layers(z)
    prob = problem_from(gncde, z, params, data=True).with_compute("bf16_mfma")
    t = torch.tensor(z["t"], dtype=torch.float32, device="cuda")
    y = torch.tensor(z["y"], dtype=torch.float32, device="cuda")
    with pytest.raises(gncde._lib.GncdeError, match="not supported"):
        gncde.vf_eval(prob, t, y)
    B = prob.B
    spec = gncde.SolverSpec(method=gncde._lib.TSIT5, save_mode=gncde._lib.SAVE_T1,
                            grid=prob.ts[:, [0, -1]].contiguous(), nsteps=torch.ones(B, dtype=torch.int32, device="cuda"))
    with pytest.raises(gncde._lib.GncdeError):
        gncde.integrate_path(prob, spec)
    with pytest.raises(gncde._lib.GncdeError):
        gncde.integrate(prob, spec, y)


def rows_envelope(z, data):
    """The one-launch evaluation's shapes (gncde_rows.hip rows_supported): n <= 256, one width H in {16, 32, 64}
    for every hidden layer, and an ODE output of width H or the de = 8 read-out with h = H."""
    L = int(z["L"])
    n = z["y"].shape[1]
    dims = [z[f"l{l}_W"].shape[1] for l in range(L)] + [z[f"l{L - 1}_W"].shape[0]]
    H = dims[0]
    if n > 256 or H not in (16, 32, 64) or any(d != H for d in dims[:-1]):
        return False
    if data:
        return int(z["de"]) == 8 and int(z["h"]) == H and dims[-1] == 16 * H
    return dims[-1] == H


def bf16_model_vf(z, params, data, t, y, ts=None, coeffs=None, xcoeffs=None, noise_seed=None):
    """(fp64 oracle, fp64 bf16-rounding model) of one evaluation on the bf16-rounded coefficients; with noise_seed,
    the model's pre-rounding values are perturbed by +-2^-22 relative (its sensitivity to fp32-class differences)."""
    from oracle import bf16_model as BM
    ts = z["ts"] if ts is None else ts
    q = BM.coef_bf16(tuple(z[k] for k in ("d", "c", "b", "a")) if coeffs is None else coeffs)
    base = BM.bf16
    if noise_seed is not None:
        rng = np.random.default_rng(noise_seed)
        BM.bf16 = lambda x: base(np.asarray(x, np.float64) * (1.0 + 2.0 ** -22 * rng.choice([-1.0, 1.0], np.shape(x))))
    try:
        exact, model = [], []
        for b in range(ts.shape[0]):
            ctrl = O.CubicInterpolation(ts[b], tuple(c[b] for c in q))
            if data:
                xc = tuple(z[k] for k in ("xd", "xc", "xb", "xa")) if xcoeffs is None else xcoeffs
                h, de = (int(z["h"]), int(z["de"])) if xcoeffs is None else (y.shape[-1], 8)
                cx = O.CubicInterpolation(ts[b], tuple(c[b] for c in xc))
                exact.append(O.cde_wrapper(params, h, de, t[b], y[b], ctrl, cx))
                model.append(BM.cde_wrapper(params, h, de, t[b], y[b], ctrl, cx))
            else:
                exact.append(O.vector_field(params, t[b], y[b], ctrl))
                model.append(BM.vector_field(params, t[b], y[b], ctrl))
    finally:
        BM.bf16 = base
    return np.stack(exact), np.stack(model)


def check_vs_model(label, dy, args, kwargs):
    exact, model = bf16_model_vf(*args, **kwargs)
    _, noisy = bf16_model_vf(*args, noise_seed=0, **kwargs)
    em, ee, spread = rel_err(dy, model), rel_err(dy, exact), rel_err(noisy, model)
    bound = max(AGREE_BF16M, 10.0 * spread)
    print(f"{label} bf16_mfma: vs rounding model {em:.3e} (bound {bound:.2e}: model spread {spread:.2e}), "
          f"vs exact products {ee:.3e}")
    assert em <= bound
    assert ee <= RTOL_BF16M_EXACT


BF16M_CASES = VF_CASES + [("vf_undirected_n4_L2.npz", False), ("cde_n20_h64_de8.npz", True)]


@experiment_bf16m
@pytest.mark.parametrize("name,data", BF16M_CASES)
def test_bf16_mfma_vf_eval_vs_rounding_model(gncde, golden_dir, name, data):
    z = np.load(os.path.join(golden_dir, name))
    params = MG.load_layers(z)
    prob = problem_from(gncde, z, params, data=data).with_compute("bf16_mfma")
    assert prob.coef.dtype == torch.bfloat16
    t = torch.tensor(z["t"], dtype=torch.float32, device="cuda")
    y = torch.tensor(z["y"], dtype=torch.float32, device="cuda")
    if not rows_envelope(z, data):  # no other kernel implements the mode: a loud refusal, never a fallback
        with pytest.raises(gncde._lib.GncdeError):
            gncde.vf_eval(prob, t, y)
        return
    dy = gncde.vf_eval(prob, t, y).cpu().numpy()
    check_vs_model(name, dy, (z, params, data, z["t"], z["y"]), {})


@experiment_bf16m
@pytest.mark.parametrize("n,H,cde", [(200, 32, False), (255, 32, True), (129, 64, True), (256, 16, False)])
def test_bf16_mfma_large_n_vs_rounding_model(gncde, n, H, cde):
    """n in (128, 256]: both 32-wide K chunks of every wave, odd n (funnel-shifted coefficient loads), the padded
    tail chunk; the H = 64 read-out (bf16 only)."""
    rng = np.random.default_rng(1000 + n + H)
    B, T, L = 2, 5, 3
    dims = [H] * L + [16 * H if cde else H]
    ts, coeffs, params = MG.problem(rng, B, n, T, "undirected", dims)
    y = rng.standard_normal((B, n, H))
    t = np.array([rng.uniform(ts[b, 0], ts[b, -1]) for b in range(B)], dtype=np.float32).astype(np.float64)
    xcoeffs = None
    kw = {}
    if cde:
        xs = [O.backward_hermite_coefficients(ts[b], rng.standard_normal((T, n, 8, 2))) for b in range(B)]
        xcoeffs = tuple(np.stack([x[q] for x in xs]) for q in range(4))
        kw = dict(data_coeffs=xcoeffs, cde_hidden=H, cde_embed=8)
    prob = gncde.make_problem(ts, coeffs, params.kind, params.layers, compute="bf16_mfma", **kw)
    assert gncde.integrate_path(prob, gncde.SolverSpec(
        method=gncde._lib.TSIT5, save_mode=gncde._lib.SAVE_T1,
        grid=torch.tensor(np.stack([ts[:, 0], ts[:, -1]], 1).astype(np.float32), device="cuda"),
        nsteps=torch.ones(B, dtype=torch.int32, device="cuda"))) == "rows_bf16"
    dy = gncde.vf_eval(prob, torch.tensor(t, dtype=torch.float32, device="cuda"),
                       torch.tensor(y, dtype=torch.float32, device="cuda")).cpu().numpy()
    check_vs_model(f"n={n} H={H} cde={cde}", dy, ({}, params, cde, t, y),
                   dict(ts=ts, coeffs=coeffs, xcoeffs=xcoeffs))


# one evaluation of the single-plane mode at L = 4: each of the L + 1 products rounds both operands to bf16 (unit
# roundoff 2^-8 each, so <= 2^-7 per product term relative to sum |a b|), and the errors add to first order through
# the stack (RMSNorm renormalises, it does not amplify): (L + 1) 2^-7 = 3.9e-2 when the sums do not cancel
# (measured 1.4e-2 at n = 255, 7.7e-3 at n = 64)
RTOL_BF16_CFG5_VF = 5 * 2.0 ** -7
BF16M_SOLVE_CAP = {255: 0.15, 64: 0.04}


@experiment_bf16m
@pytest.mark.parametrize("n", [255, 64])
def test_bf16_mfma_config5_shape_vs_fp32(gncde, n):
    """TGB-trade-shaped CDE (n = 255 / 64, h = 32, L = 4, de = 8): one evaluation and a 20-step Tsit5 solve in the
    single-plane mode against the fp32 path on the same (fp32) inputs.

    Bound on the solve's deviation: BF16M_SOLVE_CAP[n], about twice the deviation measured at HEAD (round 4:
    7.7e-2 at n = 255, 1.8e-2 at n = 64), so a regression of the mode's solve fails instead of hiding under a
    clamp.  The fp32 solve's own response to a 1-ulp change of y0 is printed for scale."""
    from gncde import layout, synthetic
    prob, y0 = synthetic.cde_batch(4, n, 3, 32, 8, 4, 1.0)
    t = torch.full((prob.B,), 0.37, device="cuda")
    ref = gncde.vf_eval(prob, t, y0).cpu().numpy()
    got = gncde.vf_eval(prob.with_compute("bf16_mfma"), t, y0).cpu().numpy()
    err = rel_err(got, ref)
    # a grid in fixed-step Tsit5's stable regime on this problem (h = 0.015; at h >= 0.05 the fp32 solve itself
    # amplifies a 1-ulp change of y0 x2000: see tests/test_gpu_configs.py)
    grid, ns = layout.stack_grids([layout.constant_step_grid(0.0, 0.3, 0.015)] * prob.B)
    spec = gncde.SolverSpec(method=gncde._lib.TSIT5, save_mode=gncde._lib.SAVE_T1, grid=grid, nsteps=ns)
    yr = gncde.integrate(prob, spec, y0).cpu().numpy()
    ym = gncde.integrate(prob.with_compute("bf16_mfma"), spec, y0).cpu().numpy()
    yq = gncde.integrate(prob.with_compute("bf16_storage"), spec, y0).cpu().numpy()
    sign = torch.where(torch.rand(y0.shape, generator=torch.Generator().manual_seed(9)) < 0.5, -1.0, 1.0).cuda()
    sens = rel_err(gncde.integrate(prob, spec, y0 * (1.0 + sign * 2.0 ** -24)).cpu().numpy(), yr)
    dev = rel_err(ym, yr)
    bound = BF16M_SOLVE_CAP[n]
    print(f"config-5 shape n={n}: one eval bf16_mfma vs fp32 {err:.3e}; 20-step solve: bf16_mfma {dev:.3e} "
          f"(bound {bound:.3e}; the fp32 1-ulp response {sens:.3e}), bf16_storage {rel_err(yq, yr):.3e}")
    assert np.isfinite(ym).all()
    assert err <= RTOL_BF16_CFG5_VF
    assert dev <= bound
