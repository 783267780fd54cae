"""GPU: the bf16 MFMA paths (GNCDE_COMPUTE_BF16 / _BF16_STORAGE / _BF16_MFMA, BASELINE config 5).

COMPUTE_BF16 runs the n x n products on v_mfma_f32_16x16x32_bf16 with both operands split into bf16 (hi, lo) pairs:
three products, fp32 accumulation, ~2^-16 relative per product, so it is held to fp32-class tolerances (5x the fp32
path's).  COMPUTE_BF16_STORAGE also quantises the operator coefficients to bf16; it is compared with the fp64 oracle
evaluated on the same bf16-rounded coefficients (the quantisation is an input change, not an arithmetic error).
Tolerances (relative to the max magnitude of the reference tensor):
  * one vector-field evaluation:   RTOL_BF16_VF    = 1e-4
  * a fixed-grid solve trajectory: RTOL_BF16_SOLVE = 5e-4
"""
import math
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


# one evaluation of the single-plane mode at L = 4: each of the L + 1 products rounds both operands to bf16 (unit
# roundoff 2^-8 each, so <= 2^-7 per product term relative to sum |a b|), and the errors add to first order through
# the stack (RMSNorm renormalises, it does not amplify): (L + 1) 2^-7 = 3.9e-2 when the sums do not cancel
# (measured 1.4e-2 at n = 255, 7.7e-3 at n = 64)
RTOL_BF16_CFG5_VF = 5 * 2.0 ** -7


@pytest.mark.parametrize("n", [255, 64])
def test_bf16_mfma_config5_shape_vs_fp32(gncde, n):
    """TGB-trade-shaped CDE (n = 255 / 64, h = 32, L = 4, de = 8): one evaluation and a 20-step Tsit5 solve in the
    single-plane mode against the fp32 path on the same (fp32) inputs.

    Bound on the solve's deviation, derived from the fp32 solve's own sensitivity: ``sens`` = its relative response
    to a relative 2^-24 (fp32 unit roundoff) perturbation of every element of y0.  The mode rounds operands to bf16
    (unit roundoff 2^-9, 2^15 times fp32's) at each of the solve's 121 evaluations; treating each as an independent
    perturbation of that size propagated like the initial one gives sqrt(121) * 2^15 * sens, and a factor 4 covers
    the operand count per product (the rounding of both operands and of the coefficients).  The deviation must
    also stay below 1 (a solve, not noise)."""
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
    bound = min(4.0 * math.sqrt(121) * 2.0 ** 15 * sens, 1.0)
    print(f"config-5 shape n={n}: one eval bf16_mfma vs fp32 {err:.3e}; 20-step solve: bf16_mfma {dev:.3e} "
          f"(bound {bound:.3e} from the fp32 1-ulp response {sens:.3e}), bf16_storage {rel_err(yq, yr):.3e}")
    assert np.isfinite(ym).all()
    assert err <= RTOL_BF16_CFG5_VF
    assert dev <= bound
