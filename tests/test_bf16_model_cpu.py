"""CPU: the fp64 model of GNCDE_COMPUTE_BF16_MFMA's rounding points (oracle/bf16_model.py).

With its bf16 rounding switched off the model must be the reference vector field restated by the oracle
(gncde_oracle.vector_field / cde_wrapper): its reassociation (RMSNorm folded into W', the bias through
q = (I + Abar) 1, the de = 8 read-out contracted without forming the widening layer) is exact algebra.  With rounding
on, it must differ by the ~2^-8 the mode defines — not more, not zero.
"""
import os

import numpy as np
import pytest

from oracle import bf16_model as BM
from oracle import gncde_oracle as O
from tests.golden import make_golden as MG


def _eval(z, params, data, model):
    out = []
    for b in range(z["ts"].shape[0]):
        ctrl = O.CubicInterpolation(z["ts"][b], tuple(z[k][b] for k in ("d", "c", "b", "a")))
        if data:
            cx = O.CubicInterpolation(z["ts"][b], tuple(z[k][b] for k in ("xd", "xc", "xb", "xa")))
            out.append(model.cde_wrapper(params, int(z["h"]), int(z["de"]), z["t"][b], z["y"][b], ctrl, cx))
        else:
            out.append(model.vector_field(params, z["t"][b], z["y"][b], ctrl))
    return np.stack(out)


@pytest.mark.parametrize("name,data", [("vf_undirected_n16_L3.npz", False), ("vf_directed_n48_h64_L2.npz", False),
                                       ("cde_n33_h32_de8.npz", True), ("cde_n20_h64_de8.npz", True)])
def test_model_without_rounding_is_the_oracle(golden_dir, name, data, monkeypatch):
    z = np.load(os.path.join(golden_dir, name))
    params = MG.load_layers(z)
    ref = _eval(z, params, data, O)
    np.testing.assert_allclose(ref, z["dy"], rtol=0, atol=1e-9 * np.abs(z["dy"]).max())
    rounded = _eval(z, params, data, BM)
    monkeypatch.setattr(BM, "bf16", lambda x: np.asarray(x, dtype=np.float64))
    exact = _eval(z, params, data, BM)
    scale = np.abs(ref).max()
    assert np.abs(exact - ref).max() <= 1e-10 * scale
    dev = np.abs(rounded - ref).max() / scale
    assert 1e-5 < dev < 5e-2, dev


def test_bf16_rounding_is_nearest_even():
    x = np.array([1.0, 1.0 + 2 ** -8, 1.0 + 3 * 2 ** -8, -2.5, 1.0 + 2 ** -8 + 2 ** -20], dtype=np.float32)
    np.testing.assert_array_equal(BM.bf16(x), [1.0, 1.0, 1.0 + 2 ** -6, -2.5, 1.0 + 2 ** -7])
