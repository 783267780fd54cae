"""The C restatement (bench.py's cpu_baseline) agrees with the numpy fp64 oracle."""
import os

import numpy as np

from oracle import c_oracle
from oracle import gncde_oracle as O
from tests.golden import make_golden as MG


def test_c_oracle_matches_numpy_oracle(golden_dir):
    z = np.load(os.path.join(golden_dir, "rk4_undirected_n10_L3.npz"))
    params = MG.load_layers(z)
    coef = np.stack([z["d"][..., 1], z["c"][..., 1], z["b"][..., 1], z["a"][..., 1]], axis=2)
    tcoef = np.stack([z["d"][..., 0].mean(-2), z["c"][..., 0].mean(-2), z["b"][..., 0].mean(-2)], axis=2)
    yT, nev = c_oracle.rk4(z["ts"], coef, tcoef, params.layers, z["grid"], z["nsteps"], z["y0"], nthreads=2)
    ref = z["ys"][:, -1]
    err = np.max(np.abs(yT - ref)) / np.max(np.abs(ref))
    assert err < 1e-4, err
    assert nev == int(4 * z["nsteps"].sum())
