"""ctypes wrapper of oracle/build/libgncde_oracle.so (the C restatement) — TEST INFRASTRUCTURE ONLY.

Used by tests/test_c_oracle.py (cross-check vs the numpy oracle) and bench.py's cpu_baseline leg.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# GNCDE_ORACLE_LIB selects another build of the same source (the ASan/UBSan one: `make -C oracle asan`).
LIB = os.environ.get("GNCDE_ORACLE_LIB") or os.path.join(HERE, "build", "libgncde_oracle.so")
_lib = None


def build():
    target = os.path.relpath(LIB, HERE) if os.path.dirname(os.path.abspath(LIB)).startswith(HERE) else "all"
    subprocess.run(["make", "-C", HERE, "-s", target], check=True)


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        lib = ctypes.CDLL(LIB)
        f = lib.gncde_oracle_rk4
        f.restype = ctypes.c_long
        f.argtypes = [ctypes.c_int] * 4 + [ctypes.c_void_p] * 8 + [ctypes.c_int, ctypes.c_void_p,
                                                                    ctypes.c_void_p, ctypes.c_int]
        _lib = lib
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def raw_fusion_params(layers):
    """[L, 8, 2] float32: param1..param8 (undirected ConvEquivFusionLayer order)."""
    names = ("param1", "param2", "param3", "param4", "param5", "param6", "param7", "param8")
    return np.ascontiguousarray(np.array([[np.asarray(lay[nm]).reshape(2) for nm in names] for lay in layers],
                                         dtype=np.float32))


def packed_params(layers):
    return np.ascontiguousarray(np.concatenate(
        [np.concatenate([np.asarray(lay[k], dtype=np.float32).ravel() for k in ("rms_w", "rms_b", "W", "b")])
         for lay in layers]).astype(np.float32))


def rk4(ts, coef, tcoef, layers, grid, nsteps, y0, nthreads=0):
    """Fixed-grid RK4 for B samples (undirected PermEquivGraphVectorField).  Arrays in the engine layout
    (include/gncde.h).  Returns (yT [B, n, H] float32, number of VF evaluations)."""
    lib = load()
    ts = np.ascontiguousarray(ts, dtype=np.float32)
    coef = np.ascontiguousarray(coef, dtype=np.float32)
    tcoef = np.ascontiguousarray(tcoef, dtype=np.float32)
    grid = np.ascontiguousarray(grid, dtype=np.float32)
    nsteps = np.ascontiguousarray(nsteps, dtype=np.int32)
    y0 = np.ascontiguousarray(y0, dtype=np.float32)
    B, T = ts.shape
    n = coef.shape[-1]
    dims = np.array([np.asarray(layers[0]["W"]).shape[1]] + [np.asarray(l["W"]).shape[0] for l in layers],
                    dtype=np.int32)
    fp = raw_fusion_params(layers)
    pp = packed_params(layers)
    yT = np.empty_like(y0)
    nev = lib.gncde_oracle_rk4(B, n, T, len(layers), _p(dims), _p(ts), _p(coef), _p(tcoef), _p(fp), _p(pp),
                               _p(grid), _p(nsteps), grid.shape[1], _p(y0), _p(yT), int(nthreads))
    return yT, int(nev)
