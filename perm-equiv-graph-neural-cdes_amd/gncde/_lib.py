"""ctypes binding of libgncde_hip.so (the C-ABI declared in include/gncde.h).

The library is built in-tree (``make -C perm-equiv-graph-neural-cdes_amd``) and loaded from this
directory.  There is deliberately NO fallback: if the shared object is missing, fails to load, or no
GPU is visible, every entry point raises.
"""
from __future__ import annotations

import ctypes
import glob
import hashlib
import os
import sys
from ctypes import POINTER, c_char_p, c_float, c_int32, c_size_t, c_void_p

MAX_LAYERS = 8
FC = 24
ABI_VERSION = 8

RK4, TSIT5 = 0, 1
CTRL_GRID, CTRL_PID = 0, 1
SAVE_T1, SAVE_STEPS, SAVE_TS = 0, 1, 2
FLAG_GENERIC = 1  # GncdeSolver.flags: force the generic forward and reverse sweep
COMPUTE_FP32, COMPUTE_BF16, COMPUTE_BF16_STORAGE, COMPUTE_BF16_MFMA = 0, 1, 2, 3  # GncdeProblem.compute (gncde.h)
BF16_COEF_MODES = (COMPUTE_BF16_STORAGE, COMPUTE_BF16_MFMA)  # modes whose coefficients are stored as bfloat16
STAT_STEPS, STAT_REJECTS, STAT_EVALS, STAT_STATUS = 0, 1, 2, 3
STATUS_OK, STATUS_MAX_STEPS, STATUS_NONFINITE, STATUS_STEP_RECORD = 0, 1, 2, 3
OP_NORM_LAP, OP_NORM_ADJ, OP_KIPF, OP_NORMALIZED_PLUS = 0, 1, 2, 3

LIB_NAME = "libgncde_hip.so"
LIB_PATH = os.environ.get("GNCDE_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), LIB_NAME)  # GNCDE_LIB: an alternative build of the same library (kernel experiments)

# Every symbol include/gncde.h declares (checked by tests/test_abi.py).
EXPORTED_SYMBOLS = (
    "gncde_abi_version",
    "gncde_strerror",
    "gncde_source_sha256",
    "gncde_integrate_path",
    "gncde_stage_record_floats",
    "gncde_activation_record_floats",
    "gncde_workspace_bytes",
    "gncde_vf_eval",
    "gncde_integrate",
    "gncde_vjp_workspace_bytes",
    "gncde_integrate_vjp",
    "gncde_integrate_vjp_data",
    "gncde_integrate_vjp_ex",
    "gncde_node_affine",
    "gncde_node_affine_grad",
    "gncde_adamw_workspace_bytes",
    "gncde_clip_adamw",
    "gncde_interval_index",
    "gncde_graph_operator",
    "gncde_hermite_coefficients",
    "gncde_hermite_coefficients_vjp",
)


class GncdeProblem(ctypes.Structure):
    _fields_ = [
        ("B", c_int32),
        ("n", c_int32),
        ("T", c_int32),
        ("L", c_int32),
        ("dims", c_int32 * (MAX_LAYERS + 1)),
        ("cde_hidden", c_int32),
        ("cde_embed", c_int32),
        ("ts", c_void_p),
        ("coef", c_void_p),
        ("tcoef", c_void_p),
        ("data_coef", c_void_p),
        ("fusion", c_void_p),
        ("params", c_void_p),
        ("compute", c_int32),
    ]


class GncdeSolver(ctypes.Structure):
    _fields_ = [
        ("method", c_int32),
        ("controller", c_int32),
        ("save_mode", c_int32),
        ("max_steps", c_int32),
        ("grid_len", c_int32),
        ("n_save", c_int32),
        ("rtol", c_float),
        ("atol", c_float),
        ("grid", c_void_p),
        ("nsteps", c_void_p),
        ("t0", c_void_p),
        ("t1", c_void_p),
        ("dt0", c_void_p),
        ("save_ts", c_void_p),
        ("step_ts", c_void_p),
        ("step_ts_len", c_int32),
        ("stage_rec", c_void_p),
        ("stage_rec_len", ctypes.c_int64),
        ("flags", c_int32),
        ("act_rec", c_void_p),
        ("act_rec_len", ctypes.c_int64),
        ("pid_ckpt", c_void_p),
        ("rec_steps", c_int32),
    ]


class GncdeError(RuntimeError):
    pass


_PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))  # perm-equiv-graph-neural-cdes_amd/


def source_files() -> list[str]:
    """The files whose bytes the library's build-provenance sha covers, in the Makefile's order (SHA_SRC)."""
    csrc = os.path.join(_PKG_ROOT, "csrc")
    files = sorted(glob.glob(os.path.join(csrc, "*.hip")) + glob.glob(os.path.join(csrc, "*.h")),
                   key=lambda f: os.path.basename(f))
    return files + [os.path.join(os.path.dirname(_PKG_ROOT), "include", "gncde.h")]


def source_sha256() -> str:
    """sha256 of the kernel sources in this tree (what `make` compiles into gncde_source_sha256())."""
    files = source_files()
    missing = [f for f in files if not os.path.exists(f)]
    if len(files) < 2 or missing:
        raise GncdeError(f"kernel sources not found ({missing or 'csrc/'}): cannot verify the library's build")
    h = hashlib.sha256()
    for f in files:
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()


def verify_provenance(lib) -> str:
    """Refuse a library that was not compiled from this tree's kernel sources.  An explicit experiment build
    (GNCDE_LIB with GNCDE_LIB_UNVERIFIED=1, tools/ab_*.sh only) is loaded with a warning instead."""
    built = lib.gncde_source_sha256().decode()
    if os.environ.get("GNCDE_LIB") and os.environ.get("GNCDE_LIB_UNVERIFIED") == "1":
        # The opt-out is checked first, so it also works where no csrc/ tree lies next to the package.
        try:
            tree = source_sha256()
        except GncdeError:
            tree = "no-sources"
        if built != tree:
            print(f"gncde: WARNING experiment library {LIB_PATH} built from sources {built[:16]}, tree "
                  f"{tree[:16]}", file=sys.stderr)
        return built
    tree = source_sha256()
    if built != tree:
        raise GncdeError(f"{LIB_PATH} was built from kernel sources {built[:16]}..., this tree's are "
                         f"{tree[:16]}...: rebuild with `make -C perm-equiv-graph-neural-cdes_amd`")
    return built


_lib = None


def load(path: str | None = None):
    """Load (once) and return the shared library; raise if it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise GncdeError(
            f"{p} not found: build it with `make -C perm-equiv-graph-neural-cdes_amd` "
            "(there is no CPU fallback for the GNCDE hot path)")
    lib = ctypes.CDLL(p)
    lib.gncde_abi_version.restype = c_int32
    lib.gncde_strerror.restype = c_char_p
    lib.gncde_strerror.argtypes = [c_int32]
    lib.gncde_source_sha256.restype = c_char_p
    lib.gncde_source_sha256.argtypes = []
    lib.gncde_integrate_path.restype = c_int32
    lib.gncde_integrate_path.argtypes = [POINTER(GncdeProblem), POINTER(GncdeSolver), c_char_p, c_size_t]
    lib.gncde_stage_record_floats.restype = c_size_t
    lib.gncde_stage_record_floats.argtypes = [POINTER(GncdeProblem), POINTER(GncdeSolver)]
    lib.gncde_activation_record_floats.restype = c_size_t
    lib.gncde_activation_record_floats.argtypes = [POINTER(GncdeProblem), POINTER(GncdeSolver)]
    lib.gncde_workspace_bytes.restype = c_size_t
    lib.gncde_workspace_bytes.argtypes = [POINTER(GncdeProblem), POINTER(GncdeSolver)]
    lib.gncde_vf_eval.restype = c_int32
    lib.gncde_vf_eval.argtypes = [POINTER(GncdeProblem), c_void_p, c_void_p, c_void_p, c_void_p, c_size_t,
                                  c_void_p]
    lib.gncde_integrate.restype = c_int32
    lib.gncde_integrate.argtypes = [POINTER(GncdeProblem), POINTER(GncdeSolver), c_void_p, c_void_p,
                                    c_void_p, c_void_p, c_size_t, c_void_p]
    lib.gncde_vjp_workspace_bytes.restype = c_size_t
    lib.gncde_vjp_workspace_bytes.argtypes = [POINTER(GncdeProblem), POINTER(GncdeSolver)]
    lib.gncde_integrate_vjp.restype = c_int32
    lib.gncde_integrate_vjp.argtypes = [POINTER(GncdeProblem), POINTER(GncdeSolver), c_void_p, c_void_p,
                                        c_void_p, c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]
    lib.gncde_integrate_vjp_data.restype = c_int32
    lib.gncde_integrate_vjp_data.argtypes = [POINTER(GncdeProblem), POINTER(GncdeSolver), c_void_p, c_void_p,
                                             c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]
    lib.gncde_integrate_vjp_ex.restype = c_int32
    lib.gncde_integrate_vjp_ex.argtypes = [POINTER(GncdeProblem), POINTER(GncdeSolver), c_void_p, c_void_p,
                                           c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_size_t,
                                           c_void_p]
    lib.gncde_node_affine.restype = c_int32
    lib.gncde_node_affine.argtypes = [c_int32, c_int32, c_int32, c_void_p, c_void_p, c_void_p, c_void_p,
                                      c_void_p]
    lib.gncde_node_affine_grad.restype = c_int32
    lib.gncde_node_affine_grad.argtypes = [c_int32, c_int32, c_int32, c_void_p, c_void_p, c_void_p, c_void_p,
                                           c_void_p, c_void_p, c_void_p]
    lib.gncde_adamw_workspace_bytes.restype = c_size_t
    lib.gncde_adamw_workspace_bytes.argtypes = [c_int32]
    lib.gncde_clip_adamw.restype = c_int32
    lib.gncde_clip_adamw.argtypes = [c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_int32, c_float, c_float,
                                     c_float, c_float, c_float, c_float, c_void_p, c_void_p, c_size_t, c_void_p]
    lib.gncde_interval_index.restype = c_int32
    lib.gncde_interval_index.argtypes = [c_void_p, c_int32, c_int32, c_void_p, c_void_p, c_void_p, c_int32,
                                         c_void_p]
    lib.gncde_graph_operator.restype = c_int32
    lib.gncde_graph_operator.argtypes = [c_int32, c_int32, c_int32, c_void_p, c_void_p, c_void_p, c_void_p]
    lib.gncde_hermite_coefficients.restype = c_int32
    lib.gncde_hermite_coefficients.argtypes = [c_int32, c_int32, c_int32, c_int32, c_void_p, c_void_p, c_void_p,
                                               c_void_p]
    lib.gncde_hermite_coefficients_vjp.restype = c_int32
    lib.gncde_hermite_coefficients_vjp.argtypes = [c_int32, c_int32, c_int32, c_int32, c_void_p, c_void_p,
                                                   c_void_p, c_void_p]
    v = lib.gncde_abi_version()
    if v != ABI_VERSION:
        raise GncdeError(f"ABI mismatch: library {v}, bindings {ABI_VERSION}")
    verify_provenance(lib)
    _lib = lib
    return lib


def check(rc: int):
    if rc != 0:
        msg = load().gncde_strerror(rc).decode()
        raise GncdeError(f"gncde error {rc}: {msg}")
