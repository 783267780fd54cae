"""MI355X-native GNCDE integration engine (host side).

The compute lives in ``libgncde_hip.so`` (hand-written gfx950 HIP kernels behind the C-ABI of
``include/gncde.h``); this package packs reference-layout inputs into the engine's HBM layout and
mirrors the reference's module interface (``models.vector_fields.PermEquivGraphVectorField`` etc.).
There is no CPU fallback anywhere in this package.
"""
from . import _lib, layout  # noqa: F401
from ._lib import GncdeError  # noqa: F401
from .engine import (Problem, SolverSpec, integrate, integrate_path, interval_index,  # noqa: F401
                     make_problem, node_affine, vf_eval)

__all__ = ["Problem", "SolverSpec", "integrate", "integrate_path", "interval_index", "make_problem",
           "node_affine", "vf_eval", "layout", "GncdeError"]
