"""MI355X-native GNCDE integration engine (host side).

The compute lives in ``libgncde_hip.so`` (hand-written gfx950 HIP kernels behind the C-ABI of
``include/gncde.h``); this package packs reference-layout inputs into the engine's HBM layout and
mirrors the reference's module interface (``models.vector_fields.PermEquivGraphVectorField`` etc.).
There is no CPU fallback anywhere in this package.
"""
from . import _lib, autograd, engine, layout, train  # noqa: F401
from ._lib import GncdeError  # noqa: F401
from .engine import (Problem, SolverSpec, clip_adamw, integrate, integrate_path, integrate_vjp,  # noqa: F401
                     interval_index, make_problem, node_affine, node_affine_grad, vf_eval)

__all__ = ["Problem", "SolverSpec", "integrate", "integrate_path", "integrate_vjp", "interval_index",
           "make_problem", "node_affine", "node_affine_grad", "clip_adamw", "vf_eval", "layout", "autograd",
           "train", "engine", "GncdeError"]
