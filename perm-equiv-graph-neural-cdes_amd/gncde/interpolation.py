"""Device-resident control paths: the ``args`` object the vector fields receive.

``CubicInterpolation(ts, coeffs)`` mirrors ``diffrax.CubicInterpolation`` as constructed at
``graph_neural_cde.py:82`` / ``pgt_graph_neural_cde.py:105-106`` / ``tgb_graph_neural_cde.py:133-134``:
``coeffs`` is the ``backward_hermite_coefficients`` tuple (d, c, b, a).  It is packed ONCE into the
engine's HBM layout (``layout.pack_control``): operator channel ``coef [B,T-1,4,n,n]`` and the time
channel's column means ``tcoef [B,T-1,3,n]`` for graph controls (knots ``[T, n, n, 2]``), or
``[B,T-1,4,n,de,2]`` for a node-data control (knots ``[T, n, de, 2]``).  ``evaluate`` / ``derivative``
are provided for API compatibility (device tensors, diffrax interval rule).
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib, layout


def _tensor(x, device):
    return (x if torch.is_tensor(x) else torch.as_tensor(np.asarray(x))).to(device=device, dtype=torch.float32)


class CubicInterpolation:
    def __init__(self, ts, coeffs, device="cuda"):
        if not torch.cuda.is_available():
            raise _lib.GncdeError("CubicInterpolation lives in HBM: no HIP device visible")
        self.ts = _tensor(ts, device).contiguous()
        self.coeffs = tuple(_tensor(c, device) for c in coeffs)  # (d, c, b, a)
        self._packed = {}

    @classmethod
    def from_layout(cls, ts, coef=None, tcoef=None, data_coef=None):
        """A control already in the engine layout (e.g. from ``layout.control_from_knots`` /
        ``engine.hermite_coefficients``): graph (ts [B,T], coef [B,T-1,4,n,n], tcoef [B,T-1,3,n]) or node data
        (ts, data_coef [B,T-1,4,n,de,2]).  ``coeffs`` stays empty: evaluate/derivative are not available."""
        self = cls.__new__(cls)
        self.ts = _tensor(ts, "cuda").contiguous()
        self.coeffs = ()
        self._packed = {}
        if coef is not None:
            self._packed["graph"] = (self.ts, coef.contiguous(), tcoef.contiguous())
        if data_coef is not None:
            self._packed["data"] = data_coef.contiguous()
        return self

    @property
    def batched(self) -> bool:
        return self.ts.dim() == 2

    def _index(self, t):
        ts = self.ts if not self.batched else self.ts[0]
        t = torch.as_tensor(t, dtype=torch.float32, device=ts.device).reshape(1)
        i = torch.searchsorted(ts, t, side="left") - 1
        return int(i.clamp(0, ts.shape[0] - 2).item()), float(t.item()) - float(ts[i.clamp(0, ts.shape[0] - 2)])

    def evaluate(self, t):
        """X(t) = a + f (b + f (c + f d)) on the active interval (single-sample control)."""
        d, c, b, a = self.coeffs
        i, f = self._index(t)
        return a[i] + f * (b[i] + f * (c[i] + f * d[i]))

    def derivative(self, t):
        """X'(t) = b + f (2c + 3 f d)."""
        d, c, b, a = self.coeffs
        i, f = self._index(t)
        return b[i] + f * (2.0 * c[i] + 3.0 * f * d[i])

    # -- engine layouts ----------------------------------------------------------------------------
    def graph_layout(self):
        """(ts [B,T], coef [B,T-1,4,n,n], tcoef [B,T-1,3,n]) — packed on first use."""
        if "graph" not in self._packed:
            coef, tcoef = layout.pack_control(self.coeffs, device=self.ts.device)
            ts = self.ts if self.batched else self.ts.unsqueeze(0)
            self._packed["graph"] = (ts.contiguous(), coef, tcoef)
        return self._packed["graph"]

    def data_layout(self):
        """[B, T-1, 4, n, de, 2] for a node-data control (CDE wrapper)."""
        if "data" not in self._packed:
            self._packed["data"] = layout.pack_data_control(self.coeffs, device=self.ts.device)
        return self._packed["data"]
