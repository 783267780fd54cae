"""Parameter containers mirroring ``src/models/vector_fields/layers.py`` (leaf names kept).

The arithmetic of these layers runs inside the HIP kernels (the fused integrate kernel or the generic
VF path); these modules only own the parameters, initialised with the reference's distributions:
fusion params U(-1, 1)/15 (layers.py:86-95, :223-247), ``eqx.nn.Linear`` U(+-1/sqrt(d_in)) (torch's
nn.Linear default is the same distribution), ``eqx.nn.RMSNorm`` weight 1 / bias 0.
"""
from __future__ import annotations

import torch
from torch import nn


def _gen(key):
    if isinstance(key, torch.Generator):
        return key
    g = torch.Generator()
    g.manual_seed(int(key) if key is not None else 0)
    return g


def _fusion_param(g):
    return nn.Parameter(1.0 / 15.0 * (2.0 * torch.rand(2, generator=g) - 1.0))


class RMSNorm(nn.Module):
    """equinox ``nn.RMSNorm(shape)``: x * rsqrt(mean(x^2) + 1e-5) * weight + bias."""

    def __init__(self, dim: int, eps: float = 1e-5):
        super().__init__()
        self.eps = eps
        self.weight = nn.Parameter(torch.ones(dim))
        self.bias = nn.Parameter(torch.zeros(dim))


class ConvLayer(nn.Module):
    """``ConvLayer`` (layers.py:11-48): RMSNorm -> Linear -> m + adj @ m."""

    def __init__(self, input_dim: int, output_dim: int, *, key=None):
        super().__init__()
        g = _gen(key)
        self.linear = nn.Linear(input_dim, output_dim)
        lim = 1.0 / input_dim ** 0.5
        with torch.no_grad():
            self.linear.weight.copy_((2 * torch.rand(output_dim, input_dim, generator=g) - 1) * lim)
            self.linear.bias.copy_((2 * torch.rand(output_dim, generator=g) - 1) * lim)
        self.norm = RMSNorm(input_dim)

    def as_dict(self):
        return {"W": self.linear.weight.detach(), "b": self.linear.bias.detach(),
                "rms_w": self.norm.weight.detach(), "rms_b": self.norm.bias.detach()}

    def fusion_params(self):
        return []  # GraphVectorField: A + dA, no fusion parameters

    def packed(self) -> torch.Tensor:
        """Differentiable packed parameters in the engine layout (rms_w, rms_b, W row-major, b; gncde.h)."""
        return torch.cat([self.norm.weight, self.norm.bias, self.linear.weight.reshape(-1), self.linear.bias])


class ConvEquivFusionLayer(nn.Module):
    """``ConvEquivFusionLayer`` (layers.py:51-177): 8 (A, dA) coefficient pairs + ConvLayer."""

    names = ("param1", "param2", "param3", "param4", "param5", "param6", "param7", "param8")
    kind = "undirected"

    def __init__(self, input_dim: int, output_dim: int, *, key=None):
        super().__init__()
        g = _gen(key)
        for nm in self.names:
            setattr(self, nm, _fusion_param(g))
        self.conv_layer = ConvLayer(input_dim, output_dim, key=g)

    def as_dict(self):
        d = {nm: getattr(self, nm).detach() for nm in self.names}
        d.update(self.conv_layer.as_dict())
        return d

    def fusion_params(self):
        return [getattr(self, nm) for nm in self.names]

    def packed(self) -> torch.Tensor:
        return self.conv_layer.packed()


class ConvEquivFusionDirectedLayer(ConvEquivFusionLayer):
    """``ConvEquivFusionDirectedLayer`` (layers.py:180-362): 11 coefficient pairs.  As in the reference
    (layers.py:245-247) ``param6_prime`` is drawn from ``param5_prime``'s key, i.e. equal at init."""

    names = ("param1", "param2", "param3", "param4", "param4_prime", "param5", "param5_prime", "param6",
             "param6_prime", "param7", "param8")
    kind = "directed"

    def __init__(self, input_dim: int, output_dim: int, *, key=None):
        nn.Module.__init__(self)
        g = _gen(key)
        for nm in self.names:
            if nm == "param6_prime":
                self.param6_prime = nn.Parameter(self.param5_prime.detach().clone())
            else:
                setattr(self, nm, _fusion_param(g))
        self.conv_layer = ConvLayer(input_dim, output_dim, key=g)


class PlainConvLayer(nn.Module):
    """A ConvLayer driven by the unfused message matrix A + dA (``GraphVectorField``)."""

    kind = "plain"

    def __init__(self, input_dim: int, output_dim: int, *, key=None):
        super().__init__()
        self.conv_layer = ConvLayer(input_dim, output_dim, key=key)

    def as_dict(self):
        return self.conv_layer.as_dict()

    def fusion_params(self):
        return []

    def packed(self) -> torch.Tensor:
        return self.conv_layer.packed()
