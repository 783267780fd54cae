"""Vector fields with the reference's names, constructor kwargs and ``__call__(t, y, args)`` signature
(``src/models/vector_fields/*.py``), registered for ``getattr(vector_fields, name)`` lookup exactly
as ``VectorFieldCfg.build`` does (``src/configs/vector_field_configs.py:52``).

Single-sample calls route to ``gncde_vf_eval`` with B = 1; batched solves go through
``problem(...)`` + ``gncde.integrate`` (the fused persistent kernel).  No CPU path exists.
"""
from __future__ import annotations

import torch
from torch import nn

from ... import engine, layout
from ...interpolation import CubicInterpolation
from .layers import (ConvEquivFusionDirectedLayer, ConvEquivFusionLayer, ConvLayer,  # noqa: F401
                     PlainConvLayer, _gen)

__all__ = ["PermEquivGraphVectorField", "PermEquivDirGraphVectorField", "GraphVectorField",
           "CDEWrapperVectorField", "CubicInterpolation"]


class _GraphVectorFieldBase(nn.Module):
    layer_cls = ConvEquivFusionLayer
    kind = "undirected"

    def __init__(self, input_dim: int, hidden_dim: int, output_dim: int, num_layers: int, data_embed_dim: int,
                 num_nodes: int, enc_idx: bool = False, enc_type: str = "mlp", idx_dim: int = 512, *, key=None,
                 **kwargs):
        super().__init__()
        if enc_idx:
            # perm_equiv_graph_vector_field.py:69 comments out idx_enc but :105 uses it: the reference
            # path raises there too.
            raise NotImplementedError("enc_idx=True is broken in the reference (idx_enc never built)")
        g = _gen(key)
        dims = [input_dim] + [hidden_dim] * (num_layers - 1) + [output_dim]
        self.gnn_layers = nn.ModuleList(self.layer_cls(dims[l], dims[l + 1], key=g) for l in range(num_layers))
        self.data_embed_dim = data_embed_dim
        self.num_nodes = num_nodes
        self.enc_idx = enc_idx
        self.dims = dims

    # -- engine plumbing ----------------------------------------------------------------------------
    def layer_dicts(self):
        return [lay.as_dict() for lay in self.gnn_layers]

    def problem(self, control_adj: CubicInterpolation, control_data: CubicInterpolation | None = None,
                cde_hidden: int = 0, data_coef: torch.Tensor | None = None) -> engine.Problem:
        ts, coef, tcoef = control_adj.graph_layout()
        n = coef.shape[-1]
        dev = coef.device
        layers = self.layer_dicts()
        fusion = layout.fusion_table(self.kind, layers, n).to(torch.float32).to(dev).contiguous()
        params = layout.pack_params(layers, device=dev)
        dc = data_coef if data_coef is not None else (control_data.data_layout() if control_data is not None
                                                      else None)
        return engine.Problem(ts=ts, coef=coef, tcoef=tcoef, fusion=fusion, params=params, dims=list(self.dims),
                              data_coef=dc, cde_hidden=cde_hidden,
                              cde_embed=self.data_embed_dim if cde_hidden else 0)

    def problem_from_layout(self, ts: torch.Tensor, coef: torch.Tensor, tcoef: torch.Tensor,
                            data_coef: torch.Tensor | None = None, cde_hidden: int = 0) -> engine.Problem:
        """Problem over an engine-layout control (layout.control_from_knots / gncde.data) with this module's
        current parameters."""
        n = int(coef.shape[-1])
        dev = coef.device
        layers = self.layer_dicts()
        fusion = layout.fusion_table(self.kind, layers, n).to(torch.float32).to(dev).contiguous()
        params = layout.pack_params(layers, device=dev)
        return engine.Problem(ts=ts.to(dev, torch.float32).contiguous(), coef=coef.contiguous(),
                              tcoef=tcoef.contiguous(), fusion=fusion, params=params, dims=list(self.dims),
                              data_coef=data_coef, cde_hidden=cde_hidden,
                              cde_embed=self.data_embed_dim if cde_hidden else 0)

    def diff_tensors(self, n: int, device) -> tuple:
        """(params, fusion) as differentiable device tensors: the packed parameter buffer and the factored
        fusion table [L, 24] (layout.fusion_table_torch), for ``autograd.solve``."""
        params = torch.cat([lay.packed() for lay in self.gnn_layers]).to(device=device, dtype=torch.float32)
        fusion = layout.fusion_table_torch(self.kind, [lay.fusion_params() for lay in self.gnn_layers], n)
        return params, fusion.to(device=device, dtype=torch.float32)

    def __call__(self, t, y, args):
        """``vf(t, y [n, d_0], control) -> [n, d_L]`` for one sample (reference signature)."""
        prob = self.problem(args)
        yb = torch.as_tensor(y, dtype=torch.float32, device=prob.ts.device).reshape(1, *y.shape)
        tb = torch.as_tensor([float(t)], dtype=torch.float32, device=prob.ts.device)
        return engine.vf_eval(prob, tb, yb)[0]


class PermEquivGraphVectorField(_GraphVectorFieldBase):
    """``perm_equiv_graph_vector_field.py:10-129``."""

    layer_cls = ConvEquivFusionLayer
    kind = "undirected"


class PermEquivDirGraphVectorField(_GraphVectorFieldBase):
    """``perm_equiv_dir_graph_vector_field.py:10-130`` (11-term directed fusion)."""

    layer_cls = ConvEquivFusionDirectedLayer
    kind = "directed"


class GraphVectorField(_GraphVectorFieldBase):
    """``graph_vector_field.py:10-115``: ConvLayers driven by A + dA (no fusion parameters)."""

    kind = "plain"

    def __init__(self, input_dim, hidden_dim, output_dim, num_layers, data_embed_dim, num_nodes, enc_idx=False,
                 enc_type="mlp", idx_dim=512, *, key=None, **kwargs):
        nn.Module.__init__(self)
        if enc_idx:
            raise NotImplementedError("enc_idx=True is not part of the hot path")
        g = _gen(key)
        dims = [input_dim] + [hidden_dim] * (num_layers - 1) + [output_dim]
        self.gnn_layers = nn.ModuleList(ConvLayer(dims[l], dims[l + 1], key=g) for l in range(num_layers))
        self.data_embed_dim, self.num_nodes, self.enc_idx, self.dims = data_embed_dim, num_nodes, enc_idx, dims


class CDEWrapperVectorField(nn.Module):
    """``cde_wrapper_vector_field.py:5-26``: contracts the VF output [n, h, de, 2] with dX_data/dt."""

    def __init__(self, vector_field: _GraphVectorFieldBase, hidden_dim: int):
        super().__init__()
        self.vector_field = vector_field
        self.hidden_dim = hidden_dim

    def problem(self, control_adj, control_data, data_coef=None):
        return self.vector_field.problem(control_adj, control_data, cde_hidden=self.hidden_dim, data_coef=data_coef)

    def __call__(self, t, y, args):
        control_adj, control_data = args
        prob = self.problem(control_adj, control_data)
        yb = torch.as_tensor(y, dtype=torch.float32, device=prob.ts.device).reshape(1, *y.shape)
        tb = torch.as_tensor([float(t)], dtype=torch.float32, device=prob.ts.device)
        return engine.vf_eval(prob, tb, yb)[0]
