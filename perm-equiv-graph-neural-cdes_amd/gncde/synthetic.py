"""Synthetic Heat-Diffusion-shaped inputs built directly in HBM (torch on the device).

Mirrors the reference's input construction for the dyn configs: a grid graph
(``data_tools.py`` 8-neighbour grid, N = ceil(sqrt(num_nodes)) per side, ``ode_dataset.py:56``) whose
edges drop/appear at random events, mapped through the normalised Laplacian (``misc.py:83-99``, the
default ``get_graph_operator``), sampled at irregular knots on [0, final_time], stacked with the time
channel and turned into backward-Hermite coefficients (``dataset_configs.py:147-173``).  Used by
bench.py and the GPU tests; values do not change the fixed-step work.
"""
from __future__ import annotations

import math

import torch

from . import engine, layout
from .engine import Problem


def grid_adjacency(side: int, device="cuda") -> torch.Tensor:
    """8-neighbour grid graph on side x side nodes (corner degree 3, centre 8)."""
    n = side * side
    A = torch.zeros(n, n, device=device)
    for r in range(side):
        for c in range(side):
            i = r * side + c
            for dr in (-1, 0, 1):
                for dc in (-1, 0, 1):
                    if dr == 0 and dc == 0:
                        continue
                    rr, cc = r + dr, c + dc
                    if 0 <= rr < side and 0 <= cc < side:
                        A[i, rr * side + cc] = 1.0
    return A


def community_adjacency(n: int, seed: int = 1234, device="cuda") -> torch.Tensor:
    """The reference's community graph on exactly n nodes (the gene-dynamics ``graph_type: community`` of
    SURVEY §8d C4): networkx.random_partition_graph([n/3, n/3, n/4, rest], 0.25, 0.01, seed) in the community
    layout (ode_dataset.py:189-202, data.community_graph)."""
    from .data import community_graph
    return torch.tensor(community_graph(n, seed, "community"), dtype=torch.float32, device=device)


def normalized_laplacian(A: torch.Tensor) -> torch.Tensor:
    """I - D_out^-1/2 (A + I) D_in^-1/2, batched over leading dims (misc.py:83-99)."""
    n = A.shape[-1]
    eye = torch.eye(n, device=A.device, dtype=A.dtype)
    Ap = A + eye
    dout = Ap.sum(-1).rsqrt()
    din = Ap.sum(-2).rsqrt()
    return eye - dout.unsqueeze(-1) * Ap * din.unsqueeze(-2)


def hermite_coefficients(ts: torch.Tensor, ys: torch.Tensor):
    """Backward-Hermite (d, c, b, a) over dim 1 of ys [B, T, ...] with ts [B, T] (torch restatement of
    diffrax.backward_hermite_coefficients, as used at dataset_configs.py:170)."""
    B, T = ts.shape
    shape = (B, T - 1) + (1,) * (ys.dim() - 2)
    dt = (ts[:, 1:] - ts[:, :-1]).reshape(shape)
    slope = (ys[:, 1:] - ys[:, :-1]) / dt
    deriv = torch.cat([slope[:, :1], slope[:, :-1]], dim=1)
    dd = slope - deriv
    return -dd / (dt * dt), 2.0 * dd / dt, deriv, ys[:, :-1]


def init_layers(kind: str, dims, generator: torch.Generator, fusion_scale: float = 1.0 / 15):
    """Reference init distributions: fusion U(-1,1)/15 (layers.py:86-95), Linear U(+-1/sqrt(d_in)),
    RMSNorm weight 1 / bias 0 (equinox defaults).  Host tensors."""
    names = {"undirected": ("param1", "param2", "param3", "param4", "param5", "param6", "param7", "param8"),
             "directed": ("param1", "param2", "param3", "param4", "param4_prime", "param5", "param5_prime",
                          "param6", "param6_prime", "param7", "param8"),
             "plain": ()}[kind]
    layers = []
    for l in range(len(dims) - 1):
        din, dout = dims[l], dims[l + 1]
        lim = 1.0 / math.sqrt(din)
        lay = {nm: fusion_scale * (2 * torch.rand(2, generator=generator, dtype=torch.float64) - 1) for nm in names}
        lay["W"] = (2 * torch.rand(dout, din, generator=generator, dtype=torch.float64) - 1) * lim
        lay["b"] = (2 * torch.rand(dout, generator=generator, dtype=torch.float64) - 1) * lim
        lay["rms_w"] = torch.ones(din, dtype=torch.float64)
        lay["rms_b"] = torch.zeros(din, dtype=torch.float64)
        layers.append(lay)
    return layers


def heat_batch(B: int, num_nodes: int = 64, hidden: int = 16, num_layers: int = 3, T: int = 120,
               final_time: float = 5.0, events: int = 12, kind: str = "undirected", seed: int = 1234,
               device="cuda", chunk: int = 128, graph: str = "grid"):
    """Returns (Problem, y0 [B, n, hidden], layers).  graph "grid": n = ceil(sqrt(num_nodes))^2 like the
    reference grid; "community": exactly num_nodes nodes in 4 blocks (config 4)."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    if graph == "grid":
        side = int(math.ceil(math.sqrt(num_nodes)))
        n = side * side
        base = grid_adjacency(side, device=device)
    elif graph == "community":
        n = num_nodes
        base = community_adjacency(n, seed=seed, device=device)
    else:
        raise ValueError(graph)
    inner = torch.sort(torch.rand(B, T - 2, generator=g) * final_time, dim=1).values
    ts = torch.cat([torch.zeros(B, 1), inner, torch.full((B, 1), final_time)], dim=1).to(device)
    coef = torch.empty(B, T - 1, 4, n, n, device=device)
    for s in range(0, B, chunk):
        e = min(B, s + chunk)
        b = e - s
        # edge-drop / edge-add events at random knots; adjacency constant between events
        ev = torch.sort(torch.randint(1, T, (b, events), generator=g), dim=1).values.to(device)
        which = torch.zeros(b, T, dtype=torch.long, device=device)
        which.scatter_add_(1, ev, torch.ones_like(ev))
        which = which.cumsum(1).clamp(max=events)  # event epoch per knot
        flips = (torch.rand(b, events + 1, n, n, generator=g) < 0.02).to(device)
        flips[:, 0] = False
        flips = flips.cumsum(1) % 2 == 1  # cumulative toggles per epoch
        A = torch.where(flips, 1.0 - base, base)  # [b, E+1, n, n]
        ops = engine.graph_operator(A, "norm_lap")  # [b, E+1, n, n] (gncde_graph_operator)
        X = torch.gather(ops, 1, which[:, :, None, None].expand(b, T, n, n))  # [b, T, n, n]
        coef[s:e] = engine.hermite_coefficients(ts[s:e], X)  # engine layout directly (gncde_hermite_coefficients)
        del A, ops, X
    # time channel: knots = ts -> d = c = 0, b = 1 exactly (column means identical)
    tcoef = torch.zeros(B, T - 1, 3, n, device=device)
    tcoef[:, :, 2] = 1.0
    dims = [hidden] * (num_layers + 1)
    layers = init_layers(kind, dims, g)
    fusion = layout.fusion_table(kind, layers, n).to(torch.float32).to(device).contiguous()
    params = layout.pack_params(layers, device=device)
    prob = Problem(ts=ts.contiguous(), coef=coef, tcoef=tcoef, fusion=fusion, params=params, dims=dims)
    y0 = torch.randn(B, n, hidden, generator=g).to(device)
    return prob, y0, layers


def to_reference_coeffs(prob: Problem, b: int):
    """One sample of a Problem back in the reference layout: (d, c, b, a) each [T-1, n, n, 2] (float64, host)."""
    co = prob.coef[b].double().cpu()
    tc = prob.tcoef[b].double().cpu()
    n = co.shape[-1]
    ts = prob.ts[b].double().cpu()
    out = []
    for q in range(4):
        time_ch = torch.zeros_like(co[:, q]) if q < 3 else ts[:-1, None, None].expand(-1, n, n)
        if q < 3:
            time_ch = tc[:, q, None, :].expand(-1, n, n).clone()
        out.append(torch.stack([time_ch, co[:, q]], dim=-1).numpy())
    return ts.numpy(), tuple(out)


def cde_batch(B: int, n: int, T: int, hidden: int, embed: int, num_layers: int, t1: float, kind: str = "undirected",
              seed: int = 1234, device="cuda", chunk: int = 16):
    """PGT/TGB-shaped CDE-wrapper batch: a community graph with log-normal edge weights
    whose edges toggle between knots, normalised-Laplacian operator path, node data x [T, n, embed] stacked
    with time into the data spline; knots evenly spaced on [0, t1].  Returns (Problem, y0 [B, n, hidden])."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    ts = torch.linspace(0.0, t1, T).repeat(B, 1).to(device)
    coef = torch.empty(B, T - 1, 4, n, n, device=device)
    base = community_adjacency(n, seed=seed, device=device)
    for s in range(0, B, chunk):
        e = min(B, s + chunk)
        b = e - s
        w = torch.exp(torch.randn(b, T, n, n, generator=g)).to(device)
        keep = (torch.rand(b, T, n, n, generator=g) > 0.05).to(device)
        A = base * w * keep
        coef[s:e] = engine.hermite_coefficients(ts[s:e], engine.graph_operator(A, "norm_lap"))
    tcoef = torch.zeros(B, T - 1, 3, n, device=device)
    tcoef[:, :, 2] = 1.0
    x = torch.randn(B, T, n, embed, generator=g).to(device)
    X = torch.stack([ts[:, :, None, None].expand(B, T, n, embed), x], dim=-1)
    data_coef = engine.hermite_coefficients(ts, X)  # [B, T-1, 4, n, de, 2]
    dims = [hidden] * num_layers + [hidden * embed * 2]
    layers = init_layers(kind, dims, g)
    fusion = layout.fusion_table(kind, layers, n).to(torch.float32).to(device).contiguous()
    params = layout.pack_params(layers, device=device)
    prob = Problem(ts=ts.contiguous(), coef=coef, tcoef=tcoef, fusion=fusion, params=params, dims=dims,
                   data_coef=data_coef, cde_hidden=hidden, cde_embed=embed)
    y0 = torch.randn(B, n, hidden, generator=g).to(device)
    return prob, y0
