"""Dynamical-system graph datasets: heat diffusion and gene regulation on grid / community
graphs whose edges change at random events, sampled at equal or irregular times — restating
``src/dataset/ode_dataset.py`` (ODEDataset), ``src/dataset/data_tools.py`` (grid graph, events) and the
graph-path preparation of ``src/configs/dataset_configs.py:107-199`` (padding by events, graph operator,
backward-Hermite coefficients).

The ground truth restates the reference's solve (ode_dataset.py:251-300, gen_all_data :388-470):
``diffrax.diffeqsolve(ODETerm, cfg.method (Tsit5 | Dopri5), dt0=cfg.dt0, SaveAt(ts=t))`` with diffrax's default
ConstantStepSize controller, per sample, one solve per event segment of the time axis, each segment starting from
the previous segment's LAST saved state (gen_all_data's hand-over: the state jumps unchanged across the gap between
the last time of one segment and the first of the next).  It runs batched in float64 torch on the device (data
generation, not the hot path).  The graph operators and spline coefficients go through the engine's kernels
(``gncde_graph_operator``, ``gncde_hermite_coefficients``) straight into the engine layout.  Community graphs are
the reference's own (ode_dataset.py:189-202): ``networkx.random_partition_graph([n/3, n/3, n/4, rest], 0.25, 0.01,
seed=seed + i)`` for sample i, reordered by ``networkx_reorder_nodes(G, layout)`` (data_tools.py:32-72; the dyn
YAMLs set ``layout: community``, greedy-modularity order).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field, fields

import numpy as np
import torch

from . import engine, layout


@dataclass
class DynDataCfg:
    """The ``dataset:`` block of configs/dynamical_systems/*.yaml (unknown keys are ignored)."""

    name: str = "heat"
    batch_size: int = 4
    dynamic_graph: bool = True
    all_dynamic: bool = True
    graph_type: str = "grid"
    split_ratio: tuple = (0.8, 0.2)
    num_nodes: int = 400
    final_time: float = 5.0
    time_tick: int = 100
    sampling_type: str = "irregular"
    method: str = "Dopri5"  # dataset_configs.py:70-73 default; the dyn YAMLs set Tsit5
    operator_type: str = "norm_lap"
    seed: int = 1234
    padding_mode: str = "same"
    interpolation: str = "cubic"
    amp_range: tuple = (1.0, 1.0)
    layout: str | None = None  # node reordering of generated graphs: "community" | "degree" | None (data_tools.py:32)
    dt0: float = 0.01  # dataset_configs.py:74 (ConstantStepSize step of the ground-truth solve)

    @classmethod
    def from_dict(cls, d: dict) -> "DynDataCfg":
        names = {f.name for f in fields(cls)}
        return cls(**{k: v for k, v in (d or {}).items() if k in names})


def grid_8_neighbor_graph(N: int) -> np.ndarray:
    """data_tools.py:8-30: N x N grid, 8-neighbour connectivity."""
    A = np.zeros((N * N, N * N))
    for r in range(N):
        for c in range(N):
            for dr in (-1, 0, 1):
                for dc in (-1, 0, 1):
                    if (dr or dc) and 0 <= r + dr < N and 0 <= c + dc < N:
                        A[r * N + c, (r + dr) * N + c + dc] = 1.0
    return A


def reorder_nodes(G, kind=None):
    """networkx_reorder_nodes (data_tools.py:55-72) with generate_node_mapping (:32-52): a label -> position map by
    descending degree ("degree") or greedy-modularity community ("community"); None keeps G.  The reference applies
    that map to the COO row / column POSITIONS of nx.to_scipy_sparse_array(G) (positions in G's node order, which
    for random_partition_graph is not sorted), i.e. a position is looked up as if it were a label; that quirk is
    kept, since it decides which adjacency the model sees."""
    import networkx as nx
    import scipy.sparse as sp
    if kind == "degree":
        order = [v for v, _ in sorted(G.degree, key=lambda x: x[1], reverse=True)]
    elif kind == "community":
        order = [v for c in nx.community.greedy_modularity_communities(G) for v in c]
    else:
        return G
    pos = {v: i for i, v in enumerate(order)}
    C = nx.to_scipy_sparse_array(G, format="coo")
    remap = np.vectorize(lambda x: pos[int(x)], otypes=[np.int64])
    return nx.from_scipy_sparse_array(sp.coo_matrix((C.data, (remap(C.row), remap(C.col))), shape=C.shape))


def community_graph(n: int, seed: int, layout_kind=None) -> np.ndarray:
    """ODEDataset._gen_community_graph for one sample (ode_dataset.py:189-202): four blocks of n/3, n/3, n/4 and
    the rest nodes, edge probability 0.25 inside a block and 0.01 across, networkx's generator with this seed
    (the reference passes seed + i for sample i), then the layout reordering.  Dense [n, n] float adjacency."""
    import networkx as nx
    n1, n2, n3 = int(n / 3), int(n / 3), int(n / 4)
    G = nx.random_partition_graph([n1, n2, n3, n - n1 - n2 - n3], 0.25, 0.01, seed=seed)
    G = reorder_nodes(G, layout_kind)
    return np.array(nx.to_numpy_array(G), dtype=float)


def events_happen_time(rng, t: np.ndarray, event_times: int, split_ratio, all_dynamic: bool):
    """data_tools.py:75-108 (the returned indices are the last batch row's, as in the reference)."""
    B, num_t = t.shape
    n_train = int(num_t * split_ratio[0])
    if not all_dynamic:
        idx = (rng.permutation(n_train - 2) + 2)[:event_times]
        return t[:, np.sort(idx)], np.sort(idx)
    train_events = math.ceil(event_times * split_ratio[0])
    test_events = event_times - train_events
    ev_t = []
    for i in range(B):
        tr = rng.permutation(n_train - 2) + 2
        te = rng.permutation(num_t - n_train) + n_train
        idx = np.sort(np.concatenate((tr[:train_events], te[:test_events])))
        ev_t.append(t[i, idx])
    return np.stack(ev_t), idx


def events_happen_graph(rng, A: np.ndarray, event_times: int, p: float):
    """data_tools.py:111-158: each event drops edges with prob 20 p and adds edges with prob p."""
    out = [A.copy()]
    for _ in range(event_times):
        A_new = A.copy()
        A_new[rng.random(A.shape) < 20 * p] = 0.0
        A_new[rng.random(A.shape) < p] = 1.0
        out.append(A_new.copy())
        A = A_new
    return np.stack(out, axis=1)  # [B, E+1, n, n]


def split_indices(rng, sampling_type: str, time_tick: int, split_ratio):
    """ode_dataset.py:344-386 -> (id_train, id_test_extra, id_test_inter)."""
    if sampling_type == "equal":
        k = round(time_tick * split_ratio[0])
        return list(range(k)), list(range(k, time_tick)), None
    extra = list(range(time_tick, round(time_tick * (1.0 + split_ratio[1]))))
    inter = sorted(rng.permutation(list(range(1, time_tick)))[: round(time_tick * split_ratio[1])].tolist())
    train = sorted(set(range(time_tick)) - set(inter))
    return train, extra, inter


def padding_by_time(num_knots: int, events_indices: np.ndarray) -> np.ndarray:
    """dataset_configs.py:107-150 (padding_mode 'same'): epoch of every knot, events beyond the knots
    invisible (prepare_graph_path's truncation)."""
    visible = events_indices[events_indices < num_knots]
    mark = np.zeros(num_knots, dtype=np.int64)
    mark[visible] = 1
    return np.cumsum(mark)


# ---- diffrax.diffeqsolve(ODETerm, Tsit5 | Dopri5, ConstantStepSize(dt0), SaveAt(ts)) restated (data side) ------------
_TSIT5_C = (0.0, 0.161, 0.327, 0.9, 0.9800255409045097, 1.0, 1.0)
_TSIT5_A = ((), (0.161,), (-0.008480655492356989, 0.335480655492357),
            (2.897153057105493, -6.359448489975075, 4.3622954328695815),
            (5.325864828439257, -11.748883564062828, 7.4955393428898365, -0.09249506636175525),
            (5.86145544294642, -12.92096931784711, 8.159367898576159, -0.071584973281401, -0.028269050394068383),
            (0.09646076681806523, 0.01, 0.4798896504144996, 1.379008574103742, -3.290069515436081, 2.324710524099774))
_DOPRI5_C = (0.0, 0.2, 0.3, 0.8, 8.0 / 9.0, 1.0, 1.0)
_DOPRI5_A = ((), (0.2,), (3.0 / 40.0, 9.0 / 40.0), (44.0 / 45.0, -56.0 / 15.0, 32.0 / 9.0),
             (19372.0 / 6561.0, -25360.0 / 2187.0, 64448.0 / 6561.0, -212.0 / 729.0),
             (9017.0 / 3168.0, -355.0 / 33.0, 46732.0 / 5247.0, 49.0 / 176.0, -5103.0 / 18656.0),
             (35.0 / 384.0, 0.0, 500.0 / 1113.0, 125.0 / 192.0, -2187.0 / 6784.0, 11.0 / 84.0))
# Dopri5 dense output: the midpoint y(t + h/2) from these weights, then the quartic through y0, y1, y_mid, f0, f1
_DOPRI5_CMID = (6025192743.0 / 30085553152.0 / 2, 0.0, 51252292925.0 / 65400821598.0 / 2,
                -2691868925.0 / 45128329728.0 / 2, 187940372067.0 / 1594534317056.0 / 2,
                -1776094331.0 / 19743644256.0 / 2, 11237099.0 / 235043384.0 / 2)


def _tsit5_dense(th):
    t2 = th * th
    return torch.stack([
        -1.0530884977290216 * th * (th - 1.3299890189751412) * (t2 - 1.4364028541716351 * th + 0.7139816917074209),
        0.1017 * t2 * (t2 - 2.1966568338249754 * th + 1.2949852507374631),
        2.490627285651252793 * t2 * (t2 - 2.38535645472061657 * th + 1.57803468208092486),
        -16.54810288924490272 * (th - 1.21712927295533244) * (th - 0.61620406037800089) * t2,
        47.37952196281928122 * (th - 1.203071208372362603) * (th - 0.658047292653547382) * t2,
        -34.87065786149660974 * (th - 1.2) * (th - 0.666666666666666667) * t2,
        2.5 * (th - 1.0) * (th - 0.6) * t2], dim=-1)


def _dense(method, th, h, y0, y1, K):
    """y(t + th h) inside one step from its start / end states and its 7 stage values K [7, ...]."""
    if method == "tsit5":
        w = _tsit5_dense(th.reshape(-1))  # [m, 7]
        return y0 + h * torch.einsum("mj,jm...->m...", w, K)
    ymid = y0 + h * sum(c * K[j] for j, c in enumerate(_DOPRI5_CMID) if c != 0.0)
    f0, f1 = h * K[0], h * K[6]
    a = 2.0 * (f1 - f0) - 8.0 * (y1 + y0) + 16.0 * ymid
    b = 5.0 * f0 - 3.0 * f1 + 18.0 * y0 + 14.0 * y1 - 32.0 * ymid
    c = f1 - 4.0 * f0 - 11.0 * y0 - 5.0 * y1 + 16.0 * ymid
    return y0 + th * (f0 + th * (c + th * (b + th * a)))


def diffeqsolve_constant(f, ts: np.ndarray, y0: torch.Tensor, method: str = "Tsit5", dt0: float = 0.01):
    """Per sample b: diffrax.diffeqsolve(ODETerm(f), method, t0=ts[b, 0], t1=ts[b, -1], dt0, y0[b],
    SaveAt(ts=ts[b])) with the default ConstantStepSize (ode_dataset.py:279-293).  f is autonomous (heat / gene,
    batched over samples); the step grids follow ConstantStepSize (t + dt0 in fp32, snapped to t1 within 1e-6) and
    the save times are read off the solver's dense interpolant (Tsit5: its free interpolant; Dopri5: the quartic
    through y0, y1, f0, f1 and the Dopri5 midpoint).  ts [B, S] (numpy), y0 [B, ...] -> [B, S, ...]."""
    m = method.lower()
    if m not in ("tsit5", "dopri5"):
        raise NotImplementedError(f"ground-truth solver {method}: Tsit5 and Dopri5 are restated")
    A = _TSIT5_A if m == "tsit5" else _DOPRI5_A
    B, S = ts.shape
    dev = y0.device
    grids = [layout.constant_step_grid(float(ts[b, 0]), float(ts[b, -1]), dt0).astype(np.float64) for b in range(B)]
    ns = np.array([len(g) - 1 for g in grids])
    G = int(ns.max()) + 1
    grid = np.stack([np.concatenate([g, np.full(G - len(g), g[-1])]) for g in grids])
    # the step of every save time: t_k < ts <= t_{k+1} (k = -1: ts <= t0, the initial state)
    kk = np.full((B, S), -1, dtype=np.int64)
    th = np.zeros((B, S))
    for b in range(B):
        tsb = np.asarray(ts[b], np.float64)
        for s_ in range(S):
            if tsb[s_] <= grid[b, 0] or ns[b] == 0:
                continue
            k = min(max(int(np.searchsorted(grid[b, :ns[b] + 1], tsb[s_], side="left")) - 1, 0), ns[b] - 1)
            kk[b, s_] = k
            th[b, s_] = (tsb[s_] - grid[b, k]) / (grid[b, k + 1] - grid[b, k])
    out = torch.empty((B, S) + tuple(y0.shape[1:]), dtype=y0.dtype, device=dev)
    out[torch.as_tensor(kk < 0, device=dev)] = y0.unsqueeze(1).expand_as(out)[torch.as_tensor(kk < 0, device=dev)]
    hs = torch.tensor(np.diff(grid, axis=1), dtype=y0.dtype, device=dev)  # [B, G-1]; 0 on padded steps
    bshape = (B,) + (1,) * (y0.dim() - 1)
    y, k0 = y0, f(y0)
    for k in range(G - 1):
        h = hs[:, k].reshape(bshape)
        K = [k0]
        for i in range(1, 7):
            K.append(f(y + h * sum(a * K[j] for j, a in enumerate(A[i]) if a != 0.0)))
        y1 = y + h * sum(a * K[j] for j, a in enumerate(A[6]) if a != 0.0)  # stage 7 input = y1 (FSAL)
        sel = np.nonzero(kk == k)
        if len(sel[0]):
            bi = torch.as_tensor(sel[0], device=dev)
            si = torch.as_tensor(sel[1], device=dev)
            thv = torch.as_tensor(th[sel], dtype=y0.dtype, device=dev).reshape((-1,) + (1,) * (y0.dim() - 1))
            Ks = torch.stack([Kj[bi] for Kj in K])
            out[bi, si] = _dense(m, thv, hs[bi, k].reshape(thv.shape), y[bi], y1[bi], Ks)
        y, k0 = y1, K[6]
    return out


class DynDataset:
    """Generates the data and exposes the engine-layout graph paths.

    Attributes: t [B, Tt] (np), true_y [B, Tt, n] (torch, device), x0 [B, n, 1] (torch), A [B, E+1, n, n]
    (np adjacencies), events_indices, id_train / id_test_extra / id_test_inter.
    """

    def __init__(self, cfg: DynDataCfg, device="cuda"):
        self.cfg = cfg
        rng = np.random.default_rng(cfg.seed)
        B = cfg.batch_size
        if cfg.graph_type == "grid":
            self.N = int(math.ceil(math.sqrt(cfg.num_nodes)))
            base = np.tile(grid_8_neighbor_graph(self.N)[None], (B, 1, 1))
        elif cfg.graph_type == "community":
            base = np.stack([community_graph(cfg.num_nodes, cfg.seed + i, cfg.layout) for i in range(B)])
            self.N = None
        else:
            raise NotImplementedError(f"graph_type {cfg.graph_type}: grid and community are generated here")
        self.n = base.shape[-1]
        event_times = 10
        if cfg.all_dynamic:  # ode_dataset.py:79-91
            event_times += int(event_times / cfg.split_ratio[0] * cfg.split_ratio[1])
        self.t = self._sampling(rng)
        self.x0 = torch.tensor(self._initial(rng), dtype=torch.float32, device=device)
        if cfg.dynamic_graph:
            _, self.events_indices = events_happen_time(rng, self.t, event_times, cfg.split_ratio, cfg.all_dynamic)
            self.A = events_happen_graph(rng, base, event_times, 0.001)
        else:
            self.events_indices = np.zeros(0, dtype=np.int64)
            self.A = base[:, None]
        self.true_y = self._solve(device)
        self.id_train, self.id_test_extra, self.id_test_inter = split_indices(
            rng, cfg.sampling_type, cfg.time_tick, cfg.split_ratio)
        self.device = device

    def _sampling(self, rng) -> np.ndarray:
        """ode_dataset.py:303-342."""
        c = self.cfg
        if c.sampling_type == "equal":
            return np.tile(np.linspace(0.0, c.final_time, c.time_tick), (c.batch_size, 1))
        full = np.linspace(0.0, c.final_time, c.time_tick * 10)
        k = int(c.time_tick * 1.2)
        rows = []
        for _ in range(c.batch_size):
            ts = np.sort(rng.permutation(full)[:k])
            ts[0] = 0.0
            rows.append(ts)
        return np.stack(rows)

    def _initial(self, rng) -> np.ndarray:
        """ode_dataset.py:93-140: three non-overlapping patches of amplitude ~U(amp_range) (grid layout);
        a community graph gets three random node blocks instead."""
        c = self.cfg
        B, n = c.batch_size, self.n
        x0 = np.zeros((B, n))
        if self.N is not None:
            N = self.N
            grid = np.zeros((B, N, N))
            for i in range(B):
                placed = []
                for fh, fw in ((0.2, 0.2), (0.3, 0.3), (0.2, 0.3)):
                    h, w = max(1, int(fh * N)), max(1, int(fw * N))
                    for _ in range(1000):
                        r1, c1 = rng.integers(0, N - h + 1), rng.integers(0, N - w + 1)
                        if all(r1 + h <= a or a + hh <= r1 or c1 + w <= b or b + ww <= c1
                               for a, b, hh, ww in placed):
                            break
                    placed.append((r1, c1, h, w))
                    grid[i, r1:r1 + h, c1:c1 + w] = rng.uniform(*c.amp_range)
            x0 = grid.reshape(B, -1)
        else:
            for i in range(B):
                for _ in range(3):
                    s = rng.integers(0, n)
                    x0[i, s:s + max(1, n // 10)] = rng.uniform(*c.amp_range)
        return x0[..., None]

    def _rhs(self, A: torch.Tensor):
        if self.cfg.name == "heat":  # heat_diffusion_model.py: dX/dt = -k L X, L = D - A, k = 1
            L = torch.diag_embed(A.sum(-1)) - A
            return lambda x: -torch.bmm(L, x)
        if self.cfg.name == "gene":  # gene_dynamic_model.py: -b x^f + A x^h / (x^h + 1), b=1, f=1, h=2
            return lambda x: -x + torch.bmm(A, x * x) / (x * x + 1.0)
        raise NotImplementedError(f"dataset {self.cfg.name}: heat and gene are generated here")

    def _solve(self, device) -> torch.Tensor:
        """gen_all_data (ode_dataset.py:388-470): static graph -> one solve over every time; dynamic graph -> one
        solve per event segment t[:, :e_0], t[:, e_0:e_1], ..., t[:, e_last:] on graph A_k, segment k + 1 started
        from segment k's last saved state."""
        t = torch.tensor(self.t, dtype=torch.float64, device=device)
        A_all = torch.tensor(self.A, dtype=torch.float64, device=device)
        x = self.x0.to(torch.float64)
        T = self.t.shape[1]
        if not self.cfg.dynamic_graph:
            bounds = [0, T]
        else:
            bounds = [0] + [int(e) for e in np.sort(self.events_indices)] + [T]
        outs = []
        for k in range(len(bounds) - 1):
            s0, s1 = bounds[k], bounds[k + 1]
            ys = diffeqsolve_constant(self._rhs(A_all[:, k]), self.t[:, s0:s1], x, self.cfg.method, self.cfg.dt0)
            outs.append(ys)
            x = ys[:, -1]
        return torch.cat(outs, dim=1)[..., 0].to(torch.float32)  # [B, Tt, n]

    def graph_path(self, idx):
        """Engine-layout control over the knots ``idx`` (dataset_configs.py:159-199): graph operator of every
        event epoch (gncde_graph_operator), padded to the knots, backward-Hermite coefficients
        (gncde_hermite_coefficients).  Returns (ts [B, K] device, coef, tcoef)."""
        idx = np.asarray(idx)
        ts = torch.tensor(self.t[:, idx], dtype=torch.float32, device=self.device)
        ops = engine.graph_operator(torch.tensor(self.A, dtype=torch.float32), self.cfg.operator_type)
        epoch = padding_by_time(len(idx), self.events_indices) if self.cfg.dynamic_graph else \
            np.zeros(len(idx), dtype=np.int64)
        X = ops[:, torch.as_tensor(epoch, device=ops.device)]  # [B, K, n, n]
        coef, tcoef = layout.control_from_knots(ts, X)
        return ts, coef, tcoef


# ------------------------------------------------------------------------------------------------------------
# Snapshot-window datasets (PGT england-covid, TGB tgbn-trade shapes) — dataset_configs.py:461-815 (TGB),
# :900-1135 (PGT)
# ------------------------------------------------------------------------------------------------------------

@dataclass
class WindowDataCfg:
    """The ``dataset:`` block of configs/pgt/*/*.yaml and configs/tgb/*/*.yaml (unknown keys ignored).

    The reference reads england-covid from a JAX-era pickle and tgbn-trade through the tgb downloader; neither
    can be used here (no unpickling of shipped files, no network), so ``synthetic_snapshots`` generates
    snapshot sequences of the same shapes: england-covid n=129 with 8 node features (lagged case counts) and a
    per-node target; tgbn-trade n=255 with node features = adjacency rows and next-period rows as targets."""

    name: str = "england-covid"
    window_size: int = 5
    stride: int = 5
    split_ratio: tuple = (0.6, 0.2, 0.2)
    seed: int = 1234
    normalise_features: bool = False
    num_snapshots: int = 0  # 0: the dataset's own length (england-covid 61 days, tgbn-trade 32 years)

    @classmethod
    def from_dict(cls, d: dict) -> "WindowDataCfg":
        names = {f.name for f in fields(cls)}
        return cls(**{k: v for k, v in (d or {}).items() if k in names})


def window_nodes(name: str) -> int:
    """Nodes of the snapshot graphs ``synthetic_snapshots`` generates for a dataset name (england-covid: the 129
    NHS regions; tgbn-trade: 255 countries)."""
    if name.startswith("england"):
        return 129
    if name.startswith("tgbn-trade") or name.startswith("trade"):
        return 255
    raise NotImplementedError(f"dataset {name}: england-covid and tgbn-trade shapes are generated here")


def synthetic_snapshots(name: str, rng: np.random.Generator, num_snapshots: int = 0):
    """Snapshot sequence (list of dicts adj [n,n], x, y, src) shaped like the reference's datasets."""
    if name.startswith("england"):
        n, S, F = window_nodes(name), num_snapshots or 61, 8
        base = community_graph(n, int(rng.integers(1 << 30)))
        signal = np.abs(rng.standard_normal(n)) * 10.0
        hist = [signal.copy() for _ in range(F)]
        snaps = []
        for _ in range(S):
            adj = base * rng.lognormal(3.0, 1.5, (n, n)) * (rng.random((n, n)) > 0.1)
            deg = adj.sum(1, keepdims=True) + 1e-9
            nxt = np.maximum(0.7 * signal + 0.3 * (adj / deg) @ signal + rng.standard_normal(n), 0.0)
            x = np.stack(hist[-F:], axis=1)  # [n, 8] lagged values
            snaps.append(dict(adj=adj, x=x, y=nxt, src=np.nonzero(adj.sum(1))[0]))
            hist.append(nxt)
            signal = nxt
        return snaps
    if name.startswith("tgbn-trade") or name.startswith("trade"):
        n, S = window_nodes(name), num_snapshots or 32
        pattern = rng.random((n, n)) < 0.08
        np.fill_diagonal(pattern, False)
        vol = rng.lognormal(2.0, 2.0, (n, n))
        snaps = []
        for _ in range(S):
            vol = vol * rng.lognormal(0.0, 0.2, (n, n))
            active = pattern & (rng.random((n, n)) > 0.2)
            adj = np.where(active, vol, 0.0)
            snaps.append(dict(adj=adj, x=adj, src=np.nonzero(active.any(1))[0]))
        return snaps
    raise NotImplementedError(f"dataset {name}: england-covid and tgbn-trade shapes are generated here")


def sample_disjoint_windows(rng: np.random.Generator, num_snapshots: int, window_size: int, stride: int,
                            split_ratio):
    """dataset_configs.py:692-735: shuffled window starts split into disjoint train / val / test."""
    starts = np.arange(0, num_snapshots - window_size + 1, stride)
    rng.shuffle(starts)
    n_tr = int(len(starts) * split_ratio[0])
    n_va = int(len(starts) * split_ratio[1])
    return starts[:n_tr], starts[n_tr:n_tr + n_va], starts[n_tr + n_va:]


class WindowDataset:
    """Windows of ``window_size`` snapshots; the last snapshot of a window is its target (process_window,
    dataset_configs.py:772-811 / :1103-1131), the rest become the graph path (raw adjacency knots, no operator)
    and the node-data path, knots at t = 0 .. window_size-2."""

    def __init__(self, cfg: WindowDataCfg, device="cuda"):
        self.cfg, self.device = cfg, device
        rng = np.random.default_rng(cfg.seed)
        self.snaps = synthetic_snapshots(cfg.name, rng, cfg.num_snapshots)
        self.n = self.snaps[0]["adj"].shape[0]
        self.tgb = not cfg.name.startswith("england")
        self.train, self.val, self.test = sample_disjoint_windows(rng, len(self.snaps), cfg.window_size, cfg.stride,
                                                                  cfg.split_ratio)

    def batch(self, starts):
        """Model inputs for the windows starting at ``starts`` (engine layout, on the device):
        PGT: (ts, control_adj, control_x, x0, y); TGB: (ts, control_adj, x_t, x0, y, source_mask)."""
        from .interpolation import CubicInterpolation
        w = self.cfg.window_size
        dev = self.device
        T = w - 1
        wins = [self.snaps[s:s + w] for s in starts]
        ts = torch.arange(T, dtype=torch.float32, device=dev).repeat(len(wins), 1)
        A = torch.tensor(np.stack([[s["adj"] for s in win[:-1]] for win in wins]), dtype=torch.float32, device=dev)
        coef, tcoef = layout.control_from_knots(ts, A)
        adj = CubicInterpolation.from_layout(ts, coef=coef, tcoef=tcoef)
        x_t = torch.tensor(np.stack([[s["x"] for s in win[:-1]] for win in wins]), dtype=torch.float32, device=dev)
        if self.tgb and self.cfg.normalise_features:
            x_t = torch.softmax(x_t, dim=-1)
        x0 = torch.tensor(np.stack([win[0]["x"] for win in wins]), dtype=torch.float32, device=dev)
        if not self.tgb:
            X = torch.stack([ts[:, :, None, None].expand_as(x_t), x_t], dim=-1)
            xc = CubicInterpolation.from_layout(ts, data_coef=engine.hermite_coefficients(ts, X))
            y = torch.tensor(np.stack([win[-1]["y"] for win in wins]), dtype=torch.float32, device=dev)
            return ts, adj, xc, x0, y
        y = torch.tensor(np.stack([win[-1]["x"] for win in wins]), dtype=torch.float32, device=dev)
        mask = torch.zeros(len(wins), self.n, dtype=torch.bool, device=dev)
        for i, win in enumerate(wins):
            mask[i, torch.as_tensor(win[-1]["src"], device=dev, dtype=torch.long)] = True
        return ts, adj, x_t, x0, y, mask
