"""Fixture for the dyn datasets' community graphs (tests/test_data_cpu.py): the reference's generator call
(ode_dataset.py:189-202, ODEDataset._gen_community_graph) written out directly against networkx, with
data_tools.py:32-72's node reordering done the reference's way (scipy COO relabel + from_scipy_sparse_array),
independently of gncde.data.  Run: python tests/golden/make_community.py (networkx 3.4.2 in this image)."""
import os

import networkx as nx
import numpy as np
import scipy.sparse as sp

HERE = os.path.dirname(os.path.abspath(__file__))
CASES = [(128, 1234, "community"), (128, 1235, "community"), (10, 7, None), (40, 3, "degree"), (129, 99, None)]


def reference_like(n, seed, layout):
    n1, n2, n3 = int(n / 3), int(n / 3), int(n / 4)
    G = nx.random_partition_graph([n1, n2, n3, n - n1 - n2 - n3], 0.25, 0.01, seed=seed)
    if layout == "degree":
        s = sorted(G.degree, key=lambda x: x[1], reverse=True)
        m = {s[i][0]: i for i in range(len(s))}
    elif layout == "community":
        order = []
        for c in nx.community.greedy_modularity_communities(G):
            order += list(c)
        m = {order[i]: i for i in range(len(order))}
    else:
        m = None
    if m is not None:
        C = nx.to_scipy_sparse_array(G, format="coo")
        C = sp.coo_matrix((C.data, (np.array([m[x] for x in C.row]), np.array([m[x] for x in C.col]))), shape=C.shape)
        G = nx.from_scipy_sparse_array(C)
    return np.array(nx.to_numpy_array(G), dtype=float)


if __name__ == "__main__":
    out = {f"A_n{n}_s{seed}_{layout}": np.packbits(reference_like(n, seed, layout).astype(np.uint8))
           for n, seed, layout in CASES}
    out["networkx_version"] = np.array(nx.__version__)
    np.savez_compressed(os.path.join(HERE, "community_graphs.npz"), **out)
