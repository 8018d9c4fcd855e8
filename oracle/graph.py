"""ORACLE (test infrastructure): integer/graph restatements, bit-exact targets.

bfs_multi_hop      <- reference src/datasets/features.py:82-150
                      (build_numba_adjacency_list + compute_multi_hop_edges_bfs_numba)
collate_edges      <- reference src/datasets/molecular.py:339-458 (MyBatch.from_data_list,
                      steps 1, 5 and 8: atom offsets, batch_indices, [E,2] edge tensor)
stable_csr         <- the order in which CPU ATen scatter_add_ (layers.py:158 via torch_scatter)
                      visits edges: ascending edge index within each target row.
"""
import numpy as np


def adjacency_list(adj):
    """features.py:82-94: neighbours of v in ascending index order, self loops skipped."""
    n = adj.shape[0]
    out = []
    for v in range(n):
        nz = np.where(adj[v] > 0)[0]
        out.append([int(w) for w in nz if w != v])
    return out


def bfs_multi_hop(adj_list, max_hops):
    """features.py:97-150: list of `max_hops` int32 [2, E_h] arrays of first-visit (u, w) pairs."""
    n = len(adj_list)
    visited = np.zeros((n, n), dtype=bool)
    hop1 = []
    for v in range(n):
        for w in adj_list[v]:
            if not visited[v, w]:
                visited[v, w] = True
                hop1.append((v, w))
    results = [np.array(hop1, dtype=np.int32).reshape(-1, 2).T.copy()]
    frontier = hop1
    for _ in range(1, max_hops):
        new = []
        for (u, v) in frontier:
            for w in adj_list[v]:
                if w != u and not visited[u, w]:
                    visited[u, w] = True
                    new.append((u, w))
        if len(new) == 0:
            results.append(np.empty((2, 0), dtype=np.int32))
            break
        results.append(np.array(new, dtype=np.int32).T.copy())
        frontier = new
    while len(results) < max_hops:
        results.append(np.empty((2, 0), dtype=np.int32))
    return results


def collate_edges(per_mol_hops, n_atoms):
    """molecular.py:350-436: edges offset by the molecule's atom offset only (never by hop),
    concatenated molecule-major then hop-major, transposed to [E, 2] int64.
    Returns (edges [E,2] int64, batch_indices [N] int64, atom_offsets [G] int64)."""
    n_atoms = np.asarray(n_atoms, dtype=np.int64)
    offsets = np.concatenate([[0], np.cumsum(n_atoms[:-1])]).astype(np.int64)
    parts = []
    for i, hops in enumerate(per_mol_hops):
        for e in hops:
            if e.size > 0:
                parts.append(e.astype(np.int64) + offsets[i])
    if parts:
        edges = np.concatenate(parts, axis=1).T.copy()
    else:
        edges = np.empty((0, 2), dtype=np.int64)
    batch = np.repeat(np.arange(len(n_atoms), dtype=np.int64), n_atoms)
    return edges, batch, offsets


def stable_csr(keys, vals, n_rows):
    """Rows sorted by key, ties in ascending item order. Returns (rowptr int32[n_rows+1], col int32)."""
    keys = np.asarray(keys, dtype=np.int64)
    order = np.argsort(keys, kind="stable")
    counts = np.bincount(keys, minlength=n_rows)
    rowptr = np.zeros(n_rows + 1, dtype=np.int64)
    np.cumsum(counts, out=rowptr[1:])
    return rowptr.astype(np.int32), np.asarray(vals, dtype=np.int64)[order].astype(np.int32)
