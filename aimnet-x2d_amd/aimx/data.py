"""Host-side batch construction: multi-hop pair lists and the collate step.

Product implementation of the two host stages that define the hot path's inputs:
  * multi-hop BFS pair lists — reference src/datasets/features.py:82-150
    (build_numba_adjacency_list + compute_multi_hop_edges_bfs_numba): hop 1 = every (v, w)
    neighbour pair ordered by v then w; hop k expands the previous hop's frontier in order and
    keeps first-visit (u, w) pairs, w != u;
  * collate — reference src/datasets/molecular.py:339-458 (MyBatch.from_data_list): per-molecule
    hop arrays offset by the molecule's atom offset ONLY (never by hop), concatenated molecule-
    major then hop-major and transposed to [E, 2] int64; batch_indices = repeat(arange(G), atoms).
Both are bit-exact against the reference (tests/test_data.py vs tests/golden/edges.npz).
"""
from __future__ import annotations

import numpy as np
import torch

FEATURE_KEYS = ("atom_type", "hydrogen_count", "degree", "hybridization")


def bfs_multi_hop(n_atoms, bonds, max_hops):
    """List of `max_hops` int32 [2, E_h] arrays for one molecule (bonds: [B, 2] undirected)."""
    nbr = [[] for _ in range(n_atoms)]
    for a, b in np.asarray(bonds).reshape(-1, 2).tolist():
        if a != b:
            nbr[a].append(b)
            nbr[b].append(a)
    for lst in nbr:
        lst.sort()
    seen = set()
    frontier = []
    for v in range(n_atoms):
        for w in nbr[v]:
            key = v * n_atoms + w
            if key not in seen:
                seen.add(key)
                frontier.append((v, w))
    out = [frontier]
    for _ in range(1, max_hops):
        nxt = []
        for u, v in frontier:
            base = u * n_atoms
            for w in nbr[v]:
                if w != u and (base + w) not in seen:
                    seen.add(base + w)
                    nxt.append((u, w))
        if not nxt:
            out.append([])
            break
        out.append(nxt)
        frontier = nxt
    while len(out) < max_hops:
        out.append([])
    return [np.array(h, dtype=np.int32).reshape(-1, 2).T.copy() for h in out]


def collate(mols, max_hops, hops=None):
    """mols: list of (n_atoms, bonds, feats [n,4]). Returns numpy arrays of the collated batch."""
    n_atoms = np.array([m[0] for m in mols], dtype=np.int64)
    offsets = np.concatenate([[0], np.cumsum(n_atoms)[:-1]]).astype(np.int64)
    parts = []
    for i, (n, bonds, _) in enumerate(mols):
        per = hops[i] if hops is not None else bfs_multi_hop(n, bonds, max_hops)
        for e in per:
            if e.shape[1]:
                parts.append(e.astype(np.int64) + offsets[i])
    edges = np.concatenate(parts, axis=1).T.copy() if parts else np.empty((0, 2), np.int64)
    feats = np.concatenate([m[2] for m in mols], axis=0).astype(np.int64)
    batch = np.repeat(np.arange(len(mols), dtype=np.int64), n_atoms)
    return {"edges": edges, "feats": feats, "batch": batch, "n_atoms": n_atoms}


def blob_layout(fields):
    """Byte layout of DeviceBatch fields [(dtype, shape)]: 256-byte aligned offsets.
    Returns ([(offset, dtype, shape)], total bytes)."""
    out, off = [], 0
    for dt, shape in fields:
        out.append((off, np.dtype(dt), tuple(shape)))
        off += (int(np.prod(shape)) * np.dtype(dt).itemsize + 255) // 256 * 256
    return out, max(off, 256)


def batch_fields(n_rows, e_rows, g_rows, n_tasks, csr_hops=0):
    """DeviceBatch field (dtype, shape) list: 4 feature columns, edges, batch, charges, targets, and
    with csr_hops > 0 the host-built CSR views (fwd / bwd / graph rowptr + col, int32;
    aimx_csr_host_build) for a model of that many hops."""
    f = ([(np.int64, (n_rows,))] * len(FEATURE_KEYS) + [(np.int64, (e_rows, 2)), (np.int64, (n_rows,)),
                                                        (np.float32, (g_rows,)), (np.float32, (g_rows, n_tasks))])
    if csr_hops > 0:
        f += [(np.int32, (csr_hops * n_rows + 1,)), (np.int32, (max(e_rows, 1),)), (np.int32, (n_rows + 1,)),
              (np.int32, (max(e_rows, 1),)), (np.int32, (g_rows + 1,)), (np.int32, (max(n_rows, 1),))]
    return f


class HostCSR:
    """The CSR views a DeviceBatch carries (host-built, aimx_csr_host_build), attached to its edges
    tensor as `_aimx_csr`; aimx.plan.GraphPlan uses them instead of building on the device when
    the plan's (hops, N, E, G, batch tensor) match."""
    __slots__ = ("hops", "N", "E", "G", "batch", "fwd_rowptr", "fwd_col", "bwd_rowptr", "bwd_col",
                 "graph_rowptr", "graph_col")

    def __init__(self, hops, N, E, G, batch, views):
        self.hops, self.N, self.E, self.G, self.batch = hops, N, E, G, batch
        (self.fwd_rowptr, self.fwd_col, self.bwd_rowptr, self.bwd_col, self.graph_rowptr, self.graph_col) = views


def host_csr_into(views, edges, batch, n_graphs, hops):
    """Run aimx_csr_host_build on host arrays / pinned views (numpy or CPU tensors) in place."""
    from .feed import _check, load_host
    lib = load_host()

    def p(a):
        if isinstance(a, torch.Tensor):
            return a.data_ptr() if a.numel() else None
        return a.ctypes.data if a.size else None
    n = int(batch.shape[0])
    e = int(edges.shape[0])
    _check(lib.aimx_csr_host_build(p(edges), e, p(batch), n, int(n_graphs), int(hops), *[p(v) for v in views]),
           "csr_host_build (index out of range: target >= hops*N or batch index >= G)")


class DeviceBatch:
    """A collated batch resident in HBM, in the reference trainer's argument layout.

    All fields are typed views into ONE device byte buffer, so re-filling a static (graph-captured)
    batch is a single copy (copy_) instead of one per tensor."""

    _FIELDS = ("feat0", "feat1", "feat2", "feat3", "edges", "batch", "total_charges", "targets")

    def __init__(self, col, device, targets=None, total_charges=None, csr_hops=0):
        g = len(col["n_atoms"])
        self.num_graphs = g
        self.num_atoms = int(col["batch"].shape[0])
        tc = total_charges if total_charges is not None else np.zeros(g, np.float32)
        tg = targets if targets is not None else np.zeros((g, 1), np.float32)
        parts = [np.ascontiguousarray(col["feats"][:, i]).astype(np.int64) for i in range(len(FEATURE_KEYS))]
        parts += [np.ascontiguousarray(col["edges"], np.int64), np.ascontiguousarray(col["batch"], np.int64),
                  np.ascontiguousarray(tc, np.float32), np.ascontiguousarray(tg, np.float32)]
        fields = [(a.dtype, a.shape) for a in parts]
        self.csr_hops = int(csr_hops)
        if self.csr_hops > 0:
            fields = batch_fields(self.num_atoms, parts[len(FEATURE_KEYS)].shape[0], g, tg.shape[1], self.csr_hops)
        self._layout, off = blob_layout(fields)
        host = np.zeros(off, np.uint8)
        for (o, _, _), a in zip(self._layout, parts):
            host[o:o + a.nbytes] = a.view(np.uint8).reshape(-1)
        if self.csr_hops > 0:
            views = [host[o:o + int(np.prod(sh)) * 4].view(np.int32) for o, _, sh in self._layout[len(parts):]]
            host_csr_into(views, parts[len(FEATURE_KEYS)], parts[len(FEATURE_KEYS) + 1], g, self.csr_hops)
        self._blob = torch.from_numpy(host).to(device)
        self._bind()
        self.tetrahedral = torch.empty(0, 4, dtype=torch.long, device=device)
        self.cis = torch.empty(0, 2, dtype=torch.long, device=device)
        self.trans = torch.empty(0, 2, dtype=torch.long, device=device)

    @classmethod
    def from_blob(cls, blob, layout, num_graphs, num_atoms, csr_hops=0):
        """Wrap a device byte buffer already holding the fields at `layout` (blob_layout())."""
        b = cls.__new__(cls)
        b.num_graphs, b.num_atoms = int(num_graphs), int(num_atoms)
        b.csr_hops = int(csr_hops)
        b._layout, b._blob = list(layout), blob
        b._bind()
        dev = blob.device
        b.tetrahedral = torch.empty(0, 4, dtype=torch.long, device=dev)
        b.cis = torch.empty(0, 2, dtype=torch.long, device=dev)
        b.trans = torch.empty(0, 2, dtype=torch.long, device=dev)
        return b

    def _bind(self):
        views = []
        for o, dt, shape in self._layout:
            tdt = {np.dtype(np.int64): torch.int64, np.dtype(np.int32): torch.int32}.get(np.dtype(dt), torch.float32)
            n = int(np.prod(shape)) if len(shape) else 1
            views.append(self._blob[o:o + n * (8 if tdt == torch.int64 else 4)].view(tdt).view(*shape))
        nf = len(FEATURE_KEYS)
        self.atom_features = {k: views[i] for i, k in enumerate(FEATURE_KEYS)}
        self.edges, self.batch, self.total_charges, self.targets = views[nf:nf + 4]
        if getattr(self, "csr_hops", 0) > 0:
            csr = views[nf + 4:nf + 10]
            csr[1], csr[3], csr[5] = csr[1][:self.edges.shape[0]], csr[3][:self.edges.shape[0]], csr[5][:self.num_atoms]
            self.edges._aimx_csr = HostCSR(self.csr_hops, self.num_atoms, self.edges.shape[0], self.num_graphs,
                                           self.batch, csr)

    def copy_(self, other):
        """In-place copy of another batch of identical layout (static graph inputs): one copy."""
        if other._layout != self._layout:
            raise ValueError("DeviceBatch.copy_: layouts differ")
        self._blob.copy_(other._blob, non_blocking=True)

    def clone(self):
        import copy
        b = copy.copy(self)
        b._blob = self._blob.clone()
        b._bind()
        return b

    def model_args(self):
        return (self.atom_features, self.edges, self.batch, self.total_charges, self.tetrahedral, self.cis,
                self.trans)


def pad_mols_for(n_max, n_min, atoms_per_pad=64, least=8):
    """Padding molecules for a static batch of n_max atoms whose real atom count may drop to n_min:
    the slack is split over enough molecules that none exceeds atoms_per_pad atoms (at least
    `least` of them). A padding molecule above 128 atoms leaves the attention pool's row-resident
    path (pool.hip): 8 molecules over c4's ~1.3 k slack atoms made k_attn_fwd / bwd ~6x slower."""
    return max(least, -(-(int(n_max) - int(n_min)) // atoms_per_pad))


def pad_collated(col, n_max, e_max, g_real, n_pad_mols=8):
    """Pad a collated batch to static shapes for graph replay (SURVEY.md §8d "padded batches").

    The slack atoms form `n_pad_mols` extra padding molecules (indices g_real .. g_real+n_pad_mols-1,
    sizes as equal as possible; some may be empty) and the slack edges are self-pairs spread over
    the padding atoms, so every real molecule's values are untouched (molecules never interact);
    callers drop rows >= g_real of the per-molecule outputs from the loss. Several small padding
    molecules instead of one large one keep the per-molecule kernels (one workgroup per molecule)
    free of a long serial tail. Requires n_max > N (at least one padding atom) and e_max >= E.
    """
    n = col["batch"].shape[0]
    e = col["edges"].shape[0]
    if n_max <= n or e_max < e or n_pad_mols < 1:
        raise ValueError(f"padding too small: atoms {n}/{n_max}, edges {e}/{e_max}, molecules {n_pad_mols}")
    n_pad = n_max - n
    feats = np.zeros((n_max, col["feats"].shape[1]), np.int64)
    feats[:n] = col["feats"]
    sizes = np.full(n_pad_mols, n_pad // n_pad_mols, np.int64)
    sizes[: n_pad % n_pad_mols] += 1
    batch = np.empty(n_max, np.int64)
    batch[:n] = col["batch"]
    batch[n:] = g_real + np.repeat(np.arange(n_pad_mols, dtype=np.int64), sizes)
    edges = np.empty((e_max, 2), np.int64)
    edges[:e] = col["edges"]
    # slack edges: self-pairs spread over the padding atoms (no long CSR row)
    pad = n + (np.arange(e_max - e, dtype=np.int64) % n_pad)
    edges[e:, 0] = pad
    edges[e:, 1] = pad
    n_atoms = np.concatenate([col["n_atoms"], sizes])
    return {"edges": edges, "feats": feats, "batch": batch, "n_atoms": n_atoms, "real_atoms": n, "real_edges": e}
