"""Graph plan: the device-side CSR views of one collated batch, built once per forward.

Inputs are the reference's own tensors (MyBatch.from_data_list, molecular.py:339-458):
  multi_hop_edge_indices [E, 2] int64, column 0 = target, column 1 = source (gnn.py:302-306)
  batch_indices [N] int64, molecule id per atom
From them, on the device and without a host synchronisation (sizes come from tensor shapes and
from total_charges.shape[0] = G):
  fwd CSR: rows = num_hops*N keyed by target, col = source % N  (the hop, layers.py:154-163)
  bwd CSR: rows = N keyed by source % N,   col = target          (the hop's backward)
  graph CSR: rows = G keyed by batch index, col = atom id         (pooling / partial charges)
All three keep ascending item order inside a row (stable), i.e. the reference summation order.
"""
from __future__ import annotations

import os

import torch

from . import _lib

_VALIDATE = os.environ.get("AIMX_VALIDATE", "0") == "1"
# use the CSR views a DeviceBatch carries from the batch builder (False: always build on the device)
_HOST_CSR = True
_ZERO = {}


def _zero_status(device):
    """A status word that stays 0 (plans whose indices were checked on the host)."""
    z = _ZERO.get(device)
    if z is None:
        z = _ZERO[device] = torch.zeros(1, dtype=torch.int32, device=device)
    return z


def _col(t2d, j):
    """(base pointer, element stride) of column j of an int64 [E, 2] tensor (any strides)."""
    return t2d.data_ptr() + j * t2d.stride(1) * t2d.element_size(), t2d.stride(0)


def _as_i64(t):
    return t if t.dtype == torch.int64 else t.long()


class CSR:
    __slots__ = ("rowptr", "col", "rows")

    def __init__(self, rowptr, col, rows):
        self.rowptr, self.col, self.rows = rowptr, col, rows


def build_csr(key_ptr, key_stride, key_mod, val_ptr, val_stride, val_mod, n_items, n_rows, device, status):
    lib = _lib.load()
    rowptr = torch.empty(n_rows + 1, dtype=torch.int32, device=device)
    col = torch.empty(max(n_items, 1), dtype=torch.int32, device=device)
    wsb = lib.aimx_csr_workspace_bytes(n_items, n_rows)
    ws = torch.empty(wsb, dtype=torch.uint8, device=device)
    rc = lib.aimx_csr_build(key_ptr, key_stride, key_mod, val_ptr, val_stride, val_mod, n_items, n_rows,
                            rowptr.data_ptr(), col.data_ptr(), ws.data_ptr(), wsb, status.data_ptr(),
                            _lib.stream_ptr(device))
    _lib.check(rc, "csr_build")
    return CSR(rowptr, col, n_rows)


def build_csrs(specs, device, status):
    """All CSRs of a plan in one pass (aimx_csr_build_multi: one launch per phase for all)."""
    lib = _lib.load()
    arr = (_lib.CsrSpec * len(specs))()
    out = []
    for i, (kp, ks, km, vp, vs, vm, n_items, n_rows, _) in enumerate(specs):
        rowptr = torch.empty(n_rows + 1, dtype=torch.int32, device=device)
        col = torch.empty(max(n_items, 1), dtype=torch.int32, device=device)
        arr[i].key, arr[i].key_stride, arr[i].key_mod = kp, ks, km
        arr[i].val, arr[i].val_stride, arr[i].val_mod = vp, vs, vm
        arr[i].n_items, arr[i].n_rows = n_items, n_rows
        arr[i].rowptr, arr[i].col = rowptr.data_ptr(), col.data_ptr()
        out.append(CSR(rowptr, col, n_rows))
    wsb = lib.aimx_csr_build_multi_workspace_bytes(arr, len(specs))
    ws = torch.empty(max(wsb, 1), dtype=torch.uint8, device=device)
    _lib.check(lib.aimx_csr_build_multi(arr, len(specs), ws.data_ptr(), wsb, status.data_ptr(),
                                        _lib.stream_ptr(device)), "csr_build_multi")
    return out


class GraphPlan:
    """CSR views for one batch. `edges` [E,2] (target, source) or separate target/src vectors."""

    def __init__(self, num_atoms, num_hops, edges=None, target=None, src=None, batch=None, num_graphs=None):
        self.N = int(num_atoms)
        self.num_hops = int(num_hops)
        ref = edges if edges is not None else (target if target is not None else batch)
        self.device = ref.device
        _lib.require_device(ref)
        self.status = torch.empty(1, dtype=torch.int32, device=self.device)  # zeroed by the CSR build
        self.fwd = self.bwd = self.graph = None
        if edges is not None:
            e = _as_i64(edges)
            self._keep = [e]
            self.E = e.shape[0]
            (t_ptr, t_st), (s_ptr, s_st) = _col(e, 0), _col(e, 1)
        elif target is not None:
            t, s = _as_i64(target), _as_i64(src)
            self._keep = [t, s]
            self.E = t.shape[0]
            t_ptr, t_st, s_ptr, s_st = t.data_ptr(), t.stride(0), s.data_ptr(), s.stride(0)
        else:
            self._keep = []
            self.E = 0
            e = torch.zeros(0, 2, dtype=torch.int64, device=self.device)
            (t_ptr, t_st), (s_ptr, s_st) = _col(e, 0), _col(e, 1)
        self.batch = batch
        self.G = None
        hc = getattr(edges, "_aimx_csr", None) if edges is not None and _HOST_CSR else None
        if hc is not None and batch is not None and hc.hops == self.num_hops and hc.N == self.N and \
                hc.E == self.E and (num_graphs is None or int(num_graphs) == hc.G) and \
                batch.data_ptr() == hc.batch.data_ptr() and tuple(batch.shape) == tuple(hc.batch.shape) and \
                batch.dtype == torch.int64:
            # the batch builder already made this batch's CSRs (aimx.data.HostCSR, in the batch blob)
            self._keep.append(batch)
            self.G = hc.G
            self.fwd = CSR(hc.fwd_rowptr, hc.fwd_col, self.num_hops * self.N)
            self.bwd = CSR(hc.bwd_rowptr, hc.bwd_col, self.N)
            self.graph = CSR(hc.graph_rowptr, hc.graph_col, hc.G)
            self.status = _zero_status(self.device)  # validated on the host (aimx_csr_host_build)
            self.host_csr = True
            return
        self.host_csr = False
        specs = []  # (key, key_stride, key_mod, val, val_stride, val_mod, n_items, n_rows, attribute)
        if self.N > 0:  # E == 0 gives all-empty rows: every hop chunk is zero (layers.py:148-149)
            n, h = self.N, self.num_hops
            specs.append((t_ptr, t_st, 0, s_ptr, s_st, n, self.E, h * n, "fwd"))
            specs.append((s_ptr, s_st, n, t_ptr, t_st, 0, self.E, n, "bwd"))
        if batch is not None:
            b = _as_i64(batch)
            self._keep.append(b)
            g = int(num_graphs) if num_graphs is not None else int(b.max().item()) + 1 if b.numel() else 0
            self.G = g
            specs.append((b.data_ptr(), b.stride(0), 0, None, 0, 0, b.shape[0], g, "graph"))
        if specs:
            for name, c in zip([sp[-1] for sp in specs], build_csrs(specs, self.device, self.status)):
                setattr(self, name, c)
        else:
            self.status.zero_()
        if _VALIDATE:
            self.validate()

    def row_seg(self):
        """(pointer, stride) of the molecule id per atom (the batch indices) for segment-aligned
        hop tiles, or (None, 0) when the plan has no batch (the result never depends on it)."""
        if self.batch is None or self.batch.dim() != 1 or self.batch.shape[0] != self.N:
            return None, 0
        b = self._keep[-1]  # the int64 batch tensor kept alive by the plan
        return b.data_ptr(), b.stride(0)

    def validate(self):
        """Synchronising check (opt-in via AIMX_VALIDATE=1): the reference raises on bad indices."""
        if int(self.status.item()) != 0:
            raise RuntimeError("aimx: index out of range in edge/batch tensors "
                               "(target >= num_hops * N, or batch index >= num_graphs)")
