"""ctypes binding of the C ABI in include/aimx.h (libaimx.so, HIP / gfx950).

The library is built in-tree (`make -C aimnet-x2d_amd/csrc`, or __graft_entry__.build()). There is
no fallback: if the library or a HIP device is missing, every op raises AimxError.
"""
from __future__ import annotations

import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
# AIMX_LIB_PATH: a variant build of the same sources (A/B experiments on the GPU box)
LIB_PATH = os.environ.get("AIMX_LIB_PATH") or os.path.join(os.path.dirname(_HERE), "lib", "libaimx.so")

c_i64 = ctypes.c_int64
c_i32 = ctypes.c_int32
c_u32 = ctypes.c_uint32
c_f32 = ctypes.c_float
c_ptr = ctypes.c_void_p
c_size = ctypes.c_size_t

ACT_KIND = {"relu": 0, "leakyrelu": 1, "elu": 2, "gelu": 3, "silu": 4}
GATHER_SKIP_TAIL = 1  # AIMX_GATHER_SKIP_TAIL (include/aimx.h)


class AimxError(RuntimeError):
    pass


class Stereo(ctypes.Structure):
    """AimxStereo (include/aimx.h): the stereochemistry feature op's arguments."""
    _fields_ = [("x", ctypes.c_void_p), ("ldx", ctypes.c_int64), ("N", ctypes.c_int64), ("D", ctypes.c_int64),
                ("tet", ctypes.c_void_p), ("tet_stride0", ctypes.c_int64), ("tet_stride1", ctypes.c_int64),
                ("M", ctypes.c_int64),
                ("cis", ctypes.c_void_p), ("cis_stride0", ctypes.c_int64), ("cis_stride1", ctypes.c_int64),
                ("n_cis", ctypes.c_int64),
                ("trans", ctypes.c_void_p), ("trans_stride0", ctypes.c_int64), ("trans_stride1", ctypes.c_int64),
                ("n_trans", ctypes.c_int64),
                ("t_rowptr", ctypes.c_void_p), ("t_col", ctypes.c_void_p),
                ("scratch", ctypes.c_void_p), ("stats", ctypes.c_void_p),
                ("out", ctypes.c_void_p), ("ldo", ctypes.c_int64)]


class LossAccum(ctypes.Structure):
    """AimxLossAccum (include/aimx.h): the train step's device-side loss / NaN / step bookkeeping."""
    _fields_ = [("loss_sum", ctypes.c_void_p), ("nan_count", ctypes.c_void_p), ("steps", ctypes.c_void_p),
                ("scale", ctypes.c_float), ("d_loss", ctypes.c_void_p), ("d_pred", ctypes.c_void_p),
                ("ldd", ctypes.c_int64), ("rows_total", ctypes.c_int64)]


class PadBatch(ctypes.Structure):
    """AimxPadBatch (include/aimx.h): static padded inputs of one autograph shape bucket."""
    _fields_ = [("feat", ctypes.c_void_p * 4), ("feat_stride", ctypes.c_int64 * 4),
                ("edges", ctypes.c_void_p), ("edge_s0", ctypes.c_int64), ("edge_s1", ctypes.c_int64),
                ("batch", ctypes.c_void_p), ("batch_stride", ctypes.c_int64),
                ("charges", ctypes.c_void_p), ("charge_stride", ctypes.c_int64),
                ("N", ctypes.c_int64), ("E", ctypes.c_int64), ("G", ctypes.c_int64),
                ("out_feat", ctypes.c_void_p), ("out_edges", ctypes.c_void_p), ("out_batch", ctypes.c_void_p),
                ("out_charges", ctypes.c_void_p), ("Np", ctypes.c_int64), ("Ep", ctypes.c_int64),
                ("pad_mols", ctypes.c_int64)]


class GemmArgs(ctypes.Structure):
    _fields_ = [
        ("M", c_i64), ("N", c_i64), ("K", c_i64),
        ("A", c_ptr), ("sam", c_i64), ("sak", c_i64),
        ("B", c_ptr), ("sbk", c_i64), ("sbn", c_i64),
        ("C", c_ptr), ("ldc", c_i64),
        ("beta", c_f32),
        ("bias", c_ptr),
        ("res", c_ptr * 3), ("ldres", c_i64 * 3),
        ("act", c_i32), ("act_ncols", c_i64),
        ("pre", c_ptr), ("ldpre", c_i64),
        ("dact_pre", c_ptr), ("lddact", c_i64), ("dact_kind", c_i32),
        ("drop_p", c_f32), ("drop_seed", c_ptr), ("drop_salt", c_u32),
        ("mask_out", c_ptr), ("mask_in", c_ptr), ("ldmask", c_i64),
        ("ones_col", c_i32), ("col_out", c_ptr),
        ("splits", c_i32), ("workspace", c_ptr), ("workspace_bytes", c_size),
        ("counters", c_ptr), ("n_counters", c_i64),
        ("zc_rowptr", c_ptr), ("zc_rows", c_i64), ("zc_chunks", c_i32), ("zc_width", c_i64), ("zc_dim", c_i32),
        ("precision", c_i32), ("m_base", c_i64),
    ]


class ShellStack(ctypes.Structure):
    _fields_ = [
        ("N", c_i64), ("D", c_i64), ("num_hops", c_i64), ("num_layers", c_i64), ("num_mlp", c_i64),
        ("act", c_i32), ("use_pc", c_i32), ("training", c_i32), ("mode_single", c_i32),
        ("drop_p", c_f32), ("drop_seed", c_ptr),
        ("fwd_rowptr", c_ptr), ("fwd_col", c_ptr), ("bwd_rowptr", c_ptr), ("bwd_col", c_ptr),
        ("gptr", c_ptr), ("gperm", c_ptr), ("G", c_i64), ("total_charges", c_ptr),
        ("row_seg", c_ptr), ("row_seg_stride", c_i64),
        ("w_ig", c_ptr), ("b_ig", c_ptr), ("w1", c_ptr), ("b1", c_ptr), ("w2", c_ptr), ("b2", c_ptr),
        ("F", c_ptr), ("X", c_ptr), ("UG", c_ptr), ("U", c_ptr),
        ("V", c_ptr), ("R", c_ptr), ("A", c_ptr), ("M", c_ptr),
        ("x_in", c_ptr), ("x_in_ld", c_i64),
        ("out", c_ptr), ("out_ld", c_i64),
        ("workspace", c_ptr), ("workspace_bytes", c_size),
        ("counters", c_ptr), ("n_counters", c_i64), ("precision", c_i32), ("ld_f", c_i64), ("ld_ug", c_i64),
        ("ld_act", c_i64),
    ]


class ShellStackGrad(ctypes.Structure):
    _fields_ = [
        ("d_out", c_ptr), ("d_out_ld", c_i64),
        ("d_x_in", c_ptr), ("d_x_in_ld", c_i64),
        ("d_w_ig", c_ptr), ("d_b_ig", c_ptr), ("d_w1", c_ptr), ("d_b1", c_ptr), ("d_w2", c_ptr), ("d_b2", c_ptr),
        ("workspace", c_ptr), ("workspace_bytes", c_size),
    ]


HEAD_MAX_BLOCKS = 8
HEAD_SYNC_WORDS = 68


class Head(ctypes.Structure):
    _fields_ = [
        ("G", c_i64), ("F", c_i64), ("H_in", c_i64), ("T", c_i64),
        ("nb", c_i32), ("act", c_i32), ("training", c_i32),
        ("drop_p", c_f32), ("seed", c_ptr),
        ("x0", c_ptr), ("ldx0", c_i64),
        ("wp", c_ptr), ("bp", c_ptr),
        ("w1", c_ptr * HEAD_MAX_BLOCKS), ("b1", c_ptr * HEAD_MAX_BLOCKS),
        ("w2", c_ptr * HEAD_MAX_BLOCKS), ("b2", c_ptr * HEAD_MAX_BLOCKS),
        ("skip", c_i32 * HEAD_MAX_BLOCKS),
        ("ws", c_ptr), ("bs", c_ptr), ("wo", c_ptr), ("bo", c_ptr),
        ("y0", c_ptr), ("v", c_ptr * HEAD_MAX_BLOCKS), ("hid", c_ptr * HEAD_MAX_BLOCKS),
        ("mask", c_ptr * HEAD_MAX_BLOCKS), ("z", c_ptr * HEAD_MAX_BLOCKS), ("cat", c_ptr),
        ("out", c_ptr), ("ldo", c_i64),
        ("sync", c_ptr), ("cluster", c_i32),
        ("fwd_ws", c_ptr), ("fwd_ws_bytes", c_size),
    ]


class HeadGrad(ctypes.Structure):
    _fields_ = [
        ("d_out", c_ptr), ("ld_dout", c_i64),
        ("d_x0", c_ptr), ("ld_dx0", c_i64),
        ("ds", c_ptr), ("dz", c_ptr * HEAD_MAX_BLOCKS), ("dv", c_ptr * HEAD_MAX_BLOCKS), ("dy0", c_ptr),
        ("workspace", c_ptr), ("workspace_bytes", c_size),
    ]


class EmbeddingTables(ctypes.Structure):
    _fields_ = [
        ("n_tables", c_i32), ("dim", c_i64),
        ("table", c_ptr * 8), ("index", c_ptr * 8), ("rows", c_i64 * 8), ("grad", c_ptr * 8),
        ("seed_state", c_ptr), ("seeds", c_ptr), ("n_seeds", c_i32),
    ]


class CopyItem(ctypes.Structure):
    _fields_ = [("src", c_ptr), ("dst", c_ptr), ("n", c_i64)]


class CsrSpec(ctypes.Structure):
    _fields_ = [("key", c_ptr), ("key_stride", c_i64), ("key_mod", c_i64), ("val", c_ptr), ("val_stride", c_i64),
                ("val_mod", c_i64), ("n_items", c_i64), ("n_rows", c_i64), ("rowptr", c_ptr), ("col", c_ptr)]


class WgradProblem(ctypes.Structure):
    _fields_ = [("dY", c_ptr), ("ld_dy", c_i64), ("X", c_ptr), ("ld_x", c_i64), ("dW", c_ptr), ("ld_dw", c_i64),
                ("col_out", c_ptr), ("M", c_i64), ("N", c_i64), ("K", c_i64),
                ("zc_rowptr", c_ptr), ("zc_rows", c_i64), ("zc_chunks", c_i32), ("zc_width", c_i64)]


class AdamTensor(ctypes.Structure):
    _fields_ = [("param", c_ptr), ("grad", c_ptr), ("exp_avg", c_ptr), ("exp_avg_sq", c_ptr), ("numel", c_i64),
                ("group", c_i32), ("step_slot", c_i32)]


class AdamHyper(ctypes.Structure):
    _fields_ = [("beta1", c_f32), ("beta2", c_f32), ("one_minus_beta1", c_f32), ("one_minus_beta2", c_f32),
                ("eps", c_f32), ("weight_decay", c_f32), ("max_grad_norm", c_f32)]


_SIGS = {
    "aimx_version": (ctypes.c_char_p, []),
    "aimx_csr_workspace_bytes": (c_size, [c_i64, c_i64]),
    "aimx_csr_build": (c_i32, [c_ptr, c_i64, c_i64, c_ptr, c_i64, c_i64, c_i64, c_i64, c_ptr, c_ptr, c_ptr, c_size,
                               c_ptr, c_ptr]),
    "aimx_csr_build_multi_workspace_bytes": (c_size, [ctypes.POINTER(CsrSpec), c_i32]),
    "aimx_csr_build_multi": (c_i32, [ctypes.POINTER(CsrSpec), c_i32, c_ptr, c_size, c_ptr, c_ptr]),
    "aimx_segment_gather_sum": (c_i32, [c_ptr, c_i64, c_i64, c_i64, c_i64, c_ptr, c_ptr, c_i64, c_ptr, c_i64, c_i64,
                                        c_i64, c_ptr, c_i64, c_ptr, c_i64, c_ptr, c_i64, c_ptr]),
    "aimx_segment_gather_sum_ex": (c_i32, [c_ptr, c_i64, c_i64, c_i64, c_i64, c_ptr, c_ptr, c_i64, c_ptr, c_i64,
                                           c_i64, c_i64, c_ptr, c_i64, c_ptr, c_i64, c_ptr, c_i64, c_i32, c_ptr]),
    "aimx_gemm_workspace_bytes": (c_size, [ctypes.POINTER(GemmArgs)]),
    "aimx_gemm": (c_i32, [ctypes.POINTER(GemmArgs), c_ptr]),
    "aimx_shell_stack_workspace_bytes": (c_size, [ctypes.POINTER(ShellStack)]),
    "aimx_shell_stack_forward": (c_i32, [ctypes.POINTER(ShellStack), c_ptr]),
    "aimx_shell_stack_backward": (c_i32, [ctypes.POINTER(ShellStack), ctypes.POINTER(ShellStackGrad), c_ptr]),
    "aimx_shell_stack_backward_workspace_bytes": (c_size, [ctypes.POINTER(ShellStack)]),
    "aimx_partial_charge_forward": (c_i32, [c_ptr, c_i64, c_i64, c_i64, c_ptr, c_ptr, c_i64, c_ptr, c_ptr, c_i64,
                                            c_ptr]),
    "aimx_partial_charge_backward": (c_i32, [c_ptr, c_i64, c_i64, c_i64, c_ptr, c_ptr, c_i64, c_ptr, c_ptr, c_i64,
                                             c_ptr, c_i64, c_ptr]),
    "aimx_attn_pool_workspace_bytes": (c_size, [c_i64, c_i64, c_i64, c_i64]),
    "aimx_attn_pool_forward": (c_i32, [c_ptr, c_i64, c_i64, c_i64, c_ptr, c_ptr, c_ptr, c_i64, c_ptr, c_ptr, c_i64,
                                       c_ptr, c_ptr, c_ptr, c_ptr]),
    "aimx_attn_pool_backward": (c_i32, [c_ptr, c_i64, c_i64, c_i64, c_ptr, c_ptr, c_i64, c_ptr, c_ptr, c_i64, c_ptr,
                                        c_ptr, c_ptr, c_ptr, c_ptr, c_i64, c_ptr, c_ptr, c_ptr, c_ptr, c_size, c_ptr]),
    "aimx_segment_pool_forward": (c_i32, [c_i32, c_ptr, c_i64, c_i64, c_i64, c_ptr, c_ptr, c_i64, c_ptr, c_ptr,
                                          c_ptr]),
    "aimx_segment_pool_backward": (c_i32, [c_i32, c_ptr, c_i64, c_i64, c_ptr, c_ptr, c_i64, c_ptr, c_ptr, c_i64,
                                           c_ptr]),
    "aimx_embedding_gather": (c_i32, [ctypes.POINTER(EmbeddingTables), c_i64, c_ptr, c_i64, c_ptr]),
    "aimx_embedding_backward_workspace_bytes": (c_size, [ctypes.POINTER(EmbeddingTables), c_i64]),
    "aimx_embedding_backward": (c_i32, [ctypes.POINTER(EmbeddingTables), c_i64, c_ptr, c_i64, c_ptr, c_size, c_ptr]),
    "aimx_act_backward": (c_i32, [c_i32, c_ptr, c_i64, c_ptr, c_i64, c_i64, c_i64, c_ptr, c_i64, c_ptr]),
    "aimx_act_backward2": (c_i32, [c_i32, c_ptr, c_i64, c_i64, c_ptr, c_i64, c_ptr, c_i64, c_i64, c_i64, c_ptr, c_i64,
                                   c_ptr]),
    "aimx_head_forward": (c_i32, [ctypes.POINTER(Head), c_ptr]),
    "aimx_head_backward_workspace_bytes": (c_size, [ctypes.POINTER(Head)]),
    "aimx_head_forward_workspace_bytes": (c_size, [ctypes.POINTER(Head)]),
    "aimx_head_backward": (c_i32, [ctypes.POINTER(Head), ctypes.POINTER(HeadGrad), c_ptr]),
    "aimx_dropout_seeds": (c_i32, [c_ptr, c_ptr, c_i32, c_ptr]),
    "aimx_pad_batch": (c_i32, [c_ptr, c_ptr]),
    "aimx_stereo_forward": (c_i32, [ctypes.c_void_p, c_ptr]),
    "aimx_stereo_backward": (c_i32, [ctypes.c_void_p, c_ptr, c_i64, c_ptr, c_i64, c_ptr, c_ptr]),
    "aimx_l1_loss_forward": (c_i32, [c_ptr, c_i64, c_ptr, c_i64, c_i64, c_i64, c_ptr, c_i32, c_ptr, c_ptr]),
    "aimx_l1_loss_forward_accum": (c_i32, [c_ptr, c_i64, c_ptr, c_i64, c_i64, c_i64, c_ptr, c_i32, c_ptr,
                                           ctypes.c_void_p, c_ptr]),
    "aimx_l1_loss_backward": (c_i32, [c_ptr, c_i64, c_ptr, c_i64, c_i64, c_i64, c_ptr, c_i32, c_ptr, c_ptr, c_i64,
                                      c_ptr]),
    "aimx_l1_loss_backward_padded": (c_i32, [c_ptr, c_i64, c_ptr, c_i64, c_i64, c_i64, c_i64, c_ptr, c_i32, c_ptr,
                                             c_ptr, c_i64, c_ptr]),
    "aimx_wgrad_grouped_workspace_bytes": (c_size, [ctypes.POINTER(WgradProblem), c_i32]),
    "aimx_wgrad_grouped": (c_i32, [ctypes.POINTER(WgradProblem), c_i32, c_ptr, c_size, c_ptr, c_i64, c_ptr]),
    "aimx_fused_adam_workspace_bytes": (c_size, [ctypes.POINTER(AdamTensor), c_i32]),
    "aimx_multi_copy": (c_i32, [ctypes.POINTER(CopyItem), c_i32, c_ptr]),
    "aimx_set_option": (c_i32, [ctypes.c_char_p, c_i64]),
    "aimx_clear_options": (c_i32, []),
    "aimx_comm_load": (c_i32, [ctypes.c_char_p]),
    "aimx_comm_unique_id": (c_i32, [c_ptr, c_size]),
    "aimx_comm_init": (c_i32, [ctypes.POINTER(c_ptr), c_ptr, c_size, c_i32, c_i32]),
    "aimx_comm_allreduce": (c_i32, [c_ptr, c_ptr, c_i64, c_i32, c_ptr]),
    "aimx_comm_destroy": (c_i32, [c_ptr]),
    "aimx_comm_version": (c_i32, [ctypes.POINTER(c_i32)]),
    "aimx_comm_count": (c_i32, [c_ptr, ctypes.POINTER(c_i32)]),
    "aimx_fused_adam": (c_i32, [ctypes.POINTER(AdamTensor), c_i32, ctypes.POINTER(AdamHyper), c_ptr, c_ptr, c_ptr,
                                c_ptr, c_size, c_ptr]),
}

EXPORTED_SYMBOLS = tuple(_SIGS)

_lib = None


def load():
    """Load libaimx.so (once). Raises AimxError if it is missing or incomplete."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise AimxError(f"aimx: HIP library not built: {LIB_PATH} (run `make -C aimnet-x2d_amd/csrc`)")
    try:
        lib = ctypes.CDLL(LIB_PATH)
    except OSError as e:  # pragma: no cover
        raise AimxError(f"aimx: cannot load {LIB_PATH}: {e}") from e
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name, None)
        if fn is None:
            raise AimxError(f"aimx: {LIB_PATH} does not export {name}")
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(rc, what):
    if rc != 0:
        if rc < 0:
            raise AimxError(f"aimx: {what}: invalid arguments (code {rc})")
        raise AimxError(f"aimx: {what}: HIP error {rc}")


def require_device(*tensors):
    for t in tensors:
        if t is not None and not t.is_cuda:
            raise AimxError("aimx: tensors must live on the HIP device (MI355X); there is no CPU path")


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def stream_ptr(device=None):
    """The current HIP stream of `device` as an integer handle (hot path: one C call, no Stream
    object; torch.cuda.current_stream builds a Python Stream per call)."""
    if _raw_stream is not None:
        if device is None:
            idx = torch.cuda.current_device()
        elif isinstance(device, int):
            idx = device
        else:
            if isinstance(device, str):
                device = torch.device(device)
            idx = device.index if device.index is not None else torch.cuda.current_device()
        return _raw_stream(idx)
    return torch.cuda.current_stream(device).cuda_stream


_COUNTERS = {}
N_COUNTERS = 1 << 16


def counters(device, slot=0):
    """Per-device split-K arrival counters: zeroed once, kept zero by the kernels themselves. A
    different slot is a separate array (for kernels a caller runs concurrently on another stream:
    two streams' split-K tickets must never share a counter)."""
    key = torch.device(device).index if torch.device(device).index is not None else torch.cuda.current_device()
    buf = _COUNTERS.get((key, slot))
    if buf is None:
        buf = torch.zeros(N_COUNTERS, dtype=torch.int32, device=device)
        _COUNTERS[(key, slot)] = buf
    return buf


_HEAD_SYNC = {}


def head_sync(device):
    """Per-device sync words of the clustered head kernels: zeroed once, kept zero by the kernels
    (word 0 is the sticky timeout flag, see include/aimx.h AimxHead)."""
    key = torch.device(device).index if torch.device(device).index is not None else torch.cuda.current_device()
    buf = _HEAD_SYNC.get(key)
    if buf is None:
        buf = torch.zeros(HEAD_SYNC_WORDS, dtype=torch.int32, device=device)
        _HEAD_SYNC[key] = buf
    return buf


def head_sync_flag(device):
    """The sticky timeout word of the clustered head as a float64 device scalar (0 when no
    clustered head ran on `device`): no host synchronisation, so it can ride along in a collective."""
    key = torch.device(device).index if torch.device(device).index is not None else torch.cuda.current_device()
    buf = _HEAD_SYNC.get(key)
    if buf is None:
        return torch.zeros((), dtype=torch.float64, device=device)
    return buf[0].to(torch.float64)


def head_sync_timed_out(device):
    """True if a clustered head launch on `device` ever gave up waiting (host read: synchronises)."""
    key = torch.device(device).index if torch.device(device).index is not None else torch.cuda.current_device()
    buf = _HEAD_SYNC.get(key)
    return buf is not None and int(buf[0].item()) != 0


HEAD_CLUSTER_FORCE = None


def head_cluster(F=256):
    """Workgroups per 16-molecule tile of the fused head (F: the ffn width).

    The clustered head (2 workgroups per tile, about 5 % of the c2 step) relies on both workgroups
    of a cluster running at once, which holds while no other process's kernels share the GPU and
    no kernel of this process runs beside the head (see head_cluster_allowed). Otherwise the default
    is 1, which has no inter-workgroup wait at all. A wait that
    still gives up poisons that launch's outputs with NaN (head.hip cluster_poisoned), so the
    per-step NaN count of the train loop sees it on the step it happens. At F = 512 (c4) the
    chain is 4x the work per tile and 4 workgroups per tile measured best (c4 step 3.278 ms vs
    3.337 / 3.558 / 3.416 ms with 2 / 1 / 8; profiles/r03_head_f512_ab.txt). HEAD_CLUSTER_FORCE (a
    module attribute, tests and A/Bs) overrides both."""
    if HEAD_CLUSTER_FORCE is not None:
        return int(HEAD_CLUSTER_FORCE)
    if not head_cluster_allowed():
        return 1
    return 4 if F > 256 else 2


def head_cluster_allowed():
    """False when other kernels may share the CUs with the clustered head.

    * Several ranks on one GPU (the gloo rehearsal, spawned test ranks): two processes' clustered
      launches can each hold part of the CUs while their partners wait for the rest.
    Data parallelism with one GPU per rank (torchrun: LOCAL_WORLD_SIZE <= the visible GPUs, this
    rank on cuda:LOCAL_RANK) keeps the clusters: the gradient all-reduces cannot run beside the
    head. The head is the last stage of the forward, so every parameter gradient (and with it every
    bucket's collective) follows the head's backward, and the step joins every collective before the
    optimizer, ahead of the next forward's head (stream order in eager steps, graph edges in
    captured ones). Other ranks' kernels run on other GPUs. A cluster that still times out poisons
    its outputs (see head_cluster)."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1):
        return True
    try:
        lws = int(os.environ["LOCAL_WORLD_SIZE"])
        lr = int(os.environ["LOCAL_RANK"])
    except (KeyError, ValueError):
        return False
    import torch
    n = torch.cuda.device_count()
    return 0 < lws <= n and torch.cuda.current_device() == lr


def ptr(t):
    return None if t is None else t.data_ptr()


def ptr_array(tensors):
    arr = (c_ptr * max(1, len(tensors)))(*[ptr(t) for t in tensors])
    return arr


COMM_ID_BYTES = 128


def rccl_path():
    """The RCCL this process uses: PyTorch's bundled librccl.so (what torch.distributed's "nccl"
    backend runs on), else the system one."""
    cand = [os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so"), "/opt/rocm/lib/librccl.so.1",
            "/opt/rocm/lib/librccl.so"]
    for c in cand:
        if os.path.exists(c):
            return c
    raise AimxError("aimx: no librccl found")


class Comm:
    """An RCCL communicator of our own (include/aimx.h aimx_comm_*), built over an initialised
    torch.distributed group: rank 0's ncclUniqueId is broadcast through that group. Its all-reduce
    is enqueued on any stream the caller picks and captures into HIP graphs as a plain node."""

    def __init__(self, group=None, device=None):
        import torch.distributed as dist
        lib = load()
        check(lib.aimx_comm_load(rccl_path().encode()), "comm_load")
        self.rank, self.world = dist.get_rank(group), dist.get_world_size(group)
        dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        uid = (ctypes.c_uint8 * COMM_ID_BYTES)()
        if self.rank == 0:
            check(lib.aimx_comm_unique_id(uid, COMM_ID_BYTES), "comm_unique_id")
        t = torch.tensor(list(bytes(uid)), dtype=torch.uint8,
                         device=dev if dist.get_backend(group) == "nccl" else "cpu")
        dist.broadcast(t, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
        uid = (ctypes.c_uint8 * COMM_ID_BYTES)(*t.cpu().tolist())
        h = c_ptr()
        with torch.cuda.device(dev):
            check(lib.aimx_comm_init(ctypes.byref(h), uid, COMM_ID_BYTES, self.world, self.rank), "comm_init")
        self.handle = h
        # what the transport itself reports (the bench line's ddp.rccl): RCCL's version and the
        # communicator's rank count, which must equal the group's world size
        v, n = c_i32(0), c_i32(0)
        check(lib.aimx_comm_version(ctypes.byref(v)), "comm_version")
        check(lib.aimx_comm_count(h, ctypes.byref(n)), "comm_count")
        if n.value != self.world:
            raise AimxError(f"aimx.Comm: RCCL communicator has {n.value} ranks, the process group {self.world}")
        self.info = {"version": f"{v.value // 10000}.{v.value // 100 % 100}.{v.value % 100}",
                     "nranks": n.value, "library": rccl_path()}

    def all_reduce(self, buf, average=True, stream=None):
        """In-place fp32 all-reduce of `buf` on `stream` (default: the current stream)."""
        if buf.dtype != torch.float32 or not buf.is_cuda or not buf.is_contiguous():
            raise AimxError("aimx.Comm.all_reduce: contiguous fp32 device tensor")
        s = (stream or torch.cuda.current_stream(buf.device)).cuda_stream
        check(load().aimx_comm_allreduce(self.handle, buf.data_ptr(), buf.numel(), 1 if average else 0, s),
              "comm_allreduce")

    def close(self):
        if self.handle:
            load().aimx_comm_destroy(self.handle)
            self.handle = None


def copy_items(pairs):
    """The aimx_multi_copy item array of `pairs` (see multi_copy), built once for reuse: the caller
    keeps every tensor alive while the array is in use."""
    arr = (CopyItem * max(1, len(pairs)))()
    for i, (src, dst) in enumerate(pairs):
        arr[i].src = None if src is None else src.data_ptr()
        arr[i].dst = dst.data_ptr()
        arr[i].n = dst.numel()
    return arr, len(pairs)


def multi_copy_items(items, device):
    """One aimx_multi_copy launch over a prebuilt copy_items() array, on the current stream."""
    arr, n = items
    if n:
        check(load().aimx_multi_copy(arr, n, stream_ptr(device)), "multi_copy")


def multi_copy(pairs, device):
    """pairs: [(src tensor or None, dst tensor)] of fp32 contiguous tensors: dst <- src (None: 0),
    one launch (aimx_multi_copy) on the current stream."""
    if not pairs:
        return
    multi_copy_items(copy_items(pairs), device)


class options:
    """Set library path options (include/aimx.h aimx_set_option: test hooks such as AIMX_MLPW=0 for
    the per-GEMM MLP path) for the duration of a with-block; the previous table is restored on exit.
    The product library reads no environment variable for them."""

    _active = {}

    def __init__(self, **kw):
        self.kw = {k: int(v) for k, v in kw.items()}

    def __enter__(self):
        self.saved = dict(options._active)
        options._active.update(self.kw)
        _apply_options()
        return self

    def __exit__(self, *exc):
        options._active = self.saved
        _apply_options()
        return False


def _apply_options():
    lib = load()
    check(lib.aimx_clear_options(), "clear_options")
    for k, v in options._active.items():
        check(lib.aimx_set_option(k.encode(), v), f"set_option {k}")
