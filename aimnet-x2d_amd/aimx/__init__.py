"""aimx — MI355X-native runtime of the AIMNet-X2D message-passing / attention-pool hot path.

libaimx.so (HIP, gfx950) implements the kernels behind the C ABI in include/aimx.h; this package
binds it (ctypes) and exposes autograd operators (aimx.ops), the per-batch graph plan
(aimx.plan), batch construction (aimx.data) and synthetic inputs (aimx.synth).
"""
from ._lib import AimxError, LIB_PATH, load  # noqa: F401

__version__ = "0.1.0"
