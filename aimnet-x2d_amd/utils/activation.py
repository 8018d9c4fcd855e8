"""Activation functions (mirror of reference src/utils/activation.py:9-47).

The HIP kernels fuse these by kind (include/aimx.h AIMX_ACT_*); the nn.Module instances are kept so
module structure, repr and state_dict match the reference.
"""
import torch.nn as nn

_ACTIVATIONS = {
    "relu": nn.ReLU,
    "leakyrelu": nn.LeakyReLU,
    "elu": nn.ELU,
    "gelu": nn.GELU,
    "silu": nn.SiLU,
}


def get_activation_function(activation_type: str) -> nn.Module:
    """Return a fresh activation module for `activation_type`; ValueError if unsupported."""
    if activation_type not in _ACTIVATIONS:
        supported = ", ".join(_ACTIVATIONS)
        raise ValueError(f"Invalid activation type: {activation_type}. Supported: {supported}")
    return _ACTIVATIONS[activation_type]()


def get_activation_by_name(name: str) -> nn.Module:
    """Alias kept for backwards compatibility (reference activation.py:38-47)."""
    return get_activation_function(name)


def activation_name(module: nn.Module) -> str:
    """Inverse map: module instance -> kernel activation name."""
    for k, cls in _ACTIVATIONS.items():
        if type(module) is cls:
            return k
    raise ValueError(f"aimx: unsupported activation module {type(module).__name__}")
