"""Losses of the train step — drop-ins for the reference's L1 criteria (fused HIP kernels).

reference src/training/trainer.py:24-35 picks nn.L1Loss() for a single task and
WeightedL1Loss(weights) (src/models/losses.py:14-48) for multitask; both run here as one
forward and one backward launch (aimx.ops.l1_loss) instead of ATen's 4-8 elementwise/reduction
kernels. Same call signature criterion(y_pred, y_true) -> scalar, same math, same gradient
(sign(0) = 0). The MSE and evidential criteria are not on the hot path and stay the reference's.
"""
import torch
import torch.nn as nn

from aimx import ops


class L1Loss(nn.Module):
    """nn.L1Loss() (reduction='mean') on the fused kernel."""

    def forward(self, y_pred: torch.Tensor, y_true: torch.Tensor) -> torch.Tensor:
        return ops.l1_loss(y_pred, y_true)

    def padded(self, y_pred: torch.Tensor, y_true: torch.Tensor, rows: int, accum=None, grad_of=None) -> torch.Tensor:
        """forward(y_pred[:rows], y_true) for a static padded batch, the padding rows' zero gradient
        written by the same backward launch (no slice-backward fill + copy); accum, grad_of:
        ops.l1_loss."""
        return ops.l1_loss(y_pred, y_true, rows=rows, accum=accum, grad_of=grad_of)


class WeightedL1Loss(nn.Module):
    """sum over tasks of w_t |y_pred - y_true|, averaged over samples (reference losses.py:14-48)."""

    def __init__(self, weights: torch.Tensor):
        super().__init__()
        self.register_buffer("weights", weights)

    def forward(self, y_pred: torch.Tensor, y_true: torch.Tensor) -> torch.Tensor:
        return ops.l1_loss(y_pred, y_true, self.weights.to(y_pred.device), per_sample=True)

    def padded(self, y_pred: torch.Tensor, y_true: torch.Tensor, rows: int, accum=None, grad_of=None) -> torch.Tensor:
        return ops.l1_loss(y_pred, y_true, self.weights.to(y_pred.device), per_sample=True, rows=rows, accum=accum,
                           grad_of=grad_of)
