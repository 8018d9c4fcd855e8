"""Graph pooling — MI355X-native drop-in for reference src/models/pooling.py.

Same classes, constructor signatures and parameter names (MeanPoolingLayer 15-34,
MaxPoolingLayer 37-57, SumPoolingLayer 60-80, MultiHeadAttentionPoolingLayer 83-172,
SetAttentionPoolingLayer 175-243, create_pooling_layer 246-273). Mean/max/sum and attention
pooling run as one-molecule-per-workgroup HIP kernels (aimx.ops); forward hooks on these modules
fire as before because they are still called through nn.Module.__call__.

Number of molecules: the reference lets torch_scatter infer it as batch_indices.max()+1 (a host
sync). GNN.forward hands the pooling layer its GraphPlan built with G = total_charges.shape[0];
a standalone call builds the plan itself with the reference's max()+1 rule.
"""
from typing import Optional, Tuple

import torch
import torch.nn as nn

from aimx import _lib, ops
from aimx.plan import GraphPlan


def _plan_for(module, x, batch_indices):
    plan = getattr(module, "_aimx_plan", None)
    if plan is not None and plan.graph is not None and plan.batch is batch_indices:
        return plan
    _lib.require_device(x, batch_indices)
    return GraphPlan(x.shape[0], 1, batch=batch_indices)


class MeanPoolingLayer(nn.Module):
    """Per-molecule mean of node features (torch_scatter.scatter_mean)."""

    def forward(self, x: torch.Tensor, batch_indices: torch.Tensor) -> Tuple[torch.Tensor, None]:
        x = x.to(batch_indices.device)
        return ops.segment_pool(_plan_for(self, x, batch_indices), "mean", x), None


class MaxPoolingLayer(nn.Module):
    """Per-molecule channel-wise max (torch_scatter.scatter_max; gradient to the first arg-max)."""

    def forward(self, x: torch.Tensor, batch_indices: torch.Tensor) -> Tuple[torch.Tensor, None]:
        x = x.to(batch_indices.device)
        return ops.segment_pool(_plan_for(self, x, batch_indices), "max", x), None


class SumPoolingLayer(nn.Module):
    """Per-molecule sum of node features (torch_scatter.scatter_add)."""

    def forward(self, x: torch.Tensor, batch_indices: torch.Tensor) -> Tuple[torch.Tensor, None]:
        x = x.to(batch_indices.device)
        return ops.segment_pool(_plan_for(self, x, batch_indices), "sum", x), None


class MultiHeadAttentionPoolingLayer(nn.Module):
    """Multi-head attention pooling: per head h, s = Linear_h(x)/temperature, a = per-molecule
    softmax(s), pooled = mean over heads of sum_atoms a*x. Returns (pooled [G, C], a [H, N])."""

    def __init__(self, input_dim: int, num_heads: int = 4, initial_temperature: float = 1.0,
                 learnable_temperature: bool = True, dropout_prob: float = 0.0):
        super().__init__()
        self.num_heads = num_heads
        self.input_dim = input_dim
        self.attention_weights = nn.ModuleList([nn.Linear(input_dim, 1) for _ in range(num_heads)])
        if learnable_temperature:
            self.temperature = nn.Parameter(torch.tensor(initial_temperature))
        else:
            self.register_buffer("temperature", torch.tensor(initial_temperature))
        self.dropout = nn.Dropout(dropout_prob)
        self._pack_heads()

    def _pack_heads(self):
        """Lay the heads' weights [1, C] and biases [1] out as consecutive rows of one [H, C] / [H]
        block (same Parameters, same state_dict; values unchanged), so the kernels read them in
        place (ops.attention_pool_heads). Re-done after .to() / .cuda() (_apply)."""
        lins = list(self.attention_weights)
        if not lins:
            return
        with torch.no_grad():
            for name in ("weight", "bias"):
                ps = [getattr(lin, name) for lin in lins]
                if ops._packed_rows(ps) is not None:
                    continue
                block = torch.cat([p.detach().reshape(1, -1) for p in ps], 0)
                for i, p in enumerate(ps):
                    p.data = block[i].view(p.shape)

    def _apply(self, fn, *args, **kwargs):
        out = super()._apply(fn, *args, **kwargs)
        self._pack_heads()
        return out

    def forward(self, x: torch.Tensor, batch_indices: Optional[torch.Tensor]) -> Tuple[torch.Tensor, torch.Tensor]:
        if batch_indices is None:  # whole input is one graph (pooling.py:146-147, 163-166)
            batch_indices = torch.zeros(x.shape[0], dtype=torch.long, device=x.device)
        plan = _plan_for(self, x, batch_indices)
        pooled, attn = ops.attention_pool_heads(plan, x, [lin.weight for lin in self.attention_weights],
                                                [lin.bias for lin in self.attention_weights], self.temperature)
        if self.dropout.p > 0:
            pooled = self.dropout(pooled)
        return pooled, attn


class SetAttentionPoolingLayer(nn.Module):
    """Set2Set-style pooling (pooling.py:175-243). Not selectable from the reference CLI
    (cli.py:97-99) and not on the hot path: composed from PyTorch ops + the aimx segment kernels."""

    def __init__(self, input_dim: int, hidden_dim: int, num_steps: int = 3):
        super().__init__()
        self.input_dim = input_dim
        self.hidden_dim = hidden_dim
        self.num_steps = num_steps
        self.lstm = nn.LSTM(input_dim, hidden_dim, batch_first=True)
        self.attention = nn.Linear(hidden_dim + input_dim, 1)

    def forward(self, x: torch.Tensor, batch_indices: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        plan = _plan_for(self, x, batch_indices)
        g = plan.G
        h = torch.zeros(1, g, self.hidden_dim, device=x.device)
        c = torch.zeros(1, g, self.hidden_dim, device=x.device)
        weights = []
        a = None
        for _ in range(self.num_steps):
            out, (h, c) = self.lstm(h.transpose(0, 1), (h, c))
            per_atom = out.squeeze(1)[batch_indices]
            s = self.attention(torch.cat([x, per_atom], dim=-1)).squeeze(-1)
            a = _segment_softmax(s, batch_indices, g)
            weights.append(a)
            h = ops.segment_pool(plan, "sum", x * a.unsqueeze(-1)).unsqueeze(0)
        pooled = ops.segment_pool(plan, "sum", x * a.unsqueeze(-1))
        return pooled, torch.stack(weights, dim=0)


def _segment_softmax(s, batch, g):
    mx = torch.full((g,), float("-inf"), device=s.device, dtype=s.dtype).scatter_reduce(0, batch, s, "amax")
    e = (s - mx[batch]).exp()
    den = torch.zeros(g, device=s.device, dtype=s.dtype).index_add(0, batch, e)
    return e / den[batch]


def create_pooling_layer(pooling_type: str, input_dim: int, **kwargs) -> nn.Module:
    """Factory (pooling.py:246-273): 'attention', 'mean', 'max', 'sum', 'set_attention'."""
    if pooling_type == "attention":
        return MultiHeadAttentionPoolingLayer(input_dim, **kwargs)
    if pooling_type == "mean":
        return MeanPoolingLayer()
    if pooling_type == "max":
        return MaxPoolingLayer()
    if pooling_type == "sum":
        return SumPoolingLayer()
    if pooling_type == "set_attention":
        return SetAttentionPoolingLayer(input_dim, **kwargs)
    supported = ["attention", "mean", "max", "sum", "set_attention"]
    raise ValueError(f"Unsupported pooling type: {pooling_type}. Supported: {supported}")
