"""Layers of the molecular GNN — MI355X-native drop-in for reference src/models/layers.py.

Same classes, constructor signatures, submodule names and state_dict keys as the reference
(ShellConvolutionLayer layers.py:17-167, LinearBlock 170-219, MultiLayerPerceptron 222-267).
ShellConvolutionLayer's message passing and node-update MLP run as HIP kernels through
aimx.ops (hop = stable-CSR segmented gather-sum, MLP = fused fp32 MFMA GEMMs); LinearBlock and
MultiLayerPerceptron act on per-molecule rows (G << N) and stay on PyTorch/hipBLASLt.
"""
from typing import List

import torch
import torch.nn as nn

from aimx import ops
from aimx.plan import GraphPlan
from utils.activation import activation_name, get_activation_function


class ShellConvolutionLayer(nn.Module):
    """Shell-based graph convolution (reference layers.py:17-108).

    forward(x [N,D], target [E], src [E]) = a_L + global_skip, where
      F = [x | hop_1 | ... | hop_h] (hop_j = chunk j of scatter_add(x[src % N], target)),
      a_0 = act(input_proj(F)), a_{k+1} = linear_2(dropout(act(linear_1(a_k)))) + a_k,
      global_skip = global_skip_proj(F), or a_0.clone() when the reference builds no
      global_skip_proj (input_dim == output_dim, layers.py:61,86-89).

    Every configuration the reference accepts runs on the HIP kernels: any number of MLP blocks
    (0 included, cli.py:106-107) on the fused stack when the layer is square (atom_input_dim ==
    output_dim, the GNN's layers), else the composed path (hop kernel, MFMA GEMMs with fused
    epilogues, the fused LinearBlock operator; `_stacked`).
    """

    def __init__(self, atom_input_dim: int, output_dim: int, num_hops: int = 3, dropout: float = 0.00,
                 activation_type: str = "silu", num_mlp_layers: int = 2):
        super().__init__()
        self.num_hops = num_hops
        input_dim = atom_input_dim * (num_hops + 1)
        self.activation = get_activation_function(activation_type)
        self.input_proj = nn.Linear(input_dim, output_dim)
        self.mlp_blocks = nn.ModuleList()
        for _ in range(num_mlp_layers):
            self.mlp_blocks.append(nn.ModuleDict({
                "linear_1": nn.Linear(output_dim, output_dim),
                "activation": get_activation_function(activation_type),
                "dropout": nn.Dropout(dropout),
                "linear_2": nn.Linear(output_dim, output_dim),
            }))
        self.global_skip_proj = nn.Linear(input_dim, output_dim) if input_dim != output_dim else None
        self._atom_input_dim = atom_input_dim
        self._output_dim = output_dim

    # -- kernel plumbing -------------------------------------------------------------------
    def _stacked(self):
        """The fused stack's layer shape (aimx_shell_stack_*): atom_input_dim == output_dim (so a
        global_skip_proj exists) and at most 8 MLP blocks — every layer the reference GNN builds."""
        return self.global_skip_proj is not None and self._atom_input_dim == self._output_dim and \
            len(self.mlp_blocks) <= 8

    def _aimx_params(self):
        """[input_proj.W, global_skip_proj.W, input_proj.b, global_skip_proj.b, (w1, b1, w2, b2) per
        block]; the operator packs [Wi ; Wg] of all layers with one cat kernel."""
        if not self._stacked():
            raise ValueError("aimx: the fused message-passing stack takes square shell layers with a "
                             "global_skip_proj (GNN layers); ShellConvolutionLayer.forward handles the rest")
        p = [self.input_proj.weight, self.global_skip_proj.weight, self.input_proj.bias, self.global_skip_proj.bias]
        for b in self.mlp_blocks:
            p += [b["linear_1"].weight, b["linear_1"].bias, b["linear_2"].weight, b["linear_2"].bias]
        return p

    def _aimx_dropout(self):
        d = self.mlp_blocks[0]["dropout"] if len(self.mlp_blocks) else None
        return (bool(d is not None and d.training and d.p > 0), float(d.p) if d is not None else 0.0)

    def _aimx_act(self):
        return activation_name(self.activation)

    # -- reference API ---------------------------------------------------------------------
    def forward(self, x: torch.Tensor, target: torch.Tensor, src: torch.Tensor) -> torch.Tensor:
        plan = getattr(self, "_aimx_plan", None)
        if plan is None or plan.N != x.shape[0] or plan.num_hops != self.num_hops:
            plan = GraphPlan(x.shape[0], self.num_hops, target=target, src=src)
        training, p = self._aimx_dropout()
        if not self._stacked():
            return self._composed(plan, x, training, p)
        seed = torch.randint(0, 2 ** 62, (1,), device=x.device, dtype=torch.int64) if training else None
        return ops.message_passing_stack(plan, x, self._aimx_params(), num_hops=self.num_hops, num_layers=1,
                                         num_mlp=len(self.mlp_blocks), act=self._aimx_act(), training=training,
                                         drop_p=p, drop_seed=seed, single=True)

    def _composed(self, plan, x, training, p):
        """layers.py:75-108 for the shapes the fused stack does not take (rectangular layers, no
        global_skip_proj): the hop kernel, MFMA GEMMs with the activation fused in the epilogue and
        the fused LinearBlock operator (linear_1 -> act -> dropout -> linear_2 + skip, layers.py:92-103)."""
        n = x.shape[0]
        F = torch.cat([x] + list(torch.split(ops.hop(plan, x), n, dim=0)), dim=-1)
        act = self._aimx_act()
        a = ops.linear(F, self.input_proj.weight, self.input_proj.bias, act)
        skip = ops.linear(F, self.global_skip_proj.weight, self.global_skip_proj.bias) \
            if self.global_skip_proj is not None else a.clone()
        for b in self.mlp_blocks:
            a = ops.linear_block(a, b["linear_1"].weight, b["linear_1"].bias, b["linear_2"].weight, b["linear_2"].bias,
                                 act, p, training, True)
        return a + skip

    def message_passing(self, atom_features: torch.Tensor, target: torch.Tensor, src: torch.Tensor) -> List[torch.Tensor]:
        """Per-hop aggregated features (reference layers.py:133-167): chunk j of
        scatter_add(atom_features[src % N], target, dim_size = num_hops * N)."""
        n = atom_features.shape[0]
        if target.numel() == 0:
            return [torch.zeros_like(atom_features) for _ in range(self.num_hops)]
        plan = getattr(self, "_aimx_plan", None)
        if plan is None or plan.N != n or plan.num_hops != self.num_hops:
            plan = GraphPlan(n, self.num_hops, target=target, src=src)
        agg = ops.hop(plan, atom_features)
        return list(torch.split(agg, n, dim=0))


class AimxLinear(nn.Linear):
    """nn.Linear whose forward runs on the fused fp32 MFMA GEMM (aimx.ops.linear): same parameters,
    state_dict keys, isinstance and hook behaviour as nn.Linear; the weight/bias gradients come from
    one split-K GEMM with the bias column fused (deterministic)."""

    def forward(self, x: torch.Tensor, act: str = None) -> torch.Tensor:
        return ops.linear(x, self.weight, self.bias, act)


class LinearBlock(nn.Module):
    """Linear -> activation -> dropout -> linear with an optional identity skip (layers.py:170-219)."""

    def __init__(self, input_dim: int, output_dim: int, activation_type: str = "silu", dropout: float = 0.0,
                 use_skip: bool = True):
        super().__init__()
        self.use_skip = use_skip and (input_dim == output_dim)
        self.linear1 = AimxLinear(input_dim, output_dim)
        self.activation = get_activation_function(activation_type)
        self.dropout = nn.Dropout(dropout)
        self.linear2 = AimxLinear(output_dim, output_dim)
        # the reference's projection branch is unreachable (use_skip implies equal widths)
        self.skip_proj = None

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        # one fused operator: linear1 + activation + dropout (hash mask, honours self.dropout's
        # training flag) + linear2 + skip, with a fused backward (aimx.ops.linear_block)
        # (GNN.forward may hand every block its dropout seed from one draw: _aimx_seed)
        return ops.linear_block(x, self.linear1.weight, self.linear1.bias, self.linear2.weight, self.linear2.bias,
                                activation_name(self.activation), self.dropout.p, self.dropout.training,
                                self.use_skip, seed=getattr(self, "_aimx_seed", None))


class MultiLayerPerceptron(nn.Module):
    """Stack of LinearBlocks: in->hidden, (num_layers-2) x hidden->hidden with skips, hidden->out
    (layers.py:222-267)."""

    def __init__(self, input_dim: int, hidden_dim: int, output_dim: int, num_layers: int = 2,
                 activation_type: str = "silu", dropout: float = 0.0, use_skip: bool = True):
        super().__init__()
        if num_layers == 1:
            blocks = [LinearBlock(input_dim, output_dim, activation_type, dropout, False)]
        else:
            blocks = [LinearBlock(input_dim, hidden_dim, activation_type, dropout, False)]
            blocks += [LinearBlock(hidden_dim, hidden_dim, activation_type, dropout, use_skip)
                       for _ in range(num_layers - 2)]
            blocks.append(LinearBlock(hidden_dim, output_dim, activation_type, dropout, False))
        self.layers = nn.ModuleList(blocks)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        for layer in self.layers:
            x = layer(x)
        return x
