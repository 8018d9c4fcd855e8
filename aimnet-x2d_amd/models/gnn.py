"""Main GNN — MI355X-native drop-in for reference src/models/gnn.py.

Constructor signature, attribute names, submodule registration order (hence the 73 state_dict
keys at defaults), forward signature and return tuple are the reference's (gnn.py:19-780), so
checkpoints, the unchanged trainer (trainer.py:151-159), evaluators, predictors and the forward
hooks on `pooling` / `concat_self_other` (extractors.py:110-116) keep working.

What changes is where the hot path runs:
  * one GraphPlan per forward builds the stable CSR views of the batch on the device
    (aimx/plan.py) — no torch_scatter, no host syncs (G = total_charges.shape[0]);
  * the message-passing stack (gnn.py:276-308: partial charges -> ShellConvolutionLayer -> +x,
    for every layer) is ONE fused HIP operator (aimx.ops.message_passing_stack);
  * pooling runs the one-molecule-per-workgroup HIP kernels (models/pooling.py).
Stereochemistry (off in every BASELINE config) runs per layer between the HIP layer operators, as
the reference computes it (gnn.py:288-306): the [x | cis/trans | tetrahedral] features are one HIP
operator (ops.stereo_features, csrc/stereo.hip) feeding stereochemical_embedding_2.
"""
import os
import sys
import weakref
from typing import Dict, Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from aimx import _lib, autograph, ops
from aimx.plan import GraphPlan
from utils.activation import activation_name, get_activation_function

from .layers import AimxLinear, MultiLayerPerceptron, ShellConvolutionLayer
from .pooling import create_pooling_layer


_FEATURE_KEYS = ("atom_type", "hydrogen_count", "degree", "hybridization")
# the fused post-pool head (aimx.ops.head) where it applies; False: the module path (tests, A/Bs)
FUSED_HEAD = True


def _calling_ddp():
    """The DistributedDataParallel whose constructor is reading GNN._ddp_params_and_buffers_to_ignore
    (its `self`, a few frames up: the property is read by hasattr/getattr inside DDP.__init__, after
    DDP has set its process_group), or None when something else reads it."""
    try:
        from torch.nn.parallel import DistributedDataParallel
    except ImportError:  # pragma: no cover
        return None
    f = sys._getframe(2)
    for _ in range(8):
        if f is None:
            break
        s = f.f_locals.get("self")
        if isinstance(s, DistributedDataParallel):
            return s
        f = f.f_back
    return None


def _nondefault_group(pg):
    """None for the default (world) process group, else the group itself."""
    import torch.distributed as dist
    if pg is None or not (dist.is_available() and dist.is_initialized()):
        return None
    return None if pg == dist.distributed_c10d._get_default_group() else pg


class GNN(nn.Module):
    """Graph neural network for molecular property prediction (reference gnn.py:19-149)."""

    def __init__(self, feature_sizes: Dict[str, int], hidden_dim: int, output_dim: int, num_shells: int = 3,
                 num_message_passing_layers: int = 3, dropout: float = 0.05, ffn_hidden_dim: Optional[int] = None,
                 ffn_num_layers: int = 3, pooling_type: str = "attention", task_type: str = "regression",
                 embedding_dim: int = 64, use_partial_charges: bool = False, use_stereochemistry: bool = False,
                 ffn_dropout: float = 0.05, activation_type: str = "silu", shell_conv_num_mlp_layers: int = 2,
                 shell_conv_dropout: float = 0.05, attention_num_heads: int = 4, attention_temperature: float = 1.0,
                 loss_function: str = "l1"):
        super().__init__()
        self.hidden_dim = hidden_dim
        self.num_shells = num_shells
        self.task_type = task_type
        self.embedding_dim = embedding_dim
        self.use_partial_charges = use_partial_charges
        self.use_stereochemistry = use_stereochemistry
        self.loss_function = loss_function
        if ffn_hidden_dim is None:
            ffn_hidden_dim = hidden_dim

        self._create_embeddings(feature_sizes, embedding_dim)
        self.embedding_projection = AimxLinear(embedding_dim * len(feature_sizes), hidden_dim)
        self.activation = get_activation_function(activation_type)

        self.x_other_dim = int(0.3 * hidden_dim)
        self.x_self_dim = hidden_dim - self.x_other_dim

        self._create_message_passing_layers(num_message_passing_layers, num_shells, activation_type,
                                            shell_conv_dropout, shell_conv_num_mlp_layers)
        self.pooling = create_pooling_layer(pooling_type, hidden_dim, num_heads=attention_num_heads,
                                            initial_temperature=attention_temperature)
        self._create_processing_layers(hidden_dim, activation_type)

        self.post_pooling_projection = AimxLinear(hidden_dim, ffn_hidden_dim)
        self.ffn = MultiLayerPerceptron(input_dim=ffn_hidden_dim, hidden_dim=ffn_hidden_dim, output_dim=ffn_hidden_dim,
                                        num_layers=ffn_num_layers, activation_type=activation_type,
                                        dropout=ffn_dropout, use_skip=True)
        self.skip_transform = AimxLinear(ffn_hidden_dim, ffn_hidden_dim)
        final_output_dim = output_dim * 4 if loss_function == "evidential" else output_dim
        self.output_layer = AimxLinear(ffn_hidden_dim * 2, final_output_dim)
        # constructed by the reference (gnn.py:146) but never used in forward
        self.long_range_projection = AimxLinear(hidden_dim, ffn_hidden_dim)
        self.init_weights()
        self._aimx_pack_ig()

    def _aimx_pack_ig(self):
        """Input-projection weights of every shell layer laid out as the fused stack's packed block
        (ops.pack_ig_params): read in place each step instead of one cat per forward."""
        layers = self.message_passing_layers
        if len(layers) == 0 or self.use_stereochemistry:
            return
        params = []
        for layer in layers:
            params += layer._aimx_params()
        d = layers[0].input_proj.weight.shape[0]
        k = layers[0].input_proj.weight.shape[1]
        ops.pack_ig_params(params, len(layers), len(layers[0].mlp_blocks), d, k)

    def _apply(self, fn, *args, **kwargs):
        out = super()._apply(fn, *args, **kwargs)
        self._aimx_pack_ig()
        autograph.bump_structure()  # parameters may now live in new storage
        return out

    def _create_embeddings(self, feature_sizes: Dict[str, int], embedding_dim: int):
        self.atom_type_embedding = nn.Embedding(feature_sizes["atom_type"], embedding_dim)
        self.hydrogen_count_embedding = nn.Embedding(feature_sizes["hydrogen_count"], embedding_dim)
        self.degree_embedding = nn.Embedding(feature_sizes["degree"], embedding_dim)
        self.hybridization_embedding = nn.Embedding(feature_sizes["hybridization"], embedding_dim)

    def _create_message_passing_layers(self, num_layers: int, num_shells: int, activation_type: str, dropout: float,
                                       num_mlp_layers: int):
        self.message_passing_layers = nn.ModuleList([
            ShellConvolutionLayer(atom_input_dim=self.x_other_dim, output_dim=self.x_other_dim, num_hops=num_shells,
                                  activation_type=activation_type, dropout=dropout, num_mlp_layers=num_mlp_layers)
            for _ in range(num_layers)])

    def _create_processing_layers(self, hidden_dim: int, activation_type: str):
        self.concat_self_other = AimxLinear(hidden_dim, hidden_dim)
        if self.use_stereochemistry:
            self.stereochemical_embedding = AimxLinear(hidden_dim * 3, hidden_dim)
            self.stereochemical_embedding_2 = AimxLinear(self.x_other_dim * 3, self.x_other_dim)

    # ------------------------------------------------------------------------------------------
    def forward(self, atom_features: Dict[str, torch.Tensor], multi_hop_edge_indices: torch.Tensor,
                batch_indices: torch.Tensor, total_charges: torch.Tensor, tetrahedral_indices: torch.Tensor,
                cis_indices: torch.Tensor, trans_indices: torch.Tensor
                ) -> Tuple[torch.Tensor, Optional[torch.Tensor], Optional[torch.Tensor]]:
        args = (atom_features, multi_hop_edge_indices, batch_indices, total_charges, tetrahedral_indices,
                cis_indices, trans_indices)
        _lib.require_device(multi_hop_edge_indices, batch_indices, total_charges)
        if self.training and torch.is_grad_enabled():
            sync = self._aimx_native_sync()  # wrapped by DDP: our gradient sync exists before the backward
            if sync is not None:
                sync.new_step()
        if autograph.wanted(self, args):  # per-shape-bucket graph replay (aimx/autograph.py; AIMX_AUTOGRAPH=0: off)
            return autograph.run(self, args)
        return self._aimx_forward(*args)

    def _aimx_forward(self, atom_features, multi_hop_edge_indices, batch_indices, total_charges,
                      tetrahedral_indices, cis_indices, trans_indices):
        """gnn.py:197-260 eagerly: one HIP operator per reference stage."""
        # every dropout seed of this forward (message-passing stack + FFN blocks) from ONE draw, made
        # by the embedding gather's launch
        blocks = list(self.ffn.layers)
        need = (self.message_passing_layers[0]._aimx_dropout()[0] if len(self.message_passing_layers) else False) or \
            any(b.dropout.training and b.dropout.p > 0 for b in blocks)
        slots = ops.dropout_seed_slots(self, 1 + len(blocks), multi_hop_edge_indices.device) if need else None
        # gnn.py:221-225: four lookups + cat + projection + activation, fused on the device
        # (the split of gnn.py:227-231 comes back as the two column views, so the backward needs no
        # concatenation of their gradients)
        x_self, x_other = ops.embed_project(
            [atom_features[k] for k in _FEATURE_KEYS],
            [self.atom_type_embedding.weight, self.hydrogen_count_embedding.weight, self.degree_embedding.weight,
             self.hybridization_embedding.weight],
            self.embedding_projection.weight, self.embedding_projection.bias, act=activation_name(self.activation),
            split=self.x_self_dim, seeds=slots)

        plan = GraphPlan(x_self.shape[0], self.num_shells, edges=multi_hop_edge_indices,
                         batch=batch_indices, num_graphs=total_charges.shape[0])
        if need:  # (MC-dropout may switch single Dropout modules on in eval mode: follow their flags)
            seeds = slots[1]
            self._aimx_stack_seed = seeds[0:1]
            for i, blk in enumerate(blocks):
                blk._aimx_seed = seeds[1 + i:2 + i]
        try:
            x_other_updated = self._message_passing_forward(x_other, multi_hop_edge_indices, batch_indices,
                                                            total_charges, tetrahedral_indices, cis_indices,
                                                            trans_indices, plan=plan)
        finally:
            self._aimx_stack_seed = None
        partial_charges = None
        if self.use_partial_charges and x_other_updated.shape[-1] >= 2:
            partial_charges = x_other_updated[:, 0].clone()

        x = self.concat_self_other(torch.cat([x_self, x_other_updated], dim=-1))
        self.pooling._aimx_plan = plan
        try:
            x_pooled, attention_weights = self.pooling(x, batch_indices)
        finally:
            self.pooling._aimx_plan = None

        # a caller that reads only the first rows of the output (GraphedTrainStep, the autograph: the
        # rows after them are padding molecules) sets _aimx_head_rows, and the post-pool chain
        # (gnn.py:252-258: a per-molecule function) runs on those rows alone
        # (only for the module path: the fused head's tiles of 4-8 molecules gain nothing from a
        # padding molecule less, while the slice's backward costs a zero fill and a copy)
        rows = self.__dict__.get("_aimx_head_rows")
        if rows is not None and 0 < rows < x_pooled.shape[0] and not self._aimx_head_ok():
            x_pooled = x_pooled[:rows]
        try:
            if self._aimx_head_ok():
                # gnn.py:252-258 as one fused operator forward and backward (aimx.ops.head)
                b0 = blocks[0]
                output = ops.head(
                    x_pooled, self.post_pooling_projection.weight, self.post_pooling_projection.bias,
                    [(b.linear1.weight, b.linear1.bias, b.linear2.weight, b.linear2.bias) for b in blocks],
                    self.skip_transform.weight, self.skip_transform.bias, self.output_layer.weight,
                    self.output_layer.bias, act=activation_name(b0.activation), drop_p=b0.dropout.p,
                    training=b0.dropout.training, seed=getattr(b0, "_aimx_seed", None),
                    skips=[b.use_skip for b in blocks])
            else:
                x = self.ffn(self.post_pooling_projection(x_pooled))
                skip_connection = self.skip_transform(x)
                output = self.output_layer(torch.cat([x, skip_connection], dim=-1))
        finally:
            for blk in blocks:
                blk._aimx_seed = None
        return output, attention_weights, partial_charges

    def _aimx_head_ok(self) -> bool:
        """The fused head covers the reference's post-pool chain when every LinearBlock is F -> F
        with one activation and one dropout setting, F <= 256, F and the input width multiples of 32
        (FUSED_HEAD = False, a module attribute for tests and A/Bs, disables it). Wider chains run
        the module path, whose G x F x F products take k_gemm_deep: at c4 (F = 512) it measured
        2.370 vs 2.388 ms per step on the fused 8-molecule kernels; at c2 (F = 256) the fused
        kernels keep 0.707 vs 0.815 ms (profiles/r06_head_path_ab.txt). (ops.head itself still
        takes F up to HEAD_MAX_F = 512.)"""
        if not FUSED_HEAD:
            return False
        pp, blocks = self.post_pooling_projection, list(self.ffn.layers)
        F = pp.out_features
        if not (32 <= F <= 256 and F % 32 == 0 and pp.in_features % 32 == 0 and 1 <= len(blocks) <= 8):
            return False
        if self.skip_transform.in_features != F or self.skip_transform.out_features != F or \
                self.output_layer.in_features != 2 * F:
            return False
        b0 = blocks[0]
        for b in blocks:
            if b.skip_proj is not None or b.linear1.in_features != F or b.linear1.out_features != F or \
                    b.linear2.out_features != F or type(b.activation) is not type(b0.activation) or \
                    b.dropout.p != b0.dropout.p or b.dropout.training != b0.dropout.training:
                return False
        # the fused kernels read the weight matrices with 16-byte loads: weights moved into other
        # storage (torch.nn.utils.vector_to_parameters puts them at arbitrary float offsets of one
        # vector) take the module path, which accepts any alignment
        ws = [pp.weight, self.skip_transform.weight, self.output_layer.weight]
        ws += [w for b in blocks for w in (b.linear1.weight, b.linear2.weight)]
        return all(w.data_ptr() % 16 == 0 and w.is_contiguous() for w in ws)

    def _embed_atomic_features(self, atom_features: Dict[str, torch.Tensor]) -> torch.Tensor:
        return torch.cat([
            self.atom_type_embedding(atom_features["atom_type"]),
            self.hydrogen_count_embedding(atom_features["hydrogen_count"]),
            self.degree_embedding(atom_features["degree"]),
            self.hybridization_embedding(atom_features["hybridization"]),
        ], dim=-1)

    def _message_passing_forward(self, x_other, multi_hop_edge_indices, batch_indices, total_charges,
                                 tetrahedral_indices, cis_indices, trans_indices, plan=None):
        """gnn.py:276-308. Skipped entirely when there are no edges (gnn.py:287)."""
        if multi_hop_edge_indices.numel() == 0:
            return x_other
        if plan is None:
            plan = GraphPlan(x_other.shape[0], self.num_shells, edges=multi_hop_edge_indices, batch=batch_indices,
                             num_graphs=total_charges.shape[0])
        layers = self.message_passing_layers
        first = layers[0]
        training, p = first._aimx_dropout()
        seed = getattr(self, "_aimx_stack_seed", None)
        if training and seed is None:
            seed = ops.dropout_seeds(self, 1, x_other.device)
        if not self.use_stereochemistry:
            params = []
            for layer in layers:
                params += layer._aimx_params()
            return ops.message_passing_stack(plan, x_other, params, num_hops=self.num_shells,
                                             num_layers=len(layers), num_mlp=len(first.mlp_blocks),
                                             act=activation_name(first.activation), use_pc=self.use_partial_charges,
                                             total_charges=total_charges, training=training, drop_p=p,
                                             drop_seed=seed, single=False)
        # stereochemistry: PyTorch ops between the per-layer HIP operators (gnn.py:288-306)
        x = x_other
        for layer in layers:
            if self.use_partial_charges:
                x = ops.partial_charges(plan, x, total_charges)
            x = self._apply_stereochemistry(x, tetrahedral_indices, cis_indices, trans_indices)
            layer._aimx_plan = plan
            try:
                x = layer(x, multi_hop_edge_indices[:, 0], multi_hop_edge_indices[:, 1]) + x
            finally:
                layer._aimx_plan = None
        return x

    # -- stereochemistry (plain PyTorch; reference gnn.py:310-509) ----------------------------
    def _apply_stereochemistry(self, x_other, tetrahedral_indices, cis_indices, trans_indices):
        # [x | cis/trans | tetrahedral] in one HIP op (csrc/stereo.hip) forward and backward; the
        # two methods below keep the reference's PyTorch formulation as module API
        return self.stereochemical_embedding_2(ops.stereo_features(x_other, tetrahedral_indices, cis_indices,
                                                                   trans_indices))

    def _tetrahedral_feature_calculation_physics_inspired(self, atom_features, tetrahedral_indices):
        """Chirality term on unit-normalised neighbour features, rescaled by tanh(mean |x| / 3),
        added onto the centre's neighbours; rows of atoms not named in any centre are zeroed."""
        if tetrahedral_indices.numel() == 0:
            return atom_features
        out = atom_features.clone()
        nb = out[tetrahedral_indices]                                    # [M, 4, D]
        mag = nb.norm(dim=-1, keepdim=True)                              # [M, 4, 1]
        u = F.normalize(nb, dim=-1, eps=1e-8)
        sq = u * u
        r1, r2, r3 = [1, 2, 3, 0], [2, 3, 0, 1], [3, 0, 1, 2]            # cyclic shifts by -1, -2, -3
        chir = sq[:, r1] * (u[:, r2] - u[:, r3]) + sq[:, r2] * (u[:, r3] - u[:, r1]) + sq[:, r3] * (u[:, r1] - u[:, r2])
        chir = chir * torch.tanh(mag.mean(dim=1, keepdim=True) / 3.0)
        flat_idx = tetrahedral_indices.reshape(-1)
        out.index_add_(0, flat_idx, chir.reshape(-1, out.shape[-1]))
        keep = torch.zeros(out.shape[0], dtype=torch.bool, device=out.device)
        keep[flat_idx] = True
        out[~keep] = 0.0
        return out

    def _cis_trans_calculation(self, atom_features, cis_indices, trans_indices):
        """Adds -x[cis_indices[0]] at cis_indices[1] and +x[trans_indices[0]] at trans_indices[1]
        (rows 0 and 1 of the collated [M, 2] tensors, exactly as the reference indexes them)."""
        if cis_indices.numel() == 0 and trans_indices.numel() == 0:
            return atom_features
        dev, d = atom_features.device, atom_features.shape[1]
        tgts, vals = [], []
        if cis_indices.numel() > 0:
            tgts.append(cis_indices[1])
            vals.append(-atom_features[cis_indices[0]])
        if trans_indices.numel() > 0:
            tgts.append(trans_indices[1])
            vals.append(atom_features[trans_indices[0]])
        t = torch.cat(tgts) if tgts else torch.empty(0, dtype=torch.long, device=dev)
        v = torch.cat(vals) if vals else torch.empty(0, d, device=dev)
        if t.numel() == 0:
            return atom_features
        return atom_features.scatter_add(0, t.unsqueeze(1).expand(-1, d), v)

    def _partial_charge_calculation(self, atom_features, batch_indices, total_charges):
        """Charge equilibration (gnn.py:622-658) as the HIP segment kernel."""
        plan = GraphPlan(atom_features.shape[0], 1, batch=batch_indices, num_graphs=total_charges.shape[0])
        return ops.partial_charges(plan, atom_features, total_charges)

    # ------------------------------------------------------------------------------------------
    def init_weights(self) -> None:
        """Xavier init of the top-level projections, embeddings and attention heads; biases zero;
        message-passing layers keep PyTorch's default init (reference gnn.py:660-703)."""
        linear_layers = [self.embedding_projection, self.concat_self_other, self.post_pooling_projection,
                         self.skip_transform, self.output_layer, self.long_range_projection]
        if hasattr(self, "stereochemical_embedding"):
            linear_layers += [self.stereochemical_embedding, self.stereochemical_embedding_2]
        for layer in linear_layers:
            nn.init.xavier_uniform_(layer.weight)
            if layer.bias is not None:
                nn.init.zeros_(layer.bias)
        for emb in (self.atom_type_embedding, self.degree_embedding, self.hybridization_embedding,
                    self.hydrogen_count_embedding):
            nn.init.xavier_uniform_(emb.weight)
        for layer in self.message_passing_layers:
            if hasattr(layer, "init_weights"):
                layer.init_weights()
        if hasattr(self.pooling, "attention_weights"):
            for head in self.pooling.attention_weights:
                nn.init.xavier_uniform_(head.weight)
                if head.bias is not None:
                    nn.init.zeros_(head.bias)

    # -- DistributedDataParallel (reference runner.py:703-707) -----------------------------------
    # DDP's constructor reads `module._ddp_params_and_buffers_to_ignore` (the hook it offers modules
    # for parameters whose gradients they synchronise themselves). Here it is a property: reading it
    # is how the model learns it is being wrapped. It then keeps ONE used parameter (_DDP_ANCHOR) in
    # DDP's reducer — DDP refuses a module with none, and that parameter's hook is what DDP's own
    # end-of-backward bookkeeping runs on — and averages every other gradient itself
    # (utils.distributed.GradientSync: bucketed RCCL all-reduce over our own communicator), which a
    # graph replay can do in a handful of launches where DDP's reducer copies each of the 73
    # gradients into its buckets and back. AIMX_NATIVE_DDP=0 leaves every parameter to DDP.
    _DDP_ANCHOR = "output_layer.bias"

    @property
    def _ddp_params_and_buffers_to_ignore(self):
        user = list(self.__dict__.get("_aimx_ddp_user_ignore", ()))
        if os.environ.get("AIMX_NATIVE_DDP", "1") == "0":
            if user:
                return user
            raise AttributeError("_ddp_params_and_buffers_to_ignore")
        if not self.__dict__.get("_aimx_ddp_native", False):
            # the wrapper whose constructor is asking: its process group is the one to average over
            # (DDP(module, process_group=subgroup)) and its require_backward_grad_sync flag says
            # whether a backward syncs at all (ddp.no_sync() micro-batches)
            ddp = _calling_ddp()
            group = _nondefault_group(ddp.process_group) if ddp is not None else None
            self.__dict__["_aimx_ddp_native"] = True
            self.__dict__["_aimx_ddp_group"] = group
            self.__dict__["_aimx_ddp_ref"] = weakref.ref(ddp) if ddp is not None else None
            # DDP's constructor broadcasts the start state of what it syncs; this is ours (the same
            # collective order on every member: every member is inside DDP's constructor)
            from utils.distributed import broadcast_parameters
            broadcast_parameters([p for n, p in self.named_parameters() if n != self._DDP_ANCHOR and n not in user],
                                 0, group)
        return [n for n, _ in self.named_parameters() if n != self._DDP_ANCHOR] + \
            [n for n in user if n not in dict(self.named_parameters())]

    @_ddp_params_and_buffers_to_ignore.setter
    def _ddp_params_and_buffers_to_ignore(self, names):
        # DistributedDataParallel._set_params_and_buffers_to_ignore_for_model(module, names)
        self.__dict__["_aimx_ddp_user_ignore"] = list(names)

    def _aimx_native_sync(self):
        """The gradient sync of the parameters DDP was told to ignore (None unless wrapped)."""
        if not self.__dict__.get("_aimx_ddp_native", False):
            return None
        import torch.distributed as dist
        if not (dist.is_available() and dist.is_initialized()):
            return None
        ref = self.__dict__.get("_aimx_ddp_ref")
        ddp = ref() if ref is not None else None
        join = getattr(ddp, "_join_config", None)
        if join is not None and join.enable:
            raise _lib.AimxError(
                "aimx native DDP: DistributedDataParallel.join() (uneven inputs) is not supported by the "
                "model's own gradient sync; construct the model with AIMX_NATIVE_DDP=0 to let DDP's reducer "
                "sync every parameter")
        sync = self.__dict__.get("_aimx_sync")
        if sync is None:
            # built once: DDP itself holds the Parameter objects it wrapped, so a wrapped model's
            # parameters are not replaced or moved afterwards (DDP would break first)
            from utils.distributed import GradientSync
            named = dict(self.named_parameters())
            params = [p for n, p in named.items() if n != self._DDP_ANCHOR and
                      n not in self.__dict__.get("_aimx_ddp_user_ignore", ())]
            # always: the collectives run at world size 1 too, as DDP's do; auto_finish: the
            # reference trainer never calls finish() (DDP finalises in an engine callback); the
            # wrapper's group, and its no_sync() flag as the gate of every backward's sync
            gate = (lambda r=ref: (r() is None) or bool(r().require_backward_grad_sync)) if ref is not None else None
            sync = GradientSync(params, process_group=self.__dict__.get("_aimx_ddp_group"),
                                unused=self.unused_parameters(), always=True, broadcast_params=False,
                                auto_finish=True, gate=gate)
            sync.anchor_param = named.get(self._DDP_ANCHOR)
            self.__dict__["_aimx_sync"] = sync
        return sync

    def unused_parameters(self):
        """Parameters the forward never touches: long_range_projection (gnn.py:146) and, with
        stereochemistry, stereochemical_embedding (gnn.py:194) — the reference constructs both and
        never calls them. Data-parallel sync leaves them out (GradientSync(unused=))."""
        out = list(self.long_range_projection.parameters())
        if hasattr(self, "stereochemical_embedding"):
            out += list(self.stereochemical_embedding.parameters())
        return out

    def get_model_info(self) -> Dict[str, object]:
        total = sum(p.numel() for p in self.parameters())
        trainable = sum(p.numel() for p in self.parameters() if p.requires_grad)
        return {
            "total_parameters": total,
            "trainable_parameters": trainable,
            "hidden_dim": self.hidden_dim,
            "num_shells": self.num_shells,
            "embedding_dim": self.embedding_dim,
            "task_type": self.task_type,
            "use_partial_charges": self.use_partial_charges,
            "use_stereochemistry": self.use_stereochemistry,
            "loss_function": self.loss_function,
            "num_message_passing_layers": len(self.message_passing_layers),
            "pooling_type": type(self.pooling).__name__,
        }

    def __repr__(self) -> str:
        info = self.get_model_info()
        return (f"GNN(\n  parameters={info['total_parameters']:,}\n  hidden_dim={info['hidden_dim']}\n"
                f"  num_shells={info['num_shells']}\n  task_type='{info['task_type']}'\n"
                f"  loss_function='{info['loss_function']}'\n"
                f"  features=[partial_charges={info['use_partial_charges']}, "
                f"stereochemistry={info['use_stereochemistry']}]\n)")


class GNNConfig:
    """Build GNN kwargs from parsed CLI arguments (reference gnn.py:738-780)."""

    FEATURE_SIZES = {"atom_type": 119, "hydrogen_count": 9, "degree": 7, "hybridization": 7}

    @staticmethod
    def from_args(args) -> Dict[str, object]:
        keys = ["hidden_dim", "num_shells", "num_message_passing_layers", "ffn_hidden_dim", "ffn_num_layers",
                "pooling_type", "task_type", "embedding_dim", "use_partial_charges", "use_stereochemistry",
                "ffn_dropout", "activation_type", "shell_conv_num_mlp_layers", "shell_conv_dropout",
                "attention_num_heads", "attention_temperature", "loss_function"]
        cfg = {"feature_sizes": dict(GNNConfig.FEATURE_SIZES), "output_dim": getattr(args, "output_dim", 1)}
        for k in keys:
            cfg[k] = getattr(args, k)
        return cfg

    @staticmethod
    def create_model_from_args(args) -> GNN:
        return GNN(**GNNConfig.from_args(args))
