"""ORACLE (test infrastructure): functional fp32 torch-CPU restatement of the reference GNN.

Every function cites the reference lines it restates (paths relative to the reference root).
Parameters are passed as a flat dict with the reference's state_dict keys (73 at defaults), so the
same weights drive the reference, this oracle and the HIP implementation. Backward comes from
torch autograd over these CPU ops (the same ATen ops the reference reaches).

Eval-mode semantics (dropout off) unless `training=True`, in which case torch's own dropout is
used (bitwise parity in training mode is not a goal: the reference's dropout masks come from the
torch CPU RNG).
"""
import math

import torch
import torch.nn.functional as F

ACTS = ("relu", "leakyrelu", "elu", "gelu", "silu")


def act(name, x):
    """utils/activation.py:9-34 (nn.ReLU / LeakyReLU(0.01) / ELU(1.0) / GELU(erf) / SiLU)."""
    if name == "relu":
        return F.relu(x)
    if name == "leakyrelu":
        return F.leaky_relu(x, 0.01)
    if name == "elu":
        return F.elu(x)
    if name == "gelu":
        return F.gelu(x)
    if name == "silu":
        return F.silu(x)
    raise ValueError(f"Invalid activation type: {name}")


def linear(p, name, x):
    return F.linear(x, p[name + ".weight"], p[name + ".bias"])


def dropout(x, prob, training):
    return F.dropout(x, prob, training) if training and prob > 0 else x


def message_passing(x, target, src, num_hops):
    """layers.py:133-167: out = zeros(h*N, D).scatter_add_(0, target, x[src % N]); split into h chunks."""
    n, d = x.shape
    if target.numel() == 0:
        return [torch.zeros_like(x) for _ in range(num_hops)]
    true_src = src % n
    rows = x[true_src]
    agg = torch.zeros(num_hops * n, d, dtype=x.dtype, device=x.device).scatter_add_(
        0, target.unsqueeze(1).expand(-1, d), rows)
    return list(torch.split(agg, n, dim=0))


def shell_layer(p, pre, x, target, src, cfg, training=False):
    """layers.py:63-108 (ShellConvolutionLayer.forward)."""
    a = cfg["activation"]
    chunks = message_passing(x, target, src, cfg["num_shells"])
    feats = torch.cat([x] + chunks, dim=-1)
    h = act(a, linear(p, pre + "input_proj", feats))
    # layers.py:61,86-89: no global_skip_proj when input_dim (= D_in (h+1)) == output_dim
    skip = linear(p, pre + "global_skip_proj", feats) if pre + "global_skip_proj.weight" in p else h.clone()
    for k in range(cfg["shell_conv_num_mlp_layers"]):
        b = f"{pre}mlp_blocks.{k}."
        y = linear(p, b + "linear_1", h)
        y = act(a, y)
        y = dropout(y, cfg["shell_conv_dropout"], training)
        y = linear(p, b + "linear_2", y)
        h = y + h
    return h + skip


def partial_charges(x, batch, total_charges):
    """gnn.py:622-658 (_partial_charge_calculation)."""
    q, f, rest = x.split([1, 1, x.shape[-1] - 2], dim=-1)
    f = torch.clamp(f, min=1e-6)
    g = total_charges.shape[0]
    qu = torch.zeros(g, 1, dtype=q.dtype, device=q.device).scatter_add(0, batch.unsqueeze(1), q)
    fu = torch.zeros(g, 1, dtype=q.dtype, device=q.device).scatter_add(0, batch.unsqueeze(1), f) + 1e-6
    fu = torch.clamp(fu, min=1e-6)
    dq = total_charges.unsqueeze(-1) - qu
    f_new = f / fu[batch]
    q_new = q + f_new * dq[batch]
    return torch.cat([q_new, f_new, rest], dim=-1)


def segment_softmax(scores, batch, num_graphs):
    """torch_scatter.scatter_softmax along dim 1 of [H, N] (pooling.py:143-145)."""
    h, n = scores.shape
    idx = batch.unsqueeze(0).expand(h, n)
    mx = torch.full((h, num_graphs), float("-inf"), dtype=scores.dtype, device=scores.device).scatter_reduce(1, idx, scores, "amax", include_self=True)
    mx = torch.where(torch.isinf(mx) & (mx < 0), torch.zeros_like(mx), mx)
    e = (scores - mx.gather(1, idx)).exp()
    s = torch.zeros(h, num_graphs, dtype=scores.dtype, device=scores.device).scatter_add_(1, idx, e)
    return e / s.gather(1, idx)


def attention_pool(p, pre, x, batch, num_heads, num_graphs, capture=None):
    """pooling.py:122-172 (MultiHeadAttentionPoolingLayer.forward), dropout p=0. `capture` (dict)
    receives the scores [H, N] (their .grad is retained) and tau: temperature_scale() below."""
    tau = p[pre + "temperature"]
    scores = torch.stack([linear(p, f"{pre}attention_weights.{i}", x).squeeze(-1) / tau
                          for i in range(num_heads)], 0)
    if capture is not None and scores.requires_grad:
        scores.retain_grad()
        capture["pool_scores"], capture["pool_tau"] = scores, tau
    a = segment_softmax(scores, batch, num_graphs)
    weighted = x.unsqueeze(0).expand(num_heads, -1, -1) * a.unsqueeze(-1)
    idx = batch.view(1, -1, 1).expand_as(weighted)
    pooled = torch.zeros(num_heads, num_graphs, x.shape[1], dtype=x.dtype, device=x.device).scatter_add_(1, idx, weighted)
    return pooled.mean(dim=0), a


def temperature_scale(capture):
    """After backward: sum_hj |dL/ds_hj * s_hj| / |tau| — the magnitude of the terms whose signed sum
    is dL/dtau (s = x.W_h / tau + ..., ds/dtau = -s / tau). The temperature gradient sums H*N terms of
    both signs (softmax shift invariance makes them cancel to a few % of that magnitude), so its fp32
    rounding is judged against this scale (tests/conftest.py _scale_for)."""
    s = capture["pool_scores"]
    return float((s.grad * s).detach().abs().sum() / capture["pool_tau"].detach().abs())


def simple_pool(kind, x, batch, num_graphs):
    """pooling.py:15-80 (Mean / Max / Sum pooling via torch_scatter)."""
    idx = batch.unsqueeze(1).expand_as(x)
    s = torch.zeros(num_graphs, x.shape[1], dtype=x.dtype, device=x.device).scatter_add_(0, idx, x)
    if kind == "sum":
        return s
    if kind == "mean":
        cnt = torch.zeros(num_graphs, dtype=x.dtype, device=x.device).scatter_add_(0, batch, torch.ones(x.shape[0], dtype=x.dtype, device=x.device)).clamp(min=1)
        return s / cnt.unsqueeze(1)
    if kind == "max":
        m = torch.full((num_graphs, x.shape[1]), float("-inf"), dtype=x.dtype, device=x.device).scatter_reduce(0, idx, x, "amax", include_self=True)
        return torch.where(torch.isinf(m) & (m < 0), torch.zeros_like(m), m)
    raise ValueError(kind)


def linear_block(p, pre, x, activation, drop, use_skip, training):
    """layers.py:170-219 (LinearBlock.forward)."""
    out = linear(p, pre + "linear1", x)
    out = act(activation, out)
    out = dropout(out, drop, training)
    out = linear(p, pre + "linear2", out)
    return out + x if use_skip else out


def mlp(p, pre, x, cfg, training):
    """layers.py:222-267 (MultiLayerPerceptron), use_skip=True, in = hidden = out = ffn_hidden_dim."""
    n = cfg["ffn_num_layers"]
    d = cfg["ffn_hidden_dim"]
    for i in range(n):
        first_or_last = (n == 1) or i == 0 or i == n - 1
        use_skip = (not first_or_last) and True  # input_dim == output_dim == d
        x = linear_block(p, f"{pre}layers.{i}.", x, cfg["activation"], cfg["ffn_dropout"], use_skip, training)
    del d
    return x


def cis_trans(x, cis, trans):
    """gnn.py:452-497 (_cis_trans_calculation): rows 0 and 1 of the collated [M, 2] cis / trans
    tensors are the source and target atom lists (as the reference indexes them); cis sources are
    subtracted, trans sources added, by one scatter_add onto a copy of x."""
    if cis.numel() == 0 and trans.numel() == 0:
        return x
    tg, sv = [], []
    if cis.numel() > 0:
        tg.append(cis[1])
        sv.append(-x[cis[0]])
    if trans.numel() > 0:
        tg.append(trans[1])
        sv.append(x[trans[0]])
    t = torch.cat(tg)
    return x.scatter_add(0, t.unsqueeze(1).expand(-1, x.shape[1]), torch.cat(sv))


def tetrahedral(x, tet):
    """gnn.py:376-450 (_tetrahedral_feature_calculation_physics_inspired): for every chiral centre's
    4 neighbour rows e (unit-normalised, eps 1e-8), chi = e1^2 (e2 - e3) + e2^2 (e3 - e1) +
    e3^2 (e1 - e2) with e_k = roll(e, -k) over the 4 neighbours, scaled by tanh(mean |row| / 3),
    index_add_-ed onto a copy of x at the neighbour rows; rows named by no centre become 0."""
    if tet.numel() == 0:
        return x
    out = x.clone()
    raw = out[tet]
    mag = torch.norm(raw, dim=-1, keepdim=True)
    e = F.normalize(raw, dim=-1, eps=1e-8)
    sq = e ** 2
    r = lambda t, k: torch.roll(t, shifts=-k, dims=1)  # noqa: E731
    chi = r(sq, 1) * (r(e, 2) - r(e, 3)) + r(sq, 2) * (r(e, 3) - r(e, 1)) + r(sq, 3) * (r(e, 1) - r(e, 2))
    chi = chi * torch.tanh(torch.mean(mag, dim=1, keepdim=True) / 3.0)
    idx = tet.reshape(-1)
    out.index_add_(0, idx, chi.reshape(-1, out.shape[-1]))
    keep = torch.zeros(out.shape[0], dtype=torch.bool, device=out.device)
    keep[torch.unique(idx)] = True
    out[~keep] = 0.0
    return out


def stereo(p, x, tet, cis, trans):
    """gnn.py:310-326 (_apply_stereochemistry): Linear(3D -> D) of [x | cis_trans(x) | tetrahedral(x)]."""
    return linear(p, "stereochemical_embedding_2", torch.cat([x, cis_trans(x, cis, trans), tetrahedral(x, tet)], -1))


def default_config(**kw):
    """GNN.__init__ defaults (gnn.py:50-70)."""
    cfg = dict(hidden_dim=512, output_dim=1, num_shells=3, num_message_passing_layers=3,
               ffn_hidden_dim=None, ffn_num_layers=3, pooling_type="attention", embedding_dim=64,
               use_partial_charges=False, ffn_dropout=0.05, activation="silu",
               shell_conv_num_mlp_layers=2, shell_conv_dropout=0.05, attention_num_heads=4,
               attention_temperature=1.0, loss_function="l1", use_stereochemistry=False)
    cfg.update(kw)
    if cfg["ffn_hidden_dim"] is None:
        cfg["ffn_hidden_dim"] = cfg["hidden_dim"]
    cfg["x_other_dim"] = int(0.3 * cfg["hidden_dim"])
    return cfg


def gnn_forward(p, cfg, atom_features, edges, batch, total_charges, training=False, capture=None, tet=None, cis=None,
                trans=None):
    """gnn.py:197-260 (GNN.forward); stereochemistry (gnn.py:297-300) when cfg['use_stereochemistry'],
    from the collated tetrahedral [M, 4] / cis [C, 2] / trans [T, 2] tensors.

    Returns (output [G, T or 4T], attention [H, N] or None, partial_charges [N] or None).
    `capture` (dict) receives intermediate tensors: 'x_other_in', 'layer{l}', 'chunks0', 'pre_pool'.
    """
    emb = torch.cat([
        F.embedding(atom_features["atom_type"], p["atom_type_embedding.weight"]),
        F.embedding(atom_features["hydrogen_count"], p["hydrogen_count_embedding.weight"]),
        F.embedding(atom_features["degree"], p["degree_embedding.weight"]),
        F.embedding(atom_features["hybridization"], p["hybridization_embedding.weight"]),
    ], dim=-1)  # gnn.py:262-274
    h = act(cfg["activation"], linear(p, "embedding_projection", emb))  # gnn.py:224-225
    d = cfg["x_other_dim"]
    x_self, x_other = torch.split(h, [cfg["hidden_dim"] - d, d], dim=-1)  # gnn.py:227-231
    if capture is not None:
        capture["x_other_in"] = x_other
    if edges.numel() > 0:  # gnn.py:287
        for l in range(cfg["num_message_passing_layers"]):
            if cfg["use_partial_charges"]:
                x_other = partial_charges(x_other, batch, total_charges)
            if cfg.get("use_stereochemistry"):
                e0 = torch.empty(0, 2, dtype=torch.long)
                x_other = stereo(p, x_other, tet if tet is not None else torch.empty(0, 4, dtype=torch.long),
                                 cis if cis is not None else e0, trans if trans is not None else e0)
            if capture is not None and l == 0:
                capture["chunks0"] = message_passing(x_other, edges[:, 0], edges[:, 1], cfg["num_shells"])
            x_other = shell_layer(p, f"message_passing_layers.{l}.", x_other, edges[:, 0], edges[:, 1],
                                  cfg, training) + x_other
            if capture is not None:
                capture[f"layer{l}"] = x_other
    q = x_other[:, 0].clone() if (cfg["use_partial_charges"] and x_other.shape[-1] >= 2) else None
    x = linear(p, "concat_self_other", torch.cat([x_self, x_other], dim=-1))  # gnn.py:245-246
    if capture is not None:
        capture["pre_pool"] = x
    g = total_charges.shape[0]
    if cfg["pooling_type"] == "attention":
        pooled, attn = attention_pool(p, "pooling.", x, batch, cfg["attention_num_heads"], g, capture=capture)
    else:
        pooled, attn = simple_pool(cfg["pooling_type"], x, batch, g), None
    x = linear(p, "post_pooling_projection", pooled)
    x = mlp(p, "ffn.", x, cfg, training)
    skip = linear(p, "skip_transform", x)
    out = linear(p, "output_layer", torch.cat([x, skip], dim=-1))
    return out, attn, q


def param_shapes(cfg, feature_sizes=None):
    """Parameter names and shapes in the reference's registration order (state_dict order)."""
    fs = feature_sizes or {"atom_type": 119, "hydrogen_count": 9, "degree": 7, "hybridization": 7}
    e, hd, d = cfg["embedding_dim"], cfg["hidden_dim"], cfg["x_other_dim"]
    fh = cfg["ffn_hidden_dim"]
    s = []
    for k in ("atom_type", "hydrogen_count", "degree", "hybridization"):
        s.append((f"{k}_embedding.weight", (fs[k], e)))
    s += [("embedding_projection.weight", (hd, 4 * e)), ("embedding_projection.bias", (hd,))]
    k_in = d * (cfg["num_shells"] + 1)
    for l in range(cfg["num_message_passing_layers"]):
        pre = f"message_passing_layers.{l}."
        s += [(pre + "input_proj.weight", (d, k_in)), (pre + "input_proj.bias", (d,))]
        for b in range(cfg["shell_conv_num_mlp_layers"]):
            for nm in ("linear_1", "linear_2"):
                s += [(f"{pre}mlp_blocks.{b}.{nm}.weight", (d, d)), (f"{pre}mlp_blocks.{b}.{nm}.bias", (d,))]
        s += [(pre + "global_skip_proj.weight", (d, k_in)), (pre + "global_skip_proj.bias", (d,))]
    if cfg["pooling_type"] == "attention":
        s.append(("pooling.temperature", ()))
        for i in range(cfg["attention_num_heads"]):
            s += [(f"pooling.attention_weights.{i}.weight", (1, hd)), (f"pooling.attention_weights.{i}.bias", (1,))]
    s += [("concat_self_other.weight", (hd, hd)), ("concat_self_other.bias", (hd,))]
    if cfg.get("use_stereochemistry"):  # gnn.py:192-195
        s += [("stereochemical_embedding.weight", (hd, 3 * hd)), ("stereochemical_embedding.bias", (hd,)),
              ("stereochemical_embedding_2.weight", (d, 3 * d)), ("stereochemical_embedding_2.bias", (d,))]
    s += [("post_pooling_projection.weight", (fh, hd)), ("post_pooling_projection.bias", (fh,))]
    for i in range(cfg["ffn_num_layers"]):
        for nm in ("linear1", "linear2"):
            s += [(f"ffn.layers.{i}.{nm}.weight", (fh, fh)), (f"ffn.layers.{i}.{nm}.bias", (fh,))]
    t = cfg["output_dim"] * (4 if cfg["loss_function"] == "evidential" else 1)
    s += [("skip_transform.weight", (fh, fh)), ("skip_transform.bias", (fh,))]
    s += [("output_layer.weight", (t, 2 * fh)), ("output_layer.bias", (t,))]
    s += [("long_range_projection.weight", (fh, hd)), ("long_range_projection.bias", (fh,))]
    return s


def seeded_params(cfg, seed, dtype=torch.float32):
    """Deterministic weights by (seed, key): every framework under test loads these same values.

    Distributions follow the reference's own initialisation so activations have realistic scale:
    GNN.init_weights (gnn.py:660-703) = xavier_uniform on embeddings, the top-level Linear layers and
    the attention heads; nn.Linear default U(+-1/sqrt(fan_in)) on the message-passing and FFN layers.
    Biases that the reference zeroes get a small non-zero value (0.01*N(0,1)) so the bias paths are
    exercised; temperature = 1 + 0.25*u. Streams are independent per key:
    default_rng([seed, crc32(key)]).
    """
    import zlib

    import numpy as np

    top = ("embedding_projection.", "concat_self_other.", "post_pooling_projection.", "skip_transform.",
           "output_layer.", "long_range_projection.", "pooling.attention_weights.", "stereochemical_embedding")
    out = {}
    for name, shape in param_shapes(cfg):
        rng = np.random.default_rng([seed, zlib.crc32(name.encode())])
        xavier = name.startswith(top) or (name.endswith("_embedding.weight"))
        if name.endswith("temperature"):
            v = np.array(1.0 + 0.25 * rng.random(), dtype=np.float64)
        elif name.endswith("weight") and xavier:
            a = math.sqrt(6.0 / (shape[0] + shape[1]))
            v = rng.uniform(-a, a, shape)
        elif name.endswith("bias") and xavier:
            v = rng.standard_normal(shape) * 0.01
        else:
            fan_in = shape[1] if len(shape) == 2 else param_fan_in(cfg, name)
            a = 1.0 / math.sqrt(fan_in)
            v = rng.uniform(-a, a, shape)
        out[name] = torch.tensor(np.asarray(v), dtype=dtype).reshape(shape)
    return out


def param_fan_in(cfg, bias_name):
    """fan_in of the Linear a bias belongs to (nn.Linear.reset_parameters bias bound)."""
    d = cfg["x_other_dim"]
    if "input_proj" in bias_name or "global_skip_proj" in bias_name:
        return d * (cfg["num_shells"] + 1)
    if "mlp_blocks" in bias_name:
        return d
    return cfg["ffn_hidden_dim"]
