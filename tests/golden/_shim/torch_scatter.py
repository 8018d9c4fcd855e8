"""Stand-in for torch_scatter 2.1.2 (requirements.txt:6 of the reference), used ONLY by
tests/golden/make_golden.py to import the reference model in the development container.

torch_scatter is not installed here and there is no network. The functions below restate the
published 2.1.2 semantics (torch_scatter/scatter.py, composite/softmax.py):
  scatter_sum/add: zeros(size).scatter_add_(dim, broadcast(index), src), dim_size=None -> index.max()+1
  scatter_mean:   sum / count.clamp(min=1) (integer-division for int dtypes not needed here)
  scatter_max:    per-segment max, empty segments filled with 0, argmax = src.size(dim) for empty
  scatter_softmax: exp(src - max[index]) / sum(exp)[index]
This is "parity unpinned" at the torch_scatter boundary (no offline tests exist for it).
"""
import torch


def _broadcast(src, other, dim):
    if dim < 0:
        dim = other.dim() + dim
    if src.dim() == 1:
        for _ in range(0, dim):
            src = src.unsqueeze(0)
    for _ in range(src.dim(), other.dim()):
        src = src.unsqueeze(-1)
    src = src.expand(other.size())
    return src


def scatter_sum(src, index, dim=-1, out=None, dim_size=None):
    index = _broadcast(index, src, dim)
    if out is None:
        size = list(src.size())
        if dim_size is not None:
            size[dim] = dim_size
        elif index.numel() == 0:
            size[dim] = 0
        else:
            size[dim] = int(index.max()) + 1
        out = torch.zeros(size, dtype=src.dtype, device=src.device)
        return out.scatter_add_(dim, index, src)
    return out.scatter_add_(dim, index, src)


def scatter_add(src, index, dim=-1, out=None, dim_size=None):
    return scatter_sum(src, index, dim, out, dim_size)


def scatter_mean(src, index, dim=-1, out=None, dim_size=None):
    out = scatter_sum(src, index, dim, out, dim_size)
    dim_size = out.size(dim)
    index_dim = dim
    if index_dim < 0:
        index_dim = index_dim + src.dim()
    if index.dim() <= index_dim:
        index_dim = index.dim() - 1
    ones = torch.ones(index.size(), dtype=src.dtype, device=src.device)
    count = scatter_sum(ones, index, index_dim, None, dim_size)
    count[count < 1] = 1
    count = _broadcast(count, out, dim)
    if out.is_floating_point():
        out.true_divide_(count)
    else:
        out.div_(count, rounding_mode="floor")
    return out


def scatter_max(src, index, dim=-1, out=None, dim_size=None):
    if dim < 0:
        dim = src.dim() + dim
    index_b = _broadcast(index, src, dim)
    size = list(src.size())
    if dim_size is not None:
        size[dim] = dim_size
    elif index_b.numel() == 0:
        size[dim] = 0
    else:
        size[dim] = int(index_b.max()) + 1
    res = torch.full(size, float("-inf"), dtype=src.dtype, device=src.device)
    res = res.scatter_reduce(dim, index_b, src, reduce="amax", include_self=True)
    empty = torch.isinf(res) & (res < 0)
    res = res.masked_fill(empty, 0.0)
    # argmax: first position attaining the max (CPU kernel iterates in order)
    arg = torch.full(size, src.size(dim), dtype=torch.long, device=src.device)
    pos = torch.arange(src.size(dim), device=src.device)
    shape = [1] * src.dim()
    shape[dim] = -1
    pos = pos.view(shape).expand_as(src)
    hit = src == res.gather(dim, index_b)
    cand = torch.where(hit, pos, torch.full_like(pos, src.size(dim)))
    arg = arg.scatter_reduce(dim, index_b, cand, reduce="amin", include_self=True)
    return res, arg


def scatter_softmax(src, index, dim=-1, dim_size=None):
    if not torch.is_floating_point(src):
        raise ValueError("`scatter_softmax` can only be computed over tensors with floating point data types.")
    index = _broadcast(index, src, dim)
    max_value_per_index = scatter_max(src, index, dim=dim, dim_size=dim_size)[0]
    max_per_src_element = max_value_per_index.gather(dim, index)
    recentered_scores = src - max_per_src_element
    recentered_scores_exp = recentered_scores.exp_()
    sum_per_index = scatter_sum(recentered_scores_exp, index, dim, dim_size=dim_size)
    normalizing_constants = sum_per_index.gather(dim, index)
    return recentered_scores_exp.div(normalizing_constants)
