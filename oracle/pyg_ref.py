"""ORACLE (test infrastructure only): CPU restatement of the PyG / torch_scatter ops
buck-gnn calls (Models/BuckGNN.py:3-6; Utils/Losses.py:4).

Everything is the textbook gather -> scatter formulation PyG's MessagePassing
uses on the CPU: messages x_j = x.index_select(0, edge_index[0]) and an
index_add_ / scatter_reduce_ into edge_index[1]. No fused or reordered math.
"""
from __future__ import annotations

import math
from typing import List, Optional, Sequence

import torch
import torch.nn.functional as F
from torch import Tensor, nn


# ----------------------------------------------------------------------------- scatter
class _ScatterMaxFirst(torch.autograd.Function):
    """Segment max along dim 0 whose gradient goes to the FIRST position (in src order) that
    attains the maximum of its (segment, column): torch_scatter's scatter_max convention
    (its CPU kernel keeps the first strict '>' winner as `arg`; the backward scatters the whole
    output gradient to `arg`). Empty segments give 0 and pass no gradient.

    Tie convention (SURVEY §7 "Max aggregation tie-breaking"): PyG's `utils.scatter(reduce='max')`
    calls torch_scatter when it is installed and the input is a CUDA tensor that requires grad
    (one winner per tie; on CUDA the winner among ties is unspecified), and
    `Tensor.scatter_reduce_('amax')` otherwise (the gradient split evenly over the ties). The
    reference imports torch_scatter (Models/BuckGNN.py:6) and trained on CUDA, so the one-winner
    form is the reference's; the first occurrence is its deterministic instance, the one
    bgnn's kernels implement (csrc/spmm.hip: strict '>' in CSR = edge_index order)."""

    @staticmethod
    def forward(ctx, src, index, dim_size):
        idx = index.view(-1, *([1] * (src.dim() - 1))).expand_as(src)
        out = src.new_zeros((dim_size,) + tuple(src.shape[1:])).scatter_reduce_(0, idx, src, reduce="amax",
                                                                                 include_self=False)
        n = src.size(0)
        pos = torch.arange(n, device=src.device).view(-1, *([1] * (src.dim() - 1))).expand_as(src)
        hit = src == out.index_select(0, index)
        first = torch.full(out.shape, n, dtype=torch.long, device=src.device)
        first.scatter_reduce_(0, idx, torch.where(hit, pos, torch.full_like(pos, n)), reduce="amin",
                              include_self=True)
        ctx.save_for_backward(first)
        ctx.n = n
        return out

    @staticmethod
    def backward(ctx, g):
        (first,) = ctx.saved_tensors
        n = ctx.n
        valid = first < n
        gs = g.new_zeros((n + 1,) + tuple(g.shape[1:]))   # row n absorbs the empty segments
        gs.scatter_(0, torch.where(valid, first, torch.full_like(first, n)), torch.where(valid, g, torch.zeros_like(g)))
        return gs[:n], None, None


def scatter(src: Tensor, index: Tensor, dim_size: int, reduce: str) -> Tensor:
    """Segment reduce along dim 0 (torch_scatter / PyG utils.scatter semantics):
    sum, mean (sum / max(count, 1)), max (empty segments -> 0; gradient to the first maximum,
    _ScatterMaxFirst)."""
    out_shape = (dim_size,) + tuple(src.shape[1:])
    if reduce in ("sum", "add"):
        return src.new_zeros(out_shape).index_add_(0, index, src)
    if reduce == "mean":
        s = src.new_zeros(out_shape).index_add_(0, index, src)
        cnt = torch.zeros(dim_size, dtype=src.dtype, device=src.device).index_add_(
            0, index, torch.ones(index.numel(), dtype=src.dtype, device=src.device))
        return s / cnt.clamp_min(1).view(-1, *([1] * (src.dim() - 1)))
    if reduce == "max":
        return _ScatterMaxFirst.apply(src, index, dim_size)
    raise ValueError(reduce)


def scatter_add(src, index, dim=0, out=None, dim_size=None):
    n = dim_size if dim_size is not None else (int(index.max()) + 1 if index.numel() else 0)
    return scatter(src, index, n, "sum")


def scatter_mean(src, index, dim=0, out=None, dim_size=None):
    n = dim_size if dim_size is not None else (int(index.max()) + 1 if index.numel() else 0)
    return scatter(src, index, n, "mean")


# ----------------------------------------------------------------------------- pooling
def _pool(x: Tensor, batch: Optional[Tensor], size: Optional[int], reduce: str) -> Tensor:
    if batch is None:
        kd = x.dim() == 2
        if reduce == "mean":
            return x.mean(dim=-2, keepdim=kd)
        if reduce == "sum":
            return x.sum(dim=-2, keepdim=kd)
        return x.max(dim=-2, keepdim=kd)[0]
    n = size if size is not None else (int(batch.max()) + 1 if batch.numel() else 0)
    return scatter(x, batch, n, reduce)


def global_mean_pool(x, batch, size=None):
    return _pool(x, batch, size, "mean")


def global_add_pool(x, batch, size=None):
    return _pool(x, batch, size, "sum")


def global_max_pool(x, batch, size=None):
    return _pool(x, batch, size, "max")


# ----------------------------------------------------------------------------- SAGEConv
class Linear(nn.Linear):
    def reset_parameters(self):
        bound = math.sqrt(6.0 / (6.0 * self.in_features)) if self.in_features else 0.0
        with torch.no_grad():
            self.weight.uniform_(-bound, bound)
            if self.bias is not None:
                b = 1.0 / math.sqrt(self.in_features) if self.in_features else 0.0
                self.bias.uniform_(-b, b)


def sage_aggregate(x: Tensor, edge_index: Tensor, aggr: str) -> Tensor:
    """AGG_{j: (j -> i)} x_j with j = edge_index[0], i = edge_index[1]."""
    msg = x.index_select(0, edge_index[0])
    return scatter(msg, edge_index[1], x.size(0), "sum" if aggr == "add" else aggr)


class SAGEConv(nn.Module):
    def __init__(self, in_channels, out_channels, aggr="mean", normalize=False, root_weight=True,
                 project=False, bias=True, **kw):
        super().__init__()
        self.in_channels, self.out_channels = in_channels, out_channels
        self.aggr, self.normalize, self.root_weight, self.project = aggr, normalize, root_weight, project
        if project:
            self.lin = Linear(in_channels, in_channels, bias=True)
        self.lin_l = Linear(in_channels, out_channels, bias=bias)
        if root_weight:
            self.lin_r = Linear(in_channels, out_channels, bias=False)

    def forward(self, x, edge_index, size=None):
        x_src = x
        if self.project:
            x_src = F.relu(self.lin(x_src))
        out = self.lin_l(sage_aggregate(x_src, edge_index, self.aggr))
        if self.root_weight:
            out = out + self.lin_r(x)
        if self.normalize:
            out = F.normalize(out, p=2.0, dim=-1)
        return out


# ----------------------------------------------------------------------------- SAGPooling
def topk(score: Tensor, ratio: float, batch: Tensor) -> Tensor:
    """PyG's topk (torch_geometric.nn.pool.select.topk, ratio < 1 form) [PyG-doc]: per graph
    the k_g = ceil(ratio * n_g) highest scores (k_g computed in the score dtype), graphs in
    order, scores descending. PyG's first sort is unstable, so its tie order is unspecified;
    here both sorts are stable (ties: lower node index first)."""
    n_graphs = int(batch.max()) + 1 if batch.numel() else 0
    num_nodes = torch.zeros(n_graphs, dtype=torch.long).index_add_(0, batch, torch.ones_like(batch))
    k = (float(ratio) * num_nodes.to(score.dtype)).ceil().to(torch.long)
    _, x_perm = torch.sort(score.view(-1), descending=True, stable=True)
    b = batch[x_perm]
    b, b_perm = torch.sort(b, descending=False, stable=True)
    ptr = torch.cat([num_nodes.new_zeros(1), num_nodes.cumsum(0)[:-1]])
    mask = (torch.arange(score.numel()) - ptr[b]) < k[b]
    return x_perm[b_perm[mask]]


def filter_adj(edge_index: Tensor, edge_attr: Optional[Tensor], perm: Tensor, num_nodes: int):
    """PyG's filter_adj [PyG-doc]: keep the edges whose two ends are in perm, in edge_index
    order, relabelled to positions in perm."""
    mask = perm.new_full((num_nodes,), -1)
    mask[perm] = torch.arange(perm.numel(), dtype=torch.long)
    row, col = mask[edge_index[0]], mask[edge_index[1]]
    keep = (row >= 0) & (col >= 0)
    return torch.stack([row[keep], col[keep]], 0), (edge_attr[keep] if edge_attr is not None else None)


class _SelectTopK(nn.Module):
    """The scoring projection of PyG's SelectTopK(in_channels=1): weight [1, 1],
    score = act((attn * w).sum(-1) / ||w||), i.e. act(sign(w) * attn)."""

    def __init__(self):
        super().__init__()
        self.weight = nn.Parameter(torch.empty(1, 1))
        with torch.no_grad():
            self.weight.uniform_(-1.0, 1.0)   # PyG: uniform(in_channels=1, weight)


class SAGPooling(nn.Module):
    """torch_geometric.nn.SAGPooling restated [PyG-doc] for the form the reference builds
    (Models/BuckGNN.py:203-208,231-236: GNN=SAGEConv, aggr='add', ratio=0.5, min_score=None):
    attn = GNN(x, edge_index) [N, 1]; score = tanh(sign(w) attn) (select.weight w);
    perm = topk(score, ratio, batch); x' = x[perm] * score[perm] (* multiplier);
    edge_index', edge_attr' = filter_adj(...); batch' = batch[perm].
    Returns (x', edge_index', edge_attr', batch', perm, score[perm])."""

    def __init__(self, in_channels, ratio=0.5, GNN=None, min_score=None, multiplier=1.0, nonlinearity="tanh",
                 **kwargs):
        super().__init__()
        if GNN is None:
            raise NotImplementedError("SAGPooling: only an explicit GNN (the reference passes SAGEConv)")
        if min_score is not None:
            raise NotImplementedError("SAGPooling: min_score (softmax selection) is not restated")
        self.in_channels, self.ratio, self.multiplier = in_channels, ratio, multiplier
        self.nonlinearity = torch.tanh if nonlinearity == "tanh" else nonlinearity
        self.gnn = GNN(in_channels, 1, **kwargs)
        self.select = _SelectTopK()

    def forward(self, x, edge_index, edge_attr=None, batch=None, attn=None):
        if batch is None:
            batch = edge_index.new_zeros(x.size(0))
        attn = x if attn is None else attn
        attn = attn.view(-1, 1) if attn.dim() == 1 else attn
        attn = self.gnn(attn, edge_index)
        w = self.select.weight
        score = self.nonlinearity((attn * w).sum(dim=-1) / w.norm(p=2, dim=-1))
        perm = topk(score, self.ratio, batch)
        s = score[perm]
        x = x[perm] * s.view(-1, 1)
        x = self.multiplier * x if self.multiplier != 1 else x
        edge_index, edge_attr = filter_adj(edge_index, edge_attr, perm, score.numel())
        return x, edge_index, edge_attr, batch[perm], perm, s


# ----------------------------------------------------------------------------- batching
class Data:
    def __init__(self, **kw):
        self.__dict__.update(kw)


def collate(graphs: Sequence[dict]) -> dict:
    """PyG Batch.from_data_list restated: x/edge_attr/y concatenated, edge_index offset
    by the running node count, batch = graph id per node."""
    xs, eis, eas, ys, bs = [], [], [], [], []
    off = 0
    for g, d in enumerate(graphs):
        n = d["x"].shape[0]
        xs.append(torch.as_tensor(d["x"]))
        eis.append(torch.as_tensor(d["edge_index"]) + off)
        if d.get("edge_attr") is not None:
            eas.append(torch.as_tensor(d["edge_attr"]))
        ys.append(torch.as_tensor(d["y"]).reshape(-1))
        bs.append(torch.full((n,), g, dtype=torch.long))
        off += n
    return {"x": torch.cat(xs), "edge_index": torch.cat(eis, 1),
            "edge_attr": torch.cat(eas) if eas else None, "y": torch.cat(ys), "batch": torch.cat(bs)}
