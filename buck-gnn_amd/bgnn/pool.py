"""SAGPooling's node selection and graph coarsening on libbgnn (no CPU fallback).

torch_geometric.nn.SAGPooling, as the reference builds it for GraphSAGE_SAG / EAGNN_SAG
(Models/BuckGNN.py:203-208,231-236; called at :364,502), does [PyG-doc]

    perm   = topk(score, ratio, batch)          # per graph ceil(ratio * n_g) best, descending
    x'     = x[perm] * score[perm]
    edges' = filter_adj(edge_index, perm)        # both ends kept, edge_index order, relabelled
    batch' = batch[perm]

* `topk_select` — bgnn_topk_rank (each node's position in its graph's stable descending
  order) + bgnn_topk_select (scatter of the kept nodes to their output positions, new node
  ids, pooled batch vector). One host sync for the kept-node count (PyG's boolean-mask
  indexing syncs there too).
* `gather_scale` — bgnn_gather_scale / _bwd as an autograd Function (gradients to x and
  to the score, which is how the scoring GNN trains).
* `filter_edges` — bgnn_filter_edges (deterministic stream compaction); one host sync for
  the kept-edge count.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch

from . import _lib
from .graph import _stream, require_cuda


def _graph_offsets(batch: torch.Tensor) -> Tuple[torch.Tensor, int]:
    """ptr [B+1] of a non-decreasing `batch` vector and B (one host sync, which also checks
    the order: every PyG Batch has its graphs' nodes contiguous and in graph order)."""
    last, unsorted, first = torch.stack([batch[-1], (batch[1:] < batch[:-1]).any().to(batch.dtype),
                                         batch[0]]).tolist()
    if unsorted:
        raise ValueError("SAGPooling: `batch` must be non-decreasing (graphs contiguous, in order)")
    if first < 0:
        raise ValueError("SAGPooling: negative graph id in `batch`")
    B = int(last) + 1
    ptr = torch.searchsorted(batch, torch.arange(B + 1, dtype=batch.dtype, device=batch.device))
    return ptr, B


def topk_select(score: torch.Tensor, ratio: float, batch: torch.Tensor):
    """(perm [K] int64, new_id [N] int32 (-1 = dropped), batch' [K] int64): PyG's topk with
    ties broken towards the lower node index (a stable descending sort)."""
    require_cuda(score, batch, what="topk_select")
    score = score.detach().reshape(-1).contiguous()
    if score.dtype != torch.float32:
        raise TypeError("topk_select: score must be float32")
    # the kernels read `batch` as int64 (an int32 edge_index gives an int32 batch upstream)
    batch = batch.to(torch.long).contiguous()
    N = score.numel()
    dev = score.device
    if batch.numel() != N:
        raise ValueError(f"topk_select: batch has {batch.numel()} entries, score {N}")
    if N == 0:
        e = torch.empty(0, dtype=torch.long, device=dev)
        return e, torch.empty(0, dtype=torch.int32, device=dev), e
    ptr, B = _graph_offsets(batch)
    counts = ptr[1:] - ptr[:-1]
    if ratio >= 1:
        k = counts.new_full((B,), int(ratio)).minimum(counts)
    else:   # PyG: (float(ratio) * num_nodes.to(score.dtype)).ceil()
        k = (float(ratio) * counts.to(score.dtype)).ceil().to(torch.long)
    new_ptr = torch.zeros(B + 1, dtype=torch.long, device=dev)
    torch.cumsum(k, 0, out=new_ptr[1:])
    K = int(new_ptr[-1].item())
    rank = torch.empty(N, dtype=torch.int32, device=dev)
    perm = torch.empty(K, dtype=torch.long, device=dev)
    new_id = torch.empty(N, dtype=torch.int32, device=dev)
    batch_out = torch.empty(K, dtype=torch.long, device=dev)
    s = _stream()
    _lib.call("bgnn_topk_rank", score.data_ptr(), batch.data_ptr(), ptr.data_ptr(), N, rank.data_ptr(), s)
    _lib.call("bgnn_topk_select", rank.data_ptr(), batch.data_ptr(), k.data_ptr(), new_ptr.data_ptr(), N,
              perm.data_ptr(), new_id.data_ptr(), batch_out.data_ptr(), s)
    return perm, new_id, batch_out


class _GatherScale(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, score, perm, new_id):
        N, H = x.shape
        K = perm.numel()
        out = torch.empty(K, H, dtype=x.dtype, device=x.device)
        _lib.call("bgnn_gather_scale", x.data_ptr(), x.stride(0), H, perm.data_ptr(), score.data_ptr(), K,
                  out.data_ptr(), out.stride(0), _stream())
        ctx.save_for_backward(x, score, new_id)
        return out

    @staticmethod
    def backward(ctx, g):
        x, score, new_id = ctx.saved_tensors
        g = g.contiguous()
        N, H = x.shape
        dx = torch.empty_like(x)
        ds = torch.empty_like(score) if ctx.needs_input_grad[1] else None
        _lib.call("bgnn_gather_scale_bwd", g.data_ptr(), g.stride(0), x.data_ptr(), x.stride(0), H,
                  new_id.data_ptr(), score.data_ptr(), N, dx.data_ptr(), dx.stride(0),
                  None if ds is None else ds.data_ptr(), _stream())
        return dx, ds, None, None


def gather_scale(x: torch.Tensor, score: torch.Tensor, perm: torch.Tensor, new_id: torch.Tensor) -> torch.Tensor:
    """x[perm] * score[perm].view(-1, 1) (Models/BuckGNN.py:364,502 via SAGPooling), differentiable
    in x and score."""
    require_cuda(x, score, perm, new_id, what="gather_scale")
    if x.dtype != torch.float32 or x.dim() != 2:
        raise TypeError("gather_scale: x must be a float32 [N, H] tensor")
    x = x.contiguous()
    score = score.reshape(-1).contiguous()
    if score.numel() != x.size(0) or new_id.numel() != x.size(0):
        raise ValueError("gather_scale: score / new_id must have one entry per row of x")
    if new_id.dtype != torch.int32 or perm.dtype != torch.long:
        raise TypeError("gather_scale: new_id must be int32 and perm int64 (topk_select's outputs)")
    if score.dtype != torch.float32:
        raise TypeError("gather_scale: score must be float32")
    return _GatherScale.apply(x, score, perm.contiguous(), new_id.contiguous())


def filter_edges(edge_index: torch.Tensor, new_id: torch.Tensor, num_nodes: int):
    """(edge_index' [2, E'] int64, kept [E'] int64): PyG's filter_adj on device; `kept` holds
    the original positions of the kept edges (edge_attr' = edge_attr[kept])."""
    require_cuda(edge_index, new_id, what="filter_edges")
    if edge_index.dim() != 2 or edge_index.size(0) != 2:
        raise ValueError(f"filter_edges: edge_index must be [2, E], got {tuple(edge_index.shape)}")
    if new_id.dtype != torch.int32 or new_id.numel() != int(num_nodes):
        raise TypeError("filter_edges: new_id must be an int32 vector with one entry per node")
    new_id = new_id.contiguous()
    ei = edge_index.to(torch.long).contiguous()
    E = ei.size(1)
    dev = ei.device
    out = torch.empty(2 * E, dtype=torch.long, device=dev)
    kept = torch.empty(E, dtype=torch.long, device=dev)
    n = torch.empty(1, dtype=torch.long, device=dev)
    ws_bytes = _lib.query("bgnn_filter_edges_ws_bytes", E)
    ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=dev)
    _lib.call("bgnn_filter_edges", ei.data_ptr(), E, new_id.data_ptr(), int(num_nodes), out.data_ptr(),
              kept.data_ptr(), n.data_ptr(), ws.data_ptr(), ws_bytes, _stream())
    M = int(n.item())
    return out[:2 * M].view(2, M), kept[:M]


def sag_pool(x: torch.Tensor, score: torch.Tensor, ratio: float, edge_index: torch.Tensor,
             edge_attr: Optional[torch.Tensor], batch: torch.Tensor, multiplier: float = 1.0):
    """The selection + coarsening half of SAGPooling.forward given the node scores:
    returns (x', edge_index', edge_attr', batch', perm, score[perm])."""
    perm, new_id, batch_out = topk_select(score, ratio, batch)
    xo = gather_scale(x, score, perm, new_id)
    if multiplier != 1:
        xo = multiplier * xo
    ei, kept = filter_edges(edge_index, new_id, x.size(0))
    ea = edge_attr.index_select(0, kept) if edge_attr is not None else None
    return xo, ei, ea, batch_out, perm, score.reshape(-1)[perm]
