"""Autograd-wrapped segment reductions on libbgnn (no CPU fallback).

* `aggregate(x, graph, reduce)` — SAGEConv's neighbour aggregation
  (PyG semantics: sum over in-edges of target = edge_index[1]; 'add' == 'sum';
  mean divides by the in-degree; max takes the element-wise maximum; empty
  rows are 0 for all three). Used at Models/BuckGNN.py:342,393,434,449,463.
* `segment_reduce(src, segments, reduce)` — global_mean_pool
  (Models/BuckGNN.py:274) and torch_scatter.scatter_add / scatter_mean
  (Models/BuckGNN.py:561,605).
"""
from __future__ import annotations

import torch

from . import _lib
from .graph import Graph, SegmentIndex, _stream, require_cuda

REDUCE = {"sum": 0, "add": 0, "mean": 1, "max": 2}


def _check_x(x: torch.Tensor, what: str) -> torch.Tensor:
    require_cuda(x, what=what)
    if x.dtype != torch.float32:
        raise TypeError(f"{what}: only float32 features are supported (got {x.dtype})")
    if x.dim() != 2:
        raise ValueError(f"{what}: expected a 2-D [rows, channels] tensor, got {tuple(x.shape)}")
    return x.contiguous()


def _partial(csr, H: int, reduce: int, dev) -> torch.Tensor:
    n = csr.plan.n_chunks
    if n == 0:
        return None
    # MAX keeps an int32 arg plane after the float plane
    return torch.empty(n * H * (2 if reduce == 2 else 1), dtype=torch.float32, device=dev)


def spmm_fwd(csr, x: torch.Tensor, reduce: int, out_rows: int, want_arg: bool = False):
    """AGG over the CSR rows; for MAX with want_arg also the argmax state (a uint8 buffer of
    bgnn_spmm_max_arg_bytes: per-row edge offsets, int32 for heavy rows; max_arg_positions decodes)."""
    H = x.size(1)
    out = torch.empty(out_rows, H, dtype=torch.float32, device=x.device)
    arg = None
    if reduce == 2 and want_arg:
        arg = torch.empty(_lib.query("bgnn_spmm_max_arg_bytes", out_rows, H, csr.plan.n_heavy), dtype=torch.uint8,
                          device=x.device)
    part = _partial(csr, H, reduce, x.device)
    if out_rows > 0 and H > 0:
        _lib.call("bgnn_spmm_fwd", csr.ref(), x.data_ptr(), x.stride(0), H, reduce, out.data_ptr(), out.stride(0),
                  None if arg is None else arg.data_ptr(), None if part is None else part.data_ptr(), _stream())
    return out, arg


def spmm_bwd(csr_t, perm_t, fwd_rowptr, g: torch.Tensor, reduce: int, arg, out_rows: int, amax=None):
    """Transpose aggregation (rows = sources); MAX routes each (target, column) gradient to the
    argmax edge recorded in `arg` (the forward's state; the forward had g.size(0) rows)."""
    g = g.contiguous()
    H = g.size(1)
    gx = torch.empty(out_rows, H, dtype=torch.float32, device=g.device)
    part = _partial(csr_t, H, 0, g.device)
    if out_rows > 0 and H > 0:
        if reduce == 2:
            _lib.call("bgnn_spmm_bwd_max", csr_t.ref(), perm_t.data_ptr(), fwd_rowptr.data_ptr(), g.size(0),
                      g.data_ptr(), g.stride(0), H, arg.data_ptr(), None, 0, gx.data_ptr(), gx.stride(0),
                      None if part is None else part.data_ptr(), None if amax is None else amax.data_ptr(), _stream())
        else:
            _lib.call("bgnn_spmm_bwd", csr_t.ref(), None if perm_t is None else perm_t.data_ptr(),
                      None if fwd_rowptr is None else fwd_rowptr.data_ptr(), g.data_ptr(), g.stride(0), H, reduce,
                      gx.data_ptr(), gx.stride(0), None if part is None else part.data_ptr(),
                      None if amax is None else amax.data_ptr(), 0, _stream())
    return gx


def max_arg_positions(csr, arg: torch.Tensor, rows: int, H: int) -> torch.Tensor:
    """Decode spmm_fwd's MAX argmax state into int64 CSR positions [rows, H] (-1 for empty rows):
    test / inspection helper (torch ops on the device)."""
    from .graph import Plan  # noqa: F401  (documentation: heavy rows come from csr.plan)
    n = rows * H
    hoff = (n + 255) // 256 * 256
    aoff = hoff + (rows * 4 + 255) // 256 * 256
    a8 = arg[:n].view(rows, H).long()
    rp = csr.rowptr.long()
    deg = rp[1:] - rp[:-1]
    pos = rp[:-1].view(-1, 1) + a8
    nh = csr.plan.n_heavy
    if nh > 0:
        heavy_of = arg[hoff:hoff + rows * 4].view(torch.int32)
        ah = arg[aoff:aoff + nh * H * 4].view(torch.int32).view(nh, H).long()
        hr = csr.plan.heavy_row[:nh].long()
        pos[hr] = rp[hr].view(-1, 1) + ah[heavy_of[hr].long()]
    return torch.where(deg.view(-1, 1) > 0, pos, torch.full_like(pos, -1))


class _Aggregate(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, graph: Graph, reduce: int):
        out, arg = spmm_fwd(graph.fwd, x, reduce, graph.num_nodes, want_arg=x.requires_grad)
        ctx.graph = graph
        ctx.reduce = reduce
        ctx.save_for_backward(arg if arg is not None else torch.empty(0, device=x.device))
        return out

    @staticmethod
    def backward(ctx, g):
        (arg,) = ctx.saved_tensors
        graph = ctx.graph
        gx = spmm_bwd(graph.bwd, graph.perm_t, graph.fwd.rowptr, g, ctx.reduce,
                      arg if ctx.reduce == 2 else None, graph.num_nodes)
        return gx, None, None


def aggregate(x: torch.Tensor, graph: Graph, reduce: str = "sum") -> torch.Tensor:
    """out[i] = AGG_{j: (j -> i) in E} x[j]  (PyG SAGEConv aggregation)."""
    x = _check_x(x, "aggregate")
    if x.size(0) != graph.num_nodes:
        raise ValueError(f"aggregate: x has {x.size(0)} rows, graph has {graph.num_nodes} nodes")
    r = REDUCE[reduce]
    return _Aggregate.apply(x, graph, r)


class _SegmentReduce(torch.autograd.Function):
    @staticmethod
    def forward(ctx, src, seg: SegmentIndex, reduce: int):
        out, arg = spmm_fwd(seg.fwd, src, reduce, seg.num_rows, want_arg=src.requires_grad)
        ctx.seg = seg
        ctx.reduce = reduce
        ctx.save_for_backward(arg if arg is not None else torch.empty(0, device=src.device))
        return out

    @staticmethod
    def backward(ctx, g):
        seg = ctx.seg
        r = ctx.reduce
        if r == 2:
            (arg,) = ctx.saved_tensors
            # position i receives g[seg(i), c] where arg[seg(i), c] is i's slot in the forward CSR.
            slot = torch.empty(seg.n, dtype=torch.int32, device=g.device)
            slot[seg.fwd.col[:seg.n].long()] = torch.arange(seg.n, dtype=torch.int32, device=g.device)
            return spmm_bwd(seg.bwd, slot, seg.fwd.rowptr, g, 2, arg, seg.n), None, None
        # sum / mean: every position receives its segment's gradient row (a broadcast;
        # one HBM write of the output, no gather structure needed)
        g = g.contiguous()
        if r == 1:
            cnt = seg.fwd.degree().clamp_min(1).to(g.dtype)
            g = g / cnt.unsqueeze(1)
        return g.index_select(0, seg.index), None, None


class _SegmentReduceBf16(torch.autograd.Function):
    """sum / mean over segments of a bf16 [n, H] source into f32 [R, H] (bgnn_segment_sum_bf16);
    backward: every position receives its segment's (scaled) gradient row, in bf16."""

    @staticmethod
    def forward(ctx, src, seg: SegmentIndex, mean: bool):
        H = src.size(1)
        out = torch.empty(seg.num_rows, H, dtype=torch.float32, device=src.device)
        _lib.call("bgnn_segment_sum_bf16", seg.fwd.rowptr.data_ptr(), seg.fwd.col.data_ptr(), seg.num_rows,
                  src.data_ptr(), src.stride(0), H, int(mean), out.data_ptr(), out.stride(0), _stream())
        ctx.seg, ctx.mean = seg, mean
        return out

    @staticmethod
    def backward(ctx, g):
        seg = ctx.seg
        g = g.contiguous()
        H = g.size(1)
        if g.dtype == torch.float32 and g.is_cuda and H % 8 == 0 and H <= 512 and g.data_ptr() % 16 == 0:
            # one pass: scale, bf16 rounding and the broadcast to every position (bgnn_segment_bcast_bf16)
            out = torch.empty(seg.n, H, dtype=torch.bfloat16, device=g.device)
            _lib.call("bgnn_segment_bcast_bf16", seg.fwd.rowptr.data_ptr(), seg.fwd.col.data_ptr(), seg.num_rows,
                      g.data_ptr(), g.stride(0), H, int(ctx.mean), out.data_ptr(), out.stride(0), _stream())
            return out, None, None
        if ctx.mean:
            g = g / seg.fwd.degree().clamp_min(1).to(g.dtype).unsqueeze(1)
        return g.to(torch.bfloat16).index_select(0, seg.index), None, None


def segment_reduce(src: torch.Tensor, seg: SegmentIndex, reduce: str = "sum") -> torch.Tensor:
    if src.dtype == torch.bfloat16 and reduce in ("sum", "add", "mean"):
        require_cuda(src, what="segment_reduce")
        src = src.contiguous()
        if src.dim() != 2 or src.size(0) != seg.n or src.size(1) % 8 or src.size(1) > 512:
            raise ValueError("segment_reduce(bf16): need [n, H] with H % 8 == 0, H <= 512")
        return _SegmentReduceBf16.apply(src, seg, reduce == "mean")
    src = _check_x(src, "segment_reduce")
    if src.size(0) != seg.n:
        raise ValueError(f"segment_reduce: src has {src.size(0)} rows, index has {seg.n} entries")
    return _SegmentReduce.apply(src, seg, REDUCE[reduce])
