"""EA_GNN's GraphNetBlock (Models/BuckGNN.py:528-566) on bgnn kernels, transform-first.

The reference block runs three MLPs on per-edge concatenations:

    e'  = edge_mlp( [x[row] | x[col] | e] )          Linear(3H->H) . ReLU . Linear(H->H)
    m   = phi     ( [x[col] | e'] )                   Linear(2H->H) . ReLU . Linear(H->H)
    agg = scatter_mean(m, row)                        (row = edge_index[0])
    out = gamma([x | agg]);  out = out + beta(out)

A Linear on a concatenation splits by column blocks of its weight, and the node-indexed blocks
are the same for every edge of a node, so they are computed per NODE and gathered:

    [P_row | P_col | Q] = x . [W1[:, :H] ; W1[:, H:2H] ; Wphi[:, :H]]^T       (N x 3H, one GEMM)
    h1  = ReLU( e . W1[:, 2H:]^T + b1 + P_row[row] + P_col[col] )
    e'  = h1 . W2^T + b2
    m1  = ReLU( e' . Wphi[:, H:]^T + bphi + Q[col] )
    m   = m1 . Wphi2^T + bphi2

which removes 2 of the 4 per-edge K = H products of the first layers (3H + 2H -> H + H) and
leaves every per-edge GEMM at K = H. All GEMMs run on the bgnn split kernels
(f32-accurate f16x3, or bf16 operands with f32 accumulation when `bf16=True`, the precision
of BASELINE configs[4]); gathers are row index_selects, their backward and the scatter_mean
are deterministic bgnn segment reductions over the edge index (no atomics).
"""
from __future__ import annotations

import torch

from .fused import linear, mlp
from .graph import SegmentIndex, _index_cache
from .ops import segment_reduce


def edge_segments(edge_index: torch.Tensor, num_nodes: int):
    """Segment structures of edge_index[0] (row) and edge_index[1] (col), cached per tensor."""
    row = _index_cache.get(edge_index, ("ea_row", int(num_nodes)),
                           lambda: SegmentIndex.build(edge_index[0], num_nodes))
    col = _index_cache.get(edge_index, ("ea_col", int(num_nodes)),
                           lambda: SegmentIndex.build(edge_index[1], num_nodes))
    return row, col


class _GatherAdd(torch.autograd.Function):
    """out = act(a + p1[i1] (+ p2[i2])) over edge rows; backward: da = g', dp1 = segment_sum
    of g' by i1 (and dp2 by i2), g' = g masked by the ReLU."""

    @staticmethod
    def forward(ctx, a, p1, seg1: SegmentIndex, p2, seg2: SegmentIndex, relu: bool):
        out = a + p1.index_select(0, seg1.index)
        if p2 is not None:
            out += p2.index_select(0, seg2.index)
        if relu:
            out.relu_()
        ctx.seg1, ctx.seg2, ctx.relu, ctx.has2 = seg1, seg2, relu, p2 is not None
        ctx.save_for_backward(out if relu else torch.empty(0, device=a.device))
        return out

    @staticmethod
    def backward(ctx, g):
        (out,) = ctx.saved_tensors
        g = g.contiguous()
        if ctx.relu:
            g = g * (out > 0)
        d1 = segment_reduce(g, ctx.seg1, "sum")
        d2 = segment_reduce(g, ctx.seg2, "sum") if ctx.has2 else None
        return g, d1, None, d2, None, None


def gather_add(a, p1, seg1, p2=None, seg2=None, relu=False):
    return _GatherAdd.apply(a, p1, seg1, p2, seg2, relu)


def graphnet_block(blk, x: torch.Tensor, e: torch.Tensor, edge_index: torch.Tensor, bf16: bool = False):
    """(x_out, e_out) of one GraphNetBlock `blk` (bgnn.buckgnn.GraphNetBlock: same parameters
    as the reference's) on the bgnn kernels."""
    N, H = x.shape
    seg_row, seg_col = edge_segments(edge_index, N)
    W1, b1 = blk.edge_mlp[0].weight, blk.edge_mlp[0].bias
    W2, b2 = blk.edge_mlp[2].weight, blk.edge_mlp[2].bias
    Wp, bp = blk.node_mlp_phi[0].weight, blk.node_mlp_phi[0].bias
    Wp2, bp2 = blk.node_mlp_phi[2].weight, blk.node_mlp_phi[2].bias
    x = x.contiguous()
    # node-level blocks of the two concatenation Linears, one GEMM
    P = linear(x, torch.cat([W1[:, :H], W1[:, H:2 * H], Wp[:, :H]], 0), None, False, bf16=bf16)
    h1 = gather_add(linear(e, W1[:, 2 * H:], b1, False, bf16=bf16), P[:, :H], seg_row, P[:, H:2 * H], seg_col,
                    relu=True)
    e_out = linear(h1, W2, b2, False, bf16=bf16)
    m1 = gather_add(linear(e_out, Wp[:, H:], bp, False, bf16=bf16), P[:, 2 * H:], seg_col, relu=True)
    msg = linear(m1, Wp2, bp2, False, bf16=bf16)
    agg = segment_reduce(msg, seg_row, "mean")
    out = mlp(blk.node_mlp_gamma, torch.cat([x, agg], 1), bf16=bf16)
    out = out + mlp(blk.node_mlp_beta, out, bf16=bf16)
    return out, e_out
