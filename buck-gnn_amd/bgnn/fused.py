"""Fused GraphSAGE layer for the BuckGNN layer loop (Models/BuckGNN.py:430-444).

One autograd node per layer computes, for train or eval mode,

    x_next = Dropout_p( ReLU( BN( normalize( SAGEConv(x_prev, edge_index) ) ) ) + [skip] x_prev )

with SAGEConv(aggr in {add, sum, mean}, normalize=True) evaluated transform-first:

    z   = x_prev · [W_l ; W_r]^T                 one fp32 MFMA GEMM, stored as planes
                                                  z_l [N, H] and z_r [N, H]
    h_i = AGG_{j->i} z_l[j] + z_r[i] + b_l        (= lin_l(AGG x) + lin_r(x): AGG is linear)
    o_i = h_i / max(||h_i||, 1e-12)               fused into the aggregation kernel,
                                                  which also emits BatchNorm partial sums

The backward mirrors it: BN statistics of dL/dx_next, a row-wise kernel for the
BN + normalize backward giving dh, the transpose aggregation dz_l = A^T dh, and
two GEMMs  dx = [dz_l | dh] · [W_l ; W_r]  and  d[W_l ; W_r] = [dz_l | dh]^T · x_prev.
"""
from __future__ import annotations

import torch

from . import _lib
from .graph import Graph, _stream, require_cuda

# "hip" = bgnn_gemm_f32 (hand-written f32 MFMA); "torch" = torch.mm (rocBLAS/hipBLASLt),
# kept only for A/B measurement. Both run on the GPU.
GEMM_BACKEND = "hip"

# z = [z_l | z_r] and dz = [dz_l | dh] are stored either interleaved ([N, 2H], row i holds
# both halves) or as two dense [N, H] planes (needs H % PLANE_TILE == 0, the GEMM tile width).
# Measured on MI355X (cfg2, tools/tune_agg.py + tools/ab_step.py): the forward aggregation is
# 5% faster on interleaved z (z_l[i], z_r[i] in one DRAM page), the transpose aggregation 4%
# faster on dz planes, but the plane-operand GEMMs lose more than that: whole step 18.83 ms
# interleaved vs 18.92 (dz planes) / 19.12 (z planes) / 19.23 (both).
PLANE_TILE = 128
Z_PLANES = False
DZ_PLANES = False
# dgrad B operand: transposed copy of [W_l;W_r] (K-contiguous loads) instead of strided reads
DGRAD_WT = True
# folded input transform: the weight-by-weight products (Wf = Wcat W_in, its gradients; no node
# dimension, <= 0.3 GFLOP each) on torch.mm instead of bgnn_gemm (A/B switch; default bgnn:
# both are f32-class, torch.mm saved ~1 % of the step but shifts the BN-amplified gradient
# rounding noise, tools/fold_ab.py)
FOLD_WEIGHTS_TORCH = False
# skip layers' dgrad adds the dropout-masked incoming gradient in its epilogue
# (bgnn_gemm_f32_dropadd) instead of reading a skip gradient bgnn_sage_bwd_rows wrote
DGRAD_DROPADD = True

# bf16-stored Linear backward (EA_GNN's bf16 configuration): ReLU mask + f32 bias-gradient sums
# in one bgnn pass (bgnn_linear_bwd_prep_bf16) instead of torch threshold_backward + sum (A/B switch)
BF16_PREP = True
# per-layer weight maxima of a SAGE layer loop in one launch (bgnn_absmax_items_f32)
ABSMAX_ITEMS = True
# [W_l;W_r] of all layers packed by a multi-tensor copy into a persistent buffer (not torch.cat)
PERSISTENT_WPACK = True
# max aggregation: the two input-gradient products as one GEMM [dh W_l | dh W_r (+ drop(g))] and
# the two weight gradients as one [agg | x]^T dh (A/B switch)
MAX_MERGED = True
# forward / input-gradient GEMMs of the K = H layers take [W_l;W_r] (and its transpose) as images
# pre-split once per step (bgnn_gemm_wsplit), staged by LDS-DMA in the GEMM (bgnn_gemm_f32_w);
# bit-identical to the register-staged path (A/B switch)
WSPLIT = True

# Optional per-launch timing (bench.py): name -> list of (start, end) HIP events recorded
# on the launching stream around the named launch.
TIMERS = None
# event factory for TIMERS (None: torch.cuda.Event(enable_timing=True)); bench.py installs HIP events
# created with hipEventDisableSystemFence: a default event's record does a system-scope release (cache
# writeback + invalidate) that leaves the GPU idle ~5 us per event between the timed kernels
TIMER_EVENT = None


class _timed:
    __slots__ = ("name", "ev")

    def __init__(self, name):
        self.name = name
        self.ev = None

    def __enter__(self):
        if TIMERS is not None:
            mk = TIMER_EVENT or (lambda: torch.cuda.Event(enable_timing=True))
            self.ev = (mk(), mk())
            self.ev[0].record()
        return self

    def __exit__(self, *exc):
        if self.ev is not None:
            self.ev[1].record()
            TIMERS.setdefault(self.name, []).append(self.ev)
        return False


class Planes:
    """A row-major matrix [rows, P*blk] stored as P contiguous [rows, blk] planes (tensor t of
    shape [P, rows, blk]). Used for z = [z_l | z_r] and dz = [dz_l | dh], whose halves the
    aggregation kernels read as separate dense arrays."""
    __slots__ = ("t",)

    def __init__(self, t: torch.Tensor):
        if t.dim() != 3 or not t.is_contiguous():
            raise ValueError("Planes: need a contiguous [P, rows, blk] tensor")
        self.t = t

    def size(self, d):
        return self.t.size(1) if d == 0 else self.t.size(0) * self.t.size(2)

    def dense(self) -> torch.Tensor:
        return self.t.permute(1, 0, 2).reshape(self.size(0), self.size(1))


class Pair:
    """The row-wise concatenation [a | b] of two [rows, blk] fp32 matrices with the same row
    stride, read in place as one GEMM A operand (the plane-split addressing of the bgnn GEMM:
    plane 1 lives (b - a) elements after plane 0). The aggregate-first max-aggregation layer
    multiplies [AGG x | x] by [W_l | W_r]^T this way without building the concatenation."""
    __slots__ = ("a", "b")

    def __init__(self, a: torch.Tensor, b: torch.Tensor):
        if (a.dim() != 2 or a.shape != b.shape or a.stride() != b.stride() or a.stride(1) != 1
                or a.dtype != torch.float32 or b.dtype != torch.float32 or a.device != b.device):
            raise ValueError("Pair: need two fp32 [rows, blk] matrices of one shape and row stride")
        self.a, self.b = a, b

    def size(self, d):
        return self.a.size(0) if d == 0 else 2 * self.a.size(1)

    def dense(self) -> torch.Tensor:
        return torch.cat([self.a, self.b], 1)


def _operand(x):
    """(ptr, ld, blk, pstride) of a dense tensor, Planes or Pair operand."""
    if isinstance(x, Planes):
        P, R, blk = x.t.shape
        return x.t.data_ptr(), blk, (blk if P > 1 else 0), R * blk
    if isinstance(x, Pair):
        diff = x.b.data_ptr() - x.a.data_ptr()
        if diff % 16:   # (the GEMM's float4 loads test plane 0's alignment only)
            raise ValueError("Pair: the two halves must be 16-byte aligned relative to each other")
        return x.a.data_ptr(), x.a.stride(0), x.a.size(1), diff // 4
    if x.stride(1) != 1:
        raise ValueError("gemm: operands must have unit column stride")
    return x.data_ptr(), x.stride(0), 0, 0


def absmax(x: torch.Tensor, out: torch.Tensor = None, accumulate: bool = False) -> torch.Tensor:
    """max |x| of a row-major fp32 matrix (unit column stride) into a 1-element device tensor
    (bgnn_absmax_f32; accumulate folds into out's current value)."""
    if out is None:
        out = torch.empty(1, dtype=torch.float32, device=x.device)
        accumulate = False
    x2 = x.reshape(x.size(0), -1) if x.dim() != 2 else x
    _lib.call("bgnn_absmax_f32", x2.data_ptr(), x2.size(0), x2.size(1), x2.stride(0), out.data_ptr(),
              int(accumulate), _stream())
    return out


def gemm(a, b: torch.Tensor, trans_a: bool, trans_b: bool, out=None, beta: float = 0.0, alpha: float = 1.0,
         bias: torch.Tensor = None, relu: bool = False, a_amax: torch.Tensor = None,
         b_amax: torch.Tensor = None, c_amax: torch.Tensor = None, bf16: bool = False):
    """C = act(alpha * op(a) @ op(b) + beta * C + bias) (fp32, row-major operands, unit column
    stride). `a` and `out` may be Planes. a_amax / b_amax: optional device scalars holding
    max|a| / max|b| (the f16x3 operand scales; computed inside when absent); c_amax: optional
    device scalar that max |C| is folded into (bgnn_gemm_f32_scaled). bf16: round both operands
    to bf16 (one MFMA product, f32 accumulation and output) instead of the f32-accurate split."""
    M = a.size(1) if trans_a else a.size(0)
    K = a.size(0) if trans_a else a.size(1)
    N = b.size(0) if trans_b else b.size(1)
    Kb = b.size(1) if trans_b else b.size(0)
    if K != Kb:
        raise ValueError(f"gemm: inner dims differ ({K} vs {Kb})")
    if out is None:
        out = torch.empty(M, N, dtype=torch.float32, device=b.device)
        beta = 0.0
    if out.size(0) != M or out.size(1) != N:
        raise ValueError(f"gemm: out is {out.size(0)}x{out.size(1)}, expected {M}x{N}")
    if GEMM_BACKEND == "torch":
        ad = a.dense() if isinstance(a, (Planes, Pair)) else a
        od = out.dense() if isinstance(out, Planes) else out
        ra = ad.t() if trans_a else ad
        rb = b.t() if trans_b else b
        if beta == 0.0:
            torch.mm(ra, rb, out=od)
            if alpha != 1.0:
                od.mul_(alpha)
        else:
            od.mul_(beta).addmm_(ra, rb, alpha=alpha)
        if bias is not None:
            od.add_(bias)
        if relu:
            od.relu_()
        if isinstance(out, Planes):
            out.t.copy_(od.view(M, out.t.size(0), out.t.size(2)).permute(1, 0, 2))
        return out
    pa, lda, a_blk, a_ps = _operand(a)
    pb, ldb, _, _ = _operand(b)
    pc, ldc, c_blk, c_ps = _operand(out)
    prec = 1 if bf16 else 0
    ws_bytes = _lib.query("bgnn_gemm_ws_bytes_ex", M, N, K, int(trans_a), int(trans_b), prec)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=b.device) if ws_bytes else None
    _lib.call("bgnn_gemm_f32_scaled", int(trans_a), int(trans_b), M, N, K, float(alpha), pa, lda, a_blk, a_ps,
              pb, ldb, float(beta), pc, ldc, c_blk, c_ps, None if bias is None else bias.data_ptr(), int(relu),
              _ptr(a_amax), _ptr(b_amax), _ptr(c_amax), prec, None if ws is None else ws.data_ptr(), ws_bytes,
              _stream())
    return out


_BF16_BUILT = {(0, 1): (0, 1, 3, 4, 5, 7), (1, 0): (0, 1, 2, 3)}
# bf16-stored A times an f32 weight (A B^T, K % 64 == 0): round the weight to bf16 once (torch's
# round-to-nearest-even, the rounding the GEMM applies in-tile) so that both operands are bf16 and
# the LDS-DMA bf16 kernel (gemm_b16.hip, bit-identical) takes the product. False: the
# register-staged kernel reads the f32 weight (A/B).
B16_WEIGHTS = True


def b16_weight(a: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """w (the B^T operand of a K-contiguous product with a) as bf16 when a is stored bf16 and
    the LDS-DMA bf16 kernel applies; else w unchanged."""
    if B16_WEIGHTS and a.dtype == torch.bfloat16 and w.dtype == torch.float32 and w.size(1) % 64 == 0:
        return w.to(torch.bfloat16)
    return w


def gemm_bf16(a: torch.Tensor, b: torch.Tensor, trans_a: bool, trans_b: bool, out=None, out_bf16: bool = False,
              bias: torch.Tensor = None, relu: bool = False):
    """C = act(op(a) @ op(b) + bias) on the bf16-operand GEMM (one bf16 MFMA product, f32
    accumulation) with each of a / b / C stored as float32 or bfloat16 (bgnn_gemm_bf16): the bf16
    configuration of EA_GNN keeps its per-edge activations in bf16 (half the HBM bytes)."""
    for t in (a, b):
        if t.dtype not in (torch.float32, torch.bfloat16) or t.stride(1) != 1:
            raise ValueError("gemm_bf16: operands must be float32 / bfloat16 with unit column stride")
    M = a.size(1) if trans_a else a.size(0)
    K = a.size(0) if trans_a else a.size(1)
    N = b.size(0) if trans_b else b.size(1)
    if (b.size(1) if trans_b else b.size(0)) != K:
        raise ValueError("gemm_bf16: inner dims differ")
    if out is None:
        out = torch.empty(M, N, dtype=torch.bfloat16 if out_bf16 else torch.float32, device=b.device)
    if not trans_a and trans_b:
        b = b16_weight(a, b)
    storage = ((1 if a.dtype == torch.bfloat16 else 0) | (2 if b.dtype == torch.bfloat16 else 0)
               | (4 if out.dtype == torch.bfloat16 else 0))
    if storage not in _BF16_BUILT.get((int(trans_a), int(trans_b)), (0,)):
        raise ValueError(f"gemm_bf16: storage {storage} with trans_a={trans_a}, trans_b={trans_b} is not built")
    ws_bytes = _lib.query("bgnn_gemm_ws_bytes_ex", M, N, K, int(trans_a), int(trans_b), 1)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=b.device) if ws_bytes else None
    _lib.call("bgnn_gemm_bf16", int(trans_a), int(trans_b), M, N, K, 1.0, a.data_ptr(), a.stride(0), b.data_ptr(),
              b.stride(0), 0.0, out.data_ptr(), out.stride(0), _ptr(bias), int(relu), storage, _ptr(ws), ws_bytes,
              _stream())
    return out


class LinearBf16Fn(torch.autograd.Function):
    """y = act(x W^T + b) with bf16 operands and bf16 storage of x and / or y (EA_GNN's bf16
    configuration: per-edge activations in bf16, like torch autocast's bf16 Linear). Backward:
    ReLU mask and bias gradient (f32 sum) in torch, dgrad / wgrad on bgnn_gemm_bf16 (dx in x's
    dtype, dW f32)."""

    @staticmethod
    def forward(ctx, x, weight, bias, relu: bool, out_bf16: bool):
        x = x.contiguous()
        y = gemm_bf16(x, weight.contiguous(), False, True, out_bf16=out_bf16, bias=bias, relu=relu)
        ctx.relu, ctx.has_bias = relu, bias is not None
        ctx.save_for_backward(x, weight, y if relu else torch.empty(0, device=x.device))
        return y

    @staticmethod
    def backward(ctx, g):
        x, weight, y = ctx.saved_tensors
        if g.dtype == torch.bfloat16 and BF16_PREP:
            g, db = relu_bias_grad_bf16(g, y if ctx.relu else None, ctx.has_bias)
        else:
            g = g.contiguous()
            if ctx.relu:
                g = torch.ops.aten.threshold_backward(g, y, 0.0)
            db = torch.sum(g, 0, dtype=torch.float32) if ctx.has_bias else None
        dx = None
        if ctx.needs_input_grad[0]:
            dx = gemm_bf16(g, weight.t().contiguous(), False, True, out_bf16=x.dtype == torch.bfloat16)
        dw = gemm_bf16(g, x, True, False)
        return dx, dw, db, None, None


def linear_bf16(x, weight, bias=None, relu=False, out_bf16=True):
    return LinearBf16Fn.apply(x, weight, bias, relu, out_bf16)


def mlp_bf16(seq: torch.nn.Sequential, x: torch.Tensor, out_bf16: bool = True):
    """An nn.Sequential of Linear/ReLU with bf16 operands, every activation stored in bf16
    (out_bf16: also the last one), each ReLU fused into the preceding Linear's epilogue."""
    mods = list(seq)
    i = 0
    while i < len(mods):
        m = mods[i]
        if isinstance(m, torch.nn.Linear):
            fuse = i + 1 < len(mods) and isinstance(mods[i + 1], torch.nn.ReLU)
            last = i + (2 if fuse else 1) >= len(mods)
            x = linear_bf16(x, m.weight, m.bias, fuse, out_bf16 or not last)
            i += 2 if fuse else 1
        else:
            x = m(x)
            i += 1
    return x


def relu_bias_grad_bf16(g: torch.Tensor, y=None, bias: bool = True):
    """(g', db) for the backward of act(x W^T + b) with bf16 g (and bf16 ReLU output y): g' = g
    masked by y > 0 (bf16; g itself when y is None), db = f32 column sums of g' (None when bias is
    False). One pass over g (bgnn_linear_bwd_prep_bf16) instead of torch's threshold_backward plus
    a float32 sum, each of which torch splits in two launches at E x 512 bf16 (> 2^31 bytes)."""
    g = g.contiguous()
    C = g.size(1)
    ok = (C % 8 == 0 and 8 <= C <= 2048 and 256 % (C // 8) == 0 and g.data_ptr() % 16 == 0
          and (y is None or (y.dtype == torch.bfloat16 and y.is_contiguous() and y.data_ptr() % 16 == 0)))
    if not ok:
        if y is not None:
            g = torch.ops.aten.threshold_backward(g, y, 0.0)
        return g, (torch.sum(g, 0, dtype=torch.float32) if bias else None)
    if y is None and not bias:
        return g, None
    gm = torch.empty_like(g) if y is not None else g
    slots = _lib.query("bgnn_linear_bwd_prep_slots")
    part = torch.empty(slots, 2, C, dtype=torch.float32, device=g.device)
    s = _stream()
    _lib.call("bgnn_linear_bwd_prep_bf16", g.data_ptr(), None if y is None else y.data_ptr(), g.size(0), C,
              gm.data_ptr() if y is not None else None, part.data_ptr(), s)
    db = None
    if bias:
        db = torch.empty(C, dtype=torch.float32, device=g.device)
        _lib.call("bgnn_reduce_partials", part.data_ptr(), slots, C, db.data_ptr(), None, 0, s)
    return gm, db


def relu_bias_grad(g: torch.Tensor, y=None, bias: bool = True):
    """(g', db, max|g'|) for the backward of act(x W^T + b): g' = g masked by y > 0 (y = the ReLU
    output; None = no ReLU), db = column sums of g' (None when bias is False). One pass over g
    (bgnn_linear_bwd_prep: mask, bias-gradient partials and max|g'|) where the width allows,
    else torch threshold_backward + sum + a max pass."""
    g = g.contiguous()
    C = g.size(1)
    if C % 4 == 0 and 4 <= C <= 1024 and 256 % (C // 4) == 0:
        gm = torch.empty_like(g) if y is not None else g
        slots = _lib.query("bgnn_linear_bwd_prep_slots")
        part = torch.empty(slots, 2, C, dtype=torch.float32, device=g.device)
        g_amax = torch.zeros(1, dtype=torch.float32, device=g.device)
        s = _stream()
        _lib.call("bgnn_linear_bwd_prep", g.data_ptr(), None if y is None else y.data_ptr(), g.size(0), C,
                  gm.data_ptr() if y is not None else None, part.data_ptr(), g_amax.data_ptr(), s)
        db = None
        if bias:
            db = torch.empty(C, dtype=torch.float32, device=g.device)
            _lib.call("bgnn_reduce_partials", part.data_ptr(), slots, C, db.data_ptr(), None, 0, s)
        return gm, db, g_amax
    if y is not None:
        g = torch.ops.aten.threshold_backward(g, y, 0.0)   # ReLU mask in one pass
    return g, (g.sum(0) if bias else None), absmax(g)


class LinearFn(torch.autograd.Function):
    """(y, max|y|) with y = act(x W^T + b) on the bgnn GEMM (bias + ReLU fused in the epilogue,
    max|y| folded in there too: the next Linear's operand scale); backward: dgrad and wgrad
    GEMMs on the same kernel, sharing one max|g| pass (Models/BuckGNN.py:67-74 encoder)."""

    @staticmethod
    def forward(ctx, x, weight, bias, relu: bool, x_amax, bf16: bool = False, amax=None):
        x = x.contiguous()
        if amax is None:   # [max|W|, max|y|], zeroed (callers batch these: one fill per MLP)
            amax = torch.zeros(2, dtype=torch.float32, device=x.device)
        w_amax, y_amax = amax[0:1], amax[1:2]
        if not bf16:   # (bf16 operands need no scales)
            absmax(weight, w_amax, accumulate=True)
            if x_amax is None:
                x_amax = absmax(x)
        y = gemm(x, weight.contiguous(), trans_a=False, trans_b=True, bias=bias, relu=relu,
                 a_amax=None if bf16 else x_amax, b_amax=None if bf16 else w_amax,
                 c_amax=None if bf16 else y_amax, bf16=bf16)
        ctx.relu = relu
        ctx.bf16 = bf16
        ctx.has_bias = bias is not None
        ctx.save_for_backward(x, weight, y if relu else torch.empty(0, device=x.device),
                              x_amax if x_amax is not None else torch.empty(0, device=x.device), w_amax)
        ctx.mark_non_differentiable(y_amax)
        ctx.set_materialize_grads(False)   # no zero-filled gradient for y_amax
        return y, y_amax

    @staticmethod
    def backward(ctx, g, _g_amax):
        if g is None:
            return None, None, None, None, None, None, None
        x, weight, y, x_amax, w_amax = ctx.saved_tensors
        bf16 = ctx.bf16
        g, db, g_amax = relu_bias_grad(g, y if ctx.relu else None, ctx.has_bias)
        if bf16:
            g_amax = None
        w_amax = None if bf16 else w_amax
        x_amax = None if bf16 else x_amax
        dx = None
        if ctx.needs_input_grad[0]:
            dx = (gemm(g, weight.t().contiguous(), trans_a=False, trans_b=True, a_amax=g_amax, b_amax=w_amax,
                       bf16=bf16)
                  if DGRAD_WT else
                  gemm(g, weight.contiguous(), trans_a=False, trans_b=False, a_amax=g_amax, b_amax=w_amax,
                       bf16=bf16))
        dw = gemm(g, x, trans_a=True, trans_b=False, a_amax=g_amax, b_amax=x_amax, bf16=bf16)
        return dx, dw, db, None, None, None, None


def linear(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor = None, relu: bool = False,
           x_amax: torch.Tensor = None, return_amax: bool = False, bf16: bool = False, amax_buf=None):
    """act(x W^T + b) on the bgnn GEMM; bf16: bf16 operands, f32 accumulation and output.
    amax_buf: optional zeroed 2-float device scratch for [max|W|, max|y|]."""
    y, y_amax = LinearFn.apply(x, weight, bias, relu, x_amax, bf16, amax_buf)
    return (y, y_amax) if return_amax else y


# the node encoder's leading Linear(16,64).ReLU.Linear(64,128).ReLU as one VALU kernel
# (bgnn_mlp2_fwd / _bwd) instead of two GEMM launches with their operand-max passes:
# fwd 57 us, bwd 108 us + 11 us slot sums on cfg2; the step 9.94 -> 9.82 ms (tools/ab_step.py);
# round 4: conflict-free W2^T load, backward at 512 threads: fwd 54 us, bwd 94 us (bit-identical)
FUSED_MLP2 = True


class _Mlp2Fn(torch.autograd.Function):
    """(h, max|h|) with h = ReLU(ReLU(x W1^T + b1) W2^T + b2) on bgnn_mlp2_fwd; backward: the
    four weight / bias gradients from bgnn_mlp2_bwd (x gets none: node features are data)."""

    @staticmethod
    def forward(ctx, x, W1, b1, W2, b2):
        N, F = x.shape
        D1, D2 = W1.size(0), W2.size(0)
        h = torch.empty(N, D2, dtype=torch.float32, device=x.device)
        amax = torch.zeros(1, dtype=torch.float32, device=x.device)
        _lib.call("bgnn_mlp2_fwd", x.data_ptr(), N, F, D1, D2, W1.data_ptr(), b1.data_ptr(), W2.data_ptr(),
                  b2.data_ptr(), h.data_ptr(), amax.data_ptr(), _stream())
        ctx.save_for_backward(x, W1, b1, W2, h)
        ctx.mark_non_differentiable(amax)
        ctx.set_materialize_grads(False)
        return h, amax

    @staticmethod
    def backward(ctx, dh, _g_amax):
        if dh is None:
            return None, None, None, None, None
        x, W1, b1, W2, h = ctx.saved_tensors
        dh = dh.contiguous()
        N, F = x.shape
        D1, D2 = W1.size(0), W2.size(0)
        dW1, db1 = torch.empty_like(W1), torch.empty_like(b1)
        dW2 = torch.empty_like(W2)
        db2 = torch.empty(D2, dtype=torch.float32, device=x.device)
        ws_bytes = _lib.query("bgnn_mlp2_bwd_ws_bytes", N)
        ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=x.device)
        _lib.call("bgnn_mlp2_bwd", x.data_ptr(), N, F, D1, D2, W1.data_ptr(), b1.data_ptr(), W2.data_ptr(),
                  h.data_ptr(), dh.data_ptr(), dW1.data_ptr(), db1.data_ptr(), dW2.data_ptr(), db2.data_ptr(),
                  ws.data_ptr(), ws_bytes, _stream())
        return None, dW1, db1, dW2, db2


class SmallMLPFn(torch.autograd.Function):
    """An nn.Sequential of Linear (+ ReLU) layers on a few rows (the decoder on the pooled
    [graphs, H] features, Models/BuckGNN.py:94-100) with one bgnn_small_linear_fwd launch per layer
    (bias and ReLU inside) and one bgnn_small_linear_bwd per layer backward (ReLU mask, dW, db and
    dx together) instead of a library GEMM, a ReLU kernel, bias reductions and ReLU-mask kernels
    per layer. Inputs: x, then (W, b, relu) per layer flattened as weights / biases."""

    @staticmethod
    def forward(ctx, x, relus, *params):
        x = x.contiguous()
        B = x.size(0)
        s = _stream()
        acts = [x]
        for i, relu in enumerate(relus):
            W, b = params[2 * i], params[2 * i + 1]
            N, K = W.shape
            y = torch.empty(B, N, dtype=torch.float32, device=x.device)
            _lib.call("bgnn_small_linear_fwd", acts[-1].data_ptr(), B, K, W.data_ptr(), _ptr(b), N, int(relu),
                      y.data_ptr(), s)
            acts.append(y)
        ctx.relus = relus
        ctx.has_bias = [params[2 * i + 1] is not None for i in range(len(relus))]
        ctx.save_for_backward(*acts, *[params[2 * i] for i in range(len(relus))])
        return acts[-1]

    @staticmethod
    def backward(ctx, g):
        L = len(ctx.relus)
        saved = ctx.saved_tensors
        acts, Ws = saved[:L + 1], saved[L + 1:]
        s = _stream()
        g = g.contiguous()
        B = g.size(0)
        grads = [None] * (2 * L)
        gx = None
        for i in reversed(range(L)):
            W = Ws[i]
            N, K = W.shape
            dW = torch.empty_like(W)
            db = torch.empty(N, dtype=torch.float32, device=W.device) if ctx.has_bias[i] else None
            need_dx = i > 0 or ctx.needs_input_grad[0]
            dx = torch.empty(B, K, dtype=torch.float32, device=W.device) if need_dx else None
            _lib.call("bgnn_small_linear_bwd", g.data_ptr(), acts[i + 1].data_ptr() if ctx.relus[i] else None,
                      acts[i].data_ptr(), B, K, W.data_ptr(), N, _ptr(dx), dW.data_ptr(), _ptr(db), s)
            grads[2 * i], grads[2 * i + 1] = dW, db
            g = dx
            gx = dx
        return (gx, None, *grads)


# the decoder on the pooled features as bgnn_small_linear layers (SmallMLPFn) when it qualifies
SMALL_MLP = True
SMALL_MLP_MAX_ROWS = 256


def small_mlp(seq: torch.nn.Sequential, x: torch.Tensor):
    """seq(x) through SmallMLPFn when seq is Linear (ReLU) ... Linear with f32 weights, x on the
    GPU with at most SMALL_MLP_MAX_ROWS rows and every in_features a multiple of 4; else None."""
    if not (SMALL_MLP and x.is_cuda and x.dtype == torch.float32 and x.dim() == 2
            and 0 < x.size(0) <= SMALL_MLP_MAX_ROWS):
        return None
    mods = list(seq)
    relus, params = [], []
    i = 0
    while i < len(mods):
        m = mods[i]
        if not (isinstance(m, torch.nn.Linear) and m.weight.dtype == torch.float32 and m.in_features % 4 == 0
                and m.weight.is_contiguous()):
            return None
        relu = i + 1 < len(mods) and isinstance(mods[i + 1], torch.nn.ReLU)
        relus.append(relu)
        params += [m.weight, m.bias]
        i += 2 if relu else 1
    return SmallMLPFn.apply(x, tuple(relus), *params)


def _mlp2_prefix(mods, x: torch.Tensor) -> bool:
    """Whether mods starts with Linear . ReLU . Linear . ReLU that bgnn_mlp2 covers for x."""
    if not FUSED_MLP2 or len(mods) < 4 or x.requires_grad or x.dtype != torch.float32 or x.dim() != 2:
        return False
    l1, r1, l2, r2 = mods[:4]
    if not (isinstance(l1, torch.nn.Linear) and isinstance(l2, torch.nn.Linear) and isinstance(r1, torch.nn.ReLU)
            and isinstance(r2, torch.nn.ReLU) and l1.bias is not None and l2.bias is not None):
        return False
    if l2.in_features != l1.out_features or x.size(1) != l1.in_features:
        return False
    return bool(_lib.query("bgnn_mlp2_supported", l1.in_features, l1.out_features, l2.out_features))


def mlp(seq: torch.nn.Sequential, x: torch.Tensor, return_amax: bool = False, bf16: bool = False):
    """Run an nn.Sequential of Linear/ReLU through bgnn GEMMs, fusing each ReLU into the
    preceding Linear's epilogue (same parameters, same result as seq(x)); a leading
    Linear(16,64).ReLU.Linear(64,128).ReLU runs as one bgnn_mlp2 kernel. With return_amax,
    also returns max|output| (device scalar) when the last module is a Linear or that kernel's
    ReLU, else None."""
    mods = list(seq)
    i = 0
    amax = None
    if not bf16 and _mlp2_prefix(mods, x):
        x, amax = _Mlp2Fn.apply(x.contiguous(), mods[0].weight, mods[0].bias, mods[2].weight, mods[2].bias)
        if len(mods) == 4:
            return (x, amax) if return_amax else x
        mods = mods[4:]
    n_lin = sum(isinstance(m, torch.nn.Linear) for m in mods)
    bufs = torch.zeros(n_lin, 2, dtype=torch.float32, device=x.device)   # one fill for the whole MLP
    k = 0
    while i < len(mods):
        m = mods[i]
        if isinstance(m, torch.nn.Linear):
            fuse = i + 1 < len(mods) and isinstance(mods[i + 1], torch.nn.ReLU)
            x, amax = linear(x, m.weight, m.bias, fuse, x_amax=amax, return_amax=True, bf16=bf16, amax_buf=bufs[k])
            k += 1
            i += 2 if fuse else 1
        else:
            x = m(x)
            amax = None
            i += 1
    return (x, amax) if return_amax else x


def _ptr(t):
    return None if t is None else t.data_ptr()


class RangeRows:
    """Range-row plumbing of one fused sum / mean layer (csrc/ranges.hip; Csr.ensure_ranges): the
    super nodes of a stiffened batch (VirtualEdgeCreate.py:81-113) aggregate their graph's whole
    contiguous real-node range, so
      forward   the previous layer's bgnn_sage_apply also writes the range sums S of x_next as R
                extra rows after it ([N + R, H], x_full); this layer's GEMM runs on all N + R rows,
                and z_l's extra rows (S W_l^T = the summed z_l rows) are the range rows' aggregates
                (bgnn_sage_fwd heavy_agg) -- no chunk pass over the real rows;
      backward  bgnn_sage_bwd_rows also sums dh over each transposed range row's targets, and
                bgnn_range_sums_finish writes those dz_l rows (bgnn_spmm_bwd heavy_done).
    x_full / x_amax: the input's [N + R, H] buffer and a device scalar >= its max |.| (the GEMM's A
    scale), or None; out: write the range sums of x_next into `out_amax`'s layer buffer, appended
    to `holder`; bwd: the backward takes the range path."""
    __slots__ = ("x_full", "x_amax", "out", "out_amax", "bwd", "holder")

    def __init__(self, x_full=None, x_amax=None, out=False, out_amax=None, bwd=True):
        self.x_full, self.x_amax, self.out, self.out_amax, self.bwd = x_full, x_amax, out, out_amax, bwd
        self.holder = []


# range rows (RangeRows) for stiffened batches; False: the chunk + combine path for every heavy row
RANGE_ROWS = True


class LayerConfig:
    __slots__ = ("reduce", "bn", "training", "momentum", "eps", "skip", "p", "seed", "famax", "rng")

    def __init__(self, reduce: int, bn: bool, training: bool, momentum: float, eps: float, skip: bool,
                 p: float, seed: int):
        self.reduce = reduce
        self.bn = bn
        self.training = training
        self.momentum = momentum
        self.eps = eps
        self.skip = skip
        self.p = p if training else 0.0
        self.seed = seed
        # folded layer: 5 zeroed device slots for the maxima of the weight-product operands
        # (max|Wcat|, max|W_in|, max|b_in|, max|dWf|, max|dbf|), so those small f16x3 GEMMs need no
        # max pass (and no zero fill) of their own
        self.famax = None
        self.rng = None     # RangeRows (range rows of a stiffened batch) or None


def _glue_fwd(o, bn_part, slots, x_prev, gamma, beta, running_mean, running_var, cfg: LayerConfig, next_amax,
              graph: Graph = None):
    """The layer glue after the normalised SAGE output o (Models/BuckGNN.py:436-444): BatchNorm
    finalize (train: batch statistics from the aggregation's partial sums, running stats updated;
    eval: running stats), then x_next = drop(relu(o * scale + shift) + skip * x_prev) with
    max|x_next| folded into next_amax. Returns (x_next, (scale, shift, mean, invstd)) (None
    coefficients without BN).

    The BatchNorm partials here are the UNSHIFTED f32 per-block sums of o and o^2 from the
    aggregation epilogue, reduced in fp64 (the per-module BatchNorm1d shifts by the first row,
    bgnn_bn_finalize_shifted, because its input can have |mean| >> std). o is L2-normalised per row,
    so sum_c E[o_c^2] = 1 and each channel's E[o_c^2] <= 1: the E[o^2] - E[o]^2 cancellation costs
    at most the f32 rounding of a block's ~80-row sum, <= 80 * 2^-24 * E[o_c^2] <= 5e-6 * E[o_c^2]
    (typically 1e-8 at h = 512, E[o_c^2] ~ 1/512), next to BatchNorm's eps = 1e-5 in var + eps.
    The shift would need o's first row before the kernel that produces it; the full-size tests
    bound the running statistics against fp64 at rtol 1e-5 (tests/test_gpu_fullsize.py)."""
    N, H = o.shape
    dev = o.device
    s = _stream()
    scale = shift = mean = invstd = None
    if cfg.bn:
        scale = torch.empty(H, dtype=torch.float32, device=dev)
        shift = torch.empty(H, dtype=torch.float32, device=dev)
        mean = torch.empty(H, dtype=torch.float32, device=dev)
        invstd = torch.empty(H, dtype=torch.float32, device=dev)
        if cfg.training:
            _lib.call("bgnn_bn_finalize", bn_part.data_ptr(), slots, H, N, _ptr(gamma), _ptr(beta), cfg.eps,
                      cfg.momentum, _ptr(running_mean), _ptr(running_var), mean.data_ptr(), invstd.data_ptr(),
                      scale.data_ptr(), shift.data_ptr(), s)
        else:
            _lib.call("bgnn_bn_eval_coeffs", H, _ptr(gamma), _ptr(beta), cfg.eps, running_mean.data_ptr(),
                      running_var.data_ptr(), scale.data_ptr(), shift.data_ptr(), s)
            mean.copy_(running_mean)
            invstd.copy_(torch.rsqrt(running_var + cfg.eps))
    rng = cfg.rng
    if rng is not None and rng.out:
        # x_next and the next layer's range sums S in one [N + R, H] buffer (RangeRows)
        R = graph.fwd.plan.n_heavy
        full = torch.empty(N + R, H, dtype=torch.float32, device=dev)
        x_next = full[:N]
        rp = torch.empty(_lib.query("bgnn_range_partial_bytes", N, H) // 4, dtype=torch.float32, device=dev)
        _lib.call("bgnn_sage_apply", o.data_ptr(), _ptr(scale), _ptr(shift), x_prev.data_ptr(), int(cfg.skip),
                  float(cfg.p), cfg.seed, N, H, x_next.data_ptr(), next_amax.data_ptr(), graph.fwd.ranges.data_ptr(),
                  rp.data_ptr(), s)
        _lib.call("bgnn_range_sums_finish", rp.data_ptr(), N, H, graph.fwd.ref(), 0, full[N:].data_ptr(), H,
                  next_amax.data_ptr(), rng.out_amax.data_ptr(), s)
        rng.holder.append(full)
        return x_next, (scale, shift, mean, invstd)
    x_next = torch.empty(N, H, dtype=torch.float32, device=dev)
    _lib.call("bgnn_sage_apply", o.data_ptr(), _ptr(scale), _ptr(shift), x_prev.data_ptr(), int(cfg.skip),
              float(cfg.p), cfg.seed, N, H, x_next.data_ptr(), next_amax.data_ptr(), None, None, s)
    return x_next, (scale, shift, mean, invstd)


def _glue_bwd_stats(g, o, scale, shift, mean, invstd, cfg: LayerConfig, g_rows=None):
    """BatchNorm backward statistics of the layer glue (bgnn_sage_bwd_stats + one slot reduce):
    (dgamma, dbeta, sum_g2, sum_g2xhat) -- all None without BN; eval mode uses zero sums.
    g_rows (int64 [N] or None): row r's gradient is row g_rows[r] of g (the pooled gradient)."""
    if not cfg.bn:
        return None, None, None, None
    N, H = o.shape
    dev = o.device
    s = _stream()
    rs = _lib.query("bgnn_rows_slots", N)
    part2 = torch.empty(rs, 2, H, dtype=torch.float32, device=dev)
    _lib.call("bgnn_sage_bwd_stats", g.data_ptr(), _ptr(g_rows), o.data_ptr(), scale.data_ptr(), shift.data_ptr(),
              mean.data_ptr(), invstd.data_ptr(), float(cfg.p), cfg.seed, N, H, part2.data_ptr(), s)
    sums = torch.empty(2, H, dtype=torch.float32, device=dev)
    _lib.call("bgnn_reduce_partials", part2.data_ptr(), rs, H, sums[0].data_ptr(), sums[1].data_ptr(), 0, s)
    dbeta, dgamma = sums[0], sums[1]
    if cfg.training:
        return dgamma, dbeta, sums[0], sums[1]
    z = torch.zeros(H, dtype=torch.float32, device=dev)
    return dgamma, dbeta, z, z


class SageLayerFn(torch.autograd.Function):
    """Outputs (x_next, max|x_next|): the second output (non-differentiable) is the f16x3 GEMM
    operand scale of the next layer, folded in by bgnn_sage_apply at no extra pass.
    pool (a SegmentIndex, the batch vector's segments): a third output, the mean pool of x_next
    per segment (global_mean_pool, Models/BuckGNN.py:246-249; the same segment kernel as
    bgnn.ops.segment_reduce). Its gradient reaches the backward row passes as the pooled
    gradient / count read through the batch vector (g_rows), not as a materialised [N, H]
    broadcast (the pool's index_select) read twice -- the same g values, so the same bits."""

    @staticmethod
    def forward(ctx, x_prev, x_amax, w_l, b_l, w_r, gamma, beta, running_mean, running_var, graph: Graph,
                cfg: LayerConfig, amax=None, w_in=None, b_in=None, wprep=None, pool=None):
        dev = x_prev.device
        x_prev = x_prev.contiguous()
        H = w_l.size(0)
        N = x_prev.size(0)
        # [W_l;W_r] [2H, H] and its transpose (dgrad operand): from prepare_weights (all layers in
        # a few launches; the amax slot then already holds max|W|) or built here
        if isinstance(wprep, WPrep):
            wcat, wcat_t_pre, img_f, img_d = wprep.wcat, wprep.wcat_t, wprep, wprep
        elif wprep is not None:
            (wcat, wcat_t_pre), img_f, img_d = wprep, None, None
        else:
            wcat, wcat_t_pre, img_f, img_d = torch.cat([w_l, w_r], 0).contiguous(), None, None, None
        img_f = img_f if (img_f is not None and img_f.img_f is not None) else None
        img_d = img_d if (img_d is not None and img_d.img_d is not None) else None
        # operand maxima: [0] = max|W|, [1] = max|x_next| (this layer's output), [2] = max|dz|
        # (zeroed; the layer loop passes one slice of a single per-step fill)
        if amax is None:
            amax = torch.zeros(3, dtype=torch.float32, device=dev)
        w_amax, next_amax, dz_amax = amax[0:1], amax[1:2], amax[2:3]
        folded = w_in is not None
        if folded:
            # the encoder's last Linear folded into this layer's transform (x_prev = its input h):
            # x = h W_in^T + b_in never materialised; z = x [W_l;W_r]^T = h Wf^T + bf with
            # Wf = [W_l;W_r] W_in [2H, K_in], bf = [W_l;W_r] b_in
            if cfg.skip:
                raise ValueError("sage_layer: a folded input transform needs a layer without skip")
            if FOLD_WEIGHTS_TORCH:
                wf = torch.mm(wcat, w_in)
                bf = torch.mv(wcat, b_in)
            else:
                fs = cfg.famax
                fa = (fs[0:1], fs[1:2], fs[2:3]) if fs is not None else (None, None, None)
                if fs is not None:   # the same maxima the GEMMs would compute, without their fills
                    absmax(wcat, fa[0], accumulate=True)
                    absmax(w_in, fa[1], accumulate=True)
                    absmax(b_in.view(1, -1), fa[2], accumulate=True)
                wf = gemm(wcat, w_in.contiguous(), trans_a=False, trans_b=False, a_amax=fa[0], b_amax=fa[1])
                # (bgnn GEMM, not torch.mv: rocBLAS's GEMV moved the BN-amplified gradients of the
                # Shared variant 50x further from fp64, tests/test_gpu_fold.py)
                bf = gemm(wcat, b_in.contiguous().view(H, 1), trans_a=False, trans_b=False, a_amax=fa[0],
                          b_amax=fa[2]).view(-1)
            absmax(wf, w_amax, accumulate=True)
            wmat = wf
        else:
            if wprep is None:
                absmax(wcat, w_amax, accumulate=True)
            wmat, bf = wcat, None
        if x_amax is None:
            x_amax = absmax(x_prev)
        planes = Z_PLANES and H % PLANE_TILE == 0 and not folded
        # range rows (RangeRows): x_prev is the head of an [N + R, H] buffer whose last R rows are the
        # range sums of x_prev; the GEMM runs on all N + R rows and z_l's extra rows are the range
        # rows' aggregates
        rng = cfg.rng
        x_full = rng.x_full if (rng is not None and rng.x_full is not None and not folded and not planes) else None
        if x_full is not None and x_full.data_ptr() != x_prev.data_ptr():
            raise RuntimeError("sage_layer: RangeRows.x_full must start at x_prev")
        xa, a_amax_g = (x_full, rng.x_amax) if x_full is not None else (x_prev, x_amax)
        M = xa.size(0)
        # (the folded layer's transform has K = K_in, not H: timed under its own name so the
        # bench's flops per launch are right for every launch it averages)
        with _timed("gemm_fwd_fold" if folded else "gemm_fwd"):
            if planes:   # z = [z_l ; z_r] as two dense [N, H] planes
                z = torch.empty(2, N, H, dtype=torch.float32, device=dev)
                gemm(x_prev, wmat, trans_a=False, trans_b=True, out=Planes(z), a_amax=x_amax, b_amax=w_amax)
                zl, zr, ldz = z[0], z[1], H
            elif (img_f is not None and not folded
                  and _lib.query("bgnn_gemm_w_tile", M, 2 * H, H) == img_f.bn_f):   # pre-split [W_l;W_r]
                z = torch.empty(M, 2 * H, dtype=torch.float32, device=dev)
                _lib.call("bgnn_gemm_f32_w", M, 2 * H, H, xa.data_ptr(), xa.stride(0), img_f.img_f.data_ptr(),
                          img_f.bn_f, z.data_ptr(), 2 * H, None, 0, a_amax_g.data_ptr(), w_amax.data_ptr(), None, None,
                          0, 0.0, 0, _stream())
                zl, zr, ldz = z, z[:, H:], 2 * H
            else:        # interleaved [M, 2H]
                z = gemm(xa, wmat, trans_a=False, trans_b=True, bias=bf, a_amax=a_amax_g, b_amax=w_amax)
                zl, zr, ldz = z, z[:, H:], 2 * H
        hagg = z[N:] if x_full is not None else None
        o = torch.empty(N, H, dtype=torch.float32, device=dev)
        nrm = torch.empty(N, dtype=torch.float32, device=dev)
        slots = _lib.query("bgnn_sage_fwd_slots", graph.fwd.ref())
        bn_part = torch.empty(slots, 2, H, dtype=torch.float32, device=dev)
        part = (torch.empty(graph.fwd.plan.n_chunks * H, dtype=torch.float32, device=dev)
                if graph.fwd.plan.n_chunks else None)
        s = _stream()
        with _timed("sage_fwd"):
            _lib.call("bgnn_sage_fwd", graph.fwd.ref(), zl.data_ptr(), ldz, zr.data_ptr(), ldz, b_l.data_ptr(), H,
                      cfg.reduce, o.data_ptr(), nrm.data_ptr(), bn_part.data_ptr(), _ptr(part), _ptr(hagg),
                      2 * H if hagg is not None else 0, s)
        del z, zl, zr, hagg
        x_next, (scale, shift, mean, invstd) = _glue_fwd(o, bn_part, slots, x_prev, gamma, beta, running_mean,
                                                         running_var, cfg, next_amax, graph)
        ctx.graph = graph
        ctx.cfg = cfg
        ctx.folded = folded
        ctx.wcat_t = wcat_t_pre
        ctx.img_d = img_d if not folded else None
        ctx.set_materialize_grads(False)   # the amax output never gets a gradient: no zero fill for it
        ctx.fold = (w_in, b_in, wf) if folded else None
        ctx.save_for_backward(x_prev, o, nrm, wcat, gamma if gamma is not None else torch.empty(0, device=dev),
                              scale if scale is not None else torch.empty(0, device=dev),
                              shift if shift is not None else torch.empty(0, device=dev),
                              mean if mean is not None else torch.empty(0, device=dev),
                              invstd if invstd is not None else torch.empty(0, device=dev),
                              x_amax, w_amax, dz_amax)
        ctx.mark_non_differentiable(next_amax)
        ctx.pool = pool
        if pool is not None:
            from .ops import spmm_fwd
            pooled, _ = spmm_fwd(pool.fwd, x_next, 1, pool.num_rows)
            return x_next, next_amax, pooled
        return x_next, next_amax

    @staticmethod
    def backward(ctx, g, _g_amax, g_pool=None):
        cfg: LayerConfig = ctx.cfg
        g_rows = None
        if g_pool is not None:   # mean pool: segment gradient / count (bgnn.ops._SegmentReduce.backward)
            seg = ctx.pool
            gp = g_pool.contiguous() / seg.fwd.degree().clamp_min(1).to(g_pool.dtype).unsqueeze(1)
            if g is None and not cfg.skip:
                g, g_rows = gp, seg.index
            else:
                gb = gp.index_select(0, seg.index)
                g = gb if g is None else g + gb
        if g is None:   # (materialize_grads off: the layer output did not reach the loss)
            return (None,) * 16
        x_prev, o, nrm, wcat, gamma, scale, shift, mean, invstd, x_amax, w_amax, dz_amax = ctx.saved_tensors
        graph: Graph = ctx.graph
        g = g.contiguous()
        N, H = o.shape
        planes = DZ_PLANES and H % PLANE_TILE == 0
        dev = o.device
        s = _stream()
        bn = cfg.bn
        dgamma, dbeta, sum_g2, sum_g2xhat = _glue_bwd_stats(g, o, scale, shift, mean, invstd, cfg, g_rows)
        if planes:   # dz = [dz_l ; dh] as two dense [N, H] planes
            dzt = torch.empty(2, N, H, dtype=torch.float32, device=dev)
            dz, dzl, dh, lddz = Planes(dzt), dzt[0], dzt[1], H
        else:
            dz = torch.empty(N, 2 * H, dtype=torch.float32, device=dev)
            dzl, dh, lddz = dz, dz[:, H:], 2 * H
        # skip layers: the dgrad's epilogue adds drop(g) itself (bgnn_gemm_f32_dropadd), so
        # bgnn_sage_bwd_rows does not write the [N, H] skip gradient
        dropadd = (cfg.skip and DGRAD_DROPADD and GEMM_BACKEND == "hip" and DGRAD_WT and not planes
                   and H % 4 == 0 and _lib.query("bgnn_get_tuning", 5) == 2)
        gskip = torch.empty(N, H, dtype=torch.float32, device=dev) if (cfg.skip and not dropadd) else None
        rs = _lib.query("bgnn_rows_slots", N)
        part_db = torch.empty(rs, 2, H, dtype=torch.float32, device=dev)
        # range rows (RangeRows): the transposed range rows' dz_l rows summed by this pass
        bw = graph.bwd
        rb = (cfg.rng is not None and cfg.rng.bwd and not planes and bw.ranges is not None)
        rp = (torch.empty(_lib.query("bgnn_range_partial_bytes", N, H) // 4, dtype=torch.float32, device=dev)
              if rb else None)
        _lib.call("bgnn_sage_bwd_rows", g.data_ptr(), _ptr(g_rows), o.data_ptr(), nrm.data_ptr(),
                  _ptr(scale) if bn else None, _ptr(shift) if bn else None,
                  _ptr(gamma) if (bn and gamma.numel()) else None,
                  _ptr(mean) if bn else None, _ptr(invstd) if bn else None, _ptr(sum_g2), _ptr(sum_g2xhat),
                  float(cfg.p), cfg.seed, int(cfg.skip and not dropadd), N, H, dh.data_ptr(), lddz, _ptr(gskip),
                  part_db.data_ptr(), dz_amax.data_ptr(), graph.fwd.rowptr.data_ptr() if ctx.folded else None,
                  (2 if cfg.reduce == 1 else 1) if ctx.folded else 0, _ptr(bw.ranges) if rb else None,
                  graph.fwd.rowptr.data_ptr() if (rb and cfg.reduce == 1) else None, _ptr(rp), s)
        if rb:   # the super nodes' dz_l rows (and their max |.| into dz_amax)
            _lib.call("bgnn_range_sums_finish", rp.data_ptr(), N, H, bw.ref(), 1, dzl.data_ptr(), lddz, None,
                      dz_amax.data_ptr(), s)
        db2 = torch.empty(2 if ctx.folded else 1, H, dtype=torch.float32, device=dev)
        # sum of dh (db_l) into the last row; folded input transform: the column sums of dz_l = A^T dh
        # into row 0, so that db2 viewed flat is [sum dz_l ; sum dh], the folded layer's dbf
        _lib.call("bgnn_reduce_partials", part_db.data_ptr(), rs, H, db2[-1].data_ptr(),
                  db2[0].data_ptr() if ctx.folded else None, 0, s)
        db, db_zl = db2[-1], (db2[0] if ctx.folded else None)
        # dz_l = A^T dh (transpose CSR; MEAN scales by the target's in-degree)
        part = torch.empty(bw.plan.n_chunks * H, dtype=torch.float32, device=dev) if bw.plan.n_chunks else None
        with _timed("spmm_bwd"):
            _lib.call("bgnn_spmm_bwd", bw.ref(), graph.perm_t.data_ptr(), graph.fwd.rowptr.data_ptr(),
                      dh.data_ptr(), lddz, H, cfg.reduce, dzl.data_ptr(), lddz, _ptr(part),
                      dz_amax.data_ptr(), int(rb), s)
        has_affine = bn and gamma.numel() > 0
        if ctx.folded:
            # x = h W_in^T + b_in folded in: dh = dz Wf; dWf = dz^T h; dbf = column sums of dz;
            # then dWcat = dWf W_in^T + dbf b_in^T (= dz^T x), dW_in = Wcat^T dWf, db_in = Wcat^T dbf
            w_in, b_in, wf = ctx.fold
            wf_t = wf.t().contiguous() if DGRAD_WT else wf
            with _timed("gemm_dgrad_fold"):
                dx = gemm(dz, wf_t, trans_a=False, trans_b=DGRAD_WT, a_amax=dz_amax, b_amax=w_amax)
            fs = cfg.famax
            fa = (fs[0:1], fs[1:2], fs[2:3], fs[3:4], fs[4:5]) if fs is not None else (None,) * 5
            with _timed("gemm_wgrad_fold"):
                dwf = gemm(dz, x_prev, trans_a=True, trans_b=False, a_amax=dz_amax, b_amax=x_amax,
                           c_amax=fa[3])                                                   # [2H, K_in]
            dbf = db2.view(-1)                                                              # Σ dz_l ; Σ dh
            if fs is not None:
                absmax(db2, fa[4], accumulate=True)
            if FOLD_WEIGHTS_TORCH:
                dw = torch.addmm(torch.outer(dbf, b_in), dwf, w_in.t())                    # [2H, H]
                dw_in = torch.mm(wcat.t(), dwf)                                            # [H, K_in]
                db_in = torch.mv(wcat.t(), dbf)                                            # [H]
            else:
                dw = gemm(dwf, w_in.contiguous(), trans_a=False, trans_b=True, a_amax=fa[3],
                          b_amax=fa[1])                                                    # [2H, H]
                dw.add_(torch.outer(dbf, b_in))
                dw_in = gemm(wcat, dwf, trans_a=True, trans_b=False, a_amax=fa[0], b_amax=fa[3])  # [H, K_in]
                db_in = gemm(wcat, dbf.view(-1, 1), trans_a=True, trans_b=False, a_amax=fa[0],
                             b_amax=fa[4]).view(-1)                                        # [H]
            return (dx, None, dw[:H], db, dw[H:], dgamma if has_affine else None, dbeta if has_affine else None,
                    None, None, None, None, None, dw_in, db_in, None, None)
        # dx = dz · Wcat (+ skip gradient);  dWcat = dz^T · x_prev
        # [W_l;W_r] transposed once (2 MB) so the dgrad reads its B operand K-contiguous
        wcat_t = (ctx.wcat_t if ctx.wcat_t is not None else wcat.t().contiguous()) if DGRAD_WT else wcat
        img_d = ctx.img_d if (not planes and DGRAD_WT) else None
        if (img_d is not None and (dropadd or gskip is None)
                and _lib.query("bgnn_gemm_w_tile", N, H, 2 * H) == img_d.bn_d):   # pre-split [W_l;W_r]^T
            dx = torch.empty(N, H, dtype=torch.float32, device=dev)
            with _timed("gemm_dgrad"):
                _lib.call("bgnn_gemm_f32_w", N, H, 2 * H, dz.data_ptr(), lddz, img_d.img_d.data_ptr(), img_d.bn_d,
                          dx.data_ptr(), H, None, 0, dz_amax.data_ptr(), w_amax.data_ptr(), None,
                          g.data_ptr() if dropadd else None, H, float(cfg.p) if dropadd else 0.0,
                          cfg.seed if dropadd else 0, s)
        elif dropadd:
            dx = torch.empty(N, H, dtype=torch.float32, device=dev)
            M_, K_ = N, 2 * H
            ws_bytes = _lib.query("bgnn_gemm_ws_bytes_ex", M_, H, K_, 0, 1, 0)
            ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev) if ws_bytes else None
            with _timed("gemm_dgrad"):
                _lib.call("bgnn_gemm_f32_dropadd", 0, 1, M_, H, K_, dz.data_ptr(), lddz, wcat_t.data_ptr(),
                          wcat_t.stride(0), dx.data_ptr(), H, dz_amax.data_ptr(), w_amax.data_ptr(), g.data_ptr(),
                          H, float(cfg.p), cfg.seed, _ptr(ws), ws_bytes, s)
        elif gskip is not None:
            with _timed("gemm_dgrad"):
                dx = gemm(dz, wcat_t, trans_a=False, trans_b=DGRAD_WT, out=gskip, beta=1.0, a_amax=dz_amax,
                          b_amax=w_amax)
        else:
            with _timed("gemm_dgrad"):
                dx = gemm(dz, wcat_t, trans_a=False, trans_b=DGRAD_WT, a_amax=dz_amax, b_amax=w_amax)
        with _timed("gemm_wgrad"):
            dw = gemm(dz, x_prev, trans_a=True, trans_b=False, a_amax=dz_amax, b_amax=x_amax)  # [2H, H]
        dw_l, dw_r = dw[:H], dw[H:]
        return (dx, None, dw_l, db, dw_r, dgamma if has_affine else None, dbeta if has_affine else None,
                None, None, None, None, None, None, None, None, None)


def _max_transform(x, w_l, w_r, graph: Graph, x_amax, w_amax, name: str):
    """Aggregate-first SAGEConv(aggr='max') transform (max is not linear, so the transform-first
    algebra of the sum / mean layers does not apply):
        agg = max_{j->i} x_j                 bgnn_spmm_fwd(MAX) with the per-element CSR argmax
        y   = [agg | x] [W_l | W_r]^T        one f16x3 GEMM, K = 2 C_in, [agg | x] read in place
    max|[agg | x]| = max|x| (every agg element is an x element or 0), so x's maximum scales A.
    Returns (y, agg, arg)."""
    from .ops import spmm_fwd
    N, C = x.shape
    with _timed("agg_max"):
        agg, arg = spmm_fwd(graph.fwd, x, 2, N, want_arg=True)
    wk = torch.cat([w_l, w_r], 1)                                    # [H, 2C]
    in_place = C % 32 == 0 and (x.data_ptr() - agg.data_ptr()) % 16 == 0
    a = Pair(agg, x) if in_place else torch.cat([agg, x], 1)
    with _timed(name):
        y = gemm(a, wk, trans_a=False, trans_b=True, a_amax=x_amax, b_amax=w_amax)
    return y, agg, arg


def _max_rows_fwd(y, b_l, H: int):
    """o = normalize(y + b_l), its row norms and the BatchNorm partial sums of o: bgnn_sage_fwd
    over a CSR without entries (graph.empty_csr), i.e. the SAGE row epilogue alone (the same
    arithmetic as the fused sum / mean layers' epilogue)."""
    from .graph import empty_csr
    N = y.size(0)
    dev = y.device
    csr = empty_csr(N, dev)
    bias = b_l if b_l is not None else torch.zeros(H, dtype=torch.float32, device=dev)
    o = torch.empty(N, H, dtype=torch.float32, device=dev)
    nrm = torch.empty(N, dtype=torch.float32, device=dev)
    slots = _lib.query("bgnn_sage_fwd_slots", csr.ref())
    bn_part = torch.empty(slots, 2, H, dtype=torch.float32, device=dev)
    _lib.call("bgnn_sage_fwd", csr.ref(), y.data_ptr(), y.stride(0), y.data_ptr(), y.stride(0), bias.data_ptr(), H,
              0, o.data_ptr(), nrm.data_ptr(), bn_part.data_ptr(), None, None, 0, _stream())
    return o, nrm, bn_part, slots


def _max_backward(dh, dz_amax, wcat_t, x, agg, arg, graph: Graph, x_amax, w_amax, addend_beta_src,
                  need_dx: bool, p: float = 0.0, seed: int = 0):
    """Backward of y = [agg | x] [W_l | W_r]^T with agg = max-aggregate(x), given dh = dL/dy:
        dagg = dh W_l, then dx = A_max^T dagg + (dh W_r [+ drop(g)])   (bgnn_spmm_bwd_max: the
             gradient of each (target, column) goes to its argmax edge's source, CSR-first on ties)
        dW_l = dh^T agg,  dW_r = dh^T x
    wcat_t = [W_l ; W_r]^T ([C, 2H]); addend_beta_src: the skip connection's incoming gradient g
    (added through its dropout mask in the dW_r product's epilogue) or None."""
    N, H = dh.shape
    C = x.size(1)
    dev = dh.device
    dx = None
    hip16 = GEMM_BACKEND == "hip" and _lib.query("bgnn_get_tuning", 5) == 2
    if need_dx and MAX_MERGED and hip16 and C % 256 == 0:
        # one GEMM [dagg | t] = dh [W_l | W_r] (B^T = [W_l^T ; W_r^T], [2C, H]), the skip layers'
        # drop(g) added to the t columns only (bgnn_gemm_f32_dropadd_cols): one launch at N = 2C
        # instead of two at N = C
        wkt = torch.cat([wcat_t[:, :H], wcat_t[:, H:]], 0)          # [W_l^T ; W_r^T]
        with _timed("gemm_dgrad"):
            dt = torch.empty(N, 2 * C, dtype=torch.float32, device=dev)
            if addend_beta_src is not None:
                ws_bytes = _lib.query("bgnn_gemm_ws_bytes_ex", N, 2 * C, H, 0, 1, 0)
                ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev) if ws_bytes else None
                _lib.call("bgnn_gemm_f32_dropadd_cols", N, 2 * C, H, dh.data_ptr(), dh.stride(0), wkt.data_ptr(), H,
                          dt.data_ptr(), 2 * C, dz_amax.data_ptr(), w_amax.data_ptr(), addend_beta_src.data_ptr(),
                          addend_beta_src.stride(0), C, float(p), seed, _ptr(ws), ws_bytes, _stream())
            else:
                gemm(dh, wkt, trans_a=False, trans_b=True, out=dt, a_amax=dz_amax, b_amax=w_amax)
        dagg, t = dt[:, :C], dt[:, C:]
        dx = torch.empty(N, C, dtype=torch.float32, device=dev)
        bw = graph.bwd
        part = torch.empty(bw.plan.n_chunks * C, dtype=torch.float32, device=dev) if bw.plan.n_chunks else None
        with _timed("spmm_bwd"):
            _lib.call("bgnn_spmm_bwd_max", bw.ref(), graph.perm_t.data_ptr(), graph.fwd.rowptr.data_ptr(), N,
                      dagg.data_ptr(), 2 * C, C, arg.data_ptr(), t.data_ptr(), 2 * C,
                      dx.data_ptr(), dx.stride(0), _ptr(part), None, _stream())
        del dt, dagg, t
    elif need_dx:
        wl_t, wr_t = wcat_t[:, :H], wcat_t[:, H:]                    # W_l^T, W_r^T: [C, H], ld 2H
        with _timed("gemm_dgrad"):
            dagg = gemm(dh, wl_t, trans_a=False, trans_b=True, a_amax=dz_amax, b_amax=w_amax)
            if addend_beta_src is not None and hip16:
                t = torch.empty(N, wcat_t.size(0), dtype=torch.float32, device=dev)
                ws_bytes = _lib.query("bgnn_gemm_ws_bytes_ex", N, t.size(1), H, 0, 1, 0)
                ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev) if ws_bytes else None
                _lib.call("bgnn_gemm_f32_dropadd", 0, 1, N, t.size(1), H, dh.data_ptr(), dh.stride(0),
                          wr_t.data_ptr(), wr_t.stride(0), t.data_ptr(), t.stride(0), dz_amax.data_ptr(),
                          w_amax.data_ptr(), addend_beta_src.data_ptr(), addend_beta_src.stride(0), float(p), seed,
                          _ptr(ws), ws_bytes, _stream())
            else:
                t = gemm(dh, wr_t, trans_a=False, trans_b=True, a_amax=dz_amax, b_amax=w_amax)
                if addend_beta_src is not None:   # (torch GEMM backend / other GEMM modes: an explicit add)
                    t.add_(_dropped(addend_beta_src, p, seed))
        dx = torch.empty(N, x.size(1), dtype=torch.float32, device=dev)
        bw = graph.bwd
        part = torch.empty(bw.plan.n_chunks * x.size(1), dtype=torch.float32, device=dev) if bw.plan.n_chunks else None
        with _timed("spmm_bwd"):
            _lib.call("bgnn_spmm_bwd_max", bw.ref(), graph.perm_t.data_ptr(), graph.fwd.rowptr.data_ptr(), N,
                      dagg.data_ptr(), dagg.stride(0), x.size(1), arg.data_ptr(), t.data_ptr(), t.stride(0),
                      dx.data_ptr(), dx.stride(0), _ptr(part), None, _stream())
    with _timed("gemm_wgrad"):
        if (MAX_MERGED and GEMM_BACKEND == "hip" and C % 256 == 0 and agg.shape == x.shape
                and agg.stride() == x.stride() and (x.data_ptr() - agg.data_ptr()) % 16 == 0):
            # [dW_l^T ; dW_r^T] = [agg | x]^T dh in one GEMM ([agg | x] read in place as two planes
            # of the M dimension; max|[agg | x]| = max|x|)
            dwt = gemm(Pair(agg, x), dh, trans_a=True, trans_b=False, a_amax=x_amax, b_amax=dz_amax)   # [2C, H]
            dw_l, dw_r = dwt[:C].t(), dwt[C:].t()
        else:
            dw_l = gemm(dh, agg, trans_a=True, trans_b=False, a_amax=dz_amax, b_amax=x_amax)
            dw_r = gemm(dh, x, trans_a=True, trans_b=False, a_amax=dz_amax, b_amax=x_amax)
    return dx, dw_l, dw_r


def _dropped(g, p: float, seed: int):
    """drop(g) with the layer's counter-based mask (bgnn_add_dropout with a zero addend): the skip
    gradient for the GEMM modes without the drop-add epilogue."""
    out = torch.empty_like(g)
    _lib.call("bgnn_add_dropout", g.data_ptr(), None, g.numel(), float(p), seed, out.data_ptr(), _stream())
    return out


class SageMaxLayerFn(torch.autograd.Function):
    """The fused layer of GraphSage_maxAggr (Models/BuckGNN.py:165-180,459-471): SAGEConv(aggr='max',
    normalize=True) -> BatchNorm -> ReLU -> skip -> Dropout, aggregate-first (_max_transform), then
    the same row epilogue and glue kernels as the sum / mean layers. Outputs (x_next, max|x_next|)."""

    @staticmethod
    def forward(ctx, x_prev, x_amax, w_l, b_l, w_r, gamma, beta, running_mean, running_var, graph: Graph,
                cfg: LayerConfig, amax=None, wprep=None):
        dev = x_prev.device
        x_prev = x_prev.contiguous()
        H = w_l.size(0)
        if amax is None:
            amax = torch.zeros(3, dtype=torch.float32, device=dev)
        w_amax, next_amax, dz_amax = amax[0:1], amax[1:2], amax[2:3]
        if wprep is not None:   # (prepare_weights has folded max|[W_l;W_r]| into the slot)
            w0, w1 = (wprep.wcat, wprep.wcat_t) if isinstance(wprep, WPrep) else wprep
            wcat_t = w1 if w1 is not None else w0.t().contiguous()
        else:
            wcat_t = torch.cat([w_l, w_r], 0).t().contiguous()
            absmax(wcat_t, w_amax, accumulate=True)
        if x_amax is None:
            x_amax = absmax(x_prev)
        y, agg, arg = _max_transform(x_prev, w_l, w_r, graph, x_amax, w_amax, "gemm_fwd_max")
        with _timed("sage_fwd"):
            o, nrm, bn_part, slots = _max_rows_fwd(y, b_l, H)
        del y
        x_next, (scale, shift, mean, invstd) = _glue_fwd(o, bn_part, slots, x_prev, gamma, beta, running_mean,
                                                         running_var, cfg, next_amax)
        ctx.graph = graph
        ctx.cfg = cfg
        ctx.set_materialize_grads(False)
        e = torch.empty(0, device=dev)
        ctx.save_for_backward(x_prev, agg, arg, o, nrm, wcat_t, gamma if gamma is not None else e,
                              scale if scale is not None else e, shift if shift is not None else e,
                              mean if mean is not None else e, invstd if invstd is not None else e,
                              x_amax, w_amax, dz_amax)
        ctx.mark_non_differentiable(next_amax)
        return x_next, next_amax

    @staticmethod
    def backward(ctx, g, _g_amax):
        if g is None:
            return (None,) * 13
        (x_prev, agg, arg, o, nrm, wcat_t, gamma, scale, shift, mean, invstd, x_amax, w_amax,
         dz_amax) = ctx.saved_tensors
        cfg: LayerConfig = ctx.cfg
        g = g.contiguous()
        N, H = o.shape
        dev = o.device
        s = _stream()
        bn = cfg.bn
        dgamma, dbeta, sum_g2, sum_g2xhat = _glue_bwd_stats(g, o, scale, shift, mean, invstd, cfg)
        dh = torch.empty(N, H, dtype=torch.float32, device=dev)
        rs = _lib.query("bgnn_rows_slots", N)
        part_db = torch.empty(rs, 2, H, dtype=torch.float32, device=dev)
        _lib.call("bgnn_sage_bwd_rows", g.data_ptr(), None, o.data_ptr(), nrm.data_ptr(),
                  _ptr(scale) if bn else None, _ptr(shift) if bn else None,
                  _ptr(gamma) if (bn and gamma.numel()) else None,
                  _ptr(mean) if bn else None, _ptr(invstd) if bn else None, _ptr(sum_g2), _ptr(sum_g2xhat),
                  float(cfg.p), cfg.seed, 0, N, H, dh.data_ptr(), H, None, part_db.data_ptr(), dz_amax.data_ptr(),
                  None, 0, None, None, None, s)
        db = torch.empty(H, dtype=torch.float32, device=dev)
        _lib.call("bgnn_reduce_partials", part_db.data_ptr(), rs, H, db.data_ptr(), None, 0, s)
        dx, dw_l, dw_r = _max_backward(dh, dz_amax, wcat_t, x_prev, agg, arg, ctx.graph, x_amax, w_amax,
                                       g if cfg.skip else None, ctx.needs_input_grad[0], cfg.p, cfg.seed)
        has_affine = bn and gamma.numel() > 0
        return (dx, None, dw_l, db, dw_r, dgamma if has_affine else None, dbeta if has_affine else None,
                None, None, None, None, None, None)


def _weight_pack(pairs, L: int, H: int):
    """[L, 2H, H] / [L, H, 2H] buffers holding one layer loop's [W_l;W_r] (and its transpose),
    filled by one multi-tensor copy and one transpose on every call (~20 us of GPU time per
    step; a fresh torch.cat of the 2L weights each step blocked the host ~0.4 ms,
    tools/host_profile.py). Every call packs into NEW buffers, never into ones a live autograd
    graph may have saved, so a second forward before the first backward (two micro-batches, an
    eval forward in between) keeps the first graph's operands intact. (Round 4 reused the pack
    while the weights' data pointers and autograd versions were unchanged; round-4 ADVICE: a
    freed model's addresses can be handed to a new model with equal versions, and writes through
    p.data bump no version, so a reused pack could be stale. Refilling costs nothing measurable.)"""
    dev = pairs[0][0].device
    W = torch.empty(L, 2 * H, H, dtype=torch.float32, device=dev)
    Wt = torch.empty(L, H, 2 * H, dtype=torch.float32, device=dev) if DGRAD_WT else None
    torch._foreach_copy_([W[i, k * H:(k + 1) * H] for i in range(L) for k in (0, 1)], [t for pr in pairs for t in pr])
    if Wt is not None:
        Wt.copy_(W.transpose(1, 2))
    return W, Wt


class WPrep:
    """One layer's prepared weight operands (prepare_weights): [W_l;W_r] [2H, H], its transpose
    [H, 2H] (dgrad B operand), and optionally their pre-split images (fwd: img_f with column tile
    bn_f; dgrad: img_d, bn_d) for bgnn_gemm_f32_w."""
    __slots__ = ("wcat", "wcat_t", "img_f", "bn_f", "img_d", "bn_d")

    def __init__(self, wcat, wcat_t, img_f=None, bn_f=0, img_d=None, bn_d=0):
        self.wcat, self.wcat_t = wcat, wcat_t
        self.img_f, self.bn_f, self.img_d, self.bn_d = img_f, bn_f, img_d, bn_d


def _wsplit_run(W, i, j, amax_bufs, M):
    """Pre-split images of W[i:j] ([n, N, K] fp32 contiguous, the B^T operands of C = A W^T with
    M rows) in one launch, each scaled by its layer's max|W| (amax_bufs[k, 0]); (images, bn) or
    (None, 0) when the shape has no pre-split path."""
    _, N, K = W.shape
    bn = _lib.query("bgnn_gemm_w_tile", M, N, K)
    if bn == 0:
        return None, 0
    nb = _lib.query("bgnn_gemm_wsplit_bytes", N, K)
    img = torch.empty(j - i, nb, dtype=torch.uint8, device=W.device)
    _lib.call("bgnn_gemm_wsplit", W[i].data_ptr(), j - i, W.stride(0), N, K, W.stride(1), amax_bufs[i].data_ptr(),
              amax_bufs.stride(0), img.data_ptr(), nb, bn, _stream())
    return img, bn


def prepare_weights(pairs, amax_bufs: torch.Tensor, fill_amax, n_rows: int = 0):
    """[W_l;W_r] and its transpose for every layer of a loop in a few launches (one multi-tensor
    copy into a fresh pack, one transpose, one max|W|
    launch per run of layers that take it) instead of three launches per layer. pairs:
    [(w_l, w_r)] per layer; amax_bufs: the loop's zeroed [L, 3] operand-max slots, whose slot 0
    receives max|[W_l;W_r]| for the layers where fill_amax[i] (a folded layer scales by max|Wf|
    instead). Returns [(wcat, wcat_t)] per layer (views of two [L, ...] buffers)."""
    L = len(pairs)
    H = pairs[0][0].size(0)
    with torch.no_grad():   # operands only: the layers return the weight gradients themselves
        if PERSISTENT_WPACK and all(a.dtype == torch.float32 and b.dtype == torch.float32 and a.is_contiguous()
                                    and b.is_contiguous() and a.shape == (H, H) and b.shape == (H, H)
                                    for a, b in pairs):
            W, Wt = _weight_pack(pairs, L, H)
        else:
            W = torch.cat([t for pr in pairs for t in pr], 0).view(L, 2 * H, H)
            Wt = W.transpose(1, 2).contiguous() if DGRAD_WT else None
        # max|W| per layer with bgnn_absmax (torch's dim=(1, 2) max-reduction took 128 us here),
        # one launch per run of consecutive layers that take it (the folded first layer does not)
        i = 0
        while i < L:
            if not fill_amax[i]:
                i += 1
                continue
            j = i
            while j < L and fill_amax[j]:
                j += 1
            if ABSMAX_ITEMS and amax_bufs.is_contiguous() and H % 4 == 0:
                _lib.call("bgnn_absmax_items_f32", W[i].data_ptr(), j - i, 2 * H * H, 2 * H, H, H,
                          amax_bufs[i].data_ptr(), amax_bufs.stride(0), _stream())
            else:
                for k in range(i, j):
                    absmax(W[k], amax_bufs[k, 0:1], accumulate=True)
            i = j
        out = [WPrep(W[i], Wt[i] if Wt is not None else None) for i in range(L)]
        # pre-split images (after the maxima they are scaled by): the layers that scale by
        # max|[W_l;W_r]| (not a folded layer, whose transform is a per-step weight product)
        if (WSPLIT and n_rows > 0 and GEMM_BACKEND == "hip" and Wt is not None and not Z_PLANES and not DZ_PLANES
                and amax_bufs.is_contiguous() and _lib.query("bgnn_get_tuning", 5) == 2):
            i = 0
            while i < L:
                if not fill_amax[i]:
                    i += 1
                    continue
                j = i
                while j < L and fill_amax[j]:
                    j += 1
                img_f, bn_f = _wsplit_run(W, i, j, amax_bufs, n_rows)
                img_d, bn_d = _wsplit_run(Wt, i, j, amax_bufs, n_rows)
                for k in range(i, j):
                    o = out[k]
                    if img_f is not None:
                        o.img_f, o.bn_f = img_f[k - i], bn_f
                    if img_d is not None:
                        o.img_d, o.bn_d = img_d[k - i], bn_d
                i = j
    return out


def sage_layer(x_prev: torch.Tensor, w_l: torch.Tensor, b_l: torch.Tensor, w_r: torch.Tensor,
               bn_module, graph: Graph, reduce: int, skip: bool, p: float, training: bool,
               seed: int, x_amax: torch.Tensor = None, return_amax: bool = False, amax_buf=None,
               w_in: torch.Tensor = None, b_in: torch.Tensor = None, wprep=None, count_batch: bool = True,
               fold_amax: torch.Tensor = None, rng: RangeRows = None, pool=None):
    """Run one fused layer. `bn_module` is a torch.nn.BatchNorm1d (or None for no BN).
    x_amax: optional device scalar >= max|x_prev| (the previous layer's second output), which
    spares the GEMM a pass over x_prev; return_amax: also return max|x_next|.
    w_in / b_in: fold a preceding Linear into this layer (x_prev is then that Linear's INPUT h,
    and the layer computes on x = h W_in^T + b_in without materialising x); only for a layer
    without skip connection (the reference's first SAGE layer after the node encoder).
    rng: the range-row plumbing of a stiffened batch (RangeRows; sum / mean only).
    pool: a SegmentIndex (sum / mean only): also return the mean pool of x_next per segment as the
    last element (SageLayerFn)."""
    require_cuda(x_prev, w_l, b_l, w_r, what="sage_layer")
    H = w_l.size(0)
    if w_in is None and x_prev.size(1) != H:
        raise ValueError(f"sage_layer: x has {x_prev.size(1)} features, the layer {H}")
    if H % 4 or H > 512:
        raise ValueError(f"sage_layer: fused path needs H % 4 == 0 and H <= 512 (got {H})")
    if reduce not in (0, 1, 2):
        raise ValueError("sage_layer: reduce must be 0 (sum), 1 (mean) or 2 (max)")
    if reduce == 2 and w_in is not None:
        raise ValueError("sage_layer: max aggregation needs its input rows (no folded input transform)")
    if reduce == 2 and pool is not None:
        raise ValueError("sage_layer: the fused mean pool is for sum / mean layers")
    if bn_module is not None:
        use_batch_stats = training or not bn_module.track_running_stats
        momentum = bn_module.momentum
        if training and bn_module.track_running_stats:
            if count_batch:
                bn_module.num_batches_tracked.add_(1)
            if momentum is None:   # cumulative average (torch: 1 / num_batches_tracked after the increment;
                # with count_batch=False the caller has already incremented the counter)
                momentum = 1.0 / float(bn_module.num_batches_tracked.item())
        cfg = LayerConfig(reduce, True, use_batch_stats, float(momentum or 0.0) if bn_module.track_running_stats
                          else 0.0, float(bn_module.eps), skip, p, seed)
        cfg.p = p if training else 0.0
        cfg.famax = fold_amax if w_in is not None else None
        cfg.rng = rng if reduce != 2 else None
        if reduce == 2:
            out = SageMaxLayerFn.apply(x_prev, x_amax, w_l, b_l, w_r, bn_module.weight, bn_module.bias,
                                       bn_module.running_mean, bn_module.running_var, graph, cfg, amax_buf, wprep)
        else:
            out = SageLayerFn.apply(x_prev, x_amax, w_l, b_l, w_r, bn_module.weight, bn_module.bias,
                                    bn_module.running_mean, bn_module.running_var, graph, cfg, amax_buf, w_in, b_in,
                                    wprep, pool)
    else:
        cfg = LayerConfig(reduce, False, training, 0.0, 0.0, skip, p, seed)
        cfg.famax = fold_amax if w_in is not None else None
        cfg.rng = rng if reduce != 2 else None
        if reduce == 2:
            out = SageMaxLayerFn.apply(x_prev, x_amax, w_l, b_l, w_r, None, None, None, None, graph, cfg, amax_buf,
                                       wprep)
        else:
            out = SageLayerFn.apply(x_prev, x_amax, w_l, b_l, w_r, None, None, None, None, graph, cfg, amax_buf,
                                    w_in, b_in, wprep, pool)
    if pool is not None:
        return out if return_amax else (out[0], out[2])
    return out if return_amax else out[0]


class SageConvFn(torch.autograd.Function):
    """One SAGEConv(normalize=True, aggr in {add, sum, mean, max}) module on the hand-written path:
    the per-module form of SageLayerFn without the layer glue, for the PyG call surface
    (bgnn.nn.SAGEConv, i.e. the reference's unchanged Models/BuckGNN.py:434 under the shim,
    whose BatchNorm / ReLU / skip / Dropout stay torch modules).

        z = x [W_l;W_r]^T                 f16x3 MFMA GEMM (bgnn_gemm_f32_scaled)
        o = normalize(AGG z_l + z_r + b)  bgnn_sage_fwd (aggregation + bias + L2 normalize)

    backward: bgnn_l2norm_bwd (dh, bias-gradient partials, max|dh|), the transpose aggregation
    dz_l = A^T dh (bgnn_spmm_bwd) and the dgrad / wgrad GEMMs on [dz_l | dh].
    aggr='max' runs aggregate-first (_max_transform / _max_rows_fwd / _max_backward)."""

    @staticmethod
    def forward(ctx, x, w_l, b_l, w_r, graph: Graph, reduce: int):
        dev = x.device
        x = x.contiguous()
        N = x.size(0)
        H = w_l.size(0)
        wcat = torch.cat([w_l, w_r], 0).contiguous()            # [2H, C_in]
        amax = torch.zeros(2, dtype=torch.float32, device=dev)   # max|W|, max|x|
        w_amax, x_amax = amax[0:1], amax[1:2]
        absmax(wcat, w_amax, accumulate=True)
        absmax(x, x_amax, accumulate=True)
        ctx.graph = graph
        ctx.reduce = reduce
        ctx.has_bias = b_l is not None
        if reduce == 2:   # aggregate-first (max is not linear): SageMaxLayerFn's transform + row epilogue
            y, agg, arg = _max_transform(x, w_l, w_r, graph, x_amax, w_amax, "conv_gemm_fwd")
            with _timed("conv_sage_fwd"):
                o, nrm, _, _ = _max_rows_fwd(y, b_l, H)
            ctx.save_for_backward(x, o, nrm, wcat, x_amax, w_amax, agg, arg)
            return o
        with _timed("conv_gemm_fwd"):
            z = gemm(x, wcat, trans_a=False, trans_b=True, a_amax=x_amax, b_amax=w_amax)   # [N, 2H]
        bias = b_l if b_l is not None else torch.zeros(H, dtype=torch.float32, device=dev)
        o = torch.empty(N, H, dtype=torch.float32, device=dev)
        nrm = torch.empty(N, dtype=torch.float32, device=dev)
        slots = _lib.query("bgnn_sage_fwd_slots", graph.fwd.ref())
        bn_part = torch.empty(slots, 2, H, dtype=torch.float32, device=dev)   # (BN sums: unused here)
        part = (torch.empty(graph.fwd.plan.n_chunks * H, dtype=torch.float32, device=dev)
                if graph.fwd.plan.n_chunks else None)
        with _timed("conv_sage_fwd"):
            _lib.call("bgnn_sage_fwd", graph.fwd.ref(), z.data_ptr(), 2 * H, z[:, H:].data_ptr(), 2 * H,
                      bias.data_ptr(), H, reduce, o.data_ptr(), nrm.data_ptr(), bn_part.data_ptr(), _ptr(part),
                      None, 0, _stream())
        ctx.save_for_backward(x, o, nrm, wcat, x_amax, w_amax)
        return o

    @staticmethod
    def backward(ctx, g):
        x, o, nrm, wcat, x_amax, w_amax = ctx.saved_tensors[:6]
        graph: Graph = ctx.graph
        g = g.contiguous()
        N, H = o.shape
        dev = o.device
        s = _stream()
        mx = ctx.reduce == 2
        # max aggregation: dh alone ([N, H]); sum / mean: dz = [dz_l | dh] for the K = 2H GEMMs
        dz = torch.empty(N, H if mx else 2 * H, dtype=torch.float32, device=dev)
        dh = dz if mx else dz[:, H:]
        rs = _lib.query("bgnn_rows_slots", N)
        part_db = torch.empty(rs, 2, H, dtype=torch.float32, device=dev)
        dz_amax = torch.zeros(1, dtype=torch.float32, device=dev)   # max|dz| (fresh: re-entrant backward)
        _lib.call("bgnn_l2norm_bwd", g.data_ptr(), o.data_ptr(), nrm.data_ptr(), N, H, dh.data_ptr(), dh.stride(0),
                  part_db.data_ptr(), dz_amax.data_ptr(), s)
        db = None
        if ctx.has_bias and ctx.needs_input_grad[2]:
            db = torch.empty(H, dtype=torch.float32, device=dev)
            _lib.call("bgnn_reduce_partials", part_db.data_ptr(), rs, H, db.data_ptr(), None, 0, s)
        if mx:
            agg, arg = ctx.saved_tensors[6:]
            dx, dw_l, dw_r = _max_backward(dh, dz_amax, wcat.t().contiguous(), x, agg, arg, graph, x_amax, w_amax,
                                           None, ctx.needs_input_grad[0])
            return dx, dw_l, db, dw_r, None, None
        bw = graph.bwd
        part = torch.empty(bw.plan.n_chunks * H, dtype=torch.float32, device=dev) if bw.plan.n_chunks else None
        with _timed("conv_spmm_bwd"):
            _lib.call("bgnn_spmm_bwd", bw.ref(), graph.perm_t.data_ptr(), graph.fwd.rowptr.data_ptr(),
                      dh.data_ptr(), 2 * H, H, ctx.reduce, dz.data_ptr(), 2 * H, _ptr(part),
                      dz_amax.data_ptr(), 0, s)
        dx = None
        if ctx.needs_input_grad[0]:
            with _timed("conv_gemm_dgrad"):
                dx = gemm(dz, wcat.t().contiguous(), trans_a=False, trans_b=True, a_amax=dz_amax, b_amax=w_amax)
        dw = None
        if ctx.needs_input_grad[1] or ctx.needs_input_grad[3]:
            with _timed("conv_gemm_wgrad"):
                dw = gemm(dz, x, trans_a=True, trans_b=False, a_amax=dz_amax, b_amax=x_amax)   # [2H, C_in]
        return (dx, None if dw is None else dw[:H], db, None if dw is None else dw[H:], None, None)


def sage_conv(x: torch.Tensor, w_l: torch.Tensor, b_l, w_r: torch.Tensor, graph: Graph, reduce: int):
    """normalize(lin_l(AGG x) + lin_r(x)) of one SAGEConv module on the hand-written path
    (SageConvFn); reduce 0 = sum/add, 1 = mean, 2 = max (aggregate-first)."""
    require_cuda(x, w_l, w_r, what="sage_conv")
    return SageConvFn.apply(x, w_l, b_l, w_r, graph, reduce)
