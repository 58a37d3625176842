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
of BASELINE configs[4]). The gathers, the adds and the ReLU of h1 and m1 run in the GEMM
epilogue (bgnn_gemm_gather_add); their backward and the scatter_mean are deterministic bgnn
segment reductions over the edge index (no atomics).
"""
from __future__ import annotations

import torch

from . import _lib
from . import fused
from .fused import Pair, Planes, b16_weight, gemm, gemm_bf16, linear, linear_bf16, mlp, relu_bias_grad
from .graph import SegmentIndex, _index_cache, _stream
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
            g = torch.ops.aten.threshold_backward(g, out, 0.0)   # one pass: g where out > 0
        d1 = segment_reduce(g, ctx.seg1, "sum")
        d2 = segment_reduce(g, ctx.seg2, "sum") if ctx.has2 else None
        return g, d1, None, d2, None, None


def gather_add(a, p1, seg1, p2=None, seg2=None, relu=False):
    return _GatherAdd.apply(a, p1, seg1, p2, seg2, relu)


class _LinearGatherReLU(torch.autograd.Function):
    """out = ReLU(e W^T + b + p1[i1] (+ p2[i2])) as ONE bgnn GEMM whose epilogue gathers the
    node rows (bgnn_gemm_gather_add): no [E, H] temporaries for the gathers, the adds or the
    ReLU. Backward: g' = g masked by out > 0; de = g' W, dW = g'^T e, db = sum g', and
    dp1 / dp2 = deterministic segment sums of g' by i1 / i2."""

    @staticmethod
    def forward(ctx, e, W, b, p1, seg1: SegmentIndex, p2, seg2: SegmentIndex, bf16: bool, out_bf16: bool = False,
                slot=None, dp=None):
        e = e.contiguous()
        Wc = W.contiguous()
        M, K = e.shape
        N = Wc.size(0)
        if p1.stride(1) != 1 or (p2 is not None and p2.stride(1) != 1):
            raise ValueError("gather rows must have unit column stride")
        Wg = b16_weight(e, Wc) if bf16 else Wc
        storage = ((1 if e.dtype == torch.bfloat16 else 0) | (2 if Wg.dtype == torch.bfloat16 else 0)
                   | (4 if out_bf16 else 0))
        out = torch.empty(M, N, dtype=torch.bfloat16 if out_bf16 else torch.float32, device=e.device)
        prec = 1 if bf16 else 0
        ws_bytes = _lib.query("bgnn_gemm_ws_bytes_ex", M, N, K, 0, 1, prec)
        ws = torch.empty(ws_bytes, dtype=torch.uint8, device=e.device) if ws_bytes else None
        args = (e.data_ptr(), e.stride(0), Wg.data_ptr(), Wg.stride(0), out.data_ptr(), N,
                None if b is None else b.contiguous().data_ptr(), 1,
                p1.data_ptr(), seg1.index.data_ptr(), p1.stride(0),
                None if p2 is None else p2.data_ptr(), None if p2 is None else seg2.index.data_ptr(),
                0 if p2 is None else p2.stride(0))
        if storage:   # bf16 edge activations (bf16 operands only)
            if not bf16:
                raise ValueError("linear_gather_relu: bf16 storage needs bf16 operands")
            _lib.call("bgnn_gemm_gather_add_bf16", M, N, K, *args, storage, None if ws is None else ws.data_ptr(),
                      ws_bytes, _stream())
        else:
            _lib.call("bgnn_gemm_gather_add", 0, 1, M, N, K, *args, prec, None if ws is None else ws.data_ptr(),
                      ws_bytes, _stream())
        ctx.seg1, ctx.seg2, ctx.has2, ctx.bf16, ctx.has_bias = seg1, seg2, p2 is not None, bf16, b is not None
        ctx.storage = storage
        ctx.slot = slot
        ctx.dp = dp   # (ColGrad, block of p1, block of p2): the segment sums go into its columns
        ctx.save_for_backward(e, W, out)
        return out

    @staticmethod
    def backward(ctx, g):
        e, W, out = ctx.saved_tensors
        if ctx.storage:   # bf16 storage: mask + f32 bias sum in one pass, GEMMs on bgnn_gemm_bf16
            if g.dtype == torch.bfloat16 and fused.BF16_PREP:
                g, db = fused.relu_bias_grad_bf16(g, out, ctx.has_bias)
            else:
                g = torch.ops.aten.threshold_backward(g.contiguous(), out, 0.0)
                db = torch.sum(g, 0, dtype=torch.float32) if ctx.has_bias else None
            de = None
            if ctx.needs_input_grad[0]:
                slot = ctx.slot
                if (slot is not None and slot.armed and GEMM_DROPADD and e.dtype == torch.bfloat16
                        and g.dtype == torch.bfloat16):
                    # + the skip + dropout's share of e's gradient in the dgrad GEMM's epilogue
                    de = slot.gemm_dropadd(g, W)
                else:
                    de = gemm_bf16(g, W.t().contiguous(), False, True, out_bf16=e.dtype == torch.bfloat16)
                    if slot is not None:
                        de = slot.add_to(de)   # + the skip + dropout's share of e's gradient, one pass
            dW = gemm_bf16(g, e, True, False)
            if ctx.dp is not None:
                cg, i1, i2 = ctx.dp
                H = g.size(1)
                d1 = _segment_sum_into(g, ctx.seg1, cg.block(i1, H))
                d2 = _segment_sum_into(g, ctx.seg2, cg.block(i2, H)) if ctx.has2 else None
            else:
                d1 = segment_reduce(g, ctx.seg1, "sum")
                d2 = segment_reduce(g, ctx.seg2, "sum") if ctx.has2 else None
            return de, dW, db, d1, None, d2, None, None, None, None, None
        # ReLU mask, bias gradient and max|g'| (the f16x3 operand scale of both GEMMs) in one pass
        g, db, g_amax = relu_bias_grad(g, out, ctx.has_bias)
        bf16 = ctx.bf16
        if bf16:
            g_amax = None
        de = (gemm(g, W.t().contiguous(), trans_a=False, trans_b=True, a_amax=g_amax, bf16=bf16)
              if ctx.needs_input_grad[0] else None)
        dW = gemm(g, e, trans_a=True, trans_b=False, a_amax=g_amax, bf16=bf16)
        d1 = segment_reduce(g, ctx.seg1, "sum")
        d2 = segment_reduce(g, ctx.seg2, "sum") if ctx.has2 else None
        return de, dW, db, d1, None, d2, None, None, None, None, None


def _segment_sum_into(g: torch.Tensor, seg: SegmentIndex, out: torch.Tensor) -> torch.Tensor:
    """Segment sums of the bf16 rows of g by seg into the f32 view out (a column block of a
    ColGrad buffer): bgnn_segment_sum_bf16 with out's row stride."""
    g = g.contiguous()
    _lib.call("bgnn_segment_sum_bf16", seg.fwd.rowptr.data_ptr(), seg.fwd.col.data_ptr(), seg.num_rows, g.data_ptr(),
              g.stride(0), g.size(1), 0, out.data_ptr(), out.stride(0), _stream())
    return out


def _epilogue_gather_available() -> bool:
    """bgnn_gemm_gather_add runs on the split GEMM family (f16x3 / bf16x6); the f32-MFMA family
    (BGNN_TUNE_GEMM_MODE = 0) and the torch.mm A/B backend take the two-step form."""
    from . import fused
    return fused.GEMM_BACKEND == "hip" and _lib.query("bgnn_get_tuning", 5) != 0


def linear_gather_relu(e, W, b, p1, seg1, p2=None, seg2=None, bf16=False, out_bf16=False, slot=None, dp=None):
    if not _epilogue_gather_available():
        if e.dtype == torch.bfloat16 or out_bf16:
            raise ValueError("linear_gather_relu: bf16 storage needs the epilogue gather (split GEMM family)")
        return gather_add(linear(e, W, b, False, bf16=bf16), p1, seg1, p2, seg2, relu=True)
    return _LinearGatherReLU.apply(e, W, b, p1, seg1, p2, seg2, bf16, out_bf16, slot, dp)


class GradSlot:
    """Hand-off of one edge activation's skip + dropout gradient to the edge Linear that also
    consumes it (EA_GNN bf16 storage, `FUSED_GRAD_ADD`). EA_GNN's block output e' (and, with the
    skip, its input e) feeds both an edge Linear of the block (phi's first Linear; edge_mlp's) and
    `Dropout(e' + e)` (Models/BuckGNN.py:382-387). Autograd would sum the two gradients with an
    add over [E, H] after a dropout pass wrote drop(g); here the skip + dropout's backward leaves g
    in the slot and returns no gradient for e' / e, and the Linear's backward adds drop(g) to its
    input gradient in one pass (bgnn_add_dropped_bf16: the same mask, nothing stored).
    Order: the skip + dropout node is created after the block's Linears, so autograd runs its
    backward first; a consumer that finds the slot armed but empty raises instead of dropping a
    gradient."""
    __slots__ = ("armed", "g", "p", "seed")

    def __init__(self):
        self.armed, self.g, self.p, self.seed = False, None, 0.0, 0

    def _arrived(self):
        if self.g is None:
            raise RuntimeError("GradSlot: the skip + dropout gradient had not arrived when the edge Linear's "
                               "backward ran (autograd order)")
        return self.g

    def gemm_dropadd(self, g: torch.Tensor, W: torch.Tensor) -> torch.Tensor:
        """The consumer Linear's input gradient g W plus drop(slot gradient), both bf16, in one
        launch (bgnn_gemm_bf16_dropadd: the same bits as gemm_bf16 followed by add_to)."""
        src = self._arrived()
        g = g.contiguous()
        M, K = g.shape
        N = W.size(1)
        if src.shape != (M, N) or src.dtype != torch.bfloat16 or not src.is_contiguous():
            raise RuntimeError("GradSlot: gradient shape / dtype mismatch")
        wt = b16_weight(g, W.t().contiguous())   # W^T rounded to bf16 once (the B operand, [N, K])
        if wt.dtype != torch.bfloat16 or K % 64 or N % 8:   # not the LDS-DMA kernel's shapes: two steps
            return self.add_to(gemm_bf16(g, W.t().contiguous(), False, True, out_bf16=True))
        de = torch.empty(M, N, dtype=torch.bfloat16, device=g.device)
        _lib.call("bgnn_gemm_bf16_dropadd", M, N, K, g.data_ptr(), g.stride(0), wt.data_ptr(), wt.stride(0),
                  de.data_ptr(), N, src.data_ptr(), N, float(self.p), self.seed, _stream())
        return de

    def add_to(self, de: torch.Tensor) -> torch.Tensor:
        if not self.armed:
            return de
        self._arrived()
        de = de.contiguous()
        g = self.g
        if g.shape != de.shape or g.dtype != torch.bfloat16 or de.dtype != torch.bfloat16:
            raise RuntimeError("GradSlot: gradient shape / dtype mismatch")
        _lib.call("bgnn_add_dropped_bf16", de.data_ptr(), g.data_ptr(), de.numel(), float(self.p), self.seed,
                  de.data_ptr(), _stream())
        return de


class _SkipDropoutToSlot(torch.autograd.Function):
    """drop(a + b) like _SkipDropout, whose backward hands g to `slot` (see GradSlot) instead of
    returning drop(g) for a and b."""

    @staticmethod
    def forward(ctx, a, b, p: float, seed: int, slot: GradSlot):
        ctx.slot = slot
        slot.armed, slot.g, slot.p, slot.seed = True, None, p, seed
        return _add_dropout(a, b, p, seed)

    @staticmethod
    def backward(ctx, g):
        ctx.slot.g = g.contiguous()
        return None, None, None, None, None


class ColGrad:
    """One [N, k*H] f32 gradient buffer shared by the k column blocks of P (_ColumnBlocks): the
    consumers' backward writes each block's segment sums straight into its columns (one block each),
    so _ColumnBlocks' backward returns the buffer instead of concatenating k [N, H] gradients (EA_GNN
    cfg5: a 2 GB copy per block per step)."""
    __slots__ = ("shape", "device", "buf")

    def __init__(self, shape, device):
        self.shape, self.device, self.buf = shape, device, None

    def block(self, i: int, H: int) -> torch.Tensor:
        if self.buf is None:
            self.buf = torch.empty(self.shape, dtype=torch.float32, device=self.device)
        return self.buf[:, i * H:(i + 1) * H]


class _ColumnBlocks(torch.autograd.Function):
    """Split [N, k*H] into k column views whose backward is ONE concatenation of the k
    gradients (autograd's slice backward would zero-fill and add k full [N, k*H] buffers), or no
    copy at all when the k gradients are the blocks of the layer's ColGrad buffer."""

    @staticmethod
    def forward(ctx, P, k: int, cg=None):
        ctx.k, ctx.cg = k, cg
        ctx.set_materialize_grads(False)   # unused blocks arrive as None: no zero-filled buffers
        H = P.size(1) // k
        return tuple(P[:, i * H:(i + 1) * H] for i in range(k))

    @staticmethod
    def backward(ctx, *gs):
        ref = next((g for g in gs if g is not None), None)
        if ref is None:
            return None, None, None
        cg = ctx.cg
        if cg is not None and cg.buf is not None:
            H = cg.buf.size(1) // ctx.k
            if all(g is not None and g.data_ptr() == cg.buf[:, i * H:].data_ptr() and g.stride() == cg.buf.stride()
                   for i, g in enumerate(gs)):
                buf, cg.buf = cg.buf, None
                return buf, None, None
        gs = [torch.zeros_like(ref) if g is None else g for g in gs]
        return torch.cat(gs, 1), None, None


class _PairLinear(torch.autograd.Function):
    """act([x | agg] W^T + b) with bf16 operands for node_mlp_gamma's first Linear
    (Models/BuckGNN.py:560, `node_mlp_gamma(torch.cat([x, agg], 1))`), [x | agg] read in place as
    two planes of the GEMM's A operand (fused.Pair) instead of a [N, 2H] torch.cat; backward: the
    ReLU mask and bias sum (relu_bias_grad), [dx | dagg] = g' W written as two planes (each a dense
    [N, H] gradient, no slicing of a [N, 2H] one), dW = ([x | agg]^T g')^T. The forward and dx / dagg
    are the bits of LinearFn on the concatenation (the bf16 tiles all sum in increasing k); dW is
    the transposed product (its split-K grouping may differ: rounding-equal)."""

    @staticmethod
    def forward(ctx, x, agg, weight, bias, relu: bool):
        y = gemm(Pair(x, agg), weight.contiguous(), trans_a=False, trans_b=True, bias=bias, relu=relu, bf16=True)
        ctx.relu, ctx.has_bias = relu, bias is not None
        ctx.save_for_backward(x, agg, weight, y if relu else torch.empty(0, device=x.device))
        return y

    @staticmethod
    def backward(ctx, g):
        x, agg, weight, y = ctx.saved_tensors
        g, db, _ = relu_bias_grad(g, y if ctx.relu else None, ctx.has_bias)
        dx = dagg = None
        if ctx.needs_input_grad[0] or ctx.needs_input_grad[1]:
            N, H = x.shape
            t = torch.empty(2, N, H, dtype=torch.float32, device=x.device)
            gemm(g, weight.t().contiguous(), trans_a=False, trans_b=True, out=Planes(t), bf16=True)
            dx, dagg = t[0], t[1]
        dwt = gemm(Pair(x, agg), g, trans_a=True, trans_b=False, bf16=True)   # [2H, H_out]
        return dx, dagg, dwt.t(), db, None


def _gamma_mlp(seq: torch.nn.Sequential, x: torch.Tensor, agg: torch.Tensor) -> torch.Tensor:
    """node_mlp_gamma([x | agg]) in bf16 operands: the first Linear on the two planes (_PairLinear)
    when the halves qualify, the rest through fused.mlp; else mlp over torch.cat."""
    mods = list(seq)
    ok = (PAIR_GAMMA and fused.GEMM_BACKEND == "hip" and len(mods) >= 1 and isinstance(mods[0], torch.nn.Linear)
          and x.shape == agg.shape and x.dtype == agg.dtype == torch.float32 and x.is_contiguous()
          and agg.is_contiguous() and x.size(1) % 256 == 0 and (agg.data_ptr() - x.data_ptr()) % 16 == 0)
    if not ok:
        return mlp(seq, torch.cat([x, agg], 1), bf16=True)
    relu = len(mods) > 1 and isinstance(mods[1], torch.nn.ReLU)
    h = _PairLinear.apply(x, agg, mods[0].weight, mods[0].bias, relu)
    rest = mods[2 if relu else 1:]
    return mlp(torch.nn.Sequential(*rest), h, bf16=True) if rest else h


_IDENTITY = {}


def _identity_index(n: int, device) -> torch.Tensor:
    """arange(n) as a view of one per-device arange sized to the largest n seen (batches have varying
    node counts: a cache keyed by n would grow without bound)."""
    key = str(device)
    t = _IDENTITY.get(key)
    if t is None or t.numel() < n:
        t = _IDENTITY[key] = torch.arange(max(n, 1), dtype=torch.int64, device=device)
    return t[:n]


class _LinearResidual(torch.autograd.Function):
    """r + (h W^T + b) with bf16 operands as ONE GEMM whose epilogue adds row r[i] to output row i
    (bgnn_gemm_gather_add with the identity index): node_mlp_beta's last Linear and the residual
    `out + node_mlp_beta(out)` (Models/BuckGNN.py:561), the bits of LinearFn followed by torch's add
    (the epilogue adds bias, then the row) without the [N, H] add pass. Backward: LinearFn's
    (relu_bias_grad for the bias sum, dgrad and wgrad GEMMs), and g itself for r."""

    @staticmethod
    def forward(ctx, h, weight, bias, r):
        h = h.contiguous()
        M, K = h.shape
        N = weight.size(0)
        W = weight.contiguous()
        out = torch.empty(M, N, dtype=torch.float32, device=h.device)
        idx = _identity_index(M, h.device)
        ws_bytes = _lib.query("bgnn_gemm_ws_bytes_ex", M, N, K, 0, 1, 1)
        ws = torch.empty(ws_bytes, dtype=torch.uint8, device=h.device) if ws_bytes else None
        _lib.call("bgnn_gemm_gather_add", 0, 1, M, N, K, h.data_ptr(), h.stride(0), W.data_ptr(), W.stride(0),
                  out.data_ptr(), N, None if bias is None else bias.contiguous().data_ptr(), 0,
                  r.data_ptr(), idx.data_ptr(), r.stride(0), None, None, 0, 1,
                  None if ws is None else ws.data_ptr(), ws_bytes, _stream())
        ctx.has_bias = bias is not None
        ctx.save_for_backward(h, weight)
        return out

    @staticmethod
    def backward(ctx, g):
        h, weight = ctx.saved_tensors
        gg, db, _ = relu_bias_grad(g, None, ctx.has_bias)
        dh = gemm(gg, weight.t().contiguous(), trans_a=False, trans_b=True, bf16=True) if ctx.needs_input_grad[0] else None
        dw = gemm(gg, h, trans_a=True, trans_b=False, bf16=True)
        return dh, dw, db, g


def _beta_residual(seq: torch.nn.Sequential, out: torch.Tensor) -> torch.Tensor:
    """out + node_mlp_beta(out) in bf16 operands: the last Linear and the add as one GEMM
    (_LinearResidual) when it qualifies, else fused.mlp and torch's add."""
    mods = list(seq)
    ok = (RESIDUAL_EPILOGUE and fused.GEMM_BACKEND == "hip" and _epilogue_gather_available() and len(mods) >= 1
          and isinstance(mods[-1], torch.nn.Linear) and out.dtype == torch.float32 and out.is_contiguous()
          and out.size(1) == mods[-1].weight.size(0) and out.size(1) % 4 == 0 and out.data_ptr() % 16 == 0)
    if not ok:
        return out + mlp(seq, out, bf16=True)
    h = mlp(torch.nn.Sequential(*mods[:-1]), out, bf16=True) if len(mods) > 1 else out
    return _LinearResidual.apply(h, mods[-1].weight, mods[-1].bias, out)


# the two-step form (linear, then _GatherAdd) is kept for A/B measurement
FUSED_GATHER = True
# bf16 storage: node_mlp_beta's last Linear adds the residual in its epilogue (no [N, H] add pass).
# Off: measured equal to the separate add (cfg5 204.0-204.7 either way, tools/ab_ea_residual.sh,
# profiles/r05_ab_ea_residual.txt) -- the gathered-row epilogue costs what the add pass did
RESIDUAL_EPILOGUE = False
# bf16 storage: node_mlp_gamma's first Linear reads [x | agg] as two GEMM planes (no torch.cat)
PAIR_GAMMA = True
# bf16 storage: the P column blocks' gradients written into one shared buffer (ColGrad, A/B switch)
COLGRAD = True
# EA_GNN's skip add + dropout over [E, H] / [N, H] as one pass (bgnn_add_dropout)
FUSED_SKIP_DROPOUT = True
# bf16 configuration (model.ea_bf16): the per-edge activations (edge encoder output, h1, e',
# m1, messages and their gradients) are STORED in bf16 as well, like torch autocast's bf16
# Linear outputs; node-level tensors, weights and their gradients stay f32. False = bf16
# operands with f32 storage (round-2 form, A/B)
BF16_STORAGE = True
# bf16 storage: the two gradients of every edge activation (an edge Linear's input gradient and the
# skip + dropout's) summed by the Linear's backward in one pass (GradSlot) instead of autograd's add
FUSED_GRAD_ADD = True
# ... and that sum in the dgrad GEMM's epilogue (bgnn_gemm_bf16_dropadd) instead of a pass over the
# GEMM's stored output (A/B switch; the same bits)
GEMM_DROPADD = True


def _add_dropout(a: torch.Tensor, b, p: float, seed: int) -> torch.Tensor:
    out = torch.empty_like(a)
    fn = "bgnn_add_dropout_bf16" if a.dtype == torch.bfloat16 else "bgnn_add_dropout"
    _lib.call(fn, a.data_ptr(), None if b is None else b.data_ptr(), a.numel(), float(p), seed, out.data_ptr(),
              _stream())
    return out


class _SkipDropout(torch.autograd.Function):
    """drop(a + b) with the counter-based mask (nothing stored); backward drop(g) to both."""

    @staticmethod
    def forward(ctx, a, b, p: float, seed: int):
        ctx.p, ctx.seed, ctx.has_b = p, seed, b is not None
        return _add_dropout(a, b, p, seed)

    @staticmethod
    def backward(ctx, g):
        gd = _add_dropout(g.contiguous(), None, ctx.p, ctx.seed)
        return gd, (gd if ctx.has_b else None), None, None


def skip_dropout(a: torch.Tensor, b, p: float, training: bool, seed: int, slot: GradSlot = None) -> torch.Tensor:
    """Dropout_p(a + b) (b may be None) as one pass: Models/BuckGNN.py:382-387. With a slot
    (EA_GNN bf16 storage), the backward hands the gradient to the edge Linears that consume a and b
    (GradSlot) -- only for bf16 a / b, whose consumers were given the same slot."""
    if not training or p == 0.0:
        return a + b if b is not None else a
    ok = (FUSED_SKIP_DROPOUT and a.is_cuda and a.dtype in (torch.float32, torch.bfloat16) and a.is_contiguous()
          and a.numel() % (8 if a.dtype == torch.bfloat16 else 4) == 0 and a.data_ptr() % 16 == 0
          and (b is None or (b.is_contiguous() and b.shape == a.shape and b.dtype == a.dtype
                             and b.data_ptr() % 16 == 0)))
    if not ok:
        return torch.nn.functional.dropout(a + b if b is not None else a, p, True)
    if slot is not None and a.dtype == torch.bfloat16 and FUSED_GRAD_ADD:
        return _SkipDropoutToSlot.apply(a, b, p, seed, slot)
    return _SkipDropout.apply(a, b, p, seed)


def graphnet_block(blk, x: torch.Tensor, e: torch.Tensor, edge_index: torch.Tensor, bf16: bool = False,
                   slot: GradSlot = None, slot_in: bool = False):
    """(x_out, e_out) of one GraphNetBlock `blk` (bgnn.buckgnn.GraphNetBlock: same parameters
    as the reference's) on the bgnn kernels. slot (bf16 storage): the GradSlot the caller passes to
    the skip + dropout of this block's edge output; phi's first Linear (consumer of e_out) adds its
    gradient, and edge_mlp's first Linear (consumer of e) too when slot_in (the skip uses e)."""
    N, H = x.shape
    seg_row, seg_col = edge_segments(edge_index, N)
    W1, b1 = blk.edge_mlp[0].weight, blk.edge_mlp[0].bias
    W2, b2 = blk.edge_mlp[2].weight, blk.edge_mlp[2].bias
    Wp, bp = blk.node_mlp_phi[0].weight, blk.node_mlp_phi[0].bias
    Wp2, bp2 = blk.node_mlp_phi[2].weight, blk.node_mlp_phi[2].bias
    x = x.contiguous()
    # node-level blocks of the two concatenation Linears, one GEMM
    P = linear(x, torch.cat([W1[:, :H], W1[:, H:2 * H], Wp[:, :H]], 0), None, False, bf16=bf16)
    # the four per-edge K = H forward products, timed for the bench's EA_GNN roofline (each reads
    # an [E, H] f32 operand and writes an [E, H] f32 result)
    st = bf16 and BF16_STORAGE and FUSED_GATHER and _epilogue_gather_available() and H % 8 == 0
    cg = ColGrad(P.shape, P.device) if (st and COLGRAD) else None
    P_row, P_col, Q = _ColumnBlocks.apply(P, 3, cg)
    if st:   # bf16 edge activations end to end
        with fused._timed("ea_edge_fwd"):
            h1 = linear_gather_relu(e, W1[:, 2 * H:], b1, P_row, seg_row, P_col, seg_col, bf16=True, out_bf16=True,
                                    slot=slot if slot_in else None, dp=(cg, 0, 1) if cg is not None else None)
        with fused._timed("ea_edge_fwd"):
            e_out = linear_bf16(h1, W2, b2, False, True)
        with fused._timed("ea_edge_fwd"):
            m1 = linear_gather_relu(e_out, Wp[:, H:], bp, Q, seg_col, bf16=True, out_bf16=True, slot=slot,
                                    dp=(cg, 2, None) if cg is not None else None)
        with fused._timed("ea_edge_fwd"):
            msg = linear_bf16(m1, Wp2, bp2, False, True)
        agg = segment_reduce(msg, seg_row, "mean")
        out = _gamma_mlp(blk.node_mlp_gamma, x, agg)
        out = _beta_residual(blk.node_mlp_beta, out)
        return out, e_out
    with fused._timed("ea_edge_fwd"):
        if FUSED_GATHER:
            h1 = linear_gather_relu(e, W1[:, 2 * H:], b1, P_row, seg_row, P_col, seg_col, bf16=bf16)
        else:
            h1 = gather_add(linear(e, W1[:, 2 * H:], b1, False, bf16=bf16), P_row, seg_row, P_col,
                            seg_col, relu=True)
    with fused._timed("ea_edge_fwd"):
        e_out = linear(h1, W2, b2, False, bf16=bf16)
    with fused._timed("ea_edge_fwd"):
        if FUSED_GATHER:
            m1 = linear_gather_relu(e_out, Wp[:, H:], bp, Q, seg_col, bf16=bf16)
        else:
            m1 = gather_add(linear(e_out, Wp[:, H:], bp, False, bf16=bf16), Q, seg_col, relu=True)
    with fused._timed("ea_edge_fwd"):
        msg = linear(m1, Wp2, bp2, False, bf16=bf16)
    agg = segment_reduce(msg, seg_row, "mean")
    out = mlp(blk.node_mlp_gamma, torch.cat([x, agg], 1), bf16=bf16)
    out = out + mlp(blk.node_mlp_beta, out, bf16=bf16)
    return out, e_out
