"""PyG-compatible module / functional surface backed by libbgnn.

Mirrors exactly the parts of torch_geometric / torch_scatter that buck-gnn calls
(Models/BuckGNN.py:3-6, Utils/Losses.py:4):

    SAGEConv(in_channels, out_channels, aggr='mean', normalize=False,
             root_weight=True, project=False, bias=True)      -> forward(x, edge_index)
    global_mean_pool / global_add_pool / global_max_pool(x, batch, size=None)
    scatter_add / scatter_mean / scatter_max(src, index, dim=0, out=None, dim_size=None)

State-dict keys of SAGEConv are PyG's (`lin_l.weight`, `lin_l.bias`, `lin_r.weight`,
plus `lin.*` when project=True), so reference checkpoints load unchanged.
PyG is not installed here and its version is not pinned by the reference
(README.md:64-70); the semantics restated are those of PyG's documented
SAGEConv: out_i = lin_l(AGG_{j->i} x_j) + lin_r(x_i), then F.normalize when
normalize=True, with 'add' == 'sum' and empty neighbourhoods giving 0.
"""
from __future__ import annotations

import math
from typing import Optional, Tuple, Union

import torch
import torch.nn.functional as F
from torch import Tensor, nn

from .graph import graph_for, segments_for
from .ops import REDUCE, aggregate, segment_reduce

# SAGEConv(normalize=True, aggr in {add, sum, mean}) modules run on the hand-written path
# (bgnn.fused.SageConvFn: MFMA transform + fused aggregation/bias/normalize) when the input is
# on the GPU; False = aggregate-first through torch Linear + F.normalize (A/B and tests)
FAST_SAGECONV = True


class Linear(nn.Linear):
    """torch.nn.Linear with PyG's initialisation (kaiming_uniform(a=sqrt(5)) weight,
    uniform(±1/sqrt(in)) bias) — same distribution as nn.Linear's default."""

    def reset_parameters(self) -> None:
        bound_w = math.sqrt(6.0 / ((1 + 5.0) * self.in_features)) if self.in_features > 0 else 0.0
        with torch.no_grad():
            self.weight.uniform_(-bound_w, bound_w)
            if self.bias is not None:
                b = 1.0 / math.sqrt(self.in_features) if self.in_features > 0 else 0.0
                self.bias.uniform_(-b, b)


class SAGEConv(nn.Module):
    """GraphSAGE operator with PyG's constructor, forward and state-dict layout."""

    def __init__(self, in_channels: Union[int, Tuple[int, int]], out_channels: int, aggr: str = "mean",
                 normalize: bool = False, root_weight: bool = True, project: bool = False, bias: bool = True,
                 **kwargs):
        super().__init__()
        if isinstance(in_channels, int):
            in_channels = (in_channels, in_channels)
        if aggr not in REDUCE:
            raise ValueError(f"SAGEConv: unsupported aggr '{aggr}' (supported: {sorted(REDUCE)})")
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.aggr = aggr
        self.normalize = normalize
        self.root_weight = root_weight
        self.project = project
        if project:
            self.lin = Linear(in_channels[0], in_channels[0], bias=True)
        self.lin_l = Linear(in_channels[0], out_channels, bias=bias)
        if root_weight:
            self.lin_r = Linear(in_channels[1], out_channels, bias=False)
        self.reset_parameters()

    def reset_parameters(self) -> None:
        if self.project:
            self.lin.reset_parameters()
        self.lin_l.reset_parameters()
        if self.root_weight:
            self.lin_r.reset_parameters()

    def forward(self, x: Union[Tensor, Tuple[Tensor, Tensor]], edge_index: Tensor, size=None) -> Tensor:
        if size is not None:
            raise NotImplementedError("SAGEConv: bipartite `size` is not supported by bgnn")
        if isinstance(x, Tensor):
            x = (x, x)
        x_src, x_dst = x
        if x_src.size(0) != x_dst.size(0):
            raise NotImplementedError("SAGEConv: bipartite graphs are not supported by bgnn")
        if self.project:
            x_src = F.relu(self.lin(x_src))
        graph = graph_for(edge_index, x_src.size(0))
        if self._fast(x_src, x_dst):
            # the hand-written path: f16x3 MFMA transform [W_l;W_r] + fused aggregation, bias and
            # L2 normalize, with its own backward (bgnn.fused.SageConvFn)
            from .fused import sage_conv
            return sage_conv(x_src, self.lin_l.weight, self.lin_l.bias, self.lin_r.weight, graph,
                             {"mean": 1, "max": 2}.get(self.aggr, 0))
        if self.aggr in ("add", "sum", "mean") and 2 * self.out_channels <= self.in_channels[0]:
            # narrow output (e.g. SAGPooling's 1-channel scorer): transform first, then aggregate
            # the narrow rows -- lin_l(AGG x) = AGG(x W_l^T) + b_l, since sum / mean are linear
            out = aggregate(F.linear(x_src, self.lin_l.weight), graph, self.aggr)
            if self.lin_l.bias is not None:
                out = out + self.lin_l.bias
        else:
            out = self.lin_l(aggregate(x_src, graph, self.aggr))
        if self.root_weight and x_dst is not None:
            out = out + self.lin_r(x_dst)
        if self.normalize:
            out = F.normalize(out, p=2.0, dim=-1)
        return out

    def _fast(self, x_src: Tensor, x_dst: Tensor) -> bool:
        """Whether this call runs on bgnn.fused.SageConvFn: normalize=True, sum/mean/max
        aggregation, root weight, no projection, fp32 CUDA input, out_channels a multiple of
        4 up to 512 and not narrower than half the input (the narrow scorer of SAGPooling
        aggregates its 1-wide transform instead)."""
        return (FAST_SAGECONV and self.normalize and self.root_weight and not self.project
                and self.aggr in ("add", "sum", "mean", "max") and x_src is x_dst and x_src.is_cuda
                and x_src.dtype == torch.float32 and x_src.dim() == 2
                and self.out_channels % 4 == 0 and 4 <= self.out_channels <= 512
                and 2 * self.out_channels > self.in_channels[0] and self.in_channels[0] % 4 == 0
                and self.lin_l.weight.dtype == torch.float32)

    def __repr__(self) -> str:
        return f"{self.__class__.__name__}({self.in_channels[0]}, {self.out_channels}, aggr={self.aggr})"


class _BatchNormFn(torch.autograd.Function):
    """torch.nn.functional.batch_norm over a [N, C] fp32 CUDA activation on libbgnn (csrc/bn.hip):
    train (batch statistics; running stats updated in place by bgnn_bn_finalize) or eval (running
    statistics), forward one stats pass + one apply pass, backward one stats pass + one row pass."""

    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, batch_stats: bool, momentum: float, eps: float):
        from . import _lib
        from .graph import _stream
        x = x.contiguous()
        N, C = x.shape
        dev = x.device
        s = _stream()
        coef = torch.empty(4, C, dtype=torch.float32, device=dev)   # mean, invstd, scale, shift
        mean, invstd, scale, shift = coef[0], coef[1], coef[2], coef[3]
        w = None if weight is None else weight.contiguous()
        b = None if bias is None else bias.contiguous()
        if batch_stats:
            slots = _lib.query("bgnn_bn_slots", N, C)
            part = torch.empty(slots, 2, C, dtype=torch.float32, device=dev)
            _lib.call("bgnn_bn_stats", x.data_ptr(), N, C, part.data_ptr(), s)
            _lib.call("bgnn_bn_finalize_shifted", part.data_ptr(), slots, C, N, x.data_ptr(),
                      None if w is None else w.data_ptr(),
                      None if b is None else b.data_ptr(), float(eps), float(momentum),
                      None if running_mean is None else running_mean.data_ptr(),
                      None if running_var is None else running_var.data_ptr(), mean.data_ptr(), invstd.data_ptr(),
                      scale.data_ptr(), shift.data_ptr(), s)
        else:
            _lib.call("bgnn_bn_eval_coeffs", C, None if w is None else w.data_ptr(), None if b is None else b.data_ptr(),
                      float(eps), running_mean.data_ptr(), running_var.data_ptr(), scale.data_ptr(), shift.data_ptr(),
                      s)
            mean.copy_(running_mean)
            invstd.copy_(torch.rsqrt(running_var + eps))
        y = torch.empty_like(x)
        _lib.call("bgnn_bn_apply", x.data_ptr(), N, C, scale.data_ptr(), shift.data_ptr(), y.data_ptr(), s)
        ctx.batch_stats = batch_stats
        ctx.affine = (weight is not None, bias is not None)
        ctx.save_for_backward(x, coef, w if w is not None else torch.empty(0, device=dev))
        return y

    @staticmethod
    def backward(ctx, g):
        from . import _lib
        from .graph import _stream
        x, coef, w = ctx.saved_tensors
        g = g.contiguous()
        N, C = x.shape
        dev = x.device
        s = _stream()
        mean, invstd, scale = coef[0], coef[1], coef[2]
        slots = _lib.query("bgnn_bn_slots", N, C)
        part = torch.empty(slots, 2, C, dtype=torch.float32, device=dev)
        _lib.call("bgnn_bn_bwd_stats", g.data_ptr(), x.data_ptr(), mean.data_ptr(), invstd.data_ptr(), N, C,
                  part.data_ptr(), s)
        sums = torch.empty(2, C, dtype=torch.float32, device=dev)   # dbeta, dgamma
        _lib.call("bgnn_reduce_partials", part.data_ptr(), slots, C, sums[0].data_ptr(), sums[1].data_ptr(), 0, s)
        dx = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(x)
            if ctx.batch_stats:
                _lib.call("bgnn_bn_bwd_dx", g.data_ptr(), x.data_ptr(), mean.data_ptr(), invstd.data_ptr(),
                          w.data_ptr() if w.numel() else None, sums.data_ptr(), N, C, dx.data_ptr(), s)
            else:   # eval: dx = g * gamma * invstd (the scale of the forward)
                zero = torch.zeros(C, dtype=torch.float32, device=dev)
                _lib.call("bgnn_bn_apply", g.data_ptr(), N, C, scale.data_ptr(), zero.data_ptr(), dx.data_ptr(), s)
        has_w, has_b = ctx.affine
        return (dx, sums[1] if has_w else None, sums[0] if has_b else None, None, None, None, None, None)


class BatchNorm1d(nn.BatchNorm1d):
    """torch.nn.BatchNorm1d with the same constructor, parameters, buffers and state-dict keys,
    whose forward over a 2-D fp32 CUDA input runs on libbgnn (_BatchNormFn: csrc/bn.hip) -- the
    opt-in replacement bgnn.install_pyg_shim(batchnorm=True) installs for the BatchNorm1d modules
    the reference's unchanged Models/BuckGNN.py builds (torch's channels-last BatchNorm kernels
    take ~1.7 ms per cfg2 layer on ROCm). Anything else (3-D input, other dtypes,
    CPU) takes torch's forward. The momentum / num_batches_tracked / running-stats logic is
    torch's _BatchNorm.forward, restated."""

    def forward(self, input: Tensor) -> Tensor:
        C = input.size(-1) if input.dim() == 2 else -1
        if not (input.is_cuda and input.dim() == 2 and input.dtype == torch.float32 and C == self.num_features
                and C % 4 == 0 and C <= 1024 and 256 % (C // 4) == 0 and input.size(0) > 0
                and (self.weight is None or self.weight.dtype == torch.float32)):
            return super().forward(input)
        eaf = 0.0 if self.momentum is None else self.momentum
        if self.training and self.track_running_stats and self.num_batches_tracked is not None:
            self.num_batches_tracked.add_(1)
            if self.momentum is None:   # cumulative moving average (one host read, as torch's)
                eaf = 1.0 / float(self.num_batches_tracked.item())
        batch_stats = self.training or (self.running_mean is None and self.running_var is None)
        if batch_stats and input.size(0) < 2:
            raise ValueError(f"Expected more than 1 value per channel when training, got input size {tuple(input.shape)}")
        # (train: the running buffers are updated unless they are not tracked; eval: used)
        rm = self.running_mean if (not self.training or self.track_running_stats) else None
        rv = self.running_var if (not self.training or self.track_running_stats) else None
        return _BatchNormFn.apply(input, self.weight, self.bias, rm, rv, batch_stats, eaf, self.eps)


def use_bgnn_batchnorm(module: nn.Module) -> nn.Module:
    """Make every torch.nn.BatchNorm1d inside `module` a bgnn.nn.BatchNorm1d in place (the class
    only: parameters, buffers and state-dict keys are unchanged) and return the module."""
    torch_bn = torch.nn.modules.batchnorm.BatchNorm1d   # (torch's class even while the shim replaces nn's)
    for m in module.modules():
        if type(m) is torch_bn:
            m.__class__ = BatchNorm1d
    return module


def _num_segments(index: Tensor, size: Optional[int]) -> int:
    if size is not None:
        return int(size)
    return int(index.max().item()) + 1 if index.numel() else 0


def _pool(x: Tensor, batch: Optional[Tensor], size: Optional[int], reduce: str) -> Tensor:
    if batch is None:
        if reduce == "mean":
            return x.mean(dim=-2, keepdim=x.dim() == 2)
        if reduce == "sum":
            return x.sum(dim=-2, keepdim=x.dim() == 2)
        return x.max(dim=-2, keepdim=x.dim() == 2)[0]
    n = _num_segments(batch, size)
    return segment_reduce(x, segments_for(batch, n), reduce)


def global_mean_pool(x: Tensor, batch: Optional[Tensor], size: Optional[int] = None) -> Tensor:
    return _pool(x, batch, size, "mean")


def global_add_pool(x: Tensor, batch: Optional[Tensor], size: Optional[int] = None) -> Tensor:
    return _pool(x, batch, size, "sum")


def global_max_pool(x: Tensor, batch: Optional[Tensor], size: Optional[int] = None) -> Tensor:
    return _pool(x, batch, size, "max")


def _scatter(src: Tensor, index: Tensor, dim: int, out: Optional[Tensor], dim_size: Optional[int],
             reduce: str) -> Tensor:
    if src.dim() != 2 or dim not in (0, -2) or index.dim() != 1:
        raise NotImplementedError("bgnn scatter: only 2-D src with a 1-D index along dim 0 is supported")
    n = dim_size if dim_size is not None else (out.size(0) if out is not None else None)
    n = _num_segments(index, n)
    res = segment_reduce(src, segments_for(index, n), reduce)
    if out is not None:
        if reduce == "sum":
            out.add_(res)
        else:
            out.copy_(res)
        return out
    return res


def scatter_add(src: Tensor, index: Tensor, dim: int = 0, out: Optional[Tensor] = None,
                dim_size: Optional[int] = None) -> Tensor:
    return _scatter(src, index, dim, out, dim_size, "sum")


def scatter_sum(src: Tensor, index: Tensor, dim: int = 0, out: Optional[Tensor] = None,
                dim_size: Optional[int] = None) -> Tensor:
    return _scatter(src, index, dim, out, dim_size, "sum")


def scatter_mean(src: Tensor, index: Tensor, dim: int = 0, out: Optional[Tensor] = None,
                 dim_size: Optional[int] = None) -> Tensor:
    return _scatter(src, index, dim, out, dim_size, "mean")


class _SelectTopK(nn.Module):
    """The scoring projection of PyG's SelectTopK(in_channels=1) inside SAGPooling: weight
    [1, 1], score = act((attn * w).sum(-1) / ||w||) = act(sign(w) * attn). PyG releases
    before the select/connect refactor have no such weight (score = act(attn)); their
    checkpoints load with w = 1, which is the same function."""

    def __init__(self):
        super().__init__()
        self.weight = nn.Parameter(torch.empty(1, 1))
        with torch.no_grad():
            self.weight.uniform_(-1.0, 1.0)   # PyG: uniform(in_channels=1, weight)

    def _load_from_state_dict(self, state_dict, prefix, *args, **kwargs):
        if prefix + "weight" not in state_dict:
            state_dict[prefix + "weight"] = torch.ones(1, 1)
        super()._load_from_state_dict(state_dict, prefix, *args, **kwargs)


class SAGPooling(nn.Module):
    """torch_geometric.nn.SAGPooling in the form the reference builds it for GraphSAGE_SAG /
    EAGNN_SAG (Models/BuckGNN.py:203-208,231-236: `SAGPooling(h, ratio=0.5, GNN=SAGEConv,
    aggr='add')`, called at :364,502) [PyG-doc]:

        attn  = GNN(x, edge_index)                     [N, 1] (bgnn SAGEConv, HIP aggregation)
        score = tanh(sign(w) * attn)                   select.weight w
        perm  = topk(score, ratio, batch)              bgnn_topk_rank / bgnn_topk_select
        x'    = x[perm] * score[perm] (* multiplier)   bgnn_gather_scale (+ backward)
        edge_index', edge_attr' = filter_adj(...)      bgnn_filter_edges

    forward returns (x', edge_index', edge_attr', batch', perm, score[perm]). State-dict keys:
    `gnn.*` (the GNN's own) and `select.weight`. Ties in the score go to the lower node index.
    Not supported (the reference does not use them): the default GNN (GraphConv) and
    min_score (softmax selection)."""

    def __init__(self, in_channels: int, ratio: float = 0.5, GNN=None, min_score: Optional[float] = None,
                 multiplier: float = 1.0, nonlinearity="tanh", **kwargs):
        super().__init__()
        if GNN is None:
            raise NotImplementedError("SAGPooling: pass GNN= explicitly (GraphConv, PyG's default, is not provided)")
        if min_score is not None:
            raise NotImplementedError("SAGPooling: min_score (softmax selection) is not supported")
        if not ratio > 0:
            raise ValueError(f"SAGPooling: ratio must be > 0 (got {ratio})")
        self.in_channels = in_channels
        self.ratio = ratio
        self.min_score = min_score
        self.multiplier = multiplier
        self.nonlinearity = torch.tanh if nonlinearity == "tanh" else nonlinearity
        if not callable(self.nonlinearity):
            raise ValueError(f"SAGPooling: unsupported nonlinearity {nonlinearity!r}")
        self.gnn = GNN(in_channels, 1, **kwargs)
        self.select = _SelectTopK()

    def forward(self, x: Tensor, edge_index: Tensor, edge_attr: Optional[Tensor] = None,
                batch: Optional[Tensor] = None, attn: Optional[Tensor] = None):
        from .pool import sag_pool
        if batch is None:
            batch = torch.zeros(x.size(0), dtype=torch.long, device=x.device)
        attn = x if attn is None else attn
        attn = attn.view(-1, 1) if attn.dim() == 1 else attn
        attn = self.gnn(attn, edge_index)
        w = self.select.weight
        score = self.nonlinearity((attn * w).sum(dim=-1) / w.norm(p=2, dim=-1))
        return sag_pool(x, score, self.ratio, edge_index, edge_attr, batch, self.multiplier)

    def __repr__(self) -> str:
        return f"{self.__class__.__name__}({self.gnn.__class__.__name__}, {self.in_channels}, ratio={self.ratio})"
