"""BuckGNN on MI355X: same constructor, same submodules / state-dict keys, same
forward contract as Models/BuckGNN.py:9-526, with the SAGE layer loop run as
fused HIP layers (bgnn.fused) instead of per-op modules.

Variants and where their loop is defined in the reference:
    GraphSage_addAggr / _sumAggr / _meanAggr      :430-458 -> fused (BN, ReLU, skip, dropout)
    GraphSage_addAggr_Shared (TRAIN_FINAL default)  :338-352 -> fused (no BN)
    GraphSage_maxAggr                               :459-471 -> fused, aggregate-first (max aggregation,
                                                       [agg | x] GEMM, same BN / ReLU / skip / dropout kernels)
    EA_GNN / EA_GNN_Shared                          :326-336,375-387 -> per-op (GraphNetBlock on bgnn scatter_mean)
    GraphSAGE_SAG                                   :190-217,493-511 -> fused SAGE layers (skip added
                                                       after dropout), SAGPooling on bgnn kernels
    EAGNN_SAG                                       :219-244,354-373 -> GraphNetBlocks + SAGPooling
    GraphSage_MLP / *_woBatchNorm -> reproduce the reference's behaviour (AttributeError: their
      ModuleLists are never built, :404-429,472-492).
Pooling (get_pooling_layer, :246-307) is vectorised: the reference's per-node Python
loop over `batch` (:256-271) is `last index of every run of equal batch ids`.
"""
from __future__ import annotations

from typing import Optional

import torch
from torch import Tensor, nn

from . import ea as ea_mod
from .ea import GradSlot as EAGradSlot, graphnet_block, skip_dropout
from . import _lib
from . import fused as _fused
from .fused import RangeRows, mlp, mlp_bf16, prepare_weights, sage_layer, small_mlp
from .graph import SegmentIndex, graph_for, _index_cache
from .nn import SAGEConv, SAGPooling, global_mean_pool, scatter_mean
from .ops import segment_reduce

# run the node encoder on bgnn GEMMs (fused bias+ReLU) instead of torch nn.Linear
# (with the bf16x6 GEMM: 14.79 vs 14.82 ms/step, tools/ab_step.py)
FUSED_ENCODER = True
# fold the node encoder's last Linear into the first fused SAGE layer (BuckGNN._foldable_encoder)
FOLD_ENCODER = True
# buckling + mean pooling on the fused sum / mean layer loop: the last layer also returns the
# per-graph mean pool (fused.SageLayerFn pool), so its backward reads the pooled gradient through
# the batch vector instead of an [N, H] broadcast (A/B switch; the same bits)
FUSED_POOL = True

_SAGE_VARIANTS = {
    # model_name: (ModuleList attribute, aggr, has BatchNorm)
    "GraphSage_sumAggr": ("sage_blocks_sum", "sum", True),
    "GraphSage_addAggr": ("sage_blocks_add", "add", True),
    "GraphSage_meanAggr": ("sage_blocks_mean", "mean", True),
    "GraphSage_maxAggr": ("sage_blocks_max", "max", True),
}


def _mlp(dims, final_relu=False):
    layers = []
    for a, b in zip(dims[:-1], dims[1:]):
        layers += [nn.Linear(a, b), nn.ReLU()]
    if not final_relu:
        layers.pop()
    return nn.Sequential(*layers)


class GraphNetBlock(nn.Module):
    """Edge-feature message block (Models/BuckGNN.py:528-566): edge MLP on
    [x_row, x_col, e], message MLP phi on [x_col, e'], scatter_mean at row =
    edge_index[0], node MLPs gamma and beta."""

    def __init__(self, hidden_channels: int):
        super().__init__()
        h = hidden_channels
        self.edge_mlp = _mlp([3 * h, h, h])
        self.node_mlp_phi = _mlp([2 * h, h, h])
        self.node_mlp_gamma = _mlp([2 * h, h, h])
        self.node_mlp_beta = _mlp([h, h, h])

    def forward(self, x: Tensor, edge_index: Tensor, edge_attr: Tensor):
        row, col = edge_index[0], edge_index[1]
        e = self.edge_mlp(torch.cat([x[row], x[col], edge_attr], 1))
        m = self.node_mlp_phi(torch.cat([x[col], e], 1))
        agg = scatter_mean(m, row, dim=0, dim_size=x.size(0))
        out = self.node_mlp_gamma(torch.cat([x, agg], 1))
        return out + self.node_mlp_beta(out), e


class MLPPooling(nn.Module):
    """global mean pool then Linear+ReLU (Models/BuckGNN.py:568-581)."""

    def __init__(self, in_channels: int, hidden_channels: int, out_channels: int):
        super().__init__()
        self.mlp = nn.Sequential(nn.Linear(in_channels, hidden_channels), nn.ReLU())

    def forward(self, x: Tensor, batch: Optional[Tensor]):
        return self.mlp(global_mean_pool(x, batch))


def _output_dim(prediction_type: str, use_z_coord: bool, use_rotations: bool) -> int:
    if prediction_type == "buckling":
        return 1
    if prediction_type == "static_disp":
        return {(True, True): 6, (True, False): 3, (False, True): 4, (False, False): 2}[(use_z_coord, use_rotations)]
    if prediction_type == "static_stress":
        return 3
    if prediction_type == "mode_shape":
        return 6 if use_rotations else 3
    return 1


def batch_segments(batch: Tensor) -> SegmentIndex:
    """Segment structure of a `batch` vector, cached per tensor (one host sync per new batch)."""
    def build():
        n = int(batch.max().item()) + 1 if batch.numel() else 0
        return SegmentIndex.build(batch, n)
    return _index_cache.get(batch, ("batch",), build)


def super_node_index(batch: Optional[Tensor], n_nodes: int, device) -> Tensor:
    """Index of the last node of every graph (the super node, VirtualEdgeCreate.py:106-107);
    vectorised form of the reference's loop at Models/BuckGNN.py:256-266."""
    if batch is None:
        return torch.tensor([n_nodes - 1], device=device)
    if batch.numel() == 0:
        return torch.zeros(0, dtype=torch.long, device=device)
    change = torch.nonzero(batch[1:] != batch[:-1]).flatten()
    return torch.cat([change, torch.tensor([batch.numel() - 1], device=batch.device)])


def _range_rows_on(graph, red: int, n_rows: int, H: int) -> bool:
    """Whether the fused sum / mean layer loop takes the range-row path (fused.RangeRows) on this
    graph: it has heavy rows, the row passes' blocks are short enough for the 3 range slots
    (bgnn_range_sums_finish: rows per block <= 2 (chunk + 1)), and the transposed and forward ranges
    are computed (Csr.ensure_ranges)."""
    if not _fused.RANGE_ROWS or red == 2 or H > 512 or graph.fwd.plan.n_heavy <= 0:
        return False
    slots = _lib.query("bgnn_rows_slots", n_rows)
    if (n_rows + slots - 1) // slots > 2 * (graph.fwd.plan.chunk + 1):
        return False
    graph.fwd.ensure_ranges()
    graph.bwd.ensure_ranges()
    return True


class BuckGNN(nn.Module):
    def __init__(self, num_node_features, num_edge_features, hidden_channels=128, num_layers=6,
                 pooling_layer="mean", prediction_type="buckling", use_z_coord=False, use_rotations=False,
                 dropout_rate=0.1, model_name="GraphSAGE_MLP"):
        super().__init__()
        h = hidden_channels
        self.hidden_channels = h
        self.prediction_type = prediction_type
        self.pooling_layer = pooling_layer
        self.num_layers = num_layers
        self.model_name = model_name
        out_dim = _output_dim(prediction_type, use_z_coord, use_rotations)
        dec_in = 2 * h if (pooling_layer == "supernode_with_pooling" and prediction_type == "buckling") else h
        # encoders / decoder (Models/BuckGNN.py:41-100; nothing is built for 128 < h < 256)
        if h <= 128:
            self.node_encoder = _mlp([num_node_features, 64, h])
            self.edge_encoder = _mlp([num_edge_features, 64, h])
            self.decoder = _mlp([dec_in, 64, out_dim])
        elif h >= 256:
            self.node_encoder = _mlp([num_node_features, 64, 128, h])
            self.edge_encoder = _mlp([num_edge_features, 64, 128, h])
            self.decoder = _mlp([dec_in, 128, 64, out_dim])
        # processors (Models/BuckGNN.py:103-180)
        if model_name == "EA_GNN_Shared":
            self.shared_gn_block = GraphNetBlock(h)
        if model_name == "EA_GNN":
            self.gn_blocks = nn.ModuleList([GraphNetBlock(h) for _ in range(num_layers)])
        if model_name == "GraphSage_addAggr_Shared":
            self.shared_graphsage_block = SAGEConv(in_channels=h, out_channels=h, normalize=True, aggr="add")
        if model_name in _SAGE_VARIANTS:
            attr, aggr, _ = _SAGE_VARIANTS[model_name]
            setattr(self, attr, nn.ModuleList())
            self.batch_norms = nn.ModuleList()
            self.sage_mlps = nn.ModuleList()
            for _ in range(num_layers):
                getattr(self, attr).append(SAGEConv(in_channels=h, out_channels=h, normalize=True, aggr=aggr))
                self.batch_norms.append(nn.BatchNorm1d(h))
                self.sage_mlps.append(nn.Linear(h, h))
        self.batch_norm = nn.BatchNorm1d(h)
        self.relu = nn.ReLU()
        self.dropout = nn.Dropout(p=dropout_rate)
        self.pooling_mpl = MLPPooling(h, h, h)
        if model_name in ("GraphSAGE_SAG", "EAGNN_SAG"):   # Models/BuckGNN.py:190-244
            n_before = num_layers // 2
            n_after = num_layers - n_before
            sag = model_name == "GraphSAGE_SAG"
            pre, bns = ("sage_layers_", True) if sag else ("gnn_layers_", False)

            def block():
                return SAGEConv(h, h, normalize=True, aggr="add") if sag else GraphNetBlock(h)
            setattr(self, pre + "1", nn.ModuleList([block() for _ in range(n_before)]))
            self.batch_norms_1 = nn.ModuleList([nn.BatchNorm1d(h) for _ in range(n_before)] if bns else [])
            self.pool = SAGPooling(h, ratio=0.5, GNN=SAGEConv, aggr="add")
            setattr(self, pre + "2", nn.ModuleList([block() for _ in range(n_after)]))
            self.batch_norms_2 = nn.ModuleList([nn.BatchNorm1d(h) for _ in range(n_after)] if bns else [])
        # fused-path switch (tests compare both paths)
        self.use_fused = True
        # EA_GNN GEMM precision on the fused path: False = f32-accurate (f16x3), True = bf16
        # operands with f32 accumulation and bf16 storage of the per-edge activations
        # (BASELINE configs[4]; bgnn.ea.BF16_STORAGE)
        self.ea_bf16 = False
        self._step = 0

    # ------------------------------------------------------------------ pooling
    def get_pooling_layer(self, x: Tensor, edge_index: Tensor, batch: Optional[Tensor]) -> Tensor:
        mode = self.pooling_layer
        if mode == "mean":
            if batch is None:
                return global_mean_pool(x, None)
            return segment_reduce(x, batch_segments(batch), "mean")
        if mode == "hybrid":
            raise AttributeError("'BuckGNN' object has no attribute 'hybrid_pooling'")  # Models/BuckGNN.py:188,276
        if mode == "mlp":
            return self.pooling_mpl(x, batch)
        if "super" not in mode and mode != "mlp_no_super" and mode != "mean_no_super":
            raise ValueError(f"Unknown pooling layer: {mode}")
        sup = super_node_index(batch, x.size(0), x.device)
        keep = torch.ones(x.size(0), dtype=torch.bool, device=x.device)
        keep[sup] = False
        real = torch.nonzero(keep).flatten()
        if batch is None:
            rb = torch.zeros(real.numel(), dtype=torch.long, device=x.device)
        else:
            rb = batch[real]
        if mode == "mean_no_super":
            return global_mean_pool(x[real], rb)
        if mode == "supernode_only":
            return x[sup]
        if mode == "supernode_with_pooling":
            return torch.cat([global_mean_pool(x[real], rb), x[sup]], 1)
        if mode == "mlp_no_super":
            return self.pooling_mpl(x[real], rb)
        raise ValueError(f"Unknown pooling layer: {mode}")

    # ------------------------------------------------------------------ forward
    def _seed(self) -> int:
        # dropout mask seed drawn from torch's CPU generator: reproducible under torch.manual_seed
        return int(torch.randint(0, 2 ** 62, (1,)).item())

    def _decode(self, h: Tensor) -> Tensor:
        """The decoder on the pooled per-graph features: bgnn small-batch Linear layers on the
        fused path (bgnn.fused.small_mlp), the torch modules otherwise."""
        dec = self.decoder
        # (a module with hooks is called as a module, so the hooks see its input and output)
        hooked = bool(dec._forward_pre_hooks or dec._forward_hooks)
        out = small_mlp(dec, h) if (self.use_fused and not hooked) else None
        return dec(h) if out is None else out

    def _fused_ok(self, x: Tensor) -> bool:
        return self.use_fused and x.is_cuda and self.hidden_channels % 4 == 0 and self.hidden_channels <= 512

    def _sage_fused(self, x: Tensor, aggr: str) -> bool:
        return self._fused_ok(x) and aggr in ("add", "sum", "mean", "max")

    def _foldable_encoder(self, x: Tensor) -> bool:
        """The node encoder's last Linear can be folded into the first fused SAGE layer (which
        has no skip connection): the encoder output x0 = h W^T + b feeds only that layer's
        transform [W_l;W_r], so z = h ([W_l;W_r] W)^T + [W_l;W_r] b (fused.sage_layer w_in)."""
        enc = self.node_encoder
        return (FOLD_ENCODER and FUSED_ENCODER and isinstance(enc, nn.Sequential) and len(enc) >= 2
                and isinstance(enc[-1], nn.Linear) and enc[-1].out_features == self.hidden_channels
                and x.size(0) >= 1024 and self.num_layers >= 1)

    def _sage_loop(self, x: Tensor, edge_index: Tensor, convs, bns, aggr: str, skip_last_excluded: bool,
                   x_amax: Optional[Tensor] = None, x_in: Optional[nn.Linear] = None, pool=None):
        """The SAGE layer loop; pool (a SegmentIndex; fused sum / mean loop only): returns
        (x, mean pool of x per segment) from the last fused layer instead of x."""
        L = len(convs) if convs is not None else self.num_layers
        p = self.dropout.p
        if self._sage_fused(x, aggr):
            graph = graph_for(edge_index, x.size(0))
            red = {"mean": 1, "max": 2}.get(aggr, 0)
            amax = x_amax   # max|x| of the running features: each layer's apply kernel folds it in
            # per-layer operand maxima (slot 3: max|.| of the layer output's [N + R, H] range-row
            # buffer, fused.RangeRows) and the folded layer's weight-product maxima, one fill
            scratch = torch.zeros(4 * L + 5, dtype=torch.float32, device=x.device)
            bufs, fold_amax = scratch[:4 * L].view(L, 4), scratch[4 * L:]
            layers = [convs[i] if convs is not None else self.shared_graphsage_block for i in range(L)]
            rng_on = _range_rows_on(graph, red, x.size(0), layers[0].lin_l.weight.size(0))
            R = graph.fwd.plan.n_heavy if rng_on else 0
            wprep = prepare_weights([(c.lin_l.weight, c.lin_r.weight) for c in layers], bufs,
                                    [not (i == 0 and x_in is not None) for i in range(L)],
                                    n_rows=x.size(0) + R if red != 2 else 0)
            self._count_bn_batches(bns)
            x_full = None
            for i in range(L):
                conv = layers[i]
                bn = bns[i] if bns is not None else None
                skip = 0 < i < L - 1
                fold = x_in if i == 0 else None
                rng = (RangeRows(x_full=x_full, x_amax=bufs[i - 1, 3:4] if x_full is not None else None,
                                 out=i < L - 1, out_amax=bufs[i, 3:4]) if rng_on else None)
                pl = pool if (i == L - 1 and red != 2) else None
                out = sage_layer(x, conv.lin_l.weight, conv.lin_l.bias, conv.lin_r.weight, bn, graph, red,
                                 skip, p, self.training, self._seed(), x_amax=amax, return_amax=True,
                                 amax_buf=bufs[i], w_in=None if fold is None else fold.weight,
                                 b_in=None if fold is None else fold.bias, wprep=wprep[i], count_batch=False,
                                 fold_amax=fold_amax, rng=rng, pool=pl)
                x, amax = out[0], out[1]
                x_full = rng.holder[0] if (rng is not None and rng.holder) else None
            if pool is not None:
                return x, (out[2] if (red != 2 and L > 0) else segment_reduce(x, pool, "mean"))
            return x
        if x_in is not None:   # (only reached when the caller folded the encoder's last Linear)
            x = x_in(x)
        for i in range(L):
            x_prev = x
            conv = convs[i] if convs is not None else self.shared_graphsage_block
            x = conv(x, edge_index)
            if bns is not None:
                x = bns[i](x)
            x = self.relu(x)
            if 0 < i < L - 1:
                x = x + x_prev
            x = self.dropout(x)
        return (x, segment_reduce(x, pool, "mean")) if pool is not None else x

    def _count_bn_batches(self, bns) -> None:
        """BatchNorm1d's num_batches_tracked += 1 for every module of a fused loop in one launch
        (the fused layers are then called with count_batch=False)."""
        if bns is None or not self.training:
            return
        ts = [bn.num_batches_tracked for bn in bns if bn.track_running_stats]
        if ts:
            torch._foreach_add_(ts, 1)

    def _sag_sage_loop(self, x: Tensor, edge_index: Tensor, convs, bns, first_skip: bool,
                       x_amax: Optional[Tensor] = None, x_in: Optional[nn.Linear] = None) -> Tensor:
        """GraphSAGE_SAG's layer loops (Models/BuckGNN.py:494-501 with first_skip=False,
        :505-511 with first_skip=True): conv -> BN -> ReLU -> Dropout, then + identity. The
        fused layer computes the first four (no skip inside: here the skip follows dropout)."""
        p = self.dropout.p
        if self._sage_fused(x, "add"):
            graph = graph_for(edge_index, x.size(0))
            bufs = torch.zeros(len(convs), 3, dtype=torch.float32, device=x.device)
            for i, (conv, bn) in enumerate(zip(convs, bns)):
                skip = first_skip or i > 0
                fold = x_in if i == 0 else None
                y, y_amax = sage_layer(x, conv.lin_l.weight, conv.lin_l.bias, conv.lin_r.weight, bn, graph, 0,
                                       False, p, self.training, self._seed(), x_amax=x_amax, return_amax=True,
                                       amax_buf=bufs[i], w_in=None if fold is None else fold.weight,
                                       b_in=None if fold is None else fold.bias)
                x, x_amax = (y + x, None) if skip else (y, y_amax)
            return x
        if x_in is not None:
            x = x_in(x)
        for i, (conv, bn) in enumerate(zip(convs, bns)):
            identity = x
            x = self.dropout(self.relu(bn(conv(x, edge_index))))
            if first_skip or i > 0:
                x = x + identity
        return x

    def _skip_dropout(self, x, e, x_prev, e_prev, skip: bool, fused: bool, e_slot=None):
        """EA_GNN's `if 0 < i < L-1: x, e = x + x_prev, e + e_prev` then Dropout on both
        (Models/BuckGNN.py:382-387); one bgnn_add_dropout pass each on the fused path (e_slot:
        the edge gradient goes to the block's edge Linears, bgnn.ea.GradSlot)."""
        if not fused:
            if skip:
                x, e = x + x_prev, e + e_prev
            return self.dropout(x), self.dropout(e)
        p = self.dropout.p
        return (skip_dropout(x, x_prev if skip else None, p, self.training, self._seed()),
                skip_dropout(e, e_prev if skip else None, p, self.training, self._seed(), slot=e_slot))

    def _ea_block(self, blk, x, e, edge_index, fused: bool):
        return graphnet_block(blk, x, e, edge_index, self.ea_bf16) if fused else blk(x, edge_index, e)

    def forward(self, x, edge_index, edge_attr, batch=None, mask=None):
        name = self.model_name
        if "super" in self.pooling_layer:
            is_real_node = x[:, -1] == 0 if x.size(1) > 0 else torch.ones(x.size(0), dtype=torch.bool,
                                                                           device=x.device)
            real_node_batch = batch[is_real_node] if batch is not None else None
        x_amax = None   # max|x| after the encoder (f16x3 operand scale of the first SAGE GEMM)
        x_in = None     # the encoder's last Linear when it is folded into the first SAGE layer
        sage = _SAGE_VARIANTS.get(name, (None, "add", None))[1] if name != "GraphSage_addAggr_Shared" else "add"
        # (GraphSAGE_SAG folds into sage_layers_1[0]: not when that list is empty, num_layers == 1)
        if (name in _SAGE_VARIANTS or name == "GraphSage_addAggr_Shared"
                or (name == "GraphSAGE_SAG" and len(self.sage_layers_1) >= 1)) \
                and self._sage_fused(x, sage) and sage != "max" and self._foldable_encoder(x):
            x_in = self.node_encoder[-1]
            x, x_amax = mlp(self.node_encoder[:-1], x, return_amax=True)
        elif self._fused_ok(x) and x.size(0) >= 1024 and FUSED_ENCODER:
            x, x_amax = mlp(self.node_encoder, x, return_amax=True)   # GEMMs with fused bias+ReLU epilogues
        else:
            x = self.node_encoder(x)
        ea_fused = name in ("EA_GNN", "EA_GNN_Shared", "EAGNN_SAG") and self._fused_ok(x)
        if ea_fused:
            if self.ea_bf16 and ea_mod.BF16_STORAGE and edge_attr.size(0) >= 1024 and FUSED_ENCODER:
                e = mlp_bf16(self.edge_encoder, edge_attr)   # bf16 edge activations from the start
            else:
                e = (mlp(self.edge_encoder, edge_attr) if edge_attr.size(0) >= 1024 and FUSED_ENCODER
                     else self.edge_encoder(edge_attr))
        if name == "EA_GNN_Shared":
            if not ea_fused:
                e = self.edge_encoder(edge_attr)
            for i in range(self.num_layers):
                x_prev, e_prev = x, e
                if ea_fused:
                    x, e = graphnet_block(self.shared_gn_block, x, e, edge_index, self.ea_bf16)
                else:
                    x, e = self.shared_gn_block(x, edge_index, e)
                x, e = self._skip_dropout(x, e, x_prev, e_prev, 0 < i < self.num_layers - 1, ea_fused)
        # the buckling decoder's mean pool from the last fused sum / mean layer (FUSED_POOL)
        pool = (batch_segments(batch) if (FUSED_POOL and self.prediction_type == "buckling"
                                          and self.pooling_layer == "mean" and batch is not None
                                          and (name == "GraphSage_addAggr_Shared" or name in _SAGE_VARIANTS)
                                          and self._sage_fused(x, sage) and sage != "max") else None)
        pooled = None
        if name == "GraphSage_addAggr_Shared":
            x = self._sage_loop(x, edge_index, None, None, "add", True, x_amax, x_in, pool=pool)
            if pool is not None:
                x, pooled = x
        elif name == "EA_GNN":
            if not ea_fused:
                e = self.edge_encoder(edge_attr)
            L = len(self.gn_blocks)
            for i, blk in enumerate(self.gn_blocks):
                x_prev, e_prev = x, e
                # the last block's edge output feeds nothing: no gradient hand-off there
                slot = EAGradSlot() if (ea_fused and self.ea_bf16 and self.training and i < L - 1) else None
                if ea_fused:   # transform-first GraphNetBlock on bgnn GEMMs (bgnn/ea.py)
                    x, e = graphnet_block(blk, x, e, edge_index, self.ea_bf16, slot=slot, slot_in=0 < i < L - 1)
                else:
                    x, e = blk(x, edge_index, e)
                x, e = self._skip_dropout(x, e, x_prev, e_prev, 0 < i < L - 1, ea_fused, e_slot=slot)
        elif name in _SAGE_VARIANTS:
            attr, aggr, _ = _SAGE_VARIANTS[name]
            x = self._sage_loop(x, edge_index, getattr(self, attr), self.batch_norms, aggr, True, x_amax, x_in,
                                pool=pool)
            if pool is not None:
                x, pooled = x
        elif name in ("GraphSage_addAggr_woBatchNorm", "GraphSage_MLP"):
            getattr(self, "sage_blocks_add")  # AttributeError, as in the reference (:405,473)
        elif name == "GraphSage_sumAggr_woBatchNorm":
            getattr(self, "sage_blocks_sum")  # AttributeError, as in the reference (:418)
        elif name == "GraphSAGE_SAG":   # Models/BuckGNN.py:493-511
            x = self._sag_sage_loop(x, edge_index, self.sage_layers_1, self.batch_norms_1, False, x_amax, x_in)
            x, edge_index, edge_attr, batch, _perm, _score = self.pool(x, edge_index, edge_attr, batch)
            x = self._sag_sage_loop(x, edge_index, self.sage_layers_2, self.batch_norms_2, True)
        elif name == "EAGNN_SAG":       # Models/BuckGNN.py:354-373
            if not ea_fused:
                e = self.edge_encoder(edge_attr)
            for i, blk in enumerate(self.gnn_layers_1):
                x_prev, e_prev = x, e
                x, e = self._ea_block(blk, x, e, edge_index, ea_fused)
                x, e = self.dropout(x), self.dropout(e)
                if i > 0:
                    x, e = x + x_prev, e + e_prev
            x, edge_index, e, batch, _perm, _score = self.pool(x, edge_index, e, batch)
            for blk in self.gnn_layers_2:
                x_prev, e_prev = x, e
                x, e = self._ea_block(blk, x, e, edge_index, ea_fused)
                x, e = self.dropout(x), self.dropout(e)
                x, e = x + x_prev, e + e_prev

        if self.prediction_type == "buckling":
            if pooled is None:
                pooled = self.get_pooling_layer(x, edge_index, batch)
            return self._decode(pooled).squeeze(), batch
        if "static" in self.prediction_type or "mode_shape" in self.prediction_type:
            if "super" in self.pooling_layer:
                return self.decoder(x[is_real_node]), real_node_batch
            return self.decoder(x), batch
        raise ValueError(f"Unknown prediction type: {self.prediction_type}")
