"""ORACLE (test infrastructure only): CPU restatement of BuckGNN's SAGE forward and
train step, in functional form over a state dict with the reference's key names.

Follows, line for line in meaning:
  encoder            Models/BuckGNN.py:41-74   (h<=128: F->64->h; h>=256: F->64->128->h)
  decoder            Models/BuckGNN.py:55-65,85-100
  SAGE layer loops   Models/BuckGNN.py:338-352 (Shared, no BN), :389-403 (sum),
                     :430-444 (add), :445-458 (mean), :459-471 (max)
  pooling 'mean'     Models/BuckGNN.py:273-274 (global_mean_pool incl. super node)
  pooling super*     Models/BuckGNN.py:248-271,277-293
  loss               Utils/Losses.py:755-761 on Normalizer.py:207-215 denormalised values
  step               TRAIN_FINAL.py:190 (Adam lr, wd), :253-298 (fwd, loss, zero_grad, bwd, step)
  EA_GNN loop        Models/BuckGNN.py:375-387 with GraphNetBlock :528-566 (edge encoder :76-82)
  SAG variants       Models/BuckGNN.py:493-511 (GraphSAGE_SAG), :354-373 (EAGNN_SAG), with
                     SAGPooling :203-208,231-236 restated in oracle.pyg_ref (topk, filter_adj)
The SAGEConv arithmetic is oracle.pyg_ref (gather -> index_add -> lin_l + lin_r -> normalize).
"""
from __future__ import annotations

from typing import Dict, Optional

import torch
import torch.nn.functional as F
from torch import Tensor

from .pyg_ref import filter_adj, global_mean_pool, sage_aggregate, topk

SAGE = {  # model_name -> (ModuleList attribute, aggr, batchnorm)
    "GraphSage_sumAggr": ("sage_blocks_sum", "sum", True),
    "GraphSage_addAggr": ("sage_blocks_add", "add", True),
    "GraphSage_meanAggr": ("sage_blocks_mean", "mean", True),
    "GraphSage_maxAggr": ("sage_blocks_max", "max", True),
    "GraphSage_addAggr_Shared": ("shared_graphsage_block", "add", False),
}


def _mlp(sd: Dict[str, Tensor], prefix: str, x: Tensor) -> Tensor:
    idx = sorted({int(k[len(prefix) + 1:].split(".")[0]) for k in sd if k.startswith(prefix + ".")})
    for n, i in enumerate(idx):
        x = F.linear(x, sd[f"{prefix}.{i}.weight"], sd[f"{prefix}.{i}.bias"])
        if n < len(idx) - 1:
            x = F.relu(x)
    return x


def sage_conv(sd, pre, x, edge_index, aggr):
    agg = sage_aggregate(x, edge_index, aggr)
    out = F.linear(agg, sd[pre + ".lin_l.weight"], sd[pre + ".lin_l.bias"]) + F.linear(x, sd[pre + ".lin_r.weight"])
    return F.normalize(out, p=2.0, dim=-1)


def super_index(batch: Optional[Tensor], n: int) -> Tensor:
    if batch is None:
        return torch.tensor([n - 1])
    last = [i for i in range(n - 1) if batch[i] != batch[i + 1]] + [n - 1]
    return torch.tensor(last)


def forward(sd: Dict[str, Tensor], model_name: str, x: Tensor, edge_index: Tensor, batch: Optional[Tensor],
            training: bool, pooling: str = "mean", dropout: float = 0.0, num_layers: int = 6,
            bn_momentum: float = 0.1, bn_eps: float = 1e-5, return_nodes: bool = False):
    attr, aggr, use_bn = SAGE[model_name]
    x = _mlp(sd, "node_encoder", x)
    for i in range(num_layers):
        x_prev = x
        pre = attr if model_name.endswith("_Shared") else f"{attr}.{i}"
        x = sage_conv(sd, pre, x, edge_index, aggr)
        if use_bn:
            b = f"batch_norms.{i}"
            x = F.batch_norm(x, sd[b + ".running_mean"], sd[b + ".running_var"], sd[b + ".weight"],
                             sd[b + ".bias"], training, bn_momentum, bn_eps)
        x = F.relu(x)
        if 0 < i < num_layers - 1:
            x = x + x_prev
        x = F.dropout(x, dropout, training)
    nodes = x
    if pooling == "mean":
        pooled = global_mean_pool(x, batch)
    else:
        sup = super_index(batch, x.size(0))
        keep = torch.ones(x.size(0), dtype=torch.bool)
        keep[sup] = False
        real = torch.nonzero(keep).flatten()
        rb = batch[real] if batch is not None else torch.zeros(real.numel(), dtype=torch.long)
        if pooling == "mean_no_super":
            pooled = global_mean_pool(x[real], rb)
        elif pooling == "supernode_only":
            pooled = x[sup]
        elif pooling == "supernode_with_pooling":
            pooled = torch.cat([global_mean_pool(x[real], rb), x[sup]], 1)
        else:
            raise ValueError(pooling)
    pred = _mlp(sd, "decoder", pooled).squeeze()
    return (pred, nodes) if return_nodes else pred


def graphnet_block(sd: Dict[str, Tensor], pre: str, x: Tensor, edge_index: Tensor, e: Tensor):
    """GraphNetBlock.forward (Models/BuckGNN.py:552-566): concatenation MLPs on gathered node
    rows, scatter_mean of the messages at row = edge_index[0]."""
    row, col = edge_index[0], edge_index[1]
    e = _mlp(sd, pre + ".edge_mlp", torch.cat([x[row], x[col], e], 1))
    m = _mlp(sd, pre + ".node_mlp_phi", torch.cat([x[col], e], 1))
    deg = torch.zeros(x.size(0), dtype=x.dtype, device=x.device).index_add_(
        0, row, torch.ones(row.numel(), dtype=x.dtype, device=x.device))
    agg = torch.zeros(x.size(0), m.size(1), dtype=m.dtype, device=m.device).index_add_(0, row, m)
    agg = agg / deg.clamp_min(1).unsqueeze(1)
    x = _mlp(sd, pre + ".node_mlp_gamma", torch.cat([x, agg], 1))
    return x + _mlp(sd, pre + ".node_mlp_beta", x), e


def ea_forward(sd: Dict[str, Tensor], x: Tensor, edge_index: Tensor, edge_attr: Tensor, batch: Optional[Tensor],
               training: bool, dropout: float = 0.0, num_layers: int = 6, shared: bool = False) -> Tensor:
    """EA_GNN forward (Models/BuckGNN.py:323,375-387,515-516) with mean pooling; shared=True:
    EA_GNN_Shared (:326-336), one GraphNetBlock (`shared_gn_block`) applied num_layers times
    with the same skip / dropout pattern."""
    x = _mlp(sd, "node_encoder", x)
    e = _mlp(sd, "edge_encoder", edge_attr)
    for i in range(num_layers):
        x_prev, e_prev = x, e
        x, e = graphnet_block(sd, "shared_gn_block" if shared else f"gn_blocks.{i}", x, edge_index, e)
        if 0 < i < num_layers - 1:
            x, e = x + x_prev, e + e_prev
        x, e = F.dropout(x, dropout, training), F.dropout(e, dropout, training)
    return _mlp(sd, "decoder", global_mean_pool(x, batch)).squeeze()


def sag_pool(sd: Dict[str, Tensor], x: Tensor, edge_index: Tensor, edge_attr: Optional[Tensor],
             batch: Tensor, ratio: float = 0.5):
    """SAGPooling(h, ratio, GNN=SAGEConv, aggr='add') at key prefix `pool`: returns
    (x', edge_index', edge_attr', batch', perm, score[perm])."""
    agg = sage_aggregate(x, edge_index, "add")
    attn = F.linear(agg, sd["pool.gnn.lin_l.weight"], sd["pool.gnn.lin_l.bias"]) + \
        F.linear(x, sd["pool.gnn.lin_r.weight"])
    w = sd["pool.select.weight"]
    score = torch.tanh((attn * w).sum(-1) / w.norm(p=2, dim=-1))
    perm = topk(score, ratio, batch)
    s = score[perm]
    ei, ea = filter_adj(edge_index, edge_attr, perm, x.size(0))
    return x[perm] * s.view(-1, 1), ei, ea, batch[perm], perm, s


def sag_forward(sd: Dict[str, Tensor], model_name: str, x: Tensor, edge_index: Tensor, edge_attr: Tensor,
                batch: Optional[Tensor], training: bool, dropout: float = 0.0, num_layers: int = 6,
                bn_momentum: float = 0.1, bn_eps: float = 1e-5):
    """GraphSAGE_SAG / EAGNN_SAG forward with mean pooling: returns (pred, perm)."""
    x = _mlp(sd, "node_encoder", x)
    if batch is None:
        batch = torch.zeros(x.size(0), dtype=torch.long)
    n1 = num_layers // 2
    n2 = num_layers - n1
    if model_name == "GraphSAGE_SAG":
        def run(x, ei, part, n, first_skip):
            for i in range(n):
                identity = x
                x = sage_conv(sd, f"sage_layers_{part}.{i}", x, ei, "add")
                b = f"batch_norms_{part}.{i}"
                x = F.batch_norm(x, sd[b + ".running_mean"], sd[b + ".running_var"], sd[b + ".weight"],
                                 sd[b + ".bias"], training, bn_momentum, bn_eps)
                x = F.dropout(F.relu(x), dropout, training)
                if first_skip or i > 0:
                    x = x + identity
            return x
        x = run(x, edge_index, 1, n1, False)
        x, edge_index, _, batch, perm, _ = sag_pool(sd, x, edge_index, edge_attr, batch)
        x = run(x, edge_index, 2, n2, True)
    elif model_name == "EAGNN_SAG":
        e = _mlp(sd, "edge_encoder", edge_attr)

        def run(x, e, ei, part, n, first_skip):
            for i in range(n):
                x_prev, e_prev = x, e
                x, e = graphnet_block(sd, f"gnn_layers_{part}.{i}", x, ei, e)
                x, e = F.dropout(x, dropout, training), F.dropout(e, dropout, training)
                if first_skip or i > 0:
                    x, e = x + x_prev, e + e_prev
            return x, e
        x, e = run(x, e, edge_index, 1, n1, False)
        x, edge_index, e, batch, perm, _ = sag_pool(sd, x, edge_index, e, batch)
        x, e = run(x, e, edge_index, 2, n2, True)
    else:
        raise ValueError(model_name)
    return _mlp(sd, "decoder", global_mean_pool(x, batch)).squeeze(), perm


def relative_error_loss(pred: Tensor, target: Tensor, eps: float = 1e-8) -> Tensor:
    return torch.mean(torch.abs(pred - target) / (torch.abs(target) + eps))


class TrainStep:
    """fwd + RelativeErrorLoss + bwd + Adam over the used parameters (CPU)."""

    def __init__(self, sd: Dict[str, Tensor], model_name: str, lr: float = 1e-2, weight_decay: float = 1e-8,
                 dropout: float = 0.1, pooling: str = "mean", num_layers: int = 6):
        self.sd = {k: v.detach().clone() for k, v in sd.items()}
        self.params = []
        for k, v in self.sd.items():
            if v.is_floating_point() and not k.endswith(("running_mean", "running_var")):
                v.requires_grad_(True)
                self.params.append(v)
        self.model_name, self.dropout, self.pooling, self.num_layers = model_name, dropout, pooling, num_layers
        self.opt = torch.optim.Adam(self.params, lr=lr, weight_decay=weight_decay)

    def __call__(self, x, edge_index, batch, y):
        pred = forward(self.sd, self.model_name, x, edge_index, batch, True, self.pooling, self.dropout,
                       self.num_layers)
        loss = relative_error_loss(pred, y)
        self.opt.zero_grad(set_to_none=True)
        loss.backward()
        self.opt.step()
        return loss.detach()
