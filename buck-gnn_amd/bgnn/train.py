"""Training-step driver and data-parallel gradient exchange.

`train_step` is the body of the reference's inner loop (TRAIN_FINAL.py:253-298)
for buckling targets: forward, RelativeErrorLoss on denormalised eigenvalues
(Utils/Losses.py:755-761, Dataset_Preparation/Normalizer.py:207-215), backward,
Adam step (TRAIN_FINAL.py:190). The reference's per-step `.item()` host syncs
(TRAIN_FINAL.py:263,298) are optional here (`sync_metrics`).

`GradAllReduce` is the one collective of the multi-GPU path: the
mini-batch is split by whole mesh graphs (no edge cuts), each rank runs its own
graphs, and the gradients of the parameters that received one are summed with a
single flat RCCL all-reduce and divided by the world size. Parameters the
forward never touches (edge_encoder, batch_norm, pooling_mpl, sage_mlps of the
addAggr variant) have no gradient and are skipped, exactly like the unused
modules in the reference.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.distributed as dist
from torch import nn

from .graph import prepare


class RelativeErrorLoss(nn.Module):
    """mean(|pred - target| / (|target| + eps))  (Utils/Losses.py:755-761)."""

    def __init__(self, epsilon: float = 1e-8):
        super().__init__()
        self.epsilon = epsilon

    def forward(self, pred, target):
        return torch.mean(torch.abs(pred - target) / (torch.abs(target) + self.epsilon))


def mape_error(pred, target, normalizer=None):
    """MAPE in percent for buckling targets (Dataset_Preparation/Metrics.py:4-12)."""
    if normalizer is not None:
        pred = normalizer.denormalize_eigenvalue(pred)
        target = normalizer.denormalize_eigenvalue(target)
    return torch.mean(torch.abs((target - pred) / target)) * 100


class EigenvalueScaler:
    """The affine eigenvalue (de)normalisation of DatasetNormalizer (Normalizer.py:203-215):
    value * scale + center (RobustScaler center_/scale_)."""

    def __init__(self, center: float = 0.0, scale: float = 1.0):
        self.center = float(center)
        self.scale = float(scale)

    def normalize_eigenvalue(self, v):
        return (v - self.center) / self.scale

    def denormalize_eigenvalue(self, v):
        return v * self.scale + self.center


class GradAllReduce:
    """Sum-then-average gradients across ranks with one flat all-reduce."""

    def __init__(self, model: nn.Module, group: Optional[dist.ProcessGroup] = None):
        self.model = model
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self._flat = None

    def __call__(self) -> None:
        if self.world <= 1:
            return
        grads = [p.grad for p in self.model.parameters() if p.grad is not None]
        if not grads:
            return
        total = sum(g.numel() for g in grads)
        if self._flat is None or self._flat.numel() != total or self._flat.device != grads[0].device:
            self._flat = torch.empty(total, dtype=grads[0].dtype, device=grads[0].device)
        views = []
        off = 0
        for g in grads:
            n = g.numel()
            views.append(self._flat[off:off + n].view_as(g))
            off += n
        torch._foreach_copy_(views, grads)
        dist.all_reduce(self._flat, op=dist.ReduceOp.SUM, group=self.group)
        self._flat.mul_(1.0 / self.world)
        torch._foreach_copy_(grads, views)


def train_step(model, batch, optimizer, criterion, normalizer=None, allreduce: Optional[GradAllReduce] = None,
               sync_metrics: bool = False):
    # graph + pooling structure for this batch, one host sync (cached per tensor)
    prepare(batch.edge_index, batch.x.size(0), batch.batch, getattr(batch, "num_graphs", None) or None)
    pred, _ = model(batch.x, batch.edge_index, batch.edge_attr, batch.batch)
    if normalizer is not None:
        loss = criterion(normalizer.denormalize_eigenvalue(pred), normalizer.denormalize_eigenvalue(batch.y))
    else:
        loss = criterion(pred, batch.y)
    optimizer.zero_grad(set_to_none=True)
    loss.backward()
    if allreduce is not None:
        allreduce()
    optimizer.step()
    if sync_metrics:
        return float(loss.item()), float(mape_error(pred.detach(), batch.y, normalizer).item())
    return loss.detach()
