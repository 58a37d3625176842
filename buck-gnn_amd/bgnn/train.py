"""Training-step driver and data-parallel gradient exchange.

`train_step` is the body of the reference's inner loop (TRAIN_FINAL.py:253-298)
for buckling targets: forward, RelativeErrorLoss on denormalised eigenvalues
(Utils/Losses.py:755-761, Dataset_Preparation/Normalizer.py:207-215), backward,
Adam step (TRAIN_FINAL.py:190). The reference's per-step `.item()` host syncs
(TRAIN_FINAL.py:263,298) are optional here (`sync_metrics`).

`GradAllReduce` is the one collective of the multi-GPU path: the
mini-batch is split by whole mesh graphs (no edge cuts), each rank runs its own
graphs, and the gradients of the parameters that received one are summed by RCCL
all-reduces of ~4 MB buckets launched during the backward (overlapped with the earlier
layers' backward) and divided by the world size. Parameters the
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
    """Sum-then-average gradients across ranks (SURVEY §8e's one exchange step).

    First step: one flat blocking all-reduce of every gradient that was produced, while
    post-accumulate-grad hooks record the order in which the gradients arrive. From then on
    (overlap=True) the gradients are grouped in that order into buckets of about
    `bucket_mb` MB; a bucket's asynchronous all-reduce is launched from the hook of its last
    gradient, i.e. while autograd is still computing the earlier layers' backward, and
    __call__ (after backward) only waits, scales and copies back. Buckets launch strictly in
    bucket order, so every rank issues the same collective sequence. Parameters that receive
    no gradient (the reference's unused modules) are never part of a bucket."""

    def __init__(self, model: nn.Module, group: Optional[dist.ProcessGroup] = None, bucket_mb: float = 4.0,
                 overlap: bool = True):
        self.model = model
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.bucket_bytes = int(bucket_mb * (1 << 20))
        self.overlap = overlap and self.world > 1
        self._flat = None
        self._seen = []            # gradient arrival order of the recording step
        self._buckets = None       # [(params, flat buffer, views)]
        self._bucket_of = {}
        self._ready = []
        self._next = 0
        self._works = []
        self._hooks = []
        if self.overlap:
            for p in model.parameters():
                if p.requires_grad:
                    self._hooks.append(p.register_post_accumulate_grad_hook(self._on_grad))

    # ---------------------------------------------------------------- overlap path
    def _on_grad(self, p: torch.Tensor) -> None:
        if self._buckets is None:
            self._seen.append(p)
            return
        b = self._bucket_of.get(id(p))
        if b is None:
            raise RuntimeError("GradAllReduce: a parameter without a gradient in the first step got one")
        self._ready[b] += 1
        while self._next < len(self._buckets) and self._ready[self._next] == len(self._buckets[self._next][0]):
            params, flat, views = self._buckets[self._next]
            torch._foreach_copy_(views, [q.grad for q in params])
            self._works.append(dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=self.group, async_op=True))
            self._next += 1

    def _build_buckets(self) -> None:
        order, seen = [], set()
        for p in self._seen:
            if id(p) not in seen and p.grad is not None:
                seen.add(id(p))
                order.append(p)
        self._seen = []
        buckets, cur, nbytes = [], [], 0
        for p in order:
            cur.append(p)
            nbytes += p.numel() * p.element_size()
            if nbytes >= self.bucket_bytes:
                buckets.append(cur)
                cur, nbytes = [], 0
        if cur:
            buckets.append(cur)
        self._buckets = []
        for b, params in enumerate(buckets):
            flat = torch.empty(sum(p.numel() for p in params), dtype=params[0].dtype, device=params[0].device)
            views, off = [], 0
            for p in params:
                views.append(flat[off:off + p.numel()].view_as(p))
                self._bucket_of[id(p)] = b
                off += p.numel()
            self._buckets.append((params, flat, views))
        self._ready = [0] * len(self._buckets)

    # ---------------------------------------------------------------- per step
    def __call__(self) -> None:
        if self.world <= 1:
            return
        if self.overlap and self._buckets is not None:
            if self._next != len(self._buckets):
                raise RuntimeError("GradAllReduce: not every bucket received all its gradients this step")
            for w in self._works:
                w.wait()
            inv = 1.0 / self.world
            for params, flat, views in self._buckets:
                flat.mul_(inv)
                torch._foreach_copy_([p.grad for p in params], views)
            self._works, self._next = [], 0
            self._ready = [0] * len(self._buckets)
            return
        grads = [p.grad for p in self.model.parameters() if p.grad is not None]
        if grads:
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
        if self.overlap:
            self._build_buckets()
            self._flat = None


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
