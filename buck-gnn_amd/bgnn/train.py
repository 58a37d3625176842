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


class _RelErrorLossFn(torch.autograd.Function):
    """RelativeErrorLoss of the denormalised prediction and target in one launch
    (bgnn_rel_error_loss: loss and d loss / d pred together); backward one multiply."""

    @staticmethod
    def forward(ctx, pred, y, scale: float, center: float, eps: float):
        from . import _lib
        from .graph import _stream
        pred = pred.contiguous()
        y = y.contiguous()
        loss = torch.empty((), dtype=torch.float32, device=pred.device)
        dpred = torch.empty_like(pred)
        _lib.call("bgnn_rel_error_loss", pred.data_ptr(), y.data_ptr(), pred.numel(), float(scale), float(center),
                  float(eps), loss.data_ptr(), dpred.data_ptr(), _stream())
        ctx.save_for_backward(dpred)
        return loss

    @staticmethod
    def backward(ctx, g):
        (dpred,) = ctx.saved_tensors
        return dpred * g, None, None, None, None


# train_step's loss: RelativeErrorLoss on EigenvalueScaler-denormalised values as one HIP launch
FUSED_LOSS = True


def _fused_loss(criterion, normalizer, pred, y):
    """criterion(denorm(pred), denorm(y)) through _RelErrorLossFn when that is exactly what the
    reference computes (TRAIN_FINAL.py:267-270 with Utils/Losses.py:755-761), else None."""
    if not (FUSED_LOSS and type(criterion) is RelativeErrorLoss and pred.is_cuda and pred.dtype == torch.float32
            and y.dtype == torch.float32 and pred.shape == y.shape and pred.numel() > 0):
        return None
    if normalizer is None:
        scale, center = 1.0, 0.0
    elif type(normalizer) is EigenvalueScaler:
        scale, center = normalizer.scale, normalizer.center
    else:
        return None
    return _RelErrorLossFn.apply(pred, y, scale, center, criterion.epsilon)


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
                 overlap: bool = True, _force_collectives: bool = False):
        self.model = model
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.bucket_bytes = int(bucket_mb * (1 << 20))
        # test-only: issue the collectives (hook-launched buckets included) even at world size 1,
        # so a one-GPU box runs the RCCL path for real (tests/test_gpu_rccl.py); at world 1 the
        # sum and the 1/world scale are exact, the gradients come back unchanged
        self._force = bool(_force_collectives) and dist.is_initialized()
        self.overlap = overlap and (self.world > 1 or self._force)
        self._flat = None
        self._seen = []            # gradient arrival order of the recording step
        self._buckets = None       # [(params, flat buffer, views)]
        self._bucket_of = {}
        self._ready = []
        self._next = 0
        self._works = []
        self._extra = []
        self.layout = None         # bucket layout (parameter indices), identical on every rank
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
        if b is None:   # reported by __call__ once this step's collectives are issued
            self._extra.append(p)
            return
        self._ready[b] += 1
        while self._next < len(self._buckets) and self._ready[self._next] == len(self._buckets[self._next][0]):
            params, flat, views = self._buckets[self._next]
            torch._foreach_copy_(views, [q.grad for q in params])
            flat[-len(params):].fill_(1.0)   # every parameter of the bucket has a gradient on this rank
            self._works.append(dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=self.group, async_op=True))
            self._next += 1

    def _build_buckets(self) -> None:
        """Bucket layout from the recording step's gradient arrival order. The layout must be the
        same on every rank (a hook-launched all-reduce of bucket b sums bucket b of every rank),
        but arrival order is data-dependent (the fold / encoder paths switch on the batch size),
        so rank 0's order is broadcast and used everywhere (DDP's rebuilt-buckets approach);
        every rank checks that it has gradients for exactly the same parameters and all ranks
        raise together if any differs."""
        params = [p for p in self.model.parameters() if p.requires_grad]
        index = {id(p): i for i, p in enumerate(params)}
        order, seen = [], set()
        for p in self._seen:
            if id(p) not in seen and p.grad is not None:
                seen.add(id(p))
                order.append(index[id(p)])
        self._seen = []
        if self.world > 1:
            dev = params[0].device if params else torch.device("cpu")
            # the group's rank 0 as a global rank (broadcast's src is global)
            src = dist.get_global_rank(self.group, 0) if self.group is not None else 0
            n = torch.tensor([len(order)], dtype=torch.long, device=dev)
            dist.broadcast(n, src, group=self.group)
            ref = torch.tensor(order if dist.get_rank(self.group) == 0 else [0] * int(n.item()),
                               dtype=torch.long, device=dev)
            dist.broadcast(ref, src, group=self.group)
            ref = ref.tolist()
            ok = torch.tensor([int(sorted(ref) == sorted(order))], dtype=torch.long, device=dev)
            dist.all_reduce(ok, op=dist.ReduceOp.MIN, group=self.group)
            if not int(ok.item()):
                raise RuntimeError("GradAllReduce: the ranks produced gradients for different parameter sets "
                                   "in the recording step; the bucket layout cannot be shared")
            order = ref
        buckets, cur, nbytes = [], [], 0
        for i in order:
            p = params[i]
            cur.append(p)
            nbytes += p.numel() * p.element_size()
            if nbytes >= self.bucket_bytes:
                buckets.append(cur)
                cur, nbytes = [], 0
        if cur:
            buckets.append(cur)
        self._buckets = []
        self.layout = [[index[id(p)] for p in b] for b in buckets]   # parameter indices per bucket
        for b, bparams in enumerate(buckets):
            # [gradients | one "had a gradient" flag per parameter]: the flags are summed with the
            # gradients, so after the all-reduce a parameter some rank used is told apart from one
            # no rank used (which keeps grad None, as under DDP: Adam then skips it)
            flat = torch.empty(sum(p.numel() for p in bparams) + len(bparams), dtype=bparams[0].dtype,
                               device=bparams[0].device)
            views, off = [], 0
            for p in bparams:
                views.append(flat[off:off + p.numel()].view_as(p))
                self._bucket_of[id(p)] = b
                off += p.numel()
            self._buckets.append((bparams, flat, views))
        self._ready = [0] * len(self._buckets)

    def _launch_rest(self) -> None:
        """Launch the buckets whose gradients did not all arrive this step, with zeros (and a zero
        flag) for the missing ones, so every rank still issues the same collective sequence."""
        while self._next < len(self._buckets):
            params, flat, views = self._buckets[self._next]
            flags = flat[-len(params):]
            for i, (p, v) in enumerate(zip(params, views)):
                if p.grad is None:
                    v.zero_()
                    flags[i].fill_(0.0)
                else:
                    v.copy_(p.grad)
                    flags[i].fill_(1.0)
            self._works.append(dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=self.group, async_op=True))
            self._next += 1

    # ---------------------------------------------------------------- per step
    def __call__(self) -> None:
        if self.world <= 1 and not self._force:
            return
        if self.overlap and self._buckets is not None:
            self._launch_rest()
            for w in self._works:
                w.wait()
            inv = 1.0 / self.world
            for params, flat, views in self._buckets:
                flat.mul_(inv)
                if any(p.grad is None for p in params):
                    # unused on this rank this step: it takes the others' average (DDP), unless no
                    # rank used it -- then it keeps no gradient (one host read, this path only)
                    used = flat[-len(params):].tolist()
                    keep = [i for i, p in enumerate(params) if p.grad is not None or used[i] > 0]
                    for i in keep:
                        if params[i].grad is None:
                            params[i].grad = torch.zeros_like(params[i])
                    if keep:
                        torch._foreach_copy_([params[i].grad for i in keep], [views[i] for i in keep])
                else:
                    torch._foreach_copy_([p.grad for p in params], views)
            extra = self._extra
            self._extra = []
            self._works, self._next = [], 0
            self._ready = [0] * len(self._buckets)
            if extra:   # (after this step's collectives, so the other ranks are not left blocked)
                raise RuntimeError(f"GradAllReduce: {len(extra)} parameter(s) without a gradient in the "
                                   "recording step got one; they are in no bucket")
            return
        if self.overlap:   # layout (and the parameter-set check) before the first gradient collective
            self._build_buckets()
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
            self._flat = None


def train_step(model, batch, optimizer, criterion, normalizer=None, allreduce: Optional[GradAllReduce] = None,
               sync_metrics: bool = False):
    # graph + pooling structure for this batch, one host sync (cached per tensor)
    prepare(batch.edge_index, batch.x.size(0), batch.batch, getattr(batch, "num_graphs", None) or None)
    pred, _ = model(batch.x, batch.edge_index, batch.edge_attr, batch.batch)
    loss = _fused_loss(criterion, normalizer, pred, batch.y)
    if loss is None:
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
