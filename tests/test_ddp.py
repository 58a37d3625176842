"""Multi-process data-parallel path on CPU (gloo, world_size 2): the mini-batch is
split by whole graphs (no edge cuts) and GradAllReduce averages gradients with one
flat all-reduce, skipping parameters without gradients."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class Tiny(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.a = torch.nn.Linear(4, 3)
        self.unused = torch.nn.Linear(3, 3)   # like edge_encoder / sage_mlps in the reference


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bgnn
    from bgnn import synthetic

    torch.manual_seed(0)
    m = Tiny()
    torch.manual_seed(100 + rank)
    x = torch.randn(8, 4)
    m.a(x).pow(2).sum().backward()
    own = m.a.weight.grad.clone()
    bgnn.GradAllReduce(m)()
    # per-rank graph shards are different graphs of the same shape
    b = synthetic.make_batch(6, 2, seed0=1000 * rank)
    q.put((rank, own, m.a.weight.grad.clone(), m.a.bias.grad.clone(), m.unused.weight.grad,
           b.edge_index.shape, float(b.x.sum())))
    dist.barrier()
    dist.destroy_process_group()


def test_grad_allreduce_gloo_world2():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, PORT, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    avg = (res[0][1] + res[1][1]) / 2
    for r in res:
        torch.testing.assert_close(r[2], avg)
        assert r[4] is None                     # parameters without grads are skipped
    torch.testing.assert_close(res[0][3], res[1][3])
    assert res[0][5] == res[1][5] and res[0][6] != res[1][6]


class Deep(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.layers = torch.nn.ModuleList([torch.nn.Linear(16, 16) for _ in range(5)])
        self.unused = torch.nn.Linear(16, 16)

    def forward(self, x):
        for i, l in enumerate(self.layers):
            x = torch.relu(l(x)) + (x if i else 0)
        return x


def _worker_overlap(rank, world, port, q):
    """Three steps with bucketed all-reduces launched from the gradient hooks (several buckets)
    against the flat blocking all-reduce: identical averaged gradients every step."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bgnn

    out = []
    for overlap in (True, False):
        torch.manual_seed(0)
        m = Deep()
        ar = bgnn.GradAllReduce(m, bucket_mb=0.001, overlap=overlap)   # ~1 KB buckets: one per layer
        grads = []
        for step in range(3):
            torch.manual_seed(100 * step + rank)
            m.zero_grad(set_to_none=True)
            m(torch.randn(8, 16)).pow(2).sum().backward()
            ar()
            grads.append([p.grad.numpy().copy() for p in m.layers.parameters()])
            assert m.unused.weight.grad is None
        out.append((grads, len(ar._buckets) if ar._buckets else 0))
    q.put((rank, out))
    dist.barrier()
    dist.destroy_process_group()


def test_grad_allreduce_overlapped_buckets_gloo_world2():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_overlap, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, ((g_ov, nb), (g_flat, _)) in res:
        assert nb == 5
        for a, b in zip(g_ov, g_flat):
            for x, y in zip(a, b):
                assert (x == y).all()
    for x, y in zip(res[0][1][0][0][-1], res[1][1][0][0][-1]):
        assert (x == y).all()   # every rank holds the same average


PORT = _free_port()


class Optional_(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.layers = torch.nn.ModuleList([torch.nn.Linear(16, 16) for _ in range(3)])
        self.opt = torch.nn.Linear(16, 16)

    def forward(self, x, use_opt: bool):
        for l in self.layers:
            x = torch.relu(l(x))
        return self.opt(x) if use_opt else x


def _worker_unused(rank, world, port, q):
    """Hook-launched buckets when a module is skipped after the recording step: by one rank (it
    takes the other rank's gradient / world, like DDP) and by every rank (it keeps grad None, so
    the optimizer skips it)."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bgnn

    torch.manual_seed(0)
    m = Optional_()
    ar = bgnn.GradAllReduce(m, bucket_mb=0.001)
    res = []
    for step, use in enumerate([(True, True), (True, False), (False, False)]):
        torch.manual_seed(100 * step + rank)
        m.zero_grad(set_to_none=True)
        m(torch.randn(8, 16), use[rank]).pow(2).sum().backward()
        own = None if m.opt.weight.grad is None else m.opt.weight.grad.clone()
        ar()
        res.append((own, None if m.opt.weight.grad is None else m.opt.weight.grad.clone(),
                    m.layers[0].weight.grad.clone()))
    q.put((rank, res))
    dist.barrier()
    dist.destroy_process_group()


def test_grad_allreduce_unused_after_recording_gloo_world2():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_unused, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    r0, r1 = res[0], res[1]
    # step 1: rank 1 skipped `opt`: both ranks hold rank 0's gradient / 2
    own0 = r0[1][0]
    assert r1[1][0] is None
    torch.testing.assert_close(r0[1][1], own0 / 2)
    torch.testing.assert_close(r1[1][1], own0 / 2)
    # step 2: no rank used it: no gradient anywhere; the used layers are still averaged
    assert r0[2][1] is None and r1[2][1] is None
    torch.testing.assert_close(r0[2][2], r1[2][2])
