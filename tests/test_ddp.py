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


PORT = _free_port()
