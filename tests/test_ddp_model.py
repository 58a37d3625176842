"""GradAllReduce over the real BuckGNN parameter set (gloo, world size 2, CPU).

The fused SAGE path needs a GPU, so each rank produces its gradients with a dense CPU
surrogate of the same forward (encoder -> 6 x [lin_l + lin_r, normalize, BN, ReLU, skip] ->
mean -> decoder; the aggregation is left out): the same parameters receive gradients, in the
same per-layer order (decoder first, encoder last), and the reference's unused modules
(edge_encoder, sage_mlps, batch_norm, pooling_mpl) receive none. Checked (SURVEY §8e,
DESIGN §6): the ~4 MB bucket layout is identical on every rank even when the ranks' gradient
arrival orders differ, the hook-launched bucketed average equals the flat blocking all-reduce
bit for bit over three steps, and a rank with a different parameter set makes every rank raise.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn.functional as F


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _surrogate_loss(m, x):
    h = m.node_encoder(x)
    shared = m.model_name == "GraphSage_addAggr_Shared"
    convs = [m.shared_graphsage_block] * m.num_layers if shared else list(m.sage_blocks_add)
    L = len(convs)
    for i, conv in enumerate(convs):
        prev = h
        o = F.normalize(F.linear(h, conv.lin_l.weight, conv.lin_l.bias) + F.linear(h, conv.lin_r.weight), dim=-1)
        if not shared:
            bn = m.batch_norms[i]
            o = F.batch_norm(o, None, None, bn.weight, bn.bias, training=True)
        h = torch.relu(o)
        if 0 < i < L - 1:
            h = h + prev
    return m.decoder(h.mean(0, keepdim=True)).pow(2).sum()


def _worker(rank, world, port, name, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(2)
    import bgnn

    out = {}
    for overlap in (True, False):
        torch.manual_seed(0)
        m = bgnn.BuckGNN(16, 5, hidden_channels=512, num_layers=6, model_name=name)
        ar = bgnn.GradAllReduce(m, bucket_mb=4.0, overlap=overlap)
        grads = []
        for step in range(3):
            torch.manual_seed(100 * step + rank)
            m.zero_grad(set_to_none=True)
            _surrogate_loss(m, torch.randn(32, 16)).backward()
            if step == 0 and rank == 1 and overlap:
                ar._seen.reverse()   # a different arrival order on this rank: the layout must not follow it
            ar()
            grads.append({k: p.grad.numpy().copy() for k, p in m.named_parameters() if p.grad is not None})
        no_grad = sorted(k for k, p in m.named_parameters() if p.grad is None)
        used = sum(p.numel() for p in m.parameters() if p.grad is not None)
        out[overlap] = (grads, ar.layout, no_grad, used)
    q.put((rank, out))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("name,n_buckets,used", [("GraphSage_addAggr", 4, 3304385),
                                                 ("GraphSage_addAggr_Shared", 1, 674241)])
def test_grad_allreduce_real_model_gloo_world2(name, n_buckets, used):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, name, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank in range(world):
        (g_ov, layout, no_grad, n_used), (g_flat, _, no_grad_f, _) = res[rank][True], res[rank][False]
        assert n_used == used                                   # SURVEY §8e's used-parameter count
        assert len(layout) == n_buckets                         # ~4 MB buckets
        assert no_grad == no_grad_f
        assert any(k.startswith("edge_encoder") for k in no_grad) and any(k.startswith("pooling_mpl") for k in no_grad)
        for a, b in zip(g_ov, g_flat):
            assert a.keys() == b.keys()
            for k in a:
                assert (a[k] == b[k]).all(), k               # bucketed == flat, bit for bit
    assert res[0][True][1] == res[1][True][1]                   # same layout although rank 1's order differed
    for k in res[0][True][0][-1]:
        assert (res[0][True][0][-1][k] == res[1][True][0][-1][k]).all()   # every rank holds the same average


def _worker_mismatch(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bgnn

    torch.manual_seed(0)
    m = bgnn.BuckGNN(16, 5, hidden_channels=64, num_layers=2, model_name="GraphSage_addAggr")
    ar = bgnn.GradAllReduce(m, bucket_mb=0.01)
    loss = _surrogate_loss(m, torch.randn(8, 16))
    if rank == 1:   # a parameter set that differs from rank 0's
        loss = loss + m.sage_mlps[0].weight.sum()
    loss.backward()
    try:
        ar()
        q.put((rank, "no error"))
    except RuntimeError as e:
        q.put((rank, str(e)))
    dist.destroy_process_group()


def test_grad_allreduce_parameter_set_mismatch_raises_on_every_rank():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_mismatch, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    assert all("different parameter sets" in res[r] for r in range(world)), res
