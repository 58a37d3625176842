"""GPU: the data-parallel training loop of BASELINE configs[3] at its per-rank shape
(TRAIN_FINAL.py:246-298 over the DataLoader of :1298): two fresh worker processes
(spawned, gloo -- both ranks share cuda:0 on the one-GPU test box; the multi-GPU bench uses RCCL),
each training the fused GraphSage_addAggr (h = 512, dropout 0.1) on its DistributedSampler-style
shard of a device-resident GraphStore of cfg3 meshes (71x71 stiffened meshes with a super node of
in-degree 5,041 each, VirtualEdgeCreate.py:81-113; 16 graphs per rank and step, so the heavy-row
chunk / combine path runs under the hook-launched buckets), with GradAllReduce's ~4 MB buckets
overlapping the fused backward. Checked every step: the bucket layout is the same on both ranks;
the averaged gradients equal (g_0 + g_1) / 2 of the ranks' own gradients bit for bit; after Adam
the parameters are bit-identical across ranks. Step 0 runs with dropout 0 (torch's dropout RNG
cannot be matched) and rank 0's own step-0 gradients are bounded, whole tensor by whole tensor,
against the fp64 oracle on its batch (as tests/test_gpu_fullsize.py)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _gather(t):
    out = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return out


def _fp64_bound(sd0, batch, own, loss_g, norm):
    """Rank 0's step-0 gradients against the fp64 oracle on its batch: per parameter the L2
    distance within 1e-3 of the gradient's norm plus a floor of 1e-5 of the largest per-element
    RMS gradient (test_gpu_fullsize.py); the loss within 1e-4. Returns the largest error / bound."""
    import numpy as np
    from oracle import buckgnn_ref as R
    torch.set_num_threads(8)
    x, ei, b, y = (t.detach().cpu() for t in (batch.x, batch.edge_index, batch.batch, batch.y))
    st = {k: v.double().clone().requires_grad_(v.is_floating_point() and "running" not in k
                                               and "num_batches" not in k) for k, v in sd0.items()}
    pred_o = R.forward(st, "GraphSage_addAggr", x.double(), ei, b, True, "mean", 0.0)
    loss_o = R.relative_error_loss(norm.denormalize_eigenvalue(pred_o), norm.denormalize_eigenvalue(y.double()))
    loss_o.backward()
    assert abs(loss_g - float(loss_o)) <= 1e-4 * (1 + abs(float(loss_o))), (loss_g, float(loss_o))
    ref = {k: v.grad.numpy() for k, v in st.items() if v.grad is not None}
    got = {k: g.detach().cpu().double().numpy() for k, g in own.items() if g is not None}
    assert set(got) == set(ref), set(got) ^ set(ref)
    rms = max(np.sqrt(np.mean(r ** 2)) for r in ref.values())
    worst = 0.0
    for k in ref:
        err = float(np.linalg.norm(got[k] - ref[k]))
        bound = 1e-3 * float(np.linalg.norm(ref[k])) + 1e-5 * rms * np.sqrt(ref[k].size)
        assert err <= bound, (k, err, bound)
        worst = max(worst, err / bound)
    return worst


def _worker(rank, world, port, q):
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        import bgnn
        from bgnn import synthetic

        # 64 cfg3 meshes (71 x 71 nodes + a super node each), one store per rank holding the whole
        # dataset; each rank iterates its own shard of 32 (TRAIN_FINAL's loader, sharded)
        pool = [synthetic.make_mesh_graph(71, g, super_node=True) for g in range(64)]
        store = bgnn.GraphStore(pool, dev)
        torch.manual_seed(0)
        model = bgnn.BuckGNN(synthetic.NUM_NODE_FEATURES, synthetic.NUM_EDGE_FEATURES, hidden_channels=512,
                             num_layers=6, dropout_rate=0.1, model_name="GraphSage_addAggr")
        sd0 = {k: v.clone() for k, v in model.state_dict().items()}
        model = model.to(dev).train()
        opt = torch.optim.Adam(model.parameters(), lr=1e-2, weight_decay=1e-8)
        crit = bgnn.RelativeErrorLoss()
        norm = bgnn.EigenvalueScaler(center=1.0, scale=0.5)
        ar = bgnn.GradAllReduce(model, bucket_mb=4.0)
        params = [p for p in model.parameters()]
        stats = []
        step = 0
        epoch = 0
        while step < 3:
            for batch in store.loader(16, shuffle=True, seed=1234, epoch=epoch, rank=rank, world_size=world,
                                      drop_last=True):
                if step >= 3:
                    break
                bgnn.prepare(batch.edge_index, batch.x.size(0), batch.batch, batch.num_graphs)
                assert batch.num_graphs == 16 and batch.num_nodes == 16 * 5042
                torch.manual_seed(100 * step + rank)   # dropout seeds differ per rank, like separate runs
                model.dropout.p = 0.0 if step == 0 else 0.1
                pred, _ = model(batch.x, batch.edge_index, batch.edge_attr, batch.batch)
                loss = crit(norm.denormalize_eigenvalue(pred), norm.denormalize_eigenvalue(batch.y))
                opt.zero_grad(set_to_none=True)
                loss.backward()
                own = [None if p.grad is None else p.grad.detach().clone() for p in params]
                if step == 0 and rank == 0:
                    worst = _fp64_bound(sd0, batch, dict(zip([n for n, _ in model.named_parameters()], own)),
                                        float(loss), norm)
                ar()
                torch.cuda.synchronize()
                n_checked = 0
                for p, g in zip(params, own):
                    if g is None:
                        assert p.grad is None
                        continue
                    g0, g1 = _gather(g)
                    assert torch.equal(p.grad, (g0 + g1) / 2), "bucketed average differs from (g0 + g1) / 2"
                    n_checked += 1
                opt.step()
                flat = torch.cat([p.detach().reshape(-1) for p in params])
                f0, f1 = _gather(flat)
                assert torch.equal(f0, f1), "parameters differ across ranks after the step"
                stats.append((step, float(loss), n_checked, float(batch.num_nodes),
                              worst if (step == 0 and rank == 0) else None))
                step += 1
            epoch += 1
        layout = ar.layout
        lens = _gather(torch.tensor([len(layout)], device=dev))
        q.put((rank, "ok", layout, [int(x) for x in lens], stats))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:   # report instead of hanging the parent
        import traceback
        q.put((rank, "error", traceback.format_exc(), None, None))
        raise


def test_fused_model_ddp_two_ranks_gloo(dev):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r = q.get(timeout=170)
        res[r[0]] = r
    for p in procs:
        p.join(timeout=60)
    for r in res.values():
        assert r[1] == "ok", r[2]
    for p in procs:
        assert p.exitcode == 0
    lay0, lay1 = res[0][2], res[1][2]
    assert lay0 == lay1 and len(lay0) >= 2, (len(lay0), len(lay1))
    for rank in (0, 1):
        st = res[rank][4]
        assert [s[0] for s in st] == [0, 1, 2]
        assert all(s[2] > 20 for s in st)          # every used parameter's average checked
        assert all(s[3] == 16 * 5042 for s in st)   # cfg3's per-rank batch: 16 meshes + super nodes
    print("rank 0 step-0 gradients vs fp64: largest error / bound", res[0][4][0][4])
    # the ranks trained on different graphs
    assert [s[1] for s in res[0][4]] != [s[1] for s in res[1][4]]
