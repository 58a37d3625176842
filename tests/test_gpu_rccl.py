"""GPU: the RCCL branch of the data-parallel step, executed on the one-GPU test box.

bench.py initialises the process group with backend "nccl" (RCCL on ROCm) and a `device_id`
(bench.py setup_dist) for N > 1; the multi-GPU runs are the driver's. Here one spawned process
initialises a world-size-1 "nccl" group the same way, and GradAllReduce runs with its test-only
`_force_collectives` switch, which keeps the collectives -- the recording step's flat blocking
all-reduce and, from step 2 on, the bucketed asynchronous all-reduces launched from autograd's
post-accumulate-grad hooks and waited on after the backward -- on at world size 1. The fused
GraphSage_addAggr (h = 512) trains three steps; every step's gradients after the all-reduce must
equal the backward's own gradients bit for bit (the sum over one rank and the 1/world scale are
exact), and the hook path must have issued asynchronous RCCL all-reduces (TRAIN_FINAL.py:246-298
is the loop; the reference itself has no distributed code)."""
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


def _worker(port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1")
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)   # as bench.py setup_dist
        assert dist.get_backend() == "nccl"
        import bgnn
        from bgnn import synthetic

        issued = []
        real_all_reduce = dist.all_reduce

        def counting(t, *a, **k):
            issued.append((bool(k.get("async_op", False)), t.numel(), t.device.type))
            return real_all_reduce(t, *a, **k)
        dist.all_reduce = counting
        batch = synthetic.make_batch(31, 4).to(dev)
        torch.manual_seed(0)
        model = bgnn.BuckGNN(synthetic.NUM_NODE_FEATURES, synthetic.NUM_EDGE_FEATURES, hidden_channels=512,
                             num_layers=6, dropout_rate=0.1, model_name="GraphSage_addAggr").to(dev).train()
        opt = torch.optim.Adam(model.parameters(), lr=1e-3, weight_decay=1e-8)
        crit = bgnn.RelativeErrorLoss()
        ar = bgnn.GradAllReduce(model, bucket_mb=4.0, _force_collectives=True)
        params = list(model.parameters())
        steps = []
        for step in range(3):
            n0 = len(issued)
            pred, _ = model(batch.x, batch.edge_index, batch.edge_attr, batch.batch)
            loss = crit(pred, batch.y)
            opt.zero_grad(set_to_none=True)
            loss.backward()
            torch.cuda.synchronize()
            n_hook = len(issued) - n0   # launched from the hooks while the backward ran
            own = [None if p.grad is None else p.grad.detach().clone() for p in params]
            ar()
            torch.cuda.synchronize()
            for p, g in zip(params, own):
                if g is None:
                    assert p.grad is None
                else:
                    assert torch.equal(p.grad, g), "gradient changed by the world-1 RCCL all-reduce"
            opt.step()
            steps.append((n_hook, len(issued) - n0, sum(g is not None for g in own), float(loss)))
        q.put(("ok", steps, issued, len(ar.layout or [])))
        dist.destroy_process_group()
    except Exception:
        import traceback
        q.put(("error", traceback.format_exc(), None, None))
        raise


def test_rccl_world1_bucketed_allreduce_keeps_gradients(dev):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(_free_port(), q))
    p.start()
    res = q.get(timeout=150)
    p.join(timeout=60)
    assert res[0] == "ok", res[1]
    assert p.exitcode == 0
    steps, issued, n_buckets = res[1], res[2], res[3]
    print("per step (hook-launched all-reduces, all-reduces, gradients, loss):", steps, "buckets:", n_buckets)
    assert all(d == "cuda" for _, _, d in issued)
    # step 0: the recording step, one flat blocking all-reduce after the backward
    assert steps[0][0] == 0 and steps[0][1] == 1 and not issued[0][0]
    # steps 1, 2: every bucket's async all-reduce launched from a hook during the backward
    assert n_buckets >= 2
    for s in steps[1:]:
        assert s[0] == n_buckets and s[1] == n_buckets, steps
    assert all(a for a, _, _ in issued[1:])
