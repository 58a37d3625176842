"""GPU: EA_GNN at BASELINE configs[4]'s full per-GPU size -- 64 cfg2 meshes (64 x 71x71 with
virtual edges: N = 322,624 nodes, E = 2,863,488 directed edges), h = 512 -- the workload
`bench.py --model EA_GNN --bf16 --config cfg5` times (Models/BuckGNN.py:375-387, GraphNetBlock
:528-566).

At this size the bf16 edge GEMMs run M = E = 2.86 M rows: the ragged-last-tile whole-line bf16
epilogue, the LDS-staged gather indices and the drop-add dgrad epilogue on [E, 512] bf16 tensors of
2.9 GB, none of which the smaller EA tests reach (largest there: E = 178,968).

1. One GraphNetBlock forward + backward with bf16 GEMM operands and bf16 edge storage against the
   f32-accurate fused block on the same inputs; the bar is PyTorch's own bf16 (autocast's bf16
   Linear on the per-op block) against the same f32 result, as in
   tests/test_gpu_model.py::test_ea_gnn_bf16_block_close_to_f32: every output and input gradient
   within 1.5x of autocast's relative L2 error.
2. The whole 6-block model's Adam train steps (lr 1e-3, dropout 0): the bf16 step's loss within
   5e-2 of the f32-accurate step's, step by step, and both finite."""
import pytest
import torch

import bgnn
from bgnn import synthetic as S

pytestmark = pytest.mark.gpu

H = 512


@pytest.fixture(scope="module")
def cfg5_batch():
    b = S.make_config_batch("cfg5")
    assert (b.num_nodes, b.num_edges, int(b.batch.max()) + 1) == (322624, 2863488, 64)
    return b


def test_cfg5_graphnet_block_bf16_close_to_f32(dev, cfg5_batch):
    from bgnn.buckgnn import GraphNetBlock
    from bgnn.ea import graphnet_block
    b = cfg5_batch.to(dev)
    torch.manual_seed(0)
    blk = GraphNetBlock(H).to(dev)
    x0 = torch.randn(b.num_nodes, H, device=dev)
    e0 = torch.randn(b.num_edges, H, device=dev)
    gx, ge = torch.randn_like(x0), torch.randn_like(e0)

    def run(fn):
        x, e = x0.clone().requires_grad_(True), e0.clone().requires_grad_(True)
        xo, eo = fn(x, e)
        torch.autograd.backward([xo.float(), eo.float()], [gx, ge])
        out = [xo.detach().float(), eo.detach().float(), x.grad, e.grad]
        blk.zero_grad(set_to_none=True)
        return out

    def rel(a, r):
        return ((a - r).norm() / r.norm()).item()

    ref = run(lambda x, e: graphnet_block(blk, x, e, b.edge_index, bf16=False))
    for t in ref:
        assert bool(torch.isfinite(t).all())
    ours = [rel(o, r) for o, r in zip(run(lambda x, e: graphnet_block(blk, x, e, b.edge_index, bf16=True)), ref)]
    torch.cuda.empty_cache()

    def lin(v, m):   # autocast's bf16 Linear: bf16 operands and output, f32 accumulation
        return torch.nn.functional.linear(v.bfloat16(), m.weight.bfloat16(), m.bias.bfloat16())

    def autocast_block(x, e):
        row, col = b.edge_index
        relu = torch.relu
        xb = x.bfloat16()   # (rounded before the gathers: the same operands, a third of the bytes)
        e2 = lin(relu(lin(torch.cat([xb[row], xb[col], e.bfloat16()], 1), blk.edge_mlp[0])), blk.edge_mlp[2])
        m = lin(relu(lin(torch.cat([xb[col], e2], 1), blk.node_mlp_phi[0])), blk.node_mlp_phi[2])
        deg = torch.bincount(row, minlength=x.size(0)).clamp_min(1).float().unsqueeze(1)
        agg = torch.zeros_like(x).index_add(0, row, m.float()) / deg
        out = lin(relu(lin(torch.cat([x, agg], 1), blk.node_mlp_gamma[0])), blk.node_mlp_gamma[2]).float()
        return out + lin(relu(lin(out, blk.node_mlp_beta[0])), blk.node_mlp_beta[2]).float(), e2
    torch_bf16 = [rel(t, r) for t, r in zip(run(autocast_block), ref)]
    print("rel L2 vs the f32-accurate block (x, e, dx, de): bgnn bf16", [f"{v:.2e}" for v in ours],
          "autocast bf16", [f"{v:.2e}" for v in torch_bf16])
    for name, ro, rt in zip(("x", "e", "dx", "de"), ours, torch_bf16):
        assert 1e-6 < ro <= 1.5 * rt + 1e-4, (name, ro, rt)


def test_cfg5_ea_gnn_bf16_train_steps_follow_f32(dev, cfg5_batch):
    b = cfg5_batch.to(dev)
    crit, norm = bgnn.RelativeErrorLoss(), bgnn.EigenvalueScaler(1.0, 0.5)
    losses = {}
    for bf16 in (False, True):
        torch.manual_seed(0)
        model = bgnn.BuckGNN(16, 5, hidden_channels=H, num_layers=6, dropout_rate=0.0, model_name="EA_GNN").to(dev)
        model.train()
        model.ea_bf16 = bf16
        opt = torch.optim.Adam(model.parameters(), lr=1e-3, weight_decay=1e-8)
        losses[bf16] = [float(bgnn.train_step(model, b, opt, crit, norm)) for _ in range(3)]
        del model, opt
        torch.cuda.empty_cache()
    print("cfg5 EA_GNN losses f32-accurate", losses[False], "bf16", losses[True])
    for s, (a, r) in enumerate(zip(losses[True], losses[False])):
        assert torch.isfinite(torch.tensor(a)) and a == pytest.approx(r, rel=5e-2), (s, losses)
