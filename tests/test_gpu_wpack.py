"""GPU: the persistent [W_l;W_r] weight pack of the fused SAGE loop (bgnn.fused._weight_pack) is
safe when a second forward runs before the first backward (round-3 ADVICE, medium): two
micro-batches summed into one backward, and a no_grad eval forward between a training forward and
its backward. Gradients must equal those of the fresh-concatenation path
(fused.PERSISTENT_WPACK = False), bit for bit: the pack only changes where the operands live."""
import pytest
import torch

import bgnn
from bgnn import fused
from bgnn import synthetic as S
from bgnn.data import Batch

pytestmark = pytest.mark.gpu


def _model(dev):
    torch.manual_seed(0)
    return bgnn.BuckGNN(16, 5, hidden_channels=128, num_layers=4, dropout_rate=0.0,
                        model_name="GraphSage_addAggr").to(dev).train()


def _batches(dev):
    b1 = Batch.from_data_list([S.make_mesh_graph(30, seed=s) for s in range(3)]).to(dev)
    b2 = Batch.from_data_list([S.make_mesh_graph(30, seed=10 + s) for s in range(3)]).to(dev)
    return b1, b2


def _grads(model):
    return {n: p.grad.detach().clone() for n, p in model.named_parameters() if p.grad is not None}


@pytest.mark.parametrize("between", ["second_microbatch", "eval_forward"])
def test_second_forward_before_backward(dev, monkeypatch, between):
    b1, b2 = _batches(dev)
    out = {}
    for persistent in (False, True):
        monkeypatch.setattr(fused, "PERSISTENT_WPACK", persistent)
        fused._WPACK.clear()
        bgnn.clear_caches()
        model = _model(dev)
        model.zero_grad(set_to_none=True)
        p1, _ = model(b1.x, b1.edge_index, b1.edge_attr, b1.batch)
        loss = p1.square().sum()
        if between == "second_microbatch":
            p2, _ = model(b2.x, b2.edge_index, b2.edge_attr, b2.batch)
            loss = loss + p2.square().sum()
        else:
            model.eval()
            with torch.no_grad():
                model(b2.x, b2.edge_index, b2.edge_attr, b2.batch)
            model.train()
        loss.backward()
        out[persistent] = (float(loss), _grads(model))
    assert out[True][0] == out[False][0]
    assert out[True][1].keys() == out[False][1].keys() and len(out[True][1]) > 0
    for k in out[False][1]:
        assert torch.equal(out[True][1][k], out[False][1][k]), k


def test_pack_refilled_after_optimizer_step(dev):
    """After an in-place weight update the next forward sees the new weights (the pack follows
    the weights' autograd versions), and the pack is reused while they are unchanged."""
    b1, _ = _batches(dev)
    fused._WPACK.clear()
    bgnn.clear_caches()
    model = _model(dev)
    model.eval()
    with torch.no_grad():
        y0, _ = model(b1.x, b1.edge_index, b1.edge_attr, b1.batch)
        n_packs = len(fused._WPACK)
        y0b, _ = model(b1.x, b1.edge_index, b1.edge_attr, b1.batch)
        assert len(fused._WPACK) == n_packs and torch.equal(y0, y0b)
        for conv in model.sage_blocks_add:
            conv.lin_l.weight.mul_(0.5)
        y1, _ = model(b1.x, b1.edge_index, b1.edge_attr, b1.batch)
    assert not torch.equal(y0, y1)
    fused._WPACK.clear()
    with torch.no_grad():
        y1_fresh, _ = model(b1.x, b1.edge_index, b1.edge_attr, b1.batch)
    assert torch.equal(y1, y1_fresh)
