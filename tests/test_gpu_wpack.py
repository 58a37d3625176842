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


def _fwd(model, b):
    with torch.no_grad():
        return model(b.x, b.edge_index, b.edge_attr, b.batch)[0]


def _fresh_fwd(model, b, monkeypatch):
    monkeypatch.setattr(fused, "PERSISTENT_WPACK", False)
    try:
        return _fwd(model, b)
    finally:
        monkeypatch.setattr(fused, "PERSISTENT_WPACK", True)


def test_pack_follows_in_place_writes(dev, monkeypatch):
    """Weight writes that bump no autograd version (through p.data) and ones that do (no_grad
    in-place ops) are both seen by the next forward: the pack is refilled on every call."""
    b1, _ = _batches(dev)
    bgnn.clear_caches()
    model = _model(dev).eval()
    y0 = _fwd(model, b1)
    assert torch.equal(y0, _fwd(model, b1))
    for conv in model.sage_blocks_add:
        conv.lin_l.weight.data.mul_(0.5)          # (no version bump)
    y1 = _fwd(model, b1)
    assert not torch.equal(y0, y1)
    assert torch.equal(y1, _fresh_fwd(model, b1, monkeypatch))
    with torch.no_grad():
        for conv in model.sage_blocks_add:
            conv.lin_r.weight.mul_(2.0)           # (version bump)
    y2 = _fwd(model, b1)
    assert not torch.equal(y1, y2)
    assert torch.equal(y2, _fresh_fwd(model, b1, monkeypatch))


def test_new_model_at_freed_addresses(dev, monkeypatch):
    """Model A evaluated and freed, model B of the same shapes built with different weights (the
    caching allocator may hand B A's addresses, with equal autograd versions): B's forward uses
    B's weights (INFERENCE.py evaluates one checkpoint after another this way)."""
    b1, _ = _batches(dev)
    bgnn.clear_caches()
    torch.manual_seed(1)
    a = bgnn.BuckGNN(16, 5, hidden_channels=128, num_layers=4, dropout_rate=0.0,
                     model_name="GraphSage_addAggr").to(dev).eval()
    ya = _fwd(a, b1)
    del a
    torch.manual_seed(2)
    b = bgnn.BuckGNN(16, 5, hidden_channels=128, num_layers=4, dropout_rate=0.0,
                     model_name="GraphSage_addAggr").to(dev).eval()
    yb = _fwd(b, b1)
    assert not torch.equal(ya, yb)
    assert torch.equal(yb, _fresh_fwd(b, b1, monkeypatch))


@pytest.mark.parametrize("variant", ["foreach", "fused", "for_loop"])
def test_adam_steps_match_fresh_pack(dev, monkeypatch, variant):
    """Three training steps under a real torch.optim.Adam (foreach, fused and for-loop forms):
    losses and parameters bit-identical to the fresh-concatenation path."""
    b1, b2 = _batches(dev)
    res = {}
    for persistent in (True, False):
        monkeypatch.setattr(fused, "PERSISTENT_WPACK", persistent)
        bgnn.clear_caches()
        model = _model(dev)
        kw = {"foreach": dict(foreach=True), "fused": dict(fused=True), "for_loop": dict(foreach=False)}[variant]
        opt = torch.optim.Adam(model.parameters(), lr=1e-2, **kw)
        losses = []
        for b in (b1, b2, b1):
            opt.zero_grad(set_to_none=True)
            p, _ = model(b.x, b.edge_index, b.edge_attr, b.batch)
            loss = p.square().mean()
            loss.backward()
            opt.step()
            losses.append(float(loss))
        res[persistent] = (losses, {n: t.detach().clone() for n, t in model.state_dict().items()})
    assert res[True][0] == res[False][0]
    for k, v in res[False][1].items():
        assert torch.equal(res[True][1][k], v), k
