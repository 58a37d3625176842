"""GPU: the PyG-surface SAGEConv module (bgnn.nn.SAGEConv) on its hand-written path
(bgnn.fused.SageConvFn: f16x3 MFMA transform + fused aggregation / bias / L2 normalize, and
its backward) against the fp64 oracle SAGEConv (oracle/pyg_ref.py, PyG's documented formula),
output and every gradient at the north star's 1e-4; it is the module the reference's unchanged
Models/BuckGNN.py:135-149,434 builds and calls under bgnn.install_pyg_shim()."""
import pytest
import torch

import bgnn
from bgnn import fused, nn as bnn
from bgnn import synthetic as S
from oracle import pyg_ref as P

pytestmark = pytest.mark.gpu
TOL = dict(rtol=1e-4, atol=1e-4)


def _run(dev, aggr, H, Cin, super_node, bias=True, seed=0):
    b = S.make_batch(11, 3, super_node=super_node)
    torch.manual_seed(seed)
    conv = bnn.SAGEConv(in_channels=Cin, out_channels=H, normalize=True, aggr=aggr, bias=bias)
    ref = P.SAGEConv(Cin, H, aggr=aggr, normalize=True, bias=bias).double()
    ref.load_state_dict({k: v.double() for k, v in conv.state_dict().items()})
    conv = conv.to(dev)
    x = torch.randn(b.num_nodes, Cin)
    up = torch.randn(b.num_nodes, H)
    xd = x.to(dev).requires_grad_(True)
    out = conv(xd, b.edge_index.to(dev))
    out.backward(up.to(dev))
    xr = x.double().requires_grad_(True)
    ro = ref(xr, b.edge_index)
    ro.backward(up.double())
    return conv, ref, out, ro, xd, xr


@pytest.mark.parametrize("aggr", ["add", "sum", "mean", "max"])
@pytest.mark.parametrize("H,Cin", [(64, 64), (512, 512), (512, 128)])
@pytest.mark.parametrize("super_node", [False, True])
def test_sageconv_module_fast_path_matches_oracle(dev, monkeypatch, aggr, H, Cin, super_node):
    calls = []
    real = fused.SageConvFn.apply
    monkeypatch.setattr(fused.SageConvFn, "apply", lambda *a: calls.append(1) or real(*a))
    conv, ref, out, ro, xd, xr = _run(dev, aggr, H, Cin, super_node)
    assert calls, "SAGEConv did not take the hand-written path"
    torch.testing.assert_close(out.detach().cpu(), ro.detach().float(), **TOL)
    torch.testing.assert_close(xd.grad.cpu(), xr.grad.float(), **TOL)
    for (k, p), (_, q) in zip(conv.named_parameters(), ref.named_parameters()):
        torch.testing.assert_close(p.grad.cpu(), q.grad.float(), **TOL, msg=k)


def test_sageconv_module_no_bias(dev):
    conv, ref, out, ro, xd, xr = _run(dev, "add", 128, 128, True, bias=False)
    torch.testing.assert_close(out.detach().cpu(), ro.detach().float(), **TOL)
    torch.testing.assert_close(conv.lin_l.weight.grad.cpu(), ref.lin_l.weight.grad.float(), **TOL)


def test_sageconv_module_paths_agree(dev, monkeypatch):
    """Fast path against the aggregate-first path (torch Linear + F.normalize) of the same module."""
    res = []
    for fast in (True, False):
        monkeypatch.setattr(bnn, "FAST_SAGECONV", fast)
        conv, ref, out, ro, xd, xr = _run(dev, "add", 512, 512, True, seed=3)
        res.append((out.detach(), xd.grad, conv.lin_l.weight.grad, conv.lin_r.weight.grad, conv.lin_l.bias.grad))
    for a, c in zip(*res):
        torch.testing.assert_close(a, c, rtol=1e-4, atol=1e-5)


def test_per_op_model_uses_hand_written_gemm(dev, monkeypatch):
    """bgnn.BuckGNN with use_fused=False (the module graph the PyG shim gives the reference's
    Models/BuckGNN.py) runs every SAGE layer's transform on the bgnn GEMM, not torch.mm."""
    n_gemm = []
    real = fused.gemm
    monkeypatch.setattr(fused, "gemm", lambda *a, **k: n_gemm.append(1) or real(*a, **k))
    b = S.make_batch(20, 4).to(dev)
    torch.manual_seed(0)
    m = bgnn.BuckGNN(16, 5, hidden_channels=512, num_layers=6, dropout_rate=0.0,
                     model_name="GraphSage_addAggr").to(dev)
    m.use_fused = False
    pred, _ = m(b.x, b.edge_index, b.edge_attr, b.batch)
    assert len(n_gemm) == 6
    pred.sum().backward()
    assert len(n_gemm) == 6 + 12   # dgrad + wgrad per layer
