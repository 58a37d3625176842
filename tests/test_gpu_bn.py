"""GPU: bgnn.nn.BatchNorm1d (csrc/bn.hip, the opt-in BatchNorm of the per-module path) against
torch.nn.BatchNorm1d in fp64 on the CPU: train and eval, affine or not, tracked or untracked
running statistics, momentum None (cumulative average); output, input gradient, weight and bias
gradients at 1e-4 and the running statistics at 1e-5 (Models/BuckGNN.py:133,148,163,179,436)."""
import copy

import pytest
import torch

import bgnn
from bgnn import nn as bnn

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("training", [True, False])
@pytest.mark.parametrize("affine,track,momentum", [(True, True, 0.1), (False, True, 0.1), (True, False, 0.1),
                                                  (True, True, None)])
@pytest.mark.parametrize("N,C", [(5041, 512), (1000, 64), (37, 128)])
def test_bgnn_batchnorm_matches_torch(dev, training, affine, track, momentum, N, C):
    torch.manual_seed(N + C)
    ref = torch.nn.BatchNorm1d(C, affine=affine, track_running_stats=track, momentum=momentum).double()
    if affine:
        with torch.no_grad():
            ref.weight.uniform_(0.5, 1.5)
            ref.bias.uniform_(-0.2, 0.2)
    if track:
        with torch.no_grad():
            ref.running_mean.uniform_(-0.1, 0.1)
            ref.running_var.uniform_(0.8, 1.2)
            ref.num_batches_tracked.fill_(3)
    ours = bnn.use_bgnn_batchnorm(copy.deepcopy(ref).float().to(dev))
    assert type(ours) is bnn.BatchNorm1d
    ref.train(training)
    ours.train(training)
    x = torch.randn(N, C, dtype=torch.float64) * 0.3 + 0.05
    g = torch.randn(N, C, dtype=torch.float64)
    calls = []
    real = bnn._BatchNormFn.apply
    bnn._BatchNormFn.apply = lambda *a: calls.append(1) or real(*a)
    try:
        for step in range(2):   # two steps: running statistics and num_batches_tracked evolve alike
            xr = x.clone().requires_grad_(True)
            xo = x.float().to(dev).requires_grad_(True)
            yr = ref(xr)
            yo = ours(xo)
            yr.backward(g)
            yo.backward(g.float().to(dev))
            torch.testing.assert_close(yo.detach().cpu(), yr.detach().float(), rtol=1e-4, atol=1e-4)
            torch.testing.assert_close(xo.grad.cpu(), xr.grad.float(), rtol=1e-4, atol=1e-4)
            if affine:
                torch.testing.assert_close(ours.weight.grad.cpu(), ref.weight.grad.float(), rtol=1e-4, atol=1e-3)
                torch.testing.assert_close(ours.bias.grad.cpu(), ref.bias.grad.float(), rtol=1e-4, atol=1e-3)
                ours.weight.grad = ours.bias.grad = ref.weight.grad = ref.bias.grad = None
            if track:
                torch.testing.assert_close(ours.running_mean.cpu(), ref.running_mean.float(), rtol=1e-5, atol=1e-6)
                torch.testing.assert_close(ours.running_var.cpu(), ref.running_var.float(), rtol=1e-5, atol=1e-6)
                assert int(ours.num_batches_tracked) == int(ref.num_batches_tracked)
    finally:
        bnn._BatchNormFn.apply = real
    assert len(calls) == 2
    assert set(ours.state_dict()) == set(ref.state_dict())


def test_per_op_model_with_bgnn_batchnorm_matches_torch_batchnorm(dev):
    """The per-module model graph (bgnn.BuckGNN use_fused=False, the module graph the shim gives
    the reference's Models/BuckGNN.py) with bgnn BatchNorm1d equals the same model with torch's."""
    from bgnn import synthetic as S
    b = S.make_batch(20, 3, super_node=True).to(dev)
    res = []
    for mode in ("torch", "bgnn"):
        torch.manual_seed(0)
        m = bgnn.BuckGNN(16, 5, hidden_channels=512, num_layers=6, dropout_rate=0.0,
                         model_name="GraphSage_addAggr").to(dev)
        m.use_fused = False
        if mode == "bgnn":
            bnn.use_bgnn_batchnorm(m)
        pred, _ = m(b.x, b.edge_index, b.edge_attr, b.batch)
        pred.sum().backward()
        res.append([pred.detach()] + [p.grad for p in m.sage_blocks_add.parameters()]
                   + [p.grad for p in m.batch_norms.parameters()] + [m.batch_norms[2].running_var.clone()])
    for a, c in zip(*res):
        torch.testing.assert_close(a, c, rtol=1e-3, atol=1e-4)


@pytest.mark.parametrize("offset", [1e3, -3e3])
def test_bgnn_batchnorm_large_channel_offset(dev, offset):
    """|mean| >> std (x = offset + randn): the statistics are shifted sums (bgnn_bn_stats subtracts
    the first row, bgnn_bn_finalize_shifted adds it back), so the variance does not cancel; the
    output, input gradient and running variance stay within the fp32 tolerances against fp64 torch
    (round-4 ADVICE, low)."""
    torch.manual_seed(7)
    N, C = 5041, 512
    ref = torch.nn.BatchNorm1d(C).double()
    ours = bnn.use_bgnn_batchnorm(copy.deepcopy(ref).float().to(dev))
    x = torch.randn(N, C, dtype=torch.float64) + offset
    x32 = x.float()
    g = torch.randn(N, C, dtype=torch.float64)
    xr = x32.double().requires_grad_(True)     # (the fp32 input both sides see)
    xo = x32.to(dev).requires_grad_(True)
    yr = ref(xr)
    yo = ours(xo)
    yr.backward(g)
    yo.backward(g.float().to(dev))
    # (y = x * scale + shift in fp32 carries ~ulp(offset) of rounding: atol 1e-3 at |offset| <= 3e3;
    # the one-pass E[x^2] - E[x]^2 form missed the variance by ~10 % here)
    torch.testing.assert_close(yo.detach().cpu(), yr.detach().float(), rtol=1e-3, atol=2e-3)
    torch.testing.assert_close(ours.running_var.cpu(), ref.running_var.float(), rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(ours.running_mean.cpu(), ref.running_mean.float(), rtol=1e-5, atol=1e-3)
    torch.testing.assert_close(xo.grad.cpu(), xr.grad.float(), rtol=1e-3, atol=2e-3)
