"""GPU: the node encoder's last Linear folded into the first fused SAGE layer
(BuckGNN._foldable_encoder, fused.sage_layer w_in/b_in). The reference computes
x0 = node_encoder(x) and then SAGEConv_0(x0) (Models/BuckGNN.py:323,434); folding computes
z = h ([W_l;W_r] W)^T + [W_l;W_r] b from the encoder's hidden h without materialising x0. The
function and every gradient must match the unfolded path (and the CPU oracle) to fp32 rounding."""
import pytest
import torch

import bgnn
from bgnn import buckgnn
from bgnn import synthetic as S
from oracle import buckgnn_ref as R

pytestmark = pytest.mark.gpu


def oracle_grads(b, sd, model_name):
    """fp64 gradients of the oracle (reference orchestration over the PyG restatement)."""
    st = {k: v.double().clone().requires_grad_(v.is_floating_point() and "running" not in k
                                               and "num_batches" not in k)
          for k, v in sd.items()}
    pred = R.forward(st, model_name, b.x.double(), b.edge_index, b.batch, True, "mean", 0.0)
    R.relative_error_loss(pred, b.y.double()).backward()
    return {k: v.grad for k, v in st.items() if v.grad is not None}


def rel_err(a, r):
    return float((a.double().cpu() - r).norm() / (r.norm() + 1e-300))


def grads_close(got, ref, exact):
    """Against fp64: every folded gradient within 1e-3 relative L2 (the golden-gradient tolerance
    of tests/test_gpu_model.py) or within 4x the unfolded path's own error, and folding no less
    accurate than the unfolded path overall (mean relative error within 2x). Per parameter the
    two paths' f32 rounding noise, amplified through BatchNorm, varies either way by up to 100x
    (measured: 1e-6 .. 6e-4 for both paths; which parameters land in the 1e-6 group differs
    between them): the unfolded path alone, run once with f16x3 and once with bf16x6 GEMMs (both
    f32-class), lands at 3.1e-4 and 9.7e-6 on the same parameter (GraphSage_meanAggr layer 1
    lin_l.bias; tools/fold_ab.py)."""
    assert set(got) == set(ref)
    e_fold = {k: rel_err(got[k], exact[k]) for k in ref}
    e_ref = {k: rel_err(ref[k], exact[k]) for k in ref}
    for k in ref:
        assert e_fold[k] <= max(1e-3, 4.0 * e_ref[k]), (k, e_fold[k], e_ref[k])
    mean = lambda d: sum(d.values()) / len(d)   # noqa: E731
    assert mean(e_fold) <= 2.0 * mean(e_ref) + 1e-6, (mean(e_fold), mean(e_ref))


def run(dev, model_name, hidden, fold, super_node=False):
    b = S.make_batch(24, 4, super_node=super_node)          # N >= 1024: the fused encoder path
    assert b.num_nodes >= 1024
    torch.manual_seed(0)
    m = bgnn.BuckGNN(16, 5, hidden_channels=hidden, num_layers=6, dropout_rate=0.0, model_name=model_name)
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    m = m.to(dev).train()
    old = buckgnn.FOLD_ENCODER
    buckgnn.FOLD_ENCODER = fold
    try:
        bd = b.to(dev)
        pred, _ = m(bd.x, bd.edge_index, bd.edge_attr, bd.batch)
        loss = bgnn.RelativeErrorLoss()(pred, bd.y)
        loss.backward()
    finally:
        buckgnn.FOLD_ENCODER = old
    grads = {k: p.grad.detach().clone() for k, p in m.named_parameters() if p.grad is not None}
    return b, sd, pred.detach(), grads


@pytest.mark.parametrize("model_name,hidden", [("GraphSage_addAggr", 512), ("GraphSage_meanAggr", 512),
                                               ("GraphSage_addAggr_Shared", 512), ("GraphSage_addAggr", 64)])
def test_folded_encoder_matches_unfolded_and_oracle(dev, model_name, hidden):
    b, sd, p_fold, g_fold = run(dev, model_name, hidden, True)
    _, _, p_ref, g_ref = run(dev, model_name, hidden, False)
    torch.testing.assert_close(p_fold, p_ref, rtol=1e-4, atol=1e-5)
    grads_close(g_fold, g_ref, oracle_grads(b, sd, model_name))
    # and the CPU oracle (reference orchestration over the PyG restatement), BatchNorm in train mode
    pred_o = R.forward({k: v for k, v in sd.items()}, model_name, b.x, b.edge_index, b.batch, True, "mean", 0.0)
    torch.testing.assert_close(p_fold.cpu(), pred_o, rtol=1e-4, atol=1e-4)


def test_folded_encoder_with_super_nodes(dev):
    """cfg3-like graphs (super nodes: heavy rows in the first layer's aggregation)."""
    b, sd, p_fold, g_fold = run(dev, "GraphSage_addAggr", 512, True, super_node=True)
    _, _, p_ref, g_ref = run(dev, "GraphSage_addAggr", 512, False, super_node=True)
    torch.testing.assert_close(p_fold, p_ref, rtol=1e-4, atol=1e-5)
    grads_close(g_fold, g_ref, oracle_grads(b, sd, "GraphSage_addAggr"))
