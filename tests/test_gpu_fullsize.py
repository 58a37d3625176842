"""GPU: the bench's whole train-step forward + backward at full BASELINE size against the fp64
oracle (the reference orchestration Models/BuckGNN.py:67-74,323,430-444 over the PyG
restatement), on the exact code path bench.py times: GraphSage_addAggr h=512 L=6 on a full
cfg2 batch (16 x 71x71 meshes with virtual edges: N = 80,656, E = 715,872) and a full cfg3
batch (16 meshes with super nodes of in-degree 5,041: N = 80,672, E = 792,992), folded node
encoder + bgnn_mlp2 head, fused layers, BatchNorm in train mode, dropout 0 (torch's dropout RNG
cannot be matched). Checked: the 16 predictions and the RelativeErrorLoss within the north
star's 1e-4, every used parameter's gradient within the golden fixtures' checksum tolerance,
the whole gradient tensors within 1e-3 relative L2 per parameter (with a noise floor for the
gradients that are exactly 0 in exact arithmetic), BatchNorm running statistics, and the set of
parameters with gradients."""
import numpy as np
import pytest
import torch

import bgnn
from bgnn import buckgnn, fused
from bgnn import synthetic as S
from oracle import buckgnn_ref as R
from recipe import grad_checksum

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("cfg", ["cfg2", "cfg3"])
def test_full_size_train_step_matches_fp64_oracle(dev, monkeypatch, cfg):
    b = S.make_config_batch(cfg)
    assert (b.num_nodes, b.num_edges) == {"cfg2": (80656, 715872), "cfg3": (80672, 792992)}[cfg]
    torch.manual_seed(0)
    m = bgnn.BuckGNN(16, 5, hidden_channels=512, num_layers=6, dropout_rate=0.0, model_name="GraphSage_addAggr")
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    m = m.to(dev).train()
    folds = []
    real_layer = buckgnn.sage_layer
    monkeypatch.setattr(buckgnn, "sage_layer", lambda *a, **k: folds.append(k.get("w_in") is not None)
                        or real_layer(*a, **k))
    bd = b.to(dev)
    pred, _ = m(bd.x, bd.edge_index, bd.edge_attr, bd.batch)
    loss = bgnn.RelativeErrorLoss()(pred, bd.y)
    loss.backward()
    torch.cuda.synchronize()
    assert folds == [True] + [False] * 5                       # the bench's folded-encoder path
    got = {k: p.grad.detach().cpu().double().numpy() for k, p in m.named_parameters() if p.grad is not None}
    state = {k: v.detach().cpu() for k, v in m.state_dict().items() if "running_" in k}
    pred_g, loss_g = pred.detach().cpu().double(), float(loss.item())
    del m, bd, pred, loss
    torch.cuda.empty_cache()

    # fp64 oracle on the host (~25 s with 8-16 threads)
    torch.set_num_threads(min(16, torch.get_num_threads()))
    st = {k: v.double().clone().requires_grad_(v.is_floating_point() and "running" not in k
                                               and "num_batches" not in k) for k, v in sd.items()}
    pred_o = R.forward(st, "GraphSage_addAggr", b.x.double(), b.edge_index, b.batch, True, "mean", 0.0)
    loss_o = R.relative_error_loss(pred_o, b.y.double())
    loss_o.backward()

    np.testing.assert_allclose(pred_g.numpy(), pred_o.detach().numpy(), rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(loss_g, float(loss_o), rtol=1e-4, atol=1e-4)
    ref = {k: v.grad.numpy() for k, v in st.items() if v.grad is not None}
    assert set(got) == set(ref)
    for k in ref:
        np.testing.assert_allclose(grad_checksum(got[k]), grad_checksum(ref[k]), rtol=2e-3, atol=2e-4, err_msg=k)
    # whole gradient tensors, elementwise in aggregate: per parameter the L2 distance to fp64 within
    # 1e-3 of the parameter's own gradient norm, plus a floor of 1e-5 of the largest per-element RMS
    # gradient of the model (biases feeding a BatchNorm have an exact gradient of 0; their float
    # gradients are rounding noise that a purely relative bound cannot judge)
    rms = max(np.sqrt(np.mean(r ** 2)) for r in ref.values())
    worst = []
    for k in ref:
        err = float(np.linalg.norm(got[k] - ref[k]))
        nrm = float(np.linalg.norm(ref[k]))
        bound = 1e-3 * nrm + 1e-5 * rms * np.sqrt(ref[k].size)
        worst.append((err / max(bound, 1e-300), k, err, nrm))
        assert err <= bound, (k, err, nrm, bound)
    print("largest gradient error / bound:", max(worst)[:2])
    for k, v in state.items():   # running statistics after one train-mode step (momentum 0.1)
        np.testing.assert_allclose(v.numpy(), st[k].detach().numpy(), rtol=1e-5, atol=1e-6, err_msg=k)
