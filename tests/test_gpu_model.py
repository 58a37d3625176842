"""GPU: whole-model parity of bgnn.BuckGNN against golden vectors produced by the
REFERENCE's own Models/BuckGNN.py (tests/golden/make_golden.py): prediction,
RelativeErrorLoss, every gradient (or gradient checksums at h >= 256), BatchNorm
running statistics, pooled features and the eval-mode prediction. Both the fused
HIP layer loop and the per-op (drop-in SAGEConv) loop are checked."""
import glob
import os

import numpy as np
import pytest
import torch

import bgnn
from recipe import grad_checksum, make_weights, meta_from_array

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
FILES = sorted(glob.glob(os.path.join(GOLDEN, "*.npz")))


def build(meta, dev, fused_path):
    m = bgnn.BuckGNN(16, 5, hidden_channels=meta["hidden"], num_layers=meta["num_layers"],
                     pooling_layer=meta["pooling"], dropout_rate=0.0, model_name=meta["model_name"])
    sd = m.state_dict()
    w = make_weights({k: tuple(v.shape) for k, v in sd.items()}, meta["weight_seed"])
    m.load_state_dict({k: torch.from_numpy(w[k]) if k in w else sd[k] for k in sd})
    m.use_fused = fused_path
    return m.to(dev)


@pytest.mark.parametrize("fused_path", [True, False], ids=["fused", "per_op"])
@pytest.mark.parametrize("path", FILES, ids=os.path.basename)
def test_model_matches_reference_golden(dev, path, fused_path):
    z = np.load(path)
    meta = meta_from_array(z["meta"])
    model = build(meta, dev, fused_path)
    captured = {}
    model.decoder.register_forward_pre_hook(lambda mod, inp: captured.__setitem__("pooled", inp[0].detach()))
    x = torch.from_numpy(z["x"]).to(dev)
    ei = torch.from_numpy(z["edge_index"]).to(dev)
    ea = torch.from_numpy(z["edge_attr"]).to(dev)
    batch = None if meta["single_graph"] else torch.from_numpy(z["batch"]).to(dev)
    y = torch.from_numpy(z["y"]).to(dev)
    if meta["single_graph"]:
        y = y[0]
    model.train()
    pred, _ = model(x, ei, ea, batch)
    loss = bgnn.RelativeErrorLoss()(pred, y)
    model.zero_grad(set_to_none=True)
    loss.backward()
    tol = dict(rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(pred.detach().cpu().numpy().reshape(-1), z["pred_train"], **tol)
    np.testing.assert_allclose(loss.item(), float(z["loss_train"]), **tol)
    np.testing.assert_allclose(captured["pooled"].cpu().numpy(), z["pooled_train"], **tol)
    params = dict(model.named_parameters())
    for k in z.files:
        if k.startswith("grad/"):
            g = params[k[5:]].grad
            assert g is not None, k
            np.testing.assert_allclose(g.cpu().numpy(), z[k], rtol=1e-3, atol=2e-5, err_msg=k)
        elif k.startswith("gradsum/"):
            g = params[k[8:]].grad
            assert g is not None, k
            np.testing.assert_allclose(grad_checksum(g.cpu().numpy()), z[k], rtol=2e-3, atol=2e-4, err_msg=k)
    sd = model.state_dict()
    for k in z.files:
        if k.startswith("state/"):
            np.testing.assert_allclose(sd[k[6:]].cpu().numpy(), z[k], rtol=1e-5, atol=1e-6, err_msg=k)
    # parameters the reference never uses get no gradient here either
    for k, p in params.items():
        if ("grad/" + k) not in z.files and ("gradsum/" + k) not in z.files:
            assert p.grad is None, k
    model.eval()
    with torch.no_grad():
        pe, _ = model(x, ei, ea, batch)
    np.testing.assert_allclose(pe.cpu().numpy().reshape(-1), z["pred_eval"], **tol)
    np.testing.assert_allclose(captured["pooled"].cpu().numpy(), z["pooled_eval"], **tol)
