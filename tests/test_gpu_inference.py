"""GPU: the inference driver (bgnn.evaluate, INFERENCE.py's buckling metrics) against the fp64
oracle's eval forward and metrics, and over
host-collated batches and GraphStore batches gives the same predictions (to fp32 rounding:
the two paths group aggregation rows differently) and the metrics of a direct computation."""
import numpy as np
import pytest
import torch

import bgnn
from bgnn import synthetic as S
from bgnn.data import Batch

pytestmark = pytest.mark.gpu


def test_evaluate_matches_direct_computation(dev):
    gs = [S.make_mesh_graph(18, seed=s, super_node=(s % 2 == 1)) for s in range(6)]
    torch.manual_seed(0)
    model = bgnn.BuckGNN(16, 5, 64, 6, "mean", model_name="GraphSage_addAggr").to(dev)
    scaler = bgnn.EigenvalueScaler(2.0, 0.75)
    host = [Batch.from_data_list(gs[i:i + 4]) for i in range(0, 6, 4)]
    r1 = bgnn.evaluate(model, host, scaler, device=dev)
    store = bgnn.GraphStore(gs, dev)
    r2 = bgnn.evaluate(model, store.loader(4), scaler)
    torch.testing.assert_close(r1["predictions"], r2["predictions"], rtol=1e-5, atol=1e-6)
    assert r1["graphs"] == r2["graphs"] == 6
    # direct: eval forward, denormalise, |(true - pred) / true| in percent
    model.eval()
    with torch.no_grad():
        b = Batch.from_data_list(gs).to(dev)
        pred, _ = model(b.x, b.edge_index, b.edge_attr, b.batch)
    t = scaler.denormalize_eigenvalue(b.y).double().cpu().numpy()
    p = scaler.denormalize_eigenvalue(pred.view_as(b.y)).double().cpu().numpy()
    ape = np.abs((t - p) / t) * 100
    assert r1["mape"] == pytest.approx(ape.mean(), rel=1e-5)
    assert r1["max_mape"] == pytest.approx(ape.max(), rel=1e-5)
    assert r1["min_mape"] == pytest.approx(ape.min(), rel=1e-5)


def test_evaluate_matches_oracle(dev):
    """bgnn.evaluate (eval-mode BN with running statistics, no_grad) against the fp64 oracle's
    eval forward (Models/BuckGNN.py in eval mode over the PyG restatement) and INFERENCE.py's
    metrics computed from the oracle's predictions (INFERENCE.py:133-150): h=512, one batch of
    >= 1,024 nodes (folded encoder + bgnn_mlp2 head) and one smaller batch (unfolded path)."""
    from oracle import buckgnn_ref as R
    from recipe import make_weights
    gs = [S.make_mesh_graph(18, seed=40 + s, super_node=(s % 2 == 1)) for s in range(6)]
    torch.manual_seed(0)
    model = bgnn.BuckGNN(16, 5, 512, 6, "mean", model_name="GraphSage_addAggr")
    sd = model.state_dict()
    w = make_weights({k: tuple(v.shape) for k, v in sd.items()}, 77)   # non-trivial running statistics
    sd = {k: torch.from_numpy(w[k]) if k in w else sd[k] for k in sd}
    model.load_state_dict(sd)
    model = model.to(dev)
    scaler = bgnn.EigenvalueScaler(2.0, 0.75)
    batches = [Batch.from_data_list(gs[0:4]), Batch.from_data_list(gs[4:6])]
    assert batches[0].num_nodes >= 1024 > batches[1].num_nodes
    r = bgnn.evaluate(model, batches, scaler, device=dev)
    sd64 = {k: v.double() if v.is_floating_point() else v for k, v in sd.items()}
    preds, apes = [], []
    for b in batches:
        p = R.forward(sd64, "GraphSage_addAggr", b.x.double(), b.edge_index, b.batch, False, "mean", 0.0)
        preds.append(p)
        t = scaler.denormalize_eigenvalue(b.y.double())
        apes.append(torch.abs((t - scaler.denormalize_eigenvalue(p)) / t) * 100)
    # (evaluate returns denormalised predictions, INFERENCE.py:137-138)
    np.testing.assert_allclose(r["predictions"].cpu().numpy(),
                               scaler.denormalize_eigenvalue(torch.cat(preds)).numpy(), rtol=1e-4, atol=1e-4)
    ape = torch.cat(apes)
    assert r["mape"] == pytest.approx(float(ape.mean()), rel=1e-4, abs=1e-4)
    assert r["max_mape"] == pytest.approx(float(ape.max()), rel=1e-4, abs=1e-4)
    assert r["min_mape"] == pytest.approx(float(ape.min()), rel=1e-4, abs=1e-4)
    assert r["graphs"] == 6
