"""GPU: the inference driver (bgnn.evaluate, INFERENCE.py's buckling metrics) over
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
