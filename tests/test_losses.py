"""Per-graph losses and error metrics of the node-level heads (bgnn.losses) against the
reference's own classes and functions (Utils/Losses.py:303-507, Dataset_Preparation/Metrics.py
:4-191), pinned by tests/golden/heads/losses.npz (tests/golden/make_golden_losses.py). The reference
loops over graphs with a mask each; bgnn.losses computes the same quantities as segment
reductions. Ragged graphs, values on both sides of the 0.1 threshold, ties of the largest
|target| (first index wins) and 1-D predictions are covered."""
import os

import numpy as np
import pytest
import torch

from bgnn import losses as L

GOLD = np.load(os.path.join(os.path.dirname(__file__), "golden", "heads", "losses.npz"))
TAGS = ["s3", "d3", "v1"]
MODS = {"rel": L.GraphRelativeError, "mixed": L.GraphMixedError, "mse": L.GraphMSELoss, "mae": L.GraphMAELoss,
        "maxc": L.GraphMaxComponentRelativeError}


def case(tag, dev):
    p, t, b = (torch.from_numpy(GOLD[f"{tag}_{k}"]).to(dev) for k in ("pred", "target", "batch"))
    return p, t, b


def check_losses(dev):
    for tag in TAGS:
        p, t, b = case(tag, dev)
        for name, cls in MODS.items():
            m = cls()
            assert m(p, t, b, None).item() == pytest.approx(float(GOLD[f"{tag}_{name}"]), rel=2e-5), (tag, name)
            assert m(p, t, None, None).item() == pytest.approx(float(GOLD[f"{tag}_{name}_nobatch"]), rel=2e-5), \
                (tag, name)


def check_metrics(dev):
    for tag in ("s3", "d3"):
        p, t, b = case(tag, dev)
        for kind in ("static_stress", "static_disp"):
            d = L.stress_errors(p, t, b, prediction_type=kind)
            keys = [str(k) for k in GOLD[f"{tag}_{kind}_keys"]]
            assert sorted(d) == keys, (tag, kind)
            ref = dict(zip(keys, GOLD[f"{tag}_{kind}_vals"]))
            for k in keys:
                if np.isnan(ref[k]):
                    assert np.isnan(d[k]), (tag, kind, k)
                else:
                    assert d[k] == pytest.approx(float(ref[k]), rel=5e-5, abs=1e-6), (tag, kind, k, d[k], ref[k])
            assert L.mape_error(p, t, kind).item() == pytest.approx(float(GOLD[f"{tag}_mape_{kind}"]), rel=2e-5)
        assert L.mape_error(p, t, "mode_shape").item() == pytest.approx(float(GOLD[f"{tag}_mape_mode_shape"]),
                                                                         rel=2e-5)


def test_losses_match_reference_cpu():
    check_losses(torch.device("cpu"))


def test_metrics_match_reference_cpu():
    check_metrics(torch.device("cpu"))


def test_segment_helpers_edge_cases():
    """Empty segments (graph ids with no rows), single-row graphs, unsorted batch vectors."""
    v = torch.tensor([3.0, 1.0, 2.0, 5.0, 5.0])
    seg = torch.tensor([2, 0, 2, 3, 3])
    assert L._seg_first_argmax(v, seg, 4).tolist()[2:] == [0, 3]
    q = L._seg_quantile(v, seg, 4, 0.5)
    assert torch.isnan(q[1]) and q[0].item() == 1.0 and q[2].item() == 2.5 and q[3].item() == 5.0


@pytest.mark.gpu
def test_losses_and_metrics_on_gpu(dev):
    check_losses(dev)
    check_metrics(dev)
