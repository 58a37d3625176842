"""Reference checkpoint compatibility (bgnn.checkpoint): a file in the layout of
TRAIN_FINAL.py:391-429 -- model_state_dict, a pickled DatasetNormalizer holding sklearn
scalers and numpy arrays, config -- is read with torch.load(weights_only=True) only.
The fixture's normalizer class is a test-side stand-in registered under the reference's
module path (the reference's own class is not imported); the scalers are real sklearn
objects."""
import sys
import types

import numpy as np
import pytest
import torch

import bgnn
from bgnn import checkpoint as ck

sklearn_pre = pytest.importorskip("sklearn.preprocessing")

CONFIG = {"num_node_features": 16, "num_edge_features": 5, "hidden_channels": 64, "num_layers": 6,
          "use_edge_attr": False, "use_z_coord": False, "use_rotations": False, "prediction_type": "buckling",
          "pooling_layer": "mean", "dropout_rate": 0.1, "model_name": "GraphSage_addAggr"}


@pytest.fixture
def reference_module():
    mod = types.ModuleType("Dataset_Preparation.Normalizer")
    pkg = types.ModuleType("Dataset_Preparation")

    class DatasetNormalizer:   # attribute layout of Normalizer.py:5-42
        def __init__(self):
            self.eigenvalue_scaler = sklearn_pre.RobustScaler()
            self.displacement_scaler = sklearn_pre.RobustScaler()
            self.rotation_scaler = sklearn_pre.StandardScaler()
            self.coord_min = None
            self.coord_max = None
            self.axial_stress_mean = None

    DatasetNormalizer.__module__ = "Dataset_Preparation.Normalizer"
    DatasetNormalizer.__qualname__ = "DatasetNormalizer"
    mod.DatasetNormalizer = DatasetNormalizer
    pkg.Normalizer = mod
    saved = {k: sys.modules.get(k) for k in ("Dataset_Preparation", "Dataset_Preparation.Normalizer")}
    sys.modules["Dataset_Preparation"] = pkg
    sys.modules["Dataset_Preparation.Normalizer"] = mod
    yield DatasetNormalizer
    for k, v in saved.items():
        if v is None:
            sys.modules.pop(k, None)
        else:
            sys.modules[k] = v


def make_reference_checkpoint(path, normalizer_cls):
    torch.manual_seed(3)
    model = bgnn.BuckGNN(16, 5, 64, 6, "mean", model_name="GraphSage_addAggr")
    norm = normalizer_cls()
    eig = np.random.default_rng(0).uniform(50, 400, size=(200, 1))
    norm.eigenvalue_scaler.fit(eig)
    norm.coord_min = np.array([0.0, -1.5, 2.0])
    torch.save({"model_state_dict": model.state_dict(), "normalizer": norm, "config": dict(CONFIG)}, path)
    return model, norm


def test_reference_checkpoint_loads_with_weights_only(tmp_path, reference_module):
    path = tmp_path / "last.pt"
    model, norm = make_reference_checkpoint(path, reference_module)
    # the plain weights_only load refuses the pickled normalizer ...
    with pytest.raises(Exception):
        torch.load(path, weights_only=True)
    # ... the bgnn loader reads it with weights_only=True and stand-in classes
    m2, scaler, cfg = bgnn.load_reference_checkpoint(str(path))
    assert cfg == CONFIG
    sd1, sd2 = model.state_dict(), m2.state_dict()
    assert sd1.keys() == sd2.keys()
    for k in sd1:
        assert torch.equal(sd1[k], sd2[k]), k
    assert not m2.training
    assert scaler.center == pytest.approx(float(norm.eigenvalue_scaler.center_[0]), rel=0, abs=0)
    assert scaler.scale == pytest.approx(float(norm.eigenvalue_scaler.scale_[0]), rel=0, abs=0)
    raw = ck.safe_load(str(path))
    assert isinstance(raw["normalizer"], ck.PickledObject)
    assert np.array_equal(raw["normalizer"].coord_min, norm.coord_min)
    # denormalisation matches Normalizer.py:207-215 (float32 tensors, v * scale + center)
    v = torch.tensor([0.25, -1.0, 3.5])
    ref = v * torch.tensor(norm.eigenvalue_scaler.scale_, dtype=torch.float32) + \
        torch.tensor(norm.eigenvalue_scaler.center_, dtype=torch.float32)
    assert torch.equal(scaler.denormalize_eigenvalue(v), ref)


class NotAllowed:
    pass


def test_unknown_classes_are_refused(tmp_path):
    path = tmp_path / "evil.pt"
    torch.save({"model_state_dict": {}, "normalizer": NotAllowed(), "config": dict(CONFIG)}, path)
    with pytest.raises(Exception, match="NotAllowed"):
        ck.safe_load(str(path))


def test_save_load_round_trip(tmp_path):
    torch.manual_seed(1)
    model = bgnn.BuckGNN(16, 5, 64, 6, "mean", model_name="GraphSage_addAggr")
    path = tmp_path / "bgnn.pt"
    bgnn.save_checkpoint(str(path), model, CONFIG, bgnn.EigenvalueScaler(120.5, 33.25))
    torch.load(path, weights_only=True)      # plain safe load works for bgnn's own files
    m2, scaler, cfg = bgnn.load_checkpoint(str(path))
    assert (scaler.center, scaler.scale) == (120.5, 33.25) and cfg == CONFIG
    for k, v in model.state_dict().items():
        assert torch.equal(v, m2.state_dict()[k])
