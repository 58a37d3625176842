"""Reference checkpoint compatibility.

TRAIN_FINAL.py:391-429 saves `last.pt` / `best.pt` as
    {'model_state_dict': OrderedDict[str, Tensor],
     'normalizer': Dataset_Preparation.Normalizer.DatasetNormalizer (sklearn scalers, numpy),
     'config': {num_node_features, num_edge_features, hidden_channels, num_layers, ...}}
and INFERENCE.py:65-88 rebuilds the model from 'config' and loads the state dict with an
unrestricted `torch.load`. Here the file is read ONLY with `torch.load(weights_only=True)`:
the restricted unpickler runs no code from the file. The pickled normalizer's classes are
allowlisted as plain attribute-bag stand-ins registered under the reference's class paths
(`DatasetNormalizer`, sklearn's `RobustScaler` / `StandardScaler` / `MinMaxScaler`), so only
their attribute dictionaries are restored. numpy arrays and scalars go through numpy's own
reconstruct functions. The eigenvalue scaler's `center_` / `scale_` become an
`EigenvalueScaler` (Normalizer.py:207-215). A file holding any other class is refused by
torch, with the class name in the error message.
"""
from __future__ import annotations

import os
from typing import Any, Dict, Optional, Tuple

import numpy as np
import torch

from .buckgnn import BuckGNN
from .train import EigenvalueScaler


class PickledObject:
    """Attribute bag standing in for an allowlisted class of the reference checkpoint."""

    def __repr__(self) -> str:
        return f"{type(self).__name__}({', '.join(sorted(self.__dict__))})"


def _standin(qualname: str):
    return type(qualname.rsplit(".", 1)[-1], (PickledObject,), {"__module__": __name__})


_STANDIN_PATHS = (
    "Dataset_Preparation.Normalizer.DatasetNormalizer",
    "Normalizer.DatasetNormalizer",
    "__main__.DatasetNormalizer",
    "sklearn.preprocessing._data.RobustScaler",
    "sklearn.preprocessing._data.StandardScaler",
    "sklearn.preprocessing._data.MinMaxScaler",
)
_STANDINS = {p: _standin(p) for p in _STANDIN_PATHS}


def _numpy_globals():
    mods = []
    for name in ("numpy._core.multiarray", "numpy.core.multiarray"):
        try:
            mods.append(__import__(name, fromlist=["_reconstruct"]))
        except ImportError:
            pass
    recon = mods[0]._reconstruct
    scalar = mods[0].scalar
    out = [np.ndarray, np.dtype]
    for path in ("numpy.core.multiarray", "numpy._core.multiarray"):
        out.append((recon, f"{path}._reconstruct"))
        out.append((scalar, f"{path}.scalar"))
    # numpy dtype classes (numpy.dtypes.Float64DType, ...) pickled with the arrays
    for dt in (np.float64, np.float32, np.int64, np.int32, np.bool_):
        out.append((type(np.dtype(dt)), f"numpy.dtypes.{type(np.dtype(dt)).__name__}"))
    return out


def safe_load(path: str, map_location="cpu") -> Dict[str, Any]:
    """torch.load(weights_only=True) with the reference's normalizer classes as stand-ins."""
    allow = list(_numpy_globals()) + [(cls, p) for p, cls in _STANDINS.items()]
    with torch.serialization.safe_globals(allow):
        return torch.load(path, map_location=map_location, weights_only=True)


def eigenvalue_scaler(normalizer: Any) -> Optional[EigenvalueScaler]:
    """EigenvalueScaler from a (stand-in) DatasetNormalizer: its eigenvalue RobustScaler's
    center_ / scale_ (Normalizer.py:207-215)."""
    sc = getattr(normalizer, "eigenvalue_scaler", None) if normalizer is not None else None
    if sc is None or not hasattr(sc, "center_") or not hasattr(sc, "scale_"):
        return None
    return EigenvalueScaler(float(np.asarray(sc.center_).reshape(-1)[0]), float(np.asarray(sc.scale_).reshape(-1)[0]))


def load_reference_checkpoint(path: str, device=None) -> Tuple[BuckGNN, Optional[EigenvalueScaler], Dict]:
    """Rebuild the model of a reference `last.pt` / `best.pt` (INFERENCE.py:65-88) as a
    bgnn.BuckGNN (same constructor, same state-dict keys), in eval mode, plus its
    eigenvalue scaler and config."""
    if not os.path.exists(path):
        raise FileNotFoundError(path)
    ck = safe_load(path)
    model, _, cfg = _model_from(ck, device)
    return model, eigenvalue_scaler(ck.get("normalizer")), cfg


def save_checkpoint(path: str, model: BuckGNN, config: Dict, scaler: Optional[EigenvalueScaler] = None) -> None:
    """Save in the reference layout, loadable with weights_only=True everywhere: the normalizer
    is stored as plain numbers ({'eigenvalue_center', 'eigenvalue_scale'}) instead of a pickled
    object."""
    norm = None if scaler is None else {"eigenvalue_center": scaler.center, "eigenvalue_scale": scaler.scale}
    torch.save({"model_state_dict": model.state_dict(), "normalizer": norm, "config": dict(config)}, path)


def load_checkpoint(path: str, device=None) -> Tuple[BuckGNN, Optional[EigenvalueScaler], Dict]:
    """Load a checkpoint written by save_checkpoint or by the reference."""
    ck = safe_load(path)
    norm = ck.get("normalizer")
    if isinstance(norm, dict) and "eigenvalue_center" in norm:
        model, _, cfg = _model_from(ck, device)
        return model, EigenvalueScaler(norm["eigenvalue_center"], norm["eigenvalue_scale"]), cfg
    return load_reference_checkpoint(path, device)


def _model_from(ck, device):
    cfg = ck["config"]
    model = BuckGNN(cfg["num_node_features"], cfg["num_edge_features"], cfg["hidden_channels"], cfg["num_layers"],
                    cfg["pooling_layer"], prediction_type=cfg["prediction_type"],
                    use_z_coord=cfg.get("use_z_coord", False), use_rotations=cfg.get("use_rotations", False),
                    dropout_rate=cfg.get("dropout_rate", 0.1), model_name=cfg.get("model_name", "EA_GNN"))
    model.load_state_dict(ck["model_state_dict"])
    if device is not None:
        model = model.to(device)
    model.eval()
    return model, None, cfg
