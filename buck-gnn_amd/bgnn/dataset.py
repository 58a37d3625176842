"""PyG-free loader for the reference's on-disk dataset cache.

Dataset_Preparation/GraphCreate.py:562-568 returns `pickle.load(f)` of
`dataset_cache_{buckling|static|mode_shape}.pkl`, which :636-638 wrote with `pickle.dump(dataset)`:
a `list[torch_geometric.data.Data]` (x, edge_index, edge_attr, y, plus file_path and, for
buckling, mode_shapes; GraphCreate.py:544-552). TRAIN_FINAL.py:1161-1217 reads it through
load_folder_dataset. PyG is not installed here, and an unrestricted pickle.load would execute
whatever the file names, so `load_dataset_cache` uses a restricted unpickler:

* `find_class` allowlists exactly the globals such a file holds -- PyG's `Data` (both the 2.x
  layout with a `GlobalStorage` in `_store` and the `DataEdgeAttr` / `DataTensorAttr` class
  markers, and the 1.x layout with plain attributes), the tensor rebuild function
  `torch._utils._rebuild_tensor_v2`, `collections.OrderedDict`, and numpy's array / scalar
  reconstructors -- and refuses every other global with the module and name in the error;
* PyG's Data becomes a bgnn Data with the same attributes (`PygData.__setstate__`, which reads
  the state dictionary only; no PyG code runs), its storage and class markers attribute bags;
* tensor storages, which plain pickle writes as `torch.storage._load_from_bytes(bytes)` (a
  nested torch.save blob that torch itself would load with weights_only=False), are loaded
  with `torch.load(weights_only=True)` instead.

The result is a list of plain `bgnn.data.Data`, ready for `bgnn.GraphStore(...)` or
`bgnn.Batch.from_data_list(...)`.
"""
from __future__ import annotations

import collections
import io
import pickle
from typing import Any, Dict, List

import numpy as np
import torch

from .data import Data


class _PygBag:
    """Attribute bag for an allowlisted PyG helper class (GlobalStorage, class markers)."""

    def __setstate__(self, state: Any) -> None:
        if isinstance(state, tuple) and len(state) == 2:   # (dict state, slot state)
            state = {**(state[0] or {}), **(state[1] or {})}
        if not isinstance(state, dict):
            raise pickle.UnpicklingError(f"dataset cache: unexpected state of {type(self).__name__}")
        self.__dict__.update(state)


class PygStorage(_PygBag):
    """Stands in for torch_geometric.data.storage.GlobalStorage (its `_mapping` holds the attributes)."""


class PygClassMarker(_PygBag):
    """Stands in for DataEdgeAttr / DataTensorAttr, the classes PyG 2.x keeps in Data.__dict__."""


class PygData(Data):
    """Unpickles a torch_geometric.data.Data (2.x: attributes in `_store._mapping`; 1.x: plain
    attributes) as a bgnn Data with the same attributes. Also what bgnn.install_pyg_shim registers
    as torch_geometric.data.data.Data, so the reference's own pickle.load of a cache
    (GraphCreate.py:566-568) yields bgnn graphs."""

    def __setstate__(self, state: Any) -> None:
        if isinstance(state, tuple) and len(state) == 2:
            state = {**(state[0] or {}), **(state[1] or {})}
        if not isinstance(state, dict):
            raise pickle.UnpicklingError("dataset cache: unexpected PyG Data state")
        store = state.get("_store")
        if store is not None:
            mapping = store.__dict__.get("_mapping") if hasattr(store, "__dict__") else None
            if not isinstance(mapping, dict):
                raise pickle.UnpicklingError("dataset cache: PyG Data without a storage mapping")
        else:
            mapping = {k: v for k, v in state.items() if not k.startswith("_")}
        self.__dict__["_store"] = {k: (torch.from_numpy(v) if isinstance(v, np.ndarray) else v)
                                   for k, v in mapping.items()}


def _safe_load_from_bytes(b: bytes):
    """torch.storage._load_from_bytes restricted to weights_only (a nested storage blob)."""
    return torch.load(io.BytesIO(b), weights_only=True)


def _allowed() -> Dict[tuple, Any]:
    allow = {
        ("torch._utils", "_rebuild_tensor_v2"): torch._utils._rebuild_tensor_v2,
        ("torch.storage", "_load_from_bytes"): _safe_load_from_bytes,
        ("collections", "OrderedDict"): collections.OrderedDict,
        ("torch", "Size"): torch.Size,
    }
    for mod in ("torch_geometric.data.data", "torch_geometric.data"):
        allow[(mod, "Data")] = PygData
        allow[(mod, "DataEdgeAttr")] = PygClassMarker
        allow[(mod, "DataTensorAttr")] = PygClassMarker
    for name in ("GlobalStorage", "NodeStorage", "EdgeStorage", "BaseStorage"):
        allow[("torch_geometric.data.storage", name)] = PygStorage
    try:
        from numpy._core import multiarray as ma
    except ImportError:   # numpy < 2
        from numpy.core import multiarray as ma
    for path in ("numpy.core.multiarray", "numpy._core.multiarray"):
        allow[(path, "_reconstruct")] = ma._reconstruct
        allow[(path, "scalar")] = ma.scalar
    allow[("numpy", "ndarray")] = np.ndarray
    allow[("numpy", "dtype")] = np.dtype
    for dt in (np.float64, np.float32, np.int64, np.int32, np.bool_, np.uint8):
        allow[("numpy.dtypes", type(np.dtype(dt)).__name__)] = type(np.dtype(dt))
    return allow


class _RestrictedUnpickler(pickle.Unpickler):
    _ALLOWED = None

    def find_class(self, module: str, name: str):
        if _RestrictedUnpickler._ALLOWED is None:
            _RestrictedUnpickler._ALLOWED = _allowed()
        fn = _RestrictedUnpickler._ALLOWED.get((module, name))
        if fn is None:
            raise pickle.UnpicklingError(f"dataset cache: refused global {module}.{name} (not a PyG Data list)")
        return fn


def _convert(obj: Any) -> Data:
    if not isinstance(obj, Data):
        raise ValueError(f"dataset cache: expected PyG Data objects, got {type(obj).__name__}")
    out = Data()
    out.__dict__["_store"] = dict(obj._store)
    return out


def load_dataset_cache(path: str) -> List[Data]:
    """The reference's `dataset_cache_*.pkl` (GraphCreate.py:562-568) as a list of bgnn Data,
    read without PyG and without executing anything from the file."""
    with open(path, "rb") as f:
        obj = _RestrictedUnpickler(f).load()
    if isinstance(obj, tuple):
        obj = list(obj)
    if not isinstance(obj, list):
        raise ValueError(f"dataset cache: expected a list of graphs, got {type(obj).__name__}")
    return [_convert(o) for o in obj]
