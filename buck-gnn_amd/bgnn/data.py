"""Minimal PyG-compatible graph containers: Data, Batch, DataLoader.

Covers what buck-gnn uses (GraphCreate.py:544-552; TRAIN_FINAL.py:253-255,1298-1302;
INFERENCE.py:114,134-136): arbitrary attributes (x, edge_index, edge_attr, y,
file_path, mode_shapes, ...), `.to(device)`, `.clone()`, `num_nodes`,
`num_node_features`, `num_edge_features`, and mini-batching into a disjoint
union with `batch` (graph id per node, nodes of a graph contiguous) and `ptr`.

PyG collation rules restated: attributes whose name contains "index" are
concatenated along their last dim and offset by the running node count; other
tensors are concatenated along dim 0 (0-d tensors are stacked); non-tensors are
collected into a list.
"""
from __future__ import annotations

import copy
from typing import Any, Iterable, List, Optional, Sequence

import torch
from torch import Tensor


def _is_index_key(key: str) -> bool:
    return "index" in key or key == "face"


class Data:
    def __init__(self, x: Optional[Tensor] = None, edge_index: Optional[Tensor] = None,
                 edge_attr: Optional[Tensor] = None, y: Optional[Tensor] = None, **kwargs: Any):
        self.__dict__["_store"] = {}
        for k, v in (("x", x), ("edge_index", edge_index), ("edge_attr", edge_attr), ("y", y)):
            if v is not None:
                self._store[k] = v
        for k, v in kwargs.items():
            self._store[k] = v

    # attribute access -------------------------------------------------------------
    def __getattr__(self, key: str):
        store = self.__dict__.get("_store", {})
        if key in store:
            return store[key]
        if key in ("x", "edge_index", "edge_attr", "y", "batch", "ptr", "pos"):
            return None
        raise AttributeError(key)

    def __setattr__(self, key: str, value: Any) -> None:
        if value is None:
            self._store.pop(key, None)
        else:
            self._store[key] = value

    def __delattr__(self, key: str) -> None:
        self._store.pop(key, None)

    def __getitem__(self, key: str):
        return self._store[key]

    def __setitem__(self, key: str, value: Any) -> None:
        self._store[key] = value

    def __contains__(self, key: str) -> bool:
        return key in self._store

    def keys(self) -> List[str]:
        return list(self._store.keys())

    def items(self):
        return self._store.items()

    # properties ---------------------------------------------------------------------
    @property
    def num_nodes(self) -> int:
        if "num_nodes" in self._store:
            return int(self._store["num_nodes"])
        if self.x is not None:
            return self.x.size(0)
        if self.edge_index is not None and self.edge_index.numel():
            return int(self.edge_index.max()) + 1
        return 0

    @property
    def num_edges(self) -> int:
        return 0 if self.edge_index is None else self.edge_index.size(-1)

    @property
    def num_node_features(self) -> int:
        return 0 if self.x is None else (1 if self.x.dim() == 1 else self.x.size(-1))

    @property
    def num_features(self) -> int:
        return self.num_node_features

    @property
    def num_edge_features(self) -> int:
        return 0 if self.edge_attr is None else (1 if self.edge_attr.dim() == 1 else self.edge_attr.size(-1))

    # transforms ---------------------------------------------------------------------
    def apply(self, fn):
        out = copy.copy(self)
        out.__dict__["_store"] = {k: (fn(v) if isinstance(v, Tensor) else v) for k, v in self._store.items()}
        return out

    def to(self, device, non_blocking: bool = False):
        return self.apply(lambda t: t.to(device, non_blocking=non_blocking))

    def cuda(self, device=None):
        return self.apply(lambda t: t.cuda(device))

    def cpu(self):
        return self.apply(lambda t: t.cpu())

    def clone(self):
        out = copy.copy(self)
        out.__dict__["_store"] = {k: (v.clone() if isinstance(v, Tensor) else copy.deepcopy(v))
                                  for k, v in self._store.items()}
        return out

    def __repr__(self) -> str:
        parts = []
        for k, v in self._store.items():
            parts.append(f"{k}={list(v.shape)}" if isinstance(v, Tensor) else f"{k}={v!r}"[:40])
        return f"{self.__class__.__name__}({', '.join(parts)})"


class Batch(Data):
    """Disjoint union of graphs with `batch` and `ptr` vectors."""

    @classmethod
    def from_data_list(cls, data_list: Sequence[Data]) -> "Batch":
        if len(data_list) == 0:
            raise ValueError("Batch.from_data_list: empty list")
        keys: List[str] = []
        for d in data_list:
            for k in d.keys():
                if k not in keys and k != "num_nodes":
                    keys.append(k)
        counts = [d.num_nodes for d in data_list]
        offsets = [0]
        for c in counts:
            offsets.append(offsets[-1] + c)
        out = cls()
        for k in keys:
            vals = [d._store.get(k) for d in data_list]
            if all(isinstance(v, Tensor) for v in vals):
                if _is_index_key(k):
                    vals = [v + off for v, off in zip(vals, offsets[:-1])]
                    out._store[k] = torch.cat(vals, dim=-1)
                elif all(v.dim() == 0 for v in vals):
                    out._store[k] = torch.stack(vals)
                else:
                    out._store[k] = torch.cat(vals, dim=0)
            else:
                out._store[k] = vals
        dev = data_list[0].x.device if data_list[0].x is not None else None
        out._store["batch"] = torch.repeat_interleave(torch.arange(len(data_list), device=dev),
                                                      torch.tensor(counts, device=dev))
        out._store["ptr"] = torch.tensor(offsets, dtype=torch.long, device=dev)
        out._store["num_graphs"] = len(data_list)
        out._store["num_nodes"] = offsets[-1]
        return out

    @property
    def num_graphs(self) -> int:
        return int(self._store.get("num_graphs", 0))

    def to_data_list(self) -> List[Data]:
        raise NotImplementedError("Batch.to_data_list is not needed by buck-gnn")


def collate(data_list: Sequence[Data]) -> Batch:
    return Batch.from_data_list(data_list)


class DataLoader(torch.utils.data.DataLoader):
    """torch DataLoader that collates lists of Data into a Batch (PyG loader API)."""

    def __init__(self, dataset, batch_size: int = 1, shuffle: bool = False, **kwargs):
        kwargs.pop("collate_fn", None)
        kwargs.pop("follow_batch", None)
        kwargs.pop("exclude_keys", None)
        super().__init__(dataset, batch_size=batch_size, shuffle=shuffle, collate_fn=collate, **kwargs)
