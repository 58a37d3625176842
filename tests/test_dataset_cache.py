"""The PyG-free loader of the reference's dataset cache (bgnn.load_dataset_cache;
Dataset_Preparation/GraphCreate.py:544-552 builds the Data objects, :562-568 loads and :636-638
writes `dataset_cache_*.pkl` with plain pickle).

PyG is absent, so the fixture pickles are written by stand-in classes registered under PyG's
module paths for the duration of the dump, laid out as PyG pickles them: 2.x (`Data` whose
`__dict__` holds a `GlobalStorage` in `_store` -- its `__getstate__` dereferences the weakref to
the parent -- and the `DataEdgeAttr` / `DataTensorAttr` class markers) and 1.x (plain
attributes). The stand-ins are removed before loading, so the loader sees only the file. Parity
with the reference's own cache files is unpinned (none ship with the reference)."""
import os
import pickle
import sys
import types
import weakref

import numpy as np
import pytest
import torch

import bgnn
from bgnn import synthetic as S
from bgnn.data import Batch


def _install_fake_pyg(layout):
    data_mod = types.ModuleType("torch_geometric.data.data")
    storage_mod = types.ModuleType("torch_geometric.data.storage")

    class GlobalStorage:
        def __init__(self, parent, mapping):
            self.__dict__["_mapping"] = dict(mapping)
            self.__dict__["_parent"] = weakref.ref(parent)

        def __getstate__(self):   # PyG BaseStorage.__getstate__
            out = self.__dict__.copy()
            out["_parent"] = out["_parent"]()
            return out

        def __setstate__(self, state):
            self.__dict__.update(state)
            self.__dict__["_parent"] = weakref.ref(state["_parent"])

    class DataEdgeAttr:
        pass

    class DataTensorAttr:
        pass

    class Data:
        def __init__(self, **kw):
            if layout == "2.x":
                self.__dict__["_store"] = GlobalStorage(self, kw)
                self.__dict__["_edge_attr_cls"] = DataEdgeAttr
                self.__dict__["_tensor_attr_cls"] = DataTensorAttr
            else:
                self.__dict__.update(kw)

    for cls, mod in ((GlobalStorage, storage_mod), (DataEdgeAttr, data_mod), (DataTensorAttr, data_mod), (Data, data_mod)):
        cls.__module__ = mod.__name__
        cls.__qualname__ = cls.__name__
        setattr(mod, cls.__name__, cls)
    saved = {k: sys.modules.get(k) for k in ("torch_geometric", "torch_geometric.data", "torch_geometric.data.data",
                                             "torch_geometric.data.storage")}
    sys.modules["torch_geometric"] = types.ModuleType("torch_geometric")
    sys.modules["torch_geometric.data"] = types.ModuleType("torch_geometric.data")
    sys.modules["torch_geometric.data.data"] = data_mod
    sys.modules["torch_geometric.data.storage"] = storage_mod
    return Data, saved


def _restore(saved):
    for k, v in saved.items():
        if v is None:
            sys.modules.pop(k, None)
        else:
            sys.modules[k] = v


def _write_cache(path, graphs, layout):
    Data, saved = _install_fake_pyg(layout)
    try:
        objs = []
        for i, g in enumerate(graphs):
            kw = dict(x=g.x, edge_index=g.edge_index, edge_attr=g.edge_attr, y=g.y, file_path=f"case_{i}.bdf",
                      mode_shapes=torch.randn(g.num_nodes, 6, dtype=torch.float32))
            objs.append(Data(**kw))
        with open(path, "wb") as f:
            pickle.dump(objs, f)   # GraphCreate.py:636-638
    finally:
        _restore(saved)


@pytest.mark.parametrize("layout", ["2.x", "1.x"])
def test_load_dataset_cache_roundtrip(tmp_path, layout):
    graphs = [S.make_mesh_graph(6 + i, seed=i, super_node=(i % 2 == 1)) for i in range(4)]
    path = os.path.join(tmp_path, "dataset_cache_buckling.pkl")
    _write_cache(path, graphs, layout)
    assert "torch_geometric.data.data" not in sys.modules
    ds = bgnn.load_dataset_cache(path)
    assert len(ds) == len(graphs)
    for i, (d, g) in enumerate(zip(ds, graphs)):
        assert isinstance(d, bgnn.Data)
        for k in ("x", "edge_index", "edge_attr", "y"):
            assert torch.equal(d[k], g[k]), k
            assert d[k].dtype == g[k].dtype
        assert d.file_path == f"case_{i}.bdf"
        assert d.mode_shapes.shape == (g.num_nodes, 6)
        assert d.num_node_features == 16 and d.num_edge_features == 5
    b = Batch.from_data_list(ds)                       # the reference's DataLoader collation
    ref = Batch.from_data_list(graphs)
    assert torch.equal(b.edge_index, ref.edge_index) and torch.equal(b.batch, ref.batch)


class _Evil:
    def __reduce__(self):
        return (os.system, ("echo pwned",))


def test_load_dataset_cache_refuses_other_globals(tmp_path):
    path = os.path.join(tmp_path, "evil.pkl")
    with open(path, "wb") as f:
        pickle.dump([_Evil()], f)
    with pytest.raises(pickle.UnpicklingError, match="refused global"):
        bgnn.load_dataset_cache(path)


def test_load_dataset_cache_rejects_non_list(tmp_path):
    path = os.path.join(tmp_path, "dict.pkl")
    with open(path, "wb") as f:
        pickle.dump({"x": 1}, f)
    with pytest.raises(ValueError):
        bgnn.load_dataset_cache(path)


@pytest.mark.gpu
def test_dataset_cache_into_graph_store(dev, tmp_path):
    """A loaded cache feeds the device-resident GraphStore; its batches equal host collation of
    the same graphs (Batch.from_data_list, the reference's DataLoader path)."""
    graphs = [S.make_mesh_graph(12, seed=50 + i, super_node=(i % 3 == 0)) for i in range(7)]
    path = os.path.join(tmp_path, "dataset_cache_buckling.pkl")
    _write_cache(path, graphs, "2.x")
    ds = bgnn.load_dataset_cache(path)
    store = bgnn.GraphStore(ds, dev)
    for ids in ([0, 1, 2], [6, 3, 5, 4]):
        got = store.batch(ids)
        ref = Batch.from_data_list([graphs[i] for i in ids]).to(dev)
        for k in ("x", "edge_index", "edge_attr", "y", "batch"):
            assert torch.equal(got[k], ref[k]), k


def test_shim_pickle_load_gives_bgnn_graphs(tmp_path):
    """With bgnn.install_pyg_shim(), the reference's own `pickle.load` of a cache
    (GraphCreate.py:566-568) resolves PyG's classes to bgnn's: the graphs come back as bgnn Data."""
    graphs = [S.make_mesh_graph(5, seed=i) for i in range(2)]
    path = os.path.join(tmp_path, "dataset_cache_buckling.pkl")
    _write_cache(path, graphs, "2.x")
    bgnn.install_pyg_shim()
    try:
        with open(path, "rb") as f:
            ds = pickle.load(f)
    finally:
        bgnn.uninstall_pyg_shim()
    assert all(isinstance(d, bgnn.Data) for d in ds)
    assert torch.equal(ds[1].edge_index, graphs[1].edge_index) and ds[0].file_path == "case_0.bdf"
