"""Install bgnn as `torch_geometric` / `torch_scatter` so the reference's own files
(Models/BuckGNN.py, TRAIN_FINAL.py, INFERENCE.py) import and run on MI355X unchanged:

    import bgnn; bgnn.install_pyg_shim()
    from Models.BuckGNN import BuckGNN            # reference module, unchanged

Provides exactly the names the reference imports (Models/BuckGNN.py:3-6,
Utils/Losses.py:4, TRAIN_FINAL.py:5, INFERENCE.py:5, GraphCreate.py:4).
"""
from __future__ import annotations

import sys
import types


def _module(name: str, **attrs) -> types.ModuleType:
    m = types.ModuleType(name)
    m.__dict__.update(attrs)
    m.__bgnn_shim__ = True
    return m


_TORCH_BN = None   # torch.nn.BatchNorm1d while install_pyg_shim(batchnorm=True) has replaced it


def install_pyg_shim(force: bool = False, batchnorm: bool = False) -> None:
    """batchnorm=True (opt-in): also make torch.nn.BatchNorm1d bgnn.nn.BatchNorm1d (a subclass with
    the same parameters, buffers and state-dict keys whose 2-D fp32 GPU forward runs on libbgnn),
    so the BatchNorm1d modules the reference builds (Models/BuckGNN.py:133-217, `nn.BatchNorm1d`
    looked up when the model is constructed) take the HIP kernels too."""
    global _TORCH_BN
    existing = sys.modules.get("torch_geometric")
    if existing is not None and not getattr(existing, "__bgnn_shim__", False) and not force:
        raise RuntimeError("a real torch_geometric is already imported; pass force=True to replace it")
    from . import data as D
    from . import dataset as DS
    from . import nn as N

    nn_mod = _module("torch_geometric.nn", SAGEConv=N.SAGEConv, SAGPooling=N.SAGPooling,
                     global_mean_pool=N.global_mean_pool, global_max_pool=N.global_max_pool,
                     global_add_pool=N.global_add_pool)
    data_mod = _module("torch_geometric.data", Data=D.Data, Batch=D.Batch)
    # unpickling targets of PyG-written dataset caches (GraphCreate.py:566-568 pickle.load):
    # PyG's Data comes back as a bgnn Data with the same attributes
    data_data_mod = _module("torch_geometric.data.data", Data=DS.PygData, DataEdgeAttr=DS.PygClassMarker,
                            DataTensorAttr=DS.PygClassMarker)
    storage_mod = _module("torch_geometric.data.storage", GlobalStorage=DS.PygStorage, NodeStorage=DS.PygStorage,
                          EdgeStorage=DS.PygStorage, BaseStorage=DS.PygStorage)
    loader_mod = _module("torch_geometric.loader", DataLoader=D.DataLoader)
    pyg = _module("torch_geometric", nn=nn_mod, data=data_mod, loader=loader_mod, __version__="bgnn-shim")
    scatter = _module("torch_scatter", scatter_add=N.scatter_add, scatter_sum=N.scatter_sum,
                      scatter_mean=N.scatter_mean)
    sys.modules.update({
        "torch_geometric": pyg,
        "torch_geometric.nn": nn_mod,
        "torch_geometric.data": data_mod,
        "torch_geometric.data.data": data_data_mod,
        "torch_geometric.data.storage": storage_mod,
        "torch_geometric.loader": loader_mod,
        "torch_scatter": scatter,
    })
    if batchnorm and _TORCH_BN is None:
        import torch
        _TORCH_BN = torch.nn.BatchNorm1d
        torch.nn.BatchNorm1d = N.BatchNorm1d


def uninstall_pyg_shim() -> None:
    global _TORCH_BN
    if _TORCH_BN is not None:
        import torch
        torch.nn.BatchNorm1d = _TORCH_BN
        _TORCH_BN = None
    for k in ("torch_geometric", "torch_geometric.nn", "torch_geometric.data", "torch_geometric.data.data",
              "torch_geometric.data.storage", "torch_geometric.loader", "torch_scatter"):
        m = sys.modules.get(k)
        if m is not None and getattr(m, "__bgnn_shim__", False):
            del sys.modules[k]
