"""Install bgnn as `torch_geometric` / `torch_scatter` so the reference's own files
(Models/BuckGNN.py, TRAIN_FINAL.py, INFERENCE.py) import and run on MI355X unchanged:

    import bgnn; bgnn.install_pyg_shim()
    from Models.BuckGNN import BuckGNN            # TRAIN_FINAL.py:38 / INFERENCE.py, unchanged

Provides exactly the names the reference imports (Models/BuckGNN.py:3-6,
Utils/Losses.py:4, TRAIN_FINAL.py:5, INFERENCE.py:5, GraphCreate.py:4).

By default (fused_model=True) the shim also installs an import hook: when the reference's
`Models.BuckGNN` module is imported (or already was), its `BuckGNN` class is replaced by
bgnn.BuckGNN -- the same constructor (Models/BuckGNN.py:9-12), submodules, state-dict keys and
forward signature (:311) -- whose SAGE layer loop runs as fused HIP layers, so the unchanged
TRAIN_FINAL.py / INFERENCE.py train and evaluate on the fused path. The reference's own class stays
reachable as `Models.BuckGNN.BuckGNN_reference` (fused_model=False keeps it in place: the per-module
route, every SAGEConv / BatchNorm1d on libbgnn and the layer glue in torch).
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
_MODEL_HOOK = None  # the import hook of install_pyg_shim(fused_model=True)
_REF_MODULE = "Models.BuckGNN"


def _bind_fused_model(mod) -> None:
    """Make module `mod` (the reference's Models.BuckGNN) export bgnn.BuckGNN as BuckGNN."""
    import types
    from .buckgnn import BuckGNN
    ref = mod.__dict__.get("BuckGNN")
    if ref is None or ref is BuckGNN:
        return
    # the reference's methods look BuckGNN up in the module globals at call time
    # (`super(BuckGNN, self).__init__()`, Models/BuckGNN.py:13): give them globals in which the name
    # still means their own class, so BuckGNN_reference stays constructible
    g = dict(mod.__dict__)
    g["BuckGNN"] = ref
    for name, f in list(vars(ref).items()):
        if isinstance(f, types.FunctionType) and f.__globals__ is mod.__dict__:
            nf = types.FunctionType(f.__code__, g, f.__name__, f.__defaults__, f.__closure__)
            nf.__kwdefaults__, nf.__qualname__, nf.__doc__ = f.__kwdefaults__, f.__qualname__, f.__doc__
            setattr(ref, name, nf)
    mod.BuckGNN_reference = ref
    mod.BuckGNN = BuckGNN


class _ModelHook:
    """sys.meta_path finder: loads the reference's Models.BuckGNN with its own loader, then binds
    bgnn.BuckGNN in place of its BuckGNN class (_bind_fused_model)."""

    def find_spec(self, fullname, path=None, target=None):
        if fullname != _REF_MODULE:
            return None
        import importlib.machinery
        spec = importlib.machinery.PathFinder.find_spec(fullname, path)
        if spec is None or spec.loader is None:
            return None
        real = spec.loader

        class _Loader:
            def create_module(self, sp):
                return real.create_module(sp) if hasattr(real, "create_module") else None

            def exec_module(self, module):
                real.exec_module(module)
                _bind_fused_model(module)

        spec.loader = _Loader()
        return spec


def install_pyg_shim(force: bool = False, batchnorm: bool = True, fused_model: bool = True) -> None:
    """batchnorm=True (default): also make torch.nn.BatchNorm1d bgnn.nn.BatchNorm1d (a subclass with
    the same parameters, buffers and state-dict keys whose 2-D fp32 GPU forward runs on libbgnn),
    so the BatchNorm1d modules the reference builds (Models/BuckGNN.py:133-217, `nn.BatchNorm1d`
    looked up when the model is constructed) take the HIP kernels too (round 5: on by default).
    fused_model=True (default): the import hook that binds bgnn.BuckGNN as the reference's
    Models.BuckGNN.BuckGNN (module docstring)."""
    global _TORCH_BN, _MODEL_HOOK
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
    if fused_model and _MODEL_HOOK is None:
        _MODEL_HOOK = _ModelHook()
        sys.meta_path.insert(0, _MODEL_HOOK)
        if _REF_MODULE in sys.modules:   # (imported before the shim: rebind in place)
            _bind_fused_model(sys.modules[_REF_MODULE])


def uninstall_pyg_shim() -> None:
    global _TORCH_BN, _MODEL_HOOK
    if _MODEL_HOOK is not None:
        if _MODEL_HOOK in sys.meta_path:
            sys.meta_path.remove(_MODEL_HOOK)
        _MODEL_HOOK = None
        m = sys.modules.get(_REF_MODULE)
        if m is not None and "BuckGNN_reference" in m.__dict__:
            m.BuckGNN = m.BuckGNN_reference
    if _TORCH_BN is not None:
        import torch
        torch.nn.BatchNorm1d = _TORCH_BN
        _TORCH_BN = None
    for k in ("torch_geometric", "torch_geometric.nn", "torch_geometric.data", "torch_geometric.data.data",
              "torch_geometric.data.storage", "torch_geometric.loader", "torch_scatter"):
        m = sys.modules.get(k)
        if m is not None and getattr(m, "__bgnn_shim__", False):
            del sys.modules[k]
