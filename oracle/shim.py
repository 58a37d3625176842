"""ORACLE (test infrastructure only): install oracle.pyg_ref as torch_geometric /
torch_scatter, so the reference's Models/BuckGNN.py can be imported in THIS
container for golden-vector generation (tests/golden/make_golden.py)."""
from __future__ import annotations

import sys
import types

from . import pyg_ref as P


def install() -> None:
    def mod(name, **a):
        m = types.ModuleType(name)
        m.__dict__.update(a)
        return m

    nn_mod = mod("torch_geometric.nn", SAGEConv=P.SAGEConv, SAGPooling=P.SAGPooling,
                 global_mean_pool=P.global_mean_pool, global_max_pool=P.global_max_pool,
                 global_add_pool=P.global_add_pool)
    data_mod = mod("torch_geometric.data", Data=P.Data)
    pyg = mod("torch_geometric", nn=nn_mod, data=data_mod)
    sc = mod("torch_scatter", scatter_add=P.scatter_add, scatter_mean=P.scatter_mean)
    sys.modules.update({"torch_geometric": pyg, "torch_geometric.nn": nn_mod,
                        "torch_geometric.data": data_mod, "torch_scatter": sc})


def uninstall() -> None:
    for k in ("torch_geometric", "torch_geometric.nn", "torch_geometric.data", "torch_scatter"):
        sys.modules.pop(k, None)
