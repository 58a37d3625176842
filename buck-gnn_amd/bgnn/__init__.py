"""bgnn — MI355X-native (gfx950) GraphSAGE message-passing hot path of buck-gnn.

Host side (this package) mirrors the PyG / torch_scatter call surface the
reference uses; all arithmetic runs in libbgnn.so (HIP kernels, C-ABI in
include/bgnn.h). Importing the package does not touch the GPU.
"""
from . import _lib
from .buckgnn import BuckGNN, GraphNetBlock, MLPPooling
from .data import Batch, Data, DataLoader
from .graph import Graph, SegmentIndex, clear_caches, graph_for, prepare, segments_for
from .nn import (SAGEConv, SAGPooling, global_add_pool, global_max_pool, global_mean_pool, scatter_add, scatter_mean,
                 scatter_sum)
from .ops import aggregate, segment_reduce
from .pyg_shim import install_pyg_shim, uninstall_pyg_shim
from .store import GraphStore
from .checkpoint import load_checkpoint, load_reference_checkpoint, save_checkpoint
from .dataset import load_dataset_cache
from .inference import evaluate
from .train import EigenvalueScaler, GradAllReduce, RelativeErrorLoss, mape_error, train_step
from . import losses
from .losses import (GraphMAELoss, GraphMaxComponentRelativeError, GraphMixedError, GraphMSELoss,
                     GraphRelativeError, stress_errors)

__all__ = [
    "BuckGNN", "GraphNetBlock", "MLPPooling", "Batch", "Data", "DataLoader", "Graph", "SegmentIndex",
    "clear_caches", "graph_for", "prepare", "segments_for", "SAGEConv", "SAGPooling", "global_add_pool", "global_max_pool",
    "global_mean_pool", "scatter_add", "scatter_mean", "scatter_sum", "aggregate", "segment_reduce",
    "install_pyg_shim", "uninstall_pyg_shim", "EigenvalueScaler", "GradAllReduce", "RelativeErrorLoss",
    "mape_error", "train_step", "load_library", "GraphStore", "load_checkpoint", "load_reference_checkpoint",
    "save_checkpoint", "load_dataset_cache", "evaluate", "losses", "GraphMAELoss", "GraphMaxComponentRelativeError", "GraphMixedError",
    "GraphMSELoss", "GraphRelativeError", "stress_errors",
]


def load_library():
    """Load libbgnn.so (raises ImportError when it is missing)."""
    return _lib.load()
