"""Seeded synthetic FE-mesh graphs shaped like buck-gnn's inputs.

Connectivity mirrors the reference data pipeline:
* an n x n quad mesh with row-major node ids (sorted Nastran ids give this
  locality, GraphCreate.py:150-151), CQUAD4 perimeter edges
  (GraphCreate.py:334-350) plus both quad diagonals as CBARs
  (Data_Generation_v3.py:233-242,264-270);
* non-stiffened: random virtual edges, int(0.1333 * #undirected) distinct pairs
  not already connected (VirtualEdgeCreate.py:21-49), edge feature 4 = 1;
* stiffened: a super node appended as the last node, wired to every real node
  (VirtualEdgeCreate.py:81-113), indicator feature = 1 on it;
* every undirected edge is emitted in both directions, int64
  (GraphCreate.py:417-422).
Node features are N(0,1) placeholders for the 15 physical features plus the
super-node indicator column (16 total); y ~ U(0.5, 1.5) per graph.
"""
from __future__ import annotations

from typing import List, Tuple

import numpy as np
import torch

from .data import Batch, Data

NUM_NODE_FEATURES = 16
NUM_EDGE_FEATURES = 5
VIRTUAL_EDGE_FRACTION = 0.1333


def mesh_edges(n: int) -> np.ndarray:
    """Undirected edges (a < b) of an n x n quad mesh with both diagonals, in element order."""
    idx = np.arange(n * n, dtype=np.int64).reshape(n, n)
    out = []
    # per quad (i, j): perimeter (top, left; bottom/right come from neighbouring quads) + diagonals
    right = np.stack([idx[:, :-1].ravel(), idx[:, 1:].ravel()], 1)
    down = np.stack([idx[:-1, :].ravel(), idx[1:, :].ravel()], 1)
    diag = np.stack([idx[:-1, :-1].ravel(), idx[1:, 1:].ravel()], 1)
    anti = np.stack([idx[:-1, 1:].ravel(), idx[1:, :-1].ravel()], 1)
    out = np.concatenate([right, down, diag, anti], 0)
    return np.sort(out, axis=1)


def random_virtual_edges(num_nodes: int, existing: np.ndarray, rng: np.random.Generator,
                         fraction: float = VIRTUAL_EDGE_FRACTION) -> np.ndarray:
    """int(fraction * len(existing)) distinct new undirected pairs (VirtualEdgeCreate.py:21-49)."""
    target = int(len(existing) * fraction)
    have = set(map(tuple, existing.tolist()))
    chosen: List[Tuple[int, int]] = []
    seen = set()
    while len(chosen) < target:
        a, b = rng.choice(num_nodes, size=2, replace=False)
        e = (int(min(a, b)), int(max(a, b)))
        if e in have or e in seen:
            continue
        seen.add(e)
        chosen.append(e)
    return np.array(chosen, dtype=np.int64).reshape(-1, 2)


def make_mesh_graph(n: int, seed: int, super_node: bool = False, virtual_edges: bool = True) -> Data:
    rng = np.random.default_rng(seed)
    base = mesh_edges(n)
    n_real = n * n
    coords = np.stack(np.meshgrid(np.arange(n), np.arange(n), indexing="xy"), -1).reshape(-1, 2).astype(np.float64)
    feats = [np.zeros((len(base), 1))]  # virtual flag per undirected edge
    und = base
    if super_node:
        s = n_real
        sup = np.stack([np.full(n_real, s, dtype=np.int64), np.arange(n_real, dtype=np.int64)], 1)
        und = np.concatenate([base, sup], 0)
        feats.append(np.ones((n_real, 1)))
        coords = np.concatenate([coords, np.zeros((1, 2))], 0)
    elif virtual_edges:
        ve = random_virtual_edges(n_real, base, rng)
        und = np.concatenate([base, ve], 0)
        feats.append(np.ones((len(ve), 1)))
    vflag = np.concatenate(feats, 0)[:, 0]
    num_nodes = n_real + (1 if super_node else 0)
    # edge features [type, length/1000, dir_x, dir_y, virtual] (GraphCreate.py:352-377, VirtualEdgeCreate.py:75-77)
    d = coords[und[:, 1]] - coords[und[:, 0]]
    length = np.sqrt((d ** 2).sum(1))
    direc = d / np.maximum(length, 1e-12)[:, None]
    ea = np.stack([np.where(vflag > 0, 0.0, 0.01), length / 1000.0, direc[:, 0], direc[:, 1], vflag], 1)
    # both directions, interleaved per undirected edge (GraphCreate.py:420-422)
    ei = np.empty((2, 2 * len(und)), dtype=np.int64)
    ei[0, 0::2], ei[1, 0::2] = und[:, 0], und[:, 1]
    ei[0, 1::2], ei[1, 1::2] = und[:, 1], und[:, 0]
    ea2 = np.repeat(ea, 2, axis=0)
    x = rng.standard_normal((num_nodes, NUM_NODE_FEATURES - 1)).astype(np.float32)
    ind = np.zeros((num_nodes, 1), dtype=np.float32)
    if super_node:
        x[-1] = 0.0
        ind[-1] = 1.0
    x = np.concatenate([x, ind], 1)
    y = rng.uniform(0.5, 1.5, size=(1,)).astype(np.float32)
    return Data(x=torch.from_numpy(x), edge_index=torch.from_numpy(ei),
                edge_attr=torch.from_numpy(ea2.astype(np.float32)), y=torch.from_numpy(y))


CONFIGS = {
    # SURVEY.md §8d / BASELINE.json configs
    "cfg1": dict(n=45, graphs=1, super_node=False),
    "cfg2": dict(n=71, graphs=16, super_node=False),
    "cfg3": dict(n=71, graphs=16, super_node=True),
    "cfg5": dict(n=71, graphs=64, super_node=False),
}


def make_batch(n: int, graphs: int, super_node: bool = False, seed0: int = 0) -> Batch:
    return Batch.from_data_list([make_mesh_graph(n, seed0 + g, super_node=super_node) for g in range(graphs)])


def make_config_batch(name: str, rank: int = 0) -> Batch:
    c = CONFIGS[name]
    return make_batch(c["n"], c["graphs"], c["super_node"], seed0=1000 * rank)
