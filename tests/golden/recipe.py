"""Deterministic recipes shared by the golden generator and the tests: weights from
numpy's PCG64 (stable across machines/versions by design) keyed by state-dict name."""
from __future__ import annotations

import json
from typing import Dict, Tuple

import numpy as np


def make_weights(shapes: Dict[str, Tuple[int, ...]], seed: int) -> Dict[str, np.ndarray]:
    rng = np.random.default_rng(seed)
    out = {}
    for k in sorted(shapes):
        shape = tuple(shapes[k])
        if k.endswith("num_batches_tracked"):
            continue
        if k.endswith("running_mean"):
            v = 0.1 * rng.standard_normal(shape)
        elif k.endswith("running_var"):
            v = 1.0 + 0.2 * rng.random(shape)
        elif "batch_norm" in k and k.endswith("weight"):
            v = 1.0 + 0.1 * rng.standard_normal(shape)
        elif "batch_norm" in k and k.endswith("bias"):
            v = 0.1 * rng.standard_normal(shape)
        elif len(shape) == 2:
            v = rng.standard_normal(shape) / np.sqrt(shape[1])
        else:
            v = 0.1 * rng.standard_normal(shape)
        out[k] = v.astype(np.float32)
    return out


def projection(shape, seed: int = 12345) -> np.ndarray:
    """Fixed random direction used to checksum large gradients."""
    rng = np.random.default_rng(seed + int(np.prod(shape)))
    return rng.standard_normal(shape).astype(np.float64)


def grad_checksum(g: np.ndarray) -> np.ndarray:
    g64 = g.astype(np.float64)
    return np.array([g64.sum(), np.abs(g64).sum(), (g64 * projection(g.shape)).sum()])


def meta_to_array(meta: dict) -> np.ndarray:
    return np.array(json.dumps(meta, sort_keys=True))


def meta_from_array(a: np.ndarray) -> dict:
    return json.loads(str(a))
