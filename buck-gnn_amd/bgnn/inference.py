"""Inference driver: INFERENCE.py's buckling evaluation on the
bgnn path.

INFERENCE.py:133-150,176-186 runs the model in eval mode under no_grad over a DataLoader
and reports, on denormalised eigenvalues, the MAPE summed over graphs divided by the
number of graphs, and the smallest and largest per-graph APE, all in percent. `evaluate`
does the same over any iterable of batches: host-collated `Batch`es, or
`GraphStore.loader(...)` batches gathered on the GPU.
"""
from __future__ import annotations

from typing import Dict, Iterable, Optional

import torch

from .graph import prepare
from .train import EigenvalueScaler


@torch.no_grad()
def evaluate(model, batches: Iterable, normalizer: Optional[EigenvalueScaler] = None,
             device=None) -> Dict[str, float]:
    """Buckling-eigenvalue metrics of INFERENCE.py: mean / min / max APE in percent."""
    model.eval()
    total, n, lo, hi = 0.0, 0, float("inf"), 0.0
    preds = []
    for batch in batches:
        if device is not None:
            batch = batch.to(device)
        prepare(batch.edge_index, batch.x.size(0), batch.batch, getattr(batch, "num_graphs", None) or None)
        pred, _ = model(batch.x, batch.edge_index, batch.edge_attr, batch.batch)
        true = batch.y
        if normalizer is not None:
            true, pred = normalizer.denormalize_eigenvalue(true), normalizer.denormalize_eigenvalue(pred)
        apes = torch.abs((true - pred.view_as(true)) / true)
        # one host read per batch for the three statistics (INFERENCE.py reads them per batch too)
        s, mx, mn = torch.stack([apes.sum(), apes.max(), apes.min()]).tolist()
        total += s * 100
        hi, lo = max(hi, mx * 100), min(lo, mn * 100)
        n += apes.numel()
        preds.append(pred.detach())
    return {"mape": total / max(n, 1), "min_mape": lo if n else 0.0, "max_mape": hi, "graphs": n,
            "predictions": torch.cat(preds) if preds else None}
