"""ORACLE — test infrastructure only, never part of the product path.

CPU restatement (plain PyTorch fp32 on the CPU) of the arithmetic on buck-gnn's
GraphSAGE hot path, used as the checker for the HIP path:

* pyg_ref.py     — the third-party ops the reference calls (torch_geometric
                   SAGEConv / global_*_pool / Batch collation, torch_scatter
                   scatter_add / scatter_mean). PyG is NOT installed and the
                   reference pins no version (README.md:64-70: "PyTorch 1.10+,
                   PyTorch Geometric"); the restatement follows PyG's published
                   SAGEConv formula (MessagePassing with flow='source_to_target',
                   message x_j = x[edge_index[0]], aggregation at edge_index[1],
                   lin_l with bias, lin_r without, F.normalize(p=2, eps=1e-12)).
* buckgnn_ref.py — the BuckGNN SAGE layer loops (Models/BuckGNN.py:338-352,
                   430-471), pooling (:246-307), decoder, RelativeErrorLoss
                   (Utils/Losses.py:755-761) and the Adam train step
                   (TRAIN_FINAL.py:190,253-298).
* shim.py        — installs pyg_ref as `torch_geometric`/`torch_scatter` so the
                   reference's own Models/BuckGNN.py can be imported IN THIS
                   CONTAINER ONLY to generate tests/golden fixtures.

Pinning: the model orchestration is pinned by golden vectors produced by the
reference's own Models/BuckGNN.py running over pyg_ref (tests/golden/make_golden.py);
the PyG op semantics themselves are pinned only by hand-derived known-answer tests
(tests/test_oracle.py) — the reference ships no tests or fixtures,
so parity at the PyG boundary is "pinned by KATs of the documented formula".

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this package.
"""
