"""Device-resident graph store and on-device mini-batching.

The reference keeps its dataset as a host list of PyG `Data` (a pickled
`dataset_cache_*.pkl`, GraphCreate.py:562-568) and collates every mini-batch on the host
(`DataLoader`, TRAIN_FINAL.py:1298-1302); the GPU then sees a new `edge_index` each step.
On MI355X the whole dataset fits in HBM (80,000 cfg4 meshes ~ 150 GB of 288 GB), so
`GraphStore` uploads it once, builds every graph's CSR / transpose CSR once (one stable
`bgnn_graph_build` per group of graphs) and keeps them graph-local. A mini-batch is then
assembled on the device by two C-ABI calls (`bgnn_store_gather_graph`,
`bgnn_store_gather_rows`) from a 16-row offset table: no host collation, no per-step
sort and no host synchronisation. The batch's graph structure and pooling segments are
registered in the caches `bgnn.prepare` / SAGEConv / BuckGNN consult, and they are
identical to what `Graph.build` would produce from the collated `edge_index`.

Collation follows PyG (and bgnn.data.Batch): per-node tensors (first dim = num_nodes)
and per-edge tensors (first dim = num_edges) are concatenated, `edge_index` is offset by
the running node count, per-graph tensors are concatenated along dim 0, `batch` and `ptr`
are added.
"""
from __future__ import annotations

from typing import Dict, Iterator, List, Optional, Sequence

import numpy as np
import torch

from . import _lib
from .data import Batch, Data
from . import graph as _graph
from .graph import (DEFAULT_CHUNK, Csr, Graph, Groups, Plan, SegmentIndex, _graph_cache, _index_cache, _stream,
                    enqueue_groups, enqueue_plan)

_GROUP_EDGES = 1 << 30   # graphs are CSR-built in groups of < 2^30 edges (int32 positions)


def _heavy_counts(rowptr: torch.Tensor, gid: torch.Tensor, G: int, chunk: int):
    """Per-graph (rows with degree > chunk, sum of their ceil(deg / chunk))."""
    deg = (rowptr[1:] - rowptr[:-1]).to(torch.int64)
    heavy = deg > chunk
    chunks = torch.where(heavy, (deg + chunk - 1) // chunk, torch.zeros_like(deg))
    h = torch.zeros(G, dtype=torch.int64, device=rowptr.device).index_add_(0, gid, heavy.to(torch.int64))
    c = torch.zeros(G, dtype=torch.int64, device=rowptr.device).index_add_(0, gid, chunks)
    return h, c


class GraphStore:
    """All graphs of a dataset resident on one GPU, with graph-local CSR structures."""

    def __init__(self, graphs: Sequence[Data], device=None, chunk: int = DEFAULT_CHUNK):
        if len(graphs) == 0:
            raise ValueError("GraphStore: empty dataset")
        dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        if dev.type != "cuda":
            raise RuntimeError("GraphStore: the store lives in GPU memory (bgnn has no CPU fallback)")
        self.device = dev
        self.chunk = chunk
        self._empty_plan = None
        G = len(graphs)
        self.num_graphs = G
        n = np.array([d.num_nodes for d in graphs], dtype=np.int64)
        e = np.array([d.num_edges for d in graphs], dtype=np.int64)
        if (e >= (1 << 31)).any() or (n >= (1 << 31)).any():
            raise ValueError("GraphStore: a single graph must have < 2^31 nodes and edges")
        self.n_nodes, self.n_edges = n, e
        self.node_off = np.concatenate([[0], np.cumsum(n)])
        self.edge_off = np.concatenate([[0], np.cumsum(e)])

        # classify attributes like PyG collation
        keys: List[str] = []
        for d in graphs:
            for k in d.keys():
                if k not in keys and k not in ("num_nodes", "batch", "ptr"):
                    keys.append(k)
        self.node_keys, self.edge_keys, self.graph_keys, self.other_keys = [], [], [], []
        for k in keys:
            vals = [d._store.get(k) for d in graphs]
            if k == "edge_index":
                continue
            if not all(isinstance(v, torch.Tensor) for v in vals):
                self.other_keys.append(k)
            # (PyG concatenates every tensor along dim 0; the class only picks the gather path)
            elif all(v.dim() > 0 and v.size(0) == d.num_nodes for v, d in zip(vals, graphs)):
                self.node_keys.append(k)
            elif all(v.dim() > 0 and v.size(0) == d.num_edges for v, d in zip(vals, graphs)):
                self.edge_keys.append(k)
            else:
                self.graph_keys.append(k)

        self.node_data: Dict[str, torch.Tensor] = {
            k: torch.cat([d._store[k] for d in graphs], 0).to(dev).contiguous() for k in self.node_keys}
        self.edge_data: Dict[str, torch.Tensor] = {
            k: torch.cat([d._store[k] for d in graphs], 0).to(dev).contiguous() for k in self.edge_keys}
        self.graph_data: Dict[str, List[torch.Tensor]] = {}
        self.graph_stacked: Dict[str, torch.Tensor] = {}
        for k in self.graph_keys:
            vals = [d._store[k] for d in graphs]
            if all(v.dim() == 0 for v in vals):
                self.graph_stacked[k] = torch.stack(vals).to(dev)
            elif all(v.shape == vals[0].shape for v in vals):
                self.graph_stacked[k] = torch.stack(vals).to(dev)     # [G, *shape]: gather + flatten dim 0
            else:
                self.graph_data[k] = [v.to(dev) for v in vals]
        self.other = {k: [d._store.get(k) for d in graphs] for k in self.other_keys}

        # graph-local edge_index (int32) and CSRs, built once per group of graphs
        sumN, sumE = int(self.node_off[-1]), int(self.edge_off[-1])
        ei_l = torch.empty(2, max(sumE, 1), dtype=torch.int32, device=dev)
        self.rowptr = torch.empty(max(sumN, 1), dtype=torch.int32, device=dev)
        self.rowptr_t = torch.empty(max(sumN, 1), dtype=torch.int32, device=dev)
        self.col = torch.empty(max(sumE, 1), dtype=torch.int32, device=dev)
        self.col_t = torch.empty(max(sumE, 1), dtype=torch.int32, device=dev)
        self.perm_t = torch.empty(max(sumE, 1), dtype=torch.int32, device=dev)
        heavy = torch.zeros(G, 4, dtype=torch.int64, device=dev)
        # row-group plans (bgnn_group_plan), per graph: groups start at the graph's first node, so
        # a batch's plan is the concatenation of its graphs' plans (bgnn_store_gather_groups)
        R = _graph.GROUP_ROWS if chunk <= 64 else 0
        self.group_rows = R
        if R > 0:
            self.n_groups = (n + R - 1) // R
            self.group_off = np.concatenate([[0], np.cumsum(self.n_groups)])
            sumG = int(self.group_off[-1])
            self.gsrc = torch.empty(max(sumE, 1), dtype=torch.int32, device=dev)
            self.gmask = torch.empty(max(sumE, 1), dtype=torch.uint8, device=dev)
            self.gsrc_t = torch.empty(max(sumE, 1), dtype=torch.int32, device=dev)
            self.gmask_t = torch.empty(max(sumE, 1), dtype=torch.uint8, device=dev)
            self.gcnt = torch.zeros(max(sumG, 1), dtype=torch.int32, device=dev)
            self.gcnt_t = torch.zeros(max(sumG, 1), dtype=torch.int32, device=dev)
        self.ranges_all = [True, True]   # (fwd, bwd): every heavy row a range row (_build_group)
        g0 = 0
        while g0 < G:
            g1 = g0 + 1
            while g1 < G and self.edge_off[g1 + 1] - self.edge_off[g0] < _GROUP_EDGES:
                g1 += 1
            self._build_group(graphs, g0, g1, ei_l, heavy)
            g0 = g1
        self.edge_index = ei_l
        self.heavy = heavy.cpu().numpy()          # per graph: fwd heavy rows, fwd chunks, bwd rows, bwd chunks
        self._ptr_cache: Dict[int, torch.Tensor] = {}

    def _build_group(self, graphs, g0, g1, ei_l, heavy):
        dev = self.device
        n0, n1 = int(self.node_off[g0]), int(self.node_off[g1])
        e0, e1 = int(self.edge_off[g0]), int(self.edge_off[g1])
        Gg = g1 - g0
        ei = torch.cat([graphs[g]._store["edge_index"].to(torch.int64) + int(self.node_off[g] - n0)
                        for g in range(g0, g1)], 1).to(dev) if e1 > e0 else \
            torch.zeros(2, 0, dtype=torch.int64, device=dev)
        gr = Graph.build(ei, n1 - n0, self.chunk)
        noff = torch.as_tensor(self.node_off[g0:g1] - n0, device=dev)
        eoff = torch.as_tensor(self.edge_off[g0:g1] - e0, device=dev)
        gid_n = torch.repeat_interleave(torch.arange(Gg, device=dev), torch.as_tensor(self.n_nodes[g0:g1], device=dev))
        gid_e = torch.repeat_interleave(torch.arange(Gg, device=dev), torch.as_tensor(self.n_edges[g0:g1], device=dev))
        if n1 > n0:
            self.rowptr[n0:n1] = (gr.fwd.rowptr[:-1].to(torch.int64) - eoff[gid_n]).to(torch.int32)
            self.rowptr_t[n0:n1] = (gr.bwd.rowptr[:-1].to(torch.int64) - eoff[gid_n]).to(torch.int32)
        if e1 > e0:
            # CSR entries of graph g occupy [edge_off[g], edge_off[g+1]) in both sorted orders
            self.col[e0:e1] = (gr.fwd.col[:e1 - e0].to(torch.int64) - noff[gid_e]).to(torch.int32)
            self.col_t[e0:e1] = (gr.bwd.col[:e1 - e0].to(torch.int64) - noff[gid_e]).to(torch.int32)
            self.perm_t[e0:e1] = (gr.perm_t[:e1 - e0].to(torch.int64) - eoff[gid_e]).to(torch.int32)
            ei_l[:, e0:e1] = (ei - noff[gid_e]).to(torch.int32)
        R = self.group_rows
        if R > 0 and n1 > n0:
            # groups of R rows from each graph's first node (graph-local after the rebase below)
            ng = self.n_groups[g0:g1]
            k = np.arange(int(ng.sum())) - np.repeat(self.group_off[g0:g1] - self.group_off[g0], ng)
            grow = np.concatenate([np.repeat(self.node_off[g0:g1] - n0, ng) + k * R, [n1 - n0]])
            grow_d = torch.from_numpy(grow.astype(np.int32)).to(dev)
            G0, G1 = int(self.group_off[g0]), int(self.group_off[g1])
            for csr, gsrc, gmask, gcnt in ((gr.fwd, self.gsrc, self.gmask, self.gcnt),
                                           (gr.bwd, self.gsrc_t, self.gmask_t, self.gcnt_t)):
                p = enqueue_groups(csr.rowptr, csr.col, n1 - n0, e1 - e0, self.chunk, R, grow_d, G1 - G0)
                gcnt[G0:G1] = p.gcnt[:G1 - G0]
                if e1 > e0:
                    # keys of a group lie inside its graph's edge range: graph-local source ids
                    gsrc[e0:e1] = (p.gsrc[:e1 - e0].to(torch.int64) - noff[gid_e]).to(torch.int32)
                    gmask[e0:e1] = p.gmask[:e1 - e0]
        hf, cf = _heavy_counts(gr.fwd.rowptr, gid_n, Gg, self.chunk)
        hb, cb = _heavy_counts(gr.bwd.rowptr, gid_n, Gg, self.chunk)
        heavy[g0:g1] = torch.stack([hf, cf, hb, cb], 1)
        # range rows (graph.Csr.ensure_ranges): whether every heavy row of these graphs is one; a
        # graph's ranges are graph-local and stay increasing and disjoint in any batch of graphs, so
        # the store-wide answer holds for every batch (its CSRs then skip the read-back)
        for i, csr in enumerate((gr.fwd, gr.bwd)):
            if csr.plan.n_heavy > 0:
                csr.ensure_ranges()
                self.ranges_all[i] = self.ranges_all[i] and csr.ranges_all == 1

    # ------------------------------------------------------------------------------------
    def batch(self, graph_ids: Sequence[int]) -> Batch:
        """Assemble the mini-batch of the given graphs on the device (PyG collation order)."""
        ids = np.asarray(graph_ids, dtype=np.int64)
        B = ids.size
        if B == 0:
            raise ValueError("GraphStore.batch: empty selection")
        if ids.min() < 0 or ids.max() >= self.num_graphs:
            raise IndexError("GraphStore.batch: graph id out of range")
        dev = self.device
        nn_, ne = self.n_nodes[ids], self.n_edges[ids]
        dn = np.concatenate([[0], np.cumsum(nn_)])
        de = np.concatenate([[0], np.cumsum(ne)])
        Nb, Eb = int(dn[-1]), int(de[-1])
        if Eb >= (1 << 31):
            raise ValueError("GraphStore.batch: a batch must have < 2^31 edges")
        table = np.stack([self.node_off[ids], dn[:-1], nn_, self.edge_off[ids], de[:-1], ne], 1)
        # every small host array of the batch in ONE pinned upload (one copy launch instead of four):
        # [table (B x 6) | graph ids (B) | ptr (B + 1) | group table (B x 7, when planned)]
        gt = self._group_table(ids, dn, de, ne)
        parts = [table.reshape(-1), ids, dn] + ([gt.reshape(-1)] if gt is not None else [])
        offs, n = [], 0
        for a in parts:   # each part starts 16-B aligned on the device
            offs.append(n)
            n += (len(a) + 1) // 2 * 2
        host = torch.zeros(n, dtype=torch.int64).pin_memory()
        hv = host.numpy()
        for o, a in zip(offs, parts):
            hv[o:o + len(a)] = a
        up = host.to(dev, non_blocking=True)
        table_d, sel_d, ptr = up[offs[0]:offs[0] + 6 * B], up[offs[1]:offs[1] + B], up[offs[2]:offs[2] + B + 1]
        gt_d = up[offs[3]:offs[3] + 7 * B] if gt is not None else None
        s = _stream()
        ei_b = torch.empty(2, Eb, dtype=torch.int64, device=dev)
        rowptr = torch.empty(Nb + 1, dtype=torch.int32, device=dev)
        rowptr_t = torch.empty(Nb + 1, dtype=torch.int32, device=dev)
        col = torch.empty(max(Eb, 1), dtype=torch.int32, device=dev)
        col_t = torch.empty(max(Eb, 1), dtype=torch.int32, device=dev)
        perm_t = torch.empty(max(Eb, 1), dtype=torch.int32, device=dev)
        batch = torch.empty(Nb, dtype=torch.int64, device=dev)
        _lib.call("bgnn_store_gather_graph", table_d.data_ptr(), B, Nb, Eb, int(nn_.max()), int(ne.max()),
                  self.edge_index.data_ptr(), self.edge_index.stride(0), self.rowptr.data_ptr(), self.col.data_ptr(),
                  self.rowptr_t.data_ptr(), self.col_t.data_ptr(), self.perm_t.data_ptr(), ei_b.data_ptr(),
                  rowptr.data_ptr(), col.data_ptr(), rowptr_t.data_ptr(), col_t.data_ptr(), perm_t.data_ptr(),
                  batch.data_ptr(), s)
        out = Batch()
        st = out._store
        for k, src in self.node_data.items():
            st[k] = self._gather_rows(table_d, B, 0, int(nn_.max()), src, Nb)
        st["edge_index"] = ei_b
        for k, src in self.edge_data.items():
            st[k] = self._gather_rows(table_d, B, 1, int(ne.max()), src, Eb)
        for k, t in self.graph_stacked.items():
            v = t.index_select(0, sel_d)
            st[k] = v if v.dim() == 1 else v.reshape(-1, *v.shape[2:])
        for k, lst in self.graph_data.items():
            st[k] = torch.cat([lst[i] for i in ids], 0)
        for k, lst in self.other.items():
            st[k] = [lst[i] for i in ids]
        st["batch"] = batch
        st["ptr"] = ptr
        st["num_graphs"] = B
        st["num_nodes"] = Nb

        # graph structure of the batch, registered for prepare()/SAGEConv/BuckGNN
        hv = self.heavy[ids].sum(0)
        gf, gb = self._groups(ids, gt_d, dn, de, ne, Nb, Eb)
        fwd = Csr(rowptr, col, Nb, Eb, self._plan(rowptr, Nb, Eb, int(hv[0]), int(hv[1])), gf,
                  ranges_all=int(self.ranges_all[0]))
        bwd = Csr(rowptr_t, col_t, Nb, Eb, self._plan(rowptr_t, Nb, Eb, int(hv[2]), int(hv[3])), gb,
                  ranges_all=int(self.ranges_all[1]))
        graph = Graph(Nb, Eb, fwd, bwd, perm_t, ei_b, None)
        _graph_cache.put(ei_b, (Nb, self.chunk), graph)
        # pooling segments: graph b owns positions [ptr[b], ptr[b+1])
        ptr32 = ptr.to(torch.int32)
        seg_f = Csr(ptr32, self._arange(Nb), B, Nb, self._plan_host(dn))
        if self._empty_plan is None:   # (constant: no heavy rows in the pooling transpose)
            self._empty_plan = Plan(torch.zeros(1, dtype=torch.int32, device=dev),
                                    torch.zeros(2, dtype=torch.int32, device=dev),
                                    torch.zeros(1, dtype=torch.int32, device=dev), 0, 0, self.chunk)
        seg_b = Csr(self._arange(Nb + 1), batch.to(torch.int32), Nb, Nb, self._empty_plan)
        _index_cache.put(batch, ("batch",), SegmentIndex(Nb, B, seg_f, seg_b, batch, None))
        return out

    def _group_table(self, ids, dn, de, ne):
        """Host table of the batch's row-group gather (None without row-group plans)."""
        if self.group_rows <= 0 or int(dn[-1]) == 0:
            return None
        ng = self.n_groups[ids]
        dg = np.concatenate([[0], np.cumsum(ng)])
        return np.stack([dn[:-1], self.edge_off[ids], de[:-1], ne, self.group_off[ids], dg[:-1], ng], 1).astype(np.int64)

    def _groups(self, ids, gt_d, dn, de, ne, Nb, Eb):
        """The batch's row-group plans (forward and transpose CSR) from the per-graph plans;
        gt_d: the uploaded _group_table."""
        R = self.group_rows
        if R <= 0 or Nb == 0:
            return None, None
        dev = self.device
        ng = self.n_groups[ids]
        Gb = int(ng.sum())
        out = [torch.empty(max(Eb, 1), dtype=torch.int32, device=dev), torch.empty(max(Eb, 1), dtype=torch.uint8, device=dev),
               torch.empty(max(Gb, 1), dtype=torch.int32, device=dev),
               torch.empty(max(Eb, 1), dtype=torch.int32, device=dev), torch.empty(max(Eb, 1), dtype=torch.uint8, device=dev),
               torch.empty(max(Gb, 1), dtype=torch.int32, device=dev)]
        grow = torch.empty(Gb + 1, dtype=torch.int32, device=dev)
        _lib.call("bgnn_store_gather_groups", gt_d.data_ptr(), len(ids), R, Nb, Gb, int(ne.max()), int(ng.max()),
                  self.gsrc.data_ptr(), self.gmask.data_ptr(), self.gcnt.data_ptr(), self.gsrc_t.data_ptr(),
                  self.gmask_t.data_ptr(), self.gcnt_t.data_ptr(), *[t.data_ptr() for t in out], grow.data_ptr(),
                  _stream())
        return (Groups(out[0], out[1], out[2], R, grow, Gb), Groups(out[3], out[4], out[5], R, grow, Gb))

    def _gather_rows(self, table_d, B, per_edge, max_rows, src, n_out):
        out = torch.empty((n_out,) + tuple(src.shape[1:]), dtype=src.dtype, device=src.device)
        row_bytes = src[0].numel() * src.element_size() if src.size(0) else 0
        if n_out == 0 or row_bytes == 0:
            return out
        if row_bytes % 4:
            raise ValueError("GraphStore: per-row attribute size must be a multiple of 4 bytes")
        _lib.call("bgnn_store_gather_rows", table_d.data_ptr(), B, per_edge, max_rows, src.data_ptr(), row_bytes,
                  out.data_ptr(), _stream())
        return out

    def _plan(self, rowptr, n_rows, nnz, n_heavy, n_chunks) -> Plan:
        if n_heavy == 0:   # no row above `chunk` (cfg2 meshes): nothing to plan, no launch
            z = self._zeros_i32()
            return Plan(z, z, z, 0, 0, self.chunk)
        counts = torch.empty(2, dtype=torch.int32, device=self.device)   # device copy unused: counts known
        p = enqueue_plan(rowptr, n_rows, nnz, counts, self.chunk)
        p.n_heavy, p.n_chunks = n_heavy, n_chunks
        return p

    def _plan_host(self, rowptr_h: np.ndarray) -> Plan:
        """Heavy-row plan of a CSR whose rowptr the host holds (the pooling segments: one row per
        graph), computed in numpy and uploaded in one copy -- the same arrays bgnn_heavy_plan
        writes: heavy rows ascending, heavy_chunk0 = running chunk counts, chunk -> heavy row."""
        deg = np.diff(np.asarray(rowptr_h, dtype=np.int64))
        heavy = np.nonzero(deg > self.chunk)[0]
        if heavy.size == 0:
            z = self._zeros_i32()
            return Plan(z, z, z, 0, 0, self.chunk)
        nch = (deg[heavy] + self.chunk - 1) // self.chunk
        c0 = np.concatenate([[0], np.cumsum(nch)])
        ch = np.repeat(np.arange(heavy.size), nch)
        pack = torch.from_numpy(np.concatenate([heavy, c0, ch]).astype(np.int32)).pin_memory()
        d = pack.to(self.device, non_blocking=True)
        h = heavy.size
        return Plan(d[:h], d[h:2 * h + 1], d[2 * h + 1:], int(h), int(c0[-1]), self.chunk)

    def _zeros_i32(self) -> torch.Tensor:
        z = self._ptr_cache.get("zeros")
        if z is None:
            z = torch.zeros(2, dtype=torch.int32, device=self.device)
            self._ptr_cache["zeros"] = z
        return z

    def _arange(self, n: int) -> torch.Tensor:
        t = self._ptr_cache.get(n)
        if t is None:
            t = torch.arange(max(n, 1), dtype=torch.int32, device=self.device)
            self._ptr_cache[n] = t
        return t

    def loader(self, batch_size: int, shuffle: bool = False, seed: int = 0, drop_last: bool = False,
               epoch: int = 0, rank: int = 0, world_size: int = 1) -> Iterator[Batch]:
        """Iterate mini-batches of one epoch (DataLoader semantics; with world_size > 1 each rank
        takes a disjoint DistributedSampler-style shard of the shuffled order)."""
        order = np.arange(self.num_graphs)
        if shuffle:
            order = np.random.default_rng(seed + epoch).permutation(self.num_graphs)
        order = order[rank::world_size]
        for i in range(0, len(order), batch_size):
            ids = order[i:i + batch_size]
            if drop_last and len(ids) < batch_size:
                break
            yield self.batch(ids)
