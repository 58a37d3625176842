"""Device-side graph structure: edge_index -> CSR (+ transpose) and heavy-row plans.

PyG's `SAGEConv(x, edge_index)` (flow='source_to_target') aggregates, for every
target i = edge_index[1, e], the source rows j = edge_index[0, e]
(Models/BuckGNN.py:342,434). Here edge_index is sorted once per distinct tensor
into a CSR over targets (for the forward) and a CSR over sources (for the
backward), both stable, by `bgnn_graph_build`. Rows with more than `chunk`
entries (the super node of VirtualEdgeCreate.py:81-113 has in-degree N_g) get a
split plan so that one wave never walks thousands of neighbours alone.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field
from typing import Optional

import torch

from . import _lib

DEFAULT_CHUNK = 64
# Rows per row-group of the sum/mean aggregation kernels (bgnn_group_plan; 0 = no plans, the
# per-row sweep kernel). Consecutive mesh rows share most neighbours: with 4 rows per group cfg2
# fetches 5.5 source rows per target row instead of 8.9 (8 rows: 4.7, but twice the registers
# and half the waves per CU; measured slower, tools/tune_agg.py).
GROUP_ROWS = 4


def _ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def require_cuda(*tensors: torch.Tensor, what: str = "bgnn") -> None:
    for t in tensors:
        if t is not None and not t.is_cuda:
            raise RuntimeError(
                f"{what}: tensors must be on a ROCm GPU (got device {t.device}); "
                "bgnn has no CPU fallback")


@dataclass
class Plan:
    """Heavy-row split plan of one CSR (rows with deg > chunk). n_heavy / n_chunks are
    filled on the host after the (single, batched) device->host copy of the counts."""

    heavy_row: torch.Tensor
    heavy_chunk0: torch.Tensor
    chunk_heavy: torch.Tensor
    n_heavy: int
    n_chunks: int
    chunk: int


def enqueue_plan(rowptr: torch.Tensor, n_rows: int, nnz: int, counts: torch.Tensor,
                 chunk: int = DEFAULT_CHUNK) -> Plan:
    """Launch bgnn_heavy_plan; its two counts land in `counts` (device int32[2])."""
    dev = rowptr.device
    heavy_row = torch.empty(max(n_rows, 1), dtype=torch.int32, device=dev)
    heavy_chunk0 = torch.empty(max(n_rows, 1) + 1, dtype=torch.int32, device=dev)
    # sum over heavy rows of ceil(deg/chunk) <= nnz/chunk + n_heavy <= 2*nnz/chunk
    chunk_heavy = torch.empty(2 * (nnz // chunk) + 2, dtype=torch.int32, device=dev)
    ws = torch.empty(_lib.query("bgnn_heavy_plan_ws_bytes", n_rows), dtype=torch.uint8, device=dev)
    _lib.call("bgnn_heavy_plan", rowptr.data_ptr(), n_rows, nnz, chunk, heavy_row.data_ptr(),
              heavy_chunk0.data_ptr(), chunk_heavy.data_ptr(), counts.data_ptr(), ws.data_ptr(), ws.numel(),
              _stream())
    return Plan(heavy_row, heavy_chunk0, chunk_heavy, -1, -1, chunk)


def make_plan(rowptr: torch.Tensor, n_rows: int, nnz: int, chunk: int = DEFAULT_CHUNK) -> Plan:
    counts = torch.empty(2, dtype=torch.int32, device=rowptr.device)
    p = enqueue_plan(rowptr, n_rows, nnz, counts, chunk)
    p.n_heavy, p.n_chunks = counts.tolist()
    return p


@dataclass
class Groups:
    """Row-group plan of a CSR (bgnn_group_plan): per group of at most `rows` consecutive rows,
    its distinct source rows (gsrc) and the mask of the group rows using each (gmask). `grow`
    (optional, [n_groups + 1]) holds each group's first row; None means g * rows."""

    gsrc: torch.Tensor
    gmask: torch.Tensor
    gcnt: torch.Tensor
    rows: int
    grow: Optional[torch.Tensor] = None
    n_groups: int = 0


def enqueue_groups(rowptr: torch.Tensor, col: torch.Tensor, n_rows: int, nnz: int, chunk: int,
                   rows: Optional[int] = None, grow: Optional[torch.Tensor] = None,
                   n_groups: Optional[int] = None) -> Optional[Groups]:
    """Launch bgnn_group_plan (asynchronous) or return None when plans are off / unsupported."""
    rows = GROUP_ROWS if rows is None else rows
    if rows <= 0 or chunk > 64 or n_rows == 0:
        return None
    dev = rowptr.device
    G = int(n_groups) if grow is not None else (n_rows + rows - 1) // rows
    gsrc = torch.empty(max(nnz, 1), dtype=torch.int32, device=dev)
    gmask = torch.empty(max(nnz, 1), dtype=torch.uint8, device=dev)
    gcnt = torch.empty(max(G, 1), dtype=torch.int32, device=dev)
    _lib.call("bgnn_group_plan", rowptr.data_ptr(), col.data_ptr(), n_rows, chunk, rows, _ptr(grow), G,
              gsrc.data_ptr(), gmask.data_ptr(), gcnt.data_ptr(), _stream())
    return Groups(gsrc, gmask, gcnt, rows, grow, G)


@dataclass
class Csr:
    rowptr: torch.Tensor
    col: torch.Tensor
    n_rows: int
    nnz: int
    plan: Plan
    groups: Optional[Groups] = None
    _struct: Optional[_lib.CsrStruct] = field(default=None, repr=False)
    # heavy-row ranges (bgnn_heavy_ranges, ensure_ranges): None until requested; ranges_all = 1 when
    # every heavy row is a range row, 0 when not, -1 unknown (ensure_ranges reads it back once)
    ranges: Optional[torch.Tensor] = field(default=None, repr=False)
    ranges_all: int = -1

    def struct(self) -> _lib.CsrStruct:
        if self._struct is None:
            p = self.plan
            assert p.n_heavy >= 0, "plan counts not resolved (call resolve())"
            gr = self.groups
            self._struct = _lib.CsrStruct(
                self.rowptr.data_ptr(), self.col.data_ptr(), p.heavy_row.data_ptr(),
                p.heavy_chunk0.data_ptr(), p.chunk_heavy.data_ptr(), self.n_rows, self.nnz,
                p.n_heavy, p.n_chunks, p.chunk, max(self.ranges_all, 0) if self.ranges is not None else 0,
                gr.gsrc.data_ptr() if gr else None, gr.gmask.data_ptr() if gr else None,
                gr.gcnt.data_ptr() if gr else None, _ptr(gr.grow) if gr else None,
                gr.n_groups if gr else 0, gr.rows if gr else 0, 0, _ptr(self.ranges))
        return self._struct

    def ensure_ranges(self) -> Optional[torch.Tensor]:
        """The heavy rows' source ranges (bgnn_heavy_ranges; include/bgnn.h): a super node wired to
        its graph's contiguous real-node range is a "range row", whose aggregation the row passes
        sum as a by-product (ranges.hip). Computed once per CSR; when ranges_all is not known (no
        GraphStore hint) it is read back with one host sync."""
        p = self.plan
        if p.n_heavy <= 0:
            return None
        if self.ranges is None:
            buf = torch.empty(_lib.query("bgnn_heavy_ranges_bytes", p.n_heavy) // 4, dtype=torch.int32,
                              device=self.rowptr.device)
            self._struct = None
            _lib.call("bgnn_heavy_ranges", self.ref(), buf.data_ptr(), _stream())
            self.ranges = buf
            if self.ranges_all < 0:
                self.ranges_all = int(int(buf[0].item()) == p.n_heavy)
            self._struct = None
        return self.ranges

    def ref(self):
        return ctypes.byref(self.struct())

    def degree(self) -> torch.Tensor:
        return (self.rowptr[1:] - self.rowptr[:-1])


@dataclass
class Graph:
    """Forward CSR (rows = targets) + transpose CSR (rows = sources) of an edge_index."""

    num_nodes: int
    num_edges: int
    fwd: Csr
    bwd: Csr
    perm_t: torch.Tensor
    edge_index: Optional[torch.Tensor] = field(default=None, repr=False)
    meta: Optional[torch.Tensor] = field(default=None, repr=False)   # device int32[5]: status, counts

    @staticmethod
    def enqueue(edge_index: torch.Tensor, num_nodes: int, chunk: int = DEFAULT_CHUNK) -> "Graph":
        """Launch every build kernel without any host synchronisation; call resolve(meta_host)."""
        require_cuda(edge_index, what="Graph.build")
        if edge_index.dim() != 2 or edge_index.size(0) != 2:
            raise ValueError(f"edge_index must have shape [2, E], got {tuple(edge_index.shape)}")
        ei = edge_index.to(torch.int64).contiguous()
        E = ei.size(1)
        N = int(num_nodes)
        dev = ei.device
        meta = torch.zeros(5, dtype=torch.int32, device=dev)
        rowptr = torch.empty(N + 1, dtype=torch.int32, device=dev)
        rowptr_t = torch.empty(N + 1, dtype=torch.int32, device=dev)
        col = torch.empty(max(E, 1), dtype=torch.int32, device=dev)
        col_t = torch.empty(max(E, 1), dtype=torch.int32, device=dev)
        perm_t = torch.empty(max(E, 1), dtype=torch.int32, device=dev)
        ws = torch.empty(_lib.query("bgnn_graph_build_ws_bytes", E, N), dtype=torch.uint8, device=dev)
        _lib.call("bgnn_graph_build", ei.data_ptr(), E, N, rowptr.data_ptr(), col.data_ptr(),
                  rowptr_t.data_ptr(), col_t.data_ptr(), perm_t.data_ptr(), ws.data_ptr(), ws.numel(),
                  meta.data_ptr(), _stream())
        fwd = Csr(rowptr, col, N, E, enqueue_plan(rowptr, N, E, meta[1:3], chunk),
                  enqueue_groups(rowptr, col, N, E, chunk))
        bwd = Csr(rowptr_t, col_t, N, E, enqueue_plan(rowptr_t, N, E, meta[3:5], chunk),
                  enqueue_groups(rowptr_t, col_t, N, E, chunk))
        return Graph(N, E, fwd, bwd, perm_t, edge_index, meta)

    def resolve(self, meta_host) -> "Graph":
        if int(meta_host[0]) != 0:
            raise IndexError(f"edge_index contains indices outside [0, {self.num_nodes})")
        self.fwd.plan.n_heavy, self.fwd.plan.n_chunks = int(meta_host[1]), int(meta_host[2])
        self.bwd.plan.n_heavy, self.bwd.plan.n_chunks = int(meta_host[3]), int(meta_host[4])
        return self

    @staticmethod
    def build(edge_index: torch.Tensor, num_nodes: int, chunk: int = DEFAULT_CHUNK) -> "Graph":
        g = Graph.enqueue(edge_index, num_nodes, chunk)
        return g.resolve(g.meta.tolist())


@dataclass
class SegmentIndex:
    """CSR of `index -> positions` (global_mean_pool's batch, scatter's index) + its transpose."""

    n: int
    num_rows: int
    fwd: Csr          # rows = segments (graphs), col = positions
    bwd: Csr          # rows = positions, exactly one entry: its segment
    index: Optional[torch.Tensor] = field(default=None, repr=False)   # int64 [n]
    meta: Optional[torch.Tensor] = field(default=None, repr=False)    # device int32[3]

    @staticmethod
    def enqueue(index: torch.Tensor, num_rows: int, chunk: int = DEFAULT_CHUNK) -> "SegmentIndex":
        require_cuda(index, what="SegmentIndex.build")
        idx = index.to(torch.int64).contiguous().view(-1)
        n = idx.numel()
        R = int(num_rows)
        dev = idx.device
        meta = torch.zeros(3, dtype=torch.int32, device=dev)
        rowptr = torch.empty(R + 1, dtype=torch.int32, device=dev)
        col = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
        ws = torch.empty(_lib.query("bgnn_graph_build_ws_bytes", n, R), dtype=torch.uint8, device=dev)
        _lib.call("bgnn_index_csr_build", idx.data_ptr(), n, R, rowptr.data_ptr(), col.data_ptr(),
                  ws.data_ptr(), ws.numel(), meta.data_ptr(), _stream())
        fwd = Csr(rowptr, col, R, n, enqueue_plan(rowptr, R, n, meta[1:3], chunk))
        rowptr_t = torch.arange(n + 1, dtype=torch.int32, device=dev)
        col_t = idx.to(torch.int32)
        empty = Plan(torch.zeros(1, dtype=torch.int32, device=dev), torch.zeros(2, dtype=torch.int32, device=dev),
                     torch.zeros(1, dtype=torch.int32, device=dev), 0, 0, chunk)
        bwd = Csr(rowptr_t, col_t if n > 0 else torch.zeros(1, dtype=torch.int32, device=dev), n, n, empty)
        return SegmentIndex(n, R, fwd, bwd, idx, meta)

    def resolve(self, meta_host) -> "SegmentIndex":
        if int(meta_host[0]) != 0:
            raise IndexError(f"index contains values outside [0, {self.num_rows})")
        self.fwd.plan.n_heavy, self.fwd.plan.n_chunks = int(meta_host[1]), int(meta_host[2])
        return self

    @staticmethod
    def build(index: torch.Tensor, num_rows: int, chunk: int = DEFAULT_CHUNK) -> "SegmentIndex":
        s = SegmentIndex.enqueue(index, num_rows, chunk)
        return s.resolve(s.meta.tolist())


class _Cache:
    """Small identity cache: structure built once per distinct index tensor (and version)."""

    def __init__(self, size: int = 8):
        self.size = size
        self.items = []  # list of (tensor, version, key, value)

    def get(self, t: torch.Tensor, key, builder):
        ver = t._version
        for i, (tt, v, k, val) in enumerate(self.items):
            if tt is t and v == ver and k == key:
                if i:
                    self.items.insert(0, self.items.pop(i))
                return val
        val = builder()
        self.items.insert(0, (t, ver, key, val))
        del self.items[self.size:]
        return val

    def peek(self, t: torch.Tensor, key):
        ver = t._version
        for tt, v, k, val in self.items:
            if tt is t and v == ver and k == key:
                return val
        return None

    def put(self, t: torch.Tensor, key, val):
        self.items.insert(0, (t, t._version, key, val))
        del self.items[self.size:]

    def clear(self):
        self.items.clear()


_graph_cache = _Cache()
_index_cache = _Cache()
_empty_csrs = {}


def empty_csr(n_rows: int, device) -> Csr:
    """A CSR of n_rows rows without entries (cached per size and device). bgnn_sage_fwd over it
    is the SAGE row epilogue alone -- o_i = normalize(z_r[i] + b), its norm and the BatchNorm
    partial sums -- which the aggregate-first max-aggregation layer (bgnn.fused) applies to its
    GEMM output."""
    key = (int(n_rows), str(device))
    c = _empty_csrs.get(key)
    if c is None:
        if len(_empty_csrs) > 8:
            _empty_csrs.clear()
        dev = torch.device(device)
        z = torch.zeros(1, dtype=torch.int32, device=dev)
        plan = Plan(z, torch.zeros(2, dtype=torch.int32, device=dev), z, 0, 0, DEFAULT_CHUNK)
        c = _empty_csrs[key] = Csr(torch.zeros(n_rows + 1, dtype=torch.int32, device=dev), z, n_rows, 0, plan)
    return c


def graph_for(edge_index: torch.Tensor, num_nodes: int, chunk: int = DEFAULT_CHUNK) -> Graph:
    return _graph_cache.get(edge_index, (int(num_nodes), chunk),
                            lambda: Graph.build(edge_index, num_nodes, chunk))


def segments_for(index: torch.Tensor, num_rows: int, chunk: int = DEFAULT_CHUNK) -> SegmentIndex:
    return _index_cache.get(index, (int(num_rows), chunk),
                            lambda: SegmentIndex.build(index, num_rows, chunk))


def clear_caches() -> None:
    _graph_cache.clear()
    _index_cache.clear()


def prepare(edge_index: torch.Tensor, num_nodes: int, batch: Optional[torch.Tensor] = None,
            num_graphs: Optional[int] = None, chunk: int = DEFAULT_CHUNK):
    """Build (or fetch from cache) the graph structure of a mini-batch and the segment
    structure of its `batch` vector with ONE host synchronisation for all status words and
    plan counts, and register them in the caches used by SAGEConv / BuckGNN / pooling."""
    key = (int(num_nodes), chunk)
    g = _graph_cache.peek(edge_index, key)
    s = None
    pending = []
    if g is None:
        g = Graph.enqueue(edge_index, num_nodes, chunk)
        pending.append(g)
    if batch is not None:
        s = _index_cache.peek(batch, ("batch",))
        if s is None:
            n = num_graphs if num_graphs is not None else int(batch.max().item()) + 1
            s = SegmentIndex.enqueue(batch, n, chunk)
            pending.append(s)
    if pending:
        host = torch.cat([p.meta for p in pending]).tolist()
        off = 0
        for p in pending:
            k = p.meta.numel()
            p.resolve(host[off:off + k])
            off += k
        if pending[0] is g:
            _graph_cache.put(edge_index, key, g)
        if s is not None and pending[-1] is s:
            _index_cache.put(batch, ("batch",), s)
    return g, s
