// Graph-structure preprocessing: COO edge_index -> forward/transpose CSR and the
// heavy-row (super node) split plan.
//
// Replaces what PyG's propagate() implies for SAGEConv(x, edge_index) with
// flow='source_to_target' (edge_index[0] = source j, edge_index[1] = target i,
// Models/BuckGNN.py:342,434) on the graphs of Dataset_Preparation/GraphCreate.py:417-422.
// Sorting is a stable LSD radix sort, so the entries of one row keep edge_index
// order and every later reduction is bit-reproducible run to run.
#include "common.h"

#include <hipcub/hipcub.hpp>

namespace bgnn {

namespace {

__global__ void k_split_coo(const int64_t* __restrict__ ei, int64_t E, int64_t N,
                            int32_t* __restrict__ src, int32_t* __restrict__ dst,
                            int32_t* __restrict__ bad) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= E) return;
    int64_t s = ei[e], d = ei[E + e];
    if (s < 0 || s >= N || d < 0 || d >= N) {
        atomicOr(bad, 1);
        s = s < 0 ? 0 : (s >= N ? N - 1 : s);
        d = d < 0 ? 0 : (d >= N ? N - 1 : d);
    }
    src[e] = (int32_t)s;
    dst[e] = (int32_t)d;
}

__global__ void k_index_to_keys(const int64_t* __restrict__ idx, int64_t n, int64_t R,
                                int32_t* __restrict__ keys, int32_t* __restrict__ vals,
                                int32_t* __restrict__ bad) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    int64_t r = idx[i];
    if (r < 0 || r >= R) {
        atomicOr(bad, 1);
        r = r < 0 ? 0 : R - 1;
    }
    keys[i] = (int32_t)r;
    vals[i] = (int32_t)i;
}

__global__ void k_iota(int32_t* __restrict__ v, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) v[i] = (int32_t)i;
}

// rowptr[r] = first position whose sorted key >= r.  Thread e (0..E) fills the
// rows in (key[e-1], key[e]] with e; key[-1] = -1, key[E] = R.
__global__ void k_rowptr_from_sorted(const int32_t* __restrict__ keys, int64_t E, int64_t R,
                                     int32_t* __restrict__ rowptr) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e > E) return;
    const int64_t lo = (e == 0) ? -1 : keys[e - 1];
    const int64_t hi = (e == E) ? R : keys[e];
    for (int64_t r = lo + 1; r <= hi; ++r) rowptr[r] = (int32_t)e;
}

__global__ void k_gather_i32(const int32_t* __restrict__ table, const int32_t* __restrict__ idx,
                             int64_t n, int32_t* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = table[idx[i]];
}

// heavy plan: per row, number of chunks if deg > chunk, else 0; and a 0/1 flag.
__global__ void k_heavy_count(const int32_t* __restrict__ rowptr, int64_t R, int32_t chunk,
                              int32_t* __restrict__ nch, int32_t* __restrict__ flag) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= R) return;
    const int32_t deg = rowptr[r + 1] - rowptr[r];
    const bool heavy = deg > chunk;
    nch[r] = heavy ? (deg + chunk - 1) / chunk : 0;
    flag[r] = heavy ? 1 : 0;
}

__global__ void k_heavy_fill(const int32_t* __restrict__ rowptr, int64_t R, int32_t chunk,
                             const int32_t* __restrict__ nch_off, const int32_t* __restrict__ flag_off,
                             int32_t* __restrict__ heavy_row, int32_t* __restrict__ heavy_chunk0,
                             int32_t* __restrict__ chunk_heavy, int64_t cap, int32_t* __restrict__ counts) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= R) return;
    const int32_t deg = rowptr[r + 1] - rowptr[r];
    if (r == R - 1) {
        const int32_t last_n = deg > chunk ? (deg + chunk - 1) / chunk : 0;
        const int32_t nh = flag_off[r] + (deg > chunk ? 1 : 0);
        const int32_t nc = nch_off[r] + last_n;
        counts[0] = nh;
        counts[1] = nc;
        heavy_chunk0[nh] = nc;
    }
    if (deg <= chunk) return;
    const int32_t h = flag_off[r], c0 = nch_off[r], n = (deg + chunk - 1) / chunk;
    heavy_row[h] = (int32_t)r;
    heavy_chunk0[h] = c0;
    for (int32_t k = 0; k < n && c0 + k < cap; ++k) chunk_heavy[c0 + k] = h;
}

inline int bits_for(int64_t n) {
    int b = 1;
    while ((int64_t(1) << b) < n + 1 && b < 31) ++b;
    return b;
}

inline unsigned grid1d(int64_t n, int t) { return (unsigned)((n + t - 1) / t); }

struct Carve {
    char* p;
    size_t left;
    bool ok = true;
    template <class T>
    T* take(size_t n) {
        size_t b = align_up(n * sizeof(T), 256);
        if (b > left) { ok = false; return nullptr; }
        T* r = reinterpret_cast<T*>(p);
        p += b;
        left -= b;
        return r;
    }
};

size_t radix_tmp_bytes(int64_t E) {
    size_t tmp = 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, tmp, (const int32_t*)nullptr, (int32_t*)nullptr,
                                       (const int32_t*)nullptr, (int32_t*)nullptr, (int)E, 0, 31);
    return tmp;
}

size_t scan_tmp_bytes(int64_t n) {
    size_t tmp = 0;
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, (const int32_t*)nullptr, (int32_t*)nullptr, (int)n);
    return tmp;
}


}  // namespace

}  // namespace bgnn

using namespace bgnn;

extern "C" size_t bgnn_graph_build_ws_bytes(int64_t E, int64_t N) {
    (void)N;
    const int64_t e = E > 0 ? E : 1;
    return 6 * align_up((size_t)e * 4, 256) + 256 + align_up(radix_tmp_bytes(e), 256) + 256;
}

extern "C" int bgnn_graph_build(const int64_t* edge_index, int64_t E, int64_t N, int32_t* rowptr,
                                int32_t* col, int32_t* rowptr_t, int32_t* col_t, int32_t* perm_t,
                                void* ws, size_t ws_bytes, int32_t* dev_status, void* stream) {
    BGNN_REQUIRE(E >= 0 && N >= 0 && N < (int64_t(1) << 31) && E < (int64_t(1) << 31),
                 "graph_build: bad sizes E=%lld N=%lld", (long long)E, (long long)N);
    BGNN_REQUIRE(rowptr && rowptr_t, "graph_build: null rowptr");
    hipStream_t s = as_stream(stream);
    if (dev_status) BGNN_HIP(hipMemsetAsync(dev_status, 0, sizeof(int32_t), s));
    if (N == 0) return BGNN_OK;
    if (E == 0) {
        BGNN_HIP(hipMemsetAsync(rowptr, 0, (N + 1) * sizeof(int32_t), s));
        BGNN_HIP(hipMemsetAsync(rowptr_t, 0, (N + 1) * sizeof(int32_t), s));
        return BGNN_OK;
    }
    BGNN_REQUIRE(edge_index && col && col_t && perm_t, "graph_build: null pointer");
    BGNN_REQUIRE(ws_bytes >= bgnn_graph_build_ws_bytes(E, N), "graph_build: workspace %zu < %zu",
                 ws_bytes, bgnn_graph_build_ws_bytes(E, N));
    Carve c{(char*)ws, ws_bytes};
    int32_t* src = c.take<int32_t>(E);
    int32_t* dst = c.take<int32_t>(E);
    int32_t* dst_sorted = c.take<int32_t>(E);
    int32_t* iota = c.take<int32_t>(E);
    int32_t* src_sorted = c.take<int32_t>(E);
    int32_t* spare = c.take<int32_t>(E);
    int32_t* bad_ws = c.take<int32_t>(64);
    size_t tmp_bytes = radix_tmp_bytes(E);
    void* tmp = c.take<char>(tmp_bytes);
    BGNN_REQUIRE(c.ok, "graph_build: workspace carve failed");
    (void)spare;
    int32_t* bad = dev_status ? dev_status : bad_ws;

    const int T = 256;
    if (!dev_status) BGNN_HIP(hipMemsetAsync(bad, 0, sizeof(int32_t), s));
    k_split_coo<<<grid1d(E, T), T, 0, s>>>(edge_index, E, N, src, dst, bad);
    BGNN_CHECK_LAUNCH();
    const int nb = bits_for(N);
    // forward CSR: key = target, value = source (stable)
    BGNN_HIP(hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, dst, dst_sorted, src, col, (int)E, 0,
                                                nb, s));
    k_rowptr_from_sorted<<<grid1d(E + 1, T), T, 0, s>>>(dst_sorted, E, N, rowptr);
    BGNN_CHECK_LAUNCH();
    // transpose CSR: key = source (in forward-CSR order), value = forward position
    k_iota<<<grid1d(E, T), T, 0, s>>>(iota, E);
    BGNN_CHECK_LAUNCH();
    BGNN_HIP(hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, col, src_sorted, iota, perm_t,
                                                (int)E, 0, nb, s));
    k_rowptr_from_sorted<<<grid1d(E + 1, T), T, 0, s>>>(src_sorted, E, N, rowptr_t);
    BGNN_CHECK_LAUNCH();
    k_gather_i32<<<grid1d(E, T), T, 0, s>>>(dst_sorted, perm_t, E, col_t);
    BGNN_CHECK_LAUNCH();
    return BGNN_OK;
}

extern "C" int bgnn_index_csr_build(const int64_t* index, int64_t n, int64_t R, int32_t* rowptr,
                                    int32_t* col, void* ws, size_t ws_bytes, int32_t* dev_status,
                                    void* stream) {
    BGNN_REQUIRE(n >= 0 && R >= 0 && n < (int64_t(1) << 31) && R < (int64_t(1) << 31),
                 "index_csr_build: bad sizes");
    hipStream_t s = as_stream(stream);
    if (dev_status) BGNN_HIP(hipMemsetAsync(dev_status, 0, sizeof(int32_t), s));
    if (R == 0) return BGNN_OK;
    if (n == 0) {
        BGNN_HIP(hipMemsetAsync(rowptr, 0, (R + 1) * sizeof(int32_t), s));
        return BGNN_OK;
    }
    BGNN_REQUIRE(ws_bytes >= bgnn_graph_build_ws_bytes(n, R), "index_csr_build: workspace too small");
    Carve c{(char*)ws, ws_bytes};
    int32_t* keys = c.take<int32_t>(n);
    int32_t* vals = c.take<int32_t>(n);
    int32_t* keys_sorted = c.take<int32_t>(n);
    c.take<int32_t>(n);
    c.take<int32_t>(n);
    c.take<int32_t>(n);
    int32_t* bad_ws = c.take<int32_t>(64);
    size_t tmp_bytes = radix_tmp_bytes(n);
    void* tmp = c.take<char>(tmp_bytes);
    BGNN_REQUIRE(c.ok, "index_csr_build: workspace carve failed");
    int32_t* bad = dev_status ? dev_status : bad_ws;
    const int T = 256;
    if (!dev_status) BGNN_HIP(hipMemsetAsync(bad, 0, sizeof(int32_t), s));
    k_index_to_keys<<<grid1d(n, T), T, 0, s>>>(index, n, R, keys, vals, bad);
    BGNN_CHECK_LAUNCH();
    BGNN_HIP(hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, keys, keys_sorted, vals, col, (int)n,
                                                0, bits_for(R), s));
    k_rowptr_from_sorted<<<grid1d(n + 1, T), T, 0, s>>>(keys_sorted, n, R, rowptr);
    BGNN_CHECK_LAUNCH();
    return BGNN_OK;
}

extern "C" size_t bgnn_heavy_plan_ws_bytes(int64_t R) {
    const int64_t r = R > 0 ? R : 1;
    return 4 * align_up((size_t)r * 4, 256) + align_up(scan_tmp_bytes(r), 256) + 512;
}

extern "C" int bgnn_heavy_plan(const int32_t* rowptr, int64_t R, int64_t nnz, int32_t chunk,
                               int32_t* heavy_row, int32_t* heavy_chunk0, int32_t* chunk_heavy,
                               int32_t* dev_counts, void* ws, size_t ws_bytes, void* stream) {
    BGNN_REQUIRE(chunk > 0, "heavy_plan: chunk must be > 0");
    BGNN_REQUIRE(dev_counts, "heavy_plan: dev_counts is required");
    hipStream_t s = as_stream(stream);
    const int64_t cap = 2 * (nnz / chunk) + 2;   // capacity of chunk_heavy (see bgnn.h)
    if (R == 0) {
        BGNN_HIP(hipMemsetAsync(dev_counts, 0, 2 * sizeof(int32_t), s));
        return BGNN_OK;
    }
    BGNN_REQUIRE(ws_bytes >= bgnn_heavy_plan_ws_bytes(R), "heavy_plan: workspace too small");
    Carve c{(char*)ws, ws_bytes};
    int32_t* nch = c.take<int32_t>(R);
    int32_t* flag = c.take<int32_t>(R);
    int32_t* nch_off = c.take<int32_t>(R);
    int32_t* flag_off = c.take<int32_t>(R);
    size_t tmp_bytes = scan_tmp_bytes(R);
    void* tmp = c.take<char>(tmp_bytes);
    BGNN_REQUIRE(c.ok, "heavy_plan: workspace carve failed");
    const int T = 256;
    k_heavy_count<<<grid1d(R, T), T, 0, s>>>(rowptr, R, chunk, nch, flag);
    BGNN_CHECK_LAUNCH();
    BGNN_HIP(hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, nch, nch_off, (int)R, s));
    BGNN_HIP(hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, flag, flag_off, (int)R, s));
    k_heavy_fill<<<grid1d(R, T), T, 0, s>>>(rowptr, R, chunk, nch_off, flag_off, heavy_row,
                                            heavy_chunk0, chunk_heavy, cap, dev_counts);
    BGNN_CHECK_LAUNCH();
    return BGNN_OK;
}

