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

// Row-group plan (bgnn.h, bgnn_group_plan): one wave per group of R consecutive rows, four
// groups per 256-thread block, all in registers (lane k of register chunk c holds entry
// 64c+k of the group). The group's light-row entries are concatenated in row order (row t =
// bit t); an entry's key is (source, occurrence of that source earlier in the same row), so a
// duplicate edge stays two entries. Keys are numbered by first appearance; each key gets the
// mask of the rows that hold it. O(n^2 / 64) wave steps for n entries (n ~ 36 on meshes at
// R = 4). The result depends only on the CSR (deterministic).
template <int C>   // register chunks: R * chunk <= 64 * C
__global__ __launch_bounds__(256) void k_group_plan(const int32_t* __restrict__ rowptr,
                                                    const int32_t* __restrict__ col, int64_t N, int32_t chunk,
                                                    int32_t R, const int32_t* __restrict__ grow, int64_t G,
                                                    int32_t* __restrict__ gsrc, uint8_t* __restrict__ gmask,
                                                    int32_t* __restrict__ gcnt) {
    const int lane = threadIdx.x & 63;
    const int64_t g = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (g >= G) return;   // whole wave
    const int64_t r0 = grow ? grow[g] : g * R;
    const int rows = (int)min((int64_t)R, (grow ? (int64_t)grow[g + 1] : N) - r0);
    const int32_t rp = lane <= rows ? rowptr[r0 + lane] : 0;
    const int32_t base = __builtin_amdgcn_readfirstlane(__shfl(rp, 0));
    // light rows' entry offsets inside the group
    int off[9], rb[8];
    off[0] = 0;
#pragma unroll
    for (int t = 0; t < 8; ++t) {
        rb[t] = 0;
        off[t + 1] = off[t];
        if (t < rows) {
            const int32_t b = __shfl(rp, t), d = __shfl(rp, t + 1) - b;
            rb[t] = b;
            if (d <= chunk) off[t + 1] += d;   // heavy row: chunk / combine kernels
        }
    }
    const int n = off[8];
    int32_t src[C], row[C], occ[C], fst[C];
#pragma unroll
    for (int c = 0; c < C; ++c) {
        const int k = c * 64 + lane;
        src[c] = -1;
        row[c] = -1;
        occ[c] = 0;
        fst[c] = k;
        if (k < n) {
            int t = 0;
#pragma unroll
            for (int q = 1; q < 8; ++q) t = (k >= off[q]) ? q : t;   // off is non-decreasing
            row[c] = t;
            src[c] = col[rb[t] + (k - off[t])];
        }
    }
    // occurrence of each entry's source earlier in the same row
#pragma unroll
    for (int ci = 0; ci < C; ++ci) {
        const int m = min(64, n - ci * 64);
        for (int ii = 0; ii < m; ++ii) {
            const int32_t si = __builtin_amdgcn_readlane(src[ci], ii);
            const int32_t ti = __builtin_amdgcn_readlane(row[ci], ii);
            const int i = ci * 64 + ii;
#pragma unroll
            for (int c = 0; c < C; ++c) occ[c] += (i < c * 64 + lane && ti == row[c] && si == src[c]) ? 1 : 0;
        }
    }
    // first entry with the same key (same source, same occurrence number)
#pragma unroll
    for (int ci = C - 1; ci >= 0; --ci) {
        const int m = min(64, n - ci * 64);
        for (int ii = m - 1; ii >= 0; --ii) {   // descending: the last hit is the first entry
            const int32_t si = __builtin_amdgcn_readlane(src[ci], ii);
            const int32_t oi = __builtin_amdgcn_readlane(occ[ci], ii);
            const int i = ci * 64 + ii;
#pragma unroll
            for (int c = 0; c < C; ++c) fst[c] = (i < c * 64 + lane && si == src[c] && oi == occ[c]) ? i : fst[c];
        }
    }
    // number the keys by first appearance
    int ent[C];
    int cnt = 0;
#pragma unroll
    for (int c = 0; c < C; ++c) {
        const int k = c * 64 + lane;
        const bool fresh = k < n && fst[c] == k;
        const uint64_t bal = __ballot(fresh);
        ent[c] = cnt + (int)__popcll(bal & ((1ull << lane) - 1ull));
        cnt += (int)__popcll(bal);
    }
    // row mask of each key: OR over the entries whose first entry it is
    uint32_t msk[C];
#pragma unroll
    for (int c = 0; c < C; ++c) msk[c] = 0u;
#pragma unroll
    for (int ci = 0; ci < C; ++ci) {
        const int m = min(64, n - ci * 64);
        for (int ii = 0; ii < m; ++ii) {
            const int32_t fi = __builtin_amdgcn_readlane(fst[ci], ii);
            const int32_t ti = __builtin_amdgcn_readlane(row[ci], ii);
#pragma unroll
            for (int c = 0; c < C; ++c) msk[c] |= (fi == c * 64 + lane) ? (1u << ti) : 0u;
        }
    }
#pragma unroll
    for (int c = 0; c < C; ++c) {
        const int k = c * 64 + lane;
        if (k < n && fst[c] == k) {
            gsrc[base + ent[c]] = src[c];
            gmask[base + ent[c]] = (uint8_t)msk[c];
        }
    }
    if (lane == 0) gcnt[g] = cnt;
}

}  // namespace bgnn

using namespace bgnn;

extern "C" int bgnn_group_plan(const int32_t* rowptr, const int32_t* col, int64_t n_rows, int32_t chunk,
                               int32_t group_rows, const int32_t* grow, int64_t n_groups, int32_t* gsrc,
                               uint8_t* gmask, int32_t* gcnt, void* stream) {
    BGNN_REQUIRE(group_rows >= 1 && group_rows <= 8, "group_plan: group_rows must be in [1, 8]");
    BGNN_REQUIRE(chunk >= 1 && chunk <= 64, "group_plan: chunk must be in [1, 64]");
    BGNN_REQUIRE(n_rows >= 0 && n_rows < (int64_t(1) << 31), "group_plan: bad n_rows");
    const int64_t G = grow ? n_groups : (n_rows + group_rows - 1) / group_rows;
    BGNN_REQUIRE(G >= 0 && G < (int64_t(1) << 31), "group_plan: bad n_groups");
    if (n_rows == 0 || G == 0) return BGNN_OK;
    BGNN_REQUIRE(rowptr && col && gsrc && gmask && gcnt, "group_plan: null pointer");
    const unsigned blocks = (unsigned)((G + 3) / 4);
    const int refs = group_rows * chunk;
    hipStream_t s = as_stream(stream);
    if (refs <= 64)
        hipLaunchKernelGGL(k_group_plan<1>, dim3(blocks), dim3(256), 0, s, rowptr, col, n_rows, chunk, group_rows,
                           grow, G, gsrc, gmask, gcnt);
    else if (refs <= 128)
        hipLaunchKernelGGL(k_group_plan<2>, dim3(blocks), dim3(256), 0, s, rowptr, col, n_rows, chunk, group_rows,
                           grow, G, gsrc, gmask, gcnt);
    else if (refs <= 256)
        hipLaunchKernelGGL(k_group_plan<4>, dim3(blocks), dim3(256), 0, s, rowptr, col, n_rows, chunk, group_rows,
                           grow, G, gsrc, gmask, gcnt);
    else
        hipLaunchKernelGGL(k_group_plan<8>, dim3(blocks), dim3(256), 0, s, rowptr, col, n_rows, chunk, group_rows,
                           grow, G, gsrc, gmask, gcnt);
    BGNN_CHECK_LAUNCH();
    return BGNN_OK;
}

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

