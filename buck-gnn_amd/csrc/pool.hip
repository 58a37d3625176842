// SAGPooling: per-graph top-k node selection, the gather-and-scale of the kept rows
// and the edge filter of torch_geometric.nn.SAGPooling, as built by the reference's
// GraphSAGE_SAG / EAGNN_SAG variants (Models/BuckGNN.py:203-208,231-236) and called at
// Models/BuckGNN.py:364,502:
//
//   perm   = topk(score, ratio, batch)      per graph the ceil(ratio * n_g) highest scores,
//                                           graphs in order, scores descending
//   x'     = x[perm] * score[perm]
//   edges' = filter_adj(edge_index, perm)   edges whose two ends are kept, in edge_index
//                                           order, relabelled to positions in perm
//
// Top-k without a sort: the position of node i inside its graph's descending order is its
// rank #{j in graph(i) : s_j > s_i, or s_j == s_i and j < i}. A block of 256 nodes counts
// against its graphs' scores staged through LDS (every lane reads the same LDS word:
// broadcast), so the result is exactly a stable descending sort (ties: lower node index
// first; -0 == +0 as in torch.sort) with no workspace, no atomics, and O(n_g^2) compares
// per graph — 2.5e7 for a 5,041-node mesh, microseconds on the chip.
//
// The edge filter is a deterministic three-pass stream compaction (per-block counts, one
// scan block, ordered write), no atomics; kept edges keep edge_index order.
#include "common.h"

namespace bgnn {

namespace {

constexpr int kRankTile = 2048;

__global__ __launch_bounds__(256) void k_topk_rank(const float* __restrict__ score,
                                                   const int64_t* __restrict__ batch,
                                                   const int64_t* __restrict__ ptr, int64_t N,
                                                   int32_t* __restrict__ rank) {
    __shared__ __attribute__((aligned(16))) float tile[kRankTile];
    const int64_t i0 = (int64_t)blockIdx.x * 256;
    const int64_t i = i0 + threadIdx.x;
    const int64_t il = min(N, i0 + 256) - 1;
    const int64_t lo = ptr[batch[i0]], hi = ptr[batch[il] + 1];   // graphs this block touches
    const bool act = i < N;
    int64_t gs = 0, ge = 0;
    float si = 0.f;
    if (act) {
        const int64_t g = batch[i];
        gs = ptr[g];
        ge = ptr[g + 1];
        si = score[i];
    }
    int32_t r = 0;
    for (int64_t t = lo; t < hi; t += kRankTile) {
        const int n = (int)min((int64_t)kRankTile, hi - t);
        __syncthreads();
        for (int k = threadIdx.x; k < n; k += 256) tile[k] = score[t + k];
        __syncthreads();
        if (!act) continue;
        const int a = (int)max((int64_t)0, gs - t), b = (int)min((int64_t)n, ge - t);
        const int own = (int)(i - t);   // position of i in this tile (may lie outside [a, b))
        // j < i: s_j >= s_i counts; j >= i: s_j > s_i counts (j == i never does)
        const int mid = min(max(own, a), b);
        for (int k = a; k < mid; ++k) r += tile[k] >= si ? 1 : 0;
        for (int k = mid; k < b; ++k) r += tile[k] > si ? 1 : 0;
    }
    if (act) rank[i] = r;
}

__global__ void k_topk_select(const int32_t* __restrict__ rank, const int64_t* __restrict__ batch,
                              const int64_t* __restrict__ k, const int64_t* __restrict__ new_ptr, int64_t N,
                              int64_t* __restrict__ perm, int32_t* __restrict__ new_id,
                              int64_t* __restrict__ batch_out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    const int64_t g = batch[i];
    const int32_t r = rank[i];
    if (r < k[g]) {
        const int64_t p = new_ptr[g] + r;
        perm[p] = i;
        new_id[i] = (int32_t)p;
        if (batch_out) batch_out[p] = g;
    } else {
        new_id[i] = -1;
    }
}

// out[p, :] = x[perm[p], :] * score[perm[p]]; one wave per output row
template <bool V4>
__global__ __launch_bounds__(256) void k_gather_scale(const float* __restrict__ x, int64_t ldx, int32_t H,
                                                      const int64_t* __restrict__ perm,
                                                      const float* __restrict__ score, int64_t K,
                                                      float* __restrict__ out, int64_t ldo) {
    const int64_t p = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (p >= K) return;
    const int lane = threadIdx.x & 63;
    const int64_t i = perm[p];
    const float s = score[i];
    const float* xr = x + i * ldx;
    float* orow = out + p * ldo;
    if constexpr (V4) {
        for (int c = lane * 4; c < H; c += 256) {
            const float4 v = *reinterpret_cast<const float4*>(xr + c);
            *reinterpret_cast<float4*>(orow + c) = make_float4(v.x * s, v.y * s, v.z * s, v.w * s);
        }
    } else {
        for (int c = lane; c < H; c += 64) orow[c] = xr[c] * s;
    }
}

// backward over ALL n input rows (rows that were not kept get zeros: no separate fill):
// dx[i, :] = g[p, :] * score[i], dscore[i] = <g[p, :], x[i, :]> with p = new_id[i]
template <bool V4>
__global__ __launch_bounds__(256) void k_gather_scale_bwd(const float* __restrict__ g, int64_t ldg,
                                                          const float* __restrict__ x, int64_t ldx, int32_t H,
                                                          const int32_t* __restrict__ new_id,
                                                          const float* __restrict__ score, int64_t n,
                                                          float* __restrict__ dx, int64_t lddx,
                                                          float* __restrict__ dscore) {
    const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= n) return;
    const int lane = threadIdx.x & 63;
    const int32_t p = new_id[i];
    float* dr = dx + i * lddx;
    if (p < 0) {
        if constexpr (V4) {
            for (int c = lane * 4; c < H; c += 256) *reinterpret_cast<float4*>(dr + c) = make_float4(0.f, 0.f, 0.f, 0.f);
        } else {
            for (int c = lane; c < H; c += 64) dr[c] = 0.f;
        }
        if (dscore && lane == 0) dscore[i] = 0.f;
        return;
    }
    const float s = score[i];
    const float* gr = g + (int64_t)p * ldg;
    const float* xr = x + i * ldx;
    float acc = 0.f;
    if constexpr (V4) {
        for (int c = lane * 4; c < H; c += 256) {
            const float4 gv = *reinterpret_cast<const float4*>(gr + c);
            const float4 xv = *reinterpret_cast<const float4*>(xr + c);
            *reinterpret_cast<float4*>(dr + c) = make_float4(gv.x * s, gv.y * s, gv.z * s, gv.w * s);
            acc = fmaf(gv.x, xv.x, acc);
            acc = fmaf(gv.y, xv.y, acc);
            acc = fmaf(gv.z, xv.z, acc);
            acc = fmaf(gv.w, xv.w, acc);
        }
    } else {
        for (int c = lane; c < H; c += 64) {
            const float gv = gr[c];
            dr[c] = gv * s;
            acc = fmaf(gv, xr[c], acc);
        }
    }
    acc = group_sum(acc, kWave);
    if (dscore && lane == 0) dscore[i] = acc;
}

// ---- edge filter: 1024 edges per block (4 per thread)
constexpr int kFiltPerThread = 4;
constexpr int kFiltBlock = 256 * kFiltPerThread;

__device__ __forceinline__ bool edge_kept(const int64_t* ei, int64_t E, int64_t e, const int32_t* new_id, int64_t N,
                                          int32_t& s, int32_t& d) {
    const int64_t a = ei[e], b = ei[E + e];
    if (a < 0 || a >= N || b < 0 || b >= N) return false;   // (validated by the caller; never read out of range)
    s = new_id[a];
    d = new_id[b];
    return s >= 0 && d >= 0;
}

// exclusive prefix of v over the 256 threads of the block; returns it and the block total
__device__ __forceinline__ int32_t block_exclusive_scan(int32_t v, int32_t* total) {
    __shared__ int32_t wsum[4];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int32_t inc = v;
    for (int o = 1; o < 64; o <<= 1) {
        const int32_t t = __shfl_up(inc, o, kWave);
        if (lane >= o) inc += t;
    }
    if (lane == 63) wsum[w] = inc;
    __syncthreads();
    int32_t base = 0;
    for (int k = 0; k < w; ++k) base += wsum[k];
    *total = wsum[0] + wsum[1] + wsum[2] + wsum[3];
    __syncthreads();
    return base + inc - v;
}

__global__ __launch_bounds__(256) void k_filter_count(const int64_t* __restrict__ ei, int64_t E,
                                                      const int32_t* __restrict__ new_id, int64_t N,
                                                      int64_t* __restrict__ block_cnt) {
    const int64_t e0 = (int64_t)blockIdx.x * kFiltBlock + (int64_t)threadIdx.x * kFiltPerThread;
    int32_t c = 0;
#pragma unroll
    for (int q = 0; q < kFiltPerThread; ++q) {
        int32_t s, d;
        if (e0 + q < E && edge_kept(ei, E, e0 + q, new_id, N, s, d)) ++c;
    }
    int32_t tot;
    block_exclusive_scan(c, &tot);
    if (threadIdx.x == 0) block_cnt[blockIdx.x] = tot;
}

// exclusive scan of the block counts in place (one block walks them in 256-wide slices);
// n_kept = the total
__global__ __launch_bounds__(256) void k_filter_scan(int64_t* __restrict__ block_cnt, int64_t nb,
                                                     int64_t* __restrict__ n_kept) {
    __shared__ int64_t part[256];
    int64_t carry = 0;
    for (int64_t b0 = 0; b0 < nb; b0 += 256) {
        const int64_t b = b0 + threadIdx.x;
        const int64_t v = b < nb ? block_cnt[b] : 0;
        part[threadIdx.x] = v;
        __syncthreads();
        for (int o = 1; o < 256; o <<= 1) {   // Hillis-Steele inclusive scan in LDS
            const int64_t t = threadIdx.x >= o ? part[threadIdx.x - o] : 0;
            __syncthreads();
            part[threadIdx.x] += t;
            __syncthreads();
        }
        if (b < nb) block_cnt[b] = carry + part[threadIdx.x] - v;
        carry += part[255];
        __syncthreads();
    }
    if (threadIdx.x == 0) *n_kept = carry;
}

// ordered write: out = [src' (n_kept) | dst' (n_kept)], kept[pos] = original edge position
__global__ __launch_bounds__(256) void k_filter_write(const int64_t* __restrict__ ei, int64_t E,
                                                      const int32_t* __restrict__ new_id, int64_t N,
                                                      const int64_t* __restrict__ block_off,
                                                      const int64_t* __restrict__ n_kept,
                                                      int64_t* __restrict__ out, int64_t* __restrict__ kept) {
    const int64_t e0 = (int64_t)blockIdx.x * kFiltBlock + (int64_t)threadIdx.x * kFiltPerThread;
    int32_t s[kFiltPerThread], d[kFiltPerThread];
    bool k[kFiltPerThread];
    int32_t c = 0;
#pragma unroll
    for (int q = 0; q < kFiltPerThread; ++q) {
        k[q] = e0 + q < E && edge_kept(ei, E, e0 + q, new_id, N, s[q], d[q]);
        c += k[q] ? 1 : 0;
    }
    int32_t tot;
    const int32_t ex = block_exclusive_scan(c, &tot);
    const int64_t M = *n_kept;
    int64_t pos = block_off[blockIdx.x] + ex;
#pragma unroll
    for (int q = 0; q < kFiltPerThread; ++q) {
        if (!k[q]) continue;
        out[pos] = s[q];
        out[M + pos] = d[q];
        if (kept) kept[pos] = e0 + q;
        ++pos;
    }
}

inline int64_t filter_blocks(int64_t E) { return (E + kFiltBlock - 1) / kFiltBlock; }

}  // namespace

}  // namespace bgnn

using namespace bgnn;

extern "C" int bgnn_topk_rank(const float* score, const int64_t* batch, const int64_t* ptr, int64_t n,
                              int32_t* rank, void* stream) {
    BGNN_REQUIRE(n >= 0, "topk_rank: n < 0");
    if (n == 0) return BGNN_OK;
    BGNN_REQUIRE(score && batch && ptr && rank, "topk_rank: null pointer");
    hipLaunchKernelGGL(k_topk_rank, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, as_stream(stream), score, batch,
                       ptr, n, rank);
    BGNN_CHECK_LAUNCH();
    return BGNN_OK;
}

extern "C" int bgnn_topk_select(const int32_t* rank, const int64_t* batch, const int64_t* k, const int64_t* new_ptr,
                                int64_t n, int64_t* perm, int32_t* new_id, int64_t* batch_out, void* stream) {
    BGNN_REQUIRE(n >= 0 && n < ((int64_t)1 << 31), "topk_select: n out of range");
    if (n == 0) return BGNN_OK;
    BGNN_REQUIRE(rank && batch && k && new_ptr && perm && new_id, "topk_select: null pointer");
    hipLaunchKernelGGL(k_topk_select, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, as_stream(stream), rank, batch,
                       k, new_ptr, n, perm, new_id, batch_out);
    BGNN_CHECK_LAUNCH();
    return BGNN_OK;
}

extern "C" int bgnn_gather_scale(const float* x, int64_t ldx, int32_t H, const int64_t* perm, const float* score,
                                 int64_t k, float* out, int64_t ldo, void* stream) {
    BGNN_REQUIRE(H >= 0 && ldx >= H && ldo >= H && k >= 0, "gather_scale: bad sizes");
    if (k == 0 || H == 0) return BGNN_OK;
    BGNN_REQUIRE(x && perm && score && out, "gather_scale: null pointer");
    const bool v4 = H % 4 == 0 && ldx % 4 == 0 && ldo % 4 == 0 && aligned16(x) && aligned16(out);
    const dim3 grid((unsigned)((k + 3) / 4));
    if (v4) hipLaunchKernelGGL(k_gather_scale<true>, grid, dim3(256), 0, as_stream(stream), x, ldx, H, perm, score, k, out, ldo);
    else hipLaunchKernelGGL(k_gather_scale<false>, grid, dim3(256), 0, as_stream(stream), x, ldx, H, perm, score, k, out, ldo);
    BGNN_CHECK_LAUNCH();
    return BGNN_OK;
}

extern "C" int bgnn_gather_scale_bwd(const float* g, int64_t ldg, const float* x, int64_t ldx, int32_t H,
                                     const int32_t* new_id, const float* score, int64_t n, float* dx, int64_t lddx,
                                     float* dscore, void* stream) {
    BGNN_REQUIRE(H >= 0 && ldg >= H && ldx >= H && lddx >= H && n >= 0, "gather_scale_bwd: bad sizes");
    if (n == 0) return BGNN_OK;
    BGNN_REQUIRE(g && x && new_id && score && dx, "gather_scale_bwd: null pointer");
    const bool v4 = H % 4 == 0 && ldg % 4 == 0 && ldx % 4 == 0 && lddx % 4 == 0 && aligned16(g) && aligned16(x) &&
                    aligned16(dx);
    const dim3 grid((unsigned)((n + 3) / 4));
    if (v4)
        hipLaunchKernelGGL(k_gather_scale_bwd<true>, grid, dim3(256), 0, as_stream(stream), g, ldg, x, ldx, H, new_id,
                           score, n, dx, lddx, dscore);
    else
        hipLaunchKernelGGL(k_gather_scale_bwd<false>, grid, dim3(256), 0, as_stream(stream), g, ldg, x, ldx, H, new_id,
                           score, n, dx, lddx, dscore);
    BGNN_CHECK_LAUNCH();
    return BGNN_OK;
}

extern "C" size_t bgnn_filter_edges_ws_bytes(int64_t num_edges) {
    return align_up((size_t)(filter_blocks(num_edges > 0 ? num_edges : 0) + 1) * sizeof(int64_t), 256);
}

extern "C" int bgnn_filter_edges(const int64_t* edge_index, int64_t num_edges, const int32_t* new_id,
                                 int64_t num_nodes, int64_t* out_edges, int64_t* kept, int64_t* n_kept, void* ws,
                                 size_t ws_bytes, void* stream) {
    BGNN_REQUIRE(num_edges >= 0 && num_nodes >= 0, "filter_edges: bad sizes");
    BGNN_REQUIRE(n_kept, "filter_edges: null n_kept");
    hipStream_t s = as_stream(stream);
    if (num_edges == 0) {
        BGNN_HIP(hipMemsetAsync(n_kept, 0, sizeof(int64_t), s));
        return BGNN_OK;
    }
    BGNN_REQUIRE(edge_index && new_id && out_edges, "filter_edges: null pointer");
    BGNN_REQUIRE(ws && ws_bytes >= bgnn_filter_edges_ws_bytes(num_edges), "filter_edges: workspace too small");
    const int64_t nb = filter_blocks(num_edges);
    BGNN_REQUIRE(nb < ((int64_t)1 << 31), "filter_edges: too many edges");
    int64_t* cnt = reinterpret_cast<int64_t*>(ws);
    hipLaunchKernelGGL(k_filter_count, dim3((unsigned)nb), dim3(256), 0, s, edge_index, num_edges, new_id, num_nodes,
                       cnt);
    BGNN_CHECK_LAUNCH();
    hipLaunchKernelGGL(k_filter_scan, dim3(1), dim3(256), 0, s, cnt, nb, n_kept);
    BGNN_CHECK_LAUNCH();
    hipLaunchKernelGGL(k_filter_write, dim3((unsigned)nb), dim3(256), 0, s, edge_index, num_edges, new_id, num_nodes,
                       cnt, n_kept, out_edges, kept);
    BGNN_CHECK_LAUNCH();
    return BGNN_OK;
}
