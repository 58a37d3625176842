// CSR segment-reduce kernels: SAGEConv neighbour aggregation (sum/mean/max),
// its transpose (backward), global_mean_pool / scatter_mean / scatter_add, and
// the fused SAGE forward epilogue (bias + lin_r term + L2 normalize + BatchNorm
// statistics).
//
// Semantics follow PyG's SAGEConv as used at Models/BuckGNN.py:113-180,434:
// target = edge_index[1], AGG over in-edges, empty segments give 0 (sum, mean,
// max). The data layout is row-major [rows, H] fp32.
//
// Mapping to CDNA4 (MI355X): one 64-lane wavefront owns one destination row
// (H = 512 fp32 = 2 KiB = two 1 KiB coalesced float4 wave-loads per neighbour).
// Neighbour rows are gathered in batches of 8 (16 x 16-B loads in flight per
// lane). A workgroup (4 waves) owns a contiguous range of rows, and the block
// index is remapped so that every XCD works on a contiguous slice of the graph:
// mesh neighbours (i±1, i±n, i±n±1; GraphCreate.py:334-350) are then L2 hits
// and HBM sees each source row about once. Rows whose degree exceeds `chunk`
// (super nodes, VirtualEdgeCreate.py:106-111) are skipped here and reduced by
// `chunk`-edge pieces in k_seg_chunk, then combined in chunk order
// (k_seg_combine) — deterministic, no atomics.
#include <vector>

#include "common.h"
#include "gemm_common.h"

namespace bgnn {

enum : int { OP_SUM = 0, OP_MEAN = 1, OP_MAX = 2, OP_MEANT = 3, OP_MAXT = 4 };
enum : int { EPI_PLAIN = 0, EPI_SAGE = 1 };

struct SegArgs {
    // structure
    const int32_t* rowptr;
    const int32_t* col;
    const int32_t* heavy_row;
    const int32_t* heavy_chunk0;
    const int32_t* chunk_heavy;
    int64_t n_rows;
    int32_t n_heavy, n_chunks, chunk;
    int32_t H;
    int64_t rows_per_block;
    // data
    const float* x;     int64_t ldx;
    float* out;         int64_t ldo;
    // MAX argmax state (bgnn_spmm_max_arg_bytes): arg8 [n_rows, H] uint8 = the argmax edge's offset
    // in its row's edge list for light rows (deg <= chunk <= 64), kArgHeavy for heavy rows, whose
    // offsets are int32 in arg_h [n_heavy, H]; heavy_of[r] = heavy index of heavy row r
    uint8_t* arg8;
    int32_t* heavy_of;
    int32_t* arg_h;
    float* partial;     // [n_chunks, H]
    int32_t* partial_arg;
    // transpose helpers
    const int32_t* fwd_rowptr;  // MEANT, MAXT
    const int32_t* perm_t;      // MAXT
    const uint8_t* arg8_in;     // MAXT: the forward argmax state (arg8 / heavy_of / arg_h above)
    const int32_t* heavy_of_in;
    const int32_t* arg_h_in;
    // SAGE epilogue
    const float* zr;    int64_t ldzr;   // lin_r term rows (z + H)
    const float* bias;
    float* nrm;
    float* bn_partial;  // [slots, 2, H]
    int32_t light_slots;
    int32_t nt;         // stream-once data (z_r rows, output rows) with non-temporal hints
    uint32_t* amax;     // plain epilogue: max |out| folded in (f32 bits, atomic max; NULL = off)
    const float* add;   // plain epilogue: out[r] += add[r] (NULL = off; bgnn_spmm_bwd_add)
    int64_t ld_add;
    // row-group plan (bgnn_group_plan): NULL = none
    const int32_t* gsrc;
    const uint8_t* gmask;
    const int32_t* gcnt;
    const int32_t* grow;    // first row of each group (NULL = g * group_rows)
    int64_t n_groups;
    int32_t group_rows;
    int32_t rev;            // row-group kernel: each eighth's groups swept from its last one down
    // range rows (ranges.hip): hfirst[h] >= 0 marks heavy row h as a range row; with hagg its
    // aggregate is row h of hagg (the forward), with hdone its output row is already written (the
    // transpose); ranges_all: every heavy row is one (host-known)
    const int32_t* hfirst;
    const float* hagg;
    int64_t ld_hagg;
    int32_t hdone;
    int32_t ranges_all;
};

// heavy row h takes the range path in this launch
__device__ __forceinline__ bool range_row(const SegArgs& A, int32_t h) {
    return A.hfirst != nullptr && (A.hagg != nullptr || A.hdone) && A.hfirst[h] >= 0;
}

// fold a lane's running max |out| into *amax: wave max, then one atomic per wave
__device__ __forceinline__ void amax_flush_wave(uint32_t* amax, uint32_t m) {
    if (!amax) return;
    for (int o = 32; o > 0; o >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, o, kWave));
    if ((threadIdx.x & 63) == 0 && m) atomicMax(amax, m);
}


// 1 / max(deg, 1), correctly rounded, identical in every kernel (MEAN backward weights)
__device__ __forceinline__ float inv_deg(int32_t d) { return __frcp_rn((float)(d > 0 ? d : 1)); }

template <int VEC>
struct Vec {
    float f[VEC];
};

template <int VEC>
__device__ __forceinline__ Vec<VEC> ld(const float* p) {
    Vec<VEC> v;
    if constexpr (VEC == 4) {
        const float4 q = *reinterpret_cast<const float4*>(p);
        v.f[0] = q.x; v.f[1] = q.y; v.f[2] = q.z; v.f[3] = q.w;
    } else {
        v.f[0] = *p;
    }
    return v;
}

template <int VEC>
__device__ __forceinline__ void st(float* p, const Vec<VEC>& v) {
    if constexpr (VEC == 4) {
        *reinterpret_cast<float4*>(p) = make_float4(v.f[0], v.f[1], v.f[2], v.f[3]);
    } else {
        *p = v.f[0];
    }
}

template <int VEC>
__device__ __forceinline__ void ldi(const int32_t* p, int32_t (&o)[VEC]) {
    if constexpr (VEC == 4) {
        const int4 q = *reinterpret_cast<const int4*>(p);
        o[0] = q.x; o[1] = q.y; o[2] = q.z; o[3] = q.w;
    } else {
        o[0] = *p;
    }
}

template <int VEC>
__device__ __forceinline__ void sti(int32_t* p, const int32_t (&o)[VEC]) {
    if constexpr (VEC == 4) {
        *reinterpret_cast<int4*>(p) = make_int4(o[0], o[1], o[2], o[3]);
    } else {
        *p = o[0];
    }
}

typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));

__device__ __forceinline__ Vec<4> ld_nt(const float* p) {
    const f32x4_t q = __builtin_nontemporal_load(reinterpret_cast<const f32x4_t*>(p));
    Vec<4> v;
    v.f[0] = q[0]; v.f[1] = q[1]; v.f[2] = q[2]; v.f[3] = q[3];
    return v;
}

__device__ __forceinline__ void st_nt(float* p, const Vec<4>& v) {
    f32x4_t q = {v.f[0], v.f[1], v.f[2], v.f[3]};
    __builtin_nontemporal_store(q, reinterpret_cast<f32x4_t*>(p));
}

// Per-lane accumulator for NV vectors of VEC floats.
template <int VEC, int NV, int OP>
struct Acc {
    float a[NV][VEC];
    int32_t g[(OP == OP_MAX) ? NV : 1][(OP == OP_MAX) ? VEC : 1];

    __device__ __forceinline__ void init() {
#pragma unroll
        for (int v = 0; v < NV; ++v)
#pragma unroll
            for (int k = 0; k < VEC; ++k) {
                a[v][k] = (OP == OP_MAX) ? -INFINITY : 0.f;
                if constexpr (OP == OP_MAX) g[v][k] = -1;
            }
    }
};

constexpr uint8_t kArgHeavy = 255;

// MAXT: the forward argmax bytes of (i, c..c+VEC-1), packed (VEC 4: one dword, VEC 1: one byte).
// Loaded in the same batch as the x rows, so that a gather batch issues all its loads at once.
template <int VEC>
__device__ __forceinline__ uint32_t maxt_bytes(const SegArgs& A, int32_t i, int c) {
    if constexpr (VEC == 4) return *reinterpret_cast<const uint32_t*>(A.arg8_in + (int64_t)i * A.H + c);
    else return A.arg8_in[(int64_t)i * A.H + c];
}

// MAXT: whether the forward edge at offset o of its target row i is the argmax of (i, c..c+VEC-1),
// one flag per column, from the bytes maxt_bytes loaded (heavy rows: the int32 offsets in arg_h)
template <int VEC>
__device__ __forceinline__ void maxt_match(const SegArgs& A, int32_t i, int32_t o, int c, uint32_t w, bool ok,
                                           bool (&m)[VEC]) {
    if ((w & 0xffu) == kArgHeavy) {   // (a heavy row: every column holds the marker; rare)
        int32_t ah[VEC];
        ldi<VEC>(A.arg_h_in + (int64_t)A.heavy_of_in[i] * A.H + c, ah);
#pragma unroll
        for (int k = 0; k < VEC; ++k) m[k] = ok && ah[k] == o;
    } else {
#pragma unroll
        for (int k = 0; k < VEC; ++k) m[k] = ok && (int32_t)((w >> (8 * k)) & 0xffu) == o;
    }
}

// Gather-accumulate the edges [e0, e1) of one row into acc. cols are shared by
// the lanes of the row (wave-uniform when LPR == 64). `cpos[v]` = column offset
// of this lane's v-th vector, `cok[v]` = whether it is inside H.
template <int VEC, int NV, int OP, int U>
__device__ __forceinline__ void gather_batch(const SegArgs& A, Acc<VEC, NV, OP>& acc, int32_t e,
                                             int32_t nvalid, const int (&cpos)[NV],
                                             const bool (&cok)[NV]) {
    int32_t j[U];
    float w[U];
    int32_t off[(OP == OP_MAXT) ? U : 1];   // MAXT: the edge's offset in its forward row
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int32_t eu = e + (u < nvalid ? u : 0);
        j[u] = A.col[eu];
        w[u] = 1.f;
        if constexpr (OP == OP_MEANT) {
            const int32_t d = A.fwd_rowptr[j[u] + 1] - A.fwd_rowptr[j[u]];
            w[u] = inv_deg(d);
        }
        if constexpr (OP == OP_MAXT) off[u] = A.perm_t[eu] - A.fwd_rowptr[j[u]];
    }
    Vec<VEC> val[U][NV];
    uint32_t aw[(OP == OP_MAXT) ? U : 1][(OP == OP_MAXT) ? NV : 1];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
        for (int v = 0; v < NV; ++v) {
            if (cok[v]) val[u][v] = ld<VEC>(A.x + (int64_t)j[u] * A.ldx + cpos[v]);
            else {
#pragma unroll
                for (int k = 0; k < VEC; ++k) val[u][v].f[k] = 0.f;
            }
            if constexpr (OP == OP_MAXT) aw[u][v] = maxt_bytes<VEC>(A, j[u], cok[v] ? cpos[v] : 0);
        }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const bool ok = u < nvalid;
#pragma unroll
        for (int v = 0; v < NV; ++v) {
            if constexpr (OP == OP_MAXT) {
                bool m[VEC];
                maxt_match<VEC>(A, j[u], off[u], cok[v] ? cpos[v] : 0, aw[u][v], ok && cok[v], m);
#pragma unroll
                for (int k = 0; k < VEC; ++k) acc.a[v][k] += m[k] ? val[u][v].f[k] : 0.f;
            } else if constexpr (OP == OP_MAX) {
#pragma unroll
                for (int k = 0; k < VEC; ++k) {
                    const bool better = ok && (val[u][v].f[k] > acc.a[v][k]);
                    acc.a[v][k] = better ? val[u][v].f[k] : acc.a[v][k];
                    acc.g[v][k] = better ? (e + u) : acc.g[v][k];
                }
            } else {
#pragma unroll
                for (int k = 0; k < VEC; ++k) acc.a[v][k] += ok ? __fmul_rn(val[u][v].f[k], w[u]) : 0.f;
            }
        }
    }
}

template <int VEC, int NV, int OP>
__device__ __forceinline__ void gather_range(const SegArgs& A, Acc<VEC, NV, OP>& acc, int32_t beg,
                                             int32_t end, const int (&cpos)[NV],
                                             const bool (&cok)[NV]) {
    int32_t e = beg;
    for (; e + 8 <= end; e += 8) gather_batch<VEC, NV, OP, 8>(A, acc, e, 8, cpos, cok);
    const int32_t rem = end - e;
    if (rem > 4) gather_batch<VEC, NV, OP, 8>(A, acc, e, rem, cpos, cok);
    else if (rem > 0) gather_batch<VEC, NV, OP, 4>(A, acc, e, rem, cpos, cok);
}

// Finish a plain reduction and store it (row r of out).
template <int VEC, int NV, int OP>
__device__ __forceinline__ void store_plain(const SegArgs& A, Acc<VEC, NV, OP>& acc, int64_t r,
                                            int32_t deg, const int (&cpos)[NV],
                                            const bool (&cok)[NV], uint32_t& tmax, int32_t h = -1) {
    int32_t rb = 0;
    if constexpr (OP == OP_MAX) {
        if (A.arg8) rb = A.rowptr[r];
    }
    const float sc = (OP == OP_MEAN) ? inv_deg(deg) : 1.f;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        if (!cok[v]) continue;
        Vec<VEC> o;
#pragma unroll
        for (int k = 0; k < VEC; ++k) {
            float t = acc.a[v][k];
            if constexpr (OP == OP_MAX) t = (deg > 0) ? t : 0.f;
            o.f[k] = t * sc;
        }
        if (A.add) {
            const Vec<VEC> ad = ld<VEC>(A.add + r * A.ld_add + cpos[v]);
#pragma unroll
            for (int k = 0; k < VEC; ++k) o.f[k] += ad.f[k];
        }
#pragma unroll
        for (int k = 0; k < VEC; ++k) tmax = max(tmax, __float_as_uint(o.f[k]) & 0x7fffffffu);
        if constexpr (VEC == 4) {
            if (A.nt) st_nt(A.out + r * A.ldo + cpos[v], o);
            else st<VEC>(A.out + r * A.ldo + cpos[v], o);
        } else {
            st<VEC>(A.out + r * A.ldo + cpos[v], o);
        }
        if constexpr (OP == OP_MAX) {
            if (A.arg8) {   // offsets in the row's edge list (heavy rows: int32 in arg_h)
                uint32_t w = 0;
#pragma unroll
                for (int k = 0; k < VEC; ++k) {
                    const uint32_t o = h >= 0 ? kArgHeavy : (deg > 0 ? (uint32_t)(acc.g[v][k] - rb) : 0u);
                    w |= (o & 0xffu) << (8 * k);
                }
                if constexpr (VEC == 4) *reinterpret_cast<uint32_t*>(A.arg8 + r * A.H + cpos[v]) = w;
                else A.arg8[r * A.H + cpos[v]] = (uint8_t)w;
                if (h >= 0) {
                    int32_t gi[VEC];
#pragma unroll
                    for (int k = 0; k < VEC; ++k) gi[k] = acc.g[v][k] - rb;
                    sti<VEC>(A.arg_h + (int64_t)h * A.H + cpos[v], gi);
                }
            }
        }
    }
}

// Fused SAGE epilogue for one row held by a full wave (LPR == 64, VEC == 4):
// h = acc*scale + z_r[r] + b; o = h / max(||h||, 1e-12); BN partial sums.
// Canonical SAGE row arithmetic, written with explicit roundings so that every kernel
// (light, sweep, combine) produces bit-identical o / nrm regardless of how the
// compiler would contract it: h = (a * sc + zr) + b, ss = fma(h, h, ss).
__device__ __forceinline__ float sage_h(float a, float sc, float zr, float b) {
    return __fadd_rn(__fadd_rn(__fmul_rn(a, sc), zr), b);
}

template <int NV, int OP>
__device__ __forceinline__ void store_sage(const SegArgs& A, Acc<4, NV, OP>& acc, int64_t r,
                                           int32_t deg, const int (&cpos)[NV], const bool (&cok)[NV],
                                           float (&bs)[NV][4], float (&bq)[NV][4]) {
    const float sc = (OP == OP_MEAN) ? inv_deg(deg) : 1.f;
    float h[NV][4];
    float ss = 0.f;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        if (cok[v]) {
            const Vec<4> zr = ld<4>(A.zr + r * A.ldzr + cpos[v]);
            const Vec<4> b = ld<4>(A.bias + cpos[v]);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                h[v][k] = sage_h(acc.a[v][k], sc, zr.f[k], b.f[k]);
                ss = fmaf(h[v][k], h[v][k], ss);
            }
        } else {
#pragma unroll
            for (int k = 0; k < 4; ++k) h[v][k] = 0.f;
        }
    }
    ss = group_sum(ss, kWave);
    const float n = sqrtf(ss);
    const float d = fmaxf(n, 1e-12f);
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        if (!cok[v]) continue;
        Vec<4> o;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            o.f[k] = h[v][k] / d;
            bs[v][k] += o.f[k];
            bq[v][k] += o.f[k] * o.f[k];
        }
        st<4>(A.out + r * A.ldo + cpos[v], o);
    }
    if ((threadIdx.x & 63) == 0) A.nrm[r] = n;
}

template <int VEC, int NV, int LPR>
__device__ __forceinline__ void lane_cols(int cb, int lir, int H, int (&cpos)[NV], bool (&cok)[NV]) {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        cpos[v] = cb + (lir + LPR * v) * VEC;
        cok[v] = cpos[v] < H;
    }
}

// ---------------------------------------------------------------------------
// Light rows: deg <= chunk. Grid: (blocks, column tiles). 256 threads.
template <int VEC, int NV, int LPR, int OP, int EPI>
__global__ __launch_bounds__(256) void k_seg_light(SegArgs A) {
    constexpr int RPW = kWave / LPR;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int sub = lane / LPR, lir = lane % LPR;
    const int lb = xcd_remap(blockIdx.x, gridDim.x);
    const int64_t r_begin = (int64_t)lb * A.rows_per_block;
    const int64_t r_end = min(A.n_rows, r_begin + A.rows_per_block);
    const int cb = blockIdx.y * (LPR * VEC * NV);
    int cpos[NV];
    bool cok[NV];
    lane_cols<VEC, NV, LPR>(cb, lir, A.H, cpos, cok);

    float bs[NV][4], bq[NV][4];
    if constexpr (EPI == EPI_SAGE) {
#pragma unroll
        for (int v = 0; v < NV; ++v)
#pragma unroll
            for (int k = 0; k < 4; ++k) bs[v][k] = bq[v][k] = 0.f;
    }
    uint32_t tmax = 0;

    for (int64_t rb = r_begin + (int64_t)wave * RPW; rb < r_end; rb += 4 * RPW) {
        const int64_t r = (RPW == 1) ? rb : rb + sub;
        if (RPW > 1 && r >= r_end) continue;
        const int32_t beg = A.rowptr[r], end = A.rowptr[r + 1];
        const int32_t deg = end - beg;
        if (deg > A.chunk) continue;  // heavy row: k_seg_chunk + k_seg_combine
        Acc<VEC, NV, OP> acc;
        acc.init();
        gather_range<VEC, NV, OP>(A, acc, beg, end, cpos, cok);
        if constexpr (EPI == EPI_SAGE) {
            store_sage<NV, OP>(A, *reinterpret_cast<Acc<4, NV, OP>*>(&acc), r, deg, cpos, cok, bs, bq);
        } else {
            store_plain<VEC, NV, OP>(A, acc, r, deg, cpos, cok, tmax);
        }
    }
    if constexpr (EPI == EPI_PLAIN) amax_flush_wave(A.amax, tmax);

    if constexpr (EPI == EPI_SAGE) {
        // block-reduce the BatchNorm partial sums over the 4 waves -> slot lb
        __shared__ __attribute__((aligned(16))) float red[4][2][512];
#pragma unroll
        for (int v = 0; v < NV; ++v)
            if (cok[v])
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    red[wave][0][cpos[v] + k] = bs[v][k];
                    red[wave][1][cpos[v] + k] = bq[v][k];
                }
        __syncthreads();
        float* dst = A.bn_partial + (int64_t)lb * 2 * A.H;
        for (int c = threadIdx.x; c < A.H; c += 256) {
            dst[c] = (red[0][0][c] + red[1][0][c]) + (red[2][0][c] + red[3][0][c]);
            dst[A.H + c] = (red[0][1][c] + red[1][1][c]) + (red[2][1][c] + red[3][1][c]);
        }
    }
}

// Heavy chunks: one wave per chunk -> partial[c, :]. 256 threads (4 chunks).
template <int VEC, int NV, int LPR, int OP>
__global__ __launch_bounds__(256) void k_seg_chunk(SegArgs A) {
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int64_t c = (int64_t)blockIdx.x * 4 + wave;
    if (c >= A.n_chunks) return;
    const int cb = blockIdx.y * (LPR * VEC * NV);
    const int lir = lane % LPR;
    if (lane / LPR != 0) return;  // one row per chunk: extra row-groups idle
    int cpos[NV];
    bool cok[NV];
    lane_cols<VEC, NV, LPR>(cb, lir, A.H, cpos, cok);
    const int32_t h = A.chunk_heavy[c];
    if (range_row(A, h)) return;   // (wave-uniform) summed by the row passes instead
    const int32_t r = A.heavy_row[h];
    const int32_t k = (int32_t)(c - A.heavy_chunk0[h]);
    const int32_t beg = A.rowptr[r] + k * A.chunk;
    const int32_t end = min(beg + A.chunk, A.rowptr[r + 1]);
    Acc<VEC, NV, OP> acc;
    acc.init();
    gather_range<VEC, NV, OP>(A, acc, beg, end, cpos, cok);
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        if (!cok[v]) continue;
        Vec<VEC> o;
#pragma unroll
        for (int q = 0; q < VEC; ++q) o.f[q] = acc.a[v][q];
        st<VEC>(A.partial + c * A.H + cpos[v], o);
        if constexpr (OP == OP_MAX) sti<VEC>(A.partial_arg + c * A.H + cpos[v], acc.g[v]);
    }
}

// Combine heavy rows: one block per heavy row (and column tile). For SUM / MEAN the block's 16
// waves (1024 threads) sum 16 contiguous runs of the row's chunks and wave 0 adds the 16 run
// sums in order: a fixed summation tree (deterministic, the same for every light-row kernel
// variant). A cfg3 super node has 79 chunks, so each wave loads 5 partial rows in one batch:
// one memory round trip instead of three (4 waves: 17 us per launch; one wave: 44 us). MAX keeps
// one wave walking the chunks in order (first-occurrence argmax), launched with 256 threads.
constexpr int kCombineWaves = 16;
template <int VEC, int NV, int LPR, int OP, int EPI>
__global__ __launch_bounds__(1024) void k_seg_combine(SegArgs A) {
    constexpr int W = (OP == OP_MAX) ? 1 : kCombineWaves;
    constexpr int TW = LPR * VEC * NV;   // columns of one column tile
    __shared__ __attribute__((aligned(16))) float red[W][TW];
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int h = blockIdx.x;
    if (h >= A.n_heavy) return;   // uniform over the block
    const bool rng = range_row(A, h);
    if (rng && !A.hagg) return;   // the transpose's range row: written by bgnn_range_sums_finish
    const bool act = (lane / LPR == 0) && wave < W;
    const int cb = blockIdx.y * TW;
    const int lir = lane % LPR;
    int cpos[NV];
    bool cok[NV];
    lane_cols<VEC, NV, LPR>(cb, lir, A.H, cpos, cok);
    const int64_t r = A.heavy_row[h];
    const int32_t deg = A.rowptr[r + 1] - A.rowptr[r];
    const int32_t c0 = A.heavy_chunk0[h], c1 = A.heavy_chunk0[h + 1];
    const int32_t per = (c1 - c0 + W - 1) / W;
    const int32_t qa = min(c1, c0 + wave * per), qb = min(c1, qa + per);
    Acc<VEC, NV, OP> acc;
    acc.init();
    if (rng) {   // the forward's range row: its aggregate is given (row h of hagg)
        if (wave != 0 || !act) return;
#pragma unroll
        for (int v = 0; v < NV; ++v) {
            if (!cok[v]) continue;
            const Vec<VEC> p = ld<VEC>(A.hagg + (int64_t)h * A.ld_hagg + cpos[v]);
#pragma unroll
            for (int q = 0; q < VEC; ++q) acc.a[v][q] = p.f[q];
        }
    } else if (act) {
#pragma unroll 8
        for (int32_t c = qa; c < qb; ++c) {
#pragma unroll
            for (int v = 0; v < NV; ++v) {
                if (!cok[v]) continue;
                const Vec<VEC> p = ld<VEC>(A.partial + (int64_t)c * A.H + cpos[v]);
                if constexpr (OP == OP_MAX) {
                    int32_t pa[VEC];
                    ldi<VEC>(A.partial_arg + (int64_t)c * A.H + cpos[v], pa);
#pragma unroll
                    for (int q = 0; q < VEC; ++q) {
                        const bool better = p.f[q] > acc.a[v][q];
                        acc.a[v][q] = better ? p.f[q] : acc.a[v][q];
                        acc.g[v][q] = better ? pa[q] : acc.g[v][q];
                    }
                } else {
#pragma unroll
                    for (int q = 0; q < VEC; ++q) acc.a[v][q] += p.f[q];
                }
            }
        }
    }
    if (W > 1 && !rng) {
        if (act) {
#pragma unroll
            for (int v = 0; v < NV; ++v)
                if (cok[v])
#pragma unroll
                    for (int q = 0; q < VEC; ++q) red[wave][cpos[v] - cb + q] = acc.a[v][q];
        }
        __syncthreads();
        if (wave != 0) return;
        if (act) {
#pragma unroll
            for (int v = 0; v < NV; ++v)
                if (cok[v])
#pragma unroll
                    for (int q = 0; q < VEC; ++q) {
                        const int i = cpos[v] - cb + q;
                        float t = red[0][i];
#pragma unroll
                        for (int w = 1; w < W; ++w) t += red[w][i];
                        acc.a[v][q] = t;
                    }
        }
    }
    if (wave != 0 || !act) return;
    if constexpr (EPI == EPI_SAGE) {
        float bs[NV][4], bq[NV][4];
#pragma unroll
        for (int v = 0; v < NV; ++v)
#pragma unroll
            for (int k = 0; k < 4; ++k) bs[v][k] = bq[v][k] = 0.f;
        store_sage<NV, OP>(A, *reinterpret_cast<Acc<4, NV, OP>*>(&acc), r, deg, cpos, cok, bs, bq);
        float* dst = A.bn_partial + (int64_t)(A.light_slots + h) * 2 * A.H;
#pragma unroll
        for (int v = 0; v < NV; ++v)
            if (cok[v]) {
                Vec<4> s1, s2;
#pragma unroll
                for (int k = 0; k < 4; ++k) { s1.f[k] = bs[v][k]; s2.f[k] = bq[v][k]; }
                st<4>(dst + cpos[v], s1);
                st<4>(dst + A.H + cpos[v], s2);
            }
    } else {
        uint32_t tmax = 0;
        store_plain<VEC, NV, OP>(A, acc, r, deg, cpos, cok, tmax, OP == OP_MAX ? h : -1);
        if constexpr (OP == OP_MAX) {
            if (A.arg8 && blockIdx.y == 0 && lane == 0) A.heavy_of[r] = h;
        }
        if (A.amax && tmax) atomicMax(A.amax, tmax);   // one heavy row per wave: few atomics
    }
}

// ---------------------------------------------------------------------------
// XCD sweep kernel (one full row per wave, LPR = 64, VEC = 4): the production
// light-row kernel for H >= 256.
//
// Row assignment: the grid (a multiple of 8 blocks) is split into the 8 groups
// of blocks that share an XCD under round-robin dispatch (b % 8). Group x owns
// the contiguous row region [x*N/8, (x+1)*N/8) and its 4*G/8 waves sweep that
// region together: wave q takes rows lo + q, lo + q + W, lo + q + 2W, ... So at
// any moment an XCD works on a ~W-row front and its mesh neighbourhood
// (±n rows), which stays in that XCD's 4 MiB L2, instead of G/8 scattered row
// ranges whose union far exceeds it. (Placement affects speed only.)
//
// Latency: rowptr of all rows of a wave is fetched with one vector load (lane l
// holds row t0+l); a row's col indices are one vector load (lane k = k-th
// neighbour, deg <= chunk <= 64) issued one row ahead; up to U neighbours are
// gathered in a single batch, so a light row costs about one memory round trip.
struct Sweep {
    int64_t lo, hi, first;
    int W, T;
};

__device__ __forceinline__ Sweep sweep_rows(int64_t n_rows, int wave) {
    Sweep s;
    const int G = gridDim.x;                 // multiple of 8
    const int x = blockIdx.x & 7, i = blockIdx.x >> 3;
    const int64_t lo = n_rows * x / kNumXcd, hi = n_rows * (x + 1) / kNumXcd;
    s.W = 4 * (G >> 3);
    s.lo = lo;
    s.hi = hi;
    s.first = lo + i * 4 + wave;
    s.T = s.first < hi ? (int)((hi - s.first + s.W - 1) / s.W) : 0;
    return s;
}

template <int NV, int OP, int U>
__device__ __forceinline__ void sweep_gather(const SegArgs& A, Acc<4, NV, OP>& acc, int32_t cur, int32_t beg,
                                             int32_t deg, int32_t e0, const int (&cpos)[NV], const bool (&cok)[NV]) {
    const int nvalid = min(U, deg - e0);
    int32_t j[U];
    float w[U];
    int32_t off[(OP == OP_MAXT) ? U : 1];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int slot = (u < nvalid) ? e0 + u : e0;   // masked slots re-read the first row (L1 hit)
        j[u] = __builtin_amdgcn_readlane(cur, slot);
        w[u] = 1.f;
        if constexpr (OP == OP_MEANT) {
            const int32_t d = A.fwd_rowptr[j[u] + 1] - A.fwd_rowptr[j[u]];
            w[u] = inv_deg(d);
        }
        if constexpr (OP == OP_MAXT) off[u] = A.perm_t[beg + slot] - A.fwd_rowptr[j[u]];
    }
    Vec<4> val[U][NV];
    uint32_t aw[(OP == OP_MAXT) ? U : 1][(OP == OP_MAXT) ? NV : 1];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
        for (int v = 0; v < NV; ++v) {
            val[u][v] = ld<4>(A.x + (int64_t)j[u] * A.ldx + (cok[v] ? cpos[v] : 0));
            if constexpr (OP == OP_MAXT) aw[u][v] = maxt_bytes<4>(A, j[u], cok[v] ? cpos[v] : 0);
        }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const bool ok = u < nvalid;
#pragma unroll
        for (int v = 0; v < NV; ++v) {
            if constexpr (OP == OP_MAXT) {
                bool m[4];
                maxt_match<4>(A, j[u], off[u], cok[v] ? cpos[v] : 0, aw[u][v], ok && cok[v], m);
#pragma unroll
                for (int k = 0; k < 4; ++k) acc.a[v][k] += m[k] ? val[u][v].f[k] : 0.f;
            } else if constexpr (OP == OP_MAX) {
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const bool better = ok && (val[u][v].f[k] > acc.a[v][k]);
                    acc.a[v][k] = better ? val[u][v].f[k] : acc.a[v][k];
                    acc.g[v][k] = better ? (beg + e0 + u) : acc.g[v][k];
                }
            } else {
#pragma unroll
                for (int k = 0; k < 4; ++k) acc.a[v][k] += ok ? __fmul_rn(val[u][v].f[k], w[u]) : 0.f;
            }
        }
    }
}

template <int NV, int OP, int EPI, int U>
__global__ __launch_bounds__(256) void k_seg_sweep(SegArgs A) {
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const Sweep sw = sweep_rows(A.n_rows, wave);
    const int cb = blockIdx.y * (64 * 4 * NV);
    int cpos[NV];
    bool cok[NV];
    lane_cols<4, NV, 64>(cb, lane, A.H, cpos, cok);
    // SAGE epilogue state lives in LDS, not VGPRs (it would cost 24 registers per lane and
    // the occupancy that a 12-neighbour gather batch needs): per-wave BatchNorm partial sums
    // red[wave][0/1][col] (each lane owns its columns: no barriers) and the bias row.
    __shared__ __attribute__((aligned(16))) float red[(EPI == EPI_SAGE) ? 4 : 1][2][(EPI == EPI_SAGE) ? 512 : 4];
    __shared__ __attribute__((aligned(16))) float sbias[(EPI == EPI_SAGE) ? 512 : 4];
    if constexpr (EPI == EPI_SAGE) {
#pragma unroll
        for (int v = 0; v < NV; ++v)
            if (cok[v]) {
                *reinterpret_cast<float4*>(&red[wave][0][cpos[v]]) = make_float4(0.f, 0.f, 0.f, 0.f);
                *reinterpret_cast<float4*>(&red[wave][1][cpos[v]]) = make_float4(0.f, 0.f, 0.f, 0.f);
            }
        for (int c = threadIdx.x; c < A.H; c += 256) sbias[c] = A.bias[c];
        __syncthreads();
    }
    const int32_t chunk = A.chunk;
    uint32_t tmax = 0;

    for (int t0 = 0; t0 < sw.T; t0 += 64) {
        const int nrow = min(64, sw.T - t0);
        int32_t rp_lo = 0, rp_hi = 0;
        if (lane < nrow) {
            const int64_t rl = sw.first + (int64_t)sw.W * (t0 + lane);
            rp_lo = A.rowptr[rl];
            rp_hi = A.rowptr[rl + 1];
        }
        int32_t nb = __builtin_amdgcn_readlane(rp_lo, 0), ndeg = __builtin_amdgcn_readlane(rp_hi, 0) - nb;
        int32_t cv = (lane < ndeg && ndeg <= chunk) ? A.col[nb + lane] : 0;
        for (int k = 0; k < nrow; ++k) {
            const int64_t r = sw.first + (int64_t)sw.W * (t0 + k);
            const int32_t beg = nb, deg = ndeg;
            const int32_t cur = cv;
            if (k + 1 < nrow) {   // prefetch the next row's neighbour list
                nb = __builtin_amdgcn_readlane(rp_lo, k + 1);
                ndeg = __builtin_amdgcn_readlane(rp_hi, k + 1) - nb;
                cv = (lane < ndeg && ndeg <= chunk) ? A.col[nb + lane] : 0;
            }
            if (deg > chunk) continue;   // heavy row: k_seg_chunk + k_seg_combine
            Acc<4, NV, OP> acc;
            acc.init();
            // issue the row's stream-once z_r load first, so it completes under the gathers
            // (one memory round trip per light row)
            Vec<4> zr[NV];
            if constexpr (EPI == EPI_SAGE) {
#pragma unroll
                for (int v = 0; v < NV; ++v) zr[v] = ld_nt(A.zr + r * A.ldzr + (cok[v] ? cpos[v] : 0));
            }
            for (int e0 = 0; e0 < deg; e0 += U) sweep_gather<NV, OP, U>(A, acc, cur, beg, deg, e0, cpos, cok);
            if constexpr (EPI == EPI_SAGE) {
                const float sc = (OP == OP_MEAN) ? inv_deg(deg) : 1.f;
                float h[NV][4];
                float ss = 0.f;
#pragma unroll
                for (int v = 0; v < NV; ++v) {
                    const float4 bv = cok[v] ? *reinterpret_cast<const float4*>(&sbias[cpos[v]])
                                             : make_float4(0.f, 0.f, 0.f, 0.f);
                    const float bb[4] = {bv.x, bv.y, bv.z, bv.w};
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        h[v][q] = cok[v] ? sage_h(acc.a[v][q], sc, zr[v].f[q], bb[q]) : 0.f;
                        ss = fmaf(h[v][q], h[v][q], ss);
                    }
                }
                ss = group_sum(ss, kWave);
                const float n = sqrtf(ss);
                const float d = fmaxf(n, 1e-12f);
#pragma unroll
                for (int v = 0; v < NV; ++v) {
                    if (!cok[v]) continue;
                    Vec<4> o;
#pragma unroll
                    for (int q = 0; q < 4; ++q) o.f[q] = h[v][q] / d;
                    st_nt(A.out + r * A.ldo + cpos[v], o);
                    float4* ps = reinterpret_cast<float4*>(&red[wave][0][cpos[v]]);
                    float4* pq = reinterpret_cast<float4*>(&red[wave][1][cpos[v]]);
                    float4 a = *ps, b = *pq;
                    a.x += o.f[0]; a.y += o.f[1]; a.z += o.f[2]; a.w += o.f[3];
                    b.x += o.f[0] * o.f[0]; b.y += o.f[1] * o.f[1]; b.z += o.f[2] * o.f[2]; b.w += o.f[3] * o.f[3];
                    *ps = a;
                    *pq = b;
                }
                if (lane == 0) A.nrm[r] = n;
            } else {
                store_plain<4, NV, OP>(A, acc, r, deg, cpos, cok, tmax);
            }
        }
    }
    if constexpr (EPI == EPI_PLAIN) amax_flush_wave(A.amax, tmax);

    if constexpr (EPI == EPI_SAGE) {
        __syncthreads();
        float* dst = A.bn_partial + (int64_t)blockIdx.x * 2 * A.H;
        for (int c = threadIdx.x; c < A.H; c += 256) {
            dst[c] = (red[0][0][c] + red[1][0][c]) + (red[2][0][c] + red[3][0][c]);
            dst[A.H + c] = (red[0][1][c] + red[1][1][c]) + (red[2][1][c] + red[3][1][c]);
        }
    }
}

// ---------------------------------------------------------------------------
// Row-group kernel (SUM / MEAN / MEANT, one full row per lane set, VEC = 4, LPR = 64): the
// production light-row kernel when the CSR carries a row-group plan (bgnn_group_plan).
//
// A wave reduces R consecutive rows at once. The plan lists every distinct source row of the
// group once, with an R-bit mask of the rows that use it: on a mesh, rows i..i+R-1 share most
// of their neighbours (i±1, the i±n bands), so a group of 8 fetches ~37 source rows instead of
// ~71 (cfg2). Each fetched row is added to the accumulators of the rows in its mask (a select
// per row and column: VALU, hidden under the loads). Groups are swept per XCD like rows in
// k_seg_sweep. Per row, the entries are summed in plan order (deterministic; for the group's
// first row it is CSR order), so results match the sweep kernel to rounding, not bitwise.
// (Measured in round 2 and dropped: issuing the group's z_r loads before its gathers, 160 -> 188
// us, and 16 source rows per gather batch, 160 -> 168 us; profiles/r02_tune_agg_knobs.txt.)
template <int NV, int OP, int EPI, int R, int U>
__global__ __launch_bounds__(256) void k_seg_group(SegArgs A) {
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const Sweep sw = sweep_rows(A.n_groups, wave);
    int cpos[NV];
    bool cok[NV];
    lane_cols<4, NV, 64>(0, lane, A.H, cpos, cok);
    __shared__ __attribute__((aligned(16))) float red[(EPI == EPI_SAGE) ? 4 : 1][2][(EPI == EPI_SAGE) ? 512 : 4];
    __shared__ __attribute__((aligned(16))) float sbias[(EPI == EPI_SAGE) ? 512 : 4];
    if constexpr (EPI == EPI_SAGE) {
#pragma unroll
        for (int v = 0; v < NV; ++v)
            if (cok[v]) {
                *reinterpret_cast<float4*>(&red[wave][0][cpos[v]]) = make_float4(0.f, 0.f, 0.f, 0.f);
                *reinterpret_cast<float4*>(&red[wave][1][cpos[v]]) = make_float4(0.f, 0.f, 0.f, 0.f);
            }
        for (int c = threadIdx.x; c < A.H; c += 256) sbias[c] = A.bias[c];
        __syncthreads();
    }
    const int32_t chunk = A.chunk;
    uint32_t tmax = 0;

    for (int t0 = 0; t0 < sw.T; t0 += 64) {
        const int ng = min(64, sw.T - t0);
        // heads of the next 64 groups of this wave: first row, row count, first CSR position
        // and key count
        int32_t hr = 0, hn = 0, hb = 0, hc = 0;
        if (lane < ng) {
            int64_t gl = sw.first + (int64_t)sw.W * (t0 + lane);
            if (A.rev) gl = sw.lo + sw.hi - 1 - gl;   // mirrored inside the eighth [lo, hi)
            if (A.grow) {
                hr = A.grow[gl];
                hn = A.grow[gl + 1] - hr;
            } else {
                hr = (int32_t)(gl * R);
                hn = (int32_t)min((int64_t)R, A.n_rows - hr);
            }
            hb = A.rowptr[hr];
            hc = A.gcnt[gl];
        }
        // prefetch of a group: its rows' rowptr (lane t <= R) and its first 64 keys
        int32_t rp_n, sl_n;
        uint32_t ml_n;
        {
            const int64_t r0 = __builtin_amdgcn_readlane(hr, 0);
            rp_n = lane <= R ? A.rowptr[min(r0 + lane, A.n_rows)] : 0;
            const int32_t b = __builtin_amdgcn_readlane(hb, 0), c = __builtin_amdgcn_readlane(hc, 0);
            sl_n = lane < c ? A.gsrc[b + lane] : 0;
            ml_n = lane < c ? (uint32_t)A.gmask[b + lane] : 0u;
        }
        for (int k = 0; k < ng; ++k) {
            const int64_t r0 = __builtin_amdgcn_readlane(hr, k);
            const int rows = __builtin_amdgcn_readlane(hn, k);
            const int32_t base = __builtin_amdgcn_readlane(hb, k), cnt = __builtin_amdgcn_readlane(hc, k);
            const int32_t rp = rp_n, sl0 = sl_n;
            const uint32_t ml0 = ml_n;
            if (k + 1 < ng) {
                const int64_t r1 = __builtin_amdgcn_readlane(hr, k + 1);
                rp_n = lane <= R ? A.rowptr[min(r1 + lane, A.n_rows)] : 0;
                const int32_t b = __builtin_amdgcn_readlane(hb, k + 1), c = __builtin_amdgcn_readlane(hc, k + 1);
                sl_n = lane < c ? A.gsrc[b + lane] : 0;
                ml_n = lane < c ? (uint32_t)A.gmask[b + lane] : 0u;
            }
            float a[R][NV][4];
#pragma unroll
            for (int t = 0; t < R; ++t)
#pragma unroll
                for (int v = 0; v < NV; ++v)
#pragma unroll
                    for (int q = 0; q < 4; ++q) a[t][v][q] = 0.f;
            for (int32_t eb = 0; eb < cnt; eb += 64) {
                const int n = min(64, cnt - eb);
                int32_t sl = sl0;
                uint32_t ml = ml0;
                if (eb > 0) {
                    sl = lane < n ? A.gsrc[base + eb + lane] : 0;
                    ml = lane < n ? (uint32_t)A.gmask[base + eb + lane] : 0u;
                }
                for (int u0 = 0; u0 < n; u0 += U) {
                    int32_t j[U];
                    uint32_t m[U];
                    float w[U];
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        const bool ok = u0 + u < n;
                        const int kk = ok ? u0 + u : u0;   // masked slots re-read the first row (L1 hit)
                        j[u] = __builtin_amdgcn_readlane(sl, kk);
                        m[u] = ok ? (uint32_t)__builtin_amdgcn_readlane((int)ml, kk) : 0u;
                        w[u] = 1.f;
                        if constexpr (OP == OP_MEANT) {
                            const int32_t d = A.fwd_rowptr[j[u] + 1] - A.fwd_rowptr[j[u]];
                            w[u] = inv_deg(d);
                        }
                    }
                    Vec<4> val[U][NV];
#pragma unroll
                    for (int u = 0; u < U; ++u)
#pragma unroll
                        for (int v = 0; v < NV; ++v)
                            val[u][v] = ld<4>(A.x + (int64_t)j[u] * A.ldx + (cok[v] ? cpos[v] : 0));
#pragma unroll
                    for (int u = 0; u < U; ++u)
#pragma unroll
                        for (int t = 0; t < R; ++t) {
                            // the mask bit is wave-uniform (j[u], m[u] come from readlane): add only
                            // where the key is used, by a scalar branch (measured: spmm_bwd 138.5 ->
                            // 135.9 us against a per-lane select, profiles/r04_ab_agg_knobs.txt)
                            if (__builtin_amdgcn_readfirstlane((int)((m[u] >> t) & 1u))) {
#pragma unroll
                                for (int v = 0; v < NV; ++v)
#pragma unroll
                                    for (int q = 0; q < 4; ++q)
                                        a[t][v][q] += (OP == OP_MEANT) ? __fmul_rn(val[u][v].f[q], w[u])
                                                                       : val[u][v].f[q];
                            }
                        }
                }
            }
            if constexpr (EPI == EPI_SAGE) {
                Vec<4> zr[R][NV];
#pragma unroll
                for (int t = 0; t < R; ++t) {
                    const int64_t r = r0 + (t < rows ? t : 0);
#pragma unroll
                    for (int v = 0; v < NV; ++v) zr[t][v] = ld_nt(A.zr + r * A.ldzr + (cok[v] ? cpos[v] : 0));
                }
#pragma unroll
                for (int t = 0; t < R; ++t) {
                    const int64_t r = r0 + t;
                    const int32_t rb = __builtin_amdgcn_readlane(rp, t);
                    const int32_t deg = __builtin_amdgcn_readlane(rp, t + 1) - rb;
                    if (t >= rows || deg > chunk) continue;   // heavy row: chunk + combine
                    const float sc = (OP == OP_MEAN) ? inv_deg(deg) : 1.f;
                    float h[NV][4];
                    float ss = 0.f;
#pragma unroll
                    for (int v = 0; v < NV; ++v) {
                        const float4 bv = cok[v] ? *reinterpret_cast<const float4*>(&sbias[cpos[v]])
                                                 : make_float4(0.f, 0.f, 0.f, 0.f);
                        const float bb[4] = {bv.x, bv.y, bv.z, bv.w};
#pragma unroll
                        for (int q = 0; q < 4; ++q) {
                            h[v][q] = cok[v] ? sage_h(a[t][v][q], sc, zr[t][v].f[q], bb[q]) : 0.f;
                            ss = fmaf(h[v][q], h[v][q], ss);
                        }
                    }
                    ss = group_sum(ss, kWave);
                    const float nr = sqrtf(ss);
                    const float d = fmaxf(nr, 1e-12f);
#pragma unroll
                    for (int v = 0; v < NV; ++v) {
                        if (!cok[v]) continue;
                        Vec<4> o;
#pragma unroll
                        for (int q = 0; q < 4; ++q) o.f[q] = h[v][q] / d;
                        st_nt(A.out + r * A.ldo + cpos[v], o);
                        float4* ps = reinterpret_cast<float4*>(&red[wave][0][cpos[v]]);
                        float4* pq = reinterpret_cast<float4*>(&red[wave][1][cpos[v]]);
                        float4 s1 = *ps, s2 = *pq;
                        s1.x += o.f[0]; s1.y += o.f[1]; s1.z += o.f[2]; s1.w += o.f[3];
                        s2.x += o.f[0] * o.f[0]; s2.y += o.f[1] * o.f[1];
                        s2.z += o.f[2] * o.f[2]; s2.w += o.f[3] * o.f[3];
                        *ps = s1;
                        *pq = s2;
                    }
                    if (lane == 0) A.nrm[r] = nr;
                }
            } else {
#pragma unroll
                for (int t = 0; t < R; ++t) {
                    const int64_t r = r0 + t;
                    const int32_t rb = __builtin_amdgcn_readlane(rp, t);
                    const int32_t deg = __builtin_amdgcn_readlane(rp, t + 1) - rb;
                    if (t >= rows || deg > chunk) continue;
                    Acc<4, NV, OP> acc;
#pragma unroll
                    for (int v = 0; v < NV; ++v)
#pragma unroll
                        for (int q = 0; q < 4; ++q) acc.a[v][q] = a[t][v][q];
                    store_plain<4, NV, OP>(A, acc, r, deg, cpos, cok, tmax);
                }
            }
        }
    }
    if constexpr (EPI == EPI_PLAIN) amax_flush_wave(A.amax, tmax);

    if constexpr (EPI == EPI_SAGE) {
        __syncthreads();
        float* dst = A.bn_partial + (int64_t)blockIdx.x * 2 * A.H;
        for (int c = threadIdx.x; c < A.H; c += 256) {
            dst[c] = (red[0][0][c] + red[1][0][c]) + (red[2][0][c] + red[3][0][c]);
            dst[A.H + c] = (red[0][1][c] + red[1][1][c]) + (red[2][1][c] + red[3][1][c]);
        }
    }
}

// ---------------------------------------------------------------------------
constexpr int kMaxLightBlocks = 1024;

// Tuning knobs (process-wide; defaults are the production choice; see bgnn_set_tuning).
// (ABI 12 removed BGNN_TUNE_MAX_GROUP, the max forward on the row-group kernel: bit-identical, but
// cfg2 156 -> 168 us, the per-(key, row) argmax resolution and tie test outweighing the
// deduplicated loads; round 5, profiles/r05_bench_max_group_j.json)
static int g_seg_kernel = 0;     // 0 = auto (row-group kernel where planned, else sweep), 1 = blocked,
                                 // 2 = sweep
static int g_grp_blocks = 1024;  // row-group kernel grid (4 blocks of 4 waves per CU)
static int g_seg_blocks = 1024;  // sweep grid (rounded to a multiple of 8)
static int g_seg_nt = 1;         // non-temporal hints on stream-once data (default on: +8 % fwd)
static int g_seg_u = 0;          // neighbours per gather batch in the sweep kernel (0 = auto = 12:
                                 // mesh rows have 8 neighbours + ~1 virtual edge, one batch)

struct Geometry {
    int vec, nv, lpr, ctiles;
};

inline int pow2ceil(int x) {
    int p = 1;
    while (p < x) p <<= 1;
    return p;
}

inline Geometry pick_geometry(int H, bool aligned16) {
    Geometry g;
    if (aligned16 && H % 4 == 0) {
        g.vec = 4;
        const int nv4 = H / 4;
        if (nv4 >= 128) { g.lpr = 64; g.nv = 2; }
        else if (nv4 > 64) { g.lpr = 64; g.nv = 2; }
        else { g.lpr = pow2ceil(nv4 < 16 ? 16 : nv4); g.nv = 1; }
        g.ctiles = (H + g.lpr * 4 * g.nv - 1) / (g.lpr * 4 * g.nv);
    } else {
        g.vec = 1;
        g.nv = 1;
        g.lpr = pow2ceil(H < 16 ? 16 : (H > 64 ? 64 : H));
        g.ctiles = (H + g.lpr - 1) / g.lpr;
    }
    return g;
}

inline int64_t light_grid(int64_t n_rows, int rows_per_wave, int max_blocks, int64_t* rpb) {
    const int64_t per_block = 4 * rows_per_wave;
    int64_t blocks = (n_rows + per_block - 1) / per_block;
    if (blocks > max_blocks) blocks = max_blocks;
    if (blocks < 1) blocks = 1;
    *rpb = (n_rows + blocks - 1) / blocks;
    return blocks;
}

inline int64_t sweep_grid(int64_t n_rows) {
    int64_t want = (n_rows + 3) / 4;                 // at most one row per wave
    int64_t blocks = g_seg_blocks;
    if (want < blocks) blocks = want;
    blocks = (blocks + 7) / 8 * 8;
    return blocks < 8 ? 8 : blocks;
}

inline int64_t group_grid(int64_t G) {
    int64_t want = (G + 3) / 4;                      // at most one group per wave
    int64_t blocks = g_grp_blocks;
    if (want < blocks) blocks = want;
    blocks = (blocks + 7) / 8 * 8;
    return blocks < 8 ? 8 : blocks;
}

// Optional timing of the heavy-row (super node) launches: while enabled, every launch_all with
// chunks records a HIP event pair around its k_seg_chunk + k_seg_combine launches (bench.py's
// cfg3 block reports the super rows' share of the aggregation; bgnn_heavy_timing).
struct HeavyEv { hipEvent_t a, b; int fwd; };
static std::vector<HeavyEv> g_heavy_ev;
static size_t g_heavy_used = 0;
static bool g_heavy_on = false;
static int g_heavy_dir = 0;   // set by the entry points: 0 = forward aggregation, 1 = transpose

inline HeavyEv* heavy_ev_next(int fwd) {
    if (!g_heavy_on) return nullptr;
    if (g_heavy_used == g_heavy_ev.size()) {
        HeavyEv e{};
        // (timing only: no system-scope fence at record, which would idle the GPU ~5 us per event)
        if (hipEventCreateWithFlags(&e.a, hipEventDisableSystemFence) != hipSuccess ||
            hipEventCreateWithFlags(&e.b, hipEventDisableSystemFence) != hipSuccess)
            return nullptr;
        g_heavy_ev.push_back(e);
    }
    HeavyEv* e = &g_heavy_ev[g_heavy_used++];
    e->fwd = fwd;
    return e;
}

// Whether launch_all runs the row-group kernel for this CSR / reduce.
inline bool use_group(const SegArgs& A, int op, int vec, int lpr) {
    return g_seg_kernel == 0 && A.gcnt != nullptr && vec == 4 && lpr == 64 && A.chunk <= 64 &&
           (op == OP_SUM || op == OP_MEAN || op == OP_MEANT);
}

inline int64_t light_blocks_sage(const SegArgs& A) {
    return use_group(A, OP_SUM, 4, 64) ? group_grid(A.n_groups) : sweep_grid(A.n_rows);
}

template <int VEC, int NV, int LPR, int OP, int EPI>
int launch_all(SegArgs A, int ctiles, int max_blocks, hipStream_t s, int64_t* blocks_out) {
    int64_t rpb = 0;
    const bool group = use_group(A, OP, VEC, LPR) && ctiles == 1;   // one wave holds a whole row
    // the sweep kernel needs one row per wave and every light row's list in one vector load
    const bool sweep = (VEC == 4 && LPR == 64 && g_seg_kernel != 1 && A.chunk <= 64);
    int64_t blocks;
    if (group) {
        blocks = group_grid(A.n_groups);
    } else if (sweep || EPI == EPI_SAGE) {   // SAGE: slot count = bgnn_sage_fwd_slots() for either kernel
        blocks = sweep_grid(A.n_rows);
        rpb = (A.n_rows + blocks - 1) / blocks;
    } else {
        blocks = light_grid(A.n_rows, kWave / LPR, max_blocks, &rpb);
    }
    A.rows_per_block = rpb;
    A.nt = g_seg_nt;
    // BGNN_TUNE_ROWS_REV bit 2 (SAGE epilogue) / bit 3 (plain): sweep each eighth downward, so it
    // starts on the rows the producing GEMM (which walks its tiles upward, one eighth per XCD)
    // wrote last
    A.rev = (rows_rev() >> (EPI == EPI_SAGE ? 2 : 3)) & 1;
    if (blocks_out) *blocks_out = blocks;
    A.light_slots = (int32_t)blocks;
    if (A.n_rows > 0) {
        if constexpr (VEC == 4 && LPR == 64 && (OP == OP_SUM || OP == OP_MEAN || OP == OP_MEANT)) {
            if (group) {
                const dim3 gr((unsigned)blocks);
                if (A.group_rows == 8)
                    hipLaunchKernelGGL((k_seg_group<NV, OP, EPI, 8, 4>), gr, dim3(256), 0, s, A);
                else
                    hipLaunchKernelGGL((k_seg_group<NV, OP, EPI, 4, 8>), gr, dim3(256), 0, s, A);
                BGNN_CHECK_LAUNCH();
            }
        }
        if (group) {
        } else if constexpr (VEC == 4 && LPR == 64) {
            if (sweep) {
                const int u = g_seg_u ? g_seg_u : 12;
                if (u == 8)
                    hipLaunchKernelGGL((k_seg_sweep<NV, OP, EPI, 8>), dim3((unsigned)blocks, ctiles), dim3(256), 0,
                                       s, A);
                else if (u == 16)
                    hipLaunchKernelGGL((k_seg_sweep<NV, OP, EPI, 16>), dim3((unsigned)blocks, ctiles), dim3(256), 0,
                                       s, A);
                else
                    hipLaunchKernelGGL((k_seg_sweep<NV, OP, EPI, 12>), dim3((unsigned)blocks, ctiles), dim3(256), 0,
                                       s, A);
            } else {
                hipLaunchKernelGGL((k_seg_light<VEC, NV, LPR, OP, EPI>), dim3((unsigned)blocks, ctiles), dim3(256),
                                   0, s, A);
            }
        } else {
            hipLaunchKernelGGL((k_seg_light<VEC, NV, LPR, OP, EPI>), dim3((unsigned)blocks, ctiles), dim3(256), 0,
                               s, A);
        }
        BGNN_CHECK_LAUNCH();
    }
    if (A.n_chunks > 0) {
        HeavyEv* ev = heavy_ev_next(g_heavy_dir == 0);
        if (ev) (void)hipEventRecord(ev->a, s);
        // every heavy row a range row (host-known): no chunks to reduce; the transpose's range
        // rows are written already (no combine either), the forward's combine applies the epilogue
        const bool all_range = A.ranges_all && A.hfirst && (A.hagg || A.hdone);
        constexpr int COP = (OP == OP_MAX) ? OP_MAX : (OP == OP_MAXT ? OP_MAXT : (OP == OP_MEANT ? OP_MEANT : OP_SUM));
        if (!all_range) {
            hipLaunchKernelGGL((k_seg_chunk<VEC, NV, LPR, COP>), dim3((A.n_chunks + 3) / 4, ctiles), dim3(256), 0, s,
                               A);
            BGNN_CHECK_LAUNCH();
        }
        constexpr int MOP = (OP == OP_MAX) ? OP_MAX : (OP == OP_MEAN ? OP_MEAN : OP_SUM);
        if (!(all_range && A.hdone)) {
            hipLaunchKernelGGL((k_seg_combine<VEC, NV, LPR, MOP, EPI>), dim3(A.n_heavy, ctiles),
                               dim3(MOP == OP_MAX ? 256 : 64 * kCombineWaves), 0, s, A);
            BGNN_CHECK_LAUNCH();
        }
        if (ev) (void)hipEventRecord(ev->b, s);
    }
    return BGNN_OK;
}

template <int OP>
int dispatch_plain(SegArgs A, const Geometry& g, hipStream_t s) {
#define BGNN_PLAIN(V, N, L)                                                              \
    if (g.vec == V && g.nv == N && g.lpr == L)                                           \
        return launch_all<V, N, L, OP, EPI_PLAIN>(A, g.ctiles, 2048, s, nullptr);
    BGNN_PLAIN(4, 2, 64)
    BGNN_PLAIN(4, 1, 64)
    BGNN_PLAIN(4, 1, 32)
    BGNN_PLAIN(4, 1, 16)
    BGNN_PLAIN(1, 1, 64)
    BGNN_PLAIN(1, 1, 32)
    BGNN_PLAIN(1, 1, 16)
#undef BGNN_PLAIN
    return fail(BGNN_E_UNSUPPORTED, "spmm: no kernel for vec=%d nv=%d lpr=%d", g.vec, g.nv, g.lpr);
}


// byte layout of the MAX argmax state buffer (bgnn_spmm_max_arg_bytes)
struct MaxArgLayout {
    int64_t heavy_of, arg_h;
};
inline MaxArgLayout max_arg_layout(int64_t rows, int64_t H) {
    MaxArgLayout L;
    L.heavy_of = (int64_t)align_up((size_t)(rows * H), 256);
    L.arg_h = L.heavy_of + (int64_t)align_up((size_t)(rows * 4), 256);
    return L;
}

inline SegArgs args_from_csr(const bgnn_csr_t* c) {
    SegArgs A{};
    A.rowptr = c->rowptr;
    A.col = c->col;
    A.heavy_row = c->heavy_row;
    A.heavy_chunk0 = c->heavy_chunk0;
    A.chunk_heavy = c->chunk_heavy;
    A.n_rows = c->n_rows;
    A.n_heavy = c->n_heavy;
    A.n_chunks = c->n_chunks;
    A.chunk = c->chunk > 0 ? c->chunk : 0x7fffffff;
    if (c->gsrc && c->gmask && c->gcnt && (c->group_rows == 4 || c->group_rows == 8)) {
        A.gsrc = c->gsrc;
        A.gmask = c->gmask;
        A.gcnt = c->gcnt;
        A.group_rows = c->group_rows;
        A.grow = c->grow;
        A.n_groups = c->grow ? c->n_groups : (c->n_rows + c->group_rows - 1) / c->group_rows;
    }
    if (c->ranges && c->n_heavy > 0) {
        A.hfirst = c->ranges + 2 + 3 * c->n_heavy;
        A.ranges_all = c->ranges_all;
    }
    return A;
}

extern int g_x6_bdma;   // gemm_x6.hip
extern int g_h3p_nsb;   // gemm_h3p.hip
#ifdef BGNN_H3P_ABLATION
extern int g_h3p_abl;
#endif

}  // namespace bgnn

using namespace bgnn;

extern "C" int bgnn_spmm_fwd(const bgnn_csr_t* csr, const float* x, int64_t ldx, int32_t H, int32_t reduce,
                             float* out, int64_t ldo, void* arg, float* partial, void* stream) {
    // (no max |out| here: nothing downstream scales by it)
    BGNN_REQUIRE(csr && csr->rowptr, "spmm_fwd: null csr");
    BGNN_REQUIRE(H > 0 && ldx >= H && ldo >= H, "spmm_fwd: bad H/ld");
    BGNN_REQUIRE(reduce >= 0 && reduce <= 2, "spmm_fwd: bad reduce %d", reduce);
    BGNN_REQUIRE(csr->n_chunks == 0 || partial, "spmm_fwd: partial scratch required for heavy rows");
    SegArgs A = args_from_csr(csr);
    g_heavy_dir = 0;
    A.H = H;
    A.x = x; A.ldx = ldx;
    A.out = out; A.ldo = ldo;
    if (arg) {
        // the compact state stores a light row's argmax as a byte offset into its edge list
        // (deg <= chunk) and marks heavy rows with 255: a chunk of 255 or more would let a light
        // row's offset wrap or collide with the marker (bgnn_spmm_bwd_max would then read a
        // heavy-row slot that was never written)
        BGNN_REQUIRE(csr->chunk > 0 && csr->chunk < 255,
                     "spmm_fwd(max, arg): the CSR's chunk must be in [1, 254] for the compact argmax (got %d)",
                     csr->chunk);
        const MaxArgLayout L = max_arg_layout(csr->n_rows, H);
        A.arg8 = static_cast<uint8_t*>(arg);
        A.heavy_of = reinterpret_cast<int32_t*>(static_cast<char*>(arg) + L.heavy_of);
        A.arg_h = reinterpret_cast<int32_t*>(static_cast<char*>(arg) + L.arg_h);
    }
    A.partial = partial;
    A.partial_arg = partial ? reinterpret_cast<int32_t*>(partial + (int64_t)csr->n_chunks * H) : nullptr;
    const bool al = aligned16(x) && aligned16(out) && ldx % 4 == 0 && ldo % 4 == 0 &&
                    (!partial || aligned16(partial)) && (!arg || aligned16(arg));
    const Geometry g = pick_geometry(H, al);
    hipStream_t s = as_stream(stream);
    switch (reduce) {
        case BGNN_REDUCE_SUM: return dispatch_plain<OP_SUM>(A, g, s);
        case BGNN_REDUCE_MEAN: return dispatch_plain<OP_MEAN>(A, g, s);
        default: return dispatch_plain<OP_MAX>(A, g, s);
    }
}

static int spmm_bwd_impl(const bgnn_csr_t* csr_t, const int32_t* perm_t, const int32_t* fwd_rowptr,
                         int64_t fwd_rows, const float* g, int64_t ldg, int32_t H, int32_t reduce, const void* arg,
                         const float* addend, int64_t ld_add, float* gx, int64_t ldgx, float* partial, float* amax,
                         int heavy_done, void* stream);

extern "C" int bgnn_spmm_bwd(const bgnn_csr_t* csr_t, const int32_t* perm_t, const int32_t* fwd_rowptr,
                             const float* g, int64_t ldg, int32_t H, int32_t reduce, float* gx, int64_t ldgx,
                             float* partial, float* amax, int32_t heavy_done, void* stream) {
    BGNN_REQUIRE(reduce != BGNN_REDUCE_MAX, "spmm_bwd: max aggregation takes bgnn_spmm_bwd_max");
    BGNN_REQUIRE(!heavy_done || (csr_t && csr_t->ranges), "spmm_bwd: heavy_done needs the CSR's ranges");
    return spmm_bwd_impl(csr_t, perm_t, fwd_rowptr, 0, g, ldg, H, reduce, nullptr, nullptr, 0, gx, ldgx, partial,
                         amax, heavy_done ? 1 : 0, stream);
}

extern "C" int bgnn_spmm_bwd_add(const bgnn_csr_t* csr_t, const int32_t* perm_t, const int32_t* fwd_rowptr,
                                 const float* g, int64_t ldg, int32_t H, int32_t reduce, const float* addend,
                                 int64_t ld_add, float* gx, int64_t ldgx, float* partial, float* amax, void* stream) {
    BGNN_REQUIRE(reduce != BGNN_REDUCE_MAX, "spmm_bwd_add: max aggregation takes bgnn_spmm_bwd_max");
    return spmm_bwd_impl(csr_t, perm_t, fwd_rowptr, 0, g, ldg, H, reduce, nullptr, addend, ld_add, gx, ldgx, partial,
                         amax, 0, stream);
}

extern "C" int bgnn_spmm_bwd_max(const bgnn_csr_t* csr_t, const int32_t* perm_t, const int32_t* fwd_rowptr,
                                 int64_t fwd_rows, const float* g, int64_t ldg, int32_t H, const void* arg,
                                 const float* addend, int64_t ld_add, float* gx, int64_t ldgx, float* partial,
                                 float* amax, void* stream) {
    BGNN_REQUIRE(perm_t && fwd_rowptr && arg && fwd_rows >= 0, "spmm_bwd_max: perm_t, fwd_rowptr and arg required");
    return spmm_bwd_impl(csr_t, perm_t, fwd_rowptr, fwd_rows, g, ldg, H, BGNN_REDUCE_MAX, arg, addend, ld_add, gx, ldgx,
                         partial, amax, 0, stream);
}

static int spmm_bwd_impl(const bgnn_csr_t* csr_t, const int32_t* perm_t, const int32_t* fwd_rowptr,
                         int64_t fwd_rows, const float* g, int64_t ldg, int32_t H, int32_t reduce, const void* arg,
                         const float* addend, int64_t ld_add, float* gx, int64_t ldgx, float* partial, float* amax,
                         int heavy_done, void* stream) {
    BGNN_REQUIRE(csr_t && csr_t->rowptr, "spmm_bwd: null csr");
    BGNN_REQUIRE(!addend || ld_add >= H, "spmm_bwd: bad ld_add");
    BGNN_REQUIRE(H > 0 && ldg >= H && ldgx >= H, "spmm_bwd: bad H/ld");
    BGNN_REQUIRE(csr_t->n_chunks == 0 || partial, "spmm_bwd: partial scratch required");
    SegArgs A = args_from_csr(csr_t);
    g_heavy_dir = 1;
    A.H = H;
    A.x = g; A.ldx = ldg;
    A.out = gx; A.ldo = ldgx;
    A.partial = partial;
    A.fwd_rowptr = fwd_rowptr;
    A.perm_t = perm_t;
    if (arg) {
        const MaxArgLayout L = max_arg_layout(fwd_rows, H);
        A.arg8_in = static_cast<const uint8_t*>(arg);
        A.heavy_of_in = reinterpret_cast<const int32_t*>(static_cast<const char*>(arg) + L.heavy_of);
        A.arg_h_in = reinterpret_cast<const int32_t*>(static_cast<const char*>(arg) + L.arg_h);
    }
    A.amax = reinterpret_cast<uint32_t*>(amax);
    A.add = addend;
    A.ld_add = ld_add;
    A.hdone = heavy_done;
    const bool al = aligned16(g) && aligned16(gx) && ldg % 4 == 0 && ldgx % 4 == 0 &&
                    (!partial || aligned16(partial)) && (!arg || aligned16(arg)) &&
                    (!addend || (aligned16(addend) && ld_add % 4 == 0));
    const Geometry geo = pick_geometry(H, al);
    hipStream_t s = as_stream(stream);
    switch (reduce) {
        case BGNN_REDUCE_SUM: return dispatch_plain<OP_SUM>(A, geo, s);
        case BGNN_REDUCE_MEAN:
            BGNN_REQUIRE(fwd_rowptr, "spmm_bwd(mean): fwd_rowptr required");
            return dispatch_plain<OP_MEANT>(A, geo, s);
        default:
            BGNN_REQUIRE(perm_t && arg && fwd_rowptr, "spmm_bwd(max): perm_t, fwd_rowptr and arg required");
            return dispatch_plain<OP_MAXT>(A, geo, s);
    }
}

extern "C" int32_t bgnn_sage_fwd_slots(const bgnn_csr_t* csr) {
    if (!csr) return -1;
    const SegArgs A = args_from_csr(csr);
    return (int32_t)(light_blocks_sage(A) + (csr->n_chunks > 0 ? csr->n_heavy : 0));
}

extern "C" int32_t bgnn_get_tuning(int32_t knob) {
    switch (knob) {
        case BGNN_TUNE_SEG_KERNEL: return g_seg_kernel;
        case BGNN_TUNE_SEG_BLOCKS: return g_seg_blocks;
        case BGNN_TUNE_SEG_U: return g_seg_u;
        case BGNN_TUNE_SEG_NT: return g_seg_nt;
        case BGNN_TUNE_GEMM_MODE: return gemm_mode();
        case BGNN_TUNE_ROWS_NT: return rows_nt();
        case BGNN_TUNE_GROUP_BLOCKS: return g_grp_blocks;
        case BGNN_TUNE_ROWS_REV: return rows_rev();
        case BGNN_TUNE_GEMM_BDMA: return g_x6_bdma == 2 && g_h3p_nsb == 4 ? 3 : g_x6_bdma;
        default: return -1;
    }
}

extern "C" int bgnn_set_tuning(int32_t knob, int32_t value) {
    switch (knob) {
        case BGNN_TUNE_SEG_KERNEL:
            BGNN_REQUIRE(value >= 0 && value <= 2, "set_tuning: kernel must be 0 (auto), 1 (blocked) or 2 (sweep)");
            g_seg_kernel = value;
            return BGNN_OK;
        case BGNN_TUNE_SEG_BLOCKS:
            BGNN_REQUIRE(value >= 8 && value <= 65536, "set_tuning: blocks out of range");
            g_seg_blocks = value;
            return BGNN_OK;
        case BGNN_TUNE_SEG_U:
            BGNN_REQUIRE(value == 0 || value == 8 || value == 12 || value == 16,
                         "set_tuning: U must be 0 (auto), 8, 12 or 16");
            g_seg_u = value;
            return BGNN_OK;
        case BGNN_TUNE_SEG_NT: g_seg_nt = value ? 1 : 0; return BGNN_OK;
        case BGNN_TUNE_GROUP_BLOCKS:
            BGNN_REQUIRE(value >= 8 && value <= 65536, "set_tuning: group blocks out of range");
            g_grp_blocks = value;
            return BGNN_OK;
        case BGNN_TUNE_ROWS_NT: set_rows_nt(value); return BGNN_OK;
        case BGNN_TUNE_ROWS_REV: set_rows_rev(value); return BGNN_OK;
        case BGNN_TUNE_GEMM_BDMA:
#ifdef BGNN_H3P_ABLATION
            if (value >= 16) {   // measurement build: the pipelined kernel (4 slots) with ablation value / 16
                g_x6_bdma = 2;
                g_h3p_nsb = 4;
                g_h3p_abl = value / 16;
                return BGNN_OK;
            }
            g_h3p_abl = 0;
#endif
#ifdef BGNN_H3P_ABLATION
            BGNN_REQUIRE(value >= 0 && value <= 4, "set_tuning: gemm B staging must be 0 .. 4");
#else
            BGNN_REQUIRE(value == 0 || value == 2 || value == 3,
                         "set_tuning: gemm B staging must be 0 (k_gemm_x6, register copy) or 2 / 3 (the pipelined "
                         "kernel, 3 / 4 slots); 1 and 4 are measurement-build forms (make abl)");
#endif
            g_x6_bdma = value == 3 ? 2 : value;
            g_h3p_nsb = value == 3 ? 4 : 3;
            return BGNN_OK;
        case BGNN_TUNE_GEMM_MODE:
            BGNN_REQUIRE(value == 0 || value == 2, "set_tuning: gemm mode must be 0 (f32 MFMA) or 2 (f16x3)");
            set_gemm_mode(value);
            return BGNN_OK;
        default: return fail(BGNN_E_ARG, "set_tuning: unknown knob %d", knob);
    }
}

extern "C" int bgnn_sage_fwd(const bgnn_csr_t* csr, const float* zl, int64_t ldzl, const float* zr, int64_t ldzr,
                             const float* bias, int32_t H, int32_t reduce, float* o, float* nrm, float* bn_partial,
                             float* partial, const float* heavy_agg, int64_t ld_heavy_agg, void* stream) {
    BGNN_REQUIRE(csr && csr->rowptr, "sage_fwd: null csr");
    BGNN_REQUIRE(H > 0 && H <= 512 && H % 4 == 0, "sage_fwd: H=%d unsupported (need H%%4==0, H<=512)", H);
    BGNN_REQUIRE(ldzl >= H && ldzl % 4 == 0 && ldzr >= H && ldzr % 4 == 0,
                 "sage_fwd: ldzl/ldzr must be >= H and multiples of 4");
    BGNN_REQUIRE(reduce == BGNN_REDUCE_SUM || reduce == BGNN_REDUCE_MEAN, "sage_fwd: reduce must be sum/mean");
    BGNN_REQUIRE(aligned16(zl) && aligned16(zr) && aligned16(o) && aligned16(bias) && aligned16(bn_partial) &&
                     (!partial || aligned16(partial)),
                 "sage_fwd: pointers must be 16-byte aligned");
    BGNN_REQUIRE(csr->n_chunks == 0 || partial, "sage_fwd: partial scratch required for heavy rows");
    SegArgs A = args_from_csr(csr);
    g_heavy_dir = 0;
    A.H = H;
    A.x = zl; A.ldx = ldzl;
    A.zr = zr; A.ldzr = ldzr;
    A.bias = bias;
    A.out = o; A.ldo = H;
    A.nrm = nrm;
    A.bn_partial = bn_partial;
    A.partial = partial;
    if (heavy_agg) {
        BGNN_REQUIRE(csr->ranges && aligned16(heavy_agg) && ld_heavy_agg >= H && ld_heavy_agg % 4 == 0,
                     "sage_fwd: heavy_agg needs the CSR's ranges, 16-B alignment and ld >= H");
        A.hagg = heavy_agg;
        A.ld_hagg = ld_heavy_agg;
    }
    hipStream_t s = as_stream(stream);
    int64_t blocks = 0;
    if (H > 256) {
        return reduce == BGNN_REDUCE_SUM
                   ? launch_all<4, 2, 64, OP_SUM, EPI_SAGE>(A, 1, kMaxLightBlocks, s, &blocks)
                   : launch_all<4, 2, 64, OP_MEAN, EPI_SAGE>(A, 1, kMaxLightBlocks, s, &blocks);
    }
    return reduce == BGNN_REDUCE_SUM ? launch_all<4, 1, 64, OP_SUM, EPI_SAGE>(A, 1, kMaxLightBlocks, s, &blocks)
                                     : launch_all<4, 1, 64, OP_MEAN, EPI_SAGE>(A, 1, kMaxLightBlocks, s, &blocks);
}

extern "C" int bgnn_heavy_timing(int32_t enable) {
    g_heavy_on = enable != 0;
    if (g_heavy_on) g_heavy_used = 0;
    return BGNN_OK;
}

extern "C" int bgnn_heavy_timing_read(int32_t which, float* total_ms, int32_t* count) {
    BGNN_REQUIRE(total_ms && count && (which == 0 || which == 1), "heavy_timing_read: bad args");
    double t = 0.0;
    int32_t n = 0;
    for (size_t i = 0; i < g_heavy_used; ++i) {
        const HeavyEv& e = g_heavy_ev[i];
        if (e.fwd != (which == 0 ? 1 : 0)) continue;
        BGNN_HIP(hipEventSynchronize(e.b));
        float ms = 0.f;
        BGNN_HIP(hipEventElapsedTime(&ms, e.a, e.b));
        t += ms;
        ++n;
    }
    *total_ms = (float)t;
    *count = n;
    return BGNN_OK;
}

extern "C" size_t bgnn_spmm_max_arg_bytes(int64_t rows, int32_t H, int32_t n_heavy) {
    if (rows < 0 || H <= 0 || n_heavy < 0) return 0;
    return (size_t)max_arg_layout(rows, H).arg_h + (size_t)n_heavy * (size_t)H * 4;
}
