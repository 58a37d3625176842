// f32-accurate GEMM on the gfx950 bf16 MFMA (v_mfma_f32_32x32x16_bf16), for the same
// SAGEConv linears as gemm.hip (Models/BuckGNN.py:135-149; fwd, dgrad, wgrad shapes).
//
// Every f32 operand element is split exactly into three bf16 pieces by round-to-nearest:
//   a0 = bf16(a), a1 = bf16(a - a0), a2 = bf16(a - a0 - a1),  a = a0 + a1 + a2
// (|a1| <= 2^-8 |a|, |a2| <= 2^-16 |a|; each residual is exact in f32). The product is
//   a.b = a0.b0 + (a0.b1 + a1.b0) + (a0.b2 + a1.b1 + a2.b0) + O(2^-23 |a||b|)
// i.e. six bf16 MFMAs per f32 product, every bf16 x bf16 product exact in f32 and all
// accumulation in the f32 MFMA accumulator. The three dropped terms are at most
// 2^-23 |a||b| together, the size of one f32 rounding of the product, so the result sits in
// the same error class as the f32 MFMA kernel (measured against fp64 in
// tests/test_gpu_gemm.py), at 6 x 32 = 192 MFMA cycles per 32x32x16 block instead of
// 8 x 64 = 512 for the f32 MFMA.
//
// Tiling: BM x BN output tile per workgroup, waves WM x WN, each wave (BM/WM) x (BN/WN) in
// 32x32 MFMA tiles; K in BK = 32 slices, double-buffered in LDS. Global operands are read as
// f32 (float4 when K-contiguous, coalesced dwords along M/N when transposed), split in
// registers and stored as three bf16 row images [R][32] per operand (K contiguous, 64-B
// rows, 16-B chunks XOR-swizzled by (row >> 2) & 3 so a 16-lane ds_read_b128 group hits 16
// distinct bank quads). Each MFMA operand is one ds_read_b128 per piece per lane.
#include "common.h"
#include "gemm_common.h"

namespace bgnn {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

constexpr int X6_BK = 32;

// two f32 -> packed bf16x2 (round to nearest even; v_cvt_pk_bf16_f32)
__device__ __forceinline__ uint32_t pack_bf16(float x, float y) {
    const f32x2 v = {x, y};
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2));
}

// exact three-way split of (x, y) into packed bf16 pieces
__device__ __forceinline__ void split2(float x, float y, uint32_t& p0, uint32_t& p1, uint32_t& p2) {
    p0 = pack_bf16(x, y);
    x -= __uint_as_float(p0 << 16);
    y -= __uint_as_float(p0 & 0xffff0000u);
    p1 = pack_bf16(x, y);
    x -= __uint_as_float(p1 << 16);
    y -= __uint_as_float(p1 & 0xffff0000u);
    p2 = pack_bf16(x, y);
}

// 16-B chunk index of (row, chunk) in a [R][32]-bf16 image
__device__ __forceinline__ int x6_pos(int row, int chunk) { return row * 4 + (chunk ^ ((row >> 2) & 3)); }

// One staging unit = 8 consecutive k of one row r (r = m or n) of the tile.
//   KCONTIG = 1: element (r, k) at P[r * ld + k];   unit idx -> r = idx / 4, chunk = idx % 4
//   KCONTIG = 0: element (r, k) at P[k * ld + r];   unit idx -> r = idx % R, chunk = idx / R
template <int KCONTIG, int R, int NT, bool FULL>
__device__ __forceinline__ void x6_load(const float* __restrict__ P, int64_t ld, int64_t Rlim, int64_t r0,
                                        int64_t k0, int64_t kend, bool vec_ok, float (&v)[R * 4 / NT][8], int t) {
    constexpr int NU = R * 4 / NT;
#pragma unroll
    for (int u = 0; u < NU; ++u) {
        const int idx = t + NT * u;
        if constexpr (KCONTIG) {
            const int r = idx >> 2, c = idx & 3;
            const int64_t gr = r0 + r, gk = k0 + c * 8;
            if (FULL || (vec_ok && gr < Rlim && gk + 7 < kend)) {
                const float4 a = *reinterpret_cast<const float4*>(P + gr * ld + gk);
                const float4 b = *reinterpret_cast<const float4*>(P + gr * ld + gk + 4);
                v[u][0] = a.x; v[u][1] = a.y; v[u][2] = a.z; v[u][3] = a.w;
                v[u][4] = b.x; v[u][5] = b.y; v[u][6] = b.z; v[u][7] = b.w;
            } else {
#pragma unroll
                for (int q = 0; q < 8; ++q) v[u][q] = (gr < Rlim && gk + q < kend) ? P[gr * ld + gk + q] : 0.f;
            }
        } else {
            const int r = idx % R, c = idx / R;
            const int64_t gr = r0 + r, gk = k0 + c * 8;
#pragma unroll
            for (int q = 0; q < 8; ++q)
                v[u][q] = (FULL || (gr < Rlim && gk + q < kend)) ? P[(gk + q) * ld + gr] : 0.f;
        }
    }
}

// split the staged units and write the three piece images (S = piece 0; piece p at S + p*R*4)
template <int KCONTIG, int R, int NT, int ABL = 0>
__device__ __forceinline__ void x6_store(uint4* __restrict__ S, const float (&v)[R * 4 / NT][8], int t) {
    constexpr int NU = R * 4 / NT;
#pragma unroll
    for (int u = 0; u < NU; ++u) {
        const int idx = t + NT * u;
        const int r = KCONTIG ? (idx >> 2) : (idx % R);
        const int c = KCONTIG ? (idx & 3) : (idx / R);
        uint4 q0, q1, q2;
        if constexpr (ABL == 1) {
            q0.x = pack_bf16(v[u][0], v[u][1]); q0.y = pack_bf16(v[u][2], v[u][3]);
            q0.z = pack_bf16(v[u][4], v[u][5]); q0.w = pack_bf16(v[u][6], v[u][7]);
            q1 = q0; q2 = q0;
        } else {
            split2(v[u][0], v[u][1], q0.x, q1.x, q2.x);
            split2(v[u][2], v[u][3], q0.y, q1.y, q2.y);
            split2(v[u][4], v[u][5], q0.z, q1.z, q2.z);
            split2(v[u][6], v[u][7], q0.w, q1.w, q2.w);
        }
        const int pos = x6_pos(r, c);
        S[pos] = q0;
        S[R * 4 + pos] = q1;
        S[2 * R * 4 + pos] = q2;
    }
}

__device__ __forceinline__ bf16x8 as_bf16x8(uint4 q) { return __builtin_bit_cast(bf16x8, q); }



// the six leading piece products of one 16-deep k-step, small terms first
template <int TM, int TN>
__device__ __forceinline__ void x6_mma(floatx16 (&acc)[TM][TN], const bf16x8 (&a)[TM][3],
                                       const bf16x8 (&b)[TN][3]) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            floatx16 t = acc[i][j];
            t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][0], b[j][2], t, 0, 0, 0);
            t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][1], b[j][1], t, 0, 0, 0);
            t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][2], b[j][0], t, 0, 0, 0);
            t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][0], b[j][1], t, 0, 0, 0);
            t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][1], b[j][0], t, 0, 0, 0);
            t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][0], b[j][0], t, 0, 0, 0);
            acc[i][j] = t;
        }
}

// write one wave's TM x TN accumulator tiles (wave origin r0, c0; tile column origin n0 for
// the plane base; split-K slab ks): C/D map of the 32x32 MFMA: col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)
template <int TM, int TN, int WTM, int WTN>
__device__ __forceinline__ void x6_epilogue(const GemmArgs& g, const floatx16 (&acc)[TM][TN], int64_t r0,
                                            int64_t c0, int64_t n0, int ks, int lane) {
    float* __restrict__ dst = g.split > 1 ? g.ws + (int64_t)ks * g.M * g.N
                                          : const_cast<float*>(plane_base(g.C, n0, g.c_blk, g.c_pstride));
    const int64_t ldd = g.split > 1 ? g.N : g.ldc;
    const int li = lane & 31, lh = lane >> 5;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int64_t col = c0 + j * 32 + li;
            if (col >= g.N) continue;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int64_t row = r0 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
                if (row >= g.M) continue;
                float v = acc[i][j][r];
                if (g.split > 1) {
                    dst[row * ldd + col] = v;
                } else {
                    v *= g.alpha;
                    if (g.beta != 0.f) v += g.beta * dst[row * ldd + col];
                    if (g.bias) v += g.bias[col];
                    if (g.relu) v = fmaxf(v, 0.f);
                    dst[row * ldd + col] = v;
                }
            }
        }
}

// ABL (timing ablations only, wrong results): 1 = no split arithmetic (piece 0 stored three
// times), 2 = no global loads, 3 = no staging at all (LDS reads + MFMA + barriers),
// 4 = MFMA + barriers only.
template <int TA, int TB, int BM, int BN, int WM, int WN, int ABL = 0>
__global__ __launch_bounds__(64 * WM * WN) void k_gemm_x6(GemmArgs g) {
    constexpr int NT = 64 * WM * WN;
    constexpr int TM = BM / WM / 32, TN = BN / WN / 32;
    constexpr int AK = (TA == 0) ? 1 : 0;   // A K-contiguous?
    constexpr int BKc = (TB == 1) ? 1 : 0;  // B K-contiguous?
    static_assert(BM * 4 % NT == 0 && BN * 4 % NT == 0, "staging units must divide evenly");
    // [buffer][piece][row][4 chunks of 8 bf16]
    __shared__ uint4 As[2][3 * BM * 4];
    __shared__ uint4 Bs[2][3 * BN * 4];

    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int wm = wave / WN, wn = wave % WN;
    const int t = threadIdx.x;
    const int64_t ntn = (g.N + BN - 1) / BN;
    const int64_t ntm = (g.M + BM - 1) / BM;
    const int tiles = (int)(ntm * ntn);
    // XCD-aware order over the whole (tile, split) grid: the workgroups one XCD runs take
    // consecutive tiles of the same K slice, so that slice's operand rows are fetched into
    // that XCD's L2 once and shared (split-K wgrad: 16 tiles x 16 slices)
    const int lt_all = xcd_remap(blockIdx.x + tiles * blockIdx.y, tiles * (int)gridDim.y);
    const int lt = lt_all % tiles, ks = lt_all / tiles;
    const int64_t tm = lt / ntn, tn = lt % ntn;
    const int64_t m0 = tm * BM, n0 = tn * BN;
    const int64_t kb = (int64_t)ks * g.kchunk;
    const int64_t ke = min(g.K, kb + g.kchunk);

    const bool a_vec = (((uintptr_t)g.A & 15) == 0) && (g.lda % 4 == 0);
    const bool b_vec = (((uintptr_t)g.B & 15) == 0) && (g.ldb % 4 == 0);

    floatx16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    float ra[BM * 4 / NT][8], rb[BN * 4 / NT][8];
    const int64_t nk = (ke > kb) ? (ke - kb + X6_BK - 1) / X6_BK : 0;
    const bool full = a_vec && b_vec && (m0 + BM <= g.M) && (n0 + BN <= g.N) && ((ke - kb) % X6_BK == 0);
    auto load_ab = [&](int64_t k0) {
        const float* Ab = plane_base(g.A, TA ? m0 : k0, g.a_blk, g.a_pstride);
        if (full) {
            x6_load<AK, BM, NT, true>(Ab, g.lda, g.M, m0, k0, ke, a_vec, ra, t);
            x6_load<BKc, BN, NT, true>(g.B, g.ldb, g.N, n0, k0, ke, b_vec, rb, t);
        } else {
            x6_load<AK, BM, NT, false>(Ab, g.lda, g.M, m0, k0, ke, a_vec, ra, t);
            x6_load<BKc, BN, NT, false>(g.B, g.ldb, g.N, n0, k0, ke, b_vec, rb, t);
        }
    };
    auto store_ab = [&](int buf) {
        x6_store<AK, BM, NT, ABL>(As[buf], ra, t);
        x6_store<BKc, BN, NT, ABL>(Bs[buf], rb, t);
    };
    // Pipeline: slice t+1 is split and written to the free LDS buffer, slice t+2 is loaded
    // into registers, then slice t is multiplied; one barrier per slice.
    if (nk > 0) {
        load_ab(kb);
        store_ab(0);
        if (nk > 1 && ABL != 2) load_ab(kb + X6_BK);
    }
    __syncthreads();

    const int li = lane & 31, lh = lane >> 5;
    for (int64_t kt = 0; kt < nk; ++kt) {
        const int cur = kt & 1;
        if (kt + 1 < nk && ABL < 3) store_ab(cur ^ 1);
        if (kt + 2 < nk && ABL != 2 && ABL < 3) load_ab(kb + (kt + 2) * X6_BK);
#pragma unroll
        for (int kk = 0; kk < X6_BK / 16; ++kk) {
            bf16x8 a[TM][3], b[TN][3];
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                const int row = wm * (BM / WM) + i * 32;
#pragma unroll
                for (int p = 0; p < 3; ++p) {
                    if constexpr (ABL == 4) {
                        a[i][p] = as_bf16x8(make_uint4(row + p, kk, i, (int)kt));
                    } else {
                        a[i][p] = as_bf16x8(As[cur][p * BM * 4 + x6_pos(row + li, 2 * kk + lh)]);
                    }
                }
            }
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                const int row = wn * (BN / WN) + j * 32;
#pragma unroll
                for (int p = 0; p < 3; ++p) {
                    if constexpr (ABL == 4) {
                        b[j][p] = as_bf16x8(make_uint4(row - p, kk, j, (int)kt));
                    } else {
                        b[j][p] = as_bf16x8(Bs[cur][p * BN * 4 + x6_pos(row + li, 2 * kk + lh)]);
                    }
                }
            }
            x6_mma<TM, TN>(acc, a, b);
        }
        __syncthreads();
    }
    x6_epilogue<TM, TN, BM / WM, BN / WN>(g, acc, m0 + wm * (BM / WM), n0 + wn * (BN / WN), n0, ks, lane);
}

const X6Cfg kX6Cfgs[] = {
    {128, 128, 4, 1},   // 0: 2x2 waves of 64x64 (1 wave / SIMD)
    {256, 128, 8, 1},   // 1: 4x2 waves of 64x64 (2 waves / SIMD)
    {128, 256, 8, 1},   // 2: 2x4 waves of 64x64
};
const int kNumX6Cfgs = 3;

template <int TA, int TB, int ABL>
static void launch_x6_a(int cfg, dim3 grid, hipStream_t s, const GemmArgs& g) {
    switch (cfg) {
        case 0: hipLaunchKernelGGL((k_gemm_x6<TA, TB, 128, 128, 2, 2, ABL>), grid, dim3(256), 0, s, g); break;
        case 1: hipLaunchKernelGGL((k_gemm_x6<TA, TB, 256, 128, 4, 2, ABL>), grid, dim3(512), 0, s, g); break;
        default: hipLaunchKernelGGL((k_gemm_x6<TA, TB, 128, 256, 2, 4, ABL>), grid, dim3(512), 0, s, g); break;
    }
}

template <int TA, int TB>
static void launch_x6_t(int cfg, int abl, dim3 grid, hipStream_t s, const GemmArgs& g) {
    if (abl == 0) { launch_x6_a<TA, TB, 0>(cfg, grid, s, g); return; }
    // ablations are built for the forward shape only (TA = 0, TB = 1)
    if constexpr (TA == 0 && TB == 1) {
        switch (abl) {
            case 1: launch_x6_a<TA, TB, 1>(cfg, grid, s, g); break;
            case 2: launch_x6_a<TA, TB, 2>(cfg, grid, s, g); break;
            case 3: launch_x6_a<TA, TB, 3>(cfg, grid, s, g); break;
            default: launch_x6_a<TA, TB, 4>(cfg, grid, s, g); break;
        }
    } else {
        launch_x6_a<TA, TB, 0>(cfg, grid, s, g);
    }
}

void launch_x6(int ta, int tb, int cfg, int abl, dim3 grid, hipStream_t s, const GemmArgs& g) {
    if (ta == 0 && tb == 0) launch_x6_t<0, 0>(cfg, abl, grid, s, g);
    else if (ta == 0 && tb == 1) launch_x6_t<0, 1>(cfg, abl, grid, s, g);
    else if (ta == 1 && tb == 0) launch_x6_t<1, 0>(cfg, abl, grid, s, g);
    else launch_x6_t<1, 1>(cfg, abl, grid, s, g);
}

}  // namespace bgnn
