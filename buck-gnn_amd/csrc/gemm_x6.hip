// GEMMs on the gfx950 16-bit MFMAs, for the same SAGEConv linears as gemm.hip
// (Models/BuckGNN.py:135-149; fwd, dgrad, wgrad shapes) and the EA_GNN edge / node MLPs.
// PREC 2 = bf16 operands (one round-to-nearest piece, one product, f32 accumulation; the
// bf16 EA_GNN path of BASELINE configs[4]). Two f32-accurate split precisions:
//
// PREC 1 = f16x3 (default). Each operand is scaled by a power of two s = 2^k chosen from its
// max |value| (max |a| * s in [2^14, 2^15), so nothing overflows the f16 range) and split
// into two round-to-nearest f16 pieces, a*s = a0 + a1 + e with |a1| <= 2^-11 |a*s| and
// |e| <= 2^-22 |a*s|. The product is a.b = (a0.b0 + a0.b1 + a1.b0) / (s_a s_b) + O(2^-21 |a||b|)
// (a1.b1 <= 2^-22, e terms <= 2^-22 each): three f16 MFMAs per f32 product, every
// f16 x f16 product (11 x 11 bits) exact in the f32 accumulator, and the unscale an exact
// power-of-two multiply. The representation error stays an order of magnitude below the
// f32 accumulation error of a K = 512 sum (measured against fp64 in tests/test_gpu_gemm.py).
// Elements below 2^-39 max|A| (f16 subnormal range after scaling) lose relative precision;
// their absolute error stays below 2^-39 max|A| |b|.
//
// Tiling: BM x BN output tile per workgroup, waves WM x WN, each wave (BM/WM) x (BN/WN) in
// 32x32 MFMA tiles; K in BK = 32 slices, double-buffered in LDS. Global operands are read as
// f32 (float4 when K-contiguous, coalesced dwords along M/N when transposed), split in
// registers and stored as 16-bit row images [R][32] per piece (K contiguous, 64-B rows, 16-B
// chunks XOR-swizzled by (row >> 2) & 3 so a 16-lane ds_read_b128 group hits 16 distinct
// bank quads). Each MFMA operand is one ds_read_b128 per piece per lane. (A bf16x6 family --
// three exact bf16 pieces, six products -- was measured and dropped in round 2: f16x3 halves
// its MFMAs at a lower error.)
#include <type_traits>

#include "common.h"
#include "gemm_common.h"
#include "gemm_x6.h"

namespace bgnn {

constexpr int X6_BK = 32;

// 16-B chunk index of (row, chunk) in a [R][32]-bf16 image
__device__ __forceinline__ int x6_pos(int row, int chunk) { return row * 4 + (chunk ^ ((row >> 2) & 3)); }

// One staging unit = 8 consecutive k of one row r (r = m or n) of the tile.
//   KCONTIG = 1: element (r, k) at P[r * ld + k];   unit idx -> r = idx / 4, chunk = idx % 4
//   KCONTIG = 0: element (r, k) at P[k * ld + r];   unit idx -> r = idx % R, chunk = idx / R
// bf16 element e of operand storage P16 (exact in f32)
__device__ __forceinline__ float bf16_at(const uint16_t* __restrict__ P16, int64_t e) {
    return __uint_as_float((uint32_t)P16[e] << 16);
}

// BF: the operand is stored as bf16 (ld in bf16 elements; the EA_GNN edge activations of the
// bf16 configuration): loaded at half the bytes and widened exactly to f32 in registers.
template <int KCONTIG, int R, int NT, bool FULL, bool BF = false>
__device__ __forceinline__ void x6_load(const float* __restrict__ P, int64_t ld, int64_t Rlim, int64_t r0,
                                        int64_t k0, int64_t kend, bool vec_ok, float (&v)[R * 4 / NT][8], int t) {
    constexpr int NU = R * 4 / NT;
    const uint16_t* __restrict__ P16 = reinterpret_cast<const uint16_t*>(P);
#pragma unroll
    for (int u = 0; u < NU; ++u) {
        const int idx = t + NT * u;
        if constexpr (BF) {
            if constexpr (KCONTIG) {
                const int r = idx >> 2, c = idx & 3;
                const int64_t gr = r0 + r, gk = k0 + c * 8;
                if (FULL || (vec_ok && gr < Rlim && gk + 7 < kend)) {
                    const uint4 q = *reinterpret_cast<const uint4*>(P16 + gr * ld + gk);
                    const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
                    for (int h = 0; h < 4; ++h) {
                        v[u][2 * h] = __uint_as_float(w[h] << 16);
                        v[u][2 * h + 1] = __uint_as_float(w[h] & 0xffff0000u);
                    }
                } else {
#pragma unroll
                    for (int q = 0; q < 8; ++q) v[u][q] = (gr < Rlim && gk + q < kend) ? bf16_at(P16, gr * ld + gk + q) : 0.f;
                }
            } else {
                const int r = idx % R, c = idx / R;
                const int64_t gr = r0 + r, gk = k0 + c * 8;
#pragma unroll
                for (int q = 0; q < 8; ++q)
                    v[u][q] = (FULL || (gr < Rlim && gk + q < kend)) ? bf16_at(P16, (gk + q) * ld + gr) : 0.f;
            }
            continue;
        }
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

// split the staged units and write the piece images (S = piece 0; piece p at S + p*R*4);
// PREC 1 scales by sc first (exact: a power of two)
template <int KCONTIG, int R, int NT, int PREC, int ABL = 0>
__device__ __forceinline__ void x6_store(uint4* __restrict__ S, const float (&v)[R * 4 / NT][8], int t, float sc) {
    constexpr int NU = R * 4 / NT;
#pragma unroll
    for (int u = 0; u < NU; ++u) {
        const int idx = t + NT * u;
        const int r = KCONTIG ? (idx >> 2) : (idx % R);
        const int c = KCONTIG ? (idx & 3) : (idx / R);
        const int pos = x6_pos(r, c);
        if constexpr (PREC == 2) {   // bf16: one round-to-nearest piece
            uint4 q0;
            q0.x = pack_bf16(v[u][0], v[u][1]); q0.y = pack_bf16(v[u][2], v[u][3]);
            q0.z = pack_bf16(v[u][4], v[u][5]); q0.w = pack_bf16(v[u][6], v[u][7]);
            S[pos] = q0;
            continue;
        }
        {
            uint4 q0, q1;
            if constexpr (ABL == 1) {
                q0.x = pack_f16(v[u][0], v[u][1]); q0.y = pack_f16(v[u][2], v[u][3]);
                q0.z = pack_f16(v[u][4], v[u][5]); q0.w = pack_f16(v[u][6], v[u][7]);
                q1 = q0;
            } else {
                split2h(v[u][0] * sc, v[u][1] * sc, q0.x, q1.x);
                split2h(v[u][2] * sc, v[u][3] * sc, q0.y, q1.y);
                split2h(v[u][4] * sc, v[u][5] * sc, q0.z, q1.z);
                split2h(v[u][6] * sc, v[u][7] * sc, q0.w, q1.w);
            }
            S[pos] = q0;
            S[R * 4 + pos] = q1;
        }
    }
}

// k-major quad staging (f16x3, both operands k-major: the weight gradient dW = dZ^T X, whose
// K is the node dimension). A quad is 4 consecutive rows r x 8 consecutive k of one operand:
// eight coalesced float4 loads along r (one per k), transposed in registers into four
// 8-k units, written as the same [row][32 k] swizzled images as the K-contiguous path (so
// the MFMA reads are unchanged). Quads of A go to threads [0, BM), of B to [BM, BM + BN).
// Measured (wgrad 1024x512x80656, 256x256 tiles): 804 -> 300 us against per-lane dword loads.
// KTAIL: rows in range and 16-B aligned, only k may run past kend (the last split-K slab of a
// K that is no multiple of the slice): float4 loads from row min(k, kend - 1), zeroed past kend.
template <int R, bool FULL, bool BF = false, bool KTAIL = false>
__device__ __forceinline__ void kq_load(const float* __restrict__ P, int64_t ld, int64_t Rlim, int64_t r0, int64_t k0,
                                        int64_t kend, bool vec_ok, float (&v)[4][8], int q) {
    const int r4 = q % (R / 4), c = q / (R / 4);
    const int64_t gr = r0 + 4 * r4, gk = k0 + 8 * c;
    if constexpr (KTAIL && !BF) {
        if (k0 + X6_BK <= kend) {   // (uniform) every slice but the last: the interior loads
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const float4 f = *reinterpret_cast<const float4*>(P + (gk + k) * ld + gr);
                v[0][k] = f.x; v[1][k] = f.y; v[2][k] = f.z; v[3][k] = f.w;
            }
            return;
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const bool ok = gk + k < kend;
            const float4 f = *reinterpret_cast<const float4*>(P + (ok ? gk + k : kend - 1) * ld + gr);
            v[0][k] = ok ? f.x : 0.f; v[1][k] = ok ? f.y : 0.f; v[2][k] = ok ? f.z : 0.f; v[3][k] = ok ? f.w : 0.f;
        }
        return;
    }
    if constexpr (BF) {   // bf16 storage: 4 consecutive rows = one 8-B load per k
        const uint16_t* __restrict__ P16 = reinterpret_cast<const uint16_t*>(P);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            if (FULL || (vec_ok && gr + 3 < Rlim && gk + k < kend)) {
                const uint2 f = *reinterpret_cast<const uint2*>(P16 + (gk + k) * ld + gr);
                v[0][k] = __uint_as_float(f.x << 16); v[1][k] = __uint_as_float(f.x & 0xffff0000u);
                v[2][k] = __uint_as_float(f.y << 16); v[3][k] = __uint_as_float(f.y & 0xffff0000u);
            } else {
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    v[i][k] = (gr + i < Rlim && gk + k < kend) ? bf16_at(P16, (gk + k) * ld + gr + i) : 0.f;
            }
        }
        return;
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        if (FULL || (vec_ok && gr + 3 < Rlim && gk + k < kend)) {
            const float4 f = *reinterpret_cast<const float4*>(P + (gk + k) * ld + gr);
            v[0][k] = f.x; v[1][k] = f.y; v[2][k] = f.z; v[3][k] = f.w;
        } else {
#pragma unroll
            for (int i = 0; i < 4; ++i) v[i][k] = (gr + i < Rlim && gk + k < kend) ? P[(gk + k) * ld + gr + i] : 0.f;
        }
    }
}

template <int R, int PREC>
__device__ __forceinline__ void kq_store(uint4* __restrict__ S, const float (&v)[4][8], int q, float sc) {
    const int r4 = q % (R / 4), c = q / (R / 4);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        if constexpr (PREC == 2) {
            uint4 q0;
            q0.x = pack_bf16(v[i][0], v[i][1]); q0.y = pack_bf16(v[i][2], v[i][3]);
            q0.z = pack_bf16(v[i][4], v[i][5]); q0.w = pack_bf16(v[i][6], v[i][7]);
            S[x6_pos(4 * r4 + i, c)] = q0;
            continue;
        }
        uint4 q0, q1;
        split2h(v[i][0] * sc, v[i][1] * sc, q0.x, q1.x);
        split2h(v[i][2] * sc, v[i][3] * sc, q0.y, q1.y);
        split2h(v[i][4] * sc, v[i][5] * sc, q0.z, q1.z);
        split2h(v[i][6] * sc, v[i][7] * sc, q0.w, q1.w);
        const int pos = x6_pos(4 * r4 + i, c);
        S[pos] = q0;
        S[R * 4 + pos] = q1;
    }
}




// k-major quads of a bf16-STORED operand kept packed (PREC 2, A and B both bf16: the EA_GNN
// weight gradient g^T e, K = E): per k one 8-B load of 4 consecutive rows, held as the raw
// 16-bit pairs (8 VGPRs per quad instead of 32 widened floats), so two register sets fit and
// the slice pipeline runs at prefetch distance 2. The LDS image is the one kq_store writes
// (bf16 values are exact, the same bits).
template <int R, bool FULL>
__device__ __forceinline__ void kq_load16(const float* __restrict__ P, int64_t ld, int64_t Rlim, int64_t r0, int64_t k0,
                                          int64_t kend, bool vec_ok, uint2 (&f)[8], int q) {
    const uint16_t* __restrict__ P16 = reinterpret_cast<const uint16_t*>(P);
    const int r4 = q % (R / 4), c = q / (R / 4);
    const int64_t gr = r0 + 4 * r4, gk = k0 + 8 * c;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        if (FULL || (vec_ok && gr + 3 < Rlim && gk + k < kend)) {
            f[k] = *reinterpret_cast<const uint2*>(P16 + (gk + k) * ld + gr);
        } else {
            uint32_t e[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) e[i] = (gr + i < Rlim && gk + k < kend) ? P16[(gk + k) * ld + gr + i] : 0u;
            f[k] = make_uint2(e[0] | (e[1] << 16), e[2] | (e[3] << 16));
        }
    }
}

template <int R>
__device__ __forceinline__ void kq_store16(uint4* __restrict__ S, const uint2 (&f)[8], int q) {
    const int r4 = q % (R / 4), c = q / (R / 4);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        uint32_t w[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) w[k] = (i < 2) ? f[k].x : f[k].y;
        uint32_t p[4];
#pragma unroll
        for (int j = 0; j < 4; ++j)
            p[j] = (i & 1) ? ((w[2 * j] >> 16) | (w[2 * j + 1] & 0xffff0000u))
                           : ((w[2 * j] & 0xffffu) | (w[2 * j + 1] << 16));
        S[x6_pos(4 * r4 + i, c)] = make_uint4(p[0], p[1], p[2], p[3]);
    }
}

// the leading piece products of one 16-deep k-step, small terms first
template <int TM, int TN, int PREC, int NP>
__device__ __forceinline__ void x6_mma(floatx16 (&acc)[TM][TN], const uint4 (&fa)[TM][NP],
                                       const uint4 (&fb)[TN][NP]) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            floatx16 t = acc[i][j];
            if constexpr (PREC == 2) {   // bf16 operands: one product
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(fa[i][0]), as_bf16x8(fb[j][0]), t, 0, 0, 0);
                continue;
            }
            // f16x3: the two cross terms, then the leading product
            t = __builtin_amdgcn_mfma_f32_32x32x16_f16(as_f16x8(fa[i][0]), as_f16x8(fb[j][1]), t, 0, 0, 0);
            t = __builtin_amdgcn_mfma_f32_32x32x16_f16(as_f16x8(fa[i][1]), as_f16x8(fb[j][0]), t, 0, 0, 0);
            t = __builtin_amdgcn_mfma_f32_32x32x16_f16(as_f16x8(fa[i][0]), as_f16x8(fb[j][0]), t, 0, 0, 0);
            acc[i][j] = t;
        }
}


// ABL (timing ablations only, wrong results): 1 = no split arithmetic (piece 0 stored in
// every piece slot), 2 = no global loads, 3 = no staging at all (LDS reads + MFMA +
// barriers), 4 = MFMA + barriers only, 5 = everything but the C stores, 6 = cached C stores,
// 7 = prefetch distance 1 (one register set) and per-lane dword staging of k-major operands.
// ABL >= 16: not an ablation but the bf16 STORAGE flags ST = ABL - 16 of the bf16-operand family
// (PREC 2): bit 0 = A, bit 1 = B, bit 2 = C stored as bf16 (EA_GNN's per-edge activations).
template <int PREC, int TA, int TB, int BM, int BN, int WM, int WN, int ABL_ = 0>
__global__ __launch_bounds__(64 * WM * WN) void k_gemm_x6(GemmArgs g) {
    constexpr int ST = ABL_ >= 16 ? ABL_ - 16 : 0;
    constexpr int ABL = ABL_ >= 16 ? 0 : ABL_;
    constexpr bool A16 = (ST & 1) != 0, B16 = (ST & 2) != 0, C16 = (ST & 4) != 0;
    static_assert(ST == 0 || PREC == 2, "bf16 storage is for the bf16-operand family only");
    static_assert(PREC == 1 || PREC == 2, "f16x3 (1) or bf16 operands (2)");
    constexpr int NT = 64 * WM * WN;
    constexpr int NP = PREC == 1 ? 2 : 1;   // pieces per operand
    constexpr int TM = BM / WM / 32, TN = BN / WN / 32;
    constexpr int AK = (TA == 0) ? 1 : 0;   // A K-contiguous?
    constexpr int BKc = (TB == 1) ? 1 : 0;  // B K-contiguous?
    static_assert(BM * 4 % NT == 0 && BN * 4 % NT == 0, "staging units must divide evenly");
    // [buffer][piece][row][4 chunks of 8 16-bit values] for A, then for B; reused by the
    // epilogue as one [TM*32][32] f32 stage per wave
    constexpr int A_U4 = NP * BM * 4, B_U4 = NP * BN * 4;
    constexpr int TILE_U4 = 2 * (A_U4 + B_U4), STAGE_U4 = WM * WN * TM * 32 * 32 * 4 / 16;
    static_assert((TILE_U4 > STAGE_U4 ? TILE_U4 : STAGE_U4) * 16 <= 160 * 1024, "LDS over 160 KiB");
    __shared__ uint4 smem[TILE_U4 > STAGE_U4 ? TILE_U4 : STAGE_U4];
    uint4 (*As)[A_U4] = reinterpret_cast<uint4 (*)[A_U4]>(smem);
    uint4 (*Bs)[B_U4] = reinterpret_cast<uint4 (*)[B_U4]>(smem + 2 * A_U4);

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

    // vector loads need 16-B aligned rows (bf16 storage: 8 elements; k-major quads: 8 B, 4 elements)
    const bool a_vec = (((uintptr_t)g.A & 15) == 0) && (g.lda % ((A16 && AK) ? 8 : 4) == 0);
    const bool b_vec = (((uintptr_t)g.B & 15) == 0) && (g.ldb % ((B16 && BKc) ? 8 : 4) == 0);

    float sa = 1.f, sb = 1.f, ia = 1.f, ib = 1.f;
    if constexpr (PREC == 1) {
        h3_scale(*g.a_amax, sa, ia);
        h3_scale(*g.b_amax, sb, ib);
    }

    floatx16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    constexpr bool KQ = !AK && !BKc && PREC >= 1 && ABL != 7 && BM + BN <= NT && BM % 64 == 0 && BN % 64 == 0 &&
                        BM * BN >= 256 * 128;   // (128x128: measured slower than the dword path)
    // two register sets for the staged slices: slice kt+1 is split into LDS while slices kt+2
    // and kt+3 are in flight (prefetch distance 2; ABL 7 = distance 1 for measurement). The
    // second set fits the VGPR budget only for K-contiguous operands and tiles up to 256x128
    // (measured: fwd 363 -> 334 us, dgrad 384 -> 322 us at 256x128).
    // both k-major operands stored bf16: the quads stay packed (kq_load16), two sets fit
    constexpr bool KQ16 = KQ && A16 && B16 && PREC == 2;
    constexpr int PF = (ABL == 7 || (BM * BN > 256 * 128 && !KQ16) || (!(AK && BKc) && !KQ)) ? 1 : 2;
    // k-major quad staging for the weight gradient (both operands k-major, f16x3)
    struct RegsStd { float a[BM * 4 / NT][8]; float b[BN * 4 / NT][8]; };
    struct RegsKQ { float q[4][8]; };
    struct RegsKQ16 { uint2 q[8]; };
    using Regs = std::conditional_t<KQ16, RegsKQ16, std::conditional_t<KQ, RegsKQ, RegsStd>>;
    Regs rs[2];
    const int64_t nk = (ke > kb) ? (ke - kb + X6_BK - 1) / X6_BK : 0;
    const bool full = a_vec && b_vec && (m0 + BM <= g.M) && (n0 + BN <= g.N) && ((ke - kb) % X6_BK == 0);
    constexpr bool kStage = ABL != 3 && ABL != 4, kLoad = kStage && ABL != 2;
    // (s_setprio(1) around the MFMA block, guide T5, measured in round 3 and dropped: fwd 317 ->
    // 341 us, dgrad 324 -> 359, wgrad 303 -> 406 in an interleaved A/B, profiles/r03_*)
    // the main loop is instantiated twice (interior tiles without guards, edge tiles with
    // them) and selected once, so the hot loop carries no per-slice bounds branches
    // MODE 1 = interior tile, 2 = interior rows / columns with a ragged K range (k-major quads
    // only), 0 = edge tile (element guards)
    auto mainloop = [&](auto mode_tag) {
        constexpr int MODE = decltype(mode_tag)::value;
        constexpr bool FULL = MODE == 1, KT = MODE == 2;
        auto load_ab = [&](int64_t k0, Regs& r) {
            const float* Ab = plane_base(g.A, TA ? m0 : k0, g.a_blk, g.a_pstride);
            if constexpr (KQ16) {
                if (t < BM) kq_load16<BM, FULL>(Ab, g.lda, g.M, m0, k0, ke, a_vec, r.q, t);
                else if (t < BM + BN) kq_load16<BN, FULL>(g.B, g.ldb, g.N, n0, k0, ke, b_vec, r.q, t - BM);
            } else if constexpr (KQ) {
                if (t < BM) kq_load<BM, FULL, A16, KT>(Ab, g.lda, g.M, m0, k0, ke, a_vec, r.q, t);
                else if (t < BM + BN) kq_load<BN, FULL, B16, KT>(g.B, g.ldb, g.N, n0, k0, ke, b_vec, r.q, t - BM);
            } else {
                x6_load<AK, BM, NT, FULL, A16>(Ab, g.lda, g.M, m0, k0, ke, a_vec, r.a, t);
                x6_load<BKc, BN, NT, FULL, B16>(g.B, g.ldb, g.N, n0, k0, ke, b_vec, r.b, t);
            }
        };
        auto store_ab = [&](int buf, const Regs& r) {
            if constexpr (KQ16) {
                if (t < BM) kq_store16<BM>(As[buf], r.q, t);
                else if (t < BM + BN) kq_store16<BN>(Bs[buf], r.q, t - BM);
            } else if constexpr (KQ) {
                if (t < BM) kq_store<BM, PREC>(As[buf], r.q, t, sa);
                else if (t < BM + BN) kq_store<BN, PREC>(Bs[buf], r.q, t - BM, sb);
            } else {
                x6_store<AK, BM, NT, PREC, ABL>(As[buf], r.a, t, sa);
                x6_store<BKc, BN, NT, PREC, ABL>(Bs[buf], r.b, t, sb);
            }
        };
        const int li = lane & 31, lh = lane >> 5;
        auto mma_slice = [&](int cur, int64_t kt) {
#pragma unroll
            for (int kk = 0; kk < X6_BK / 16; ++kk) {
                uint4 a[TM][NP], b[TN][NP];
#pragma unroll
                for (int i = 0; i < TM; ++i) {
                    const int row = wm * (BM / WM) + i * 32;
#pragma unroll
                    for (int p = 0; p < NP; ++p) {
                        if constexpr (ABL == 4) a[i][p] = make_uint4(row + p, kk, i, (int)kt);
                        else a[i][p] = As[cur][p * BM * 4 + x6_pos(row + li, 2 * kk + lh)];
                    }
                }
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    const int row = wn * (BN / WN) + j * 32;
#pragma unroll
                    for (int p = 0; p < NP; ++p) {
                        if constexpr (ABL == 4) b[j][p] = make_uint4(row - p, kk, j, (int)kt);
                        else b[j][p] = Bs[cur][p * BN * 4 + x6_pos(row + li, 2 * kk + lh)];
                    }
                }
                x6_mma<TM, TN, PREC, NP>(acc, a, b);
            }
        };
        // one pipeline step: split slice kt+1 (register set S) into LDS buffer (kt+1)&1, refill
        // set S with slice kt+1+PF, multiply slice kt, barrier. S = (kt+1) & 1 for PF = 2.
        auto step = [&](int64_t kt, Regs& r) {
            const int cur = (int)(kt & 1);
            if (kt + 1 < nk && kStage) store_ab(cur ^ 1, r);
            if (kt + 1 + PF < nk && kLoad) load_ab(kb + (kt + 1 + PF) * X6_BK, r);
            // keep the staging (split VALU, LDS writes, global loads) out of the MFMA block
            __builtin_amdgcn_sched_barrier(0);
            mma_slice(cur, kt);
            __syncthreads();
        };
        if (nk > 0) {
            load_ab(kb, rs[0]);
            store_ab(0, rs[0]);
            if (nk > 1 && kLoad) load_ab(kb + X6_BK, rs[1]);
            if (PF == 2 && nk > 2 && kLoad) load_ab(kb + 2 * X6_BK, rs[0]);
        }
        __syncthreads();
        if constexpr (PF == 2) {
            int64_t kt = 0;
            for (; kt + 1 < nk; kt += 2) {
                step(kt, rs[1]);
                step(kt + 1, rs[0]);
            }
            if (kt < nk) step(kt, rs[1]);
        } else {
            for (int64_t kt = 0; kt < nk; ++kt) step(kt, rs[1]);
        }
    };
    if (full) {
        mainloop(std::integral_constant<int, 1>{});
    } else {
        // the last split-K slab of the weight gradient (K = the node count, rarely a multiple of
        // 32): interior rows and columns, only k ragged -- the guarded edge loop would set the
        // whole kernel's time (one round of workgroups: 413 vs 280 us at K = 80,656 vs 80,640)
        bool ktail = false;
        if constexpr (KQ && !A16 && !B16)
            ktail = a_vec && b_vec && (m0 + BM <= g.M) && (n0 + BN <= g.N) && (g.lda % 4 == 0) && (g.ldb % 4 == 0);
        if constexpr (KQ && !A16 && !B16) {
            if (ktail) mainloop(std::integral_constant<int, 2>{});
            else mainloop(std::integral_constant<int, 0>{});
        } else {
            mainloop(std::integral_constant<int, 0>{});
        }
    }
    // (the loop's last barrier has retired every wave's LDS reads of the operand tiles)
    float* stage = reinterpret_cast<float*>(smem) + wave * (TM * 32 * 32);
    x6_epilogue<TM, TN, ABL, C16>(g, acc, m0 + wm * (BM / WM), n0 + wn * (BN / WN), n0, ks, lane, ia, ib, stage);
}

// bm, bn, waves, workgroups per CU; configs 3 and 4 (128 KB of LDS) are built for f16x3 only
const X6Cfg kX6Cfgs[] = {
    {128, 128, 4, 1},   // 0: 2x2 waves of 64x64 (1 wave / SIMD)
    {256, 128, 8, 1},   // 1: 4x2 waves of 64x64 (2 waves / SIMD)
    {128, 256, 8, 1},   // 2: 2x4 waves of 64x64
    {256, 256, 8, 1},   // 3: 2x4 waves of 128x64
    {256, 256, 8, 1},   // 4: 4x2 waves of 64x128
};
const int kNumX6Cfgs = 5;

template <int PREC, int TA, int TB, int ABL>
static void launch_x6_a(int cfg, dim3 grid, hipStream_t s, const GemmArgs& g) {
    // 256x256 tiles (cfg 3, 4): f16x3 and bf16 (one or two pieces fit the LDS; bf16x6's three do
    // not, make_plan never picks them for it). The tile here must be the plan's tile
    // (bgnn_gemm_f32_scaled sizes the grid from it).
    if constexpr (PREC >= 1) {
        if (cfg == 3) { hipLaunchKernelGGL((k_gemm_x6<PREC, TA, TB, 256, 256, 2, 4, ABL>), grid, dim3(512), 0, s, g); return; }
        if (cfg == 4) { hipLaunchKernelGGL((k_gemm_x6<PREC, TA, TB, 256, 256, 4, 2, ABL>), grid, dim3(512), 0, s, g); return; }
    }
    switch (cfg) {
        case 0: hipLaunchKernelGGL((k_gemm_x6<PREC, TA, TB, 128, 128, 2, 2, ABL>), grid, dim3(256), 0, s, g); break;
        case 2: hipLaunchKernelGGL((k_gemm_x6<PREC, TA, TB, 128, 256, 2, 4, ABL>), grid, dim3(512), 0, s, g); break;
        default: hipLaunchKernelGGL((k_gemm_x6<PREC, TA, TB, 256, 128, 4, 2, ABL>), grid, dim3(512), 0, s, g); break;
    }
}

template <int PREC, int TA, int TB>
static void launch_x6_t(int cfg, int abl, dim3 grid, hipStream_t s, const GemmArgs& g) {
    if (abl == 0) { launch_x6_a<PREC, TA, TB, 0>(cfg, grid, s, g); return; }
    // 8 = the dgrad epilogue with the masked beta source (bgnn_gemm_f32_dropadd; f16x3, C = A B^T)
    if constexpr (PREC == 1 && TA == 0 && TB == 1) {
        if (abl == 8) { launch_x6_a<PREC, TA, TB, 8>(cfg, grid, s, g); return; }
    }
    // ablations are built for the forward shape only (TA = 0, TB = 1)
    if constexpr (TA == 0 && TB == 1) {
        switch (abl) {
            case 1: launch_x6_a<PREC, TA, TB, 1>(cfg, grid, s, g); break;
            case 2: launch_x6_a<PREC, TA, TB, 2>(cfg, grid, s, g); break;
            case 3: launch_x6_a<PREC, TA, TB, 3>(cfg, grid, s, g); break;
            case 4: launch_x6_a<PREC, TA, TB, 4>(cfg, grid, s, g); break;
            case 5: launch_x6_a<PREC, TA, TB, 5>(cfg, grid, s, g); break;
            case 6: launch_x6_a<PREC, TA, TB, 6>(cfg, grid, s, g); break;
            default: launch_x6_a<PREC, TA, TB, 7>(cfg, grid, s, g); break;
        }
    } else if constexpr (TA == 1 && TB == 0) {   // wgrad: ablation 7 (dword k-major staging)
        if (abl == 7) launch_x6_a<PREC, TA, TB, 7>(cfg, grid, s, g);
        else launch_x6_a<PREC, TA, TB, 0>(cfg, grid, s, g);
    } else {
        launch_x6_a<PREC, TA, TB, 0>(cfg, grid, s, g);
    }
}

// bf16 storage (PREC 2): st = bit 0 A, bit 1 B, bit 2 C; the combinations EA_GNN uses
static void launch_x6_bf16_storage(int ta, int tb, int cfg, int st, dim3 grid, hipStream_t s, const GemmArgs& g) {
    if (ta == 0 && tb == 1 && st == 7) launch_x6_a<2, 0, 1, 16 + 7>(cfg, grid, s, g);        // (gemm_b16.hip when K % 64 == 0)
    else if (ta == 0 && tb == 1 && st == 3) launch_x6_a<2, 0, 1, 16 + 3>(cfg, grid, s, g);
    else if (ta == 0 && tb == 1 && st == 5) launch_x6_a<2, 0, 1, 16 + 5>(cfg, grid, s, g);   // edge fwd / dgrad
    else if (ta == 0 && tb == 1 && st == 4) launch_x6_a<2, 0, 1, 16 + 4>(cfg, grid, s, g);   // f32 in, bf16 out
    else if (ta == 0 && tb == 1 && st == 1) launch_x6_a<2, 0, 1, 16 + 1>(cfg, grid, s, g);   // bf16 in, f32 out
    else if (ta == 1 && tb == 0 && st == 3) launch_x6_a<2, 1, 0, 16 + 3>(cfg, grid, s, g);   // wgrad g^T e
    else if (ta == 1 && tb == 0 && st == 1) launch_x6_a<2, 1, 0, 16 + 1>(cfg, grid, s, g);
    else if (ta == 1 && tb == 0 && st == 2) launch_x6_a<2, 1, 0, 16 + 2>(cfg, grid, s, g);
    else launch_x6_a<2, 0, 1, 16 + 5>(cfg, grid, s, g);   // (not reached: bgnn_gemm_bf16 validates st)
}

template <int PREC>
static void launch_prec(int ta, int tb, int cfg, int abl, dim3 grid, hipStream_t s, const GemmArgs& g) {
    if (ta == 0 && tb == 0) launch_x6_t<PREC, 0, 0>(cfg, abl, grid, s, g);
    else if (ta == 0 && tb == 1) launch_x6_t<PREC, 0, 1>(cfg, abl, grid, s, g);
    else if (ta == 1 && tb == 0) launch_x6_t<PREC, 1, 0>(cfg, abl, grid, s, g);
    else launch_x6_t<PREC, 1, 1>(cfg, abl, grid, s, g);
}

void launch_x6(int prec, int ta, int tb, int cfg, int abl, dim3 grid, hipStream_t s, const GemmArgs& g) {
    if (prec == 2 && g.st != 0) launch_x6_bf16_storage(ta, tb, cfg, g.st, grid, s, g);
    else if (prec == 2) launch_prec<2>(ta, tb, cfg, 0, grid, s, g);
    else launch_prec<1>(ta, tb, cfg, abl, grid, s, g);
}

// max |x| over a strided (optionally plane-split) matrix, folded into *out by an unsigned
// atomic max on the f32 bits (monotone for non-negative floats; NaN compares above Inf).
// tpr threads per row (a power of two dividing 256) sweep a row's float4 (or float) columns;
// 256 / tpr rows per block step; no integer division inside the loops.
template <bool VEC>
__global__ __launch_bounds__(256) void k_absmax(const float* __restrict__ P, int64_t rows, int64_t cols, int64_t ld,
                                                int64_t blk, int64_t pstride, int tpr, uint32_t* __restrict__ out) {
    const int rpi = 256 / tpr;
    const int tc = threadIdx.x % tpr;
    uint32_t m = 0;
    for (int64_t r = (int64_t)blockIdx.x * rpi + threadIdx.x / tpr; r < rows; r += (int64_t)gridDim.x * rpi) {
        if constexpr (VEC) {
            const float4* row = reinterpret_cast<const float4*>(P + r * ld);
            for (int64_t c = tc; c < cols / 4; c += tpr) {
                const float4 v = row[c];
                m = max(m, max(max(__float_as_uint(v.x) & 0x7fffffffu, __float_as_uint(v.y) & 0x7fffffffu),
                               max(__float_as_uint(v.z) & 0x7fffffffu, __float_as_uint(v.w) & 0x7fffffffu)));
            }
        } else {
            int64_t cb = 0;   // plane of column c (blk > 0): element at P + plane * pstride + r * ld + c - plane * blk
            int64_t c = tc;
            for (; c < cols; c += tpr) {
                if (blk > 0) cb = c / blk;
                const float* base = P + cb * (pstride - blk);
                m = max(m, __float_as_uint(base[r * ld + c]) & 0x7fffffffu);
            }
        }
    }
    for (int o = 32; o > 0; o >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, o, kWave));
    __shared__ uint32_t red[4];
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        m = max(max(red[0], red[1]), max(red[2], red[3]));
        if (m) atomicMax(out, m);
    }
}

// max |W_i| of n items of equal shape (rows x cols, ld; item i at P + i * item_stride) in one
// launch: grid.y = item, each block of an item as in k_absmax (the per-layer weight maxima of a
// SAGE loop, bgnn.fused.prepare_weights); out[i * out_stride] = max(out[.], max |W_i|).
__global__ __launch_bounds__(256) void k_absmax_items(const float* __restrict__ P, int64_t item_stride, int64_t rows,
                                                      int64_t cols4, int64_t ld, int tpr, uint32_t* __restrict__ out,
                                                      int64_t out_stride) {
    const float* Pi = P + (int64_t)blockIdx.y * item_stride;
    const int rpi = 256 / tpr;
    const int tc = threadIdx.x % tpr;
    uint32_t m = 0;
    for (int64_t r = (int64_t)blockIdx.x * rpi + threadIdx.x / tpr; r < rows; r += (int64_t)gridDim.x * rpi) {
        const float4* row = reinterpret_cast<const float4*>(Pi + r * ld);
        for (int64_t c = tc; c < cols4; c += tpr) {
            const float4 v = row[c];
            m = max(m, max(max(__float_as_uint(v.x) & 0x7fffffffu, __float_as_uint(v.y) & 0x7fffffffu),
                           max(__float_as_uint(v.z) & 0x7fffffffu, __float_as_uint(v.w) & 0x7fffffffu)));
        }
    }
    for (int o = 32; o > 0; o >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, o, kWave));
    __shared__ uint32_t red[4];
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        m = max(max(red[0], red[1]), max(red[2], red[3]));
        if (m) atomicMax(out + (int64_t)blockIdx.y * out_stride, m);
    }
}

void launch_absmax(const float* P, int64_t rows, int64_t cols, int64_t ld, int64_t blk, int64_t pstride,
                   float* out, hipStream_t s) {
    const bool vec = blk == 0 && cols % 4 == 0 && ld % 4 == 0 && (((uintptr_t)P & 15) == 0);
    const int64_t units = vec ? cols / 4 : cols;
    int tpr = 1;
    while (tpr < 256 && tpr < units) tpr <<= 1;
    const int64_t rpi = 256 / tpr;
    int64_t blocks = (rows + rpi - 1) / rpi;
    if (blocks > 2048) blocks = 2048;
    if (blocks < 1) blocks = 1;
    uint32_t* o = reinterpret_cast<uint32_t*>(out);
    if (vec) hipLaunchKernelGGL(k_absmax<true>, dim3((unsigned)blocks), dim3(256), 0, s, P, rows, cols, ld, blk, pstride, tpr, o);
    else hipLaunchKernelGGL(k_absmax<false>, dim3((unsigned)blocks), dim3(256), 0, s, P, rows, cols, ld, blk, pstride, tpr, o);
}

}  // namespace bgnn

using namespace bgnn;

extern "C" int bgnn_absmax_items_f32(const float* x, int32_t n_items, int64_t item_stride, int64_t rows, int64_t cols,
                                     int64_t ld, float* out, int64_t out_stride, void* stream) {
    BGNN_REQUIRE(x && out && n_items >= 0 && rows >= 0 && cols >= 0 && ld >= cols, "absmax_items: bad args");
    BGNN_REQUIRE(cols % 4 == 0 && ld % 4 == 0 && item_stride % 4 == 0 && (((uintptr_t)x & 15) == 0),
                 "absmax_items: cols, ld and item_stride must be multiples of 4 and x 16-B aligned");
    BGNN_REQUIRE(n_items <= 65535, "absmax_items: at most 65535 items");
    if (n_items == 0 || rows == 0 || cols == 0) return BGNN_OK;
    const int64_t cols4 = cols / 4;
    int tpr = 1;
    while (tpr < 256 && tpr < cols4) tpr <<= 1;
    const int64_t rpi = 256 / tpr;
    int64_t blocks = (rows + rpi - 1) / rpi;
    // <= 64 blocks per item: the per-layer weights are 2 MB, and 512 blocks of 2 rows each ran the
    // 6-layer pass in 32 us (launch-, not bandwidth-bound, 3,072 atomics on 6 words)
    if (blocks > 64) blocks = 64;
    hipLaunchKernelGGL(k_absmax_items, dim3((unsigned)blocks, (unsigned)n_items), dim3(256), 0, as_stream(stream), x,
                       item_stride, rows, cols4, ld, tpr, reinterpret_cast<uint32_t*>(out), out_stride);
    BGNN_CHECK_LAUNCH();
    return BGNN_OK;
}
