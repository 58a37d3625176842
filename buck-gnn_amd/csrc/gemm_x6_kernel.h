// Kernel template of the split-precision GEMMs (see gemm_x6.hip for the numerics and tiling),
// shared by the translation units that instantiate it (gemm_x6_nt.hip, gemm_x6_other.hip,
// gemm_x6_b16s.hip): one TU per instantiation family keeps the build parallel.
#pragma once
#include <type_traits>
#include <utility>

#include "common.h"
#include "gemm_common.h"
#include "gemm_x6.h"

namespace bgnn {

constexpr int X6_BK = 32;

// measurement builds only (make m16: libbgnn_m16.so, tools/fold_ab.py): the 4-wave 128x128 tile on
// 16x16x32 MFMAs as well ("MFMA shape and rounding")
#ifndef BGNN_M16_ALL
#define BGNN_M16_ALL 0
#endif

// staging units (8 k of one row) per thread for an R-row operand tile over NT threads (a unit
// count that is no multiple of NT would give the last unit to the first threads only)
constexpr int x6_nu(int R, int NT) { return (R * 4 + NT - 1) / NT; }

// 16-B chunk index of (row, chunk) in a [R][32]-bf16 image: the chunks of row r are permuted by
// chunk ^ h((r >> 2) & 3) with h = (0, 2, 3, 1), which keeps both MFMA fragment reads conflict-free
// -- 32x32x16 (lane = row, lane >> 5 = chunk within the k16 half) and 16x16x32 (lane & 15 = row,
// lane >> 4 = chunk) -- and the row-major unit stores (any per-row permutation is). (Round 4's
// h = identity left the 16x16x32 reads 2-way conflicted.)
__device__ __forceinline__ int x6_pos(int row, int chunk) {
    return row * 4 + (chunk ^ ((0x78 >> (2 * ((row >> 2) & 3))) & 3));
}

// LDS-DMA of the pre-split B image (PPV bit 3, round 6; knob BGNN_TUNE_GEMM_BDMA): address spaces
// of __builtin_amdgcn_global_load_lds, a counted vmcnt wait, and a barrier that drains only the
// LDS writes (a __syncthreads() would also drain every DMA and A load in flight, vmcnt(0))
typedef __attribute__((address_space(3))) void x6_lds_t;
typedef __attribute__((address_space(1))) void x6_gbl_t;
template <int N>
__device__ __forceinline__ void x6_wait_vmcnt() {
    static_assert(N >= 0 && N < 64, "vmcnt field is 6 bits");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void x6_barrier_lds() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}
extern int g_x6_bdma;   // 1: the pre-split f16x3 GEMMs stage B by LDS-DMA, 2-4: k_gemm_h3p (gemm_x6.hip)
struct GemmArgs;
bool h3p_ok(int cfg, const GemmArgs& g);                                // gemm_h3p.hip
void launch_h3p(int cfg, int abl, dim3 grid, hipStream_t s, const GemmArgs& g);

// one 32-deep f16x3 slice on 16x16x32 MFMAs from restrict-scoped LDS images (the DMA path: the
// scopes keep hipcc from draining the B slots' DMA in flight, vmcnt(0), before these reads); the
// same fragments, products and order as k_gemm_x6's kM16 mma_slice, so the same bits
template <int BM, int BN, int WM, int WN>
__device__ __forceinline__ void x6_mma16_h3(const uint4* __restrict__ As, const uint4* __restrict__ Bs,
                                            floatx4 (&acc)[2 * (BM / WM / 32)][2 * (BN / WN / 32)], int wm, int wn,
                                            int lane) {
    constexpr int TM = BM / WM / 32, TN = BN / WN / 32;
    const int l16 = lane & 15, lq = lane >> 4;
    auto fa = [&](int i, int p) { return As[p * BM * 4 + x6_pos(wm * (BM / WM) + i * 16 + l16, lq)]; };
    auto fb = [&](int j, int p) { return Bs[p * BN * 4 + x6_pos(wn * (BN / WN) + j * 16 + l16, lq)]; };
    auto mma3 = [&](floatx4& t, const uint4 (&a)[2], const uint4 (&b)[2]) {
        t = __builtin_amdgcn_mfma_f32_16x16x32_f16(as_f16x8(a[0]), as_f16x8(b[1]), t, 0, 0, 0);
        t = __builtin_amdgcn_mfma_f32_16x16x32_f16(as_f16x8(a[1]), as_f16x8(b[0]), t, 0, 0, 0);
        t = __builtin_amdgcn_mfma_f32_16x16x32_f16(as_f16x8(a[0]), as_f16x8(b[0]), t, 0, 0, 0);
    };
    if constexpr (TM <= TN) {
        uint4 a[2 * TM][2];
#pragma unroll
        for (int i = 0; i < 2 * TM; ++i) { a[i][0] = fa(i, 0); a[i][1] = fa(i, 1); }
#pragma unroll
        for (int j = 0; j < 2 * TN; ++j) {
            const uint4 b[2] = {fb(j, 0), fb(j, 1)};
#pragma unroll
            for (int i = 0; i < 2 * TM; ++i) mma3(acc[i][j], a[i], b);
        }
    } else {
        uint4 b[2 * TN][2];
#pragma unroll
        for (int j = 0; j < 2 * TN; ++j) { b[j][0] = fb(j, 0); b[j][1] = fb(j, 1); }
#pragma unroll
        for (int i = 0; i < 2 * TM; ++i) {
            const uint4 a[2] = {fa(i, 0), fa(i, 1)};
#pragma unroll
            for (int j = 0; j < 2 * TN; ++j) mma3(acc[i][j], a, b[j]);
        }
    }
}

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
                                        int64_t k0, int64_t kend, bool vec_ok, float (&v)[x6_nu(R, NT)][8], int t) {
    constexpr int NU = x6_nu(R, NT);
    const uint16_t* __restrict__ P16 = reinterpret_cast<const uint16_t*>(P);
#pragma unroll
    for (int u = 0; u < NU; ++u) {
        const int idx = t + NT * u;
        if (R * 4 % NT != 0 && idx >= R * 4) break;
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
template <int KCONTIG, int R, int NT, int PREC>
__device__ __forceinline__ void x6_store(uint4* __restrict__ S, const float (&v)[x6_nu(R, NT)][8], int t, float sc) {
    constexpr int NU = x6_nu(R, NT);
#pragma unroll
    for (int u = 0; u < NU; ++u) {
        const int idx = t + NT * u;
        if (R * 4 % NT != 0 && idx >= R * 4) break;
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
            split2h(v[u][0] * sc, v[u][1] * sc, q0.x, q1.x);
            split2h(v[u][2] * sc, v[u][3] * sc, q0.y, q1.y);
            split2h(v[u][4] * sc, v[u][5] * sc, q0.z, q1.z);
            split2h(v[u][6] * sc, v[u][7] * sc, q0.w, q1.w);
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
            } else {   // f16x3: the two cross terms, then the leading product
                t = __builtin_amdgcn_mfma_f32_32x32x16_f16(as_f16x8(fa[i][0]), as_f16x8(fb[j][1]), t, 0, 0, 0);
                t = __builtin_amdgcn_mfma_f32_32x32x16_f16(as_f16x8(fa[i][1]), as_f16x8(fb[j][0]), t, 0, 0, 0);
                t = __builtin_amdgcn_mfma_f32_32x32x16_f16(as_f16x8(fa[i][0]), as_f16x8(fb[j][0]), t, 0, 0, 0);
                acc[i][j] = t;
            }
        }
}


// ABL: 0 = the plain epilogue, 8 = the drop-add epilogue (bgnn_gemm_f32_dropadd: beta * drop(src)
// added with the dropout mask recomputed from its seed). ABL >= 16: the bf16 STORAGE flags
// ST = ABL - 16 of the bf16-operand family (PREC 2): bit 0 = A, bit 1 = B, bit 2 = C stored as bf16
// (EA_GNN's per-edge activations).
// PPV bit 2 (4): B arrives pre-split (bgnn_gemm_wsplit), its LDS image is copied, not split.
// (Measured and removed, records in profiles/: timing ablations, ping-pong, line-major staging, B
// fragments in registers, the interleaved schedule, the 320 x 256 tile (round 5, r05_*); a
// wave-order swap -- waves 4..7 multiply slice kt before staging slice kt+1 while waves 0..3
// stage first, so one wave of each SIMD pair is on the matrix pipe while its partner stages --
// and waves 4..7 at static s_setprio 1 (round 6, r06_gemm_ab_b.txt: dgrad 268.9 -> 292.2 /
// 272.0 us, the cfg2 step 8.66 -> 8.80 ms with the swap).)
template <int PREC, int TA, int TB, int BM, int BN, int WM, int WN, int ABL_ = 0, int PPV = 0>
__global__ __launch_bounds__(64 * WM * WN) void k_gemm_x6(GemmArgs g) {
    constexpr int ST = ABL_ >= 16 ? ABL_ - 16 : 0;
    constexpr int ABL = ABL_ >= 16 ? 0 : ABL_;
    static_assert(ABL == 0 || ABL == 8, "epilogue: plain (0) or drop-add (8)");
    constexpr bool A16 = (ST & 1) != 0, B16 = (ST & 2) != 0, C16 = (ST & 4) != 0;
    static_assert(ST == 0 || PREC == 2, "bf16 storage is for the bf16-operand family only");
    static_assert(PREC == 1 || PREC == 2, "f16x3 (1) or bf16 operands (2)");
    constexpr int NT = 64 * WM * WN;
    constexpr int NP = PREC == 1 ? 2 : 1;   // pieces per operand
    constexpr int TM = BM / WM / 32, TN = BN / WN / 32;
    constexpr int AK = (TA == 0) ? 1 : 0;   // A K-contiguous?
    constexpr int BKc = (TB == 1) ? 1 : 0;  // B K-contiguous?
    constexpr bool kWB = (PPV & 4) != 0;
    // PPV bit 3 (8, with bit 2): B's image goes global -> LDS by global_load_lds_dwordx4 into NSB
    // slots (no VGPRs, no ds_write), issued NSB - 1 slices ahead; A keeps the register split at
    // prefetch distance 2. Only the 16x16x32 8-wave tiles.
    constexpr bool kDMA = (PPV & 8) != 0;
    // PPV bit 4 (16): waves in the second half stage between the two halves of their MFMA block, so
    // that a SIMD's two waves do not leave the matrix pipe for their staging together (the guide's
    // stagger; the pre-split 256 x 256 forward)
    constexpr bool kSTG = (PPV & 16) != 0;
    static_assert(!kDMA || (kWB && PREC == 1 && 64 * WM * WN == 512), "B by LDS-DMA: pre-split f16x3, 8 waves");
    // f16x3 main loops run 16x16x32 MFMAs (four per 32x32 block, one per 32-deep slice; round 5):
    // the same cycles per FLOP as 32x32x16, but the chip holds a higher clock under them (guide
    // MI355X_MICROARCH.md, DVFS item 7): isolated dgrad 274 -> 258 us, drop-add dgrad 314 -> 303,
    // forward 277 -> 263 (profiles/r05_ab_gemm_m16.txt). The 8-wave tiles of the large GEMMs only:
    // the 4-wave 128x128 tile of the small products (the folded encoder's weight products, the
    // EA_GNN node blocks at small N) keeps 32x32x16 and its rounding ("MFMA shape and
    // rounding"). (bf16 operands, PREC 2: every tile, as the LDS-DMA bf16 kernels of gemm_b16.hip,
    // which must give the same bits)
    constexpr bool kM16 = PREC == 2 || (PREC == 1 && (NT == 512 || BGNN_M16_ALL));

    static_assert(BM * 4 % NT == 0 && BN * 4 % NT == 0, "staging units must divide evenly");

    // [buffer][piece][row][4 chunks of 8 16-bit values] for A, then for B; reused by the
    // epilogue as one [TM*32][32] f32 stage per wave
    constexpr int A_U4 = NP * BM * 4, B_U4 = NP * BN * 4;
    // B slots of the DMA path: 4 where they fit beside A's two buffers, else 3
    constexpr int NSB = (2 * A_U4 + 4 * B_U4) * 16 <= 160 * 1024 ? 4 : 3;
    constexpr int TILE_U4 = 2 * A_U4 + (kDMA ? NSB : 2) * B_U4, STAGE_U4 = WM * WN * TM * 32 * 32 * 4 / 16;
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

    floatx16 acc[kM16 ? 1 : TM][kM16 ? 1 : TN];
    floatx4 acc4[kM16 ? 2 * TM : 1][kM16 ? 2 * TN : 1];
    if constexpr (kM16) {
#pragma unroll
        for (int i = 0; i < 2 * TM; ++i)
#pragma unroll
            for (int j = 0; j < 2 * TN; ++j) acc4[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
    } else {
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    }

    constexpr bool KQ = !AK && !BKc && BM + BN <= NT && BM % 64 == 0 && BN % 64 == 0 &&
                        BM * BN >= 256 * 128;   // (128x128: measured slower than the dword path)
    // two register sets for the staged slices: slice kt+1 is split into LDS while slices kt+2
    // and kt+3 are in flight (prefetch distance 2). The second set fits the VGPR budget only for
    // K-contiguous operands and tiles up to 256x128 (measured: fwd 363 -> 334 us, dgrad 384 ->
    // 322 us at 256x128).
    // both k-major operands stored bf16: the quads stay packed (kq_load16), two sets fit
    constexpr bool KQ16 = KQ && A16 && B16 && PREC == 2;
    constexpr int PF = ((BM * BN > 256 * 128 && !KQ16) || (!(AK && BKc) && !KQ)) ? 1 : 2;
    static_assert(!kWB || (PREC == 1 && AK && BKc && !A16 && !B16 && (BN * 8) % NT == 0),
                  "pre-split B: f16x3 NT, whole 16-B pieces per thread");
    // k-major quad staging for the weight gradient (both operands k-major, f16x3)
    struct RegsStd { float a[x6_nu(BM, NT)][8]; float b[x6_nu(BN, NT)][8]; };
    // pre-split B (kWB): per thread BN * 8 / NT 16-B pieces of the slice's image, copied to LDS as is
    struct RegsWB { float a[x6_nu(BM, NT)][8]; uint4 b[BN * 8 / NT]; };
    struct RegsKQ { float q[4][8]; };
    struct RegsKQ16 { uint2 q[8]; };
    struct RegsWA { float a[x6_nu(BM, NT)][8]; };   // DMA path: A only
    using Regs = std::conditional_t<kDMA, RegsWA, std::conditional_t<KQ16, RegsKQ16, std::conditional_t<KQ, RegsKQ,
                                    std::conditional_t<kWB, RegsWB, RegsStd>>>>;
    Regs rs[2];
    const int64_t nk = (ke > kb) ? (ke - kb + X6_BK - 1) / X6_BK : 0;
    const bool full = a_vec && b_vec && (m0 + BM <= g.M) && (n0 + BN <= g.N) && ((ke - kb) % X6_BK == 0);
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
            if constexpr (kDMA) {   // (mainloop_dma)
            } else if constexpr (KQ16) {
                if (t < BM) kq_load16<BM, FULL>(Ab, g.lda, g.M, m0, k0, ke, a_vec, r.q, t);
                else if (t < BM + BN) kq_load16<BN, FULL>(g.B, g.ldb, g.N, n0, k0, ke, b_vec, r.q, t - BM);
            } else if constexpr (KQ) {
                if (t < BM) kq_load<BM, FULL, A16, KT>(Ab, g.lda, g.M, m0, k0, ke, a_vec, r.q, t);
                else if (t < BM + BN) kq_load<BN, FULL, B16, KT>(g.B, g.ldb, g.N, n0, k0, ke, b_vec, r.q, t - BM);
            } else if constexpr (kWB) {   // B: the image of slice k0 / 32 of column tile tn
                // (bgnn_gemm_f32_w passes a dense A: no plane split, no branch in the step)
                x6_load<1, BM, NT, FULL>(g.A, g.lda, g.M, m0, k0, ke, a_vec, r.a, t);
                const uint4* img = reinterpret_cast<const uint4*>(g.B) + (tn * (g.K / X6_BK) + k0 / X6_BK) * (BN * 8);
#pragma unroll
                for (int q = 0; q < BN * 8 / NT; ++q) r.b[q] = img[t + NT * q];
            } else {
                x6_load<AK, BM, NT, FULL, A16>(Ab, g.lda, g.M, m0, k0, ke, a_vec, r.a, t);
                x6_load<BKc, BN, NT, FULL, B16>(g.B, g.ldb, g.N, n0, k0, ke, b_vec, r.b, t);
            }
        };
        auto store_ab = [&](int buf, const Regs& r) {
            if constexpr (kDMA) {   // (mainloop_dma)
            } else if constexpr (KQ16) {
                if (t < BM) kq_store16<BM>(As[buf], r.q, t);
                else if (t < BM + BN) kq_store16<BN>(Bs[buf], r.q, t - BM);
            } else if constexpr (KQ) {
                if (t < BM) kq_store<BM, PREC>(As[buf], r.q, t, sa);
                else if (t < BM + BN) kq_store<BN, PREC>(Bs[buf], r.q, t - BM, sb);
            } else if constexpr (kWB) {
                x6_store<1, BM, NT, PREC>(As[buf], r.a, t, sa);
#pragma unroll
                for (int q = 0; q < BN * 8 / NT; ++q) Bs[buf][t + NT * q] = r.b[q];
            } else {
                x6_store<AK, BM, NT, PREC>(As[buf], r.a, t, sa);
                x6_store<BKc, BN, NT, PREC>(Bs[buf], r.b, t, sb);
            }
        };
        const int li = lane & 31, lh = lane >> 5;
        auto mma_slice = [&](int cur) {
            if constexpr (kM16) {   // one 32-deep step: 16-row fragments, chunk = lane >> 4
                // the side with fewer 16-row blocks is held whole, the other streamed block by block
                // (both whole would need 24 fragments = 96 VGPRs at 256x256 and spill)
                const int l16 = lane & 15, lq = lane >> 4;
                auto fa = [&](int i, int p) {
                    return (p < NP) ? As[cur][p * BM * 4 + x6_pos(wm * (BM / WM) + i * 16 + l16, lq)]
                                    : make_uint4(0, 0, 0, 0);
                };
                auto fb = [&](int j, int p) {
                    return (p < NP) ? Bs[cur][p * BN * 4 + x6_pos(wn * (BN / WN) + j * 16 + l16, lq)]
                                    : make_uint4(0, 0, 0, 0);
                };
                auto mma3 = [&](floatx4& t, const uint4 (&a)[2], const uint4 (&b)[2]) {
                    if constexpr (PREC == 2) {   // bf16 operands: one product
                        t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(a[0]), as_bf16x8(b[0]), t, 0, 0, 0);
                    } else {
                        t = __builtin_amdgcn_mfma_f32_16x16x32_f16(as_f16x8(a[0]), as_f16x8(b[1]), t, 0, 0, 0);
                        t = __builtin_amdgcn_mfma_f32_16x16x32_f16(as_f16x8(a[1]), as_f16x8(b[0]), t, 0, 0, 0);
                        t = __builtin_amdgcn_mfma_f32_16x16x32_f16(as_f16x8(a[0]), as_f16x8(b[0]), t, 0, 0, 0);
                    }
                };
                if constexpr (TM <= TN) {
                    uint4 a[2 * TM][2];
#pragma unroll
                    for (int i = 0; i < 2 * TM; ++i) { a[i][0] = fa(i, 0); a[i][1] = fa(i, 1); }
#pragma unroll
                    for (int j = 0; j < 2 * TN; ++j) {
                        const uint4 b[2] = {fb(j, 0), fb(j, 1)};
#pragma unroll
                        for (int i = 0; i < 2 * TM; ++i) mma3(acc4[i][j], a[i], b);
                    }
                } else {
                    uint4 b[2 * TN][2];
#pragma unroll
                    for (int j = 0; j < 2 * TN; ++j) { b[j][0] = fb(j, 0); b[j][1] = fb(j, 1); }
#pragma unroll
                    for (int i = 0; i < 2 * TM; ++i) {
                        const uint4 a[2] = {fa(i, 0), fa(i, 1)};
#pragma unroll
                        for (int j = 0; j < 2 * TN; ++j) mma3(acc4[i][j], a, b[j]);
                    }
                }
            } else {
#pragma unroll
            for (int kk = 0; kk < X6_BK / 16; ++kk) {
                uint4 a[TM][NP], b[TN][NP];
#pragma unroll
                for (int i = 0; i < TM; ++i) {
                    const int row = wm * (BM / WM) + i * 32;
#pragma unroll
                    for (int p = 0; p < NP; ++p) a[i][p] = As[cur][p * BM * 4 + x6_pos(row + li, 2 * kk + lh)];
                }
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    const int row = wn * (BN / WN) + j * 32;
#pragma unroll
                    for (int p = 0; p < NP; ++p) b[j][p] = Bs[cur][p * BN * 4 + x6_pos(row + li, 2 * kk + lh)];
                }
                x6_mma<TM, TN, PREC, NP>(acc, a, b);
            }
            }
        };
        // (kSTG: the held-A form of mma_slice split at column block TN, for the staggered step)
        auto mma_half = [&](int cur, const uint4 (&a)[2 * TM][2], int j0) {
            if constexpr (kSTG && kM16 && PREC == 1 && TM <= TN) {
                const int l16 = lane & 15, lq = lane >> 4;
#pragma unroll
                for (int jj = 0; jj < TN; ++jj) {
                    const int j = j0 + jj;
                    const uint4 b[2] = {Bs[cur][x6_pos(wn * (BN / WN) + j * 16 + l16, lq)],
                                        Bs[cur][BN * 4 + x6_pos(wn * (BN / WN) + j * 16 + l16, lq)]};
#pragma unroll
                    for (int i = 0; i < 2 * TM; ++i) {
                        floatx4 t = acc4[i][j];
                        t = __builtin_amdgcn_mfma_f32_16x16x32_f16(as_f16x8(a[i][0]), as_f16x8(b[1]), t, 0, 0, 0);
                        t = __builtin_amdgcn_mfma_f32_16x16x32_f16(as_f16x8(a[i][1]), as_f16x8(b[0]), t, 0, 0, 0);
                        t = __builtin_amdgcn_mfma_f32_16x16x32_f16(as_f16x8(a[i][0]), as_f16x8(b[0]), t, 0, 0, 0);
                        acc4[i][j] = t;
                    }
                }
            }
        };
        // one pipeline step: split slice kt+1 (register set S) into LDS buffer (kt+1)&1, refill
        // set S with slice kt+1+PF, multiply slice kt, barrier. S = (kt+1) & 1 for PF = 2.
        auto step = [&](int64_t kt, Regs& r) {
            const int cur = (int)(kt & 1);
            if constexpr (kSTG && kM16 && PREC == 1 && TM <= TN) {
                if (wave >= WM * WN / 2) {
                    const int l16 = lane & 15, lq = lane >> 4;
                    uint4 a[2 * TM][2];
#pragma unroll
                    for (int i = 0; i < 2 * TM; ++i) {
                        a[i][0] = As[cur][x6_pos(wm * (BM / WM) + i * 16 + l16, lq)];
                        a[i][1] = As[cur][BM * 4 + x6_pos(wm * (BM / WM) + i * 16 + l16, lq)];
                    }
                    mma_half(cur, a, 0);
                    __builtin_amdgcn_sched_barrier(0);
                    if (kt + 1 < nk) store_ab(cur ^ 1, r);
                    if (kt + 1 + PF < nk) load_ab(kb + (kt + 1 + PF) * X6_BK, r);
                    __builtin_amdgcn_sched_barrier(0);
                    mma_half(cur, a, TN);
                    __syncthreads();
                    return;
                }
            }
            if (kt + 1 < nk) store_ab(cur ^ 1, r);
            if (kt + 1 + PF < nk) load_ab(kb + (kt + 1 + PF) * X6_BK, r);
            // keep the staging (split VALU, LDS writes, global loads) out of the MFMA block
            __builtin_amdgcn_sched_barrier(0);
            mma_slice(cur);
            __syncthreads();
        };
        if (nk > 0) {
            load_ab(kb, rs[0]);
            store_ab(0, rs[0]);
            if (nk > 1) load_ab(kb + X6_BK, rs[1]);
            if (PF == 2 && nk > 2) load_ab(kb + 2 * X6_BK, rs[0]);
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
    // The DMA path (kDMA): per step, split A(kt+1) into LDS, DMA B(kt+NSB-1) into its slot, load
    // A(kt+3), multiply slice kt, wait for this wave's part of B(kt+1) with a counted vmcnt and
    // barrier. Same LDS images, fragments and MFMA order as the register path: bit-identical.
    auto mainloop_dma = [&](auto mode_tag) {
      if constexpr (kDMA) {
        constexpr bool FULL = decltype(mode_tag)::value == 1;
        constexpr int PFA = BM * BN > 256 * 128 ? 1 : 2;   // (a second A set spills at 256 x 256)
        constexpr int LA = 2 * x6_nu(BM, NT);   // A's global_load_dwordx4 per thread and slice (interior)
        constexpr int GB = BN * 8 / NT;         // B's DMA pieces per thread and slice
        // VMEM ops issued after B(kt+1) that may stay in flight at the end of step kt: the NSB - 2
        // later steps' A loads and DMA (each step issues its A loads, then its DMA)
        constexpr int WAITN = (NSB - 2) * (GB + LA);
        static_assert(WAITN < 64, "vmcnt range");
        const uint4* img = reinterpret_cast<const uint4*>(g.B) + (tn * (g.K / X6_BK) + kb / X6_BK) * (BN * 8) + t;
        uint4* const bslots = smem + 2 * A_U4;
        // every step issues its B DMA and A loads unconditionally (past the last slice they re-read
        // slice nk - 1 into a free slot / register set, never used), so that hipcc's own waits for
        // the A registers count exactly instead of draining everything (vmcnt(0)) at each step
        auto issue_b = [&](int64_t kt) {   // slice min(kt, nk - 1) into slot kt % NSB
            const uint4* src = img + (kt < nk ? kt : nk - 1) * (BN * 8);
            uint4* dst = bslots + (int)(kt % NSB) * B_U4 + wave * 64;
#pragma unroll
            for (int q = 0; q < GB; ++q)
                __builtin_amdgcn_global_load_lds((x6_gbl_t*)(src + NT * q), (x6_lds_t*)(dst + NT * q), 16, 0, 0);
        };
        auto load_a = [&](int64_t kt, Regs& r) {
            x6_load<1, BM, NT, FULL>(g.A, g.lda, g.M, m0, kb + (kt < nk ? kt : nk - 1) * X6_BK, ke, a_vec, r.a, t);
        };
        auto step = [&](int64_t kt, Regs& r) {
            const int cur = (int)(kt & 1);
            if (kt + 1 < nk) x6_store<1, BM, NT, PREC>(As[cur ^ 1], r.a, t, sa);
            // (hipcc drains all of vmcnt before the split every other step -- the DMA is a second
            // event type in the counter -- so the DMA goes after the split, never ahead of that wait)
            __builtin_amdgcn_sched_barrier(0);
            load_a(kt + 1 + PFA, r);
            issue_b(kt + NSB - 1);
            __builtin_amdgcn_sched_barrier(0);
            x6_mma16_h3<BM, BN, WM, WN>(As[cur], bslots + (int)(kt % NSB) * B_U4, acc4, wm, wn, lane);
            // this wave's part of B(kt + 1) has landed (the newer DMA and loads stay in flight); the
            // barrier then publishes every wave's part and this step's A stores
            if constexpr (FULL) x6_wait_vmcnt<WAITN>();
            else x6_wait_vmcnt<0>();
            x6_barrier_lds();
        };
        if (nk > 0) {
            for (int64_t m = 0; m < NSB - 1; ++m) issue_b(m);
            load_a(0, rs[0]);
            x6_store<1, BM, NT, PREC>(As[0], rs[0].a, t, sa);
            x6_wait_vmcnt<0>();   // B(0) .. B(NSB-2) landed (A(0) was the newest load)
            load_a(1, rs[1]);
            if constexpr (PFA == 2) load_a(2, rs[0]);
        }
        x6_barrier_lds();
        int64_t kt = 0;
        if constexpr (PFA == 2) {
            for (; kt + 1 < nk; kt += 2) {
                step(kt, rs[1]);
                step(kt + 1, rs[0]);
            }
        }
        for (; kt < nk; ++kt) step(kt, rs[1]);
        // the unused tail DMA must land before the epilogue reuses the LDS as its stage
        x6_wait_vmcnt<0>();
        x6_barrier_lds();
      }
    };
    if constexpr (kDMA) {
        if (full) mainloop_dma(std::integral_constant<int, 1>{});
        else mainloop_dma(std::integral_constant<int, 0>{});
    } else if (full) {
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
    if (ABL == 8 && n0 < g.bsrc_c0) {   // drop-add GEMM, a column tile left of the beta operand
        GemmArgs ge = g;
        ge.beta = 0.f;
        if constexpr (kM16)
            x6_epilogue<TM, TN, ABL, C16>(ge, acc4, m0 + wm * (BM / WM), n0 + wn * (BN / WN), n0, ks, lane, ia, ib, stage);
        else
            x6_epilogue<TM, TN, ABL, C16>(ge, acc, m0 + wm * (BM / WM), n0 + wn * (BN / WN), n0, ks, lane, ia, ib, stage);
        return;
    }
    if constexpr (kM16)
        x6_epilogue<TM, TN, ABL, C16>(g, acc4, m0 + wm * (BM / WM), n0 + wn * (BN / WN), n0, ks, lane, ia, ib, stage);
    else
        x6_epilogue<TM, TN, ABL, C16>(g, acc, m0 + wm * (BM / WM), n0 + wn * (BN / WN), n0, ks, lane, ia, ib, stage);
}

template <int PREC, int TA, int TB, int ABL>
inline void launch_x6_a(int cfg, dim3 grid, hipStream_t s, const GemmArgs& g) {
    if constexpr (PREC == 1 && TA == 0 && TB == 1) {
        if (g.wb && g_x6_bdma >= 2 && h3p_ok(cfg, g)) {   // the pipelined kernels (gemm_h3p.hip)
            launch_h3p(cfg, ABL, grid, s, g);
            return;
        }
#ifdef BGNN_H3P_ABLATION
        if (g.wb && g_x6_bdma == 1) {   // the same tiles with B staged by LDS-DMA (measurement build only)
            switch (cfg) {
                case 1: hipLaunchKernelGGL((k_gemm_x6<PREC, TA, TB, 256, 128, 4, 2, ABL, 12>), grid, dim3(512), 0, s, g); return;
                case 2: hipLaunchKernelGGL((k_gemm_x6<PREC, TA, TB, 128, 256, 2, 4, ABL, 12>), grid, dim3(512), 0, s, g); return;
                case 3: hipLaunchKernelGGL((k_gemm_x6<PREC, TA, TB, 256, 256, 2, 4, ABL, 12>), grid, dim3(512), 0, s, g); return;
                default: hipLaunchKernelGGL((k_gemm_x6<PREC, TA, TB, 256, 256, 4, 2, ABL, 12>), grid, dim3(512), 0, s, g); return;
            }
        }
#endif
        if (g.wb) {   // pre-split B image (bgnn_gemm_f32_w): tiles with BN = the image's column tile
            switch (cfg) {
                case 1: hipLaunchKernelGGL((k_gemm_x6<PREC, TA, TB, 256, 128, 4, 2, ABL, 4>), grid, dim3(512), 0, s, g); return;
                case 2: hipLaunchKernelGGL((k_gemm_x6<PREC, TA, TB, 128, 256, 2, 4, ABL, 4>), grid, dim3(512), 0, s, g); return;
                case 3: hipLaunchKernelGGL((k_gemm_x6<PREC, TA, TB, 256, 256, 2, 4, ABL, 4>), grid, dim3(512), 0, s, g); return;
                // (the forward's 256 x 256 tile with the staggered staging, PPV 16: 290.5 -> 283.5 us,
                // bit-identical, profiles/r06_gemm_fwd_stagger_aa.txt)
                default: hipLaunchKernelGGL((k_gemm_x6<PREC, TA, TB, 256, 256, 4, 2, ABL, 20>), grid, dim3(512), 0, s, g); return;
            }
        }
    }
    // 256x256 tiles (cfg 3, 4): f16x3 and bf16 (one or two pieces fit the LDS). The tile here must
    // be the plan's tile (bgnn_gemm_f32_scaled sizes the grid from it).
    if constexpr (PREC >= 1) {
        if (cfg == 3) { hipLaunchKernelGGL((k_gemm_x6<PREC, TA, TB, 256, 256, 2, 4, ABL>), grid, dim3(512), 0, s, g); return; }
        // (round 6: the staggered staging on the weight gradient's 256 x 256 tile measured 259.9 ->
        // 260.7 us, profiles/r06_gemm_wgrad_stagger_ac.txt; not used)
        if (cfg == 4) { hipLaunchKernelGGL((k_gemm_x6<PREC, TA, TB, 256, 256, 4, 2, ABL>), grid, dim3(512), 0, s, g); return; }
    }
    if constexpr (PREC == 1 && TA == 0 && TB == 1) {
        if (cfg == 5) { hipLaunchKernelGGL((k_gemm_x6<PREC, TA, TB, 128, 128, 2, 4, ABL>), grid, dim3(512), 0, s, g); return; }
    }
    switch (cfg) {
        case 0: hipLaunchKernelGGL((k_gemm_x6<PREC, TA, TB, 128, 128, 2, 2, ABL>), grid, dim3(256), 0, s, g); break;
        case 2: hipLaunchKernelGGL((k_gemm_x6<PREC, TA, TB, 128, 256, 2, 4, ABL>), grid, dim3(512), 0, s, g); break;
        default: hipLaunchKernelGGL((k_gemm_x6<PREC, TA, TB, 256, 128, 4, 2, ABL>), grid, dim3(512), 0, s, g); break;
    }
}


// per-family launchers (one translation unit each)
void launch_x6_nt_main(int cfg, int abl, dim3 grid, hipStream_t s, const GemmArgs& g);    // gemm_x6_nt.hip
void launch_x6_h3_other(int ta, int tb, int cfg, dim3 grid, hipStream_t s, const GemmArgs& g);  // _other
void launch_x6_prec2(int ta, int tb, int cfg, dim3 grid, hipStream_t s, const GemmArgs& g);        // _b16s
void launch_x6_bf16_storage(int ta, int tb, int cfg, int st, dim3 grid, hipStream_t s, const GemmArgs& g);

}  // namespace bgnn
