// Kernel template of the split-precision GEMMs (see gemm_x6.hip for the numerics and tiling),
// shared by the translation units that instantiate it (gemm_x6_nt.hip, gemm_x6_nt_abl.hip,
// gemm_x6_other.hip, gemm_x6_b16s.hip): one TU per instantiation family keeps the build parallel.
#pragma once
#include <type_traits>
#include <utility>

#include "common.h"
#include "gemm_common.h"
#include "gemm_x6.h"

namespace bgnn {

constexpr int X6_BK = 32;

// staging units (8 k of one row) per thread for an R-row operand tile over NT threads; a tile
// whose unit count is no multiple of NT (320 rows over 512 threads) gives the last unit to the
// first threads only (a wave-uniform guard)
constexpr int x6_nu(int R, int NT) { return (R * 4 + NT - 1) / NT; }

// 16-B chunk index of (row, chunk) in a [R][32]-bf16 image: the chunks of row r are permuted by
// chunk ^ h((r >> 2) & 3) with h = (0, 2, 3, 1), which keeps both MFMA fragment reads conflict-free
// -- 32x32x16 (lane = row, lane >> 5 = chunk within the k16 half) and 16x16x32 (lane & 15 = row,
// lane >> 4 = chunk) -- and the row-major unit stores (any per-row permutation is). (Round 4's
// h = identity left the 16x16x32 reads 2-way conflicted.)
__device__ __forceinline__ int x6_pos(int row, int chunk) {
    return row * 4 + (chunk ^ ((0x78 >> (2 * ((row >> 2) & 3))) & 3));
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
template <int KCONTIG, int R, int NT, int PREC, int ABL = 0>
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

// Line-major staging of a K-contiguous f32 operand (k_gemm_x6 with PPV bit 1): the staging unit
// is one float4 (4 consecutive k of one row); lanes 8i..8i+7 of a wave take the 8 float4 of one
// row's 32-deep slice, so each wave load instruction reads 8 whole 128-B lines (1 KiB) instead of
// 16 half lines (x6_load's 8-k units: two float4 per lane 16 B apart). Each float4 is split into
// 4 f16 of each piece and written as half of its 16-B chunk of the same swizzled image
// (ds_write_b64). Register layout: unit u2 in v[u2 / 2][4 (u2 % 2) .. +3].
template <int R, int NT, bool FULL>
__device__ __forceinline__ void lm_load(const float* __restrict__ P, int64_t ld, int64_t Rlim, int64_t r0, int64_t k0,
                                        int64_t kend, bool vec_ok, float (&v)[R * 4 / NT][8], int t) {
    constexpr int NU2 = R * 8 / NT;
#pragma unroll
    for (int u2 = 0; u2 < NU2; ++u2) {
        const int idx = t + NT * u2;
        const int64_t gr = r0 + (idx >> 3), gk = k0 + (idx & 7) * 4;
        float* d = &v[u2 >> 1][(u2 & 1) * 4];
        if (FULL || (vec_ok && gr < Rlim && gk + 3 < kend)) {
            const float4 a = *reinterpret_cast<const float4*>(P + gr * ld + gk);
            d[0] = a.x; d[1] = a.y; d[2] = a.z; d[3] = a.w;
        } else {
#pragma unroll
            for (int q = 0; q < 4; ++q) d[q] = (gr < Rlim && gk + q < kend) ? P[gr * ld + gk + q] : 0.f;
        }
    }
}

// rows [roff, roff + RH) of an R-row tile image (roff = 0, RH = R: the whole tile)
template <int RH, int NT, int R>
__device__ __forceinline__ void lm_store(uint4* __restrict__ S, const float (&v)[RH * 4 / NT][8], int t, float sc,
                                         int roff) {
    constexpr int NU2 = RH * 8 / NT;
    uint2* __restrict__ S2 = reinterpret_cast<uint2*>(S);
#pragma unroll
    for (int u2 = 0; u2 < NU2; ++u2) {
        const int idx = t + NT * u2;
        const int q = idx & 7;
        const int pos = 2 * x6_pos(roff + (idx >> 3), q >> 1) + (q & 1);
        const float* d = &v[u2 >> 1][(u2 & 1) * 4];
        uint2 h0, h1;
        split2h(d[0] * sc, d[1] * sc, h0.x, h1.x);
        split2h(d[2] * sc, d[3] * sc, h0.y, h1.y);
        S2[pos] = h0;
        S2[R * 8 + pos] = h1;
    }
}

// ping-pong staging (k_gemm_x6 with PPV): one wave group stages the rows [roff, roff + RH) of an
// R-row operand tile -- the same [piece][row][4 chunks] swizzled image x6_store writes
template <int RH, int NTG, int R>
__device__ __forceinline__ void pp_store(uint4* __restrict__ S, const float (&v)[RH * 4 / NTG][8], int t, float sc,
                                         int roff) {
    constexpr int NU = RH * 4 / NTG;
#pragma unroll
    for (int u = 0; u < NU; ++u) {
        const int idx = t + NTG * u;
        const int pos = x6_pos(roff + (idx >> 2), idx & 3);
        uint4 q0, q1;
        split2h(v[u][0] * sc, v[u][1] * sc, q0.x, q1.x);
        split2h(v[u][2] * sc, v[u][3] * sc, q0.y, q1.y);
        split2h(v[u][4] * sc, v[u][5] * sc, q0.z, q1.z);
        split2h(v[u][6] * sc, v[u][7] * sc, q0.w, q1.w);
        S[pos] = q0;
        S[R * 4 + pos] = q1;
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


// Interleaved schedule of one steady-state pipeline step of the pre-split-B GEMM (PPV bit 4):
// the step's instructions form one basic block -- the LDS fragment reads of both k16 halves of
// slice kt, the split and LDS writes of slice kt+1, the global loads of slice kt+1+PF and the
// MFMAs of slice kt -- and sched_group_barrier spreads the staging between the MFMAs (per MFMA:
// up to one fragment read of the second half, VPM VALU, one LDS write, one global load), so a
// wave's MFMA stream carries its own staging instead of leaving the matrix pipe to the partner
// wave while it stages (one MFMA gap hides about five single-issue instructions; guide
// MI355X_MICROARCH.md, cycle constants).
template <int I, int NR, int NW, int NV, int VPM>
__device__ __forceinline__ void x6_il_one() {
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);                    // one MFMA
    if constexpr (I < NR) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);   // a fragment read
    __builtin_amdgcn_sched_group_barrier(0x002, VPM, 0);                  // VALU (the split)
    if constexpr (I >= 2 && I - 2 < NW) __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);   // LDS write
    if constexpr (I >= NR && I - NR < NV) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0); // global load
}
template <int NR0, int NR, int NW, int NV, int VPM, int... I>
__device__ __forceinline__ void x6_il_schedule(std::integer_sequence<int, I...>) {
    __builtin_amdgcn_sched_group_barrier(0x100, NR0, 0);   // the first half's fragment reads
    (x6_il_one<I, NR, NW, NV, VPM>(), ...);
}

// ABL (timing ablations only, wrong results): 1 = no split arithmetic (piece 0 stored in
// every piece slot), 2 = no global loads, 3 = no staging at all (LDS reads + MFMA +
// barriers), 4 = MFMA + barriers only, 5 = everything but the C stores, 6 = cached C stores,
// 7 = prefetch distance 1 (one register set) and per-lane dword staging of k-major operands,
// 9 = no A loads, 10 = no B loads, 11 = no MFMAs (staging, LDS reads, barriers, epilogue).
// ABL >= 16: not an ablation but the bf16 STORAGE flags ST = ABL - 16 of the bf16-operand family
// (PREC 2): bit 0 = A, bit 1 = B, bit 2 = C stored as bf16 (EA_GNN's per-edge activations).
// PPV bit 1: line-major staging loads (lm_load). PPV bit 0: ping-pong main loop (f16x3, A and B
// K-contiguous): waves 0..NW/2-1 (group 0, rows
// [0, BM/2) of the tile) and NW/2..NW-1 (group 1, rows [BM/2, BM)) -- one wave of each group per
// SIMD -- alternate roles every half step: while one group runs the MFMAs of slice k, the other
// splits its half of slice k+1 (its A rows and half of the B rows) into LDS and issues the loads of
// slice k+2; a barrier between the halves. The matrix pipe of each SIMD is fed by one group while
// the other's split VALU, LDS writes and loads run beside it, instead of both waves competing for
// the pipe and then both staging with the pipe idle.
template <int PREC, int TA, int TB, int BM, int BN, int WM, int WN, int ABL_ = 0, int PPV = 0>
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
    // PPV bit 2: B arrives pre-split (bgnn_gemm_wsplit): its LDS image is copied, not split
    constexpr bool kWB = (PPV & 4) != 0;
    // PPV bit 4 (with bit 2): the steady-state steps run the interleaved schedule (x6_il_schedule)
    constexpr bool kIL = (PPV & 16) != 0;
    // f16x3 main loops run 16x16x32 MFMAs (four per 32x32 block, one per 32-deep slice; round 5):
    // the same cycles per FLOP as 32x32x16, but the chip holds a higher clock under them (guide
    // MI355X_MICROARCH.md, DVFS item 7): isolated dgrad 274 -> 258 us, drop-add dgrad 314 -> 303,
    // forward 277 -> 263 (profiles/r05_ab_gemm_m16.txt). The 8-wave tiles of the large GEMMs only:
    // the 4-wave 128x128 tile of the small products (the folded encoder's weight products, the
    // EA_GNN node blocks at small N) keeps 32x32x16 and its rounding (tests/test_gpu_fold.py
    // measures the folded path's gradients against fp64 relative to the unfolded path's). PPV bit 5
    // keeps 32x32x16 (A/B), as do the ping-pong, line-major, interleaved and B-in-registers variants.
    // (bf16 operands, PREC 2: every tile, as the LDS-DMA bf16 kernels of gemm_b16.hip, which must
    // give the same bits)
    constexpr bool kM16 = (PREC == 2 || (PREC == 1 && NT == 512)) && (PPV & 32) == 0 &&
                          (PPV & (1 | 2 | 8 | 16)) == 0;

    // (pre-split B: A may have a unit count that is no multiple of NT, x6_nu's guarded last unit)
    static_assert((BM * 4 % NT == 0 || kWB) && BN * 4 % NT == 0, "staging units must divide evenly");
    // PPV bit 3: B's MFMA fragments are loaded straight from the pre-split image into registers
    // (no LDS image of B: its writes and reads leave the LDS port to A)
    constexpr bool kWR = (PPV & 8) != 0;
    static_assert(!kWR || (PREC == 1 && AK && BKc && !A16 && !B16 && (PPV & 7) == 0 && ABL != 7),
                  "B in registers: f16x3 NT on a pre-split image");

    // [buffer][piece][row][4 chunks of 8 16-bit values] for A, then for B; reused by the
    // epilogue as one [TM*32][32] f32 stage per wave
    constexpr int A_U4 = NP * BM * 4, B_U4 = NP * BN * 4;
    constexpr int TILE_U4 = 2 * (A_U4 + (kWR ? 0 : B_U4)), STAGE_U4 = WM * WN * TM * 32 * 32 * 4 / 16;
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

    constexpr bool KQ = !AK && !BKc && PREC >= 1 && ABL != 7 && BM + BN <= NT && BM % 64 == 0 && BN % 64 == 0 &&
                        BM * BN >= 256 * 128;   // (128x128: measured slower than the dword path)
    // two register sets for the staged slices: slice kt+1 is split into LDS while slices kt+2
    // and kt+3 are in flight (prefetch distance 2; ABL 7 = distance 1 for measurement). The
    // second set fits the VGPR budget only for K-contiguous operands and tiles up to 256x128
    // (measured: fwd 363 -> 334 us, dgrad 384 -> 322 us at 256x128).
    // both k-major operands stored bf16: the quads stay packed (kq_load16), two sets fit
    constexpr bool KQ16 = KQ && A16 && B16 && PREC == 2;
    constexpr int PF = (ABL == 7 || (BM * BN > 256 * 128 && !KQ16) || (!(AK && BKc) && !KQ)) ? 1 : 2;
    static_assert(!kWB || (PREC == 1 && AK && BKc && !A16 && !B16 && (PPV & 3) == 0 && (BN * 8) % NT == 0),
                  "pre-split B: f16x3 NT, whole 16-B pieces per thread");
    // k-major quad staging for the weight gradient (both operands k-major, f16x3)
    struct RegsStd { float a[x6_nu(BM, NT)][8]; float b[x6_nu(BN, NT)][8]; };
    // pre-split B (kWB): per thread BN * 8 / NT 16-B pieces of the slice's image, copied to LDS as is
    struct RegsWB { float a[x6_nu(BM, NT)][8]; uint4 b[BN * 8 / NT]; };
    struct RegsKQ { float q[4][8]; };
    struct RegsKQ16 { uint2 q[8]; };
    using Regs = std::conditional_t<KQ16, RegsKQ16, std::conditional_t<KQ, RegsKQ,
                                    std::conditional_t<kWB, RegsWB, RegsStd>>>;
    Regs rs[2];
    const int64_t nk = (ke > kb) ? (ke - kb + X6_BK - 1) / X6_BK : 0;
    const bool full = a_vec && b_vec && (m0 + BM <= g.M) && (n0 + BN <= g.N) && ((ke - kb) % X6_BK == 0);
    constexpr bool kStage = ABL != 3 && ABL != 4, kLoad = kStage && ABL != 2;
    // line-major f32 staging (lm_load / lm_store) of K-contiguous f16x3 operands
    constexpr bool kLM = (PPV & 2) != 0;
    static_assert(!kLM || (PREC == 1 && AK && BKc && !A16 && !B16 && ABL != 1), "line-major: f16x3, K-contiguous f32");
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
            } else if constexpr (kWB) {   // B: the image of slice k0 / 32 of column tile tn
                // (bgnn_gemm_f32_w passes a dense A: no plane split, no branch in the step)
                x6_load<1, BM, NT, FULL>(g.A, g.lda, g.M, m0, k0, ke, a_vec, r.a, t);
                const uint4* img = reinterpret_cast<const uint4*>(g.B) + (tn * (g.K / X6_BK) + k0 / X6_BK) * (BN * 8);
#pragma unroll
                for (int q = 0; q < BN * 8 / NT; ++q) r.b[q] = img[t + NT * q];
            } else if constexpr (kLM) {
                lm_load<BM, NT, FULL>(Ab, g.lda, g.M, m0, k0, ke, a_vec, r.a, t);
                lm_load<BN, NT, FULL>(g.B, g.ldb, g.N, n0, k0, ke, b_vec, r.b, t);
            } else {
                if constexpr (ABL != 9) x6_load<AK, BM, NT, FULL, A16>(Ab, g.lda, g.M, m0, k0, ke, a_vec, r.a, t);
                if constexpr (ABL != 10) x6_load<BKc, BN, NT, FULL, B16>(g.B, g.ldb, g.N, n0, k0, ke, b_vec, r.b, t);
            }
        };
        auto store_ab = [&](int buf, const Regs& r) {
            if constexpr (KQ16) {
                if (t < BM) kq_store16<BM>(As[buf], r.q, t);
                else if (t < BM + BN) kq_store16<BN>(Bs[buf], r.q, t - BM);
            } else if constexpr (KQ) {
                if (t < BM) kq_store<BM, PREC>(As[buf], r.q, t, sa);
                else if (t < BM + BN) kq_store<BN, PREC>(Bs[buf], r.q, t - BM, sb);
            } else if constexpr (kWB) {
                x6_store<1, BM, NT, PREC, ABL>(As[buf], r.a, t, sa);
#pragma unroll
                for (int q = 0; q < BN * 8 / NT; ++q) Bs[buf][t + NT * q] = r.b[q];
            } else if constexpr (kLM) {
                lm_store<BM, NT, BM>(As[buf], r.a, t, sa, 0);
                lm_store<BN, NT, BN>(Bs[buf], r.b, t, sb, 0);
            } else {
                x6_store<AK, BM, NT, PREC, ABL>(As[buf], r.a, t, sa);
                x6_store<BKc, BN, NT, PREC, ABL>(Bs[buf], r.b, t, sb);
            }
        };
        const int li = lane & 31, lh = lane >> 5;
        auto mma_slice = [&](int cur, int64_t kt) {
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
                        for (int i = 0; i < 2 * TM; ++i)
                            if constexpr (ABL != 11) mma3(acc4[i][j], a[i], b);
                    }
                } else {
                    uint4 b[2 * TN][2];
#pragma unroll
                    for (int j = 0; j < 2 * TN; ++j) { b[j][0] = fb(j, 0); b[j][1] = fb(j, 1); }
#pragma unroll
                    for (int i = 0; i < 2 * TM; ++i) {
                        const uint4 a[2] = {fa(i, 0), fa(i, 1)};
#pragma unroll
                        for (int j = 0; j < 2 * TN; ++j)
                            if constexpr (ABL != 11) mma3(acc4[i][j], a, b[j]);
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
                if constexpr (ABL != 11) x6_mma<TM, TN, PREC, NP>(acc, a, b);
                else if (kt < 0) x6_mma<TM, TN, PREC, NP>(acc, a, b);   // (keeps the reads live)
            }
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
        // steady-state step of the interleaved schedule (kIL): slice kt+1 is stored and slice
        // kt+1+PF loaded unconditionally, one basic block; the four buffers are restrict-qualified
        // so the writes to buffer cur^1 may move among the reads of buffer cur
        auto step_il = [&](const uint4* __restrict__ ard, const uint4* __restrict__ brd, uint4* __restrict__ awr,
                           uint4* __restrict__ bwr, int64_t k_next, Regs& r) {
            if constexpr (kWB && kIL) {
                uint4 fa[2][TM][NP], fb[2][TN][NP];
#pragma unroll
                for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
                    for (int i = 0; i < TM; ++i)
#pragma unroll
                        for (int p = 0; p < NP; ++p)
                            fa[kk][i][p] = ard[p * BM * 4 + x6_pos(wm * (BM / WM) + i * 32 + li, 2 * kk + lh)];
#pragma unroll
                    for (int j = 0; j < TN; ++j)
#pragma unroll
                        for (int p = 0; p < NP; ++p)
                            fb[kk][j][p] = brd[p * BN * 4 + x6_pos(wn * (BN / WN) + j * 32 + li, 2 * kk + lh)];
                }
                x6_store<1, BM, NT, PREC, ABL>(awr, r.a, t, sa);
#pragma unroll
                for (int q = 0; q < BN * 8 / NT; ++q) bwr[t + NT * q] = r.b[q];
                load_ab(k_next, r);
                x6_mma<TM, TN, PREC, NP>(acc, fa[0], fb[0]);
                x6_mma<TM, TN, PREC, NP>(acc, fa[1], fb[1]);
                constexpr int NM = 2 * TM * TN * 3, NR0 = (TM + TN) * NP;
                constexpr int NW = x6_nu(BM, NT) * 2 + BN * 8 / NT, NV = x6_nu(BM, NT) * 2 + BN * 8 / NT;
                x6_il_schedule<NR0, NR0, NW, NV, 2>(std::make_integer_sequence<int, NM>{});
            }
        };
        auto il = [&](int64_t kt, Regs& r) {
            const int cur = (int)(kt & 1);
            step_il(As[cur], Bs[cur], As[cur ^ 1], Bs[cur ^ 1], kb + (kt + 1 + PF) * X6_BK, r);
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
            if constexpr (kWB && kIL) {
                for (; kt + 2 + PF < nk; kt += 2) {
                    il(kt, rs[1]);
                    il(kt + 1, rs[0]);
                }
            }
            for (; kt + 1 < nk; kt += 2) {
                step(kt, rs[1]);
                step(kt + 1, rs[0]);
            }
            if (kt < nk) step(kt, rs[1]);
        } else {
            int64_t kt = 0;
            if constexpr (kWB && kIL) {
                for (; kt + 1 + PF < nk; ++kt) il(kt, rs[1]);
            }
            for (; kt < nk; ++kt) step(kt, rs[1]);
        }
    };
    if constexpr (kWR) {
        // A through LDS as in the main loop (prefetch distance 2, split in registers); the B
        // fragments of slice kt+1 are loaded from the image (one 16-B load per lane, fragment and
        // piece: L2-resident, shared by every row tile of the column tile) while slice kt's
        // MFMAs run, into the second of two register sets
        const int li = lane & 31, lh = lane >> 5;
        const uint4* __restrict__ img = reinterpret_cast<const uint4*>(g.B) + tn * (g.K / X6_BK) * (BN * 8);
        const int64_t s0 = kb / X6_BK;
        float ra[2][x6_nu(BM, NT)][8];
        uint4 rb[2][2][TN][NP];   // [set][kk][j][piece]
        auto load_b = [&](int64_t kt, uint4 (&b)[2][TN][NP]) {
            const uint4* __restrict__ blk = img + (s0 + kt) * (BN * 8);
#pragma unroll
            for (int kk = 0; kk < 2; ++kk)
#pragma unroll
                for (int j = 0; j < TN; ++j)
#pragma unroll
                    for (int p = 0; p < NP; ++p)   // (fragment-order image: one 1-KiB wave load each)
                        b[kk][j][p] = blk[(((wn * (BN / WN) / 32 + j) * 2 + kk) * 2 + p) * 64 + lane];
        };
        auto wr_loop = [&](auto mode_tag) {
            constexpr bool FULL = decltype(mode_tag)::value == 1;
            auto load_a = [&](int64_t kt, float (&v)[x6_nu(BM, NT)][8]) {
                const int64_t k0 = kb + kt * X6_BK;
                x6_load<1, BM, NT, FULL>(plane_base(g.A, k0, g.a_blk, g.a_pstride), g.lda, g.M, m0, k0, ke, a_vec, v, t);
            };
            auto mma = [&](int cur, const uint4 (&b)[2][TN][NP]) {
#pragma unroll
                for (int kk = 0; kk < X6_BK / 16; ++kk) {
                    uint4 a[TM][NP];
#pragma unroll
                    for (int i = 0; i < TM; ++i)
#pragma unroll
                        for (int p = 0; p < NP; ++p)
                            a[i][p] = As[cur][p * BM * 4 + x6_pos(wm * (BM / WM) + i * 32 + li, 2 * kk + lh)];
                    if constexpr (ABL != 11) x6_mma<TM, TN, PREC, NP>(acc, a, b[kk]);
                }
            };
            auto step = [&](int64_t kt, float (&va)[x6_nu(BM, NT)][8], const uint4 (&bc)[2][TN][NP],
                            uint4 (&bnx)[2][TN][NP]) {
                const int cur = (int)(kt & 1);
                if (kt + 1 < nk) x6_store<1, BM, NT, PREC, 0>(As[cur ^ 1], va, t, sa);
                if (kt + 3 < nk) load_a(kt + 3, va);
                if (kt + 1 < nk) load_b(kt + 1, bnx);
                __builtin_amdgcn_sched_barrier(0);
                mma(cur, bc);
                __syncthreads();
            };
            if (nk > 0) {
                load_a(0, ra[0]);
                x6_store<1, BM, NT, PREC, 0>(As[0], ra[0], t, sa);
                load_b(0, rb[0]);
                if (nk > 1) load_a(1, ra[1]);
                if (nk > 2) load_a(2, ra[0]);
            }
            __syncthreads();
            int64_t kt = 0;
            for (; kt + 1 < nk; kt += 2) {
                step(kt, ra[1], rb[0], rb[1]);
                step(kt + 1, ra[0], rb[1], rb[0]);
            }
            if (kt < nk) step(kt, ra[1], rb[0], rb[1]);
        };
        if (full) wr_loop(std::integral_constant<int, 1>{});
        else wr_loop(std::integral_constant<int, 0>{});
    } else if constexpr ((PPV & 1) != 0) {
        static_assert(PREC == 1 && AK && BKc && ABL != 7, "ping-pong: f16x3 with K-contiguous A and B");
        constexpr int NTG = NT / 2, RA = BM / 2, RB = BN / 2;
        static_assert(RA * 4 % NTG == 0 && RB * 4 % NTG == 0 && (WM * WN) % 2 == 0 && (WM % 2 == 0 || WM == 1),
                      "ping-pong: each group stages whole units and owns half of the tile's wave rows");
        const int grp = wave >= (WM * WN) / 2;
        const int tg = t - grp * NTG;
        float va[RA * 4 / NTG][8], vb[RB * 4 / NTG][8];
        auto pp_loop = [&](auto mode_tag) {
            constexpr bool FULL = decltype(mode_tag)::value == 1;
            auto load = [&](int64_t k0) {
                if constexpr (kLoad) {
                    const float* Ab = plane_base(g.A, k0, g.a_blk, g.a_pstride);
                    if constexpr (kLM) {
                        lm_load<RA, NTG, FULL>(Ab, g.lda, g.M, m0 + grp * RA, k0, ke, a_vec, va, tg);
                        lm_load<RB, NTG, FULL>(g.B, g.ldb, g.N, n0 + grp * RB, k0, ke, b_vec, vb, tg);
                    } else {
                        x6_load<1, RA, NTG, FULL>(Ab, g.lda, g.M, m0 + grp * RA, k0, ke, a_vec, va, tg);
                        x6_load<1, RB, NTG, FULL>(g.B, g.ldb, g.N, n0 + grp * RB, k0, ke, b_vec, vb, tg);
                    }
                }
            };
            auto store = [&](int buf) {
                if constexpr (kStage) {
                    if constexpr (kLM) {
                        lm_store<RA, NTG, BM>(As[buf], va, tg, sa, grp * RA);
                        lm_store<RB, NTG, BN>(Bs[buf], vb, tg, sb, grp * RB);
                    } else {
                        pp_store<RA, NTG, BM>(As[buf], va, tg, sa, grp * RA);
                        pp_store<RB, NTG, BN>(Bs[buf], vb, tg, sb, grp * RB);
                    }
                }
            };
            const int li = lane & 31, lh = lane >> 5;
            auto mma = [&](int cur) {
#pragma unroll
                for (int kk = 0; kk < X6_BK / 16; ++kk) {
                    uint4 a[TM][NP], b[TN][NP];
#pragma unroll
                    for (int i = 0; i < TM; ++i)
#pragma unroll
                        for (int p = 0; p < NP; ++p)
                            a[i][p] = As[cur][p * BM * 4 + x6_pos(wm * (BM / WM) + i * 32 + li, 2 * kk + lh)];
#pragma unroll
                    for (int j = 0; j < TN; ++j)
#pragma unroll
                        for (int p = 0; p < NP; ++p)
                            b[j][p] = Bs[cur][p * BN * 4 + x6_pos(wn * (BN / WN) + j * 32 + li, 2 * kk + lh)];
                    x6_mma<TM, TN, PREC, NP>(acc, a, b);
                }
            };
            auto stage = [&](int64_t kt) {   // split slice kt+1 into the other buffer, load slice kt+2
                if (kt + 1 < nk) {
                    store((int)((kt + 1) & 1));
                    if (kt + 2 < nk) load(kb + (kt + 2) * X6_BK);
                }
            };
            if (nk > 0) {
                load(kb);
                store(0);
                if (nk > 1) load(kb + X6_BK);
            }
            __syncthreads();
            for (int64_t kt = 0; kt < nk; ++kt) {
                const int cur = (int)(kt & 1);
                if (grp == 0) mma(cur);
                else stage(kt);
                __syncthreads();
                if (grp == 0) stage(kt);
                else mma(cur);
                __syncthreads();
            }
        };
        if (full) pp_loop(std::integral_constant<int, 1>{});
        else pp_loop(std::integral_constant<int, 0>{});
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
    if constexpr (PREC == 1 && TA == 0 && TB == 1 && (ABL == 0 || ABL == 8)) {
        if (g.wb) {   // pre-split B image (bgnn_gemm_f32_w): tiles with BN = the image's column tile
            if (gemm_pp() == 6) {   // 32x32x16 MFMAs, the form before round 5's default (BGNN_TUNE_GEMM_PP = 6)
                switch (cfg) {
                    case 1: hipLaunchKernelGGL((k_gemm_x6<PREC, TA, TB, 256, 128, 4, 2, ABL, 36>), grid, dim3(512), 0, s, g); return;
                    case 2: hipLaunchKernelGGL((k_gemm_x6<PREC, TA, TB, 128, 256, 2, 4, ABL, 36>), grid, dim3(512), 0, s, g); return;
                    case 3: hipLaunchKernelGGL((k_gemm_x6<PREC, TA, TB, 256, 256, 2, 4, ABL, 36>), grid, dim3(512), 0, s, g); return;
                    case 4: hipLaunchKernelGGL((k_gemm_x6<PREC, TA, TB, 256, 256, 4, 2, ABL, 36>), grid, dim3(512), 0, s, g); return;
                    default: break;
                }
            }
            if (gemm_pp() == 5) {   // interleaved schedule (BGNN_TUNE_GEMM_PP = 5; 256x256: spills)
                switch (cfg) {
                    case 1: hipLaunchKernelGGL((k_gemm_x6<PREC, TA, TB, 256, 128, 4, 2, ABL, 20>), grid, dim3(512), 0, s, g); return;
                    case 2: hipLaunchKernelGGL((k_gemm_x6<PREC, TA, TB, 128, 256, 2, 4, ABL, 20>), grid, dim3(512), 0, s, g); return;
                    default: break;
                }
            }
            if (gemm_pp() == 4) {   // B fragments in registers (BGNN_TUNE_GEMM_PP = 4)
                if (cfg == 1) { hipLaunchKernelGGL((k_gemm_x6<PREC, TA, TB, 256, 128, 4, 2, ABL, 8>), grid, dim3(512), 0, s, g); return; }
                if (cfg == 2) { hipLaunchKernelGGL((k_gemm_x6<PREC, TA, TB, 128, 256, 2, 4, ABL, 8>), grid, dim3(512), 0, s, g); return; }
            }
            switch (cfg) {
                case 1: hipLaunchKernelGGL((k_gemm_x6<PREC, TA, TB, 256, 128, 4, 2, ABL, 4>), grid, dim3(512), 0, s, g); return;
                case 2: hipLaunchKernelGGL((k_gemm_x6<PREC, TA, TB, 128, 256, 2, 4, ABL, 4>), grid, dim3(512), 0, s, g); return;
                case 3: hipLaunchKernelGGL((k_gemm_x6<PREC, TA, TB, 256, 256, 2, 4, ABL, 4>), grid, dim3(512), 0, s, g); return;
                case 5: hipLaunchKernelGGL((k_gemm_x6<PREC, TA, TB, 320, 256, 2, 4, ABL, 4>), grid, dim3(512), 0, s, g); return;
                default: hipLaunchKernelGGL((k_gemm_x6<PREC, TA, TB, 256, 256, 4, 2, ABL, 4>), grid, dim3(512), 0, s, g); return;
            }
        }
    }
    if constexpr (PREC == 1 && TA == 0 && TB == 1 && (ABL == 0 || ABL == 8 || (ABL >= 2 && ABL <= 5))) {
        const int ppv = gemm_pp();
        if (ppv >= 1 && ppv <= 3) {
#define BGNN_PPV(V)                                                                                                  \
    switch (cfg) {                                                                                                   \
        case 1: hipLaunchKernelGGL((k_gemm_x6<PREC, TA, TB, 256, 128, 4, 2, ABL, V>), grid, dim3(512), 0, s, g); return; \
        case 2: hipLaunchKernelGGL((k_gemm_x6<PREC, TA, TB, 128, 256, 2, 4, ABL, V>), grid, dim3(512), 0, s, g); return; \
        case 3: hipLaunchKernelGGL((k_gemm_x6<PREC, TA, TB, 256, 256, 2, 4, ABL, V>), grid, dim3(512), 0, s, g); return; \
        case 4: hipLaunchKernelGGL((k_gemm_x6<PREC, TA, TB, 256, 256, 4, 2, ABL, V>), grid, dim3(512), 0, s, g); return; \
        default: break;                                                                                              \
    }
            if (ppv == 1) { BGNN_PPV(1) }
            else if (ppv == 2) { BGNN_PPV(2) }
            else { BGNN_PPV(3) }
#undef BGNN_PPV
        }
    }
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


// per-family launchers (one translation unit each)
void launch_x6_nt_main(int cfg, int abl, dim3 grid, hipStream_t s, const GemmArgs& g);    // gemm_x6_nt.hip
void launch_x6_nt_abl(int cfg, int abl, dim3 grid, hipStream_t s, const GemmArgs& g);     // gemm_x6_nt_abl.hip
void launch_x6_h3_other(int ta, int tb, int cfg, int abl, dim3 grid, hipStream_t s, const GemmArgs& g);  // _other
void launch_x6_prec2(int ta, int tb, int cfg, dim3 grid, hipStream_t s, const GemmArgs& g);        // _b16s
void launch_x6_bf16_storage(int ta, int tb, int cfg, int st, dim3 grid, hipStream_t s, const GemmArgs& g);

}  // namespace bgnn
