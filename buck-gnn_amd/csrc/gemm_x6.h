// Split-precision GEMM tile helpers of gemm_x6.hip (and the bf16 C stores gemm_b16.hip shares):
// operand piece splits, the f16x3 operand scale and the LDS-staged C epilogue.
#pragma once
#include "common.h"
#include "gemm_common.h"

namespace bgnn {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

// two f32 -> packed bf16x2 (round to nearest even; v_cvt_pk_bf16_f32)
__device__ __forceinline__ uint32_t pack_bf16(float x, float y) {
    const f32x2 v = {x, y};
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2));
}

// two f32 -> packed f16x2 (round to nearest even; v_cvt_pk_f16_f32)
__device__ __forceinline__ uint32_t pack_f16(float x, float y) {
    const f32x2 v = {x, y};
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, f16x2));
}

// two-way f16 split of the (already scaled) pair (x, y); scalar residuals (no packed f32 VALU)
__device__ __forceinline__ void split2h(float x, float y, uint32_t& p0, uint32_t& p1) {
    p0 = pack_f16(x, y);
    const f16x2 h = __builtin_bit_cast(f16x2, p0);
    x -= (float)h[0];
    y -= (float)h[1];
    p1 = pack_f16(x, y);
}

// power-of-two operand scale for PREC 1: s = 2^k with max|a| * s in [2^14, 2^15), k clamped to
// [-126, 126] (zero, Inf or NaN max -> s = 1); inv = 1 / s
__device__ __forceinline__ void h3_scale(float amax, float& s, float& inv) {
    const uint32_t b = __float_as_uint(amax) & 0x7fffffffu;
    int k = 0;
    if (b != 0 && b < 0x7f800000u) {
        k = 14 - ((int)(b >> 23) - 127);
        k = k < -126 ? -126 : (k > 126 ? 126 : k);
    }
    s = __uint_as_float((uint32_t)(127 + k) << 23);
    inv = __uint_as_float((uint32_t)(127 - k) << 23);
}

__device__ __forceinline__ bf16x8 as_bf16x8(uint4 q) { return __builtin_bit_cast(bf16x8, q); }
__device__ __forceinline__ f16x8 as_f16x8(uint4 q) { return __builtin_bit_cast(f16x8, q); }

// C leaves with non-temporal stores: it is streamed once, and write-allocating it in L2 / the
// Infinity Cache costs ~40 % of the kernel (fwd 360 -> 220 us, measured on MI355X).
__device__ __forceinline__ void st_nt4(float* p, const float (&e)[4]) {
    typedef float f32x4_t __attribute__((ext_vector_type(4)));
    const f32x4_t t = {e[0], e[1], e[2], e[3]};
    __builtin_nontemporal_store(t, reinterpret_cast<f32x4_t*>(p));
}

// Epilogue: each wave writes its TM x TN accumulator tiles one 32-column block at a time
// into a wave-private LDS stage [TM*32][32] f32 (C/D map of the 32x32 MFMA: col = lane & 31,
// row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5); one ds_write_b32 group per row, conflict-free)
// and reads it back as float4 rows (8 lanes per 128-B row segment, conflict-free
// ds_read_b128), so C leaves as 16-B stores, 1 KiB per wave instruction. Unscale (f16x3),
// alpha, beta, bias, ReLU and the max |C| (c_amax) are applied per float4.
// C16: C stored as bf16 (round to nearest even), 8-B stores; no beta / split-K with it.
__device__ __forceinline__ void st_bf16x4(float* p, const float (&e)[4]) {
    uint2 q;
    q.x = pack_bf16(e[0], e[1]);
    q.y = pack_bf16(e[2], e[3]);
    *reinterpret_cast<uint2*>(p) = q;
}

// the accumulators of column block j into the wave's LDS stage [TM*32][32]: 32x32x16 MFMA tiles
// (C/D map col = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5)) ...
template <int TM, int TN>
__device__ __forceinline__ void x6_stage_write(float* __restrict__ stage, const floatx16 (&acc)[TM][TN], int j,
                                               int lane) {
    const int li = lane & 31, lh = lane >> 5;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) stage[(i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh) * 32 + li] = acc[i][j][r];
}
// ... or 16x16x32 MFMA tiles, four per 32x32 block (C/D map col = lane & 15, row = 4 (lane >> 4) + r)
template <int TM, int TN>
__device__ __forceinline__ void x6_stage_write(float* __restrict__ stage, const floatx4 (&acc)[2 * TM][2 * TN], int j,
                                               int lane) {
    const int l16 = lane & 15, lq = lane >> 4;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int si = 0; si < 2; ++si)
#pragma unroll
            for (int sj = 0; sj < 2; ++sj)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    stage[(i * 32 + si * 16 + 4 * lq + r) * 32 + sj * 16 + l16] = acc[2 * i + si][2 * j + sj][r];
}

template <int TM, int TN, int ABL = 0, bool C16 = false, typename Acc>
__device__ __forceinline__ void x6_epilogue(const GemmArgs& g, const Acc& acc, int64_t r0,
                                            int64_t c0, int64_t n0, int ks, int lane, float ia, float ib,
                                            float* __restrict__ stage) {
    const bool split = g.split > 1;
    float* __restrict__ dst = split ? g.ws + (int64_t)ks * g.M * g.N
                                    : const_cast<float*>(plane_base(g.C, n0, g.c_blk, g.c_pstride));
    // bf16 C: element (row, col) at (uint16_t*)C + row * ldc + col
    auto c16_at = [&](int64_t row, int64_t col) -> float* {
        return reinterpret_cast<float*>(reinterpret_cast<uint16_t*>(g.C) + row * g.ldc + col);
    };
    const int64_t ldd = split ? g.N : g.ldc;
    const bool vec = (((uintptr_t)dst & 15) == 0) && (ldd % 4 == 0);
    const bool bias_vec = g.bias && (((uintptr_t)g.bias & 15) == 0);
    const int rq = lane >> 3, c4 = (lane & 7) * 4;
    uint32_t cmax = 0;
    // interior tile, no split-K, aligned: per-column-block bias and pointer, per-row pointer
    // increments only (the general path below recomputes everything per float4); the same
    // arithmetic in the same order as the general path (beta C accumulation included: the
    // dgrad adds the skip connection's gradient that way)
    const bool gvec = (!g.ga0 || ((((uintptr_t)g.ga0 & 15) == 0) && g.ldg0 % 4 == 0)) &&
                      (!g.ga1 || ((((uintptr_t)g.ga1 & 15) == 0) && g.ldg1 % 4 == 0));
    const bool fast = !split && vec && gvec && (!g.bias || bias_vec) && r0 + TM * 32 <= g.M && c0 + TN * 32 <= g.N;
    const float iab = ia * ib;   // exact unless the two scales over/underflow together
    const bool one_mul = iab != 0.f && iab < 3.0e38f;
    // drop-add dgrad (ABL 8), interior tile: every bsrc float4 this lane adds is loaded before the
    // first staging pass, so the HBM latency overlaps the LDS staging and only the first 32-column
    // block waits for it (the main loop's staging registers are dead here: 16 float4 fit)
    // (up to 32 float4: larger tiles keep the per-row loads, their accumulators fill the VGPRs)
    constexpr bool kPre = ABL == 8 && !C16 && TN * TM * 4 <= 32;
    float4 gpre[kPre ? TN : 1][kPre ? TM * 4 : 1];
    if constexpr (kPre) {
        if (fast && g.beta != 0.f) {
#pragma unroll
            for (int j = 0; j < TN; ++j)
#pragma unroll
                for (int q = 0; q < TM * 4; ++q)
                    gpre[j][q] = *reinterpret_cast<const float4*>(g.bsrc + (r0 + q * 8 + rq) * g.ld_bsrc + c0 + j * 32 +
                                                                  c4 - g.bsrc_c0);
        }
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        x6_stage_write<TM, TN>(stage, acc, j, lane);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (fast) {
            const int64_t col = c0 + j * 32 + c4;
            float4 bv = make_float4(0.f, 0.f, 0.f, 0.f);
            if (g.bias) bv = *reinterpret_cast<const float4*>(g.bias + col);
            float* p = dst + (r0 + rq) * ldd + col;
            const int64_t step = 8 * ldd;
#pragma unroll
            for (int q = 0; q < TM * 4; ++q, p += step) {
                const float4 sv = *reinterpret_cast<const float4*>(stage + (q * 8 + rq) * 32 + c4);
                float e[4] = {sv.x, sv.y, sv.z, sv.w};
                const float b4[4] = {bv.x, bv.y, bv.z, bv.w};
                float4 a0 = make_float4(0.f, 0.f, 0.f, 0.f), a1 = a0;
                if (g.ga0) {
                    const int64_t row = r0 + q * 8 + rq;
                    a0 = *reinterpret_cast<const float4*>(g.ga0 + g.gi0[row] * g.ldg0 + col);
                    if (g.ga1) a1 = *reinterpret_cast<const float4*>(g.ga1 + g.gi1[row] * g.ldg1 + col);
                }
                const float x0[4] = {a0.x, a0.y, a0.z, a0.w}, x1[4] = {a1.x, a1.y, a1.z, a1.w};
                float pv[4] = {0.f, 0.f, 0.f, 0.f};
                if (g.beta != 0.f) {
                    if constexpr (kPre) {   // beta operand = masked bsrc (bgnn_gemm_f32_dropadd)
                        beta_mask4(g, r0 + q * 8 + rq, col, gpre[j][q], pv);
                    } else if constexpr (ABL == 8) {
                        beta_src4(g, r0 + q * 8 + rq, col, pv);
                    } else {
                        const float4 c4 = *reinterpret_cast<const float4*>(p);
                        pv[0] = c4.x; pv[1] = c4.y; pv[2] = c4.z; pv[3] = c4.w;
                    }
                }
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    float v = one_mul ? e[k] * iab : (e[k] * ia) * ib;
                    v *= g.alpha;
                    if (g.beta != 0.f) v += g.beta * pv[k];
                    if (g.bias) v += b4[k];
                    if (g.ga0) v += x0[k];
                    if (g.ga1) v += x1[k];
                    if (g.relu) v = fmaxf(v, 0.f);
                    e[k] = v;
                    cmax = max(cmax, __float_as_uint(v) & 0x7fffffffu);
                }
                if constexpr (C16) {
                    st_bf16x4(c16_at(r0 + q * 8 + rq, col), e);
                } else {
                    st_nt4(p, e);
                }
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            continue;
        }
        const int64_t col = c0 + j * 32 + c4;
#pragma unroll
        for (int q = 0; q < TM * 4; ++q) {
            const int rr = q * 8 + rq;
            const float4 sv = *reinterpret_cast<const float4*>(stage + rr * 32 + c4);
            const int64_t row = r0 + rr;
            float e[4] = {(sv.x * ia) * ib, (sv.y * ia) * ib, (sv.z * ia) * ib, (sv.w * ia) * ib};
            if (row >= g.M || col >= g.N) continue;
            float* p = dst + row * ldd + col;
            const bool full = vec && col + 3 < g.N;
            if (!split) {
                float prev[4] = {0.f, 0.f, 0.f, 0.f}, bv[4] = {0.f, 0.f, 0.f, 0.f};
                if (g.beta != 0.f) {
                    if constexpr (ABL == 8) {   // (the host requires N % 4 == 0: every float4 is whole)
                        beta_src4(g, row, col, prev);
                    } else if (full) {
                        const float4 t = *reinterpret_cast<const float4*>(p);
                        prev[0] = t.x; prev[1] = t.y; prev[2] = t.z; prev[3] = t.w;
                    } else {
#pragma unroll
                        for (int k = 0; k < 4; ++k) prev[k] = col + k < g.N ? p[k] : 0.f;
                    }
                }
                if (g.bias) {
                    if (bias_vec && col + 3 < g.N) {
                        const float4 t = *reinterpret_cast<const float4*>(g.bias + col);
                        bv[0] = t.x; bv[1] = t.y; bv[2] = t.z; bv[3] = t.w;
                    } else {
#pragma unroll
                        for (int k = 0; k < 4; ++k) bv[k] = col + k < g.N ? g.bias[col + k] : 0.f;
                    }
                }
                float x0[4] = {0.f, 0.f, 0.f, 0.f}, x1[4] = {0.f, 0.f, 0.f, 0.f};
                if (g.ga0) {
                    const float* s0 = g.ga0 + g.gi0[row] * g.ldg0 + col;
                    const float* s1 = g.ga1 ? g.ga1 + g.gi1[row] * g.ldg1 + col : nullptr;
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        x0[k] = col + k < g.N ? s0[k] : 0.f;
                        x1[k] = (s1 && col + k < g.N) ? s1[k] : 0.f;
                    }
                }
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    float v = e[k] * g.alpha;
                    if (g.beta != 0.f) v += g.beta * prev[k];
                    if (g.bias) v += bv[k];
                    if (g.ga0) v += x0[k];
                    if (g.ga1) v += x1[k];
                    if (g.relu) v = fmaxf(v, 0.f);
                    e[k] = v;
                    if (col + k < g.N) cmax = max(cmax, __float_as_uint(v) & 0x7fffffffu);
                }
            }
            if constexpr (C16) {
                if (full && !split) {
                    st_bf16x4(c16_at(row, col), e);
                } else {
                    uint16_t* p16 = reinterpret_cast<uint16_t*>(c16_at(row, col));
#pragma unroll
                    for (int k = 0; k < 4; ++k)
                        if (col + k < g.N) p16[k] = (uint16_t)(pack_bf16(e[k], 0.f) & 0xffffu);
                }
            } else if (full) {
                st_nt4(p, e);
            } else {
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    if (col + k < g.N) p[k] = e[k];
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    if (g.c_amax && !split) {
        for (int o = 32; o > 0; o >>= 1) cmax = max(cmax, (uint32_t)__shfl_xor((int)cmax, o, kWave));
        if (lane == 0 && cmax) atomicMax(reinterpret_cast<uint32_t*>(g.c_amax), cmax);
    }
}

}  // namespace bgnn
