// bf16 GEMM on bf16-STORED operands (round 3): C = act(A B^T + bias (+ gathered rows)) with
// A [M, K] and B [N, K] both bf16, K contiguous -- the per-edge Linears of EA_GNN's bf16
// configuration (Models/BuckGNN.py:528-566 through bgnn/ea.py and fused.linear_bf16, BASELINE
// configs[4]): edge_mlp / node_mlp_phi forward (A = the bf16 edge activations, B = the weight
// rounded to bf16 once) and their input gradients (A = the bf16 output gradient, B = W^T).
//
// Arithmetic: identical to k_gemm_x6<PREC 2> bit for bit -- the same bf16 operand values (stored
// bf16 = the round-to-nearest-even x6_store applies in-tile), one v_mfma_f32_32x32x16_bf16 per
// 32x32x16 block, k16 steps in increasing k, the same x6_epilogue (bias, gathered rows, ReLU,
// bf16 or f32 C) -- so every test of the x6 storage path holds for this kernel unchanged.
//
// Why a second kernel: x6 stages operands through registers (load, widen, round, ds_write) at
// prefetch distance 1, built for the f32-accurate split; with the operands already bf16 there is
// nothing to convert, and at E = 2.86M rows the x6 form ran at ~370 TF/s (4.57 ms per edge GEMM,
// 46 % of the cfg5 step). Here operand bytes go HBM -> LDS by global_load_lds_dwordx4 alone (no
// VGPRs, no VALU), BK = 64 k per slice so every row segment is one whole 128-B line, NS slots in
// flight, one raw barrier per slice (gemm_p16.hip's pipeline with one product instead of three).
// LDS image per slice: [A rows (BM) | B rows (BN)] x BK/8 16-B chunks, chunk c of row r at
// physical chunk c ^ ((r / RPQ) mod CPR) so the 16 lanes of a ds_read_b128 group hit 16 distinct
// bank slots; glds writes lane-linearly, so the swizzle goes on the per-lane source address.
#include "common.h"
#include "gemm_common.h"
#include "gemm_x6.h"

namespace bgnn {

namespace {

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void gbl_void_t;

template <int N>
__device__ __forceinline__ void b16_wait_vmcnt() {
    static_assert(N >= 0 && N < 64, "vmcnt field is 6 bits");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// raw barrier: no vmcnt(0) drain of the glds in flight (__syncthreads() would emit one)
__device__ __forceinline__ void b16_barrier() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

template <int BK>
struct B16Slice {
    static constexpr int CPR = BK / 8;     // 16-B chunks (8 k) per row
    static constexpr int RPQ = 16 / CPR;   // rows per 256-B bank row
    static constexpr int RPI = 64 / CPR;   // rows per glds instruction (64 lanes x 16 B)
    static constexpr int H = BK / 16;      // k16 MFMA steps per slice
    __device__ static int swz(int row) { return (row / RPQ) % CPR; }
    __device__ static int at(int row, int c) { return row * CPR + (c ^ swz(row)); }
};

// the H k16 steps of one landed slice; S restrict-scoped so hipcc does not drain the glds in
// flight (vmcnt(0)) before these LDS reads (see gemm_p16.hip, p16_mma)
template <int BM, int BN, int BK, int WM, int WN>
__device__ __forceinline__ void b16_mma(const uint4* __restrict__ S, floatx16 (&acc)[BM / WM / 32][BN / WN / 32],
                                        int wm, int wn, int lane) {
    using L = B16Slice<BK>;
    constexpr int TM = BM / WM / 32, TN = BN / WN / 32;
    const int li = lane & 31, lh = lane >> 5;
#pragma unroll
    for (int h = 0; h < L::H; ++h) {
        const int kg = 2 * h + lh;
        uint4 a[TM], b[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) a[i] = S[L::at(wm * (BM / WM) + i * 32 + li, kg)];
#pragma unroll
        for (int j = 0; j < TN; ++j) b[j] = S[L::at(BM + wn * (BN / WN) + j * 32 + li, kg)];
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(a[i]), as_bf16x8(b[j]), acc[i][j], 0, 0, 0);
    }
}

// The same slice on 16x16x32 MFMAs (round 5: the chip holds a higher clock under them; the
// k_gemm_x6 bf16 kernels use them too, so both give the same bits): per k32 step the fragments of
// 16 rows (lane & 15) x 8 k (chunk 4 s + (lane >> 4)); the side with fewer 16-row blocks is held,
// the other streamed. The swizzle keeps these reads conflict-free (lane groups of ds_read_b128).
template <int BM, int BN, int BK, int WM, int WN>
__device__ __forceinline__ void b16_mma(const uint4* __restrict__ S, floatx4 (&acc)[2 * (BM / WM / 32)][2 * (BN / WN / 32)],
                                        int wm, int wn, int lane) {
    using L = B16Slice<BK>;
    constexpr int TM = BM / WM / 32, TN = BN / WN / 32;
    const int l16 = lane & 15, lq = lane >> 4;
#pragma unroll
    for (int st = 0; st < BK / 32; ++st) {
        const int kg = 4 * st + lq;
        if constexpr (TM <= TN) {
            uint4 a[2 * TM];
#pragma unroll
            for (int i = 0; i < 2 * TM; ++i) a[i] = S[L::at(wm * (BM / WM) + i * 16 + l16, kg)];
#pragma unroll
            for (int j = 0; j < 2 * TN; ++j) {
                const uint4 b = S[L::at(BM + wn * (BN / WN) + j * 16 + l16, kg)];
#pragma unroll
                for (int i = 0; i < 2 * TM; ++i)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(a[i]), as_bf16x8(b), acc[i][j], 0, 0, 0);
            }
        } else {
            uint4 b[2 * TN];
#pragma unroll
            for (int j = 0; j < 2 * TN; ++j) b[j] = S[L::at(BM + wn * (BN / WN) + j * 16 + l16, kg)];
#pragma unroll
            for (int i = 0; i < 2 * TM; ++i) {
                const uint4 a = S[L::at(wm * (BM / WM) + i * 16 + l16, kg)];
#pragma unroll
                for (int j = 0; j < 2 * TN; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(a), as_bf16x8(b[j]), acc[i][j], 0, 0, 0);
            }
        }
    }
}

// accumulator helpers for either MFMA shape: zero; the 32x32 block (i, j) into an LDS stage (rows
// row0.., columns coff.., row stride ld) with the C/D map of the MFMA; one probe value
template <int TM, int TN>
__device__ __forceinline__ void b16_acc_zero(floatx16 (&acc)[TM][TN]) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
}
template <int TM2, int TN2>
__device__ __forceinline__ void b16_acc_zero(floatx4 (&acc)[TM2][TN2]) {
#pragma unroll
    for (int i = 0; i < TM2; ++i)
#pragma unroll
        for (int j = 0; j < TN2; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
}
template <int TM, int TN>
__device__ __forceinline__ void b16_stage_block(float* __restrict__ stage, int ld, int coff, int row0,
                                                const floatx16 (&acc)[TM][TN], int i, int j, int lane) {
    const int li = lane & 31, lh = lane >> 5;
#pragma unroll
    for (int r = 0; r < 16; ++r) stage[(row0 + (r & 3) + 8 * (r >> 2) + 4 * lh) * ld + coff + li] = acc[i][j][r];
}
template <int TM2, int TN2>
__device__ __forceinline__ void b16_stage_block(float* __restrict__ stage, int ld, int coff, int row0,
                                                const floatx4 (&acc)[TM2][TN2], int i, int j, int lane) {
    const int l16 = lane & 15, lq = lane >> 4;
#pragma unroll
    for (int si = 0; si < 2; ++si)
#pragma unroll
        for (int sj = 0; sj < 2; ++sj)
#pragma unroll
            for (int r = 0; r < 4; ++r)
                stage[(row0 + si * 16 + 4 * lq + r) * ld + coff + sj * 16 + l16] = acc[2 * i + si][2 * j + sj][r];
}

// Epilogue (alpha 1, beta 0, no split-K): per 32-column block, the wave's TM x 32 x 32
// accumulators go through its LDS stage (x6_epilogue's C/D map and stage layout) and leave as
// 16-B non-temporal row stores -- f32 C: 4 columns per lane (8 lanes per 128-B row segment), bf16
// C: 8 columns per lane (4 lanes per 64-B row segment; x6_epilogue stores 8 B). Per element the
// arithmetic and its order are x6_epilogue's: acc, + bias, + ga0[gi0[row]], + ga1[gi1[row]],
// ReLU, one bf16 rounding (RNE). Edge blocks fall back to x6_epilogue's element-guarded path.
template <int TM, int TN, bool C16, bool WIDE = false, typename Acc>
__device__ __forceinline__ void b16_epilogue(const GemmArgs& g, const Acc& acc, int64_t r0,
                                             int64_t c0, int lane, float* __restrict__ stage,
                                             const int64_t* __restrict__ li0 = nullptr,
                                             const int64_t* __restrict__ li1 = nullptr) {
    constexpr int CPL = C16 ? 8 : 4;        // columns per lane
    constexpr int LPR = 32 / CPL;           // lanes per 32-column row segment
    constexpr int RPP = 64 / LPR;           // rows per pass

    const int rq = lane / LPR, cq = (lane % LPR) * CPL;
    const bool gvec = (!g.ga0 || ((((uintptr_t)g.ga0 & 15) == 0) && g.ldg0 % 4 == 0)) &&
                      (!g.ga1 || ((((uintptr_t)g.ga1 & 15) == 0) && g.ldg1 % 4 == 0));
    const bool fast_cols = gvec && (((uintptr_t)g.C & 15) == 0) && g.ldc % 8 == 0 &&
                           (!g.bias || (((uintptr_t)g.bias & 15) == 0)) && c0 + TN * 32 <= g.N;
    const bool fast = fast_cols && r0 + TM * 32 <= g.M;
    if constexpr (C16 && TN % 2 == 0 && WIDE) {
      if (fast_cols) {   // rows past M (the last row tile) are skipped row by row
        // bf16 C in whole 128-B lines: two adjacent 32-column blocks (64 bf16 columns) of 32 rows
        // staged together ([32][68] f32: the row pad keeps the two half-waves' ds_write_b32 rows
        // on different banks), then 8 lanes x 16 B per row -- a 32-column block alone is a 64-B
        // half line per row, and half-line non-temporal stores cost the HBM side about twice
        // (tools/bf16_storage_ab.py: epilogue 835 of 2161 us at E = 2.86M). Same per-element
        // arithmetic and order as below.
        constexpr int LDW = 68;
        const int rq8 = lane >> 3, cq8 = (lane & 7) * 8;
#pragma unroll
        for (int j = 0; j < TN; j += 2) {
            const int64_t col = c0 + j * 32 + cq8;
            float bv[8];
#pragma unroll
            for (int k = 0; k < 8; k += 4) {
                const float4 t = g.bias ? *reinterpret_cast<const float4*>(g.bias + col + k) : make_float4(0.f, 0.f, 0.f, 0.f);
                bv[k] = t.x; bv[k + 1] = t.y; bv[k + 2] = t.z; bv[k + 3] = t.w;
            }
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                // drop-add source rows of this 32-row block issued before the staging, so their
                // latency runs under the LDS writes and waits
                // (the gathered ga0 rows loaded the same way ran slower: 2776 -> 3003 us at E = 2.86M,
                // their 32 VGPRs beside the 128 accumulator registers; round 5, measured, removed)
                uint4 spre[4];
                if (g.st & 8) {
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const int64_t row = r0 + i * 32 + q * 8 + rq8;
                        spre[q] = row < g.M ? *reinterpret_cast<const uint4*>(reinterpret_cast<const uint16_t*>(g.bsrc) +
                                                                             row * g.ld_bsrc + col)
                                            : make_uint4(0u, 0u, 0u, 0u);
                    }
                }
#pragma unroll
                for (int h = 0; h < 2; ++h) b16_stage_block(stage, LDW, h * 32, 0, acc, i, j + h, lane);
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int rr = q * 8 + rq8;
                    const int64_t row = r0 + i * 32 + rr;
                    if (row >= g.M) continue;
                    float e[8], x0[8], x1[8];
#pragma unroll
                    for (int k = 0; k < 8; k += 4) {
                        const float4 sv = *reinterpret_cast<const float4*>(stage + rr * LDW + cq8 + k);
                        e[k] = sv.x; e[k + 1] = sv.y; e[k + 2] = sv.z; e[k + 3] = sv.w;
                    }
                    if (g.ga0) {
                        // the gather rows' indices from the tile's LDS copy when the kernel made one
                        const float* s0 = g.ga0 + (li0 ? li0[i * 32 + rr] : g.gi0[row]) * g.ldg0 + col;
#pragma unroll
                        for (int k = 0; k < 8; k += 4) {
                            const float4 t = *reinterpret_cast<const float4*>(s0 + k);
                            x0[k] = t.x; x0[k + 1] = t.y; x0[k + 2] = t.z; x0[k + 3] = t.w;
                        }
                        if (g.ga1) {
                            const float* s1 = g.ga1 + (li1 ? li1[i * 32 + rr] : g.gi1[row]) * g.ldg1 + col;
#pragma unroll
                            for (int k = 0; k < 8; k += 4) {
                                const float4 t = *reinterpret_cast<const float4*>(s1 + k);
                                x1[k] = t.x; x1[k + 1] = t.y; x1[k + 2] = t.z; x1[k + 3] = t.w;
                            }
                        }
                    }
#pragma unroll
                    for (int k = 0; k < 8; ++k) {
                        float v = e[k];
                        if (g.bias) v += bv[k];
                        if (g.ga0) v += x0[k];
                        if (g.ga1) v += x1[k];
                        if (g.relu) v = fmaxf(v, 0.f);
                        e[k] = v;
                    }
                    if (g.st & 8) {
                        // drop-add (bgnn_gemm_bf16_dropadd): the bf16 value this epilogue would store,
                        // + drop(src) in f32, one more rounding -- bgnn_add_dropped_bf16 on the stored C,
                        // bit for bit (mask group (row * ld + col) / 4, kept values * dkeep)
                        const int64_t si = row * g.ld_bsrc + col;
                        const uint4 sv = spre[q];
                        const uint32_t sw[4] = {sv.x, sv.y, sv.z, sv.w};
                        float d[8];
#pragma unroll
                        for (int h = 0; h < 4; ++h) {
                            d[2 * h] = __uint_as_float(sw[h] << 16);
                            d[2 * h + 1] = __uint_as_float(sw[h] & 0xffff0000u);
                        }
                        if (g.dthr) {
#pragma unroll
                            for (int h = 0; h < 2; ++h) {
                                const uint32_t keep = keep_bits4(g.dseed, (uint64_t)(si >> 2) + h, g.dthr);
#pragma unroll
                                for (int k = 0; k < 4; ++k) d[4 * h + k] = ((keep >> k) & 1u) ? d[4 * h + k] * g.dkeep : 0.f;
                            }
                        }
#pragma unroll
                        for (int k = 0; k < 8; ++k) e[k] = __uint_as_float(pack_bf16(e[k], 0.f) << 16) + d[k];
                    }
                    typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
                    const u32x4_t w = {pack_bf16(e[0], e[1]), pack_bf16(e[2], e[3]), pack_bf16(e[4], e[5]),
                                       pack_bf16(e[6], e[7])};
                    __builtin_nontemporal_store(w, reinterpret_cast<u32x4_t*>(reinterpret_cast<uint16_t*>(g.C) +
                                                                              row * g.ldc + col));
                }
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            }
        }
        return;
      }
    }
    if (!fast) {
        x6_epilogue<TM, TN, 0, C16>(g, acc, r0, c0, c0, 0, lane, 1.f, 1.f, stage);
        return;
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
#pragma unroll
        for (int i = 0; i < TM; ++i) b16_stage_block(stage, 32, 0, i * 32, acc, i, j, lane);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        const int64_t col = c0 + j * 32 + cq;
        float bv[CPL];
#pragma unroll
        for (int k = 0; k < CPL; k += 4) {
            const float4 t = g.bias ? *reinterpret_cast<const float4*>(g.bias + col + k) : make_float4(0.f, 0.f, 0.f, 0.f);
            bv[k] = t.x; bv[k + 1] = t.y; bv[k + 2] = t.z; bv[k + 3] = t.w;
        }
#pragma unroll 2
        for (int q = 0; q < TM * 32 / RPP; ++q) {
            const int rr = q * RPP + rq;
            const int64_t row = r0 + rr;
            float e[CPL], x0[CPL], x1[CPL];
#pragma unroll
            for (int k = 0; k < CPL; k += 4) {
                const float4 sv = *reinterpret_cast<const float4*>(stage + rr * 32 + cq + k);
                e[k] = sv.x; e[k + 1] = sv.y; e[k + 2] = sv.z; e[k + 3] = sv.w;
            }
            if (g.ga0) {
                const float* s0 = g.ga0 + g.gi0[row] * g.ldg0 + col;
#pragma unroll
                for (int k = 0; k < CPL; k += 4) {
                    const float4 t = *reinterpret_cast<const float4*>(s0 + k);
                    x0[k] = t.x; x0[k + 1] = t.y; x0[k + 2] = t.z; x0[k + 3] = t.w;
                }
                if (g.ga1) {
                    const float* s1 = g.ga1 + g.gi1[row] * g.ldg1 + col;
#pragma unroll
                    for (int k = 0; k < CPL; k += 4) {
                        const float4 t = *reinterpret_cast<const float4*>(s1 + k);
                        x1[k] = t.x; x1[k + 1] = t.y; x1[k + 2] = t.z; x1[k + 3] = t.w;
                    }
                }
            }
#pragma unroll
            for (int k = 0; k < CPL; ++k) {
                float v = e[k];
                if (g.bias) v += bv[k];
                if (g.ga0) v += x0[k];
                if (g.ga1) v += x1[k];
                if (g.relu) v = fmaxf(v, 0.f);
                e[k] = v;
            }
            if constexpr (C16) {
                typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
                const u32x4_t w = {pack_bf16(e[0], e[1]), pack_bf16(e[2], e[3]), pack_bf16(e[4], e[5]),
                                   pack_bf16(e[6], e[7])};
                __builtin_nontemporal_store(w, reinterpret_cast<u32x4_t*>(reinterpret_cast<uint16_t*>(g.C) +
                                                                          row * g.ldc + col));
            } else {
                st_nt4(g.C + row * g.ldc + col, e);
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
}

template <int BM, int BN, int BK, int NS, int WM, int WN, bool C16, int MINB = 1, bool WIDE = false>
__global__ __launch_bounds__(64 * WM * WN, MINB) void k_gemm_b16(GemmArgs g) {
    using L = B16Slice<BK>;
    constexpr int NW = WM * WN;
    constexpr int TM = BM / WM / 32, TN = BN / WN / 32;
    constexpr int GA = BM / (L::RPI * NW), GB = BN / (L::RPI * NW);   // glds per wave per slice
    constexpr int G = GA + GB;
    constexpr int SLICE_U4 = (BM + BN) * L::CPR;
    static_assert(GA * L::RPI * NW == BM && GB * L::RPI * NW == BN, "rows must split evenly over the waves");
    static_assert((NS - 2) * G < 64, "vmcnt range");
    // per-wave LDS stage (floats): TM 32-row blocks of 32 columns, or the whole-line bf16 form's
    // [32][68] pair of blocks, whichever is larger (TM = 2 tiles: the latter)
    constexpr int STG = (C16 && WIDE && TM * 32 * 32 < 32 * 68) ? 32 * 68 : TM * 32 * 32;
    constexpr int EPI_U4 = NW * STG / 4;
    constexpr int SMEM_U4 = NS * SLICE_U4 > EPI_U4 ? NS * SLICE_U4 : EPI_U4;
    // WIDE bf16 C with gathered rows: the tile's gi0 / gi1 (BM int64 each) copied to LDS by the
    // waves' first loads, so the epilogue's gather addresses wait on LDS instead of a dependent
    // global load per 32-row block (one row of 32 per wave: NW * 32 == BM)
    constexpr bool kIdx = WIDE && C16 && NW * 32 == BM;
    constexpr int IDX_U4 = kIdx ? BM : 0;
    static_assert((SMEM_U4 + IDX_U4) * 16 <= 160 * 1024, "LDS over 160 KiB");
    __shared__ uint4 smem[SMEM_U4 + IDX_U4];   // one array (a second __shared__ object costs a vmcnt(0) per slice)

    const int t = threadIdx.x;
    const int lane = t & 63;
    const int wave = t >> 6;
    const int wm = wave / WN, wn = wave % WN;
    const int64_t ntn = (g.N + BN - 1) / BN;
    // XCD-aware order: one XCD's workgroups take consecutive tiles = the column tiles of one row
    // block, so A's rows come from HBM into that XCD's L2 once
    const int lt = xcd_remap(blockIdx.x, gridDim.x);
    const int64_t tm = lt / ntn, tn = lt % ntn;
    const int64_t m0 = tm * BM, n0 = tn * BN;

    // per-lane glds sources: byte offsets from the tile's first A / B row (rows past the edge
    // re-read the last row; their results are never stored); wave-uniform LDS destinations
    const char* abase = reinterpret_cast<const char*>(g.A) + m0 * g.lda * 2;
    const char* bbase = reinterpret_cast<const char*>(g.B) + n0 * g.ldb * 2;
    uint32_t off[G];
    int dst[G];
#pragma unroll
    for (int q = 0; q < G; ++q) {
        const bool isa = q < GA;
        const int r0 = (isa ? wave * GA + q : wave * GB + (q - GA)) * L::RPI;
        int r = r0 + lane / L::CPR;
        const int c = (lane % L::CPR) ^ L::swz((isa ? 0 : BM) + r);
        const int64_t rmax = (isa ? g.M - m0 : g.N - n0) - 1;
        if (r > rmax) r = (int)rmax;
        off[q] = (uint32_t)((r * (isa ? g.lda : g.ldb) + 8 * c) * 2);
        dst[q] = ((isa ? 0 : BM) + r0) * L::CPR;
    }
    // the index copies go first: the slice waits' in-order vmcnt covers them
    const bool lidx = kIdx && g.ga0 != nullptr;
    if (lidx) {
        int64_t row = m0 + wave * 32 + (lane >> 1);
        if (row > g.M - 1) row = g.M - 1;
        uint4* dsti = smem + SMEM_U4 + wave * 16;   // 32 rows x 8 B per wave, lane l -> bytes 4 l
        __builtin_amdgcn_global_load_lds((gbl_void_t*)(reinterpret_cast<const char*>(g.gi0 + row) + (lane & 1) * 4),
                                         (lds_void_t*)dsti, 4, 0, 0);
        if (g.ga1)
            __builtin_amdgcn_global_load_lds((gbl_void_t*)(reinterpret_cast<const char*>(g.gi1 + row) + (lane & 1) * 4),
                                             (lds_void_t*)(dsti + BM / 2), 4, 0, 0);
    }
    const int64_t nm = g.K / BK;
    auto issue = [&](int64_t m) {
        if (m >= nm) return;
        const uint32_t kb = (uint32_t)(m * BK * 2);
        uint4* slot = smem + (int)(m % NS) * SLICE_U4;
#pragma unroll
        for (int q = 0; q < G; ++q)
            __builtin_amdgcn_global_load_lds((gbl_void_t*)((q < GA ? abase : bbase) + (off[q] + kb)),
                                             (lds_void_t*)(slot + dst[q]), 16, 0, 0);
    };

    floatx4 acc[2 * TM][2 * TN];   // 16x16x32 MFMA tiles (b16_mma)
    b16_acc_zero(acc);

    // slice m lives in slot m % NS: wait for this wave's part of slice m (the NS - 2 newer
    // slices stay in flight), one barrier (every wave's part landed, every wave done with slice
    // m - 1, whose slot slice m + NS - 1 now refills), issue m + NS - 1, multiply slice m
    for (int m = 0; m < NS - 1; ++m) issue(m);
    for (int64_t m = 0; m < nm; ++m) {
        if (m + NS - 2 < nm) b16_wait_vmcnt<(NS - 2) * G>();
        else b16_wait_vmcnt<0>();
        b16_barrier();
        issue(m + NS - 1);
        b16_mma<BM, BN, BK, WM, WN>(smem + (int)(m % NS) * SLICE_U4, acc, wm, wn, lane);
    }
    __syncthreads();   // every wave's fragment reads done before the epilogue reuses the LDS
    float* stage = reinterpret_cast<float*>(smem) + wave * STG;
    const int64_t* li = reinterpret_cast<const int64_t*>(smem + SMEM_U4) + wm * (BM / WM);
    b16_epilogue<TM, TN, C16, WIDE>(g, acc, m0 + wm * (BM / WM), n0 + wn * (BN / WN), lane, stage,
                                    lidx ? li : nullptr, lidx && g.ga1 ? li + BM : nullptr);
}

int g_b16_variant = 0;   // 0 = the LDS-DMA kernel (default), -1 = bf16-stored NT products on k_gemm_x6 (A/B)
// (round 6 measured a 128 x 256 form with two workgroups per CU, k32 x 3 slots, so that one's
// epilogue runs under the other's main loop: plain 2015 -> 2351 us, gathered 3635 -> 3606, drop-add
// 2841 -> 2881 at E = 2.86M, profiles/r06_b16_two_per_cu_v.txt; removed. Its stage sizing stays:
// the whole-line bf16 stage [32][68] is larger than TM = 2 blocks of 32 x 32.)

}  // namespace

bool b16_ok(const GemmArgs& g, int ta, int tb) {
    constexpr int64_t kMaxTileBytes = int64_t(1) << 31;
    return g_b16_variant >= 0 && ta == 0 && tb == 1 && (g.st & 3) == 3 && g.split <= 1 && g.K > 0 && g.K % 64 == 0 &&
           g.a_blk == 0 && g.c_blk == 0 && (g.bsrc == nullptr || (g.st & 8)) && g.lda % 8 == 0 && g.ldb % 8 == 0 &&
           aligned16(g.A) && aligned16(g.B) && 256 * g.lda * 2 < kMaxTileBytes && 256 * g.ldb * 2 < kMaxTileBytes;
}

// One form: 256x256 tiles, one per workgroup, k64 slices (whole 128-B row segments) x 2 slots,
// whole-line bf16 C stores, the gathered rows' indices staged in LDS. At E = 2,863,488 x 512 x 512
// (cfg5, tools/bf16_storage_ab.py, same box, medians) bf16 C 1985 us against 2145 with half-line
// stores and 2200 in the persistent form; gathered bf16 C 3620 against 3700 persistent. (ABI 12
// removed the measured-and-rejected forms: persistent tiles, k32 slices with 3-4 slots, 128-row
// tiles, per-row global gather indices, prefetched gather rows, the epilogue-free ablations;
// records in profiles/r0[2-5]_*.)
bool b16_dropadd_ok(const GemmArgs& g) {
    return (g.st & 7) == 7 && g.N % 256 == 0 && g.ldc % 8 == 0 && g.ld_bsrc % 8 == 0 && aligned16(g.C) &&
           aligned16(g.bsrc);
}

void launch_b16(hipStream_t s, const GemmArgs& g) {
    const dim3 grid((unsigned)(((g.M + 255) / 256) * ((g.N + 255) / 256)));
    if (g.st & 4) hipLaunchKernelGGL((k_gemm_b16<256, 256, 64, 2, 2, 4, true, 1, true>), grid, dim3(512), 0, s, g);
    else hipLaunchKernelGGL((k_gemm_b16<256, 256, 64, 2, 2, 4, false, 1, true>), grid, dim3(512), 0, s, g);
}

}  // namespace bgnn

extern "C" int bgnn_gemm_b16_variant(int32_t variant) {
    BGNN_REQUIRE(variant == -1 || variant == 0, "gemm_b16_variant: must be -1 (off) or 0 (the LDS-DMA kernel)");
    bgnn::g_b16_variant = variant;
    return BGNN_OK;
}
