// f16x3 GEMM on PRE-SPLIT operands (round 3): C = A B^T with A [M, K] and B [N, K] given as
// their two f16 pieces (the split of gemm_x6.hip's PREC 1, done once by the producer or by
// bgnn_split_f16x2 instead of inside every tile that reads the operand). The SAGE GEMMs this
// serves (Models/BuckGNN.py:135-149 through bgnn/fused.py): the forward z = x [W_l;W_r]^T and
// the dgrad dx = dz [W_l;W_r] (B = [W_l;W_r]^T), both K-contiguous.
//
// Arithmetic: identical to k_gemm_x6<PREC 1>, bit for bit -- each operand element x is stored
// as hi = f16(x s), lo = f16(x s - hi) with the power-of-two s = h3_scale(max|x|), and every
// 32x32x16 block product is the three f16 MFMAs a_hi.b_lo, a_lo.b_hi, a_hi.b_hi in that order,
// k16 steps in order, unscaled in the same epilogue (x6_epilogue).
//
// Staging: nothing to split, so operand bytes go HBM -> LDS by global_load_lds_dwordx4 alone
// (no VGPRs, no VALU), NS slices in flight, one raw barrier per slice. Piece layout
// ("k8-interleaved"): row r holds, for every group of 8 consecutive k, the 16-B hi piece then
// the 16-B lo piece ([rows][K/8][2][8] f16, row stride ld >= 2K elements), so one slice of one
// row (BKH k, both pieces) is ONE contiguous 4 BKH-byte segment: a k32 slice reads whole 128-B
// lines (separate hi / lo planes made every glds instruction touch 32 partial lines: 4x the L2
// requests, measured 2x slower). LDS image per slice: [A rows (BM) | B rows (BN)] x the same
// 4 BKH bytes per row, in 16-B chunks swizzled by (row / RPQ) mod CPR so the 16 lanes of a
// ds_read_b128 group hit 16 distinct bank slots; glds writes lane-linearly, so the swizzle
// goes on the per-lane global source address (a permutation inside the row's segment).
#include "common.h"
#include "gemm_common.h"
#include "gemm_x6.h"

namespace bgnn {

namespace {

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void gbl_void_t;

template <int N>
__device__ __forceinline__ void p16_wait_vmcnt() {
    static_assert(N >= 0 && N < 64, "vmcnt field is 6 bits");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// raw barrier: no vmcnt(0) drain of the glds in flight (__syncthreads() would emit one)
__device__ __forceinline__ void p16_barrier() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

template <int BKH>
struct P16Slice {
    static constexpr int CPR = BKH / 4;     // 16-B chunks per row: (hi, lo) per k8 group, logical chunk 2 kg + piece
    static constexpr int RPQ = 16 / CPR;    // rows per 256-B bank row
    static constexpr int RPI = 64 / CPR;    // rows per glds instruction (64 lanes x 16 B)
    static constexpr int H = BKH / 16;      // k16 MFMA steps per slice
    __device__ static int swz(int row) { return (row / RPQ) % CPR; }
    // uint4 index of logical chunk c of row `row`
    __device__ static int at(int row, int c) { return row * CPR + (c ^ swz(row)); }
};

// split an f32 matrix into its two f16 pieces (the same rounding as x6_store / split2h), written
// k8-interleaved: thread = one group of 8 consecutive columns of one row -> 16-B hi, 16-B lo
__global__ __launch_bounds__(256) void k_split_f16x2(const float* __restrict__ x, int64_t rows, int64_t cols8,
                                                     int64_t ldx, const float* __restrict__ amax,
                                                     uint4* __restrict__ out, int64_t ldo16) {
    float s, inv;
    h3_scale(*amax, s, inv);
    const int64_t n = rows * cols8;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        const int64_t r = i / cols8, c = i % cols8;
        const float4 u = *reinterpret_cast<const float4*>(x + r * ldx + 8 * c);
        const float4 v = *reinterpret_cast<const float4*>(x + r * ldx + 8 * c + 4);
        uint4 h, l;
        split2h(u.x * s, u.y * s, h.x, l.x);
        split2h(u.z * s, u.w * s, h.y, l.y);
        split2h(v.x * s, v.y * s, h.z, l.z);
        split2h(v.z * s, v.w * s, h.w, l.w);
        out[r * ldo16 + 2 * c] = h;
        out[r * ldo16 + 2 * c + 1] = l;
    }
}

}  // namespace

// The H k16 MFMA steps of one landed slice: wave fragments (A rows wm BM/WM + 32 i + (lane & 31),
// B rows likewise, k group 2 h + (lane >> 5)) as one ds_read_b128 per piece; the two cross terms,
// then the leading product (k_gemm_x6's order). S is a restrict parameter so that, once inlined,
// its LDS reads carry alias-scope metadata: hipcc then does not wait vmcnt(0) for the glds in
// flight before them (SIInsertWaitcnts disambiguates LDS-DMA stores only against scoped accesses;
// the counted waits of the pipeline order them).
template <int BM, int BN, int BKH, int WM, int WN, int ABL>
__device__ __forceinline__ void p16_mma(const uint4* __restrict__ S, floatx16 (&acc)[BM / WM / 32][BN / WN / 32],
                                        int wm, int wn, int lane) {
    using L = P16Slice<BKH>;
    constexpr int TM = BM / WM / 32, TN = BN / WN / 32;
    const int li = lane & 31, lh = lane >> 5;
#pragma unroll
    for (int h = 0; h < L::H; ++h) {
        const int kg = 2 * h + lh;
        uint4 a[TM][2], b[TN][2];
#pragma unroll
        for (int i = 0; i < TM; ++i) {
            const int row = wm * (BM / WM) + i * 32 + li;
            a[i][0] = S[L::at(row, 2 * kg)];
            a[i][1] = S[L::at(row, 2 * kg + 1)];
        }
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int row = BM + wn * (BN / WN) + j * 32 + li;
            b[j][0] = S[L::at(row, 2 * kg)];
            b[j][1] = S[L::at(row, 2 * kg + 1)];
        }
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                floatx16 tt = acc[i][j];
                if constexpr (ABL == 3) {   // ablation: no MFMAs (fragments still read)
                    tt[0] += __uint_as_float(a[i][0].x ^ a[i][1].y ^ b[j][0].z ^ b[j][1].w);
                } else {
                    tt = __builtin_amdgcn_mfma_f32_32x32x16_f16(as_f16x8(a[i][0]), as_f16x8(b[j][1]), tt, 0, 0, 0);
                    tt = __builtin_amdgcn_mfma_f32_32x32x16_f16(as_f16x8(a[i][1]), as_f16x8(b[j][0]), tt, 0, 0, 0);
                    tt = __builtin_amdgcn_mfma_f32_32x32x16_f16(as_f16x8(a[i][0]), as_f16x8(b[j][0]), tt, 0, 0, 0);
                }
                acc[i][j] = tt;
            }
    }
}

struct P16Args {
    GemmArgs g;                 // C / epilogue fields (A, B unused)
    const uint16_t* a;          // A pieces, k8-interleaved [M][K/8][2][8] (row stride g.lda elements)
    const uint16_t* b;          // B pieces [N][K/8][2][8] (row stride g.ldb)
};

template <int BM, int BN, int BKH, int NS, int WM, int WN, int ABL = 0>
__global__ __launch_bounds__(64 * WM * WN) void k_gemm_p16(P16Args P) {
    using L = P16Slice<BKH>;
    const GemmArgs& g = P.g;
    constexpr int NW = WM * WN, H = L::H;
    constexpr int TM = BM / WM / 32, TN = BN / WN / 32;
    constexpr int GA = BM / (L::RPI * NW), GB = BN / (L::RPI * NW);   // glds per wave per slice
    constexpr int G = GA + GB;
    constexpr int SLICE_U4 = (BM + BN) * L::CPR;
    static_assert(GA * L::RPI * NW == BM && GB * L::RPI * NW == BN, "rows must split evenly over the waves");
    static_assert((NS - 2) * G < 64, "vmcnt range");
    constexpr int EPI_U4 = NW * TM * 32 * 32 / 4;
    constexpr int SMEM_U4 = NS * SLICE_U4 > EPI_U4 ? NS * SLICE_U4 : EPI_U4;
    static_assert(SMEM_U4 * 16 <= 160 * 1024, "LDS over 160 KiB");
    // all LDS in one array (a second __shared__ object can make hipcc wait vmcnt(0) before
    // the first ds_read of every slice)
    __shared__ uint4 smem[SMEM_U4];

    const int t = threadIdx.x;
    const int lane = t & 63;
    const int wave = t >> 6;
    const int wm = wave / WN, wn = wave % WN;
    const int64_t ntn = (g.N + BN - 1) / BN;
    // XCD-aware order: one XCD's workgroups take consecutive tiles, i.e. the column tiles of
    // the same row block, so A's rows are fetched into that XCD's L2 once
    const int lt = xcd_remap(blockIdx.x, gridDim.x);
    const int64_t tm = lt / ntn, tn = lt % ntn;
    const int64_t m0 = tm * BM, n0 = tn * BN;

    float sa, sb, ia, ib;
    h3_scale(*g.a_amax, sa, ia);
    h3_scale(*g.b_amax, sb, ib);
    (void)sa;
    (void)sb;

    // per-lane glds sources: byte offsets from the operand's piece buffer at k = 0 (p16_ok bounds
    // them below 4 GiB: the loads take the uniform-base + VGPR-offset form); wave-uniform LDS rows
    uint32_t off[G];
    int dst[G];
#pragma unroll
    for (int q = 0; q < G; ++q) {
        const bool isa = q < GA;
        const int r0 = (isa ? wave * GA + q : wave * GB + (q - GA)) * L::RPI;
        const int r = r0 + lane / L::CPR;
        const int c = (lane % L::CPR) ^ L::swz((isa ? 0 : BM) + r);   // logical chunk this lane fetches
        const int64_t lim = isa ? g.M : g.N;
        int64_t gr = (isa ? m0 : n0) + r;
        if (gr > lim - 1) gr = lim - 1;   // rows past the edge re-read the last row (never stored)
        off[q] = (uint32_t)((gr * (isa ? g.lda : g.ldb) + 8 * c) * 2);
        dst[q] = ((isa ? 0 : BM) + r0) * L::CPR;
    }
    const int64_t nm = g.K / BKH;   // slices
    auto issue = [&](int64_t m) {
        if (m >= nm) return;
        const uint32_t kb = (uint32_t)(m * BKH * 4);   // BKH k x 2 pieces x 2 B
        uint4* slot = smem + (int)(m % NS) * SLICE_U4;
#pragma unroll
        for (int q = 0; q < G; ++q) {
            if (ABL == 2) break;
            const char* base = reinterpret_cast<const char*>(q < GA ? P.a : P.b);
            __builtin_amdgcn_global_load_lds((gbl_void_t*)(base + (off[q] + kb)), (lds_void_t*)(slot + dst[q]), 16, 0,
                                             0);
        }
    };

    floatx16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    // Slice m lives in slot m % NS. At slice m: wait until this wave's part of slice m has landed
    // (the NS - 2 newer slices it issued stay in flight; vmcnt(0) once fewer were issued), one
    // barrier (every wave's part landed, and every wave done reading slice m - 1, whose slot
    // slice m + NS - 1 now refills), issue slice m + NS - 1, multiply slice m's H k16 steps.
    for (int m = 0; m < NS - 1; ++m) issue(m);
    for (int64_t m = 0; m < nm; ++m) {
        if (ABL != 4) {
            if (m + NS - 2 < nm) p16_wait_vmcnt<(NS - 2) * G>();
            else p16_wait_vmcnt<0>();
        }
        p16_barrier();
        issue(m + NS - 1);
        if constexpr (ABL == 9) __builtin_amdgcn_s_setprio(1);
        p16_mma<BM, BN, BKH, WM, WN, ABL>(smem + (int)(m % NS) * SLICE_U4, acc, wm, wn, lane);
        if constexpr (ABL == 9) __builtin_amdgcn_s_setprio(0);
    }
    if constexpr (ABL == 15) {   // ablation: no epilogue (one value per wave keeps the MFMAs live)
        float t0 = 0.f;
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) t0 += acc[i][j][0] + acc[i][j][15];
        if (lane == 0) g.C[(m0 + wm * (BM / WM)) * g.ldc + n0 + wn * (BN / WN)] = t0;
        return;
    }
    if constexpr (ABL == 16) {   // measurement: C straight from the accumulators (no LDS staging,
        // no barrier): lane (li, lh) holds column c0 + 32 j + li of rows r0 + 32 i + (r & 3) + 8 (r >> 2) + 4 lh
        const int li = lane & 31, lh = lane >> 5;
        const int64_t r0 = m0 + wm * (BM / WM), c0 = n0 + wn * (BN / WN);
        const float iab = ia * ib;
        uint32_t cmax = 0;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int64_t col = c0 + 32 * j + li;
            const float bv = (g.bias && col < g.N) ? g.bias[col] : 0.f;
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int64_t row = r0 + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * lh;
                    float v = acc[i][j][r] * iab * g.alpha + bv;
                    if (g.relu) v = fmaxf(v, 0.f);
                    if (row < g.M && col < g.N) {
                        __builtin_nontemporal_store(v, g.C + row * g.ldc + col);
                        cmax = max(cmax, __float_as_uint(v) & 0x7fffffffu);
                    }
                }
        }
        if (g.c_amax) {
            for (int o = 32; o > 0; o >>= 1) cmax = max(cmax, (uint32_t)__shfl_xor((int)cmax, o, kWave));
            if (lane == 0 && cmax) atomicMax(reinterpret_cast<uint32_t*>(g.c_amax), cmax);
        }
        return;
    }
    __syncthreads();   // every wave's fragment reads done before the epilogue reuses the LDS
    float* stage = reinterpret_cast<float*>(smem) + wave * (TM * 32 * 32);
    x6_epilogue<TM, TN, ABL == 8 ? 8 : 0>(g, acc, m0 + wm * (BM / WM), n0 + wn * (BN / WN), n0, 0, lane, ia, ib,
                                          stage);
}

// Epilogue of one wave's TM x TN accumulator blocks for the persistent kernel: each 32x32 block
// goes through a wave-private 4 KiB LDS stage (separate from the operand slots, so the next
// tile's slices can be in flight meanwhile) and leaves as 16-B non-temporal row stores; the same
// per-element arithmetic, in the same order, as x6_epilogue's fast path (unscale, alpha, beta C or
// drop-add source, bias, ReLU, max|C|). Edge blocks store element-wise within bounds.
template <int TM, int TN, bool DROPADD, bool EXTRA>
__device__ __forceinline__ void p16p_epilogue(const GemmArgs& g, const floatx16 (&acc)[TM][TN], int64_t r0, int64_t c0,
                                              int lane, float ia, float ib, float* __restrict__ stage,
                                              uint32_t& cmax) {
    const int li = lane & 31, lh = lane >> 5;
    const int rq = lane >> 3, c4 = (lane & 7) * 4;
    const float iab = ia * ib;
    const bool one_mul = iab != 0.f && iab < 3.0e38f;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int64_t col = c0 + j * 32 + c4;
        float bv[4] = {0.f, 0.f, 0.f, 0.f};
        if (EXTRA && g.bias) {
#pragma unroll
            for (int k = 0; k < 4; ++k) bv[k] = col + k < g.N ? g.bias[col + k] : 0.f;
        }
#pragma unroll
        for (int i = 0; i < TM; ++i) {
#pragma unroll
            for (int r = 0; r < 16; ++r) stage[((r & 3) + 8 * (r >> 2) + 4 * lh) * 32 + li] = acc[i][j][r];
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            const bool full = r0 + i * 32 + 32 <= g.M && c0 + j * 32 + 32 <= g.N;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int rr = q * 8 + rq;
                const int64_t row = r0 + i * 32 + rr;
                const float4 sv = *reinterpret_cast<const float4*>(stage + rr * 32 + c4);
                float e[4] = {sv.x, sv.y, sv.z, sv.w};
                if (!full && row >= g.M) continue;
                float* p = g.C + row * g.ldc + col;
                float pv[4] = {0.f, 0.f, 0.f, 0.f};
                const bool has_beta = (DROPADD || EXTRA) && g.beta != 0.f;
                if (has_beta) {
                    if constexpr (DROPADD) {
                        beta_src4(g, row, col, pv);
                    } else {
#pragma unroll
                        for (int k = 0; k < 4; ++k) pv[k] = (full || col + k < g.N) ? p[k] : 0.f;
                    }
                }
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    float v = one_mul ? e[k] * iab : (e[k] * ia) * ib;
                    v *= g.alpha;
                    if (has_beta) v += g.beta * pv[k];
                    if (EXTRA && g.bias) v += bv[k];
                    if (g.relu) v = fmaxf(v, 0.f);
                    e[k] = v;
                    if (full || col + k < g.N) cmax = max(cmax, __float_as_uint(v) & 0x7fffffffu);
                }
                if (full) {
                    st_nt4(p, e);
                } else {
#pragma unroll
                    for (int k = 0; k < 4; ++k)
                        if (col + k < g.N) p[k] = e[k];
                }
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        }
    }
}

// Persistent form of k_gemm_p16 (round 3): one workgroup per CU walks its tiles (XCD-aware: at
// each step the workgroups of one XCD hold 32 consecutive tiles, i.e. whole row blocks, so A's
// rows are shared in that XCD's L2). The slice pipeline runs across tile boundaries -- the next
// tile's first slices are already in flight while this tile's epilogue stages and stores C --
// and the C stores drain under the next tile's MFMAs instead of every CU storing in lockstep at
// the end of each round of tiles (measured: the non-persistent fwd spends 84 of 294 us in its
// epilogue, tools/p16_ab.py v15).
// EXTRA: the epilogue reads bias / beta C; any epilogue global load waits (in-order vmcnt) for
// the next tile's glds issued before it, so then the next tile's first slice is issued after the
// epilogue instead (its latency shows once per tile, the stores still drain under the MFMAs).
template <int BM, int BN, int BKH, int NS, int WM, int WN, bool DROPADD, bool EXTRA>
__global__ __launch_bounds__(64 * WM * WN) void k_gemm_p16p(P16Args P) {
    constexpr bool kLoadFree = !DROPADD && !EXTRA;
    using L = P16Slice<BKH>;
    const GemmArgs& g = P.g;
    constexpr int NW = WM * WN;
    constexpr int TM = BM / WM / 32, TN = BN / WN / 32;
    constexpr int GA = BM / (L::RPI * NW), GB = BN / (L::RPI * NW);
    constexpr int G = GA + GB;
    constexpr int SLICE_U4 = (BM + BN) * L::CPR;
    constexpr int STAGE_U4 = NW * 32 * 32 / 4;   // one 32x32 f32 block per wave
    static_assert(GA * L::RPI * NW == BM && GB * L::RPI * NW == BN, "rows must split evenly over the waves");
    static_assert((NS - 2) * G < 64, "vmcnt range");
    static_assert((NS * SLICE_U4 + STAGE_U4) * 16 <= 160 * 1024, "LDS over 160 KiB");
    __shared__ uint4 smem[NS * SLICE_U4 + STAGE_U4];

    const int t = threadIdx.x;
    const int lane = t & 63;
    const int wave = t >> 6;
    const int wm = wave / WN, wn = wave % WN;
    const int64_t ntn = (g.N + BN - 1) / BN;
    const int64_t ntiles = ((g.M + BM - 1) / BM) * ntn;
    const int64_t first = xcd_remap(blockIdx.x, gridDim.x);
    const int64_t stride = gridDim.x;
    if (first >= ntiles) return;
    const int64_t my_tiles = (ntiles - first + stride - 1) / stride;
    const int64_t nm = g.K / BKH;
    const int64_t total = my_tiles * nm;

    float sa, sb, ia, ib;
    h3_scale(*g.a_amax, sa, ia);
    h3_scale(*g.b_amax, sb, ib);
    (void)sa;
    (void)sb;

    // per-lane glds sources of the tile currently being issued
    uint32_t off[G];
    int dst[G];
    int64_t off_tile = -1;
    auto set_tile = [&](int64_t k) {   // k-th tile of this workgroup
        const int64_t lt = first + k * stride;
        const int64_t m0 = (lt / ntn) * BM, n0 = (lt % ntn) * BN;
#pragma unroll
        for (int q = 0; q < G; ++q) {
            const bool isa = q < GA;
            const int r0 = (isa ? wave * GA + q : wave * GB + (q - GA)) * L::RPI;
            const int r = r0 + lane / L::CPR;
            const int c = (lane % L::CPR) ^ L::swz((isa ? 0 : BM) + r);
            const int64_t lim = isa ? g.M : g.N;
            int64_t gr = (isa ? m0 : n0) + r;
            if (gr > lim - 1) gr = lim - 1;
            off[q] = (uint32_t)((gr * (isa ? g.lda : g.ldb) + 8 * c) * 2);
            dst[q] = ((isa ? 0 : BM) + r0) * L::CPR;
        }
        off_tile = k;
    };
    auto issue = [&](int64_t S) {   // global slice S of this workgroup
        if (S >= total) return;
        const int64_t k = S / nm;
        if (k != off_tile) set_tile(k);
        const uint32_t kb = (uint32_t)((S % nm) * BKH * 4);
        uint4* slot = smem + (int)(S % NS) * SLICE_U4;
#pragma unroll
        for (int q = 0; q < G; ++q) {
            const char* base = reinterpret_cast<const char*>(q < GA ? P.a : P.b);
            __builtin_amdgcn_global_load_lds((gbl_void_t*)(base + (off[q] + kb)), (lds_void_t*)(slot + dst[q]), 16, 0,
                                             0);
        }
    };

    floatx16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    float* stage = reinterpret_cast<float*>(smem + NS * SLICE_U4) + wave * (32 * 32);
    uint32_t cmax = 0;

    for (int S = 0; S < NS - 1; ++S) issue(S);
    for (int64_t S = 0; S < total; ++S) {
        if (S + NS - 2 < total) p16_wait_vmcnt<(NS - 2) * G>();
        else p16_wait_vmcnt<0>();
        p16_barrier();
        const bool tile_end = S % nm == nm - 1;
        if (kLoadFree || !tile_end) issue(S + NS - 1);
        p16_mma<BM, BN, BKH, WM, WN, 0>(smem + (int)(S % NS) * SLICE_U4, acc, wm, wn, lane);
        if (tile_end) {   // last slice of a tile: its epilogue, with the next tile's slices in flight
            const int64_t lt = first + (S / nm) * stride;
            const int64_t m0 = (lt / ntn) * BM, n0 = (lt % ntn) * BN;
            p16p_epilogue<TM, TN, DROPADD, EXTRA>(g, acc, m0 + wm * (BM / WM), n0 + wn * (BN / WN), lane, ia, ib,
                                                  stage, cmax);
            if (!kLoadFree) issue(S + NS - 1);
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j)
#pragma unroll
                    for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
        }
    }
    if (g.c_amax) {
        for (int o = 32; o > 0; o >>= 1) cmax = max(cmax, (uint32_t)__shfl_xor((int)cmax, o, kWave));
        if (lane == 0 && cmax) atomicMax(reinterpret_cast<uint32_t*>(g.c_amax), cmax);
    }
}

// variant: 0 = 256x256 tiles, k16 slices (64-B rows), 4 slots; 1 = 256x256, k32 slices, 2 slots;
// 2 = 256x128, k32 slices, 3 slots; 3 = variant 1 with the MFMA block at s_setprio 1;
// 4 = persistent (k_gemm_p16p, 256x256, k32 slices, 2 slots; also with the drop-add epilogue);
// 10 + k = timing ablation k of variant 0 (12-14), 15 = variant 1 without an epilogue, 16 = variant 1
// with C stored straight from the accumulators (no LDS staging; no beta / drop-add / gather)
static void launch_p16(int variant, bool dropadd, dim3 grid, hipStream_t s, const P16Args& P) {
    if (variant == 4 || variant == 5) {   // persistent: one workgroup per CU (256 on MI355X) or fewer
        const int64_t tiles = grid.x;
        const dim3 pg((unsigned)(tiles < 256 ? tiles : 256));
        const bool extra = P.g.bias != nullptr || P.g.beta != 0.f;
        if (dropadd) hipLaunchKernelGGL((k_gemm_p16p<256, 256, 32, 2, 2, 4, true, false>), pg, dim3(512), 0, s, P);
        else if (extra) hipLaunchKernelGGL((k_gemm_p16p<256, 256, 32, 2, 2, 4, false, true>), pg, dim3(512), 0, s, P);
        else hipLaunchKernelGGL((k_gemm_p16p<256, 256, 32, 2, 2, 4, false, false>), pg, dim3(512), 0, s, P);
        return;
    }
    if (dropadd) {
        hipLaunchKernelGGL((k_gemm_p16<256, 256, 16, 4, 2, 4, 8>), grid, dim3(512), 0, s, P);
        return;
    }
    switch (variant) {
        case 1: hipLaunchKernelGGL((k_gemm_p16<256, 256, 32, 2, 2, 4>), grid, dim3(512), 0, s, P); break;
        case 2: hipLaunchKernelGGL((k_gemm_p16<256, 128, 32, 3, 4, 2>), grid, dim3(512), 0, s, P); break;
        case 3: hipLaunchKernelGGL((k_gemm_p16<256, 256, 32, 2, 2, 4, 9>), grid, dim3(512), 0, s, P); break;
        case 12: hipLaunchKernelGGL((k_gemm_p16<256, 256, 16, 4, 2, 4, 2>), grid, dim3(512), 0, s, P); break;
        case 13: hipLaunchKernelGGL((k_gemm_p16<256, 256, 16, 4, 2, 4, 3>), grid, dim3(512), 0, s, P); break;
        case 14: hipLaunchKernelGGL((k_gemm_p16<256, 256, 16, 4, 2, 4, 4>), grid, dim3(512), 0, s, P); break;
        case 15: hipLaunchKernelGGL((k_gemm_p16<256, 256, 32, 2, 2, 4, 15>), grid, dim3(512), 0, s, P); break;
        case 16: hipLaunchKernelGGL((k_gemm_p16<256, 256, 32, 2, 2, 4, 16>), grid, dim3(512), 0, s, P); break;
        default: hipLaunchKernelGGL((k_gemm_p16<256, 256, 16, 4, 2, 4>), grid, dim3(512), 0, s, P); break;
    }
}

static int64_t p16_bm(int variant) { (void)variant; return 256; }
static int64_t p16_bn(int variant) { return variant == 2 ? 128 : 256; }

}  // namespace bgnn

using namespace bgnn;

extern "C" int bgnn_split_f16x2(const float* x, int64_t rows, int64_t cols, int64_t ldx, const float* amax,
                                uint16_t* pieces, int64_t ldp, void* stream) {
    BGNN_REQUIRE(x && amax && pieces && rows >= 0 && cols >= 0, "split_f16x2: bad args");
    BGNN_REQUIRE(cols % 8 == 0 && ldx % 4 == 0 && ldp % 8 == 0 && ldx >= cols && ldp >= 2 * cols,
                 "split_f16x2: cols and ldp must be multiples of 8, ldx of 4 (ldx >= cols, ldp >= 2 cols)");
    BGNN_REQUIRE(aligned16(x) && aligned16(pieces), "split_f16x2: x and pieces must be 16-B aligned");
    if (rows == 0 || cols == 0) return BGNN_OK;
    const int64_t n = rows * (cols / 8);
    int64_t blocks = (n + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(k_split_f16x2, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream), x, rows, cols / 8, ldx,
                       amax, reinterpret_cast<uint4*>(pieces), ldp / 8);
    BGNN_CHECK_LAUNCH();
    return BGNN_OK;
}

extern "C" int bgnn_gemm_p16(int64_t M, int64_t N, int64_t K, const uint16_t* a, int64_t lda, const float* a_amax,
                             const uint16_t* b, int64_t ldb, const float* b_amax, float alpha, float beta, float* C,
                             int64_t ldc, const float* bias, int32_t relu, float* c_amax, const float* bsrc,
                             int64_t ld_bsrc, float p, uint64_t seed, int32_t variant, void* stream) {
    BGNN_REQUIRE(a && b && C && a_amax && b_amax, "gemm_p16: null pointer");
    BGNN_REQUIRE(M >= 0 && N > 0 && K > 0 && K % 32 == 0, "gemm_p16: need K > 0, K %% 32 == 0 (got %lld)", (long long)K);
    BGNN_REQUIRE(lda >= 2 * K && ldb >= 2 * K && lda % 8 == 0 && ldb % 8 == 0,
                 "gemm_p16: piece rows must hold 2K elements and be 16-B multiples");
    BGNN_REQUIRE(aligned16(a) && aligned16(b), "gemm_p16: piece buffers must be 16-B aligned");
    BGNN_REQUIRE(ldc >= N, "gemm_p16: ldc < N");
    BGNN_REQUIRE(M * lda * 2 < (int64_t(1) << 32) && N * ldb * 2 < (int64_t(1) << 32), "gemm_p16: piece buffers over 4 GiB");
    BGNN_REQUIRE(!bsrc || (beta == 1.f && N % 4 == 0 && ldc % 4 == 0 && ld_bsrc % 4 == 0 && aligned16(bsrc) &&
                           aligned16(C)),
                 "gemm_p16: the drop-add epilogue needs beta 1 and 16-B aligned rows");
    BGNN_REQUIRE(p >= 0.f && p < 1.f, "gemm_p16: dropout p must be in [0, 1)");
    BGNN_REQUIRE(variant >= 0 && (variant <= 5 || (variant >= 12 && variant <= 16)), "gemm_p16: bad variant");
    if (M == 0) return BGNN_OK;
    P16Args P{};
    GemmArgs& g = P.g;
    g.C = C;
    g.M = M; g.N = N; g.K = K; g.lda = lda; g.ldb = ldb; g.ldc = ldc;
    g.alpha = alpha; g.beta = beta;
    g.kchunk = K; g.split = 1;
    g.bias = bias; g.relu = relu;
    g.a_amax = a_amax; g.b_amax = b_amax; g.c_amax = c_amax;
    if (bsrc) {
        g.bsrc = bsrc; g.ld_bsrc = ld_bsrc; g.dseed = seed;
        g.dthr = dropout_threshold(p);
        g.dkeep = g.dthr ? 1.f / (1.f - p) : 1.f;
    }
    P.a = a; P.b = b;
    const int v = (bsrc && variant != 4) ? 0 : variant;
    const int64_t tiles = ((M + p16_bm(v) - 1) / p16_bm(v)) * ((N + p16_bn(v) - 1) / p16_bn(v));
    launch_p16(variant, bsrc != nullptr, dim3((unsigned)tiles), as_stream(stream), P);
    BGNN_CHECK_LAUNCH();
    return BGNN_OK;
}
