// f16x3 GEMM with LDS-DMA operand staging (gfx950 global_load_lds_dwordx4) for the tall,
// K-contiguous SAGE GEMMs: the forward z = x [W_l;W_r]^T and the dgrad dx = dz [W_l;W_r]
// (Models/BuckGNN.py:135-149 through bgnn/fused.py; A [M,K] and B [N,K], both K-contiguous).
//
// Same arithmetic as k_gemm_x6<PREC 1> (gemm_x6.hip) and bit-identical results: each operand
// element is scaled by its power-of-two operand scale and split into two f16 pieces, and every
// 32x32x16 block product is the same three f16 MFMAs in the same order. What differs is the
// staging:
//   * k_gemm_x6 loads a BK slice into VGPRs, splits it and writes f16 piece images to LDS. At
//     256x256 tiles the VGPRs hold one slice in flight only, and the loads' latency shows
//     (fwd 288 us against a 176 us MFMA + epilogue floor).
//   * here raw f32 slices go HBM -> LDS by global_load_lds (no VGPRs), NS stages deep, one
//     barrier per slice, and each wave splits its MFMA fragments after the ds_read.
//
// LDS image per stage: [A rows (BM) | B rows (BN)][BKS f32]. The 16-B chunk c of row r sits at
// chunk position c ^ f(r), f(r) = (r / RPQ) mod CPR (CPR chunks per row, RPQ rows per 256-B
// bank row), so the 16 lanes of a ds_read_b128 group (16 rows, one chunk) hit 16 distinct
// bank quads. glds writes lane-linearly (wave-uniform base + 16 * lane), so the swizzle goes on
// the global source address: lane l of an instruction covering RPI rows from r0 loads row
// r0 + l / CPR, chunk (l % CPR) ^ f(row). Rows past M (N) read the last valid row; their
// results are never stored.
#include "common.h"
#include "gemm_common.h"
#include "gemm_x6.h"

namespace bgnn {

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void gbl_void_t;

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
    static_assert(N >= 0 && N < 64, "vmcnt field is 6 bits");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// raw barrier: no vmcnt(0) drain of the glds in flight (a __syncthreads() would emit one);
// the empty asm statements keep the compiler from moving LDS accesses across it
__device__ __forceinline__ void raw_barrier() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// 8 consecutive f32 of one operand row (two float4 chunks), scaled and split into the two
// f16 pieces of one MFMA operand (x6_store's split)
__device__ __forceinline__ void split8(const float4 u, const float4 v, float s, uint4& hi, uint4& lo) {
    split2h(u.x * s, u.y * s, hi.x, lo.x);
    split2h(u.z * s, u.w * s, hi.y, lo.y);
    split2h(v.x * s, v.y * s, hi.z, lo.z);
    split2h(v.z * s, v.w * s, hi.w, lo.w);
}

// Geometry of one staged slice: [A rows (BM) | B rows (BN)][BKL f32], 16-B chunks swizzled.
// The pipeline steps by k16 sub-slices (H = BKL / 16 per slice).
template <int BM, int BN, int BKL>
struct H3gSlice {
    static constexpr int CPR = BKL / 4;      // 16-B chunks per row
    static constexpr int RPQ = 16 / CPR;     // rows per 256-B bank row
    static constexpr int RPI = 64 / CPR;     // rows per glds instruction (1 KiB)
    static constexpr int H = BKL / 16;       // k16 sub-slices per slice
    static constexpr int FLOATS = (BM + BN) * BKL;
    __device__ static int swz(int row) { return (row / RPQ) % CPR; }
    // float offset of logical chunk c of row `row`
    __device__ static int at(int row, int c) { return row * BKL + 4 * (c ^ swz(row)); }
    // row of the q-th (row, 2 pairs) unit of a conversion pass; for 128-B rows, bits 1-3 of q
    // are permuted so each 8-lane ds_write_b128 group spans rows {r, r+1, r+8, r+9} (conflict-free
    // with the write order of h3g_convert; checked by tools/lds_banks.py)
    __device__ static int conv_row(int q) {
        if constexpr (BKL == 32) return (q & ~15) | (q & 1) | (((q >> 1) & 1) << 3) | (((q >> 2) & 3) << 1);
        return q;
    }
};

// In-place split of sub-slice h of one landed slice: each 8-k pair (logical chunks 2p, 2p+1,
// p = 2h, 2h+1) of every row becomes its f16 hi piece in chunk 2p's slot and its lo piece in
// chunk 2p+1's slot (same bytes). The pair's two slots are one aligned 32-B physical pair (the
// swizzle XORs the chunk index). Bank-conflict-free as issued: reads chunk 2p first (16-lane
// ds_read_b128 groups cover 16 distinct bank slots), writes physical slot 2P + ((2 row / RPQ)
// & 1) first (8-lane ds_write_b128 groups, 128-B bank window).
template <int BM, int BN, int BKL, int NT, int ABL>
__device__ __forceinline__ void h3g_convert(float* __restrict__ S, int h, int t, float sa, float sb) {
    using L = H3gSlice<BM, BN, BKL>;
    constexpr int NPT = (BM + BN) * 2 / NT;
    static_assert(NPT * NT == (BM + BN) * 2, "pairs must split evenly over the threads");
#pragma unroll
    for (int u = 0; u < NPT; ++u) {
        const int idx = t + NT * u;
        const int row = L::conv_row(idx >> 1), p = 2 * h + (idx & 1);
        const int f = L::swz(row);
        float* q = S + row * BKL;
        const int c0 = (2 * p) ^ f, c1 = (2 * p + 1) ^ f;   // physical slots of chunks 2p, 2p+1
        const float4 x0 = *reinterpret_cast<const float4*>(q + 4 * c0);
        const float4 x1 = *reinterpret_cast<const float4*>(q + 4 * c1);
        uint4 hi, lo;
        if constexpr (ABL == 1) {   // ablation: no split arithmetic
            hi = __builtin_bit_cast(uint4, x0);
            lo = __builtin_bit_cast(uint4, x1);
        } else {
            split8(x0, x1, row < BM ? sa : sb, hi, lo);
        }
        const int wb = ((2 * row) / L::RPQ) & 1;   // physical half written first
        const bool hf = (c0 & 1) == wb;            // hi piece goes in the first-written slot
        const uint4 w0 = make_uint4(hf ? hi.x : lo.x, hf ? hi.y : lo.y, hf ? hi.z : lo.z, hf ? hi.w : lo.w);
        const uint4 w1 = make_uint4(hf ? lo.x : hi.x, hf ? lo.y : hi.y, hf ? lo.z : hi.z, hf ? lo.w : hi.w);
        *reinterpret_cast<uint4*>(q + 4 * ((c0 & ~1) | wb)) = w0;
        *reinterpret_cast<uint4*>(q + 4 * ((c0 & ~1) | (wb ^ 1))) = w1;
    }
}

// MFMAs of converted sub-slice h: wave fragments (A rows wm BM/WM + 32 i + (lane & 31), B rows
// likewise; k pair 2 h + (lane >> 5)) as one ds_read_b128 per piece; the two cross terms, then
// the leading product (k_gemm_x6's order).
template <int BM, int BN, int BKL, int WM, int WN, int ABL>
__device__ __forceinline__ void h3g_mma(const float* __restrict__ S, int h, floatx16 (&acc)[BM / WM / 32][BN / WN / 32],
                                        int wm, int wn, int lane) {
    using L = H3gSlice<BM, BN, BKL>;
    constexpr int TM = BM / WM / 32, TN = BN / WN / 32;
    const int li = lane & 31, lh = lane >> 5;
    const int p = 2 * h + lh;
    uint4 a[TM][2], b[TN][2];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
        const int row = wm * (BM / WM) + i * 32 + li;
        a[i][0] = *reinterpret_cast<const uint4*>(S + L::at(row, 2 * p));
        a[i][1] = *reinterpret_cast<const uint4*>(S + L::at(row, 2 * p + 1));
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int row = BM + wn * (BN / WN) + j * 32 + li;
        b[j][0] = *reinterpret_cast<const uint4*>(S + L::at(row, 2 * p));
        b[j][1] = *reinterpret_cast<const uint4*>(S + L::at(row, 2 * p + 1));
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            floatx16 t = acc[i][j];
            if constexpr (ABL == 3) {   // ablation: no MFMAs (keep the fragments live)
                t[0] += __uint_as_float(a[i][0].x ^ a[i][1].y ^ b[j][0].z ^ b[j][1].w);
            } else {
                t = __builtin_amdgcn_mfma_f32_32x32x16_f16(as_f16x8(a[i][0]), as_f16x8(b[j][1]), t, 0, 0, 0);
                t = __builtin_amdgcn_mfma_f32_32x32x16_f16(as_f16x8(a[i][1]), as_f16x8(b[j][0]), t, 0, 0, 0);
                t = __builtin_amdgcn_mfma_f32_32x32x16_f16(as_f16x8(a[i][0]), as_f16x8(b[j][0]), t, 0, 0, 0);
            }
            acc[i][j] = t;
        }
}

// One pipeline step: multiply sub-slice (cur, hc) while splitting sub-slice (nxt, hn) in place
// (with 128-B rows the two may share a slot: disjoint bytes). Both are restrict parameters so
// that, once inlined, their LDS accesses carry alias-scope metadata: hipcc then neither waits
// vmcnt(0) for the glds in flight before them (SIInsertWaitcnts only disambiguates LDS-DMA
// stores against scoped accesses; the pipeline's counted waits order them) nor keeps the
// conversion's stores from interleaving with the MFMA block's reads. The split runs
// unconditionally (one basic block with the MFMAs): in the last step it re-splits bytes
// nobody reads again.
template <int BM, int BN, int BKL, int WM, int WN, int ABL>
__device__ __forceinline__ void h3g_step(const float* __restrict__ cur, int hc, float* __restrict__ nxt, int hn,
                                         floatx16 (&acc)[BM / WM / 32][BN / WN / 32], int wm, int wn, int lane,
                                         int t, float sa, float sb) {
    h3g_convert<BM, BN, BKL, 64 * WM * WN, ABL>(nxt, hn, t, sa, sb);
    h3g_mma<BM, BN, BKL, WM, WN, ABL>(cur, hc, acc, wm, wn, lane);
}

// ABL (timing ablations only, wrong results): 1 = no split arithmetic, 2 = no glds (LDS
// never filled), 3 = no MFMAs (fragments still read), 4 = no waits for the glds in the loop
template <int BM, int BN, int BKL, int NS, int WM, int WN, int ABL = 0>
__global__ __launch_bounds__(64 * WM * WN) void k_gemm_h3g(GemmArgs g) {
    using L = H3gSlice<BM, BN, BKL>;
    constexpr int NW = WM * WN, NT = 64 * NW, H = L::H;
    constexpr int TM = BM / WM / 32, TN = BN / WN / 32;
    constexpr int GA = BM / (L::RPI * NW), GB = BN / (L::RPI * NW);   // glds per wave per slice
    constexpr int G = GA + GB;
    // slices in flight beyond the one a step converts from (steady state)
    constexpr int AHEAD = NS - 4 + H;
    static_assert(BKL == 16 || BKL == 32, "slice depth");
    static_assert(GA * L::RPI * NW == BM && GB * L::RPI * NW == BN, "rows must split evenly over the waves");
    static_assert(AHEAD >= 0 && AHEAD * G < 64, "stages");
    constexpr int EPI_F = NW * TM * 32 * 32;
    constexpr int SMEM_F = NS * L::FLOATS > EPI_F ? NS * L::FLOATS : EPI_F;
    static_assert(SMEM_F * 4 <= 160 * 1024, "LDS over 160 KiB");
    // all LDS in one array (a second __shared__ object can make hipcc wait vmcnt(0) before
    // the first ds_read of every slice)
    __shared__ __attribute__((aligned(16))) float smem[SMEM_F];

    const int t = threadIdx.x;
    const int lane = t & 63;
    const int wave = t >> 6;
    const int wm = wave / WN, wn = wave % WN;
    const int64_t ntn = (g.N + BN - 1) / BN;
    // XCD-aware order: the workgroups one XCD runs take consecutive tiles, i.e. the column
    // tiles of the same row block, so A's rows are fetched into that XCD's L2 once
    const int lt = xcd_remap(blockIdx.x, gridDim.x);
    const int64_t tm = lt / ntn, tn = lt % ntn;
    const int64_t m0 = tm * BM, n0 = tn * BN;

    float sa, sb, ia, ib;
    h3_scale(*g.a_amax, sa, ia);
    h3_scale(*g.b_amax, sb, ib);

    // per-lane glds sources: 32-bit byte offsets from A / B at k = 0 (h3g_ok bounds both below
    // 4 GiB, so the loads take the uniform-base + VGPR-offset form); wave-uniform LDS rows
    uint32_t off[G];
    int dst[G];
#pragma unroll
    for (int q = 0; q < G; ++q) {
        const bool isa = q < GA;
        const int r0 = (isa ? wave * GA + q : wave * GB + (q - GA)) * L::RPI;
        const int r = r0 + lane / L::CPR;
        const int c = (lane % L::CPR) ^ L::swz((isa ? 0 : BM) + r);
        const int64_t lim = isa ? g.M : g.N;
        int64_t gr = (isa ? m0 : n0) + r;
        if (gr > lim - 1) gr = lim - 1;
        off[q] = (uint32_t)((gr * (isa ? g.lda : g.ldb) + 4 * c) * 4);
        dst[q] = ((isa ? 0 : BM) + r0) * BKL;
    }
    const int64_t nm = g.K / BKL;   // slices
    const int64_t nj = nm * H;      // k16 steps
    auto issue = [&](int64_t m) {
        if (m >= nm) return;
        const uint32_t kb = (uint32_t)(m * BKL * 4);
        float* slot = smem + (int)(m % NS) * L::FLOATS;
#pragma unroll
        for (int q = 0; q < G; ++q) {
            if (ABL == 2) break;
            const char* base = reinterpret_cast<const char*>(q < GA ? g.A : g.B);
            __builtin_amdgcn_global_load_lds((gbl_void_t*)(base + (off[q] + kb)), (lds_void_t*)(slot + dst[q]), 16, 0,
                                             0);
        }
    };
    auto slot = [&](int64_t j) { return smem + (int)((j / H) % NS) * L::FLOATS; };

    floatx16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    // Pipeline over k16 steps j: step j multiplies sub-slice j (split in step j-1) while it
    // splits sub-slice j+1. Slice m (H sub-slices) goes to slot m % NS; slice m + NS - 1 is
    // issued at the first step of slice m, after that step's barrier has certified slice m-1
    // (the slot's previous occupant) fully multiplied. Each step first retires the slice it
    // converts from (this wave's AHEAD newer slices stay in flight; vmcnt(0) near the end,
    // where fewer were issued); the one barrier then certifies every wave's part landed, the
    // previous split done and the previous multiply done.
    for (int m = 0; m < NS - 1; ++m) issue(m);
    if (NS - 2 < nm) wait_vmcnt<(NS - 2) * G>();
    else wait_vmcnt<0>();
    raw_barrier();
    if (nj > 0) h3g_convert<BM, BN, BKL, NT, ABL>(smem, 0, t, sa, sb);
    for (int64_t j = 0; j < nj; ++j) {
        const int64_t last = (j == 0 ? 0 : (j - 1) / H + 1) + NS - 2;   // newest slice issued so far
        if (ABL != 4) {
            if (last < nm) wait_vmcnt<AHEAD * G>();
            else wait_vmcnt<0>();
        }
        raw_barrier();
        if (j % H == 0) issue(j / H + NS - 1);
        h3g_step<BM, BN, BKL, WM, WN, ABL>(slot(j), (int)(j % H), slot(j + 1), (int)((j + 1) % H), acc, wm, wn, lane,
                                           t, sa, sb);
    }
    __syncthreads();   // every wave's fragment reads done before the epilogue reuses the LDS
    float* stage = smem + wave * (TM * 32 * 32);
    x6_epilogue<TM, TN>(g, acc, m0 + wm * (BM / WM), n0 + wn * (BN / WN), n0, 0, lane, ia, ib, stage);
}

// Shapes this kernel takes (else the register-staged k_gemm_x6): f16x3, A and B K-contiguous
// and 16-B aligned rows, K a multiple of the slice, dense A, no split-K.
bool h3g_ok(const GemmArgs& g, int ta, int tb) {
    return ta == 0 && tb == 1 && g.a_blk == 0 && (g.c_blk == 0 || g.c_blk % 256 == 0) && g.split == 1 && g.K > 0 && g.K % 32 == 0 &&
           g.lda % 4 == 0 && g.ldb % 4 == 0 && ((uintptr_t)g.A & 15) == 0 && ((uintptr_t)g.B & 15) == 0 &&
           g.a_amax != nullptr && g.b_amax != nullptr && (g.M * g.lda + g.K) * 4 < (int64_t(1) << 32) &&
           (g.N * g.ldb + g.K) * 4 < (int64_t(1) << 32);
}

int64_t h3g_tiles(int variant, int64_t M, int64_t N) {
    (void)variant;   // every variant uses 256x256 tiles
    return ((M + 255) / 256) * ((N + 255) / 256);
}

// variant: 0 = 256x256 tiles, 64-B rows (k16 slices), 4 slots; 1 = 256x256 tiles, 128-B rows
// (k32 slices), 2 slots; 10 + k = timing ablation k of variant 1
void launch_h3g(int variant, int64_t tiles, hipStream_t s, const GemmArgs& g) {
    const dim3 grid((unsigned)tiles);
    switch (variant) {
        case 1: hipLaunchKernelGGL((k_gemm_h3g<256, 256, 32, 2, 2, 4>), grid, dim3(512), 0, s, g); break;
        case 11: hipLaunchKernelGGL((k_gemm_h3g<256, 256, 32, 2, 2, 4, 1>), grid, dim3(512), 0, s, g); break;
        case 12: hipLaunchKernelGGL((k_gemm_h3g<256, 256, 32, 2, 2, 4, 2>), grid, dim3(512), 0, s, g); break;
        case 13: hipLaunchKernelGGL((k_gemm_h3g<256, 256, 32, 2, 2, 4, 3>), grid, dim3(512), 0, s, g); break;
        case 14: hipLaunchKernelGGL((k_gemm_h3g<256, 256, 32, 2, 2, 4, 4>), grid, dim3(512), 0, s, g); break;
        case 24: hipLaunchKernelGGL((k_gemm_h3g<256, 256, 16, 4, 2, 4, 4>), grid, dim3(512), 0, s, g); break;
        default: hipLaunchKernelGGL((k_gemm_h3g<256, 256, 16, 4, 2, 4>), grid, dim3(512), 0, s, g); break;
    }
}

}  // namespace bgnn
