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
// (no VGPRs, no VALU), NS slices in flight, one raw barrier per slice. Pieces live in one
// buffer [2][rows][ld] (hi plane, then lo plane pstride elements later). LDS image per slice:
// [A rows (BM) | B rows (BN)] x [hi BKH k | lo BKH k] f16 = 4 BKH bytes per row, in 16-B chunks
// swizzled by (row / RPQ) mod CPR so the 16 lanes of a ds_read_b128 group hit 16 distinct bank
// slots; glds writes lane-linearly, so the swizzle goes on the per-lane global source address.
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
    static constexpr int CPR = BKH / 4;     // 16-B chunks per row: BKH/8 hi chunks + BKH/8 lo chunks
    static constexpr int HALF = CPR / 2;    // chunks per piece
    static constexpr int RPQ = 16 / CPR;    // rows per 256-B bank row
    static constexpr int RPI = 64 / CPR;    // rows per glds instruction (64 lanes x 16 B)
    static constexpr int H = BKH / 16;      // k16 MFMA steps per slice
    __device__ static int swz(int row) { return (row / RPQ) % CPR; }
    // uint4 index of logical chunk c of row `row`
    __device__ static int at(int row, int c) { return row * CPR + (c ^ swz(row)); }
};

// split an f32 matrix into its two f16 pieces (the same rounding as x6_store / split2h)
__global__ __launch_bounds__(256) void k_split_f16x2(const float* __restrict__ x, int64_t rows, int64_t cols4,
                                                     int64_t ldx, const float* __restrict__ amax,
                                                     uint2* __restrict__ hi, uint2* __restrict__ lo, int64_t ldo4) {
    float s, inv;
    h3_scale(*amax, s, inv);
    const int64_t n = rows * cols4;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        const int64_t r = i / cols4, c = i % cols4;
        const float4 v = *reinterpret_cast<const float4*>(x + r * ldx + 4 * c);
        uint2 h, l;
        split2h(v.x * s, v.y * s, h.x, l.x);
        split2h(v.z * s, v.w * s, h.y, l.y);
        hi[r * ldo4 + c] = h;
        lo[r * ldo4 + c] = l;
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
            a[i][0] = S[L::at(row, kg)];
            a[i][1] = S[L::at(row, L::HALF + kg)];
        }
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int row = BM + wn * (BN / WN) + j * 32 + li;
            b[j][0] = S[L::at(row, kg)];
            b[j][1] = S[L::at(row, L::HALF + kg)];
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
    const uint16_t* a;          // A pieces: hi plane, lo plane at + a_ps
    const uint16_t* b;          // B pieces
    int64_t a_ps, b_ps;         // plane strides (elements)
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
        const int piece = c / L::HALF, kg = c % L::HALF;
        const int64_t lim = isa ? g.M : g.N;
        int64_t gr = (isa ? m0 : n0) + r;
        if (gr > lim - 1) gr = lim - 1;   // rows past the edge re-read the last row (never stored)
        off[q] = (uint32_t)((piece * (isa ? P.a_ps : P.b_ps) + gr * (isa ? g.lda : g.ldb) + 8 * kg) * 2);
        dst[q] = ((isa ? 0 : BM) + r0) * L::CPR;
    }
    const int64_t nm = g.K / BKH;   // slices
    auto issue = [&](int64_t m) {
        if (m >= nm) return;
        const uint32_t kb = (uint32_t)(m * BKH * 2);
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
        p16_mma<BM, BN, BKH, WM, WN, ABL>(smem + (int)(m % NS) * SLICE_U4, acc, wm, wn, lane);
    }
    __syncthreads();   // every wave's fragment reads done before the epilogue reuses the LDS
    float* stage = reinterpret_cast<float*>(smem) + wave * (TM * 32 * 32);
    x6_epilogue<TM, TN, ABL == 8 ? 8 : 0>(g, acc, m0 + wm * (BM / WM), n0 + wn * (BN / WN), n0, 0, lane, ia, ib,
                                          stage);
}

// variant: 0 = 256x256 tiles, k16 slices (64-B rows), 4 slots; 1 = 256x256, k32 slices, 2 slots;
// 2 = 256x128, k32 slices, 3 slots; 10 + k = timing ablation k of variant 0
static void launch_p16(int variant, bool dropadd, dim3 grid, hipStream_t s, const P16Args& P) {
    if (dropadd) {
        hipLaunchKernelGGL((k_gemm_p16<256, 256, 16, 4, 2, 4, 8>), grid, dim3(512), 0, s, P);
        return;
    }
    switch (variant) {
        case 1: hipLaunchKernelGGL((k_gemm_p16<256, 256, 32, 2, 2, 4>), grid, dim3(512), 0, s, P); break;
        case 2: hipLaunchKernelGGL((k_gemm_p16<256, 128, 32, 3, 4, 2>), grid, dim3(512), 0, s, P); break;
        case 12: hipLaunchKernelGGL((k_gemm_p16<256, 256, 16, 4, 2, 4, 2>), grid, dim3(512), 0, s, P); break;
        case 13: hipLaunchKernelGGL((k_gemm_p16<256, 256, 16, 4, 2, 4, 3>), grid, dim3(512), 0, s, P); break;
        case 14: hipLaunchKernelGGL((k_gemm_p16<256, 256, 16, 4, 2, 4, 4>), grid, dim3(512), 0, s, P); break;
        default: hipLaunchKernelGGL((k_gemm_p16<256, 256, 16, 4, 2, 4>), grid, dim3(512), 0, s, P); break;
    }
}

static int64_t p16_bm(int variant) { (void)variant; return 256; }
static int64_t p16_bn(int variant) { return variant == 2 ? 128 : 256; }

}  // namespace bgnn

using namespace bgnn;

extern "C" int bgnn_split_f16x2(const float* x, int64_t rows, int64_t cols, int64_t ldx, const float* amax,
                                uint16_t* pieces, int64_t ldp, int64_t pstride, void* stream) {
    BGNN_REQUIRE(x && amax && pieces && rows >= 0 && cols >= 0, "split_f16x2: bad args");
    BGNN_REQUIRE(cols % 4 == 0 && ldx % 4 == 0 && ldp % 4 == 0 && pstride % 4 == 0 && ldx >= cols && ldp >= cols,
                 "split_f16x2: cols, ldx, ldp and pstride must be multiples of 4 (ld >= cols)");
    BGNN_REQUIRE(aligned16(x) && ((uintptr_t)pieces & 7) == 0, "split_f16x2: x must be 16-B, pieces 8-B aligned");
    if (rows == 0 || cols == 0) return BGNN_OK;
    const int64_t n = rows * (cols / 4);
    int64_t blocks = (n + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(k_split_f16x2, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream), x, rows, cols / 4, ldx,
                       amax, reinterpret_cast<uint2*>(pieces), reinterpret_cast<uint2*>(pieces + pstride), ldp / 4);
    BGNN_CHECK_LAUNCH();
    return BGNN_OK;
}

extern "C" int bgnn_gemm_p16(int64_t M, int64_t N, int64_t K, const uint16_t* a, int64_t lda, int64_t a_ps,
                             const float* a_amax, const uint16_t* b, int64_t ldb, int64_t b_ps, const float* b_amax,
                             float alpha, float beta, float* C, int64_t ldc, const float* bias, int32_t relu,
                             float* c_amax, const float* bsrc, int64_t ld_bsrc, float p, uint64_t seed,
                             int32_t variant, void* stream) {
    BGNN_REQUIRE(a && b && C && a_amax && b_amax, "gemm_p16: null pointer");
    BGNN_REQUIRE(M >= 0 && N > 0 && K > 0 && K % 32 == 0, "gemm_p16: need K > 0, K %% 32 == 0 (got %lld)", (long long)K);
    BGNN_REQUIRE(lda >= K && ldb >= K && lda % 8 == 0 && ldb % 8 == 0 && a_ps % 8 == 0 && b_ps % 8 == 0,
                 "gemm_p16: piece rows must hold K and be 16-B multiples");
    BGNN_REQUIRE(aligned16(a) && aligned16(b), "gemm_p16: piece buffers must be 16-B aligned");
    BGNN_REQUIRE(ldc >= N, "gemm_p16: ldc < N");
    BGNN_REQUIRE((a_ps + M * lda) * 2 < (int64_t(1) << 32) && (b_ps + N * ldb) * 2 < (int64_t(1) << 32),
                 "gemm_p16: piece buffers over 4 GiB");
    BGNN_REQUIRE(!bsrc || (beta == 1.f && N % 4 == 0 && ldc % 4 == 0 && ld_bsrc % 4 == 0 && aligned16(bsrc) &&
                           aligned16(C)),
                 "gemm_p16: the drop-add epilogue needs beta 1 and 16-B aligned rows");
    BGNN_REQUIRE(p >= 0.f && p < 1.f, "gemm_p16: dropout p must be in [0, 1)");
    BGNN_REQUIRE(variant >= 0 && (variant <= 2 || (variant >= 12 && variant <= 14)), "gemm_p16: bad variant");
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
    P.a = a; P.b = b; P.a_ps = a_ps; P.b_ps = b_ps;
    const int v = bsrc ? 0 : variant;
    const int64_t tiles = ((M + p16_bm(v) - 1) / p16_bm(v)) * ((N + p16_bn(v) - 1) / p16_bn(v));
    launch_p16(variant, bsrc != nullptr, dim3((unsigned)tiles), as_stream(stream), P);
    BGNN_CHECK_LAUNCH();
    return BGNN_OK;
}
