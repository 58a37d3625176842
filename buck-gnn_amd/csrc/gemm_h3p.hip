// Pipelined f16x3 GEMM for the pre-split NT products (round 6): C = A W^T (+ drop(src)) with A
// [M, K] f32 K-contiguous and W's pre-split image (bgnn_gemm_wsplit) -- the SAGE forward
// z = x [W_l;W_r]^T and input gradient dx = [dz_l | dh] [W_l;W_r] (Models/BuckGNN.py:430-444 through
// bgnn_gemm_f32_w), selected by knob BGNN_TUNE_GEMM_BDMA = 2.
//
// Same arithmetic as k_gemm_x6<1, 0, 1, BM, BN, WM, WN, ABL, 4> (the same operand scales and f16
// pieces, the same LDS images, the same 16x16x32 MFMAs per accumulator in the same k order, the
// same x6_epilogue), so the same bits. What differs is the schedule. k_gemm_x6 runs each 32-deep
// slice as [split A, copy B, ds_read the fragments, MFMAs, barrier]: every slice opens with the
// MFMA pipe idle while the fragments come back from LDS (8 waves x 16 KiB per slice). Here:
//   * the fragments of slice kt+1 are read into a second register set while slice kt's MFMAs run,
//     so a slice starts on registers that are already loaded;
//   * B's image goes HBM/L2 -> LDS by global_load_lds_dwordx4 into NSB slots (no VGPRs);
//   * A is loaded by asm global loads (hipcc cannot see them, so it does not drain the DMA in flight
//     with vmcnt(0) before each split -- the waits are counted here), split and stored two slices
//     ahead of its MFMAs;
//   * one barrier per slice publishes slice kt+2's A pieces and B(kt+2)'s DMA.
// Rows past M re-read row M - 1 (never stored); K % 32 == 0 (the image requires it).
#include "gemm_x6_kernel.h"

// m0 is set inside the DMA asm (no compiler-held value lives in m0 in this kernel)
#pragma clang diagnostic ignored "-Winline-asm"

namespace bgnn {

int g_h3p_nsb = 4;   // B slots (3 or 4; default 4: r06o/r06q, dgrad 269-263 us against 273 with 3)

namespace {

typedef float f32x4_t __attribute__((ext_vector_type(4)));

// A's 8-k units of one slice (NU per thread, two float4 each): loaded by asm (hipcc does not track
// them; h3p_wait ties them)
template <int NU>
struct H3pA {
    f32x4_t v[NU][2];
};

template <int NU>
__device__ __forceinline__ void h3p_load(H3pA<NU>& r, const float* p, int64_t ustride) {
#pragma unroll
    for (int u = 0; u < NU; ++u) {
        const float* q = p + u * ustride;
        asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(r.v[u][0]) : "v"(q) : "memory");
        asm volatile("global_load_dwordx4 %0, %1, off offset:16" : "=v"(r.v[u][1]) : "v"(q) : "memory");
    }
}

// wait until at most N vector-memory ops are in flight; the registers pass through the asm so no
// use of them can be scheduled above the wait
template <int N, int NU>
__device__ __forceinline__ void h3p_wait(H3pA<NU>& r) {
    static_assert(N >= 0 && N < 64, "vmcnt field is 6 bits");
    static_assert(NU == 1 || NU == 2, "units per thread");
    if constexpr (NU == 1)
        asm volatile("s_waitcnt vmcnt(%2)" : "+v"(r.v[0][0]), "+v"(r.v[0][1]) : "n"(N) : "memory");
    else
        asm volatile("s_waitcnt vmcnt(%4)"
                     : "+v"(r.v[0][0]), "+v"(r.v[0][1]), "+v"(r.v[1][0]), "+v"(r.v[1][1])
                     : "n"(N)
                     : "memory");
}

// X: timing ablations of the measurement build only (make abl; results wrong): 1 no B DMA, 2 no A
// loads, 4 no A split / store, 8 no next-fragment reads, 16 no waits / barriers in the loop, 32 no
// epilogue
// 8 waves (128 x 256, one workgroup per CU) or 4 waves (128 x 128, MINB = 2 workgroups per CU,
// whose epilogues and barriers then overlap the other's main loop)
template <int BM, int BN, int WM, int WN, int NSB, int ABL, int X = 0, int MINB = 1>
__global__ __launch_bounds__(64 * WM * WN, MINB) void k_gemm_h3p(GemmArgs g) {
    constexpr int NT = 64 * WM * WN;
    static_assert(WM * WN == 8 || WM * WN == 4, "8 or 4 waves");
    constexpr int TM = BM / WM / 32, TN = BN / WN / 32;   // 32x32 blocks per wave
    constexpr int NU = BM * 4 / NT;                        // 8-k units of A per thread and slice
    static_assert(NU * NT == BM * 4 && (NU == 1 || NU == 2), "whole units of A per thread");
    constexpr int A_U4 = 2 * BM * 4, B_U4 = 2 * BN * 4;   // [piece][row][4 chunks]
    constexpr int GB = BN * 8 / NT;                        // B DMA pieces per thread and slice
    static_assert(GB * NT == BN * 8, "whole B pieces per thread");
    constexpr int LA = 2 * NU;                             // A loads per thread and slice
    constexpr int SMEM_U4 = 2 * A_U4 + NSB * B_U4;
    constexpr int STAGE_U4 = WM * WN * TM * 32 * 32 * 4 / 16;
    static_assert(SMEM_U4 * 16 <= 160 * 1024 && STAGE_U4 <= SMEM_U4, "LDS");
    static_assert(NSB == 3 || NSB == 4, "B slots");
    __shared__ uint4 smem[SMEM_U4];
    uint4* const abuf = smem;
    uint4* const bslots = smem + 2 * A_U4;

    // (the wave index through readfirstlane: wave-uniform branches on it stay scalar)
    const int t = threadIdx.x, lane = t & 63, wave = (X & 128) ? (t >> 6) : __builtin_amdgcn_readfirstlane(t >> 6);
    const int wm = wave / WN, wn = wave % WN;
    const int64_t ntn = (g.N + BN - 1) / BN;
    const int tiles = (int)(((g.M + BM - 1) / BM) * ntn);
    const int lt = xcd_remap(blockIdx.x, tiles);
    const int64_t tm = lt / ntn, tn = lt % ntn;
    const int64_t m0 = tm * BM, n0 = tn * BN;
    const int64_t nk = g.K / X6_BK;
    if constexpr ((X & 768) != 0) {   // (measurement build: half of each XCD's first-round workgroups start late)
        if (blockIdx.x < 256 && ((blockIdx.x >> 3) & 1))
            for (int i = 0; i < ((X >> 8) & 3) * 2; ++i) __builtin_amdgcn_s_sleep(127);
    }

    float sa, ia, sb, ib;
    h3_scale(*g.a_amax, sa, ia);
    h3_scale(*g.b_amax, sb, ib);

    // A: thread t stages units t + NT u = (row (t / 4) + u NT / 4, chunk t % 4); rows past M re-read
    // row M - 1 (the second unit's row is the first's + NT / 4: clamped separately)
    const int ar = t >> 2, ac = t & 3;
    using ARegs = H3pA<NU>;
    const int64_t grow = (m0 + ar < g.M) ? m0 + ar : g.M - 1;
    const int64_t grow1 = (m0 + ar + NT / 4 < g.M) ? m0 + ar + NT / 4 : g.M - 1;
    const float* aptr = g.A + grow * g.lda + 8 * ac;
    const int64_t austride = (grow1 - grow) * g.lda;   // unit 1's rows relative to unit 0's
    auto load_a = [&](ARegs& r, int64_t kt) { h3p_load<NU>(r, aptr + (kt < nk ? kt : nk - 1) * X6_BK, austride); };
    auto store_a = [&](const ARegs& r, int64_t kt) {   // split into A buffer kt & 1 (x6_store's bits)
        uint4* S = abuf + (int)(kt & 1) * A_U4;
#pragma unroll
        for (int u = 0; u < NU; ++u) {
            const f32x4_t lo = r.v[u][0], hi = r.v[u][1];
            uint4 q0, q1;
            split2h(lo.x * sa, lo.y * sa, q0.x, q1.x);
            split2h(lo.z * sa, lo.w * sa, q0.y, q1.y);
            split2h(hi.x * sa, hi.y * sa, q0.z, q1.z);
            split2h(hi.z * sa, hi.w * sa, q0.w, q1.w);
            const int apos = x6_pos(ar + u * (NT / 4), ac);
            S[apos] = q0;
            S[BM * 4 + apos] = q1;
        }
    };
    // B: slice min(kt, nk - 1) of column tile tn into slot kt % NSB
    const uint4* img = reinterpret_cast<const uint4*>(g.B) + tn * nk * (BN * 8) + t;
    // (asm, like A's loads: hipcc would otherwise drain every DMA in flight, vmcnt(0), before each
    // LDS read it cannot prove disjoint from them -- the fragment reads of the next slice)
    // The drop-add source through LDS (ABL 8 with the plain epilogue of bgnn_gemm_f32_w): the DMA of
    // the last NSB steps, which would re-read B's last slice, brings the tile's masked-gradient source
    // rows instead -- quarter q (BM / NSB rows of 1 KiB) into slot (nk + q) % NSB, the same slots and
    // vmcnt counts -- so the epilogue reads them from LDS instead of waiting on HBM
    constexpr bool kSrcLds = ABL == 8 && (X & ~896) == 0 && BN * 4 == 1024 && NSB * GB * (NT / 64) == BM;
    const bool lsrc = kSrcLds && g.bsrc_c0 == 0 && !g.bias && !g.relu && !g.c_amax && !g.ga0 && g.alpha == 1.f &&
                      g.beta == 1.f && nk >= NSB && g.ld_bsrc % 4 == 0 && ((uintptr_t)g.bsrc & 15) == 0 &&
                      ((uintptr_t)g.C & 15) == 0 &&
                      g.ldc % 4 == 0;
    auto issue_b = [&](int64_t kt) {
        if (kSrcLds && lsrc && kt >= nk) {   // source rows (kt - nk) * BM / NSB + wave * GB + q of the tile
            const int64_t r0 = m0 + (kt - nk) * (BM / NSB) + wave * GB;
            const uint32_t dst = (uint32_t)(uintptr_t)(x6_lds_t*)(bslots + (int)(kt % NSB) * B_U4 + wave * GB * 64);
#pragma unroll
            for (int q = 0; q < GB; ++q) {
                const int64_t row = r0 + q < g.M ? r0 + q : g.M - 1;
                asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off"
                             :
                             : "s"(__builtin_amdgcn_readfirstlane(dst + q * 1024)),
                               "v"(g.bsrc + row * g.ld_bsrc + n0 + 4 * lane)
                             : "memory", "m0");
            }
            return;
        }
        const uint4* src = img + (kt < nk ? kt : nk - 1) * (BN * 8);
        const uint32_t dst = (uint32_t)(uintptr_t)(x6_lds_t*)(bslots + (int)(kt % NSB) * B_U4 + wave * 64);
#pragma unroll
        for (int q = 0; q < GB; ++q)
            asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off"
                         :
                         : "s"(__builtin_amdgcn_readfirstlane(dst + NT * q * 16)), "v"(src + NT * q)
                         : "memory", "m0");
    };

    // fragments of one slice: 16-row blocks of the wave's rows / columns, two pieces each
    struct Frag {
        uint4 a[2 * TM][2];
        uint4 b[2 * TN][2];
    };
    const int l16 = lane & 15, lq = lane >> 4;
    auto read_a = [&](Frag& f, const uint4* __restrict__ S, int i) {
#pragma unroll
        for (int p = 0; p < 2; ++p) f.a[i][p] = S[p * BM * 4 + x6_pos(wm * (BM / WM) + i * 16 + l16, lq)];
    };
    auto read_b = [&](Frag& f, const uint4* __restrict__ S, int j) {
#pragma unroll
        for (int p = 0; p < 2; ++p) f.b[j][p] = S[p * BN * 4 + x6_pos(wn * (BN / WN) + j * 16 + l16, lq)];
    };

    floatx4 acc[2 * TM][2 * TN];
#pragma unroll
    for (int i = 0; i < 2 * TM; ++i)
#pragma unroll
        for (int j = 0; j < 2 * TN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

    auto mma3 = [&](floatx4& c, const uint4 (&a)[2], const uint4 (&b)[2]) {
        c = __builtin_amdgcn_mfma_f32_16x16x32_f16(as_f16x8(a[0]), as_f16x8(b[1]), c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_f16(as_f16x8(a[1]), as_f16x8(b[0]), c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_f16(as_f16x8(a[0]), as_f16x8(b[0]), c, 0, 0, 0);
    };

    // step kt: MFMAs of slice kt from F (registers) while the fragments of slice kt+1 are read into
    // Fn; split A(kt+2) (register set R, loaded two steps ago) into A buffer kt & 1, refill R with
    // A(kt+4), DMA B(kt+NSB) into slot kt % NSB; wait for this wave's part of B(kt+2); barrier
    // (publishes A(kt+2) and B(kt+2), and every wave is done reading slice kt+1's buffers).
    // VMEM order per step: A loads, then the DMA.
    // vmcnt at the split: after A(kt+2)'s loads come its step's DMA and one whole step
    constexpr int GBW = (X & 1) ? 0 : GB;   // DMA pieces per step as issued (ablation 1 issues none)
    constexpr int WAIT_A = GBW + (LA + GBW);
    // vmcnt at the end: after B(kt+2) (issued at step kt+2-NSB) come NSB - 2 whole steps
    constexpr int WAIT_B = (NSB - 2) * (LA + GB);
    static_assert(WAIT_A < 64 && WAIT_B < 64, "vmcnt range");
    auto step = [&](int64_t kt, Frag& F, Frag& Fn, ARegs& R) {
        const bool next = kt + 1 < nk;
        const uint4* __restrict__ An = abuf + (int)((kt + 1) & 1) * A_U4;
        const uint4* __restrict__ Bn = bslots + (int)((kt + 1) % NSB) * B_U4;
#pragma unroll
        for (int j = 0; j < 2 * TN; ++j) {
            if (next && !(X & 8)) {
                read_b(Fn, Bn, j);
                if (j < 2 * TM) read_a(Fn, An, j);
            }
#pragma unroll
            for (int i = 0; i < 2 * TM; ++i) mma3(acc[i][j], F.a[i], F.b[j]);
            // waves 4-7 stage after the third column block instead of the first, so that a SIMD's two
            // waves do not both leave the MFMA pipe for their staging at once (the guide's stagger;
            // dgrad 262.5 -> 257.6 us, drop-add 311.7 -> 308.9, bit-identical, r06_gemm_stagger_u.txt)
            const int jst = (wave >= 4 && !(X & 64)) ? 2 : 0;   // (X & 64: measurement build, no stagger)
            if (j == jst) {
                // (the first two steps wait on the prologue's A(2) / A(3), fewer ops behind them)
                if (kt >= 2) h3p_wait<WAIT_A>(R);
                else if (kt == 1) h3p_wait<LA + GBW>(R);
                else h3p_wait<LA>(R);
                if (!(X & 4) && kt + 2 < nk) store_a(R, kt + 2);
                if (!(X & 2)) load_a(R, kt + 4);
                if (!(X & 1)) issue_b(kt + NSB);
            }
        }
        if constexpr (!(X & 16)) {
            x6_wait_vmcnt<WAIT_B>();
            x6_barrier_lds();
        }
    };

    // prologue: B(0 .. NSB-1) by DMA, A(0), A(1) split into buffers 0 / 1, A(2), A(3) in flight,
    // slice 0's fragments read; the second barrier frees buffer 0 / slot 0 for step 0's refills
    Frag F0, F1;
    ARegs R0, R1;
    for (int m = 0; m < NSB; ++m) issue_b(m);
    load_a(R0, 0);
    load_a(R1, 1);
    h3p_wait<0>(R0);
    h3p_wait<0>(R1);
    store_a(R0, 0);
    if (nk > 1) store_a(R1, 1);
    if constexpr (!(X & 2)) {   // (ablation 2 keeps no A load in flight past this point)
        load_a(R0, 2);
        load_a(R1, 3);
    }
    x6_barrier_lds();
    {
        const uint4* __restrict__ A0 = abuf;
        const uint4* __restrict__ B0 = bslots;
#pragma unroll
        for (int j = 0; j < 2 * TN; ++j) read_b(F0, B0, j);
#pragma unroll
        for (int i = 0; i < 2 * TM; ++i) read_a(F0, A0, i);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    x6_barrier_lds();
    int64_t kt = 0;
    for (; kt + 1 < nk; kt += 2) {
        step(kt, F0, F1, R0);
        step(kt + 1, F1, F0, R1);
    }
    if (kt < nk) step(kt, F0, F1, R0);
    // the clamped tail loads / DMA land before the epilogue reuses the LDS as its stage
    h3p_wait<0>(R0);
    h3p_wait<0>(R1);
    x6_barrier_lds();

    if constexpr ((X & 32) != 0) {   // (keeps the MFMAs live)
        float v = 0.f;
#pragma unroll
        for (int i = 0; i < 2 * TM; ++i)
#pragma unroll
            for (int j = 0; j < 2 * TN; ++j) v += acc[i][j][0];
        if (g.alpha == -7.f) g.C[t] = v;
        return;
    }
    if constexpr (kSrcLds) {
        if (lsrc) {
            // x6_epilogue's fast-path arithmetic per element (its general path, (e * ia) * ib, for a
            // wave whose rows run past M), the source from LDS; one 32 x 32 block at a time through a
            // 4 KiB per-wave stage in the (now idle) A buffers
            float* stg = reinterpret_cast<float*>(abuf) + wave * 1024;
            const int rq = lane >> 3, c4 = (lane & 7) * 4;
            const int64_t wr0 = m0 + wm * (BM / WM);
            const bool fastw = wr0 + TM * 32 <= g.M;
            const float iab = ia * ib;
            const bool one_mul = fastw && iab != 0.f && iab < 3.0e38f;
            const float* bl = reinterpret_cast<const float*>(bslots);
#pragma unroll
            for (int j = 0; j < TN; ++j)
#pragma unroll
                for (int i = 0; i < TM; ++i) {
#pragma unroll
                    for (int si = 0; si < 2; ++si)
#pragma unroll
                        for (int sj = 0; sj < 2; ++sj)
#pragma unroll
                            for (int r = 0; r < 4; ++r)
                                stg[(si * 16 + 4 * lq + r) * 32 + sj * 16 + l16] = acc[2 * i + si][2 * j + sj][r];
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const int rr = q * 8 + rq;
                        const int trow = wm * (BM / WM) + i * 32 + rr;   // row in the tile
                        const int tcol = wn * (BN / WN) + j * 32 + c4;
                        const int64_t row = m0 + trow, col = n0 + tcol;
                        const float4 sv = *reinterpret_cast<const float4*>(stg + rr * 32 + c4);
                        const float4 src = *reinterpret_cast<const float4*>(
                            bl + (int)((nk + trow / (BM / NSB)) % NSB) * (B_U4 * 4) + (trow % (BM / NSB)) * BN + tcol);
                        if (row >= g.M) continue;
                        float pv[4];
                        beta_mask4(g, row, col, src, pv);
                        const float e[4] = {sv.x, sv.y, sv.z, sv.w};
                        float o[4];
#pragma unroll
                        for (int k = 0; k < 4; ++k) {
                            float v = one_mul ? e[k] * iab : (e[k] * ia) * ib;
                            v *= g.alpha;
                            v += g.beta * pv[k];
                            o[k] = v;
                        }
                        st_nt4(g.C + row * g.ldc + col, o);
                    }
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                }
            return;
        }
    }
    float* stage = reinterpret_cast<float*>(smem) + wave * (TM * 32 * 32);
    if (ABL == 8 && n0 < g.bsrc_c0) {   // drop-add GEMM, a column tile left of the beta operand
        GemmArgs ge = g;
        ge.beta = 0.f;
        x6_epilogue<TM, TN, ABL, false>(ge, acc, m0 + wm * (BM / WM), n0 + wn * (BN / WN), n0, 0, lane, ia, ib, stage);
        return;
    }
    x6_epilogue<TM, TN, ABL, false>(g, acc, m0 + wm * (BM / WM), n0 + wn * (BN / WN), n0, 0, lane, ia, ib, stage);
}


}  // namespace

// the plan tile (cfg) must be 128 x 256 (2 x 4 waves, knob 16 = 2 / 3) or 128 x 128 (2 x 2 waves,
// knob 16 = 4); K % 32 == 0, 16-B aligned A rows
bool h3p_ok(int cfg, const GemmArgs& g) {
    // (round 6 also measured the forward, N = 1024, on 256 x 128 and 128 x 256 pipelined tiles:
    // 318 / 298 us against k_gemm_x6's 256 x 256 at 284, profiles/r06_gemm_fwd_tiles_z.txt)
    const bool tile = (cfg == 2 && g_x6_bdma == 2) || (cfg == 0 && g_x6_bdma == 4);
    return tile && g.wb && g.split <= 1 && g.a_blk == 0 && g.c_blk == 0 && g.K > 0 && g.K % X6_BK == 0 &&
           g.lda % 4 == 0 && aligned16(g.A);
}

#ifdef BGNN_H3P_ABLATION
int g_h3p_abl = 0;
template <int X>
static void launch_x(int abl, dim3 grid, hipStream_t s, const GemmArgs& g) {
    if (abl == 8) hipLaunchKernelGGL((k_gemm_h3p<128, 256, 2, 4, 4, 8, X>), grid, dim3(512), 0, s, g);
    else hipLaunchKernelGGL((k_gemm_h3p<128, 256, 2, 4, 4, 0, X>), grid, dim3(512), 0, s, g);
}
#endif

void launch_h3p(int cfg, int abl, dim3 grid, hipStream_t s, const GemmArgs& g) {
    (void)cfg;
#ifdef BGNN_H3P_ABLATION
    switch (g_h3p_abl) {
        case 1: launch_x<1>(abl, grid, s, g); return;
        case 2: launch_x<2>(abl, grid, s, g); return;
        case 3: launch_x<3>(abl, grid, s, g); return;
        case 4: launch_x<4>(abl, grid, s, g); return;
        case 7: launch_x<7>(abl, grid, s, g); return;
        case 8: launch_x<8>(abl, grid, s, g); return;
        case 16: launch_x<16>(abl, grid, s, g); return;
        case 15: launch_x<15>(abl, grid, s, g); return;
        case 31: launch_x<31>(abl, grid, s, g); return;
        case 32: launch_x<32>(abl, grid, s, g); return;
        case 63: launch_x<63>(abl, grid, s, g); return;
        case 128: launch_x<128>(abl, grid, s, g); return;
        case 256: launch_x<256>(abl, grid, s, g); return;
        case 512: launch_x<512>(abl, grid, s, g); return;
        case 768: launch_x<768>(abl, grid, s, g); return;
        case 64: launch_x<64>(abl, grid, s, g); return;
        default: break;
    }
#endif
#ifdef BGNN_H3P_ABLATION
    if (g_x6_bdma == 4) {   // 128 x 128, two workgroups per CU (measurement build only)
        if (abl == 8) hipLaunchKernelGGL((k_gemm_h3p<128, 128, 2, 2, 3, 8, 0, 2>), grid, dim3(256), 0, s, g);
        else hipLaunchKernelGGL((k_gemm_h3p<128, 128, 2, 2, 3, 0, 0, 2>), grid, dim3(256), 0, s, g);
        return;
    }
#endif
    if (abl == 8) {
        if (g_h3p_nsb == 4) hipLaunchKernelGGL((k_gemm_h3p<128, 256, 2, 4, 4, 8>), grid, dim3(512), 0, s, g);
        else hipLaunchKernelGGL((k_gemm_h3p<128, 256, 2, 4, 3, 8>), grid, dim3(512), 0, s, g);
    } else {
        if (g_h3p_nsb == 4) hipLaunchKernelGGL((k_gemm_h3p<128, 256, 2, 4, 4, 0>), grid, dim3(512), 0, s, g);
        else hipLaunchKernelGGL((k_gemm_h3p<128, 256, 2, 4, 3, 0>), grid, dim3(512), 0, s, g);
    }
}

}  // namespace bgnn
