// fp32 GEMM on the gfx950 f32-input MFMA (v_mfma_f32_32x32x2_f32): the dense
// lin_l / lin_r of SAGEConv (Models/BuckGNN.py:135-149), i.e.
//   forward  z  = x · [W_l ; W_r]^T          (M = nodes, N = 2H, K = H)
//   dgrad    dx = [dz_l | dh] · [W_l ; W_r]   (M = nodes, N = H,  K = 2H)
//   wgrad    dW = [dz_l | dh]^T · x           (M = 2H,    N = H,  K = nodes; split-K)
// The f32 MFMA is an exact k-ordered fmaf chain (no TF32/xf32 on gfx950), so the
// result is fp32-accurate like the reference's torch.mm.
//
// Tiling: 128x128 output tile per 256-thread workgroup, 4 waves as 2x2, each wave
// 64x64 = 2x2 MFMA tiles of 32x32 (64 accumulator registers). K is staged through
// LDS in BK=16 slices, double-buffered (one barrier per slice); the next slice's
// global loads are issued before the current slice's MFMAs. Both operands are kept
// in LDS as [k][m] / [k][n] images so each MFMA operand is one conflict-free
// ds_read_b32 per lane. K-contiguous operands are transposed on the LDS store (row
// pad of 2 floats makes those scalar stores conflict-free). Tile order is remapped
// so each XCD owns a contiguous band of output rows (shared A panels stay in its L2).
#include "common.h"
#include "gemm_common.h"

namespace bgnn {

extern int g_x6_bdma;   // gemm_x6.hip: knob 16 (BGNN_TUNE_GEMM_BDMA)

// LDS row pad (floats): a K-contiguous operand is transposed by scalar ds_write_b32
// into a [BK][R + PAD] image; PAD is chosen so one wave's 32-lane store groups hit 32
// distinct banks (4*(R+PAD) = 8 mod 32 for BK = 16, 4 mod 32 for BK = 32). An
// R-contiguous operand is stored as float4 rows, kept 16-B aligned.
template <int KCONTIG, int BK>
struct Pad {
    static constexpr int value = KCONTIG ? (BK == 16 ? 2 : 1) : 4;
};

// Load one BK x R slice of an operand into registers (NL float4 per thread).
//   KCONTIG = 1: element (r, k) at P[r * ld + k]  (r = m or n, k contiguous)
//   KCONTIG = 0: element (r, k) at P[k * ld + r]  (r contiguous)
template <int KCONTIG, int R, int BK, int NT, bool FULL = false>
__device__ __forceinline__ void load_slice(const float* __restrict__ P, int64_t ld, int64_t Rlim, int64_t r0,
                                           int64_t k0, int64_t kend, bool vec_ok, float (&reg)[R * BK / 4 / NT][4]) {
    constexpr int NL = R * BK / 4 / NT;
    const int t = threadIdx.x;
#pragma unroll
    for (int i = 0; i < NL; ++i) {
        const int idx = t + NT * i;
        if constexpr (FULL) {   // interior tile, aligned, whole slice in range: no guards
            const int r = KCONTIG ? idx / (BK / 4) : (idx % (R / 4)) * 4;
            const int k = KCONTIG ? (idx % (BK / 4)) * 4 : idx / (R / 4);
            const float* src = KCONTIG ? P + (r0 + r) * ld + (k0 + k) : P + (k0 + k) * ld + (r0 + r);
            const float4 v = *reinterpret_cast<const float4*>(src);
            reg[i][0] = v.x; reg[i][1] = v.y; reg[i][2] = v.z; reg[i][3] = v.w;
        } else if constexpr (KCONTIG) {
            const int r = idx / (BK / 4), kq = idx % (BK / 4);
            const int64_t gr = r0 + r, gk = k0 + kq * 4;
            if (vec_ok && gr < Rlim && gk + 3 < kend) {
                const float4 v = *reinterpret_cast<const float4*>(P + gr * ld + gk);
                reg[i][0] = v.x; reg[i][1] = v.y; reg[i][2] = v.z; reg[i][3] = v.w;
            } else {
#pragma unroll
                for (int q = 0; q < 4; ++q) reg[i][q] = (gr < Rlim && gk + q < kend) ? P[gr * ld + gk + q] : 0.f;
            }
        } else {
            const int kr = idx / (R / 4), rq = idx % (R / 4);
            const int64_t gk = k0 + kr, gr = r0 + rq * 4;
            if (vec_ok && gk < kend && gr + 3 < Rlim) {
                const float4 v = *reinterpret_cast<const float4*>(P + gk * ld + gr);
                reg[i][0] = v.x; reg[i][1] = v.y; reg[i][2] = v.z; reg[i][3] = v.w;
            } else {
#pragma unroll
                for (int q = 0; q < 4; ++q) reg[i][q] = (gk < kend && gr + q < Rlim) ? P[gk * ld + gr + q] : 0.f;
            }
        }
    }
}

template <int KCONTIG, int R, int BK, int LDS_LD, int NT>
__device__ __forceinline__ void store_slice(float* __restrict__ S, const float (&reg)[R * BK / 4 / NT][4]) {
    constexpr int NL = R * BK / 4 / NT;
    const int t = threadIdx.x;
#pragma unroll
    for (int i = 0; i < NL; ++i) {
        const int idx = t + NT * i;
        if constexpr (KCONTIG) {
            const int r = idx / (BK / 4), kq = idx % (BK / 4);
#pragma unroll
            for (int q = 0; q < 4; ++q) S[(kq * 4 + q) * LDS_LD + r] = reg[i][q];
        } else {
            const int kr = idx / (R / 4), rq = idx % (R / 4);
            *reinterpret_cast<float4*>(S + kr * LDS_LD + rq * 4) =
                make_float4(reg[i][0], reg[i][1], reg[i][2], reg[i][3]);
        }
    }
}

// C tile BM x BN per workgroup of WM x WN waves; each wave owns (BM/WM) x (BN/WN)
// = TM x TN MFMA tiles of 32x32.
// TA: 0 -> A is [M,K] (K-contiguous), 1 -> A is [K,M].
// TB: 0 -> B is [K,N] (N-contiguous), 1 -> B is [N,K] (K-contiguous).
template <int TA, int TB, int BM, int BN, int BK, int WM, int WN>
__global__ __launch_bounds__(64 * WM * WN) void k_gemm_f32(GemmArgs g) {
    constexpr int NT = 64 * WM * WN;
    constexpr int TM = BM / WM / 32, TN = BN / WN / 32;
    constexpr int AK = (TA == 0) ? 1 : 0;   // A K-contiguous?
    constexpr int BKc = (TB == 1) ? 1 : 0;  // B K-contiguous?
    constexpr int LDA_S = BM + Pad<AK, BK>::value;
    constexpr int LDB_S = BN + Pad<BKc, BK>::value;
    __shared__ __attribute__((aligned(16))) float As[2][BK * LDA_S];
    __shared__ __attribute__((aligned(16))) float Bs[2][BK * LDB_S];

    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int wm = wave / WN, wn = wave % WN;
    const int64_t ntn = (g.N + BN - 1) / BN;
    const int64_t ntm = (g.M + BM - 1) / BM;
    const int tiles = (int)(ntm * ntn);
    const int lt = xcd_remap(blockIdx.x, tiles);
    const int64_t tm = lt / ntn, tn = lt % ntn;
    const int64_t m0 = tm * BM, n0 = tn * BN;
    const int64_t kb = (int64_t)blockIdx.y * g.kchunk;
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

    float ra[BM * BK / 4 / NT][4], rb[BN * BK / 4 / NT][4];
    const int64_t nk = (ke > kb) ? (ke - kb + BK - 1) / BK : 0;
    // interior tile with whole, aligned K slices: unguarded loads (uniform branch)
    const bool full = a_vec && b_vec && (m0 + BM <= g.M) && (n0 + BN <= g.N) && ((ke - kb) % BK == 0);
    auto load_ab = [&](int64_t k0) {
        // A planes are cut along K (TA = 0, per slice) or along M (TA = 1, per tile)
        const float* Ab = plane_base(g.A, TA ? m0 : k0, g.a_blk, g.a_pstride);
        if (full) {
            load_slice<AK, BM, BK, NT, true>(Ab, g.lda, g.M, m0, k0, ke, a_vec, ra);
            load_slice<BKc, BN, BK, NT, true>(g.B, g.ldb, g.N, n0, k0, ke, b_vec, rb);
        } else {
            load_slice<AK, BM, BK, NT>(Ab, g.lda, g.M, m0, k0, ke, a_vec, ra);
            load_slice<BKc, BN, BK, NT>(g.B, g.ldb, g.N, n0, k0, ke, b_vec, rb);
        }
    };
    // Pipeline (guide T14 order): slice t+1 is written to LDS right AFTER the barrier that
    // frees its buffer, slice t+2 is loaded into registers immediately, then slice t is
    // multiplied; the LDS-write latency and the global-load latency both hide under the MFMAs.
    if (nk > 0) {
        load_ab(kb);
        store_slice<AK, BM, BK, LDA_S, NT>(As[0], ra);
        store_slice<BKc, BN, BK, LDB_S, NT>(Bs[0], rb);
        if (nk > 1) load_ab(kb + BK);
    }
    __syncthreads();

    const int li = lane & 31, lk = lane >> 5;
    for (int64_t kt = 0; kt < nk; ++kt) {
        const int cur = kt & 1;
        if (kt + 1 < nk) {
            store_slice<AK, BM, BK, LDA_S, NT>(As[cur ^ 1], ra);
            store_slice<BKc, BN, BK, LDB_S, NT>(Bs[cur ^ 1], rb);
        }
        if (kt + 2 < nk) load_ab(kb + (kt + 2) * BK);
        const float* as = As[cur] + wm * (BM / WM) + li;
        const float* bs = Bs[cur] + wn * (BN / WN) + li;
#pragma unroll
        for (int kk = 0; kk < BK / 2; ++kk) {
            const int kr = 2 * kk + lk;
            float a[TM], b[TN];
#pragma unroll
            for (int i = 0; i < TM; ++i) a[i] = as[kr * LDA_S + i * 32];
#pragma unroll
            for (int j = 0; j < TN; ++j) b[j] = bs[kr * LDB_S + j * 32];
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], b[j], acc[i][j], 0, 0, 0);
        }
        __syncthreads();
    }

    // epilogue: C/D map of 32x32 MFMA: col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)
    float* __restrict__ dst = g.split > 1 ? g.ws + (int64_t)blockIdx.y * g.M * g.N
                                          : const_cast<float*>(plane_base(g.C, n0, g.c_blk, g.c_pstride));
    const int64_t ldd = g.split > 1 ? g.N : g.ldc;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int64_t col = n0 + wn * (BN / WN) + j * 32 + li;
            if (col >= g.N) continue;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int64_t row = m0 + wm * (BM / WM) + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lk;
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

// Split-K stage 1 for many slabs over a small C (the skinny weight gradients: a few thousand
// outputs, up to 512 slabs): slab group g of `per` slabs is summed into its first slab, in
// place (each thread reads its element of the group's slabs before writing it; no other
// thread touches that element). Coalesced over the elements; fixed summation order.
__global__ __launch_bounds__(256) void k_splitk_stage1(float* __restrict__ ws, int split, int64_t total, int per) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int s0 = blockIdx.y * per, s1 = min(split, s0 + per);
    if (i >= total || s0 >= s1) return;
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    int k = s0;
    for (; k + 4 <= s1; k += 4) {
#pragma unroll
        for (int u = 0; u < 4; ++u) acc[u] += ws[(int64_t)(k + u) * total + i];
    }
    for (; k < s1; ++k) acc[0] += ws[(int64_t)k * total + i];
    ws[(int64_t)s0 * total + i] = (acc[0] + acc[1]) + (acc[2] + acc[3]);
}

// C = act(alpha * sum of the slabs s = 0, stride, 2 stride, ... < split + beta C + bias)
__global__ __launch_bounds__(256) void k_splitk_reduce(const float* __restrict__ ws, int split, int stride, int64_t M,
                                                       int64_t N, float alpha, float beta, float* __restrict__ C,
                                                       int64_t ldc, const float* __restrict__ bias, int relu,
                                                       int64_t c_blk, int64_t c_pstride) {
    const int64_t total = M * N;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (int64_t)gridDim.x * blockDim.x) {
        float s = 0.f;
        for (int k = 0; k < split; k += stride) s += ws[(int64_t)k * total + i];
        const int64_t r = i / N, c = i % N;
        float v = alpha * s;
        float* Cp = c_blk > 0 ? C + (c / c_blk) * (c_pstride - c_blk) : C;
        if (beta != 0.f) v += beta * Cp[r * ldc + c];
        if (bias) v += bias[c];
        if (relu) v = fmaxf(v, 0.f);
        Cp[r * ldc + c] = v;
    }
}

// float4 form of k_splitk_reduce (N, ldc, c_blk multiples of 4, C and bias 16-B aligned): the
// same sum over the slabs in the same order per element, four elements per thread (the SAGE
// weight gradients' 32 slabs of [1024, 512]: a scalar element per thread ran at ~4 TB/s)
__global__ __launch_bounds__(256) void k_splitk_reduce4(const float4* __restrict__ ws, int split, int stride,
                                                        int64_t M, int64_t N, float alpha, float beta,
                                                        float* __restrict__ C, int64_t ldc,
                                                        const float* __restrict__ bias, int relu, int64_t c_blk,
                                                        int64_t c_pstride) {
    const int64_t total4 = M * N / 4;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total4;
         i += (int64_t)gridDim.x * blockDim.x) {
        float sx = 0.f, sy = 0.f, sz = 0.f, sw = 0.f;
#pragma unroll 8
        for (int k = 0; k < split; k += stride) {
            const float4 t = ws[(int64_t)k * total4 + i];
            sx += t.x;
            sy += t.y;
            sz += t.z;
            sw += t.w;
        }
        const int64_t e = 4 * i;
        const int64_t r = e / N, c = e % N;
        float* Cp = c_blk > 0 ? C + (c / c_blk) * (c_pstride - c_blk) : C;
        float v[4] = {alpha * sx, alpha * sy, alpha * sz, alpha * sw};
        float4* dst = reinterpret_cast<float4*>(Cp + r * ldc + c);
        if (beta != 0.f) {
            const float4 o = *dst;
            v[0] += beta * o.x; v[1] += beta * o.y; v[2] += beta * o.z; v[3] += beta * o.w;
        }
        if (bias) {
            const float4 b = *reinterpret_cast<const float4*>(bias + c);
            v[0] += b.x; v[1] += b.y; v[2] += b.z; v[3] += b.w;
        }
        if (relu) {
#pragma unroll
            for (int q = 0; q < 4; ++q) v[q] = fmaxf(v[q], 0.f);
        }
        *dst = make_float4(v[0], v[1], v[2], v[3]);
    }
}

struct GemmCfg {
    int bm, bn, bk, waves, blocks_per_cu;
};
// tile configurations (index = bgnn_gemm_set_cfg value)
constexpr GemmCfg kCfgs[] = {
    {128, 128, 16, 4, 3},   // 0: 2x2 waves of 64x64
    {256, 256, 16, 8, 1},   // 1: 2x4 waves of 128x64 (2 waves/SIMD)
    {256, 256, 16, 4, 1},   // 2: 2x2 waves of 128x128 (1 wave/SIMD)
    {256, 128, 16, 8, 1},   // 3: 4x2 waves of 64x64
    {256, 128, 16, 4, 1},   // 4: 2x2 waves of 128x64
    {128, 256, 16, 8, 1},   // 5: 2x4 waves of 64x64
    {128, 256, 32, 8, 1},   // 6: as 5, BK = 32
    {256, 256, 32, 8, 1},   // 7: as 1, BK = 32
    {256, 128, 32, 8, 1},   // 8: as 3, BK = 32
};
constexpr int kNumCfgs = 9;
static int g_gemm_cfg = -1;   // -1 = automatic
static int g_gemm_mode = 2;   // 0 = f32 MFMA kernel (gemm.hip), 2 = f16x3 (gemm_x6.hip, default: error
                              // below the f32 MFMA's at 3 f16 MFMAs per product; tools/tune_gemm.py)

void set_gemm_mode(int mode) { g_gemm_mode = mode; }
int gemm_mode() { return g_gemm_mode; }


// f16x3 / bf16-operand tile choice (tools/tune_gemm.py)
// f16x3 (MI355X, tools/gemm_one.py under rocprofv3, cfg2 SAGE shapes): fwd 80656x1024x512
// 256x256 tiles 293 us (256x128: 341); dgrad 80656x512x1024 128x256 311 us (256x128: 329,
// 256x256: 323, under-filled last wave); wgrad 1024x512x80656 256x256 + split-K 302 us
// (256x128: 604 -- half the operand re-reads).
inline int pick_x6_cfg(int64_t M, int64_t N, int64_t K, int prec, bool h3_nt = false) {
    // (h3_nt: the f16x3 family's NT product, C = A B^T -- the only one built with cfg 5)
    if (h3_nt && M >= 4096 && N == 128 && (M + 255) / 256 < 384) {
        // a tall N = 128 product has one column tile: 256-row tiles give 1.2 rounds of 256 CUs (the
        // folded layer's input gradient, 316 tiles), 8-wave 128 x 128 tiles 2.5 rounds; the same
        // 16x16x32 MFMA order per element, so the same bits
        return 5;
    }
    if (prec == 1) {
        if (M >= 4096 && N >= 1024) return 4;
        if (M >= 4096 && N >= 256) return 2;
        if (M >= 256 && N >= 256 && K >= 8192) return 4;
    }
    if (M >= 4096 && N >= 128) return 1;              // tall (fwd / dgrad)
    if (M >= 256 && N >= 128 && K >= 8192) return 1;  // short and deep (wgrad, split-K)
    return 0;
}

// Measured on MI355X (tools/tune_gemm.py, SAGE layer shapes): 256x128 tiles of 8 waves for
// the tall GEMMs (fwd 118 TF, dgrad 118 TF), 256x256 tiles of 8 waves + split-K for the
// short-and-deep weight gradient (125 TF); small problems keep the 128x128 tile.
inline int pick_cfg(int64_t M, int64_t N, int64_t K, int ta, int tb) {
    (void)ta; (void)tb;
    if (g_gemm_cfg >= 0) return g_gemm_cfg % kNumCfgs;
    if (M >= 256 && N >= 256 && K >= 8192 && M * N <= (int64_t)4096 * 4096) return 1;
    if (M >= 4096 && N >= 128) return 3;
    return 0;
}

inline int choose_split(int64_t M, int64_t N, int64_t K, const GemmCfg& c) {
    const int64_t tiles = ((M + c.bm - 1) / c.bm) * ((N + c.bn - 1) / c.bn);
    const int64_t slots = 256 * c.blocks_per_cu;          // resident workgroups on the chip
    if (tiles >= slots / 2 || K < 4 * 256) return 1;
    int64_t s = (slots + tiles - 1) / tiles;
    const int64_t smax = K / 256;   // keep >= 256 of K per slice
    if (s > smax) s = smax;
    // skinny weight gradients (a handful of tiles, K = node count) need many slices to fill the
    // chip: the encoder's 64x128 / 16x64 wgrads ran on 64 workgroups at the old cap of 64
    if (s > 512) s = 512;
    return s < 1 ? 1 : (int)s;
}

template <int TA, int TB>
void launch_cfg(int cfg, dim3 grid, hipStream_t s, const GemmArgs& g) {
    switch (cfg) {
        case 1: hipLaunchKernelGGL((k_gemm_f32<TA, TB, 256, 256, 16, 2, 4>), grid, dim3(512), 0, s, g); break;
        case 2: hipLaunchKernelGGL((k_gemm_f32<TA, TB, 256, 256, 16, 2, 2>), grid, dim3(256), 0, s, g); break;
        case 3: hipLaunchKernelGGL((k_gemm_f32<TA, TB, 256, 128, 16, 4, 2>), grid, dim3(512), 0, s, g); break;
        case 4: hipLaunchKernelGGL((k_gemm_f32<TA, TB, 256, 128, 16, 2, 2>), grid, dim3(256), 0, s, g); break;
        case 5: hipLaunchKernelGGL((k_gemm_f32<TA, TB, 128, 256, 16, 2, 4>), grid, dim3(512), 0, s, g); break;
        case 6: hipLaunchKernelGGL((k_gemm_f32<TA, TB, 128, 256, 32, 2, 4>), grid, dim3(512), 0, s, g); break;
        case 7: hipLaunchKernelGGL((k_gemm_f32<TA, TB, 256, 256, 32, 2, 4>), grid, dim3(512), 0, s, g); break;
        case 8: hipLaunchKernelGGL((k_gemm_f32<TA, TB, 256, 128, 32, 4, 2>), grid, dim3(512), 0, s, g); break;
        default: hipLaunchKernelGGL((k_gemm_f32<TA, TB, 128, 128, 16, 2, 2>), grid, dim3(256), 0, s, g); break;
    }
}

}  // namespace bgnn

using namespace bgnn;

extern "C" int bgnn_gemm_set_cfg(int32_t cfg) {
    // (-1 = automatic; the f16x3 / bf16 families have kNumX6Cfgs tiles, the f32 MFMA family kCfgs)
    const int n = g_gemm_mode == 0 ? kNumCfgs : kNumX6Cfgs;
    BGNN_REQUIRE(cfg >= -1 && cfg < n, "gemm: config %d out of range [-1, %d)", cfg, n);
    g_gemm_cfg = cfg;
    return BGNN_OK;
}

// Launch plan of one GEMM call: kernel family, tile config and split-K factor.
struct Plan {
    int x6;            // 1 = split-precision kernel (gemm_x6.hip), 0 = f32 MFMA
    int prec;          // split kernel: 1 = f16x3, 2 = bf16 operands
    int cfg;           // index into kX6Cfgs / kCfgs
    int bm, bn, bk;    // tile
    int split;
};

static Plan make_plan(int64_t M, int64_t N, int64_t K, int ta, int tb, int64_t a_blk, int64_t c_blk,
                      int precision = 0, bool wb = false) {
    Plan p{};
    auto planes_ok = [&](int bm, int bn, int bk) {
        return (a_blk == 0 || a_blk % (ta ? bm : bk) == 0) && (c_blk == 0 || c_blk % bn == 0);
    };
    if (precision == 1) {   // bf16 operands, f32 accumulation (the split kernel with one piece)
        p.x6 = 1;
        p.prec = 2;
        p.cfg = g_gemm_cfg >= 0 ? g_gemm_cfg % kNumX6Cfgs : pick_x6_cfg(M, N, K, 1);
        if (p.cfg == 5) p.cfg = 1;   // (the 8-wave 128 x 128 tile is built for f16x3 only)
        // plane blocks must be whole tiles (every bf16 tile gives the same bits: 16x16x32 MFMAs
        // in increasing k), else the 128x128 tile
        if (!planes_ok(kX6Cfgs[p.cfg].bm, kX6Cfgs[p.cfg].bn, 32)) p.cfg = 0;
        p.bm = kX6Cfgs[p.cfg].bm; p.bn = kX6Cfgs[p.cfg].bn; p.bk = 32;
        p.split = choose_split(M, N, K, GemmCfg{p.bm, p.bn, p.bk, kX6Cfgs[p.cfg].waves, kX6Cfgs[p.cfg].blocks_per_cu});
        return p;
    }
    if (g_gemm_mode == 2) {
        p.x6 = 1;
        p.prec = 1;
        p.cfg = g_gemm_cfg >= 0 ? g_gemm_cfg % kNumX6Cfgs : pick_x6_cfg(M, N, K, p.prec, ta == 0 && tb == 1);
        // (cfg 5 is built for the f16x3 NT product only: a forced cfg 5 elsewhere takes 256 x 128)
        if (p.cfg == 5 && !(ta == 0 && tb == 1)) p.cfg = 1;
        // knob 16 = 4: the pre-split products on the pipelined 128 x 128 kernel (gemm_h3p.hip)
#ifdef BGNN_H3P_ABLATION
        if (wb && g_x6_bdma == 4 && g_gemm_cfg < 0 && N % 128 == 0 && K % 32 == 0) p.cfg = 0;
#endif
        // plane blocks must be whole tiles: fall back to an 8-wave tile that divides them (the
        // 16x16x32 MFMA family, the same rounding as the dense layout's), else the 128x128 tile
        if (!planes_ok(kX6Cfgs[p.cfg].bm, kX6Cfgs[p.cfg].bn, 32)) {
            p.cfg = 0;
            for (int c = 1; c <= 2; ++c)
                if (planes_ok(kX6Cfgs[c].bm, kX6Cfgs[c].bn, 32)) { p.cfg = c; break; }
        }
        p.bm = kX6Cfgs[p.cfg].bm; p.bn = kX6Cfgs[p.cfg].bn; p.bk = 32;
        p.split = choose_split(M, N, K, GemmCfg{p.bm, p.bn, p.bk, kX6Cfgs[p.cfg].waves,
                                                 kX6Cfgs[p.cfg].blocks_per_cu});
        return p;
    } else {
        p.cfg = pick_cfg(M, N, K, ta, tb);
        // plane blocks must be whole multiples of the tile along the split dimension; fall back
        // to the smallest tile when the shape-picked one does not divide them
        if (!planes_ok(kCfgs[p.cfg].bm, kCfgs[p.cfg].bn, kCfgs[p.cfg].bk)) p.cfg = 0;
        const GemmCfg& c = kCfgs[p.cfg];
        p.bm = c.bm; p.bn = c.bn; p.bk = c.bk;
        p.split = choose_split(M, N, K, c);
    }
    return p;
}

// workspace: [256 B operand-max head (f16x3)] [split-K slabs]
constexpr size_t kAmaxHead = 256;

static size_t ws_need(const Plan& p, int64_t M, int64_t N) {
    const size_t head = (p.x6 && p.prec == 1) ? kAmaxHead : 0;
    return head + (p.split > 1 ? (size_t)p.split * (size_t)M * (size_t)N * sizeof(float) : 0);
}

// slab reduce of a split-K GEMM: C = act(alpha * sum of slabs + beta C + bias)
static int launch_splitk_reduce(float* slabs, int split, int64_t M, int64_t N, float alpha, float beta, float* C,
                                int64_t ldc, const float* bias, int relu, int64_t c_blk, int64_t c_pstride,
                                hipStream_t s) {
    int64_t blocks = (M * N + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    // few outputs, many slabs: sum slab groups first so the reduction spreads over >= ~512
    // workgroups instead of one serial sum per output element (encoder wgrads: 100 -> ~10 us)
    int stride = 1;
    const int64_t eb = (M * N + 255) / 256;
    if (split >= 16 && eb < 512) {
        int64_t groups = (512 + eb - 1) / eb;
        if (groups > split / 4) groups = split / 4;
        if (groups >= 2) {
            stride = (int)((split + groups - 1) / groups);
            groups = (split + stride - 1) / stride;
            hipLaunchKernelGGL(k_splitk_stage1, dim3((unsigned)eb, (unsigned)groups), dim3(256), 0, s, slabs, split,
                               M * N, stride);
            BGNN_CHECK_LAUNCH();
        }
    }
    const bool vec4 = N % 4 == 0 && ldc % 4 == 0 && (c_blk == 0 || (c_blk % 4 == 0 && c_pstride % 4 == 0)) &&
                      (((uintptr_t)C & 15) == 0) && (!bias || (((uintptr_t)bias & 15) == 0)) &&
                      (((uintptr_t)slabs & 15) == 0);
    if (vec4) {
        int64_t b4 = (M * N / 4 + 255) / 256;
        if (b4 > blocks) b4 = blocks;
        if (b4 < 1) b4 = 1;
        hipLaunchKernelGGL(k_splitk_reduce4, dim3((unsigned)b4), dim3(256), 0, s, (const float4*)slabs, split, stride,
                           M, N, alpha, beta, C, ldc, bias, relu, c_blk, c_pstride);
    } else {
        hipLaunchKernelGGL(k_splitk_reduce, dim3((unsigned)blocks), dim3(256), 0, s, (const float*)slabs, split,
                           stride, M, N, alpha, beta, C, ldc, bias, relu, c_blk, c_pstride);
    }
    BGNN_CHECK_LAUNCH();
    return BGNN_OK;
}

extern "C" size_t bgnn_gemm_ws_bytes(int64_t M, int64_t N, int64_t K, int32_t ta, int32_t tb) {
    return ws_need(make_plan(M, N, K, ta, tb, 0, 0), M, N);
}

extern "C" size_t bgnn_gemm_ws_bytes_ex(int64_t M, int64_t N, int64_t K, int32_t ta, int32_t tb, int32_t precision) {
    return ws_need(make_plan(M, N, K, ta, tb, 0, 0, precision), M, N);
}

extern "C" int bgnn_absmax_f32(const float* x, int64_t rows, int64_t cols, int64_t ld, float* out,
                               int32_t accumulate, void* stream) {
    BGNN_REQUIRE(rows >= 0 && cols >= 0 && (ld >= cols || rows <= 1), "absmax: bad shape");
    BGNN_REQUIRE(out != nullptr, "absmax: null output");
    hipStream_t s = as_stream(stream);
    if (!accumulate) BGNN_HIP(hipMemsetAsync(out, 0, sizeof(float), s));
    if (rows > 0 && cols > 0) {
        launch_absmax(x, rows, cols, ld, 0, 0, out, s);
        BGNN_CHECK_LAUNCH();
    }
    return BGNN_OK;
}

// beta operand from a dropout-masked source (bgnn_gemm_f32_dropadd); NULL src = from C
struct BetaSrc {
    const float* src;
    int64_t ld;
    uint64_t seed;
    float p;
    int64_t c0;   // first column that takes it (bgnn_gemm_f32_dropadd_cols)
};

static int gemm_scaled_impl(int32_t ta, int32_t tb, int64_t M, int64_t N, int64_t K, float alpha,
                            const float* A, int64_t lda, int64_t a_blk, int64_t a_pstride, const float* B,
                            int64_t ldb, float beta, float* C, int64_t ldc, int64_t c_blk,
                            int64_t c_pstride, const float* bias, int32_t relu, const float* a_amax,
                            const float* b_amax, float* c_amax, int32_t precision, void* ws,
                            size_t ws_bytes, void* stream, const BetaSrc& bs, int st = 0);

extern "C" int bgnn_gemm_f32_scaled(int32_t ta, int32_t tb, int64_t M, int64_t N, int64_t K, float alpha,
                                    const float* A, int64_t lda, int64_t a_blk, int64_t a_pstride, const float* B,
                                    int64_t ldb, float beta, float* C, int64_t ldc, int64_t c_blk,
                                    int64_t c_pstride, const float* bias, int32_t relu, const float* a_amax,
                                    const float* b_amax, float* c_amax, int32_t precision, void* ws,
                                    size_t ws_bytes, void* stream) {
    return gemm_scaled_impl(ta, tb, M, N, K, alpha, A, lda, a_blk, a_pstride, B, ldb, beta, C, ldc, c_blk,
                            c_pstride, bias, relu, a_amax, b_amax, c_amax, precision, ws, ws_bytes, stream,
                            BetaSrc{nullptr, 0, 0, 0.f, 0});
}

extern "C" int bgnn_gemm_f32_dropadd(int32_t ta, int32_t tb, int64_t M, int64_t N, int64_t K, const float* A,
                                     int64_t lda, const float* B, int64_t ldb, float* C, int64_t ldc,
                                     const float* a_amax, const float* b_amax, const float* src, int64_t ld_src,
                                     float p, uint64_t seed, void* ws, size_t ws_bytes, void* stream) {
    BGNN_REQUIRE(src != nullptr && ld_src >= N && ld_src % 4 == 0 && N % 4 == 0 && ((uintptr_t)src & 15) == 0,
                 "gemm_dropadd: src must be 16-byte aligned with N and ld_src multiples of 4");
    BGNN_REQUIRE(gemm_mode() == 2 && ta == 0 && tb == 1,
                 "gemm_dropadd: built for the f16x3 family (BGNN_TUNE_GEMM_MODE 2) and C = A B^T only");
    return gemm_scaled_impl(ta, tb, M, N, K, 1.f, A, lda, 0, 0, B, ldb, 1.f, C, ldc, 0, 0, nullptr, 0, a_amax,
                            b_amax, nullptr, 0, ws, ws_bytes, stream, BetaSrc{src, ld_src, seed, p, 0});
}

extern "C" int bgnn_gemm_f32_dropadd_cols(int64_t M, int64_t N, int64_t K, const float* A, int64_t lda,
                                          const float* B, int64_t ldb, float* C, int64_t ldc, const float* a_amax,
                                          const float* b_amax, const float* src, int64_t ld_src, int64_t src_col0,
                                          float p, uint64_t seed, void* ws, size_t ws_bytes, void* stream) {
    BGNN_REQUIRE(src != nullptr && src_col0 >= 0 && src_col0 < N && ld_src >= N - src_col0 && ld_src % 4 == 0 &&
                     N % 4 == 0 && ((uintptr_t)src & 15) == 0,
                 "gemm_dropadd_cols: src must be 16-byte aligned, cover columns [src_col0, N), ld_src % 4 == 0");
    BGNN_REQUIRE(gemm_mode() == 2, "gemm_dropadd_cols: built for the f16x3 family (BGNN_TUNE_GEMM_MODE 2)");
    const Plan pl = make_plan(M, N, K, 0, 1, 0, 0);
    BGNN_REQUIRE(pl.x6 && pl.split == 1 && src_col0 % pl.bn == 0,
                 "gemm_dropadd_cols: src_col0 %lld must be a multiple of the column tile %d (no split-K)",
                 (long long)src_col0, pl.bn);
    return gemm_scaled_impl(0, 1, M, N, K, 1.f, A, lda, 0, 0, B, ldb, 1.f, C, ldc, 0, 0, nullptr, 0, a_amax, b_amax,
                            nullptr, 0, ws, ws_bytes, stream, BetaSrc{src, ld_src, seed, p, src_col0});
}

extern "C" int32_t bgnn_gemm_w_tile(int64_t M, int64_t N, int64_t K) {
    if (gemm_mode() != 2 || M <= 0 || N <= 0 || K <= 0) return 0;
    const Plan pl = make_plan(M, N, K, 0, 1, 0, 0, 0, true);
    if (!pl.x6 || pl.prec != 1 || pl.split != 1 || pl.cfg > 4 || (pl.cfg < 1 && g_x6_bdma != 4)) return 0;
    if (N % pl.bn != 0 || K % 32 != 0) return 0;
    return pl.bn;
}

// C = A W^T (+ drop(src)) with W given as its pre-split image (bgnn_gemm_wsplit with column tile
// bn = bgnn_gemm_w_tile(M, N, K)): the f16x3 kernel stages W by LDS-DMA, A as bgnn_gemm_f32_scaled.
extern "C" int bgnn_gemm_f32_w(int64_t M, int64_t N, int64_t K, const float* A, int64_t lda, const void* wimg,
                               int32_t bn, float* C, int64_t ldc, const float* bias, int32_t relu,
                               const float* a_amax, const float* b_amax, float* c_amax, const float* src,
                               int64_t ld_src, float p, uint64_t seed, void* stream) {
    BGNN_REQUIRE(A && wimg && C && a_amax && b_amax, "gemm_f32_w: null pointer");
    BGNN_REQUIRE(lda >= K && ldc >= N, "gemm_f32_w: bad lda / ldc");
    if (M == 0 || N == 0) return BGNN_OK;
    const int32_t tile = bgnn_gemm_w_tile(M, N, K);
    BGNN_REQUIRE(tile != 0 && tile == bn, "gemm_f32_w: image column tile %d, plan tile %d (bgnn_gemm_w_tile)", bn,
                 tile);
    BGNN_REQUIRE(!src || (ld_src >= N && ld_src % 4 == 0 && N % 4 == 0 && ((uintptr_t)src & 15) == 0),
                 "gemm_f32_w: src must be 16-byte aligned with N and ld_src multiples of 4");
    const Plan pl = make_plan(M, N, K, 0, 1, 0, 0, 0, true);
    BGNN_REQUIRE(pl.cfg != 0 || (lda % 4 == 0 && aligned16(A)),
                 "gemm_f32_w: the 128 x 128 pipelined tile needs 16-byte aligned A rows");
    GemmArgs g{A, static_cast<const float*>(wimg), C, nullptr, M, N, K, lda, K, ldc, 1.f, src ? 1.f : 0.f, 0, 1,
               bias, relu, 0, 0, 0, 0, a_amax, b_amax, c_amax};
    g.kchunk = (K + pl.bk - 1) / pl.bk * pl.bk;
    g.wb = 1;
    if (src) {
        g.bsrc = src;
        g.ld_bsrc = ld_src;
        g.dseed = seed;
        g.dthr = dropout_threshold(p);
        g.dkeep = g.dthr ? 1.f / (1.f - p) : 1.f;
    }
    const int64_t tiles = ((M + pl.bm - 1) / pl.bm) * ((N + pl.bn - 1) / pl.bn);
    launch_x6(1, 0, 1, pl.cfg, src ? 8 : 0, dim3((unsigned)tiles, 1), as_stream(stream), g);
    BGNN_CHECK_LAUNCH();
    return BGNN_OK;
}

static int gemm_scaled_impl(int32_t ta, int32_t tb, int64_t M, int64_t N, int64_t K, float alpha,
                            const float* A, int64_t lda, int64_t a_blk, int64_t a_pstride, const float* B,
                            int64_t ldb, float beta, float* C, int64_t ldc, int64_t c_blk,
                            int64_t c_pstride, const float* bias, int32_t relu, const float* a_amax,
                            const float* b_amax, float* c_amax, int32_t precision, void* ws,
                            size_t ws_bytes, void* stream, const BetaSrc& bs, int st) {
    BGNN_REQUIRE((ta == 0 || ta == 1) && (tb == 0 || tb == 1), "gemm: bad transpose flags");
    BGNN_REQUIRE(st == 0 || (precision == 1 && a_blk == 0 && c_blk == 0 && !bs.src && c_amax == nullptr &&
                             (!(st & 4) || beta == 0.f)),
                 "gemm: bf16 storage needs the bf16-operand family, dense operands, no max|C| and beta 0 for a bf16 C");
    BGNN_REQUIRE(M >= 0 && N >= 0 && K >= 0, "gemm: negative size");
    const int64_t a_inner = a_blk > 0 ? a_blk : (ta ? M : K);
    BGNN_REQUIRE((ta == 0 && lda >= a_inner) || (ta == 1 && lda >= a_inner) || M == 0 || K == 0, "gemm: bad lda");
    BGNN_REQUIRE((tb == 0 && ldb >= N) || (tb == 1 && ldb >= K) || N == 0 || K == 0, "gemm: bad ldb");
    BGNN_REQUIRE(ldc >= (c_blk > 0 ? c_blk : N) || M == 0, "gemm: bad ldc");
    BGNN_REQUIRE(a_blk >= 0 && c_blk >= 0, "gemm: negative plane block");
    BGNN_REQUIRE(precision == 0 || precision == 1, "gemm: precision must be 0 (f32-accurate) or 1 (bf16)");
    if (M == 0 || N == 0) return BGNN_OK;
    Plan pl = make_plan(M, N, K, ta, tb, a_blk, c_blk, precision);
    // the drop-add epilogue preloads its whole masked tile (32 float4 per lane at 256x256, where the
    // accumulators already fill the VGPRs: it spilled, 365 us for the max layer's N = 1024 merged
    // dgrad): 128x256 tiles, as the SAGE dgrad's
    if (bs.src && pl.x6 && pl.prec == 1 && (pl.cfg == 3 || pl.cfg == 4) && g_gemm_cfg < 0) {
        pl.cfg = 2;
        pl.bm = kX6Cfgs[2].bm;
        pl.bn = kX6Cfgs[2].bn;
    }
    BGNN_REQUIRE((a_blk == 0 || a_blk % (ta ? pl.bm : pl.bk) == 0) && (c_blk == 0 || c_blk % pl.bn == 0),
                 "gemm: plane blocks (a_blk %lld, c_blk %lld) must be multiples of the %dx%dx%d tile",
                 (long long)a_blk, (long long)c_blk, pl.bm, pl.bn, pl.bk);
    const int64_t tiles = ((M + pl.bm - 1) / pl.bm) * ((N + pl.bn - 1) / pl.bn);
    BGNN_REQUIRE(tiles < (int64_t(1) << 31), "gemm: too many tiles");
    hipStream_t s = as_stream(stream);
    const bool h3 = pl.x6 && pl.prec == 1;
    const size_t head = h3 ? kAmaxHead : 0;
    if (h3) {
        BGNN_REQUIRE(ws != nullptr && ws_bytes >= head, "gemm: f16x3 needs the workspace of bgnn_gemm_ws_bytes()");
        // operand maxima not supplied by the caller: one pass over each operand
        float* head_amax = static_cast<float*>(ws);
        if (a_amax == nullptr || b_amax == nullptr) BGNN_HIP(hipMemsetAsync(ws, 0, 2 * sizeof(float), s));
        if (a_amax == nullptr) {
            launch_absmax(A, ta ? K : M, ta ? M : K, lda, a_blk, a_pstride, head_amax, s);
            BGNN_CHECK_LAUNCH();
            a_amax = head_amax;
        }
        if (b_amax == nullptr) {
            launch_absmax(B, tb ? N : K, tb ? K : N, ldb, 0, 0, head_amax + 1, s);
            BGNN_CHECK_LAUNCH();
            b_amax = head_amax + 1;
        }
    }
    float* slabs = ws ? reinterpret_cast<float*>(static_cast<char*>(ws) + head) : nullptr;
    const size_t slab_bytes = ws_bytes > head ? ws_bytes - head : 0;
    int split = pl.split;
    if (split > 1 && (slabs == nullptr || slab_bytes < (size_t)split * M * N * sizeof(float))) split = 1;
    if (st & 4) split = 1;   // (a bf16 C has no f32 slab reduce)
    if (bs.src) {   // the masked beta source lives in the split kernels' epilogue: no split-K
        BGNN_REQUIRE(pl.x6 && pl.prec == 1, "gemm_dropadd: needs the f16x3 kernels");
        split = 1;
    }
    if ((st & 3) == 3 && alpha == 1.f && beta == 0.f) {   // bf16-stored A and B: the LDS-DMA bf16 kernel, all rows
        GemmArgs gb{A, B, C, nullptr, M, N, K, lda, ldb, ldc, 1.f, 0.f, K, 1, bias, relu,
                    0, 0, 0, 0, nullptr, nullptr, nullptr};
        gb.st = st;
        if (b16_ok(gb, ta, tb)) {
            launch_b16(s, gb);
            BGNN_CHECK_LAUNCH();
            return BGNN_OK;
        }
    }
    const int64_t Ma = M;
    GemmArgs g{A, B, C, slabs, Ma, N, K, lda, ldb, ldc, alpha, beta, 0, split, bias, relu,
               a_blk, a_pstride, c_blk, c_pstride, a_amax, b_amax, nullptr};
    g.st = st;
    if (bs.src) {
        g.bsrc = bs.src;
        g.ld_bsrc = bs.ld;
        g.dseed = bs.seed;
        g.dthr = dropout_threshold(bs.p);
        g.dkeep = g.dthr ? 1.f / (1.f - bs.p) : 1.f;
        g.bsrc_c0 = bs.c0;
    }
    // max |C| for the next GEMM's operand scale: in the split kernels' epilogue, else one pass
    const bool c_amax_fused = c_amax != nullptr && pl.x6 && split == 1;
    if (c_amax_fused) g.c_amax = c_amax;
    int64_t kc = (K + split - 1) / split;
    kc = (kc + pl.bk - 1) / pl.bk * pl.bk;
    g.kchunk = kc > 0 ? kc : pl.bk;
    const int64_t tiles_a = ((Ma + pl.bm - 1) / pl.bm) * ((N + pl.bn - 1) / pl.bn);
    dim3 grid((unsigned)tiles_a, split);
    if (pl.x6) launch_x6(pl.prec, ta, tb, pl.cfg, bs.src ? 8 : 0, grid, s, g);
    else if (ta == 0 && tb == 0) launch_cfg<0, 0>(pl.cfg, grid, s, g);
    else if (ta == 0 && tb == 1) launch_cfg<0, 1>(pl.cfg, grid, s, g);
    else if (ta == 1 && tb == 0) launch_cfg<1, 0>(pl.cfg, grid, s, g);
    else launch_cfg<1, 1>(pl.cfg, grid, s, g);
    BGNN_CHECK_LAUNCH();
    if (split > 1) {
        const int rc = launch_splitk_reduce(slabs, split, M, N, alpha, beta, C, ldc, bias, relu, c_blk, c_pstride, s);
        if (rc != BGNN_OK) return rc;
    }
    if (c_amax != nullptr && !c_amax_fused) {
        launch_absmax(C, M, N, ldc, c_blk, c_pstride, c_amax, s);
        BGNN_CHECK_LAUNCH();
    }
    return BGNN_OK;
}

extern "C" int bgnn_gemm_f32_planes(int32_t ta, int32_t tb, int64_t M, int64_t N, int64_t K, float alpha,
                                    const float* A, int64_t lda, int64_t a_blk, int64_t a_pstride, const float* B,
                                    int64_t ldb, float beta, float* C, int64_t ldc, int64_t c_blk,
                                    int64_t c_pstride, const float* bias, int32_t relu, void* ws, size_t ws_bytes,
                                    void* stream) {
    return bgnn_gemm_f32_scaled(ta, tb, M, N, K, alpha, A, lda, a_blk, a_pstride, B, ldb, beta, C, ldc, c_blk,
                                c_pstride, bias, relu, nullptr, nullptr, nullptr, 0, ws, ws_bytes, stream);
}

extern "C" int bgnn_gemm_f32_ex(int32_t ta, int32_t tb, int64_t M, int64_t N, int64_t K, float alpha,
                                const float* A, int64_t lda, const float* B, int64_t ldb, float beta, float* C,
                                int64_t ldc, const float* bias, int32_t relu, void* ws, size_t ws_bytes,
                                void* stream) {
    return bgnn_gemm_f32_planes(ta, tb, M, N, K, alpha, A, lda, 0, 0, B, ldb, beta, C, ldc, 0, 0, bias, relu, ws,
                                ws_bytes, stream);
}

extern "C" int bgnn_gemm_f32(int32_t ta, int32_t tb, int64_t M, int64_t N, int64_t K, float alpha, const float* A,
                             int64_t lda, const float* B, int64_t ldb, float beta, float* C, int64_t ldc, void* ws,
                             size_t ws_bytes, void* stream) {
    return bgnn_gemm_f32_planes(ta, tb, M, N, K, alpha, A, lda, 0, 0, B, ldb, beta, C, ldc, 0, 0, nullptr, 0, ws,
                                ws_bytes, stream);
}

// act(op(A) op(B) + bias + add0[idx0[row]] (+ add1[idx1[row]])) with the gathered rows added in
// the epilogue of the split kernels (no split-K). precision: 0 = f32-accurate (the split family of
// BGNN_TUNE_GEMM_MODE; the f32 MFMA family is not supported here), 1 = bf16 operands.
static int gather_add_impl(int32_t ta, int32_t tb, int64_t M, int64_t N, int64_t K, const float* A, int64_t lda,
                           const float* B, int64_t ldb, float* C, int64_t ldc, const float* bias, int32_t relu,
                           const float* add0, const int64_t* idx0, int64_t ld0, const float* add1,
                           const int64_t* idx1, int64_t ld1, int32_t precision, void* ws, size_t ws_bytes,
                           void* stream, int st) {
    BGNN_REQUIRE((ta == 0 || ta == 1) && (tb == 0 || tb == 1), "gemm_gather_add: bad transpose flags");
    BGNN_REQUIRE(M >= 0 && N >= 0 && K >= 0, "gemm_gather_add: negative size");
    BGNN_REQUIRE(precision == 0 || precision == 1, "gemm_gather_add: precision must be 0 or 1");
    BGNN_REQUIRE(add0 != nullptr && idx0 != nullptr && ld0 >= N, "gemm_gather_add: add0/idx0/ld0 required");
    BGNN_REQUIRE(add1 == nullptr || (idx1 != nullptr && ld1 >= N), "gemm_gather_add: bad add1/idx1/ld1");
    BGNN_REQUIRE((ta == 0 && lda >= K) || (ta == 1 && lda >= M) || M == 0 || K == 0, "gemm_gather_add: bad lda");
    BGNN_REQUIRE((tb == 0 && ldb >= N) || (tb == 1 && ldb >= K) || N == 0 || K == 0, "gemm_gather_add: bad ldb");
    BGNN_REQUIRE(ldc >= N || M == 0, "gemm_gather_add: bad ldc");
    if (M == 0 || N == 0) return BGNN_OK;
    Plan pl = make_plan(M, N, K, ta, tb, 0, 0, precision);
    BGNN_REQUIRE(pl.x6, "gemm_gather_add: needs the split GEMM family (BGNN_TUNE_GEMM_MODE 2)");
    const int64_t tiles = ((M + pl.bm - 1) / pl.bm) * ((N + pl.bn - 1) / pl.bn);
    BGNN_REQUIRE(tiles < (int64_t(1) << 31), "gemm_gather_add: too many tiles");
    hipStream_t s = as_stream(stream);
    const bool h3 = pl.prec == 1;
    const float* a_amax = nullptr;
    const float* b_amax = nullptr;
    if (h3) {
        BGNN_REQUIRE(ws != nullptr && ws_bytes >= kAmaxHead, "gemm_gather_add: f16x3 needs bgnn_gemm_ws_bytes_ex()");
        float* head_amax = static_cast<float*>(ws);
        BGNN_HIP(hipMemsetAsync(ws, 0, 2 * sizeof(float), s));
        launch_absmax(A, ta ? K : M, ta ? M : K, lda, 0, 0, head_amax, s);
        BGNN_CHECK_LAUNCH();
        launch_absmax(B, tb ? N : K, tb ? K : N, ldb, 0, 0, head_amax + 1, s);
        BGNN_CHECK_LAUNCH();
        a_amax = head_amax;
        b_amax = head_amax + 1;
    }
    GemmArgs g{A, B, C, nullptr, M, N, K, lda, ldb, ldc, 1.f, 0.f, 0, 1, bias, relu,
               0, 0, 0, 0, a_amax, b_amax, nullptr, add0, idx0, ld0, add1, idx1, ld1};
    g.st = st;
    g.kchunk = (K + pl.bk - 1) / pl.bk * pl.bk;
    if (g.kchunk == 0) g.kchunk = pl.bk;
    if (b16_ok(g, ta, tb)) launch_b16(s, g);   // bf16-stored A and B: the LDS-DMA bf16 kernel
    else launch_x6(pl.prec, ta, tb, pl.cfg, 0, dim3((unsigned)tiles, 1), s, g);
    BGNN_CHECK_LAUNCH();
    return BGNN_OK;
}

// C = round(round(A B^T) + drop(src)) with A [M, K], B [N, K], C and src [M, N] all bf16 (ABI 11):
// EA_GNN's edge Linear dgrad plus the skip + dropout's share of the same activation's gradient
// (bgnn/ea.py GradSlot), in the LDS-DMA kernel's epilogue -- the bits of bgnn_gemm_bf16 (storage 7)
// followed by bgnn_add_dropped_bf16(C, src), without C's write and read back. Mask: keep_bits4(seed,
// (row * ld_src + col) / 4), kept values / (1 - p); ld_src == N == ldc (the flat index the two-step
// form masks by). Forms other than the whole-line bf16 C kernel, and operands the LDS-DMA kernel does not
// take, run those two steps.
extern "C" int bgnn_add_dropped_bf16(const void* a, const void* b, int64_t n, float p, uint64_t seed, void* out,
                                     void* stream);
extern "C" int bgnn_gemm_bf16(int32_t ta, int32_t tb, int64_t M, int64_t N, int64_t K, float alpha, const void* A,
                              int64_t lda, const void* B, int64_t ldb, float beta, void* C, int64_t ldc,
                              const float* bias, int32_t relu, int32_t storage, void* ws, size_t ws_bytes,
                              void* stream);
extern "C" int bgnn_gemm_bf16_dropadd(int64_t M, int64_t N, int64_t K, const void* A, int64_t lda, const void* B,
                                      int64_t ldb, void* C, int64_t ldc, const void* src, int64_t ld_src, float p,
                                      uint64_t seed, void* stream) {
    BGNN_REQUIRE(M >= 0 && N >= 0 && K >= 0, "gemm_bf16_dropadd: negative size");
    BGNN_REQUIRE(p >= 0.f && p < 1.f, "gemm_bf16_dropadd: p must be in [0, 1)");
    BGNN_REQUIRE(ldc == N && ld_src == N && lda >= K && ldb >= K, "gemm_bf16_dropadd: need ldc == ld_src == N");
    if (M == 0 || N == 0) return BGNN_OK;
    BGNN_REQUIRE(A && B && C && src && N % 8 == 0, "gemm_bf16_dropadd: null pointer or N % 8 != 0");
    hipStream_t s = as_stream(stream);
    GemmArgs g{static_cast<const float*>(A), static_cast<const float*>(B), static_cast<float*>(C), nullptr,
               M, N, K, lda, ldb, ldc, 1.f, 0.f, K, 1, nullptr, 0, 0, 0, 0, 0, nullptr, nullptr, nullptr};
    g.st = 7;
    if (!b16_ok(g, 0, 1)) {   // (K % 64, alignment, lda / ldb % 8, or b16 variant -1): the two steps
        const int rc = bgnn_gemm_bf16(0, 1, M, N, K, 1.f, A, lda, B, ldb, 0.f, C, ldc, nullptr, 0, 7, nullptr, 0,
                                      stream);
        if (rc != BGNN_OK) return rc;
        return bgnn_add_dropped_bf16(C, src, M * N, p, seed, C, stream);
    }
    GemmArgs gd = g;
    gd.bsrc = static_cast<const float*>(src);
    gd.ld_bsrc = ld_src;
    gd.dseed = seed;
    gd.dthr = dropout_threshold(p);
    gd.dkeep = gd.dthr ? 1.f / (1.f - p) : 1.f;
    gd.st = 7 | 8;
    if (b16_dropadd_ok(gd)) {
        launch_b16(s, gd);
        BGNN_CHECK_LAUNCH();
        return BGNN_OK;
    }
    launch_b16(s, g);
    BGNN_CHECK_LAUNCH();
    return bgnn_add_dropped_bf16(C, src, M * N, p, seed, C, stream);
}

extern "C" int bgnn_gemm_gather_add(int32_t ta, int32_t tb, int64_t M, int64_t N, int64_t K, const float* A,
                                    int64_t lda, const float* B, int64_t ldb, float* C, int64_t ldc,
                                    const float* bias, int32_t relu, const float* add0, const int64_t* idx0,
                                    int64_t ld0, const float* add1, const int64_t* idx1, int64_t ld1,
                                    int32_t precision, void* ws, size_t ws_bytes, void* stream) {
    return gather_add_impl(ta, tb, M, N, K, A, lda, B, ldb, C, ldc, bias, relu, add0, idx0, ld0, add1, idx1, ld1,
                           precision, ws, ws_bytes, stream, 0);
}

// bf16-operand GEMM with bf16 STORAGE of any of A / B / C (EA_GNN's per-edge activations in the
// bf16 configuration, BASELINE configs[4]): storage bit 0 = A, bit 1 = B, bit 2 = C; lda / ldb /
// ldc count elements of the stored type. Operands are rounded to bf16 (exact when stored so),
// one MFMA product, f32 accumulation; a bf16 C is rounded to nearest even.
extern "C" int bgnn_gemm_bf16(int32_t ta, int32_t tb, int64_t M, int64_t N, int64_t K, float alpha, const void* A,
                              int64_t lda, const void* B, int64_t ldb, float beta, void* C, int64_t ldc,
                              const float* bias, int32_t relu, int32_t storage, void* ws, size_t ws_bytes,
                              void* stream) {
    BGNN_REQUIRE(storage >= 0 && storage < 8, "gemm_bf16: storage flags must be in [0, 8)");
    // built: NT {0, 1, 3, 4, 5, 7} (A and / or C bf16; B bf16 only with A), TN {0, 1, 2, 3}
    const bool nt_ok = ta == 0 && tb == 1 && storage != 2 && storage != 6;
    const bool tn_ok = ta == 1 && tb == 0 && storage <= 3;
    BGNN_REQUIRE(storage == 0 || nt_ok || tn_ok, "gemm_bf16: storage %d with ta=%d tb=%d is not built", storage, ta,
                 tb);
    return gemm_scaled_impl(ta, tb, M, N, K, alpha, static_cast<const float*>(A), lda, 0, 0,
                            static_cast<const float*>(B), ldb, beta, static_cast<float*>(C), ldc, 0, 0, bias, relu,
                            nullptr, nullptr, nullptr, 1, ws, ws_bytes, stream, BetaSrc{nullptr, 0, 0, 0.f}, storage);
}

// bgnn_gemm_gather_add on the bf16-operand family with bf16 storage of any of A (bit 0), B
// (bit 1) and C (bit 2); C = A B^T only (ta 0, tb 1). A and B both bf16 (bits 0 and 1) with
// K % 64 == 0 take the LDS-DMA bf16 kernel (gemm_b16.hip).
extern "C" int bgnn_gemm_gather_add_bf16(int64_t M, int64_t N, int64_t K, const void* A, int64_t lda, const void* B,
                                         int64_t ldb, void* C, int64_t ldc, const float* bias, int32_t relu,
                                         const float* add0, const int64_t* idx0, int64_t ld0, const float* add1,
                                         const int64_t* idx1, int64_t ld1, int32_t storage, void* ws,
                                         size_t ws_bytes, void* stream) {
    BGNN_REQUIRE(storage >= 0 && storage < 8 && storage != 2 && storage != 6,
                 "gemm_gather_add_bf16: storage must be one of 0, 1, 3, 4, 5, 7");
    return gather_add_impl(0, 1, M, N, K, static_cast<const float*>(A), lda, static_cast<const float*>(B), ldb,
                           static_cast<float*>(C), ldc, bias,
                           relu, add0, idx0, ld0, add1, idx1, ld1, 1, ws, ws_bytes, stream, storage);
}
