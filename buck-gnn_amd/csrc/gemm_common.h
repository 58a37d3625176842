// Shared GEMM argument block and plane-split addressing (gemm.hip, gemm_x6.hip).
#pragma once
#include "common.h"

namespace bgnn {

typedef float floatx16 __attribute__((ext_vector_type(16)));

struct GemmArgs {
    const float* A;
    const float* B;
    float* C;
    float* ws;
    int64_t M, N, K, lda, ldb, ldc;
    float alpha, beta;
    int64_t kchunk;   // K range per split-K slice (multiple of BK)
    int split;
    const float* bias;   // epilogue: + bias[col] (may be NULL)
    int relu;            // epilogue: max(., 0)
    // plane-split storage (0 = dense): A's contiguous dim (K if !TA, M if TA) and C's N dim
    // are cut into blocks of a_blk / c_blk stored a_pstride / c_pstride elements apart
    int64_t a_blk, a_pstride, c_blk, c_pstride;
    const float* a_amax;   // f16x3 (PREC 1): device max|A| and max|B|, which set the power-of-two
    const float* b_amax;   // operand scales
    float* c_amax;         // split kernels, no split-K: max |C| folded in here (NULL = off)
    // split kernels, no split-K: C[r, :] += ga0[gi0[r], :] (+ ga1[gi1[r], :]) before the ReLU
    // (EA_GNN's node-level blocks of the edge Linears, bgnn/ea.py); NULL = off
    const float* ga0; const int64_t* gi0; int64_t ldg0;
    const float* ga1; const int64_t* gi1; int64_t ldg1;
};

// Base pointer that makes plane-split storage addressable with global coordinates:
// element with split-dim index x lives at P + (x / blk) * pstride + (x % blk); for all x of
// one plane that is Q + x with Q = P + plane * (pstride - blk).
__device__ __forceinline__ const float* plane_base(const float* P, int64_t x0, int64_t blk, int64_t pstride) {
    if (blk <= 0) return P;
    const int64_t plane = x0 / blk;
    return P + plane * (pstride - blk);
}

// f32-accurate GEMMs on 16-bit MFMAs (gemm_x6.hip): prec 0 = bf16x6, 1 = f16x3; launches the
// main kernel of tile config `cfg` (index into kX6Cfgs) on grid (tiles, split); abl != 0
// selects a timing ablation.
struct X6Cfg {
    int bm, bn, waves, blocks_per_cu;
};
extern const X6Cfg kX6Cfgs[];
extern const int kNumX6Cfgs;
void launch_x6(int prec, int ta, int tb, int cfg, int abl, dim3 grid, hipStream_t s, const GemmArgs& g);
// f16x3 with LDS-DMA staging (gemm_h3g.hip): h3g_ok = the shape and operands qualify (ta 0,
// tb 1, dense 16-B aligned A and B, K % 32 == 0, no split-K, scales supplied); launches
// variant `variant` on the grid of h3g_tiles(variant, M, N) output tiles
bool h3g_ok(const GemmArgs& g, int ta, int tb);
int64_t h3g_tiles(int variant, int64_t M, int64_t N);
void launch_h3g(int variant, int64_t tiles, hipStream_t s, const GemmArgs& g);
constexpr int kNumH3gVariants = 2;
// folds max |P| over the rows x cols matrix (ld; plane-split by blk / pstride when blk > 0)
// into *out (f32 bits, unsigned atomic max; *out must hold a non-negative value)
void launch_absmax(const float* P, int64_t rows, int64_t cols, int64_t ld, int64_t blk, int64_t pstride,
                   float* out, hipStream_t s);

}  // namespace bgnn
