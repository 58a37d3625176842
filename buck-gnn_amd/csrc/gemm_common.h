// Shared GEMM argument block and plane-split addressing (gemm.hip, gemm_x6.hip).
#pragma once
#include "common.h"

namespace bgnn {

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

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
    // split kernels, no split-K: the beta operand read from bsrc [M, ld_bsrc] through a dropout
    // mask instead of from C -- the dgrad of a SAGE skip layer adds drop(g) recomputed from the
    // layer's counter-based mask (keep_bits4(dseed, (row * ld_bsrc + col) / 4, dthr), kept
    // values scaled by dkeep; dthr = 0: no mask), so bgnn_sage_bwd_rows need not write it
    const float* bsrc; int64_t ld_bsrc; uint64_t dseed; uint32_t dthr; float dkeep;
    // bf16-operand family (PREC 2) only: bf16 STORAGE of A (bit 0), B (bit 1), C (bit 2) -- the
    // pointers then address bf16 elements and lda / ldb / ldc count bf16 elements; bit 3 (LDS-DMA
    // bf16 kernel, bf16 C): bsrc holds bf16 and is added through its mask to the ROUNDED product
    int st;
    // f16x3 C = A B^T only: B points to a pre-split image of B^T (bgnn_gemm_wsplit, column tile =
    // the launch tile's BN) instead of f32 rows; the kernel copies its LDS image
    int wb;
    // drop-add epilogue: only columns >= bsrc_c0 take the beta operand, column c reading bsrc column
    // c - bsrc_c0 (a multiple of the tile width; the max layer's merged dgrad [dh W_l | dh W_r])
    int64_t bsrc_c0;
};

// the beta operand of 4 consecutive columns (col % 4 == 0) of row `row`: masked bsrc
__device__ __forceinline__ void beta_src4(const GemmArgs& g, int64_t row, int64_t col, float (&pv)[4]) {
    const int64_t i = row * g.ld_bsrc + col - g.bsrc_c0;
    const float4 t = *reinterpret_cast<const float4*>(g.bsrc + i);
    const uint32_t m = g.dthr ? keep_bits4(g.dseed, (uint64_t)(i >> 2), g.dthr) : 0xFu;
    const float kf = g.dthr ? g.dkeep : 1.f;
    pv[0] = (m & 1u) ? t.x * kf : 0.f;
    pv[1] = (m & 2u) ? t.y * kf : 0.f;
    pv[2] = (m & 4u) ? t.z * kf : 0.f;
    pv[3] = (m & 8u) ? t.w * kf : 0.f;
}

// beta_src4 on an already loaded float4 t of bsrc at (row, col) (the drop-add epilogue's prefetch)
__device__ __forceinline__ void beta_mask4(const GemmArgs& g, int64_t row, int64_t col, const float4& t,
                                           float (&pv)[4]) {
    const int64_t i = row * g.ld_bsrc + col - g.bsrc_c0;
    const uint32_t m = g.dthr ? keep_bits4(g.dseed, (uint64_t)(i >> 2), g.dthr) : 0xFu;
    const float kf = g.dthr ? g.dkeep : 1.f;
    pv[0] = (m & 1u) ? t.x * kf : 0.f;
    pv[1] = (m & 2u) ? t.y * kf : 0.f;
    pv[2] = (m & 4u) ? t.z * kf : 0.f;
    pv[3] = (m & 8u) ? t.w * kf : 0.f;
}

// Base pointer that makes plane-split storage addressable with global coordinates:
// element with split-dim index x lives at P + (x / blk) * pstride + (x % blk); for all x of
// one plane that is Q + x with Q = P + plane * (pstride - blk).
__device__ __forceinline__ const float* plane_base(const float* P, int64_t x0, int64_t blk, int64_t pstride) {
    if (blk <= 0) return P;
    const int64_t plane = x0 / blk;
    return P + plane * (pstride - blk);
}

// GEMMs on 16-bit MFMAs (gemm_x6.hip): prec 1 = f16x3 (f32-accurate), 2 = bf16 operands; launches the
// main kernel of tile config `cfg` (index into kX6Cfgs) on grid (tiles, split); abl = 8: the
// drop-add epilogue (bgnn_gemm_f32_dropadd), else 0.
struct X6Cfg {
    int bm, bn, waves, blocks_per_cu;
};
extern const X6Cfg kX6Cfgs[];
extern const int kNumX6Cfgs;
void launch_x6(int prec, int ta, int tb, int cfg, int abl, dim3 grid, hipStream_t s, const GemmArgs& g);
// bf16-operand GEMM on bf16-STORED A and B (gemm_b16.hip): b16_ok = the call qualifies (ta 0,
// tb 1, storage bits 0 and 1, K % 64 == 0, dense 16-B aligned rows, no split-K / drop-add);
// launch_b16 covers all M rows (one 256x256 tile per workgroup)
bool b16_ok(const GemmArgs& g, int ta, int tb);
void launch_b16(hipStream_t s, const GemmArgs& g);
// the launch would run the drop-add epilogue (st bit 8: bsrc = bf16 [M, ld_bsrc] through the dropout
// mask, added to the stored bf16 C) -- a whole-line bf16 C variant, N % 256 == 0, aligned C / bsrc
bool b16_dropadd_ok(const GemmArgs& g);
// folds max |P| over the rows x cols matrix (ld; plane-split by blk / pstride when blk > 0)
// into *out (f32 bits, unsigned atomic max; *out must hold a non-negative value)
void launch_absmax(const float* P, int64_t rows, int64_t cols, int64_t ld, int64_t blk, int64_t pstride,
                   float* out, hipStream_t s);

}  // namespace bgnn
