// GEMMs on the gfx950 16-bit MFMAs, for the same SAGEConv linears as gemm.hip
// (Models/BuckGNN.py:135-149; fwd, dgrad, wgrad shapes) and the EA_GNN edge / node MLPs.
// PREC 2 = bf16 operands (one round-to-nearest piece, one product, f32 accumulation; the
// bf16 EA_GNN path of BASELINE configs[4]). Two f32-accurate split precisions:
//
// PREC 1 = f16x3 (default). Each operand is scaled by a power of two s = 2^k chosen from its
// max |value| (max |a| * s in [2^14, 2^15), so nothing overflows the f16 range) and split
// into two round-to-nearest f16 pieces, a*s = a0 + a1 + e with |a1| <= 2^-11 |a*s| and
// |e| <= 2^-22 |a*s|. The product is a.b = (a0.b0 + a0.b1 + a1.b0) / (s_a s_b) + O(2^-21 |a||b|)
// (a1.b1 <= 2^-22, e terms <= 2^-22 each): three f16 MFMAs per f32 product, every
// f16 x f16 product (11 x 11 bits) exact in the f32 accumulator, and the unscale an exact
// power-of-two multiply. The representation error stays an order of magnitude below the
// f32 accumulation error of a K = 512 sum (measured against fp64 in tests/test_gpu_gemm.py).
// Elements below 2^-39 max|A| (f16 subnormal range after scaling) lose relative precision;
// their absolute error stays below 2^-39 max|A| |b|.
//
// Tiling: BM x BN output tile per workgroup, waves WM x WN, each wave (BM/WM) x (BN/WN) in
// 32x32 MFMA tiles; K in BK = 32 slices, double-buffered in LDS. Global operands are read as
// f32 (float4 when K-contiguous, coalesced dwords along M/N when transposed), split in
// registers and stored as 16-bit row images [R][32] per piece (K contiguous, 64-B rows, 16-B
// chunks XOR-swizzled by (row >> 2) & 3 so a 16-lane ds_read_b128 group hits 16 distinct
// bank quads). Each MFMA operand is one ds_read_b128 per piece per lane. (A bf16x6 family --
// three exact bf16 pieces, six products -- was measured and dropped in round 2: f16x3 halves
// its MFMAs at a lower error.)
//
// This file: the tile table, the per-family dispatch and the operand-max kernels; the kernel
// template lives in gemm_x6_kernel.h, instantiated by gemm_x6_nt.hip (forward / dgrad shapes),
// gemm_x6_other.hip (weight gradient and the other transposes) and gemm_x6_b16s.hip (bf16
// operands and storage).
#include "gemm_x6_kernel.h"

namespace bgnn {

// bm, bn, waves, workgroups per CU; configs 3 and 4 (128 KB of LDS) are built for f16x3 only
const X6Cfg kX6Cfgs[] = {
    {128, 128, 4, 1},   // 0: 2x2 waves of 64x64 (1 wave / SIMD)
    {256, 128, 8, 1},   // 1: 4x2 waves of 64x64 (2 waves / SIMD)
    {128, 256, 8, 1},   // 2: 2x4 waves of 64x64
    {256, 256, 8, 1},   // 3: 2x4 waves of 128x64
    {256, 256, 8, 1},   // 4: 4x2 waves of 64x128
    {128, 128, 8, 1},   // 5: 2x4 waves of 64x32 (f16x3 NT only: tall N = 128 products with few 256-row tiles)
};
const int kNumX6Cfgs = 6;

// knob 16 (BGNN_TUNE_GEMM_BDMA): default 2 with 4 slots = the pipelined 128 x 256 kernel (gemm_h3p.hip)
// for the pre-split products planned on that tile (the SAGE input gradients): bit-identical, dgrad
// 272 -> 263 us, drop-add 321 -> 312, cfg2 step 8.74 -> 8.67 ms (profiles/r06_gemm_h3p_q.txt)
int g_x6_bdma = 2;

void launch_x6(int prec, int ta, int tb, int cfg, int abl, dim3 grid, hipStream_t s, const GemmArgs& g) {
    if (prec == 2 && g.st != 0) launch_x6_bf16_storage(ta, tb, cfg, g.st, grid, s, g);
    else if (prec == 2) launch_x6_prec2(ta, tb, cfg, grid, s, g);
    else if (ta == 0 && tb == 1) launch_x6_nt_main(cfg, abl, grid, s, g);
    else launch_x6_h3_other(ta, tb, cfg, grid, s, g);
}

// max |x| over a strided (optionally plane-split) matrix, folded into *out by an unsigned
// atomic max on the f32 bits (monotone for non-negative floats; NaN compares above Inf).
// tpr threads per row (a power of two dividing 256) sweep a row's float4 (or float) columns;
// 256 / tpr rows per block step; no integer division inside the loops.
template <bool VEC>
__global__ __launch_bounds__(256) void k_absmax(const float* __restrict__ P, int64_t rows, int64_t cols, int64_t ld,
                                                int64_t blk, int64_t pstride, int tpr, uint32_t* __restrict__ out) {
    const int rpi = 256 / tpr;
    const int tc = threadIdx.x % tpr;
    uint32_t m = 0;
    for (int64_t r = (int64_t)blockIdx.x * rpi + threadIdx.x / tpr; r < rows; r += (int64_t)gridDim.x * rpi) {
        if constexpr (VEC) {
            const float4* row = reinterpret_cast<const float4*>(P + r * ld);
            for (int64_t c = tc; c < cols / 4; c += tpr) {
                const float4 v = row[c];
                m = max(m, max(max(__float_as_uint(v.x) & 0x7fffffffu, __float_as_uint(v.y) & 0x7fffffffu),
                               max(__float_as_uint(v.z) & 0x7fffffffu, __float_as_uint(v.w) & 0x7fffffffu)));
            }
        } else {
            int64_t cb = 0;   // plane of column c (blk > 0): element at P + plane * pstride + r * ld + c - plane * blk
            int64_t c = tc;
            for (; c < cols; c += tpr) {
                if (blk > 0) cb = c / blk;
                const float* base = P + cb * (pstride - blk);
                m = max(m, __float_as_uint(base[r * ld + c]) & 0x7fffffffu);
            }
        }
    }
    for (int o = 32; o > 0; o >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, o, kWave));
    __shared__ uint32_t red[4];
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        m = max(max(red[0], red[1]), max(red[2], red[3]));
        if (m) atomicMax(out, m);
    }
}

// max |W_i| of n items of equal shape (rows x cols, ld; item i at P + i * item_stride) in one
// launch: grid.y = item, each block of an item as in k_absmax (the per-layer weight maxima of a
// SAGE loop, bgnn.fused.prepare_weights); out[i * out_stride] = max(out[.], max |W_i|).
__global__ __launch_bounds__(256) void k_absmax_items(const float* __restrict__ P, int64_t item_stride, int64_t rows,
                                                      int64_t cols4, int64_t ld, int tpr, uint32_t* __restrict__ out,
                                                      int64_t out_stride) {
    const float* Pi = P + (int64_t)blockIdx.y * item_stride;
    const int rpi = 256 / tpr;
    const int tc = threadIdx.x % tpr;
    uint32_t m = 0;
    for (int64_t r = (int64_t)blockIdx.x * rpi + threadIdx.x / tpr; r < rows; r += (int64_t)gridDim.x * rpi) {
        const float4* row = reinterpret_cast<const float4*>(Pi + r * ld);
        for (int64_t c = tc; c < cols4; c += tpr) {
            const float4 v = row[c];
            m = max(m, max(max(__float_as_uint(v.x) & 0x7fffffffu, __float_as_uint(v.y) & 0x7fffffffu),
                           max(__float_as_uint(v.z) & 0x7fffffffu, __float_as_uint(v.w) & 0x7fffffffu)));
        }
    }
    for (int o = 32; o > 0; o >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, o, kWave));
    __shared__ uint32_t red[4];
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        m = max(max(red[0], red[1]), max(red[2], red[3]));
        if (m) atomicMax(out + (int64_t)blockIdx.y * out_stride, m);
    }
}

void launch_absmax(const float* P, int64_t rows, int64_t cols, int64_t ld, int64_t blk, int64_t pstride,
                   float* out, hipStream_t s) {
    const bool vec = blk == 0 && cols % 4 == 0 && ld % 4 == 0 && (((uintptr_t)P & 15) == 0);
    const int64_t units = vec ? cols / 4 : cols;
    int tpr = 1;
    while (tpr < 256 && tpr < units) tpr <<= 1;
    const int64_t rpi = 256 / tpr;
    int64_t blocks = (rows + rpi - 1) / rpi;
    if (blocks > 2048) blocks = 2048;
    if (blocks < 1) blocks = 1;
    uint32_t* o = reinterpret_cast<uint32_t*>(out);
    if (vec) hipLaunchKernelGGL(k_absmax<true>, dim3((unsigned)blocks), dim3(256), 0, s, P, rows, cols, ld, blk, pstride, tpr, o);
    else hipLaunchKernelGGL(k_absmax<false>, dim3((unsigned)blocks), dim3(256), 0, s, P, rows, cols, ld, blk, pstride, tpr, o);
}

// Pre-split B images (bgnn_gemm_wsplit): weight matrix W [N][K] (the B^T operand of C = A W^T)
// scaled by its f16x3 power of two and split into the two f16 pieces, stored per (column tile of
// bn rows, 32-deep slice) as exactly the [piece][row][4 chunks] swizzled LDS image k_gemm_x6
// writes (x6_store), so the GEMM copies it into LDS by LDS-DMA unchanged. One thread per 8-k unit;
// grid.y = matrix index of a batch of equal-shape matrices.
__global__ __launch_bounds__(256) void k_wsplit(const float* __restrict__ W, int64_t item_stride, int64_t N, int64_t K,
                                                int64_t ldw, const float* __restrict__ amax, int64_t amax_stride,
                                                uint4* __restrict__ img, int64_t img_stride_u4, int bn) {
    const int64_t item = blockIdx.y;
    const int64_t ku = K / 8;
    const int64_t u = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (u >= N * ku) return;
    const int64_t n = u / ku, k0 = (u % ku) * 8;
    const int64_t tn = n / bn, sl = k0 / 32;
    const int r = (int)(n % bn), c = (int)((k0 % 32) / 8);
    float sc, inv;
    h3_scale(amax[item * amax_stride], sc, inv);
    const float* w = W + item * item_stride + n * ldw + k0;
    const float4 a = *reinterpret_cast<const float4*>(w), b = *reinterpret_cast<const float4*>(w + 4);
    uint4 q0, q1;
    split2h(a.x * sc, a.y * sc, q0.x, q1.x);
    split2h(a.z * sc, a.w * sc, q0.y, q1.y);
    split2h(b.x * sc, b.y * sc, q0.z, q1.z);
    split2h(b.z * sc, b.w * sc, q0.w, q1.w);
    uint4* dst = img + item * img_stride_u4 + (tn * (K / 32) + sl) * (int64_t)(bn * 8);
    const int pos = x6_pos(r, c);
    dst[pos] = q0;
    dst[bn * 4 + pos] = q1;
}

}  // namespace bgnn

using namespace bgnn;

extern "C" size_t bgnn_gemm_wsplit_bytes(int64_t N, int64_t K) {
    return (N > 0 && K > 0) ? (size_t)N * (size_t)K * 4 : 0;
}

extern "C" int bgnn_gemm_wsplit(const float* W, int32_t n_items, int64_t item_stride, int64_t N, int64_t K,
                                int64_t ldw, const float* amax, int64_t amax_stride, void* img, int64_t img_stride,
                                int32_t bn, void* stream) {
    BGNN_REQUIRE(W && amax && img && n_items >= 0 && n_items <= 65535, "wsplit: bad args");
    BGNN_REQUIRE(bn == 128 || bn == 256, "wsplit: column tile must be 128 or 256 (got %d)", bn);
    BGNN_REQUIRE(N > 0 && K > 0 && N % bn == 0 && K % 32 == 0, "wsplit: N %% bn == 0 and K %% 32 == 0 required");
    BGNN_REQUIRE(ldw >= K && ldw % 4 == 0 && item_stride % 4 == 0 && ((uintptr_t)W & 15) == 0,
                 "wsplit: 16-B aligned rows required");
    BGNN_REQUIRE(((uintptr_t)img & 15) == 0 && img_stride >= N * K * 4 && img_stride % 16 == 0,
                 "wsplit: img must be 16-B aligned with img_stride >= bgnn_gemm_wsplit_bytes(N, K)");
    if (n_items == 0) return BGNN_OK;
    const int64_t units = N * (K / 8);
    hipLaunchKernelGGL(k_wsplit, dim3((unsigned)((units + 255) / 256), (unsigned)n_items), dim3(256), 0,
                       as_stream(stream), W, item_stride, N, K, ldw, amax, amax_stride, static_cast<uint4*>(img),
                       img_stride / 16, (int)bn);
    BGNN_CHECK_LAUNCH();
    return BGNN_OK;
}

extern "C" int bgnn_absmax_items_f32(const float* x, int32_t n_items, int64_t item_stride, int64_t rows, int64_t cols,
                                     int64_t ld, float* out, int64_t out_stride, void* stream) {
    BGNN_REQUIRE(x && out && n_items >= 0 && rows >= 0 && cols >= 0 && ld >= cols, "absmax_items: bad args");
    BGNN_REQUIRE(cols % 4 == 0 && ld % 4 == 0 && item_stride % 4 == 0 && (((uintptr_t)x & 15) == 0),
                 "absmax_items: cols, ld and item_stride must be multiples of 4 and x 16-B aligned");
    BGNN_REQUIRE(n_items <= 65535, "absmax_items: at most 65535 items");
    if (n_items == 0 || rows == 0 || cols == 0) return BGNN_OK;
    const int64_t cols4 = cols / 4;
    int tpr = 1;
    while (tpr < 256 && tpr < cols4) tpr <<= 1;
    const int64_t rpi = 256 / tpr;
    int64_t blocks = (rows + rpi - 1) / rpi;
    // <= 64 blocks per item: the per-layer weights are 2 MB, and 512 blocks of 2 rows each ran the
    // 6-layer pass in 32 us (launch-, not bandwidth-bound, 3,072 atomics on 6 words)
    if (blocks > 64) blocks = 64;
    hipLaunchKernelGGL(k_absmax_items, dim3((unsigned)blocks, (unsigned)n_items), dim3(256), 0, as_stream(stream), x,
                       item_stride, rows, cols4, ld, tpr, reinterpret_cast<uint32_t*>(out), out_stride);
    BGNN_CHECK_LAUNCH();
    return BGNN_OK;
}
