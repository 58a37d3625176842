// BatchNorm1d over a row-major [N, C] fp32 activation (torch.nn.BatchNorm1d semantics, train and
// eval) for the per-module path: the reference's unchanged Models/BuckGNN.py builds
// nn.BatchNorm1d(h) after every SAGEConv (:133,148,163,179) and calls it at :436; under
// bgnn.install_pyg_shim(batchnorm=True) those modules are bgnn.nn.BatchNorm1d, which run here.
// (The fused layer loop has its own BN, folded into the aggregation and row kernels: sage.hip.)
//
//   train:  mean, var from the batch (biased var for the normalisation, unbiased for the running
//           estimate, bgnn_bn_finalize), y = x * scale + shift with scale = gamma * invstd,
//           shift = beta - mean * scale
//   bwd:    dbeta = sum g, dgamma = sum g * xhat, xhat = (x - mean) * invstd;
//           train dx = gamma * invstd / N * (N g - dbeta - xhat dgamma); eval dx = g * scale
//
// Every kernel is one streaming pass with C4 = C / 4 threads per row (float4 columns, C4 a power
// of two dividing 256) and 256 / C4 rows per block step; per-block column partials go to
// [blocks, 2, C] and are summed by bgnn_reduce_partials / bgnn_bn_finalize (fp64, fixed order).
#include "common.h"

namespace bgnn {

namespace {

constexpr int kBnBlocks = 1024;

inline int bn_blocks(int64_t n_rows, int C, int64_t* rpb) {
    const int rpi = 256 / (C / 4);
    int64_t blocks = (n_rows + rpi - 1) / rpi;
    if (blocks > kBnBlocks) blocks = kBnBlocks;
    if (blocks < 1) blocks = 1;
    *rpb = (n_rows + blocks - 1) / blocks;
    return (int)blocks;
}

// column partials of a (and, when b != NULL, of a * xhat(b)) over the block's rows -> part[blk]
// MODE 0: sum (x - k), sum (x - k)^2 (forward statistics, shifted by k = `mean`, the input's first
// row: the variance stays free of the E[x^2] - E[x]^2 cancellation when |mean| >> std; finalized
// by bgnn_bn_finalize_shifted); MODE 1: sum g, sum g * (x - mean) * invstd
template <int MODE>
__global__ __launch_bounds__(256) void k_bn_colsums(const float* __restrict__ a, const float* __restrict__ x,
                                                    const float* __restrict__ mean, const float* __restrict__ invstd,
                                                    int64_t n_rows, int C, int64_t rows_per_block,
                                                    float* __restrict__ part) {
    __shared__ __attribute__((aligned(16))) float red[256][8];
    const int C4 = C / 4, rpi = 256 / C4;
    const int t = threadIdx.x, c4 = t % C4, ph = t / C4, c = c4 * 4;
    const int lb = xcd_remap(blockIdx.x, gridDim.x);
    const int64_t r0 = (int64_t)lb * rows_per_block, r1 = min(n_rows, r0 + rows_per_block);
    float s0[4] = {0.f, 0.f, 0.f, 0.f}, s1[4] = {0.f, 0.f, 0.f, 0.f};
    float mu[4] = {0.f, 0.f, 0.f, 0.f}, is[4] = {1.f, 1.f, 1.f, 1.f};
    {   // MODE 0: the shift k; MODE 1: mean and invstd
        const float4 m4 = *reinterpret_cast<const float4*>(mean + c);
        const float4 i4 = MODE == 1 ? *reinterpret_cast<const float4*>(invstd + c) : make_float4(1.f, 1.f, 1.f, 1.f);
        mu[0] = m4.x; mu[1] = m4.y; mu[2] = m4.z; mu[3] = m4.w;
        if (MODE == 1) { is[0] = i4.x; is[1] = i4.y; is[2] = i4.z; is[3] = i4.w; }
    }
    for (int64_t r = r0 + ph; r < r1; r += rpi) {
        const float4 av = reinterpret_cast<const float4*>(a)[r * C4 + c4];
        const float aa[4] = {av.x, av.y, av.z, av.w};
        if (MODE == 0) {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const float d = aa[k] - mu[k];
                s0[k] += d;
                s1[k] += d * d;
            }
        } else {
            const float4 xv = reinterpret_cast<const float4*>(x)[r * C4 + c4];
            const float xx[4] = {xv.x, xv.y, xv.z, xv.w};
#pragma unroll
            for (int k = 0; k < 4; ++k) { s0[k] += aa[k]; s1[k] += aa[k] * ((xx[k] - mu[k]) * is[k]); }
        }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) { red[t][k] = s0[k]; red[t][4 + k] = s1[k]; }
    __syncthreads();
    if (t < C4) {
        float a0[4] = {0.f, 0.f, 0.f, 0.f}, a1[4] = {0.f, 0.f, 0.f, 0.f};
        for (int q = 0; q < rpi; ++q)
#pragma unroll
            for (int k = 0; k < 4; ++k) { a0[k] += red[q * C4 + t][k]; a1[k] += red[q * C4 + t][4 + k]; }
        float* dst = part + (int64_t)lb * 2 * C;
        *reinterpret_cast<float4*>(dst + c) = make_float4(a0[0], a0[1], a0[2], a0[3]);
        *reinterpret_cast<float4*>(dst + C + c) = make_float4(a1[0], a1[1], a1[2], a1[3]);
    }
}

// y = x * scale + shift (forward), or the train-mode input gradient
// dx = kA g - kB - xhat kC with kA = gamma invstd, kB = kA sum_g / N, kC = kA sum_gxhat / N
template <int MODE>
__global__ __launch_bounds__(256) void k_bn_rows(const float4* __restrict__ a, const float4* __restrict__ x,
                                                 const float* __restrict__ p0, const float* __restrict__ p1,
                                                 const float* __restrict__ mean, const float* __restrict__ invstd,
                                                 const float* __restrict__ gamma, const float* __restrict__ sums,
                                                 int64_t n4, int C4, float invn, float4* __restrict__ out) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
        const int c = (int)(i % C4) * 4;
        const float4 v = a[i];
        const float vv[4] = {v.x, v.y, v.z, v.w};
        float y[4];
        if (MODE == 0) {
            const float4 sc = *reinterpret_cast<const float4*>(p0 + c);
            const float4 sh = *reinterpret_cast<const float4*>(p1 + c);
            const float scv[4] = {sc.x, sc.y, sc.z, sc.w}, shv[4] = {sh.x, sh.y, sh.z, sh.w};
#pragma unroll
            for (int k = 0; k < 4; ++k) y[k] = vv[k] * scv[k] + shv[k];
        } else {
            const float4 xv = x[i];
            const float4 mu = *reinterpret_cast<const float4*>(mean + c);
            const float4 is = *reinterpret_cast<const float4*>(invstd + c);
            const float4 gm = gamma ? *reinterpret_cast<const float4*>(gamma + c) : make_float4(1.f, 1.f, 1.f, 1.f);
            const float4 sg = *reinterpret_cast<const float4*>(sums + c);
            const float4 sx = *reinterpret_cast<const float4*>(sums + C4 * 4 + c);
            const float xx[4] = {xv.x, xv.y, xv.z, xv.w}, muv[4] = {mu.x, mu.y, mu.z, mu.w};
            const float isv[4] = {is.x, is.y, is.z, is.w}, gmv[4] = {gm.x, gm.y, gm.z, gm.w};
            const float sgv[4] = {sg.x, sg.y, sg.z, sg.w}, sxv[4] = {sx.x, sx.y, sx.z, sx.w};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const float ga = gmv[k] * isv[k];
                const float xh = (xx[k] - muv[k]) * isv[k];
                y[k] = ga * vv[k] - ga * sgv[k] * invn - xh * (ga * sxv[k] * invn);
            }
        }
        out[i] = make_float4(y[0], y[1], y[2], y[3]);
    }
}

inline unsigned rows_blocks(int64_t n4) {
    int64_t b = (n4 + 255) / 256;
    if (b > 8192) b = 8192;
    return (unsigned)(b < 1 ? 1 : b);
}

inline bool bn_shape_ok(int C) { return C >= 4 && C % 4 == 0 && C <= 1024 && 256 % (C / 4) == 0; }

}  // namespace

}  // namespace bgnn

using namespace bgnn;

extern "C" int32_t bgnn_bn_slots(int64_t n_rows, int32_t C) {
    if (!bn_shape_ok(C) || n_rows < 0) return -1;
    int64_t rpb = 0;
    return bn_blocks(n_rows, C, &rpb);
}

extern "C" int bgnn_bn_stats(const float* x, int64_t n_rows, int32_t C, float* partial, void* stream) {
    BGNN_REQUIRE(bn_shape_ok(C), "bn_stats: C=%d unsupported (C %% 4 == 0, C / 4 a power of two <= 256)", C);
    BGNN_REQUIRE(x && partial && aligned16(x) && aligned16(partial), "bn_stats: 16-byte aligned x / partial required");
    int64_t rpb = 0;
    const int blocks = bn_blocks(n_rows, C, &rpb);
    if (n_rows == 0) return BGNN_OK;
    // shift = the first row of x (bgnn_bn_finalize_shifted adds it back)
    hipLaunchKernelGGL(k_bn_colsums<0>, dim3(blocks), dim3(256), 0, as_stream(stream), x, nullptr, x, nullptr,
                       n_rows, C, rpb, partial);
    BGNN_CHECK_LAUNCH();
    return BGNN_OK;
}

extern "C" int bgnn_bn_apply(const float* x, int64_t n_rows, int32_t C, const float* scale, const float* shift,
                             float* y, void* stream) {
    BGNN_REQUIRE(bn_shape_ok(C), "bn_apply: C=%d unsupported", C);
    BGNN_REQUIRE(x && y && scale && shift && aligned16(x) && aligned16(y) && aligned16(scale) && aligned16(shift),
                 "bn_apply: 16-byte aligned pointers required");
    const int64_t n4 = n_rows * C / 4;
    if (n4 == 0) return BGNN_OK;
    hipLaunchKernelGGL(k_bn_rows<0>, dim3(rows_blocks(n4)), dim3(256), 0, as_stream(stream),
                       reinterpret_cast<const float4*>(x), nullptr, scale, shift, nullptr, nullptr, nullptr, nullptr, n4,
                       C / 4, 0.f, reinterpret_cast<float4*>(y));
    BGNN_CHECK_LAUNCH();
    return BGNN_OK;
}

extern "C" int bgnn_bn_bwd_stats(const float* g, const float* x, const float* mean, const float* invstd,
                                 int64_t n_rows, int32_t C, float* partial, void* stream) {
    BGNN_REQUIRE(bn_shape_ok(C), "bn_bwd_stats: C=%d unsupported", C);
    BGNN_REQUIRE(g && x && mean && invstd && partial && aligned16(g) && aligned16(x) && aligned16(mean) &&
                     aligned16(invstd) && aligned16(partial),
                 "bn_bwd_stats: 16-byte aligned pointers required");
    int64_t rpb = 0;
    const int blocks = bn_blocks(n_rows, C, &rpb);
    hipLaunchKernelGGL(k_bn_colsums<1>, dim3(blocks), dim3(256), 0, as_stream(stream), g, x, mean, invstd, n_rows, C,
                       rpb, partial);
    BGNN_CHECK_LAUNCH();
    return BGNN_OK;
}

extern "C" int bgnn_bn_bwd_dx(const float* g, const float* x, const float* mean, const float* invstd,
                              const float* gamma, const float* sums, int64_t n_rows, int32_t C, float* dx,
                              void* stream) {
    BGNN_REQUIRE(bn_shape_ok(C), "bn_bwd_dx: C=%d unsupported", C);
    BGNN_REQUIRE(g && x && mean && invstd && sums && dx && aligned16(g) && aligned16(x) && aligned16(dx),
                 "bn_bwd_dx: 16-byte aligned g / x / dx required");
    const int64_t n4 = n_rows * C / 4;
    if (n4 == 0) return BGNN_OK;
    hipLaunchKernelGGL(k_bn_rows<1>, dim3(rows_blocks(n4)), dim3(256), 0, as_stream(stream),
                       reinterpret_cast<const float4*>(g), reinterpret_cast<const float4*>(x), nullptr, nullptr, mean,
                       invstd, gamma, sums, n4, C / 4, 1.f / (float)(n_rows > 0 ? n_rows : 1),
                       reinterpret_cast<float4*>(dx));
    BGNN_CHECK_LAUNCH();
    return BGNN_OK;
}
