// Skip connection + dropout of the EA_GNN layer loop (Models/BuckGNN.py:382-387:
// x, e = x + x_prev, e + e_prev on the middle blocks, then Dropout on both) as one pass over
// the [E, H] edge features, with the counter-based dropout mask of the fused SAGE layers
// (keep_bits4 on (seed, element / 4): nothing stored, the backward recomputes it).
//   fwd: out = drop(a + b)    (b optional)      3 passes (a, b read; out written)
//   bwd: g' = drop(g)         (dL/da = dL/db = g')
// torch's add + dropout + masked-scale backward make 5.25 + 2.25 such passes.
#include "common.h"

namespace bgnn {

namespace {

__global__ __launch_bounds__(256) void k_add_dropout(const float4* __restrict__ a, const float4* __restrict__ b,
                                                     int64_t n4, uint32_t thr, float inv_keep, uint64_t seed,
                                                     float4* __restrict__ out) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
        float4 v = a[i];
        if (b) {
            const float4 w = b[i];
            v.x += w.x; v.y += w.y; v.z += w.z; v.w += w.w;
        }
        if (thr) {
            const uint32_t keep = keep_bits4(seed, (uint64_t)i, thr);
            v.x = (keep & 1u) ? v.x * inv_keep : 0.f;
            v.y = (keep & 2u) ? v.y * inv_keep : 0.f;
            v.z = (keep & 4u) ? v.z * inv_keep : 0.f;
            v.w = (keep & 8u) ? v.w * inv_keep : 0.f;
        }
        out[i] = v;
    }
}

// bf16 storage (the EA_GNN bf16 configuration's edge activations): 8 elements per thread, the
// same mask (group index = element / 4), sums in f32, one round to nearest even per result
__device__ __forceinline__ void bf16x8_unpack(const uint4 q, float (&f)[8]) {
    const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int h = 0; h < 4; ++h) {
        f[2 * h] = __uint_as_float(w[h] << 16);
        f[2 * h + 1] = __uint_as_float(w[h] & 0xffff0000u);
    }
}

__device__ __forceinline__ uint32_t bf16_pack2(float x, float y) {
    typedef float f32x2 __attribute__((ext_vector_type(2)));
    typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
    const f32x2 v = {x, y};
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2));
}

__global__ __launch_bounds__(256) void k_add_dropout_bf16(const uint4* __restrict__ a, const uint4* __restrict__ b,
                                                          int64_t n8, uint32_t thr, float inv_keep, uint64_t seed,
                                                          uint4* __restrict__ out) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (int64_t)gridDim.x * blockDim.x) {
        float v[8];
        bf16x8_unpack(a[i], v);
        if (b) {
            float w[8];
            bf16x8_unpack(b[i], w);
#pragma unroll
            for (int k = 0; k < 8; ++k) v[k] += w[k];
        }
        if (thr) {
#pragma unroll
            for (int hgrp = 0; hgrp < 2; ++hgrp) {
                const uint32_t keep = keep_bits4(seed, (uint64_t)(2 * i + hgrp), thr);
#pragma unroll
                for (int k = 0; k < 4; ++k) v[4 * hgrp + k] = ((keep >> k) & 1u) ? v[4 * hgrp + k] * inv_keep : 0.f;
            }
        }
        out[i] = make_uint4(bf16_pack2(v[0], v[1]), bf16_pack2(v[2], v[3]), bf16_pack2(v[4], v[5]),
                            bf16_pack2(v[6], v[7]));
    }
}

// Segment sum / mean over rows of a bf16 [n, H] matrix (H <= 512, H % 8 == 0) into f32
// out[R, H]: one wave per output row, 8 columns (16 B) per lane, the row's entries in CSR order
// (deterministic), f32 accumulation; empty rows 0. scatter_mean / scatter_add of EA_GNN's bf16
// messages (Models/BuckGNN.py:561) and their ReLU-masked gradients.
__global__ __launch_bounds__(256) void k_seg_sum_bf16(const int32_t* __restrict__ rowptr,
                                                      const int32_t* __restrict__ col, int64_t R,
                                                      const uint16_t* __restrict__ x, int64_t ldx, int H, int mean,
                                                      float* __restrict__ out, int64_t ldo) {
    const int lane = threadIdx.x & 63;
    const int64_t nw = (int64_t)gridDim.x * 4;
    const int c = lane * 8;
    const bool ok = c < H;
    for (int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); r < R; r += nw) {
        const int32_t b = rowptr[r], e = rowptr[r + 1];
        float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        int32_t p = b;
        for (; p + 8 <= e; p += 8) {   // 8 rows in flight
            uint4 q[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int64_t j = col[p + u];
                q[u] = ok ? *reinterpret_cast<const uint4*>(x + j * ldx + c) : make_uint4(0, 0, 0, 0);
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                float f[8];
                bf16x8_unpack(q[u], f);
#pragma unroll
                for (int k = 0; k < 8; ++k) acc[k] += f[k];
            }
        }
        for (; p < e; ++p) {
            const int64_t j = col[p];
            float f[8];
            bf16x8_unpack(ok ? *reinterpret_cast<const uint4*>(x + j * ldx + c) : make_uint4(0, 0, 0, 0), f);
#pragma unroll
            for (int k = 0; k < 8; ++k) acc[k] += f[k];
        }
        if (mean) {
            const float inv = __frcp_rn((float)(e - b > 0 ? e - b : 1));
#pragma unroll
            for (int k = 0; k < 8; ++k) acc[k] *= inv;
        }
        if (ok) {
            *reinterpret_cast<float4*>(out + r * ldo + c) = make_float4(acc[0], acc[1], acc[2], acc[3]);
            *reinterpret_cast<float4*>(out + r * ldo + c + 4) = make_float4(acc[4], acc[5], acc[6], acc[7]);
        }
    }
}

// Backward of k_seg_sum_bf16: every position p of segment r receives bf16(g[r] (/ max(deg, 1) for
// mean)), f32 division then one round-to-nearest-even -- torch's (g / cnt).to(bfloat16)
// .index_select(0, index) in one pass (EA_GNN's scatter_mean backward, Models/BuckGNN.py:561).
// One wave per segment, 8 columns (16 B of bf16) per lane; each position's row is written once.
__global__ __launch_bounds__(256) void k_seg_bcast_bf16(const int32_t* __restrict__ rowptr,
                                                        const int32_t* __restrict__ col, int64_t R,
                                                        const float* __restrict__ g, int64_t ldg, int H, int mean,
                                                        uint16_t* __restrict__ out, int64_t ldo) {
    const int lane = threadIdx.x & 63;
    const int64_t nw = (int64_t)gridDim.x * 4;
    const int c = lane * 8;
    const bool ok = c < H;
    for (int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); r < R; r += nw) {
        const int32_t b = rowptr[r], e = rowptr[r + 1];
        if (b == e || !ok) continue;
        const float4 v0 = *reinterpret_cast<const float4*>(g + r * ldg + c);
        const float4 v1 = *reinterpret_cast<const float4*>(g + r * ldg + c + 4);
        float v[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
        if (mean) {
            const float cnt = (float)(e - b);
#pragma unroll
            for (int k = 0; k < 8; ++k) v[k] = __fdiv_rn(v[k], cnt);
        }
        const uint4 q = make_uint4(bf16_pack2(v[0], v[1]), bf16_pack2(v[2], v[3]), bf16_pack2(v[4], v[5]),
                                   bf16_pack2(v[6], v[7]));
        for (int32_t p = b; p < e; ++p) *reinterpret_cast<uint4*>(out + (int64_t)col[p] * ldo + c) = q;
    }
}

inline unsigned elem_blocks(int64_t n4) {
    int64_t blocks = (n4 + 255) / 256;
    if (blocks > 8192) blocks = 8192;   // grid-stride beyond 32 blocks per CU
    return (unsigned)(blocks < 1 ? 1 : blocks);
}

}  // namespace

}  // namespace bgnn

using namespace bgnn;

extern "C" int bgnn_add_dropout(const float* a, const float* b, int64_t n, float p, uint64_t seed, float* out,
                                void* stream) {
    BGNN_REQUIRE(n >= 0 && n % 4 == 0, "add_dropout: n must be a multiple of 4");
    BGNN_REQUIRE(p >= 0.f && p < 1.f, "add_dropout: p must be in [0, 1)");
    if (n == 0) return BGNN_OK;
    BGNN_REQUIRE(a && out && aligned16(a) && aligned16(out) && (!b || aligned16(b)),
                 "add_dropout: 16-byte aligned a / b / out required");
    const uint32_t thr = dropout_threshold(p);
    const float inv_keep = thr ? 1.f / (1.f - p) : 1.f;
    hipLaunchKernelGGL(k_add_dropout, dim3(elem_blocks(n / 4)), dim3(256), 0, as_stream(stream),
                       reinterpret_cast<const float4*>(a), reinterpret_cast<const float4*>(b), n / 4, thr, inv_keep,
                       seed, reinterpret_cast<float4*>(out));
    BGNN_CHECK_LAUNCH();
    return BGNN_OK;
}

extern "C" int bgnn_add_dropout_bf16(const void* a, const void* b, int64_t n, float p, uint64_t seed, void* out,
                                     void* stream) {
    BGNN_REQUIRE(n >= 0 && n % 8 == 0, "add_dropout_bf16: n must be a multiple of 8");
    BGNN_REQUIRE(p >= 0.f && p < 1.f, "add_dropout_bf16: p must be in [0, 1)");
    if (n == 0) return BGNN_OK;
    BGNN_REQUIRE(a && out && aligned16(a) && aligned16(out) && (!b || aligned16(b)),
                 "add_dropout_bf16: 16-byte aligned a / b / out required");
    const uint32_t thr = dropout_threshold(p);
    const float inv_keep = thr ? 1.f / (1.f - p) : 1.f;
    hipLaunchKernelGGL(k_add_dropout_bf16, dim3(elem_blocks(n / 8)), dim3(256), 0, as_stream(stream),
                       reinterpret_cast<const uint4*>(a), reinterpret_cast<const uint4*>(b), n / 8, thr, inv_keep,
                       seed, reinterpret_cast<uint4*>(out));
    BGNN_CHECK_LAUNCH();
    return BGNN_OK;
}

// out = a + drop(b) over bf16 (ABI 8): the gradient of an edge activation that feeds both an edge
// Linear (a = that Linear's input gradient) and EA_GNN's skip + dropout (b = the dropout output's
// gradient, masked here with the forward's mask: keep_bits4(seed, i / 4), kept values / (1 - p)),
// in one pass instead of a dropout pass writing drop(b) and autograd's add reading it back.
__global__ __launch_bounds__(256) void k_add_dropped_bf16(const uint4* __restrict__ a, const uint4* __restrict__ b,
                                                          int64_t n8, uint32_t thr, float inv_keep, uint64_t seed,
                                                          uint4* __restrict__ out) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (int64_t)gridDim.x * blockDim.x) {
        float v[8], w[8];
        bf16x8_unpack(a[i], v);
        bf16x8_unpack(b[i], w);
        if (thr) {
#pragma unroll
            for (int hgrp = 0; hgrp < 2; ++hgrp) {
                const uint32_t keep = keep_bits4(seed, (uint64_t)(2 * i + hgrp), thr);
#pragma unroll
                for (int k = 0; k < 4; ++k) w[4 * hgrp + k] = ((keep >> k) & 1u) ? w[4 * hgrp + k] * inv_keep : 0.f;
            }
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] += w[k];
        out[i] = make_uint4(bf16_pack2(v[0], v[1]), bf16_pack2(v[2], v[3]), bf16_pack2(v[4], v[5]),
                            bf16_pack2(v[6], v[7]));
    }
}

// RelativeErrorLoss on denormalised values (Utils/Losses.py:755-761 after Normalizer.py:203-215's
// value * scale + center on prediction and target), forward and gradient in one launch (ABI 8):
// loss = mean(|p' - t'| / (|t'| + eps)), p' = pred * scale + center, t' = y * scale + center;
// dpred[i] = sign(p'_i - t'_i) * scale / ((|t'_i| + eps) * n). One block; the per-thread partial
// sums (f64) are reduced in a fixed order. Replaces ~16 single-element torch launches per step.
__global__ __launch_bounds__(256) void k_rel_error_loss(const float* __restrict__ pred, const float* __restrict__ y,
                                                        int64_t n, float scale, float center, float eps,
                                                        float* __restrict__ loss, float* __restrict__ dpred) {
    __shared__ double red[256];
    const int t = threadIdx.x;
    double acc = 0.0;
    const float inv_n = 1.f / (float)n;
    for (int64_t i = t; i < n; i += 256) {
        const float p = pred[i] * scale + center;
        const float q = y[i] * scale + center;
        const float d = fabsf(q) + eps;
        const float diff = p - q;
        acc += (double)(fabsf(diff) / d);
        // sign(diff) with sign(NaN) = 0: torch's abs backward (grad * sgn(x), sgn(NaN) = 0 on
        // ROCm and CPU), which the reference's loss differentiates through -- a NaN prediction
        // shows as a NaN loss, with the same zero gradient as the reference
        const float sg = diff > 0.f ? 1.f : (diff < 0.f ? -1.f : 0.f);
        if (dpred) dpred[i] = sg * scale / d * inv_n;
    }
    red[t] = acc;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (t < o) red[t] += red[t + o];
        __syncthreads();
    }
    if (t == 0) *loss = (float)(red[0] / (double)n);
}

extern "C" int bgnn_add_dropped_bf16(const void* a, const void* b, int64_t n, float p, uint64_t seed, void* out,
                                     void* stream) {
    BGNN_REQUIRE(n >= 0 && n % 8 == 0, "add_dropped_bf16: n must be a multiple of 8");
    BGNN_REQUIRE(p >= 0.f && p < 1.f, "add_dropped_bf16: p must be in [0, 1)");
    if (n == 0) return BGNN_OK;
    BGNN_REQUIRE(a && b && out && aligned16(a) && aligned16(b) && aligned16(out),
                 "add_dropped_bf16: 16-byte aligned a / b / out required");
    const uint32_t thr = dropout_threshold(p);
    const float inv_keep = thr ? 1.f / (1.f - p) : 1.f;
    hipLaunchKernelGGL(k_add_dropped_bf16, dim3(elem_blocks(n / 8)), dim3(256), 0, as_stream(stream),
                       reinterpret_cast<const uint4*>(a), reinterpret_cast<const uint4*>(b), n / 8, thr, inv_keep,
                       seed, reinterpret_cast<uint4*>(out));
    BGNN_CHECK_LAUNCH();
    return BGNN_OK;
}

extern "C" int bgnn_rel_error_loss(const float* pred, const float* y, int64_t n, float scale, float center, float eps,
                                   float* loss, float* dpred, void* stream) {
    BGNN_REQUIRE(pred && y && loss && n > 0, "rel_error_loss: null pointer or empty input");
    hipLaunchKernelGGL(k_rel_error_loss, dim3(1), dim3(256), 0, as_stream(stream), pred, y, n, scale, center, eps, loss,
                       dpred);
    BGNN_CHECK_LAUNCH();
    return BGNN_OK;
}

extern "C" int bgnn_segment_sum_bf16(const int32_t* rowptr, const int32_t* col, int64_t n_rows, const void* x,
                                     int64_t ldx, int32_t H, int32_t mean, float* out, int64_t ldo, void* stream) {
    BGNN_REQUIRE(rowptr && (n_rows == 0 || (col && x && out)), "segment_sum_bf16: null pointer");
    BGNN_REQUIRE(H > 0 && H <= 512 && H % 8 == 0 && ldx % 8 == 0 && ldx >= H && ldo >= H && ldo % 4 == 0,
                 "segment_sum_bf16: H must be a multiple of 8 up to 512, rows 16-B aligned");
    BGNN_REQUIRE(aligned16(x) && aligned16(out), "segment_sum_bf16: 16-byte aligned x / out required");
    if (n_rows == 0) return BGNN_OK;
    int64_t blocks = (n_rows + 3) / 4;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(k_seg_sum_bf16, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream), rowptr, col, n_rows,
                       static_cast<const uint16_t*>(x), ldx, H, mean, out, ldo);
    BGNN_CHECK_LAUNCH();
    return BGNN_OK;
}

extern "C" int bgnn_segment_bcast_bf16(const int32_t* rowptr, const int32_t* col, int64_t n_rows, const float* g,
                                       int64_t ldg, int32_t H, int32_t mean, void* out, int64_t ldo, void* stream) {
    BGNN_REQUIRE(rowptr && (n_rows == 0 || (col && g && out)), "segment_bcast_bf16: null pointer");
    BGNN_REQUIRE(H > 0 && H <= 512 && H % 8 == 0 && ldg % 4 == 0 && ldg >= H && ldo >= H && ldo % 8 == 0,
                 "segment_bcast_bf16: H must be a multiple of 8 up to 512, rows 16-B aligned");
    BGNN_REQUIRE(aligned16(g) && aligned16(out), "segment_bcast_bf16: 16-byte aligned g / out required");
    if (n_rows == 0) return BGNN_OK;
    int64_t blocks = (n_rows + 3) / 4;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(k_seg_bcast_bf16, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream), rowptr, col, n_rows,
                       g, ldg, H, mean, static_cast<uint16_t*>(out), ldo);
    BGNN_CHECK_LAUNCH();
    return BGNN_OK;
}
