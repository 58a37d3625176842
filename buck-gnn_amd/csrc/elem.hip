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
