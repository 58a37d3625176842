// The node encoder's leading layers as one kernel: h = ReLU(ReLU(x W1^T + b1) W2^T + b2),
// Models/BuckGNN.py:67-74 (Linear(16,64) . ReLU . Linear(64,128) . ReLU; the last Linear(128,512)
// is folded into the first SAGE layer, bgnn/fused.py). Per node that is 9,216 MACs on 16 inputs
// and 128 outputs: far too little work per byte for MFMA tiles (a K = 16 / 64 GEMM launch
// spends its time in prologue and epilogue), so a workgroup keeps both weight matrices in LDS
// and runs 64 nodes per tile through both layers on the VALU in fp32, writing only h (and
// folding max|h|, the f16x3 operand scale of the folded GEMM that reads h).
//
// The backward recomputes the hidden layer from x (cheaper than storing [N, 64]) and
// accumulates the weight and bias gradients of both layers per workgroup; a second kernel sums
// the per-workgroup partials in a fixed order (deterministic, no atomics).
#include "common.h"

namespace bgnn {

namespace {

constexpr int kT = 64;          // nodes per tile
constexpr int kMlpBlocks = 256; // persistent workgroups (partials of the backward: one slot each)

template <int F, int D1, int D2>
struct MlpSmem {
    float w1t[F][D1];          // W1^T
    float b1[D1];
    float w2t[D1][D2];         // W2^T (forward) -- the backward keeps W2 as [D2][D1] in the same space
    float b2[D2];
    float xs[kT][F + 1];
    float h1[kT][D1 + 1];
};

template <int F, int D1, int D2>
__device__ __forceinline__ void load_weights(MlpSmem<F, D1, D2>& S, const float* W1, const float* b1,
                                             const float* W2, const float* b2, bool w2_transposed) {
    for (int i = threadIdx.x; i < D1 * F; i += 256) {
        const int j = i / F, f = i % F;
        S.w1t[f][j] = W1[i];
    }
    for (int i = threadIdx.x; i < D1; i += 256) S.b1[i] = b1 ? b1[i] : 0.f;
    float* w2 = &S.w2t[0][0];
    for (int i = threadIdx.x; i < D2 * D1; i += 256) {
        const int j = i / D1, k = i % D1;
        if (w2_transposed) w2[k * D2 + j] = W2[i];   // [D1][D2]
        else w2[i] = W2[i];                          // [D2][D1]
    }
    for (int i = threadIdx.x; i < D2; i += 256) S.b2[i] = b2 ? b2[i] : 0.f;
}

// h1[n][:] = ReLU(x[n] W1^T + b1) for the tile's nodes (xs loaded): 4 threads per node,
// D1 / 4 outputs each
template <int F, int D1, int D2>
__device__ __forceinline__ void hidden(MlpSmem<F, D1, D2>& S) {
    constexpr int P = D1 / 4;
    const int n = threadIdx.x >> 2, jb = (threadIdx.x & 3) * P;
    float acc[P];
#pragma unroll
    for (int q = 0; q < P; ++q) acc[q] = S.b1[jb + q];
#pragma unroll
    for (int f = 0; f < F; ++f) {
        const float xv = S.xs[n][f];
#pragma unroll
        for (int q = 0; q < P; ++q) acc[q] = fmaf(xv, S.w1t[f][jb + q], acc[q]);
    }
#pragma unroll
    for (int q = 0; q < P; ++q) S.h1[n][jb + q] = fmaxf(acc[q], 0.f);
}

template <int F>
__device__ __forceinline__ void load_x(float (*xs)[F + 1], const float* x, int64_t n0, int64_t N) {
    for (int i = threadIdx.x; i < kT * F; i += 256) {
        const int n = i / F, f = i % F;
        xs[n][f] = (n0 + n < N) ? x[(n0 + n) * F + f] : 0.f;
    }
}

template <int F, int D1, int D2>
__global__ __launch_bounds__(256) void k_mlp2_fwd(const float* __restrict__ x, int64_t N, const float* W1,
                                                  const float* b1, const float* W2, const float* b2,
                                                  float* __restrict__ h, uint32_t* __restrict__ amax) {
    __shared__ MlpSmem<F, D1, D2> S;
    load_weights(S, W1, b1, W2, b2, true);
    constexpr int P = D2 / 4;   // outputs per thread
    const int n = threadIdx.x >> 2, jb = (threadIdx.x & 3) * P;
    uint32_t m = 0;
    const int64_t tiles = (N + kT - 1) / kT;
    for (int64_t t = blockIdx.x; t < tiles; t += gridDim.x) {
        const int64_t n0 = t * kT;
        __syncthreads();
        load_x<F>(S.xs, x, n0, N);
        __syncthreads();
        hidden(S);
        __syncthreads();
        float acc[P];
#pragma unroll
        for (int q = 0; q < P; ++q) acc[q] = S.b2[jb + q];
        for (int k = 0; k < D1; ++k) {
            const float hv = S.h1[n][k];
#pragma unroll
            for (int q = 0; q < P; q += 4) {
                const float4 w = *reinterpret_cast<const float4*>(&S.w2t[k][jb + q]);
                acc[q] = fmaf(hv, w.x, acc[q]);
                acc[q + 1] = fmaf(hv, w.y, acc[q + 1]);
                acc[q + 2] = fmaf(hv, w.z, acc[q + 2]);
                acc[q + 3] = fmaf(hv, w.w, acc[q + 3]);
            }
        }
        if (n0 + n < N) {
            float* out = h + (n0 + n) * D2 + jb;
#pragma unroll
            for (int q = 0; q < P; q += 4) {
                const float4 v = make_float4(fmaxf(acc[q], 0.f), fmaxf(acc[q + 1], 0.f), fmaxf(acc[q + 2], 0.f),
                                             fmaxf(acc[q + 3], 0.f));
                m = max(m, max(max(__float_as_uint(v.x), __float_as_uint(v.y)),
                               max(__float_as_uint(v.z), __float_as_uint(v.w))));   // (>= 0)
                *reinterpret_cast<float4*>(out + q) = v;
            }
        }
    }
    if (amax) {
        for (int o = 32; o > 0; o >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, o, kWave));
        if ((threadIdx.x & 63) == 0 && m) atomicMax(amax, m);
    }
}

// Backward. g2 = dh (.) [h > 0];  dW2 += g2^T h1, db2 += sum g2;  g1 = (g2 W2) (.) [h1 > 0];
// dW1 += g1^T x, db1 += sum g1. Per workgroup partials: [D2*D1 | D2 | D1*F | D1].
template <int F, int D1, int D2>
__global__ __launch_bounds__(256) void k_mlp2_bwd(const float* __restrict__ x, int64_t N, const float* W1,
                                                  const float* b1, const float* W2, const float* __restrict__ h,
                                                  const float* __restrict__ dh, float* __restrict__ part) {
    extern __shared__ float dyn[];   // g2 [kT][D2 + 1], g1 [kT][D1 + 1]
    __shared__ MlpSmem<F, D1, D2> S;
    float (*g2)[D2 + 1] = reinterpret_cast<float (*)[D2 + 1]>(dyn);
    float (*g1)[D1 + 1] = reinterpret_cast<float (*)[D1 + 1]>(dyn + kT * (D2 + 1));
    load_weights(S, W1, b1, W2, nullptr, false);   // W2 kept as [D2][D1] in S.w2t's space
    const float* w2 = &S.w2t[0][0];
    // dW2: thread owns row j = tid / 2, columns kb..kb+D1/2 (D2 = 128 rows x 2 halves = 256 threads)
    static_assert(D2 * 2 == 256, "k_mlp2_bwd: D2 must be 128");
    constexpr int HK = D1 / 2;
    const int j2 = threadIdx.x >> 1, kb2 = (threadIdx.x & 1) * HK;
    float dw2[HK];
#pragma unroll
    for (int q = 0; q < HK; ++q) dw2[q] = 0.f;
    float db2 = 0.f;
    // g1: 4 threads per node, D1 / 4 columns each; dW1: thread owns (k = tid / 4, F / 4 columns)
    constexpr int P1 = D1 / 4, PF = F / 4;
    static_assert(D1 * 4 == 256, "k_mlp2_bwd: D1 must be 64");
    const int n1 = threadIdx.x >> 2, kb1 = (threadIdx.x & 3) * P1;
    const int k1 = threadIdx.x >> 2, fb1 = (threadIdx.x & 3) * PF;
    float dw1[PF];
#pragma unroll
    for (int q = 0; q < PF; ++q) dw1[q] = 0.f;
    float db1 = 0.f;
    const int64_t tiles = (N + kT - 1) / kT;
    for (int64_t t = blockIdx.x; t < tiles; t += gridDim.x) {
        const int64_t n0 = t * kT;
        __syncthreads();
        load_x<F>(S.xs, x, n0, N);
        for (int i = threadIdx.x; i < kT * D2; i += 256) {
            const int n = i / D2, j = i % D2;
            float v = 0.f;
            if (n0 + n < N) {
                const int64_t o = (n0 + n) * D2 + j;
                v = h[o] > 0.f ? dh[o] : 0.f;
            }
            g2[n][j] = v;
        }
        __syncthreads();
        hidden(S);
        __syncthreads();
        // weight / bias gradients of layer 2 (rows of padded tail nodes are zero in g2)
        for (int n = 0; n < kT; ++n) {
            const float gv = g2[n][j2];
            db2 += (kb2 == 0) ? gv : 0.f;
#pragma unroll
            for (int q = 0; q < HK; ++q) dw2[q] = fmaf(gv, S.h1[n][kb2 + q], dw2[q]);
        }
        // g1 = (g2 W2) masked by h1 > 0
        {
            float acc[P1];
#pragma unroll
            for (int q = 0; q < P1; ++q) acc[q] = 0.f;
            for (int j = 0; j < D2; ++j) {
                const float gv = g2[n1][j];
#pragma unroll
                for (int q = 0; q < P1; ++q) acc[q] = fmaf(gv, w2[j * D1 + kb1 + q], acc[q]);
            }
#pragma unroll
            for (int q = 0; q < P1; ++q) g1[n1][kb1 + q] = S.h1[n1][kb1 + q] > 0.f ? acc[q] : 0.f;
        }
        __syncthreads();
        for (int n = 0; n < kT; ++n) {
            const float gv = g1[n][k1];
            db1 += (fb1 == 0) ? gv : 0.f;
#pragma unroll
            for (int q = 0; q < PF; ++q) dw1[q] = fmaf(gv, S.xs[n][fb1 + q], dw1[q]);
        }
    }
    float* p = part + (int64_t)blockIdx.x * (D2 * D1 + D2 + D1 * F + D1);
#pragma unroll
    for (int q = 0; q < HK; ++q) p[j2 * D1 + kb2 + q] = dw2[q];
    if (kb2 == 0) p[D2 * D1 + j2] = db2;
#pragma unroll
    for (int q = 0; q < PF; ++q) p[D2 * D1 + D2 + k1 * F + fb1 + q] = dw1[q];
    if (fb1 == 0) p[D2 * D1 + D2 + D1 * F + k1] = db1;
}

// sum over the slots s (in order) of part[s][i], scattered into [dW2 | db2 | dW1 | db1]
__global__ __launch_bounds__(256) void k_sum_slots(const float* __restrict__ part, int slots, int L, int L0,
                                                   int L1, int L2, float* __restrict__ o0, float* __restrict__ o1,
                                                   float* __restrict__ o2, float* __restrict__ o3) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= L) return;
    float s = 0.f;
    for (int k = 0; k < slots; ++k) s += part[(int64_t)k * L + i];
    if (i < L0) o0[i] = s;
    else if (i < L0 + L1) o1[i - L0] = s;
    else if (i < L0 + L1 + L2) o2[i - L0 - L1] = s;
    else o3[i - L0 - L1 - L2] = s;
}

constexpr int kF = 16, kD1 = 64, kD2 = 128;
constexpr int kPartLen = kD2 * kD1 + kD2 + kD1 * kF + kD1;

inline int mlp_blocks(int64_t N) {
    const int64_t tiles = (N + kT - 1) / kT;
    return (int)(tiles < kMlpBlocks ? (tiles > 0 ? tiles : 1) : kMlpBlocks);
}

}  // namespace

}  // namespace bgnn

using namespace bgnn;

extern "C" int bgnn_mlp2_supported(int32_t F, int32_t D1, int32_t D2) {
    return F == kF && D1 == kD1 && D2 == kD2;
}

extern "C" int bgnn_mlp2_fwd(const float* x, int64_t N, int32_t F, int32_t D1, int32_t D2, const float* W1,
                             const float* b1, const float* W2, const float* b2, float* h, float* h_amax,
                             void* stream) {
    BGNN_REQUIRE(bgnn_mlp2_supported(F, D1, D2), "mlp2: shape %dx%dx%d not built (16x64x128 only)", F, D1, D2);
    BGNN_REQUIRE(N >= 0, "mlp2: N < 0");
    if (N == 0) return BGNN_OK;
    BGNN_REQUIRE(x && W1 && W2 && h, "mlp2: null pointer");
    BGNN_REQUIRE(aligned16(h), "mlp2: h must be 16-byte aligned");
    hipLaunchKernelGGL((k_mlp2_fwd<kF, kD1, kD2>), dim3(mlp_blocks(N)), dim3(256), 0, as_stream(stream), x, N, W1,
                       b1, W2, b2, h, reinterpret_cast<uint32_t*>(h_amax));
    BGNN_CHECK_LAUNCH();
    return BGNN_OK;
}

extern "C" size_t bgnn_mlp2_bwd_ws_bytes(int64_t N) {
    return (size_t)mlp_blocks(N) * kPartLen * sizeof(float);
}

extern "C" int bgnn_mlp2_bwd(const float* x, int64_t N, int32_t F, int32_t D1, int32_t D2, const float* W1,
                             const float* b1, const float* W2, const float* h, const float* dh, float* dW1,
                             float* db1, float* dW2, float* db2, void* ws, size_t ws_bytes, void* stream) {
    BGNN_REQUIRE(bgnn_mlp2_supported(F, D1, D2), "mlp2: shape %dx%dx%d not built (16x64x128 only)", F, D1, D2);
    BGNN_REQUIRE(N >= 0, "mlp2: N < 0");
    BGNN_REQUIRE(dW1 && db1 && dW2 && db2, "mlp2_bwd: null gradient output");
    hipStream_t s = as_stream(stream);
    if (N == 0) {
        BGNN_HIP(hipMemsetAsync(dW1, 0, sizeof(float) * kD1 * kF, s));
        BGNN_HIP(hipMemsetAsync(db1, 0, sizeof(float) * kD1, s));
        BGNN_HIP(hipMemsetAsync(dW2, 0, sizeof(float) * kD2 * kD1, s));
        BGNN_HIP(hipMemsetAsync(db2, 0, sizeof(float) * kD2, s));
        return BGNN_OK;
    }
    BGNN_REQUIRE(x && W1 && W2 && h && dh, "mlp2_bwd: null pointer");
    BGNN_REQUIRE(ws && ws_bytes >= bgnn_mlp2_bwd_ws_bytes(N), "mlp2_bwd: workspace too small");
    const int blocks = mlp_blocks(N);
    float* part = static_cast<float*>(ws);
    const size_t dyn = sizeof(float) * kT * ((kD2 + 1) + (kD1 + 1));
    hipLaunchKernelGGL((k_mlp2_bwd<kF, kD1, kD2>), dim3(blocks), dim3(256), dyn, s, x, N, W1, b1, W2, h, dh, part);
    BGNN_CHECK_LAUNCH();
    // slot sums straight into the four gradient tensors (partial layout [dW2 | db2 | dW1 | db1])
    hipLaunchKernelGGL(k_sum_slots, dim3((kPartLen + 255) / 256), dim3(256), 0, s, part, blocks, kPartLen,
                       kD2 * kD1, kD2, kD1 * kF, dW2, db2, dW1, db1);
    BGNN_CHECK_LAUNCH();
    return BGNN_OK;
}
