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
    float xs[kT][F + 4];       // row strides multiples of 4: float4 reads
    float h1[kT][D1 + 4];
};

template <int F, int D1, int D2, int NT>
__device__ __forceinline__ void load_weights(MlpSmem<F, D1, D2>& S, const float* W1, const float* b1,
                                             const float* W2, const float* b2, bool w2_transposed) {
    for (int i = threadIdx.x; i < D1 * F; i += NT) {
        const int j = i / F, f = i % F;
        S.w1t[f][j] = W1[i];
    }
    for (int i = threadIdx.x; i < D1; i += NT) S.b1[i] = b1 ? b1[i] : 0.f;
    float* w2 = &S.w2t[0][0];
    if (w2_transposed && (((uintptr_t)W2 & 15) == 0)) {
        // W2^T [D1][D2]: lanes run over the output j, so the LDS words a wave writes are
        // consecutive (the element-order walk wrote one bank 64 times per instruction); each
        // lane reads one float4 of W2's row j
        for (int i = threadIdx.x; i < D2 * (D1 / 4); i += NT) {
            const int j = i % D2, k = (i / D2) * 4;
            const float4 v = *reinterpret_cast<const float4*>(W2 + j * D1 + k);
            w2[(k + 0) * D2 + j] = v.x;
            w2[(k + 1) * D2 + j] = v.y;
            w2[(k + 2) * D2 + j] = v.z;
            w2[(k + 3) * D2 + j] = v.w;
        }
    } else {
        for (int i = threadIdx.x; i < D2 * D1; i += NT) {
            const int j = i / D1, k = i % D1;
            if (w2_transposed) w2[k * D2 + j] = W2[i];   // [D1][D2]
            else w2[i] = W2[i];                          // [D2][D1]
        }
    }
    for (int i = threadIdx.x; i < D2; i += NT) S.b2[i] = b2 ? b2[i] : 0.f;
}

__device__ __forceinline__ void ld4(const float* p, float (&v)[4]) {
    const float4 t = *reinterpret_cast<const float4*>(p);
    v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
}

// h1 = ReLU(x W1^T + b1) for the tile's 64 nodes (xs loaded): thread = 64 / (NT / 16) nodes x 4
// hidden units (every unit's sum runs over f in order, whatever NT)
template <int F, int D1, int D2, int NT>
__device__ __forceinline__ void hidden(MlpSmem<F, D1, D2>& S) {
    static_assert(D1 == 64 && kT == 64 && (NT == 256 || NT == 512), "hidden: 16 unit groups of 4");
    constexpr int NP = kT * 16 / NT;   // nodes per thread
    const int tn = threadIdx.x >> 4, tk = threadIdx.x & 15;
    float acc[NP][4];
#pragma unroll
    for (int i = 0; i < NP; ++i)
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[i][c] = S.b1[tk * 4 + c];
#pragma unroll
    for (int f = 0; f < F; ++f) {
        float w[4];
        ld4(&S.w1t[f][tk * 4], w);
#pragma unroll
        for (int i = 0; i < NP; ++i) {
            const float xv = S.xs[tn * NP + i][f];
#pragma unroll
            for (int c = 0; c < 4; ++c) acc[i][c] = fmaf(xv, w[c], acc[i][c]);
        }
    }
#pragma unroll
    for (int i = 0; i < NP; ++i)
        *reinterpret_cast<float4*>(&S.h1[tn * NP + i][tk * 4]) =
            make_float4(fmaxf(acc[i][0], 0.f), fmaxf(acc[i][1], 0.f), fmaxf(acc[i][2], 0.f), fmaxf(acc[i][3], 0.f));
}

template <int F, int NT>
__device__ __forceinline__ void load_x(float (*xs)[F + 4], const float* x, int64_t n0, int64_t N) {
    for (int i = threadIdx.x; i < kT * F; i += NT) {
        const int n = i / F, f = i % F;
        xs[n][f] = (n0 + n < N) ? x[(n0 + n) * F + f] : 0.f;
    }
}

// forward: thread = 4 nodes x 8 outputs of layer 2 (W2^T row segments as float4 pairs). 256
// threads, two workgroups per CU: at 512 threads of 4 x 4 outputs the loop reads twice the LDS
// bytes per FMA and ran 72 us against 54 (tools/mlp2_ab.py)
template <int F, int D1, int D2>
__global__ __launch_bounds__(256) void k_mlp2_fwd(const float* __restrict__ x, int64_t N, const float* W1,
                                                  const float* b1, const float* W2, const float* b2,
                                                  float* __restrict__ h, uint32_t* __restrict__ amax) {
    static_assert(D2 == 128, "k_mlp2_fwd: 16 column groups of 8");
    __shared__ MlpSmem<F, D1, D2> S;
    load_weights<F, D1, D2, 256>(S, W1, b1, W2, b2, true);
    const int tn = threadIdx.x >> 4, tj = threadIdx.x & 15;
    uint32_t m = 0;
    const int64_t tiles = (N + kT - 1) / kT;
    for (int64_t t = blockIdx.x; t < tiles; t += gridDim.x) {
        const int64_t n0 = t * kT;
        __syncthreads();
        load_x<F, 256>(S.xs, x, n0, N);
        __syncthreads();
        hidden<F, D1, D2, 256>(S);
        __syncthreads();
        float acc[4][8];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int c = 0; c < 8; ++c) acc[i][c] = S.b2[tj * 8 + c];
        for (int k = 0; k < D1; ++k) {
            float wa[4], wb[4];
            ld4(&S.w2t[k][tj * 8], wa);
            ld4(&S.w2t[k][tj * 8 + 4], wb);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const float hv = S.h1[tn * 4 + i][k];
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    acc[i][c] = fmaf(hv, wa[c], acc[i][c]);
                    acc[i][c + 4] = fmaf(hv, wb[c], acc[i][c + 4]);
                }
            }
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int64_t node = n0 + tn * 4 + i;
            if (node >= N) continue;
            float* out = h + node * D2 + tj * 8;
#pragma unroll
            for (int c = 0; c < 8; c += 4) {
                const float4 v = make_float4(fmaxf(acc[i][c], 0.f), fmaxf(acc[i][c + 1], 0.f),
                                             fmaxf(acc[i][c + 2], 0.f), fmaxf(acc[i][c + 3], 0.f));
                m = max(m, max(max(__float_as_uint(v.x), __float_as_uint(v.y)),
                               max(__float_as_uint(v.z), __float_as_uint(v.w))));   // (>= 0)
                *reinterpret_cast<float4*>(out + c) = v;
            }
        }
    }
    if (amax) {
        for (int o = 32; o > 0; o >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, o, kWave));
        if ((threadIdx.x & 63) == 0 && m) atomicMax(amax, m);
    }
}

// Backward. g2 = dh (.) [h > 0];  dW2 += g2^T h1, db2 += sum g2;  g1 = (g2 W2) (.) [h1 > 0];
// dW1 += g1^T x, db1 += sum g1. Per workgroup partials: [D2*D1 | D2 | D1*F | D1]. 512 threads (two
// waves per SIMD: at 256 the one wave per SIMD left every LDS read's latency exposed); every
// accumulator still sums its nodes in order, so the partials do not depend on the thread count.
constexpr int kBwdThreads = 512;

template <int F, int D1, int D2>
__global__ __launch_bounds__(kBwdThreads) void k_mlp2_bwd(const float* __restrict__ x, int64_t N, const float* W1,
                                                          const float* b1, const float* W2, const float* __restrict__ h,
                                                          const float* __restrict__ dh, float* __restrict__ part) {
    static_assert(D2 == 128 && D1 == 64 && F == 16, "k_mlp2_bwd: built for 16 x 64 x 128");
    constexpr int NT = kBwdThreads;
    constexpr int G2 = D2 + 4, G1 = D1 + 4;
    extern __shared__ float dyn[];   // g2 [kT][G2], g1 [kT][G1]
    __shared__ MlpSmem<F, D1, D2> S;
    float (*g2)[G2] = reinterpret_cast<float (*)[G2]>(dyn);
    float (*g1)[G1] = reinterpret_cast<float (*)[G1]>(dyn + kT * G2);
    load_weights<F, D1, D2, NT>(S, W1, b1, W2, nullptr, false);   // W2 kept as [D2][D1] in S.w2t's space
    const float* w2 = &S.w2t[0][0];
    const int hi = threadIdx.x >> 4, lo = threadIdx.x & 15;
    // dW2: rows hi*4..+4, columns lo*4..+4 (16 accumulators); db2 by the lo == 0 threads
    float dw2[4][4], db2[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        db2[c] = 0.f;
#pragma unroll
        for (int q = 0; q < 4; ++q) dw2[c][q] = 0.f;
    }
    // dW1: row k1 = tid / 8, columns fb1..fb1+2; db1 by the fb1 == 0 threads
    const int k1 = threadIdx.x >> 3, fb1 = (threadIdx.x & 7) * 2;
    float dw1[2] = {0.f, 0.f};
    float db1 = 0.f;
    const int64_t tiles = (N + kT - 1) / kT;
    for (int64_t t = blockIdx.x; t < tiles; t += gridDim.x) {
        const int64_t n0 = t * kT;
        __syncthreads();
        load_x<F, NT>(S.xs, x, n0, N);
        for (int i = threadIdx.x; i < kT * (D2 / 4); i += NT) {
            const int n = i / (D2 / 4), j4 = (i % (D2 / 4)) * 4;
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if (n0 + n < N) {
                const int64_t o = (n0 + n) * D2 + j4;
                const float4 hv = *reinterpret_cast<const float4*>(h + o);
                const float4 gv = *reinterpret_cast<const float4*>(dh + o);
                v = make_float4(hv.x > 0.f ? gv.x : 0.f, hv.y > 0.f ? gv.y : 0.f, hv.z > 0.f ? gv.z : 0.f,
                                hv.w > 0.f ? gv.w : 0.f);
            }
            *reinterpret_cast<float4*>(&g2[n][j4]) = v;
        }
        __syncthreads();
        hidden<F, D1, D2, NT>(S);
        __syncthreads();
        // layer-2 weight / bias gradients (rows of padded tail nodes are zero in g2)
        for (int n = 0; n < kT; ++n) {
            float ga[4], hv[4];
            ld4(&g2[n][hi * 4], ga);
            ld4(&S.h1[n][lo * 4], hv);
#pragma unroll
            for (int q = 0; q < 4; ++q)
#pragma unroll
                for (int c = 0; c < 4; ++c) dw2[c][q] = fmaf(ga[c], hv[q], dw2[c][q]);
            if (lo == 0) {
#pragma unroll
                for (int c = 0; c < 4; ++c) db2[c] += ga[c];
            }
        }
        // g1 = (g2 W2) masked by h1 > 0: thread = 2 nodes (hi) x 4 hidden units (lo)
        {
            float acc[2][4];
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int q = 0; q < 4; ++q) acc[i][q] = 0.f;
            for (int j = 0; j < D2; ++j) {
                float w[4];
                ld4(&w2[j * D1 + lo * 4], w);
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    const float gv = g2[hi * 2 + i][j];
#pragma unroll
                    for (int q = 0; q < 4; ++q) acc[i][q] = fmaf(gv, w[q], acc[i][q]);
                }
            }
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                float hv[4];
                ld4(&S.h1[hi * 2 + i][lo * 4], hv);
                *reinterpret_cast<float4*>(&g1[hi * 2 + i][lo * 4]) =
                    make_float4(hv[0] > 0.f ? acc[i][0] : 0.f, hv[1] > 0.f ? acc[i][1] : 0.f,
                                hv[2] > 0.f ? acc[i][2] : 0.f, hv[3] > 0.f ? acc[i][3] : 0.f);
            }
        }
        __syncthreads();
        for (int n = 0; n < kT; ++n) {
            const float gv = g1[n][k1];
            const float2 xv = *reinterpret_cast<const float2*>(&S.xs[n][fb1]);
            db1 += (fb1 == 0) ? gv : 0.f;
            dw1[0] = fmaf(gv, xv.x, dw1[0]);
            dw1[1] = fmaf(gv, xv.y, dw1[1]);
        }
    }
    float* p = part + (int64_t)blockIdx.x * (D2 * D1 + D2 + D1 * F + D1);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        *reinterpret_cast<float4*>(p + (hi * 4 + c) * D1 + lo * 4) = make_float4(dw2[c][0], dw2[c][1], dw2[c][2], dw2[c][3]);
        if (lo == 0) p[D2 * D1 + hi * 4 + c] = db2[c];
    }
    *reinterpret_cast<float2*>(p + D2 * D1 + D2 + k1 * F + fb1) = make_float2(dw1[0], dw1[1]);
    if (fb1 == 0) p[D2 * D1 + D2 + D1 * F + k1] = db1;
}

// two-stage, fixed-order slot sums: stage 1 sums slot group y (slots [y*per, (y+1)*per)) of
// column i into tmp[y][i]; stage 2 sums the groups in order into [dW2 | db2 | dW1 | db1]
constexpr int kSumGroups = 16;

__global__ __launch_bounds__(256) void k_sum_slots1(const float* __restrict__ part, int slots, int L,
                                                    float* __restrict__ tmp) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= L) return;
    const int per = (slots + kSumGroups - 1) / kSumGroups;
    const int s0 = blockIdx.y * per, s1 = min(slots, s0 + per);
    float s = 0.f;
    for (int k = s0; k < s1; ++k) s += part[(int64_t)k * L + i];
    tmp[(int64_t)blockIdx.y * L + i] = s;
}

__global__ __launch_bounds__(256) void k_sum_slots(const float* __restrict__ tmp, int L, int L0, int L1, int L2,
                                                   float* __restrict__ o0, float* __restrict__ o1,
                                                   float* __restrict__ o2, float* __restrict__ o3) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= L) return;
    float s = 0.f;
    for (int k = 0; k < kSumGroups; ++k) s += tmp[(int64_t)k * L + i];
    if (i < L0) o0[i] = s;
    else if (i < L0 + L1) o1[i - L0] = s;
    else if (i < L0 + L1 + L2) o2[i - L0 - L1] = s;
    else o3[i - L0 - L1 - L2] = s;
}

constexpr int kF = 16, kD1 = 64, kD2 = 128;
constexpr int kPartLen = kD2 * kD1 + kD2 + kD1 * kF + kD1;

inline int mlp_blocks(int64_t N, int cap = kMlpBlocks) {
    const int64_t tiles = (N + kT - 1) / kT;
    return (int)(tiles < cap ? (tiles > 0 ? tiles : 1) : cap);
}

// ---------------------------------------------------------------------------
// Small-batch Linear layers (ABI 8): the decoder MLP Linear(512,128).ReLU.Linear(128,64).ReLU.
// Linear(64,1) (Models/BuckGNN.py:94-100) runs on the pooled [B = graphs, H] features -- a few
// thousand outputs per layer, where a library GEMM launch plus a separate ReLU kernel (and the
// backward's bias reductions and ReLU masks) cost ~8 us each for nanoseconds of work. Here one
// launch per layer and direction, bias and ReLU (mask) inside; every output is reduced by one wave
// in a fixed order (deterministic).

// y[b, n] = act(sum_k x[b, k] W[n, k] + bias[n]): one wave per output, lanes split K (K % 4 == 0)
__global__ __launch_bounds__(256) void k_small_linear_fwd(const float* __restrict__ x, int64_t B, int K,
                                                          const float* __restrict__ W, const float* __restrict__ bias,
                                                          int N, int relu, float* __restrict__ y) {
    const int lane = threadIdx.x & 63;
    const int64_t o = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (o >= B * N) return;
    const int64_t b = o / N;
    const int n = (int)(o % N);
    const float4* xr = reinterpret_cast<const float4*>(x + b * K);
    const float4* wr = reinterpret_cast<const float4*>(W + (int64_t)n * K);
    float acc = 0.f;
    for (int k4 = lane; k4 < K / 4; k4 += 64) {
        const float4 a = xr[k4], w = wr[k4];
        acc = fmaf(a.x, w.x, acc);
        acc = fmaf(a.y, w.y, acc);
        acc = fmaf(a.z, w.z, acc);
        acc = fmaf(a.w, w.w, acc);
    }
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
    if (lane == 0) {
        float v = acc + (bias ? bias[n] : 0.f);
        y[o] = relu ? fmaxf(v, 0.f) : v;
    }
}

// backward of y = act(x W^T + bias), g = gy masked by y > 0 when act is a ReLU (y != NULL):
//   dW[n, k] = sum_b g[b, n] x[b, k]     (threads 0 .. N K / 4: one float4 of k each, loop over b)
//   db[n]    = sum_b g[b, n]             (the k4 == 0 thread of each n)
//   dx[b, k] = sum_n g[b, n] W[n, k]     (one wave per float4 of dx, lanes split n)
__global__ __launch_bounds__(256) void k_small_linear_bwd_w(const float* __restrict__ gy, const float* __restrict__ y,
                                                            const float* __restrict__ x, int64_t B, int K, int N,
                                                            float* __restrict__ dW, float* __restrict__ db) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int K4 = K / 4;
    if (t >= (int64_t)N * K4) return;
    const int n = (int)(t / K4), k4 = (int)(t % K4);
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    float bs = 0.f;
    for (int64_t b = 0; b < B; ++b) {
        float g = gy[b * N + n];
        if (y && !(y[b * N + n] > 0.f)) g = 0.f;
        const float4 a = reinterpret_cast<const float4*>(x + b * K)[k4];
        acc.x = fmaf(g, a.x, acc.x);
        acc.y = fmaf(g, a.y, acc.y);
        acc.z = fmaf(g, a.z, acc.z);
        acc.w = fmaf(g, a.w, acc.w);
        bs += g;
    }
    reinterpret_cast<float4*>(dW + (int64_t)n * K)[k4] = acc;
    if (db && k4 == 0) db[n] = bs;
}

__global__ __launch_bounds__(256) void k_small_linear_bwd_x(const float* __restrict__ gy, const float* __restrict__ y,
                                                            const float* __restrict__ W, int64_t B, int K, int N,
                                                            float* __restrict__ dx) {
    // one wave per float4 of dx: lanes split N, a fixed shuffle tree sums them (a thread looping
    // over all N rows of W ran latency-bound at ~20 us for the 512-wide layer)
    const int lane = threadIdx.x & 63;
    const int64_t o = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int K4 = K / 4;
    if (o >= B * K4) return;
    const int64_t b = o / K4;
    const int k4 = (int)(o % K4);
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int n = lane; n < N; n += 64) {
        float g = gy[b * N + n];
        if (y && !(y[b * N + n] > 0.f)) g = 0.f;
        const float4 w = reinterpret_cast<const float4*>(W + (int64_t)n * K)[k4];
        acc.x = fmaf(g, w.x, acc.x);
        acc.y = fmaf(g, w.y, acc.y);
        acc.z = fmaf(g, w.z, acc.z);
        acc.w = fmaf(g, w.w, acc.w);
    }
    for (int off = 32; off > 0; off >>= 1) {
        acc.x += __shfl_xor(acc.x, off, 64);
        acc.y += __shfl_xor(acc.y, off, 64);
        acc.z += __shfl_xor(acc.z, off, 64);
        acc.w += __shfl_xor(acc.w, off, 64);
    }
    if (lane == 0) reinterpret_cast<float4*>(dx + b * K)[k4] = acc;
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
    // 2 workgroups per CU (58 KB of LDS each)
    hipLaunchKernelGGL((k_mlp2_fwd<kF, kD1, kD2>), dim3(mlp_blocks(N, 2 * kMlpBlocks)), dim3(256), 0, as_stream(stream), x, N, W1,
                       b1, W2, b2, h, reinterpret_cast<uint32_t*>(h_amax));
    BGNN_CHECK_LAUNCH();
    return BGNN_OK;
}

extern "C" size_t bgnn_mlp2_bwd_ws_bytes(int64_t N) {
    return (size_t)(mlp_blocks(N) + kSumGroups) * kPartLen * sizeof(float);
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
    const size_t dyn = sizeof(float) * kT * ((kD2 + 4) + (kD1 + 4));
    hipLaunchKernelGGL((k_mlp2_bwd<kF, kD1, kD2>), dim3(blocks), dim3(kBwdThreads), dyn, s, x, N, W1, b1, W2, h, dh, part);
    BGNN_CHECK_LAUNCH();
    // slot sums straight into the four gradient tensors (partial layout [dW2 | db2 | dW1 | db1])
    float* tmp = part + (int64_t)blocks * kPartLen;
    hipLaunchKernelGGL(k_sum_slots1, dim3((kPartLen + 255) / 256, kSumGroups), dim3(256), 0, s, part, blocks,
                       kPartLen, tmp);
    BGNN_CHECK_LAUNCH();
    hipLaunchKernelGGL(k_sum_slots, dim3((kPartLen + 255) / 256), dim3(256), 0, s, tmp, kPartLen, kD2 * kD1, kD2,
                       kD1 * kF, dW2, db2, dW1, db1);
    BGNN_CHECK_LAUNCH();
    return BGNN_OK;
}

extern "C" int bgnn_small_linear_fwd(const float* x, int64_t B, int32_t K, const float* W, const float* bias, int32_t N,
                                     int32_t relu, float* y, void* stream) {
    BGNN_REQUIRE(x && W && y && B >= 0 && K > 0 && N > 0, "small_linear_fwd: bad args");
    BGNN_REQUIRE(K % 4 == 0 && aligned16(x) && aligned16(W), "small_linear_fwd: K %% 4 == 0 and 16-B aligned x, W");
    if (B == 0) return BGNN_OK;
    const int64_t waves = B * N;
    hipLaunchKernelGGL(k_small_linear_fwd, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, as_stream(stream), x, B, K,
                       W, bias, N, relu, y);
    BGNN_CHECK_LAUNCH();
    return BGNN_OK;
}

extern "C" int bgnn_small_linear_bwd(const float* gy, const float* y, const float* x, int64_t B, int32_t K,
                                     const float* W, int32_t N, float* dx, float* dW, float* db, void* stream) {
    BGNN_REQUIRE(gy && x && W && dW && B >= 0 && K > 0 && N > 0, "small_linear_bwd: bad args");
    BGNN_REQUIRE(K % 4 == 0 && aligned16(x) && aligned16(W) && aligned16(dW) && (!dx || aligned16(dx)),
                 "small_linear_bwd: K %% 4 == 0 and 16-B aligned x, W, dW, dx");
    hipStream_t s = as_stream(stream);
    const int64_t tw = (int64_t)N * (K / 4);
    hipLaunchKernelGGL(k_small_linear_bwd_w, dim3((unsigned)((tw + 255) / 256)), dim3(256), 0, s, gy, y, x, B, K, N, dW,
                       db);
    BGNN_CHECK_LAUNCH();
    if (dx && B > 0) {
        const int64_t waves = B * (K / 4);
        hipLaunchKernelGGL(k_small_linear_bwd_x, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, s, gy, y, W, B, K, N,
                           dx);
        BGNN_CHECK_LAUNCH();
    }
    return BGNN_OK;
}
