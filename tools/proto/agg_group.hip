// Prototype: row-group aggregation with a deduplicated source list per group.
// A wave owns R consecutive target rows; the group's plan lists every distinct
// (source, occurrence) once with an R-bit mask of the targets that use it, so a
// source row shared by several targets of the group (mesh bands i±n, i±1) is
// fetched once. Experiment only (tools/proto_agg.py).
#include <hip/hip_runtime.h>
#include <stdint.h>

struct GArgs {
    const float* x;
    float* out;
    const int32_t* gptr;
    const int32_t* gsrc;
    const uint32_t* gmask;
    int64_t G, N;
    int H;
};

template <int R, int NV, int U, int MODE>
__global__ __launch_bounds__(256) void k_grp(GArgs A) {
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    constexpr int S = (NV == 2) ? 4 : 2;  // group slots per block
    const int slot = (NV == 2) ? wave : (wave >> 1);
    const int half = (NV == 2) ? 0 : (wave & 1);
    const int G8 = gridDim.x >> 3;
    const int xg = blockIdx.x & 7, bi = blockIdx.x >> 3;
    const int64_t lo = A.G * xg / 8, hi = A.G * (xg + 1) / 8;
    const int W = S * G8;
    int cpos[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) cpos[v] = half * 256 + (lane + 64 * v) * 4;
    for (int64_t g = lo + bi * S + slot; g < hi; g += W) {
        const int32_t e0 = A.gptr[g], e1 = A.gptr[g + 1];
        float4 acc[R][NV];
#pragma unroll
        for (int t = 0; t < R; ++t)
#pragma unroll
            for (int v = 0; v < NV; ++v) acc[t][v] = make_float4(0.f, 0.f, 0.f, 0.f);
        for (int32_t eb = e0; eb < e1; eb += 64) {
            const int n = min(64, e1 - eb);
            const int32_t sl = lane < n ? A.gsrc[eb + lane] : 0;
            const uint32_t ml = lane < n ? A.gmask[eb + lane] : 0u;
            for (int u0 = 0; u0 < n; u0 += U) {
                float4 val[U][NV];
                uint32_t m[U];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int k = (u0 + u < n) ? u0 + u : u0;
                    const int32_t j = __builtin_amdgcn_readlane(sl, k);
                    m[u] = (u0 + u < n) ? (uint32_t)__builtin_amdgcn_readlane((int)ml, k) : 0u;
#pragma unroll
                    for (int v = 0; v < NV; ++v)
                        val[u][v] = *reinterpret_cast<const float4*>(A.x + (int64_t)j * A.H + cpos[v]);
                }
#pragma unroll
                for (int u = 0; u < U; ++u)
#pragma unroll
                    for (int t = 0; t < R; ++t) {
                        const bool on = (m[u] >> t) & 1u;
                        if constexpr (MODE == 0) {
#pragma unroll
                            for (int v = 0; v < NV; ++v) {
                                acc[t][v].x += on ? val[u][v].x : 0.f;
                                acc[t][v].y += on ? val[u][v].y : 0.f;
                                acc[t][v].z += on ? val[u][v].z : 0.f;
                                acc[t][v].w += on ? val[u][v].w : 0.f;
                            }
                        } else if constexpr (MODE == 1) {
                            // uniform branch kept as a branch (the asm blocks if-conversion)
                            if (on) {
                                asm volatile("" ::: "memory");
#pragma unroll
                                for (int v = 0; v < NV; ++v) {
                                    acc[t][v].x += val[u][v].x;
                                    acc[t][v].y += val[u][v].y;
                                    acc[t][v].z += val[u][v].z;
                                    acc[t][v].w += val[u][v].w;
                                }
                            }
                        } else {
                            // 0/1 weight FMA (not NaN/inf-safe: experiment only)
                            const float w = on ? 1.f : 0.f;
#pragma unroll
                            for (int v = 0; v < NV; ++v) {
                                acc[t][v].x = fmaf(val[u][v].x, w, acc[t][v].x);
                                acc[t][v].y = fmaf(val[u][v].y, w, acc[t][v].y);
                                acc[t][v].z = fmaf(val[u][v].z, w, acc[t][v].z);
                                acc[t][v].w = fmaf(val[u][v].w, w, acc[t][v].w);
                            }
                        }
                    }
            }
        }
#pragma unroll
        for (int t = 0; t < R; ++t) {
            const int64_t r = g * R + t;
            if (r < A.N)
#pragma unroll
                for (int v = 0; v < NV; ++v) *reinterpret_cast<float4*>(A.out + r * A.H + cpos[v]) = acc[t][v];
        }
    }
}

#define LAUNCH1(R, NV, U, M)                                                                     \
    if (r == R && nv == NV && u == U && mode == M) {                                              \
        hipLaunchKernelGGL((k_grp<R, NV, U, M>), dim3(blocks), dim3(256), 0, (hipStream_t)s, A); \
        return (int)hipGetLastError();                                                           \
    }
#define LAUNCH(R, NV, U) LAUNCH1(R, NV, U, 0) LAUNCH1(R, NV, U, 1) LAUNCH1(R, NV, U, 2)

extern "C" int proto_grp(int r, int nv, int u, int mode, int blocks, const float* x, float* out, const int32_t* gptr,
                         const int32_t* gsrc, const uint32_t* gmask, int64_t G, int64_t N, int H, void* s) {
    GArgs A{x, out, gptr, gsrc, gmask, G, N, H};
    LAUNCH(4, 2, 8)
    LAUNCH(8, 2, 8)
    LAUNCH(4, 2, 12)
    LAUNCH(8, 1, 12)
    LAUNCH(16, 1, 12)
    return -1;
}

// ---------------------------------------------------------------------------
// Column-split XCD mapping: XCD group x = blockIdx % 8 owns column slice (x % CS) of the
// rows [(x / CS) * N / (8 / CS), ...): an XCD's working set is one graph's column slice.
// CS = 4: quarter rows (512 B) as float2 per lane; CS = 2: half rows (1 KiB) as float4.
struct QArgs {
    const float* x;
    float* out;
    const int32_t* rowptr;
    const int32_t* col;
    const int32_t* gptr;
    const int32_t* gsrc;
    const uint32_t* gmask;
    int64_t N, G;
    int H;
};

template <int CS>
struct Cols;
template <>
struct Cols<4> {
    typedef float2 T;
    static __device__ __forceinline__ void add(float2& a, const float2& b, bool on) {
        a.x += on ? b.x : 0.f;
        a.y += on ? b.y : 0.f;
    }
    static __device__ __forceinline__ float2 zero() { return make_float2(0.f, 0.f); }
    static constexpr int W = 2;
};
template <>
struct Cols<2> {
    typedef float4 T;
    static __device__ __forceinline__ void add(float4& a, const float4& b, bool on) {
        a.x += on ? b.x : 0.f;
        a.y += on ? b.y : 0.f;
        a.z += on ? b.z : 0.f;
        a.w += on ? b.w : 0.f;
    }
    static __device__ __forceinline__ float4 zero() { return make_float4(0.f, 0.f, 0.f, 0.f); }
    static constexpr int W = 4;
};

template <int CS, int U>
__global__ __launch_bounds__(256) void k_q(QArgs A) {
    typedef typename Cols<CS>::T T;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int xg = blockIdx.x & 7, bi = blockIdx.x >> 3;
    constexpr int NR = 8 / CS;
    const int q = xg % CS, rg = xg / CS;
    const int64_t lo = A.N * rg / NR, hi = A.N * (rg + 1) / NR;
    const int W = 4 * (gridDim.x >> 3);
    const int cp = q * (A.H / CS) + lane * Cols<CS>::W;
    const int64_t first = lo + bi * 4 + wave;
    const int T_ = first < hi ? (int)((hi - first + W - 1) / W) : 0;
    for (int t0 = 0; t0 < T_; t0 += 64) {
        const int nrow = min(64, T_ - t0);
        int32_t rp_lo = 0, rp_hi = 0;
        if (lane < nrow) {
            const int64_t rl = first + (int64_t)W * (t0 + lane);
            rp_lo = A.rowptr[rl];
            rp_hi = A.rowptr[rl + 1];
        }
        int32_t nb = __builtin_amdgcn_readlane(rp_lo, 0), ndeg = __builtin_amdgcn_readlane(rp_hi, 0) - nb;
        int32_t cv = (lane < ndeg) ? A.col[nb + lane] : 0;
        for (int k = 0; k < nrow; ++k) {
            const int64_t r = first + (int64_t)W * (t0 + k);
            const int32_t deg = ndeg;
            const int32_t cur = cv;
            if (k + 1 < nrow) {
                nb = __builtin_amdgcn_readlane(rp_lo, k + 1);
                ndeg = __builtin_amdgcn_readlane(rp_hi, k + 1) - nb;
                cv = (lane < ndeg) ? A.col[nb + lane] : 0;
            }
            T acc = Cols<CS>::zero();
            for (int e0 = 0; e0 < deg; e0 += U) {
                const int nvalid = min(U, deg - e0);
                T val[U];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int slot = (u < nvalid) ? e0 + u : e0;
                    const int32_t j = __builtin_amdgcn_readlane(cur, slot);
                    val[u] = *reinterpret_cast<const T*>(A.x + (int64_t)j * A.H + cp);
                }
#pragma unroll
                for (int u = 0; u < U; ++u) Cols<CS>::add(acc, val[u], u < nvalid);
            }
            *reinterpret_cast<T*>(A.out + r * A.H + cp) = acc;
        }
    }
}

template <int CS, int R, int U>
__global__ __launch_bounds__(256) void k_qg(QArgs A) {
    typedef typename Cols<CS>::T T;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int xg = blockIdx.x & 7, bi = blockIdx.x >> 3;
    constexpr int NR = 8 / CS;
    const int q = xg % CS, rg = xg / CS;
    const int64_t lo = A.G * rg / NR, hi = A.G * (rg + 1) / NR;
    const int W = 4 * (gridDim.x >> 3);
    const int cp = q * (A.H / CS) + lane * Cols<CS>::W;
    for (int64_t g = lo + bi * 4 + wave; g < hi; g += W) {
        const int32_t e0 = A.gptr[g], e1 = A.gptr[g + 1];
        T acc[R];
#pragma unroll
        for (int t = 0; t < R; ++t) acc[t] = Cols<CS>::zero();
        for (int32_t eb = e0; eb < e1; eb += 64) {
            const int n = min(64, e1 - eb);
            const int32_t sl = lane < n ? A.gsrc[eb + lane] : 0;
            const uint32_t ml = lane < n ? A.gmask[eb + lane] : 0u;
            for (int u0 = 0; u0 < n; u0 += U) {
                T val[U];
                uint32_t m[U];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int k = (u0 + u < n) ? u0 + u : u0;
                    const int32_t j = __builtin_amdgcn_readlane(sl, k);
                    m[u] = (u0 + u < n) ? (uint32_t)__builtin_amdgcn_readlane((int)ml, k) : 0u;
                    val[u] = *reinterpret_cast<const T*>(A.x + (int64_t)j * A.H + cp);
                }
#pragma unroll
                for (int u = 0; u < U; ++u)
#pragma unroll
                    for (int t = 0; t < R; ++t) Cols<CS>::add(acc[t], val[u], (m[u] >> t) & 1u);
            }
        }
#pragma unroll
        for (int t = 0; t < R; ++t) {
            const int64_t r = g * R + t;
            if (r < A.N) *reinterpret_cast<T*>(A.out + r * A.H + cp) = acc[t];
        }
    }
}

extern "C" int proto_q(int kind, int cs, int r, int u, int blocks, const float* x, float* out, const int32_t* rowptr,
                       const int32_t* col, const int32_t* gptr, const int32_t* gsrc, const uint32_t* gmask, int64_t N,
                       int64_t G, int H, void* s) {
    QArgs A{x, out, rowptr, col, gptr, gsrc, gmask, N, G, H};
    hipStream_t st = (hipStream_t)s;
#define QL(KIND, CS, R, U, KERN)                                                   \
    if (kind == KIND && cs == CS && r == R && u == U) {                            \
        hipLaunchKernelGGL(KERN, dim3(blocks), dim3(256), 0, st, A);               \
        return (int)hipGetLastError();                                             \
    }
    QL(0, 4, 1, 12, (k_q<4, 12>))
    QL(0, 4, 1, 16, (k_q<4, 16>))
    QL(0, 2, 1, 12, (k_q<2, 12>))
    QL(1, 4, 4, 12, (k_qg<4, 4, 12>))
    QL(1, 4, 8, 12, (k_qg<4, 8, 12>))
    QL(1, 4, 8, 16, (k_qg<4, 8, 16>))
    QL(1, 2, 4, 12, (k_qg<2, 4, 12>))
    QL(1, 2, 8, 12, (k_qg<2, 8, 12>))
#undef QL
    return -1;
}
