// Shared helpers for the libbgnn HIP kernels (gfx950 / CDNA4, wave64).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdarg.h>
#include <string.h>

#include "../../include/bgnn.h"

namespace bgnn {

constexpr int kWave = 64;     // CDNA wavefront width (hard-coded, see guide §1)
constexpr int kNumXcd = 8;    // MI355X: 8 XCDs, each with its own L2

// ---- error reporting (per calling thread; never crosses the ABI as an exception)
void set_error(const char* fmt, ...);
int fail(int code, const char* fmt, ...);

#define BGNN_HIP(expr)                                                              \
    do {                                                                            \
        hipError_t _e = (expr);                                                     \
        if (_e != hipSuccess)                                                       \
            return ::bgnn::fail((int)_e, "%s failed: %s (%s:%d)", #expr,            \
                                hipGetErrorString(_e), __FILE__, __LINE__);         \
    } while (0)

#define BGNN_CHECK_LAUNCH() BGNN_HIP(hipGetLastError())

#define BGNN_REQUIRE(cond, ...)                                                     \
    do {                                                                            \
        if (!(cond)) return ::bgnn::fail(BGNN_E_ARG, __VA_ARGS__);                  \
    } while (0)

static inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }
static inline bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

static inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// Bijective XCD-aware remap of a block index (cdna_hip_programming.md §5, T1):
// blocks b and b+8 share an XCD under round-robin dispatch, so give every group of
// blocks that shares an XCD a contiguous range of logical tiles (L2 locality for
// mesh neighbourhoods). Speed only — correctness never depends on placement.
__device__ __forceinline__ int xcd_remap(int b, int nblk) {
    const int q = nblk / kNumXcd, r = nblk % kNumXcd;
    const int x = b % kNumXcd, i = b / kNumXcd;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + i;
}

// xcd_remap with each XCD's share walked from its last block down
__device__ __forceinline__ int xcd_remap_rev(int b, int nblk) {
    const int q = nblk / kNumXcd, r = nblk % kNumXcd;
    const int x = b % kNumXcd, i = b / kNumXcd;
    const int len = x < r ? q + 1 : q;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + len - 1 - i;
}

// Wave-wide sum over groups of `width` lanes (width a power of two ≤ 64).
__device__ __forceinline__ float group_sum(float v, int width) {
    for (int m = width >> 1; m > 0; m >>= 1) v += __shfl_xor(v, m, kWave);
    return v;
}

// Counter-based dropout hash: 64 random bits for (seed, 4-element group index).
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// keep-mask bits for the 4 elements [4*g, 4*g+4): element k kept iff its 16-bit
// lane of the hash is >= threshold (threshold = round(p * 65536)).
__device__ __forceinline__ uint32_t keep_bits4(uint64_t seed, uint64_t g, uint32_t thr) {
    const uint64_t h = mix64(seed ^ (g * 0xD1B54A32D192ED03ull));
    uint32_t m = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) m |= (((uint32_t)(h >> (16 * k)) & 0xFFFFu) >= thr ? 1u : 0u) << k;
    return m;
}

static inline uint32_t dropout_threshold(float p) {
    if (!(p > 0.f)) return 0u;
    double t = (double)p * 65536.0 + 0.5;
    if (t > 65536.0) t = 65536.0;
    return (uint32_t)t;
}

// GEMM kernel family (gemm.hip): 0 = f32 MFMA, 1 = bf16x6, 2 = f16x3 (f32-accurate split products)
void set_gemm_mode(int mode);
int gemm_mode();
// non-temporal output stores of the row-wise SAGE kernels (sage.hip)
void set_rows_nt(int on);
int rows_nt();
void set_rows_rev(int on);
int rows_rev();

// 16-byte store, non-temporal (streamed once: no write-allocate in L2 / Infinity Cache)
__device__ __forceinline__ void store4(float* p, float a, float b, float c, float d, bool nt) {
    typedef float f32x4_t __attribute__((ext_vector_type(4)));
    const f32x4_t t = {a, b, c, d};
    if (nt) __builtin_nontemporal_store(t, reinterpret_cast<f32x4_t*>(p));
    else *reinterpret_cast<f32x4_t*>(p) = t;
}

}  // namespace bgnn
