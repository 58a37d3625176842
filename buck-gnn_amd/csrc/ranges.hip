// Range rows (round 6): the super node of a stiffened mesh (VirtualEdgeCreate.py:81-113) is
// wired to every real node of its graph, and GraphCreate.py:417-422 emits both directions, so in
// the forward CSR its row lists sources [a, a + n_g) in increasing order and in the transpose CSR
// its row lists the same targets. Such a heavy row's aggregation is a column sum over a row range:
//   forward    h_s  = sum_{j in [a, e)} z_l[j] = (sum_{j in [a, e)} x_j) W_l^T
//   transpose  dz_s = sum_{i in [a, e)} w_i dh_i        (w_i = 1, or 1 / deg_fwd(i) for MEAN)
// The row passes that produce x (bgnn_sage_apply) and dh (bgnn_sage_bwd_rows) already stream every
// one of those rows, so they accumulate the range sums as per-block partials at no extra HBM pass;
// this file detects the range rows of a CSR (bgnn_heavy_ranges) and finishes the partials
// (bgnn_range_sums_finish). The chunk + combine path (spmm.hip) stays for every other heavy row.
#include "common.h"
#include "ranges.h"

namespace bgnn {

// one block per heavy row: is the row's column list the increasing run col[e0] + t?
__global__ __launch_bounds__(256) void k_heavy_range_check(const int32_t* __restrict__ rowptr,
                                                           const int32_t* __restrict__ col,
                                                           const int32_t* __restrict__ heavy_row, int32_t n_heavy,
                                                           int32_t* __restrict__ first) {
    const int h = blockIdx.x;
    if (h >= n_heavy) return;
    const int32_t r = heavy_row[h];
    const int32_t e0 = rowptr[r], e1 = rowptr[r + 1];
    const int32_t a = col[e0];
    int ok = 1;
    for (int32_t e = e0 + (int32_t)threadIdx.x; e < e1; e += 256) ok &= (col[e] == a + (e - e0)) ? 1 : 0;
    ok = __syncthreads_and(ok);
    if (threadIdx.x == 0) first[h] = ok ? a : -1;
}

// one wave: keep the range rows whose range starts at or after the end of every earlier candidate
// range (heavy rows are in increasing row order; the kept ranges are then increasing and disjoint,
// the others go to the chunk path) and write the compact list. 64 heavy rows per step: a prefix max
// of the candidates' ends and a ballot prefix count, carried across steps.
__global__ __launch_bounds__(64) void k_heavy_range_compact(const int32_t* __restrict__ rowptr,
                                                            const int32_t* __restrict__ heavy_row, int32_t n_heavy,
                                                            int32_t* __restrict__ ranges) {
    const int lane = threadIdx.x;
    int32_t* first = ranges + 2 + 3 * n_heavy;
    int32_t nv = 0, end_carry = INT32_MIN;
    for (int32_t base = 0; base < n_heavy; base += 64) {
        const int32_t h = base + lane;
        int32_t a = -1, e = INT32_MIN;
        if (h < n_heavy) {
            a = first[h];
            if (a >= 0) {
                const int32_t r = heavy_row[h];
                e = a + (rowptr[r + 1] - rowptr[r]);
            }
        }
        int32_t inc = e;   // inclusive prefix max of the candidates' ends
        for (int o = 1; o < 64; o <<= 1) {
            const int32_t t = __shfl_up(inc, o, kWave);
            if (lane >= o) inc = max(inc, t);
        }
        int32_t excl = __shfl_up(inc, 1, kWave);
        excl = max(lane ? excl : INT32_MIN, end_carry);
        const bool keep = a >= 0 && a >= excl;
        const uint64_t kb = __ballot(keep);
        if (keep) {
            const int32_t pos = nv + (int32_t)__popcll(kb & ((1ull << lane) - 1ull));
            ranges[2 + 3 * pos] = a;
            ranges[2 + 3 * pos + 1] = e;
            ranges[2 + 3 * pos + 2] = h;
        } else if (a >= 0) {
            first[h] = -1;
        }
        nv += (int32_t)__popcll(kb);
        end_carry = max(end_carry, __shfl(inc, 63, kWave));
    }
    if (lane == 0) {
        ranges[0] = nv;
        ranges[1] = n_heavy;
    }
}

// range k of `ranges`, columns [64 blockIdx.y, +64) float4s: wave w sums the partials of the
// range's blocks b0 + w, b0 + w + 4, ... in order; the 4 wave sums are added in wave order
// (deterministic). Block b0's slot is k - range_lower(b0 rpb); every later block of the range
// starts inside it, so its slot is 0.
template <bool MODE1>
__global__ __launch_bounds__(256) void k_range_finish(const float* __restrict__ part, int64_t rpb, int32_t H,
                                                      const int32_t* __restrict__ ranges,
                                                      const int32_t* __restrict__ heavy_row, float* __restrict__ out,
                                                      int64_t ldo, const float* __restrict__ amax_floor,
                                                      uint32_t* __restrict__ amax) {
    const int32_t k = blockIdx.x;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int H4 = H / 4;
    const int c4 = (int)blockIdx.y * 64 + lane;
    const int32_t nv = ranges[0];
    if (!MODE1) {   // mode 0: a heavy row left to the chunk path gets a zero row (its GEMM row is unused)
        const int32_t nh = ranges[1];
        if (wave == 0 && c4 < H4 && k < nh && ranges[2 + 3 * nh + k] < 0)
            *reinterpret_cast<float4*>(out + (int64_t)k * ldo + 4 * c4) = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    if (k >= nv) return;
    const int32_t a = ranges[2 + 3 * k], e = ranges[2 + 3 * k + 1], h = ranges[2 + 3 * k + 2];
    const int64_t b0 = a / rpb, b1 = (e - 1) / rpb;
    const int32_t slot0 = k - range_lower(ranges, nv, b0 * rpb);
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    if (c4 < H4) {
#pragma unroll 4
        for (int64_t b = b0 + wave; b <= b1; b += 4) {
            const int32_t slot = b == b0 ? slot0 : 0;
            const float4 p = *reinterpret_cast<const float4*>(part + ((b * kRangeSlots + slot) * H) + 4 * c4);
            s.x += p.x; s.y += p.y; s.z += p.z; s.w += p.w;
        }
    }
    __shared__ float4 red[4][64];
    red[wave][lane] = s;
    __syncthreads();
    uint32_t m = 0;
    if (wave == 0) {
        float4 t = red[0][lane];
#pragma unroll
        for (int w = 1; w < 4; ++w) {
            const float4 u = red[w][lane];
            t.x += u.x; t.y += u.y; t.z += u.z; t.w += u.w;
        }
        if (c4 < H4) {
            float* dst = out + (MODE1 ? (int64_t)heavy_row[h] : (int64_t)h) * ldo;
            *reinterpret_cast<float4*>(dst + 4 * c4) = t;
            m = max(max(__float_as_uint(t.x) & 0x7fffffffu, __float_as_uint(t.y) & 0x7fffffffu),
                    max(__float_as_uint(t.z) & 0x7fffffffu, __float_as_uint(t.w) & 0x7fffffffu));
        }
        if (amax) {
            for (int o = 32; o > 0; o >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, o, kWave));
            if (lane == 0) {
                if (amax_floor) m = max(m, __float_as_uint(*amax_floor) & 0x7fffffffu);
                if (m) atomicMax(amax, m);
            }
        }
    }
}

}  // namespace bgnn

using namespace bgnn;

extern "C" size_t bgnn_heavy_ranges_bytes(int32_t n_heavy) {
    return n_heavy >= 0 ? (size_t)(2 + 4 * (size_t)n_heavy) * 4 : 0;
}

extern "C" int bgnn_heavy_ranges(const bgnn_csr_t* csr, int32_t* ranges, void* stream) {
    BGNN_REQUIRE(csr && csr->rowptr && csr->col && ranges, "heavy_ranges: null argument");
    BGNN_REQUIRE(csr->n_heavy >= 0, "heavy_ranges: plan counts not resolved");
    hipStream_t s = as_stream(stream);
    const int32_t nh = csr->n_heavy;
    if (nh > 0) {
        BGNN_REQUIRE(csr->heavy_row, "heavy_ranges: heavy plan required");
        hipLaunchKernelGGL(k_heavy_range_check, dim3((unsigned)nh), dim3(256), 0, s, csr->rowptr, csr->col,
                           csr->heavy_row, nh, ranges + 2 + 3 * nh);
        BGNN_CHECK_LAUNCH();
    }
    hipLaunchKernelGGL(k_heavy_range_compact, dim3(1), dim3(64), 0, s, csr->rowptr, csr->heavy_row, nh, ranges);
    BGNN_CHECK_LAUNCH();
    return BGNN_OK;
}

extern "C" size_t bgnn_range_partial_bytes(int64_t n_rows, int32_t H) {
    if (n_rows <= 0 || H <= 0) return 0;
    return (size_t)rows_slots_of(n_rows) * kRangeSlots * (size_t)H * 4;
}

extern "C" int bgnn_range_sums_finish(const float* range_partial, int64_t n_rows, int32_t H, const bgnn_csr_t* csr,
                                      int32_t mode, float* out, int64_t ldo, const float* amax_floor, float* amax,
                                      void* stream) {
    BGNN_REQUIRE(range_partial && csr && csr->ranges && out, "range_sums_finish: null argument");
    BGNN_REQUIRE(mode == 0 || mode == 1, "range_sums_finish: mode must be 0 or 1");
    BGNN_REQUIRE(H > 0 && H % 4 == 0 && ldo >= H && ldo % 4 == 0, "range_sums_finish: bad H / ldo");
    BGNN_REQUIRE(((uintptr_t)range_partial & 15) == 0 && ((uintptr_t)out & 15) == 0,
                 "range_sums_finish: 16-byte aligned buffers required");
    BGNN_REQUIRE(mode == 0 || csr->heavy_row, "range_sums_finish: mode 1 needs the heavy plan");
    int64_t rpb = 0;
    rows_slots_of(n_rows, &rpb);
    BGNN_REQUIRE(rpb <= 2 * ((int64_t)csr->chunk + 1),
                 "range_sums_finish: %lld rows per block exceed 2 (chunk + 1)", (long long)rpb);
    if (csr->n_heavy <= 0 || n_rows <= 0) return BGNN_OK;
    hipStream_t s = as_stream(stream);
    const dim3 grid((unsigned)csr->n_heavy, (unsigned)((H / 4 + 63) / 64));
    if (mode == 0)
        hipLaunchKernelGGL(k_range_finish<false>, grid, dim3(256), 0, s, range_partial, rpb, H, csr->ranges,
                           csr->heavy_row, out, ldo, amax_floor, reinterpret_cast<uint32_t*>(amax));
    else
        hipLaunchKernelGGL(k_range_finish<true>, grid, dim3(256), 0, s, range_partial, rpb, H, csr->ranges,
                           csr->heavy_row, out, ldo, amax_floor, reinterpret_cast<uint32_t*>(amax));
    BGNN_CHECK_LAUNCH();
    return BGNN_OK;
}
