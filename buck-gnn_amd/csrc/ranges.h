// Shared pieces of the range-row path (ranges.hip): the row-block partition of the row-wise
// passes (bgnn_rows_slots; their range partials are indexed by it) and the lookup of the range
// rows that meet a block.
#pragma once
#include "common.h"

namespace bgnn {

constexpr int kRowsBlocks = 1024;   // max partial slots for row-blocked reductions (2048: rows 112 -> 121 us, stats 58 -> 61 us)
constexpr int kRangeSlots = 3;      // range rows meeting one row block (its rpb <= 2 (chunk + 1))

inline int64_t rows_grid(int64_t n_rows, int rows_per_block_min, int64_t* rpb) {
    int64_t blocks = (n_rows + rows_per_block_min - 1) / rows_per_block_min;
    if (blocks > kRowsBlocks) blocks = kRowsBlocks;
    if (blocks < 1) blocks = 1;
    *rpb = (n_rows + blocks - 1) / blocks;
    return blocks;
}

// the partition of bgnn_rows_slots (4 rows per block minimum)
inline int64_t rows_slots_of(int64_t n_rows, int64_t* rpb = nullptr) {
    int64_t r = 0;
    const int64_t b = rows_grid(n_rows, 4, &r);
    if (rpb) *rpb = r;
    return b;
}

// first compact range k (of nv, see bgnn_heavy_ranges) with end > row: the ranges are increasing
// and disjoint, so their ends are too
__device__ __forceinline__ int32_t range_lower(const int32_t* __restrict__ ranges, int32_t nv, int64_t row) {
    int32_t lo = 0, hi = nv;
    while (lo < hi) {
        const int32_t mid = (lo + hi) >> 1;
        if (ranges[2 + 3 * mid + 1] > row) hi = mid;
        else lo = mid + 1;
    }
    return lo;
}

// the (up to kRangeSlots) ranges meeting rows [r0, r1): slot s covers rows [b[s], e[s]) (empty
// slots: b = e = 0). Wave-uniform values.
struct BlockRanges {
    int32_t b[kRangeSlots], e[kRangeSlots];
    __device__ __forceinline__ void load(const int32_t* __restrict__ ranges, int64_t r0, int64_t r1) {
        const int32_t nv = ranges[0];
        const int32_t k0 = range_lower(ranges, nv, r0);
#pragma unroll
        for (int s = 0; s < kRangeSlots; ++s) {
            const int32_t k = k0 + s;
            const bool ok = k < nv && ranges[2 + 3 * k] < r1;
            b[s] = ok ? ranges[2 + 3 * k] : 0;
            e[s] = ok ? ranges[2 + 3 * k + 1] : 0;
        }
    }
    // slot of row r, or -1
    __device__ __forceinline__ int slot(int64_t r) const {
        int s = -1;
#pragma unroll
        for (int q = kRangeSlots - 1; q >= 0; --q)
            if (r >= b[q] && r < e[q]) s = q;
        return s;
    }
};

}  // namespace bgnn
