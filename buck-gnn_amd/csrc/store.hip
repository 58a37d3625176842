// Device-resident graph store: mini-batch assembly on the GPU.
//
// The reference collates every mini-batch on the host (PyG DataLoader/Batch,
// TRAIN_FINAL.py:1298-1302, 253-255) and re-derives the graph structure per step. Here all
// graphs of a dataset stay in HBM (288 GB holds the 80,000-mesh cfg4 set) together with their
// CSR / transpose CSR, built ONCE with bgnn_graph_build. Each stored array is graph-local
// (node ids relative to the graph's first node, edge positions relative to its first edge),
// so a batch is a set of contiguous slices that only need their offsets rebased:
//   table[b] = {src_node, dst_node, n_nodes, src_edge, dst_edge, n_edges}
// Because the CSR sort is stable and graphs occupy disjoint contiguous node ranges, the
// rebased slices are exactly the CSR bgnn_graph_build would produce for the collated batch
// (tests/test_gpu_store.py checks this bit for bit).
#include "common.h"

namespace bgnn {
namespace {

struct Seg {
    int64_t sn, dn, nn, se, de, ne;
};

__device__ __forceinline__ Seg load_seg(const int64_t* __restrict__ table, int b) {
    const int64_t* t = table + 6 * (int64_t)b;
    return Seg{t[0], t[1], t[2], t[3], t[4], t[5]};
}

// grid (x, B): blockIdx.y = graph of the batch
__global__ __launch_bounds__(256) void k_store_graph(const int64_t* __restrict__ table, int B, int64_t Nb, int64_t Eb,
                                                     const int32_t* __restrict__ ei, int64_t ld_ei,
                                                     const int32_t* __restrict__ rowptr,
                                                     const int32_t* __restrict__ col,
                                                     const int32_t* __restrict__ rowptr_t,
                                                     const int32_t* __restrict__ col_t,
                                                     const int32_t* __restrict__ perm_t, int64_t* __restrict__ ei_out,
                                                     int32_t* __restrict__ rowptr_out, int32_t* __restrict__ col_out,
                                                     int32_t* __restrict__ rowptr_t_out,
                                                     int32_t* __restrict__ col_t_out, int32_t* __restrict__ perm_t_out,
                                                     int64_t* __restrict__ batch_out) {
    const int b = blockIdx.y;
    const Seg s = load_seg(table, b);
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (int64_t i = t0; i < s.nn; i += stride) {
        rowptr_out[s.dn + i] = (int32_t)(rowptr[s.sn + i] + s.de);
        rowptr_t_out[s.dn + i] = (int32_t)(rowptr_t[s.sn + i] + s.de);
        batch_out[s.dn + i] = b;
    }
    if (b == B - 1 && t0 == 0) {
        rowptr_out[Nb] = (int32_t)Eb;
        rowptr_t_out[Nb] = (int32_t)Eb;
    }
    for (int64_t e = t0; e < s.ne; e += stride) {
        col_out[s.de + e] = (int32_t)(col[s.se + e] + s.dn);
        col_t_out[s.de + e] = (int32_t)(col_t[s.se + e] + s.dn);
        perm_t_out[s.de + e] = (int32_t)(perm_t[s.se + e] + s.de);
        ei_out[s.de + e] = ei[s.se + e] + s.dn;
        ei_out[Eb + s.de + e] = ei[ld_ei + s.se + e] + s.dn;
    }
}

// row-group plans: gtable[b] = {dst_node, src_edge, dst_edge, n_edges, src_group, dst_group, n_groups}
__global__ __launch_bounds__(256) void k_store_groups(const int64_t* __restrict__ gtable, int B, int R, int64_t Nb,
                                                      int64_t Gb, const int32_t* __restrict__ gsrc,
                                                      const uint8_t* __restrict__ gmask,
                                                      const int32_t* __restrict__ gcnt,
                                                      const int32_t* __restrict__ gsrc_t,
                                                      const uint8_t* __restrict__ gmask_t,
                                                      const int32_t* __restrict__ gcnt_t, int32_t* __restrict__ gsrc_o,
                                                      uint8_t* __restrict__ gmask_o, int32_t* __restrict__ gcnt_o,
                                                      int32_t* __restrict__ gsrc_t_o, uint8_t* __restrict__ gmask_t_o,
                                                      int32_t* __restrict__ gcnt_t_o, int32_t* __restrict__ grow_o) {
    const int b = blockIdx.y;
    const int64_t* t = gtable + 7 * (int64_t)b;
    const int64_t dn = t[0], se = t[1], de = t[2], ne = t[3], sg = t[4], dg = t[5], ng = t[6];
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    // positions past a group's keys hold unwritten values: rebased too, never read
    for (int64_t e = t0; e < ne; e += stride) {
        gsrc_o[de + e] = (int32_t)((uint32_t)gsrc[se + e] + (uint32_t)dn);
        gsrc_t_o[de + e] = (int32_t)((uint32_t)gsrc_t[se + e] + (uint32_t)dn);
        gmask_o[de + e] = gmask[se + e];
        gmask_t_o[de + e] = gmask_t[se + e];
    }
    for (int64_t k = t0; k < ng; k += stride) {
        gcnt_o[dg + k] = gcnt[sg + k];
        gcnt_t_o[dg + k] = gcnt_t[sg + k];
        grow_o[dg + k] = (int32_t)(dn + k * R);
    }
    if (b == B - 1 && t0 == 0) grow_o[Gb] = (int32_t)Nb;
}

// copy the node (or edge) rows of each graph: a contiguous block per graph
__global__ __launch_bounds__(256) void k_store_rows16(const int64_t* __restrict__ table, int per_edge,
                                                      const uint4* __restrict__ src, int64_t row_vec,
                                                      uint4* __restrict__ dst) {
    const Seg s = load_seg(table, blockIdx.y);
    const int64_t r0 = per_edge ? s.se : s.sn, d0 = per_edge ? s.de : s.dn, n = per_edge ? s.ne : s.nn;
    const int64_t total = n * row_vec;
    const uint4* a = src + r0 * row_vec;
    uint4* o = dst + d0 * row_vec;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x)
        o[i] = a[i];
}

__global__ __launch_bounds__(256) void k_store_rows4(const int64_t* __restrict__ table, int per_edge,
                                                     const uint32_t* __restrict__ src, int64_t row_words,
                                                     uint32_t* __restrict__ dst) {
    const Seg s = load_seg(table, blockIdx.y);
    const int64_t r0 = per_edge ? s.se : s.sn, d0 = per_edge ? s.de : s.dn, n = per_edge ? s.ne : s.nn;
    const int64_t total = n * row_words;
    const uint32_t* a = src + r0 * row_words;
    uint32_t* o = dst + d0 * row_words;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x)
        o[i] = a[i];
}

inline unsigned blocks_for(int64_t work, int B) {
    // ~2048 workgroups in total across the batch
    int64_t per = (2048 + B - 1) / B;
    const int64_t need = (work + 255) / 256;
    if (per > need) per = need;
    return (unsigned)(per < 1 ? 1 : per);
}

}  // namespace
}  // namespace bgnn

using namespace bgnn;

extern "C" int bgnn_store_gather_graph(const int64_t* table, int32_t B, int64_t Nb, int64_t Eb, int64_t max_nodes,
                                       int64_t max_edges, const int32_t* ei, int64_t ld_ei,
                                       const int32_t* rowptr, const int32_t* col, const int32_t* rowptr_t,
                                       const int32_t* col_t, const int32_t* perm_t, int64_t* ei_out,
                                       int32_t* rowptr_out, int32_t* col_out, int32_t* rowptr_t_out,
                                       int32_t* col_t_out, int32_t* perm_t_out, int64_t* batch_out, void* stream) {
    BGNN_REQUIRE(B > 0 && B <= 65535, "store_gather_graph: batch of %d graphs unsupported", B);
    BGNN_REQUIRE(table && rowptr && rowptr_t && rowptr_out && rowptr_t_out && batch_out, "store_gather_graph: null");
    BGNN_REQUIRE(Nb >= 0 && Eb >= 0 && Eb < (int64_t(1) << 31), "store_gather_graph: Eb %lld out of range",
                 (long long)Eb);
    BGNN_REQUIRE(Eb == 0 || (ei && col && col_t && perm_t && ei_out && col_out && col_t_out && perm_t_out),
                 "store_gather_graph: null edge arrays");
    hipStream_t s = as_stream(stream);
    const int64_t work = max_nodes > max_edges ? max_nodes : max_edges;
    hipLaunchKernelGGL(k_store_graph, dim3(blocks_for(work, B), B), dim3(256), 0, s, table, B, Nb, Eb, ei, ld_ei,
                       rowptr, col, rowptr_t, col_t, perm_t, ei_out, rowptr_out, col_out, rowptr_t_out, col_t_out,
                       perm_t_out, batch_out);
    BGNN_CHECK_LAUNCH();
    return BGNN_OK;
}

extern "C" int bgnn_store_gather_groups(const int64_t* gtable, int32_t B, int32_t group_rows, int64_t Nb, int64_t Gb,
                                        int64_t max_edges, int64_t max_groups, const int32_t* gsrc,
                                        const uint8_t* gmask, const int32_t* gcnt, const int32_t* gsrc_t,
                                        const uint8_t* gmask_t, const int32_t* gcnt_t, int32_t* gsrc_out,
                                        uint8_t* gmask_out, int32_t* gcnt_out, int32_t* gsrc_t_out,
                                        uint8_t* gmask_t_out, int32_t* gcnt_t_out, int32_t* grow_out, void* stream) {
    BGNN_REQUIRE(B > 0 && B <= 65535, "store_gather_groups: batch of %d graphs unsupported", B);
    BGNN_REQUIRE(group_rows >= 1 && group_rows <= 8, "store_gather_groups: group_rows must be in [1, 8]");
    BGNN_REQUIRE(gtable && gcnt && gcnt_t && gcnt_out && gcnt_t_out && grow_out, "store_gather_groups: null");
    BGNN_REQUIRE(max_edges == 0 || (gsrc && gmask && gsrc_t && gmask_t && gsrc_out && gmask_out && gsrc_t_out &&
                                    gmask_t_out),
                 "store_gather_groups: null edge arrays");
    const int64_t work = max_edges > max_groups ? max_edges : max_groups;
    hipLaunchKernelGGL(k_store_groups, dim3(blocks_for(work, B), B), dim3(256), 0, as_stream(stream), gtable, B,
                       group_rows, Nb, Gb, gsrc, gmask, gcnt, gsrc_t, gmask_t, gcnt_t, gsrc_out, gmask_out, gcnt_out,
                       gsrc_t_out, gmask_t_out, gcnt_t_out, grow_out);
    BGNN_CHECK_LAUNCH();
    return BGNN_OK;
}

extern "C" int bgnn_store_gather_rows(const int64_t* table, int32_t B, int32_t per_edge, int64_t max_rows,
                                      const void* src, int64_t row_bytes, void* dst, void* stream) {
    BGNN_REQUIRE(B > 0 && B <= 65535, "store_gather_rows: batch of %d graphs unsupported", B);
    BGNN_REQUIRE(row_bytes > 0 && row_bytes % 4 == 0, "store_gather_rows: row_bytes must be a positive multiple of 4");
    BGNN_REQUIRE(src && dst && table, "store_gather_rows: null pointer");
    hipStream_t s = as_stream(stream);
    if (row_bytes % 16 == 0 && aligned16(src) && aligned16(dst)) {
        const int64_t rv = row_bytes / 16;
        hipLaunchKernelGGL(k_store_rows16, dim3(blocks_for(max_rows * rv, B), B), dim3(256), 0, s, table, per_edge,
                           (const uint4*)src, rv, (uint4*)dst);
    } else {
        const int64_t rw = row_bytes / 4;
        hipLaunchKernelGGL(k_store_rows4, dim3(blocks_for(max_rows * rw, B), B), dim3(256), 0, s, table, per_edge,
                           (const uint32_t*)src, rw, (uint32_t*)dst);
    }
    BGNN_CHECK_LAUNCH();
    return BGNN_OK;
}
