/*
 * bgnn.h — C-ABI of libbgnn.so, the MI355X (gfx950) kernels behind buck-gnn's
 * GraphSAGE message-passing hot path.
 *
 * The reference (omerkurt-okt/buck-gnn) is pure Python; its hot path calls into
 * third-party PyG / torch_scatter ops. Each entry point below replaces the
 * arithmetic of one of those calls:
 *
 *   bgnn_graph_build / bgnn_heavy_plan  ← the edge_index preprocessing PyG's
 *       propagate() implies for `SAGEConv(x, edge_index)` (flow='source_to_target':
 *       edge_index[0] = source j, edge_index[1] = target i), called at
 *       Models/BuckGNN.py:342,393,434,449,463; edge_index is produced at
 *       Dataset_Preparation/GraphCreate.py:417-422 (both directions, int64).
 *   bgnn_spmm_fwd / bgnn_spmm_bwd  ← SAGEConv's neighbour aggregation
 *       (aggr='add'|'sum'|'mean'|'max', Models/BuckGNN.py:118,130,145,160,175),
 *       global_mean_pool (Models/BuckGNN.py:274) and torch_scatter.scatter_add /
 *       scatter_mean (Models/BuckGNN.py:561,605).
 *   bgnn_sage_fwd_*, bgnn_bn_*, bgnn_sage_bwd_*  ← the fused layer of
 *       Models/BuckGNN.py:430-444: SAGEConv(normalize=True) → BatchNorm1d → ReLU →
 *       skip (0<i<L-1) → Dropout, and its autograd backward.
 *   bgnn_gemm_f32*  ← lin_l / lin_r of SAGEConv (dense fp32 linear, MFMA) and the
 *       node encoder's Linear+ReLU (Models/BuckGNN.py:67-74).
 *   bgnn_store_gather_*  ← the PyG DataLoader collation of TRAIN_FINAL.py:1298-1302
 *       plus the per-step edge_index preprocessing, for a device-resident dataset.
 *
 * Conventions (all functions):
 *   - every pointer is a DEVICE pointer unless named host_*;
 *   - `stream` is a hipStream_t passed as void*; the library never uses the
 *     default stream and never allocates device memory: scratch comes from the
 *     caller through (ws, ws_bytes);
 *   - return 0 on success, otherwise a hipError_t or a BGNN_E* code; the message
 *     is available from bgnn_last_error_string() (per calling thread);
 *   - no C++ exception crosses this boundary.
 */
#ifndef BGNN_H
#define BGNN_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BGNN_ABI_VERSION 13

#define BGNN_OK 0
#define BGNN_E_ARG 1001       /* invalid argument (shape, null pointer, size)    */
#define BGNN_E_WS 1002        /* workspace too small                             */
#define BGNN_E_UNSUPPORTED 1003

/* reduction selector, PyG aggr= names: 'add' == 'sum' */
#define BGNN_REDUCE_SUM 0
#define BGNN_REDUCE_MEAN 1
#define BGNN_REDUCE_MAX 2

int bgnn_abi_version(void);
const char* bgnn_last_error_string(void);

/* Process-wide tuning knobs for A/B measurement (tools/, tests). The defaults are
 * the production choice; results are identical for every setting, only speed
 * changes. Not thread-safe against concurrent launches. */
#define BGNN_TUNE_SEG_KERNEL 1   /* light rows: 0 = auto (row-group kernel where the CSR has a
                                    row-group plan and the reduce is sum/mean, else the XCD
                                    sweep), 1 = blocked, 2 = XCD sweep                       */
#define BGNN_TUNE_SEG_BLOCKS 2   /* sweep grid in blocks (default 1024)                   */
#define BGNN_TUNE_SEG_U 3        /* neighbours per gather batch: 0 = auto (12), 8, 12, 16  */
#define BGNN_TUNE_SEG_NT 4       /* non-temporal hints on stream-once rows (default 1)       */
#define BGNN_TUNE_GEMM_MODE 5    /* GEMM kernel: 0 = f32 MFMA, 2 = f16x3 (default)           */
#define BGNN_TUNE_ROWS_NT 6      /* non-temporal stores in sage_apply / sage_bwd_rows (0/1)   */
#define BGNN_TUNE_GROUP_BLOCKS 7 /* row-group kernel grid in blocks (default 1024)            */
/* (ABI 9 retired knobs 8-12 -- LDS-DMA GEMM staging, the GEMM tail split, 16-row gather
 * batches, early z_r loads, per-XCD column slices: measured, not adopted; profiles/r0[23]_*) */
#define BGNN_TUNE_ROWS_REV 13       /* bit 0: sage_bwd_rows / l2norm_bwd walk each block's rows from
                                    the last one down, so they start on the rows sage_bwd_stats
                                    read last (still in the Infinity Cache); bit 1: sage_apply
                                    sweeps each eighth of the rows from its end, where the
                                    aggregation wrote last; bits 2 / 3: the row-group
                                    aggregation (SAGE / plain epilogue) sweeps each eighth
                                    downward, starting on the rows the producing GEMM wrote
                                    last. Bits 0 and 2 are the only knob settings that change
                                    rounding (the order of the dh bias partials / of the
                                    BatchNorm statistics sums; deterministic either way).
                                    Default 1 (measured: bits 1-3 gain nothing)              */
/* (ABI 12 retired knobs 14 and 15: the round-5 GEMM main-loop variants (ping-pong, line-major
 * staging, B fragments in registers, interleaved schedule, 32x32x16 MFMAs), the round-6 wave-order
 * swap and static priority, and the row-group max aggregation -- all measured slower or equal;
 * profiles/r05_*, profiles/r06_gemm_ab_b.txt) */
#define BGNN_TUNE_GEMM_BDMA 16   /* pre-split f16x3 GEMMs (bgnn_gemm_f32_w) planned on 128 x 256
                                    tiles (the SAGE input gradients): 0 = k_gemm_x6 (B's image
                                    copied into LDS through registers), 2 / 3 = the pipelined
                                    kernel (gemm_h3p.hip: B by LDS-DMA into 3 / 4 slots, the next
                                    slice's fragments read under the current MFMAs). Default 3.
                                    Bit-identical for every setting                           */
/* Heavy-row timing (measurement only): while enabled, every aggregation launch with super-node
 * chunks records a HIP event pair around its chunk + combine kernels. Enabling resets the record.
 * read: which = 0 the forward aggregations (bgnn_sage_fwd, bgnn_spmm_fwd), 1 the transpose
 * aggregations (bgnn_spmm_bwd, bgnn_spmm_bwd_add); total_ms = summed chunk + combine time,
 * count = launches (synchronises). */
int bgnn_heavy_timing(int32_t enable);
int bgnn_heavy_timing_read(int32_t which, float* total_ms, int32_t* count);
/* Current value of a knob (-1 for an unknown knob). */
int32_t bgnn_get_tuning(int32_t knob);
int bgnn_set_tuning(int32_t knob, int32_t value);

/* ------------------------------------------------------------------------
 * Graph structure. A CSR over destination rows plus the split plan for rows
 * whose in-degree exceeds `chunk` (super nodes: VirtualEdgeCreate.py:106-111).
 * Rows with deg > chunk are reduced in chunks of `chunk` edges by separate
 * waves into a partial buffer and combined in chunk order (deterministic).
 * ---------------------------------------------------------------------- */
typedef struct bgnn_csr {
    const int32_t* rowptr;       /* [n_rows + 1]                               */
    const int32_t* col;          /* [nnz]  source row of each entry            */
    const int32_t* heavy_row;    /* [n_heavy] row id of each heavy row         */
    const int32_t* heavy_chunk0; /* [n_heavy + 1] first chunk of each heavy row*/
    const int32_t* chunk_heavy;  /* [n_chunks] heavy index owning each chunk   */
    int64_t n_rows;
    int64_t nnz;
    int32_t n_heavy;
    int32_t n_chunks;
    int32_t chunk;               /* edges per chunk; rows with deg > chunk are heavy */
    int32_t ranges_all;          /* 1: every heavy row is a range row (host-known; chunk launches
                                    skipped when the range path covers them), else 0 */
    /* Optional row-group plan (bgnn_group_plan; all NULL / 0 = none). Used by the sum/mean
     * aggregation kernels: a wave reduces up to `group_rows` consecutive rows and fetches each
     * distinct source row of the group once. */
    const int32_t* gsrc;         /* [nnz]                                      */
    const uint8_t* gmask;        /* [nnz]                                      */
    const int32_t* gcnt;         /* [n_groups]                                 */
    const int32_t* grow;         /* [n_groups + 1] first row of each group; NULL = g * group_rows */
    int64_t n_groups;            /* with grow; else ceil(n_rows / group_rows)  */
    int32_t group_rows;
    int32_t _pad2;
    /* Optional (round 6, ABI 12): the heavy rows' source ranges, bgnn_heavy_ranges' output for
     * this CSR, or NULL. A "range row" is a heavy row whose entries are exactly the contiguous
     * increasing run [a, a + deg) -- the super node of VirtualEdgeCreate.py:106-111 over its
     * graph's real nodes (GraphCreate.py:417-422 emits both directions, so its transposed row is
     * one too). Its aggregation is a column sum over that row range, which bgnn_sage_apply /
     * bgnn_sage_bwd_rows accumulate as a by-product (range partials) and
     * bgnn_range_sums_finish completes; bgnn_sage_fwd / bgnn_spmm_bwd then skip its chunks. */
    const int32_t* ranges;
} bgnn_csr_t;

/* Workspace for bgnn_graph_build (bytes). */
size_t bgnn_graph_build_ws_bytes(int64_t num_edges, int64_t num_nodes);

/* Sort a COO edge_index [2, E] (int64, row 0 = source, row 1 = target) into
 *   forward CSR (rows = targets):   rowptr[N+1], col[E] = sources,
 *   transpose CSR (rows = sources): rowptr_t[N+1], col_t[E] = targets,
 *                                   perm_t[E] = forward-CSR position of the edge.
 * Both sorts are stable, so entries of a row keep edge_index order.
 * `dev_status` (device int32, may be NULL) receives 0, or 1 if an index was outside
 * [0, N). Fully asynchronous: no host synchronisation. */
int bgnn_graph_build(const int64_t* edge_index, int64_t num_edges, int64_t num_nodes,
                     int32_t* rowptr, int32_t* col,
                     int32_t* rowptr_t, int32_t* col_t, int32_t* perm_t,
                     void* ws, size_t ws_bytes, int32_t* dev_status, void* stream);

/* CSR over segments given a sorted-or-unsorted index vector (global_mean_pool's
 * `batch`, torch_scatter's `index`): row r lists the positions i with index[i]==r,
 * in increasing i. Same workspace rule as bgnn_graph_build with E = n. Asynchronous. */
int bgnn_index_csr_build(const int64_t* index, int64_t n, int64_t num_rows,
                         int32_t* rowptr, int32_t* col,
                         void* ws, size_t ws_bytes, int32_t* dev_status, void* stream);

/* Heavy-row plan for a CSR (rows with deg > chunk). Outputs are device arrays
 * sized for the worst case: heavy_row[n_rows], heavy_chunk0[n_rows+1],
 * chunk_heavy[2 * (nnz / chunk) + 2]. dev_counts[0] = n_heavy, [1] = n_chunks
 * (device int32[2]); the caller copies them to the host (one sync for all plans of
 * a batch) before filling bgnn_csr_t. Asynchronous. */
size_t bgnn_heavy_plan_ws_bytes(int64_t n_rows);
int bgnn_heavy_plan(const int32_t* rowptr, int64_t n_rows, int64_t nnz, int32_t chunk,
                    int32_t* heavy_row, int32_t* heavy_chunk0, int32_t* chunk_heavy,
                    int32_t* dev_counts, void* ws, size_t ws_bytes, void* stream);

/* Heavy-row ranges (round 6). ranges = int32 [bgnn_heavy_ranges_bytes(n_heavy) / 4]:
 *   [0] = n_valid, [1] = n_heavy,
 *   [2 + 3k .. 2 + 3k + 2] = (first, end, heavy index) of the k-th range row, k < n_valid, in
 *                            increasing row order: a heavy row whose columns are one increasing
 *                            run is kept when its run starts at or after the end of every earlier
 *                            such row's run (so the kept ranges are sorted and disjoint); the
 *                            others are left to the chunk path,
 *   [2 + 3 n_heavy + h]    = first source row of heavy row h's range, or -1 (chunk path).
 * Asynchronous (two launches); n_heavy is csr->n_heavy. */
size_t bgnn_heavy_ranges_bytes(int32_t n_heavy);
int bgnn_heavy_ranges(const bgnn_csr_t* csr, int32_t* ranges, void* stream);

/* Range partials -> range row sums. bgnn_sage_apply / bgnn_sage_bwd_rows (given a `ranges` buffer)
 * write, per block b of bgnn_rows_slots(n_rows) row blocks (rows [b rpb, (b+1) rpb), rpb =
 * ceil(n_rows / slots)) and for the up to 3 range rows whose ranges meet the block, the column sums
 * of their rows' outputs: range_partial [slots][3][H] (bgnn_range_partial_bytes). The block's
 * ranges are those with end > b rpb, taken in order; the finish sums each range's block partials
 * in block order (deterministic):
 *   mode 0: out[h, :]               = sum (the forward: the range sums of x_next, which the next
 *                                     layer's GEMM turns into the heavy rows' aggregates)
 *   mode 1: out[heavy_row[h], :]    = sum (the backward: a super node's dz_l row)
 * for each range row h of `csr`; mode 0 also zeroes row h of every heavy row left to the chunk path
 * (its GEMM row is computed but unused); amax (optional): *amax = max(*amax, *amax_floor, max |sum|).
 * Requires rpb <= 2 (chunk + 1) (every range spans more than chunk rows). */
size_t bgnn_range_partial_bytes(int64_t n_rows, int32_t H);
int bgnn_range_sums_finish(const float* range_partial, int64_t n_rows, int32_t H, const bgnn_csr_t* csr,
                           int32_t mode, float* out, int64_t ldo, const float* amax_floor, float* amax,
                           void* stream);

/* Row-group plan of a CSR (R = group_rows <= 8, chunk <= 64). Group g = rows
 * [grow[g], grow[g+1]) (at most R rows; grow = NULL: rows [g*R, g*R+R), n_groups =
 * ceil(n_rows / R)). For each group: the light rows' (deg <= chunk) entries, concatenated in
 * row order, keyed by (source, occurrence of that source earlier in the same row) -- a
 * duplicate edge stays two keys -- numbered by first appearance; with r0 = the group's first
 * row, gsrc[rowptr[r0] + k] = source of key k and gmask[rowptr[r0] + k] = bit t set iff row
 * r0+t holds key k, for k < gcnt[g]. Each row's entries then appear in key order (the row's
 * own CSR order for the group's first row). gsrc / gmask have nnz elements (only each group's
 * own CSR range is written), gcnt n_groups. Deterministic, asynchronous, one wave per group. */
int bgnn_group_plan(const int32_t* rowptr, const int32_t* col, int64_t n_rows, int32_t chunk,
                    int32_t group_rows, const int32_t* grow, int64_t n_groups,
                    int32_t* gsrc, uint8_t* gmask, int32_t* gcnt, void* stream);

/* ------------------------------------------------------------------------
 * Generic segment reduce (SpMM with a 0/1 or 1/deg matrix):
 *   out[r, :] = REDUCE_{e in row r} x[col[e], :]
 * H columns, row strides ldx / ldo in elements. For MEAN the sum is divided by
 * max(deg, 1); empty rows give 0 for every reduce (PyG semantics).
 * MAX writes the argmax state (below) when arg != NULL.
 * `partial` is scratch of n_chunks * H floats (+ n_chunks * H int32 for MAX).
 * ---------------------------------------------------------------------- */
int bgnn_spmm_fwd(const bgnn_csr_t* csr, const float* x, int64_t ldx, int32_t H,
                  int32_t reduce, float* out, int64_t ldo, void* arg,
                  float* partial, void* stream);
/* MAX: `arg` (optional; needed for the backward) receives the argmax state, a device buffer of
 * bgnn_spmm_max_arg_bytes(n_rows, H, n_heavy) bytes (round 5, ABI 10; was an int32 [rows, H]
 * array of CSR positions): per (row, column) the argmax edge's offset in the row's edge list as
 * one byte for light rows (deg <= chunk), and for heavy rows (super nodes) a marker byte (255)
 * plus the int32 offset in a per-heavy-row array -- 1 B instead of 4 B per element written by the
 * forward and gathered per edge by the backward. Ties: the first maximising edge in CSR order.
 * Requires csr->chunk in [1, 254] when arg != NULL (BGNN_E_ARG otherwise: a larger chunk would
 * let a light row's offset reach the marker); the library's plans use chunk 64. */
size_t bgnn_spmm_max_arg_bytes(int64_t n_rows, int32_t H, int32_t n_heavy);

/* Backward of bgnn_spmm_fwd through the transpose CSR (rows = sources):
 *   SUM : gx[j] = sum_{q in rowT j} g[col_t[q]]
 *   MEAN: gx[j] = sum_{q in rowT j} g[col_t[q]] / max(deg_fwd(col_t[q]), 1)
 * `fwd_rowptr` is the forward CSR's rowptr (MEAN degrees). Deterministic (gather form, no
 * atomics on gx). amax (optional): *amax = max(*amax, max |gx|), the operand scale of the f16x3
 * GEMMs that consume gx (bgnn_gemm_f32_scaled). MAX takes bgnn_spmm_bwd_max. */
int bgnn_spmm_bwd(const bgnn_csr_t* csr_t, const int32_t* perm_t, const int32_t* fwd_rowptr,
                  const float* g, int64_t ldg, int32_t H, int32_t reduce,
                  float* gx, int64_t ldgx, float* partial, float* amax, int32_t heavy_done, void* stream);
/* heavy_done = 1 (with csr_t->ranges): the range rows' gx rows were already written (and folded
 * into amax) by bgnn_range_sums_finish (mode 1, from bgnn_sage_bwd_rows' range partials), so
 * their chunks and combine are skipped. */
/* bgnn_spmm_bwd with an addend: gx[j] = (A^T g)[j] + addend[j] (addend [rows, H], ld ld_add),
 * added after the reduction, in the same pass. */
int bgnn_spmm_bwd_add(const bgnn_csr_t* csr_t, const int32_t* perm_t, const int32_t* fwd_rowptr,
                      const float* g, int64_t ldg, int32_t H, int32_t reduce,
                      const float* addend, int64_t ld_add, float* gx, int64_t ldgx, float* partial,
                      float* amax, void* stream);
/* MAX backward: gx[j, c] = sum over j's out-edges q (target i = col_t[q]) that are the argmax of
 * (i, c) -- fwd CSR position perm_t[q] == fwd_rowptr[i] + offset in the argmax state `arg` of the
 * forward (fwd_rows = its row count) -- of g[i, c], plus the optional addend (the max-aggregation
 * SAGEConv backward adds the lin_r input gradient dh W_r (+ the skip gradient) this way,
 * bgnn/fused.py). */
int bgnn_spmm_bwd_max(const bgnn_csr_t* csr_t, const int32_t* perm_t, const int32_t* fwd_rowptr,
                      int64_t fwd_rows, const float* g, int64_t ldg, int32_t H, const void* arg,
                      const float* addend, int64_t ld_add, float* gx, int64_t ldgx, float* partial,
                      float* amax, void* stream);

/* ------------------------------------------------------------------------
 * Fused SAGE layer (Models/BuckGNN.py:430-444, transform-first order):
 *   [z_l | z_r] = x · [W_l ; W_r]^T          (bgnn_gemm_f32_planes; two [N, H] planes)
 *   h_i = AGG_{j->i} z_l[j] + z_r[i] + b_l   (SUM or MEAN)
 *   o_i = h_i / max(||h_i||_2, 1e-12)        (SAGEConv normalize=True)
 *   BatchNorm statistics of o (train mode) as per-block partial sums.
 * Outputs: o [N, H], nrm [N] = ||h_i||, bn_partial [n_slots, 2, H] with
 *   n_slots = bgnn_sage_fwd_slots(csr) (light-row blocks of the kernel that will run, plus
 *   one slot per heavy row).
 * ---------------------------------------------------------------------- */
int32_t bgnn_sage_fwd_slots(const bgnn_csr_t* csr);
int bgnn_sage_fwd(const bgnn_csr_t* csr, const float* zl, int64_t ldzl, const float* zr, int64_t ldzr,
                  const float* bias, int32_t H, int32_t reduce, float* o, float* nrm,
                  float* bn_partial, float* partial, const float* heavy_agg, int64_t ld_heavy_agg,
                  void* stream);
/* heavy_agg (optional, with csr->ranges): row h = the summed z_l rows of range row h (the GEMM of
 * the layer's input range sums: (sum_j x_j) W_l^T = sum_j z_l[j]); the range rows' epilogue takes
 * it in place of their chunk sums (MEAN divides by the degree as for every row). */

/* BatchNorm1d finalize (train): sums the partials in fp64, writes
 *   mean[H], invstd[H], scale = gamma*invstd, shift = beta - mean*scale,
 *   running_mean/var updated in place with `momentum` (unbiased var), as
 *   torch.nn.BatchNorm1d does. gamma/beta may be NULL (affine=False -> 1/0).
 * Eval mode: bgnn_bn_eval_coeffs computes scale/shift from running stats. */
int bgnn_bn_finalize(const float* bn_partial, int32_t n_slots, int32_t H, int64_t count,
                     const float* gamma, const float* beta, float eps, float momentum,
                     float* running_mean, float* running_var,
                     float* mean, float* invstd, float* scale, float* shift, void* stream);
int bgnn_bn_eval_coeffs(int32_t H, const float* gamma, const float* beta, float eps,
                        const float* running_mean, const float* running_var,
                        float* scale, float* shift, void* stream);

/* x_next = Dropout_p( ReLU(o*scale + shift) + (skip ? x_prev : 0) ).
 * scale/shift NULL => identity (no BatchNorm, the *_Shared variant).
 * The dropout mask is a counter-based hash of (seed, element index): keep with
 * probability 1-p, scaled by 1/(1-p); p == 0 disables dropout.
 * amax (optional): *amax = max(*amax, max |x_next|) (next layer's GEMM operand scale). */
int bgnn_sage_apply(const float* o, const float* scale, const float* shift,
                    const float* x_prev, int32_t skip, float p, uint64_t seed,
                    int64_t n_rows, int32_t H, float* x_next, float* amax,
                    const int32_t* ranges, float* range_partial, void* stream);
/* ranges (optional, the next layer's forward-CSR bgnn_heavy_ranges buffer): also the range
 * partials of x_next (bgnn_range_partial_bytes; finish with bgnn_range_sums_finish mode 0), by a
 * row-blocked form of the same element-wise pass (the same x_next bits). */

/* Backward pass 1: BatchNorm statistics of the incoming gradient g (= dL/dx_next):
 *   g2 = relu'(o*scale+shift) * dropout'(g);  partial sums of g2 and g2*xhat.
 * g_rows (ABI 13; NULL: g is [n_rows, H]): row r's gradient is row g_rows[r] of g -- the last
 * layer under a mean pool (Models/BuckGNN.py:246-249 global_mean_pool) reads the pooled gradient
 * [graphs, H] / count through the batch vector instead of a materialised [N, H] broadcast. */
int32_t bgnn_rows_slots(int64_t n_rows);
int bgnn_sage_bwd_stats(const float* g, const int64_t* g_rows, const float* o, const float* scale,
                        const float* shift,
                        const float* mean, const float* invstd, float p, uint64_t seed,
                        int64_t n_rows, int32_t H, float* partial2, void* stream);

/* Reduce [n_slots, 2, H] partials (fp64) into out0[H], out1[H] (either may be NULL;
 * accumulate=1 adds into the outputs). The partial buffer is used as scratch and
 * its contents are undefined afterwards (also for bgnn_bn_finalize). */
/* Output-gradient prep of a dense Linear with fused ReLU (LinearFn.backward of the encoder
 * MLP; replaces torch's threshold_backward, g.sum(0) and a max|g| pass, Models/BuckGNN.py:67-74):
 * g_out = y > 0 ? g : 0 (y NULL: no mask; g_out may then be NULL: not written), column partial sums of g_out into
 * partial[bgnn_linear_bwd_prep_slots()][2][C] (first half of each slot; reduce them with
 * bgnn_reduce_partials), max|g_out| folded into *amax (f32 bits, unsigned atomic max; *amax must
 * hold a non-negative value). Row-major [N, C], C = 4 * a power of two <= 1024, 16-B aligned. */
int32_t bgnn_linear_bwd_prep_slots(void);
int bgnn_linear_bwd_prep(const float* g, const float* y, int64_t N, int32_t C, float* g_out,
                         float* partial, float* amax, void* stream);
/* bf16 form (ABI 7; EA_GNN's bf16 edge activations, replaces torch's threshold_backward +
 * sum(g, 0, dtype=float32)): g, y, g_out bf16 [N, C] (C = 8 * a power of two <= 2048, 16-B aligned);
 * g_out = y > 0 ? g : 0 (y NULL: no mask and g_out may be NULL), f32 column sums of g_out into
 * partial[bgnn_linear_bwd_prep_slots()][2][C] (first half of each slot, for bgnn_reduce_partials). */
int bgnn_linear_bwd_prep_bf16(const void* g, const void* y, int64_t N, int32_t C, void* g_out,
                              float* partial, void* stream);
int bgnn_reduce_partials(const float* partial, int32_t n_slots, int32_t H,
                         float* out0, float* out1, int32_t accumulate, void* stream);

/* Backward pass 2 (row-wise): BatchNorm input-gradient, then the L2-normalize
 * backward, giving dh [N, H] (ld = lddh). If skip, writes dropout'(g) into
 * gskip [N, H] (the skip branch's gradient, the initial value of dL/dx_prev).
 * Partial sums go to partial_db [slots, 2, H]: [.][0] = sum of dh rows (for db_l), [.][1] =
 * sum of w_r * dh_r with row weights w_r from w_rowptr (w_mode 1: w_r = rowptr[r+1]-rowptr[r],
 * the in-degree; 2: [in-degree > 0]; 0: no weights, the half is 0). With the forward CSR and
 * the layer's reduce (1 for sum, 2 for mean) that is the column sum of dz_l = A^T dh, the bias
 * gradient of a Linear folded into the layer (fused.sage_layer w_in).
 * sum_g2 / sum_g2xhat are the reduced stats of pass 1 (NULL when BatchNorm is off).
 * amax (optional): *amax = max(*amax, max |dh|). g_rows: as for bgnn_sage_bwd_stats. */
int bgnn_sage_bwd_rows(const float* g, const int64_t* g_rows, const float* o, const float* nrm,
                       const float* scale, const float* shift, const float* gamma,
                       const float* mean, const float* invstd,
                       const float* sum_g2, const float* sum_g2xhat,
                       float p, uint64_t seed, int32_t skip,
                       int64_t n_rows, int32_t H, float* dh, int64_t lddh,
                       float* gskip, float* partial_db, float* amax,
                       const int32_t* w_rowptr, int32_t w_mode, const int32_t* ranges,
                       const int32_t* range_w_rowptr, float* range_partial, void* stream);
/* ranges (optional, the transpose CSR's bgnn_heavy_ranges buffer): also the range partials of
 * w_r dh_r (w_r = 1, or 1 / max(deg, 1) with deg from range_w_rowptr -- the forward rowptr, MEAN's
 * transposed weights), finished with bgnn_range_sums_finish mode 1 into the super nodes' dz_l rows. */

/* The L2-normalize backward of SAGEConv(normalize=True) alone (ABI 5): the per-module
 * SAGEConv of the PyG surface (bgnn.nn.SAGEConv, called by the reference's unchanged
 * Models/BuckGNN.py:434 under the shim), whose output o = h / max(||h||, 1e-12) feeds torch's
 * BatchNorm/ReLU/Dropout. dh = (g - o <o, g>) / ||h|| per row (g * 1e12 where ||h|| < 1e-12),
 * dh row stride lddh; partial_db [bgnn_rows_slots(n_rows)][2][H]: [.][0] = column sums of dh
 * (the lin_l bias gradient; reduce with bgnn_reduce_partials), [.][1] = 0; *amax = max(*amax,
 * max |dh|). nrm is bgnn_sage_fwd's row-norm output. */
int bgnn_l2norm_bwd(const float* g, const float* o, const float* nrm, int64_t n_rows, int32_t H,
                    float* dh, int64_t lddh, float* partial_db, float* amax, void* stream);

/* bf16 storage of EA_GNN's per-edge activations (ABI 5; BASELINE configs[4], bf16):
 * bgnn_gemm_bf16: C = act(alpha op(A) op(B) + beta C + bias) on the bf16-operand GEMM family
 *   (operands rounded to bf16, one MFMA product, f32 accumulation) with `storage` bits 0 / 1 / 2
 *   = A / B / C stored as bf16 (ld in elements of the stored type; a bf16 C needs beta 0 and is
 *   rounded to nearest even). Built: storage 0; ta 0 tb 1 with 1, 3, 4, 5, 7; ta 1 tb 0 with 1, 2, 3.
 *   ta 0 tb 1 with A and B both bf16 (storage 3 / 7), K % 64 == 0, alpha 1, beta 0: the LDS-DMA
 *   bf16 kernel (ABI 6, gemm_b16.hip), bit-identical to the register-staged one.
 * bgnn_gemm_gather_add_bf16: bgnn_gemm_gather_add (C = A B^T, bf16 operands) with storage
 *   0/1/3/4/5/7 (B bf16 = the weight rounded once by the caller; ABI 6 takes B as const void*).
 * bgnn_gemm_b16_variant (ABI 6, measurement): -1 = the bf16-stored NT products on the
 *   register-staged kernel instead; 0 = default (variant 11: one 256x256 tile per workgroup,
 *   whole-line bf16 C stores, a gathered epilogue's row indices staged in LDS); 1-14 = fixed
 *   forms (A/B; 13 = variant 11 reading the gather indices from global memory per row, 14 =
 *   variant 11 loading each 32-row block's first gathered rows before its staging).
 * bgnn_add_dropout_bf16: bgnn_add_dropout over bf16 (same mask; f32 sum, one rounding).
 * bgnn_segment_sum_bf16: out[r] = sum (mean: / max(deg, 1)) of the bf16 rows x[col[p]], p in
 *   [rowptr[r], rowptr[r+1]), in CSR order, f32 result (H % 8 == 0, H <= 512). */
int bgnn_gemm_bf16(int32_t trans_a, int32_t trans_b, int64_t M, int64_t N, int64_t K, float alpha,
                   const void* A, int64_t lda, const void* B, int64_t ldb, float beta, void* C, int64_t ldc,
                   const float* bias, int32_t relu, int32_t storage, void* ws, size_t ws_bytes, void* stream);
int bgnn_gemm_gather_add_bf16(int64_t M, int64_t N, int64_t K, const void* A, int64_t lda, const void* B,
                              int64_t ldb, void* C, int64_t ldc, const float* bias, int32_t relu,
                              const float* add0, const int64_t* idx0, int64_t ld0, const float* add1,
                              const int64_t* idx1, int64_t ld1, int32_t storage, void* ws, size_t ws_bytes,
                              void* stream);
int bgnn_gemm_b16_variant(int32_t variant);
int bgnn_add_dropout_bf16(const void* a, const void* b, int64_t n, float p, uint64_t seed, void* out,
                          void* stream);
/* ABI 8: out = a + drop(b) over bf16 (n a multiple of 8, 16-B aligned; out may alias a): b masked
 * with bgnn_add_dropout_bf16's mask for (p, seed) -- EA_GNN's edge-activation gradient that sums
 * an edge Linear's input gradient (a) and the skip + dropout's gradient (b) in one pass. */
int bgnn_add_dropped_bf16(const void* a, const void* b, int64_t n, float p, uint64_t seed, void* out,
                          void* stream);
/* ABI 11: C = round(round(A B^T) + drop(src)), A [M, K], B [N, K], C and src [M, N] all bf16,
 * ldc == ld_src == N -- bgnn_gemm_bf16 (storage 7) followed by bgnn_add_dropped_bf16(C, src) bit for
 * bit, the add done in the LDS-DMA kernel's epilogue (EA_GNN's edge Linear dgrad + the skip +
 * dropout's gradient of the same activation). Needs K % 64 == 0, lda / ldb % 8 == 0, 16-B aligned
 * operands; the forms without that epilogue run the two steps. */
int bgnn_gemm_bf16_dropadd(int64_t M, int64_t N, int64_t K, const void* A, int64_t lda, const void* B,
                           int64_t ldb, void* C, int64_t ldc, const void* src, int64_t ld_src, float p,
                           uint64_t seed, void* stream);
int bgnn_segment_sum_bf16(const int32_t* rowptr, const int32_t* col, int64_t n_rows, const void* x,
                          int64_t ldx, int32_t H, int32_t mean, float* out, int64_t ldo, void* stream);
/* Backward of bgnn_segment_sum_bf16 (ABI 10): every position p of segment r (the CSR's col lists
 * the positions of each segment) gets bf16(g[r] / max(deg, 1) for mean, else g[r]) -- f32 division,
 * one round-to-nearest-even -- in one pass (torch: a divide, a bf16 cast and an index_select). */
int bgnn_segment_bcast_bf16(const int32_t* rowptr, const int32_t* col, int64_t n_rows, const float* g, int64_t ldg,
                            int32_t H, int32_t mean, void* out, int64_t ldo, void* stream);

/* ------------------------------------------------------------------------
 * fp32 GEMM (f32 operands, f32 result, f32 accumulation):
 *   C[M,N] = alpha * op(A)[M,K] · op(B)[K,N] + beta * C
 * Two kernel families (BGNN_TUNE_GEMM_MODE):
 *   2 (default) f16x3: each operand is scaled by a power of two from its max |value| and
 *     split into two f16 pieces; three f16 MFMAs per product (a0b0 + a0b1 + a1b0), f32
 *     accumulation, exact unscale (dropped terms <= ~2^-21 |a||b|; measured error vs fp64 at
 *     or below the f32 MFMA's). Needs the workspace of bgnn_gemm_ws_bytes() (the operand
 *     maxima live there unless the caller passes them to bgnn_gemm_f32_scaled).
 *   0 the f32 MFMA (v_mfma_f32_32x32x2_f32, exact fp32 FMA chain).
 * trans_a = 0: A is [M,K] row-major (lda >= K); 1: A is [K,M] row-major (lda >= M).
 * trans_b = 0: B is [K,N] row-major (ldb >= N);  1: B is [N,K] row-major (ldb >= K).
 * C is [M,N] row-major (ldc >= N). `ws` is scratch for split-K (may be NULL when
 * bgnn_gemm_ws_bytes() returns 0 for the shape).
 * ---------------------------------------------------------------------- */
size_t bgnn_gemm_ws_bytes(int64_t M, int64_t N, int64_t K, int32_t trans_a, int32_t trans_b);
/* Force a tile configuration (tuning/tests; -1 = automatic, the default; 0..4 = the f16x3 /
 * bf16 tiles 128x128, 256x128, 128x256, 256x256 (2x4 waves), 256x256 (4x2 waves); values the
 * GEMM mode has no tile for are rejected). Results are identical up to the split-K partition;
 * only speed changes. (ABI 12: the timing ablations of 100 * k + cfg, which computed wrong
 * results, are gone from the library.) */
int bgnn_gemm_set_cfg(int32_t cfg);
int bgnn_gemm_f32(int32_t trans_a, int32_t trans_b, int64_t M, int64_t N, int64_t K,
                  float alpha, const float* A, int64_t lda, const float* B, int64_t ldb,
                  float beta, float* C, int64_t ldc, void* ws, size_t ws_bytes, void* stream);
/* Same with a fused epilogue: C = act(alpha*op(A)op(B) + beta*C + bias[col]),
 * act = ReLU when relu != 0 (nn.Linear + ReLU of the node encoder, Models/BuckGNN.py:67-74). */
int bgnn_gemm_f32_ex(int32_t trans_a, int32_t trans_b, int64_t M, int64_t N, int64_t K,
                     float alpha, const float* A, int64_t lda, const float* B, int64_t ldb,
                     float beta, float* C, int64_t ldc, const float* bias, int32_t relu,
                     void* ws, size_t ws_bytes, void* stream);
/* Plane-split operands (the SAGE layer's [z_l | z_r] and [dz_l | dh] kept as two
 * contiguous [N, H] planes): A's contiguous dimension (K when trans_a = 0, M when
 * trans_a = 1) is cut into blocks of a_blk elements stored a_pstride elements apart
 * (element index x -> (x / a_blk) * a_pstride + x % a_blk); C's N dimension likewise with
 * c_blk / c_pstride. 0 = dense. Blocks must be multiples of the kernel's tile. */
/* Plane-split GEMM with caller-supplied operand maxima for f16x3 (a_amax = max|A|,
 * b_amax = max|B| as device floats, e.g. from bgnn_absmax_f32 or a producer kernel; the
 * exact max gives full accuracy, a larger value loses precision gradually, a smaller one is
 * undefined). NULL = computed here (one read pass). c_amax (optional, any mode): *c_amax =
 * max(*c_amax, max |C|) over the result (fused into the epilogue when possible), so the
 * result can feed the next GEMM without another pass. precision: 0 = f32-accurate (default
 * family), 1 = bf16 operands with f32 accumulation. */
int bgnn_gemm_f32_scaled(int32_t trans_a, int32_t trans_b, int64_t M, int64_t N, int64_t K,
                         float alpha, const float* A, int64_t lda, int64_t a_blk, int64_t a_pstride,
                         const float* B, int64_t ldb, float beta, float* C, int64_t ldc,
                         int64_t c_blk, int64_t c_pstride, const float* bias, int32_t relu,
                         const float* a_amax, const float* b_amax, float* c_amax,
                         int32_t precision, void* ws, size_t ws_bytes, void* stream);
/* Workspace of bgnn_gemm_f32_scaled for a given precision (0 = f32-accurate, the family of
 * BGNN_TUNE_GEMM_MODE; 1 = bf16 operands rounded to nearest, one MFMA product, f32
 * accumulation and output: the bf16 EA_GNN path of BASELINE configs[4]). */
/* C = A' B' + drop(src): the dgrad of a SAGE skip layer (Models/BuckGNN.py:441-444) with the
 * skip gradient drop(g) recomputed from the layer's counter-based dropout mask (seed, p; the
 * mask bgnn_sage_apply / bgnn_sage_bwd_rows use, element (r, c) of src [M, ld_src]) in the
 * GEMM epilogue, instead of being written by bgnn_sage_bwd_rows and read back as C. f16x3 mode
 * (BGNN_TUNE_GEMM_MODE 2) and trans_a = 0, trans_b = 1 only; N and ld_src multiples of 4, src
 * 16-byte aligned. */
int bgnn_gemm_f32_dropadd(int32_t trans_a, int32_t trans_b, int64_t M, int64_t N, int64_t K,
                          const float* A, int64_t lda, const float* B, int64_t ldb, float* C, int64_t ldc,
                          const float* a_amax, const float* b_amax, const float* src, int64_t ld_src,
                          float p, uint64_t seed, void* ws, size_t ws_bytes, void* stream);
/* bgnn_gemm_f32_dropadd (trans_a = 0, trans_b = 1) whose masked addend covers only the columns
 * [src_col0, N) of C -- column c takes src column c - src_col0, with the mask index of that src
 * element -- and the columns left of src_col0 are a plain product: the max aggregation layer's
 * merged input gradient [dh W_l | dh W_r + drop(g)] in one launch (round 5, ABI 10). src_col0 must
 * be a multiple of the planned column tile (256 for the SAGE shapes). */
int bgnn_gemm_f32_dropadd_cols(int64_t M, int64_t N, int64_t K, const float* A, int64_t lda, const float* B,
                               int64_t ldb, float* C, int64_t ldc, const float* a_amax, const float* b_amax,
                               const float* src, int64_t ld_src, int64_t src_col0, float p, uint64_t seed, void* ws,
                               size_t ws_bytes, void* stream);
/* Pre-split weights (round 5). The f16x3 GEMM C = A W^T of the SAGE layers (forward z = x
 * [W_l;W_r]^T, input gradient dx = dz [W_l;W_r]) takes its weight operand W [N, K] as a
 * pre-split image: W scaled by the power of two of max|W| (amax) and split into two f16 pieces
 * once per step (bgnn_gemm_wsplit, n_items matrices of one shape in one launch: W_i at W + i *
 * item_stride, max|W_i| at amax[i * amax_stride], image i at img + i * img_stride bytes), stored
 * per (column tile of bn rows, 32-deep K slice) as the GEMM's own LDS image, so the GEMM copies
 * it into LDS (16-B register copies) instead of loading, splitting and storing it in every row
 * tile. The
 * product is bit-identical to bgnn_gemm_f32_scaled / bgnn_gemm_f32_dropadd on the same operands.
 *   bgnn_gemm_w_tile(M, N, K): the column tile bn the image must use for that GEMM shape, or 0
 *     when the shape has no pre-split path (then use bgnn_gemm_f32_scaled);
 *   bgnn_gemm_wsplit_bytes(N, K): bytes of one image (N % bn == 0, K % 32 == 0);
 *   bgnn_gemm_f32_w: C = A W^T (+ bias, ReLU, max|C| into c_amax) or, with src != NULL, the
 *     drop-add epilogue of bgnn_gemm_f32_dropadd (C = A W^T + drop(src)); a_amax / b_amax are
 *     max|A| and the max|W| the image was split with. */
int32_t bgnn_gemm_w_tile(int64_t M, int64_t N, int64_t K);
size_t bgnn_gemm_wsplit_bytes(int64_t N, int64_t K);
int bgnn_gemm_wsplit(const float* W, int32_t n_items, int64_t item_stride, int64_t N, int64_t K, int64_t ldw,
                     const float* amax, int64_t amax_stride, void* img, int64_t img_stride, int32_t bn,
                     void* stream);
int bgnn_gemm_f32_w(int64_t M, int64_t N, int64_t K, const float* A, int64_t lda, const void* wimg, int32_t bn,
                    float* C, int64_t ldc, const float* bias, int32_t relu, const float* a_amax,
                    const float* b_amax, float* c_amax, const float* src, int64_t ld_src, float p, uint64_t seed,
                    void* stream);
size_t bgnn_gemm_ws_bytes_ex(int64_t M, int64_t N, int64_t K, int32_t trans_a, int32_t trans_b,
                             int32_t precision);
/* C = act(op(A) op(B) + bias + add0[idx0[r], :] (+ add1[idx1[r], :])) -- gathered row adds
 * in the GEMM epilogue, no split-K (EA_GNN's edge Linears with their node-level blocks,
 * Models/BuckGNN.py:553-560 via bgnn/ea.py). idx* are int64 row indices into add* (ld*).
 * precision: 0 = f32-accurate split family, 1 = bf16 operands. ws: bgnn_gemm_ws_bytes_ex(). */
int bgnn_gemm_gather_add(int32_t trans_a, int32_t trans_b, int64_t M, int64_t N, int64_t K,
                         const float* A, int64_t lda, const float* B, int64_t ldb, float* C, int64_t ldc,
                         const float* bias, int32_t relu, const float* add0, const int64_t* idx0, int64_t ld0,
                         const float* add1, const int64_t* idx1, int64_t ld1, int32_t precision,
                         void* ws, size_t ws_bytes, void* stream);
/* *out = max(accumulate ? *out : 0, max |x|) over a row-major [rows, cols] matrix (ld). */
int bgnn_absmax_f32(const float* x, int64_t rows, int64_t cols, int64_t ld, float* out,
                    int32_t accumulate, void* stream);
/* ABI 7: out[i * out_stride] = max(out[i * out_stride], max |x_i|) for n_items matrices of equal
 * shape [rows, cols] (ld), item i at x + i * item_stride (cols, ld, item_stride multiples of 4,
 * x 16-B aligned), in one launch (the per-layer weight maxima of a SAGE layer loop). */
int bgnn_absmax_items_f32(const float* x, int32_t n_items, int64_t item_stride, int64_t rows, int64_t cols,
                          int64_t ld, float* out, int64_t out_stride, void* stream);
int bgnn_gemm_f32_planes(int32_t trans_a, int32_t trans_b, int64_t M, int64_t N, int64_t K,
                         float alpha, const float* A, int64_t lda, int64_t a_blk, int64_t a_pstride,
                         const float* B, int64_t ldb, float beta, float* C, int64_t ldc,
                         int64_t c_blk, int64_t c_pstride, const float* bias, int32_t relu,
                         void* ws, size_t ws_bytes, void* stream);

/* ------------------------------------------------------------------------
 * Device-resident graph store (replaces the host-side PyG
 * DataLoader/Batch collation of TRAIN_FINAL.py:1298-1302 and the per-step graph
 * structure build). Stored arrays are graph-local int32: edge_index [2][ld_ei] (node ids
 * relative to the graph's first node), rowptr / rowptr_t [sum N] (edge offsets relative to
 * the graph's first edge; the row end of a graph's last node is its edge count), col /
 * col_t [sum E] (local node ids), perm_t [sum E] (local forward positions).
 * table: device int64 [B][6] = {src_node, dst_node, n_nodes, src_edge, dst_edge, n_edges}
 * per batch graph (dst offsets = running sums). max_nodes / max_edges bound the per-graph
 * sizes (launch geometry only). Outputs are the batch's int64 edge_index [2][Eb], its
 * forward / transpose CSR (rowptr [Nb+1], col [Eb], rowptr_t [Nb+1], col_t [Eb],
 * perm_t [Eb]) and the int64 `batch` vector [Nb] -- identical to bgnn_graph_build on the
 * collated edge_index.
 * ---------------------------------------------------------------------- */
int bgnn_store_gather_graph(const int64_t* table, int32_t B, int64_t Nb, int64_t Eb,
                            int64_t max_nodes, int64_t max_edges,
                            const int32_t* edge_index, int64_t ld_ei,
                            const int32_t* rowptr, const int32_t* col,
                            const int32_t* rowptr_t, const int32_t* col_t, const int32_t* perm_t,
                            int64_t* edge_index_out, int32_t* rowptr_out, int32_t* col_out,
                            int32_t* rowptr_t_out, int32_t* col_t_out, int32_t* perm_t_out,
                            int64_t* batch_out, void* stream);
/* Row-group plans of the batch from per-graph plans (groups aligned to graph starts, built
 * once by bgnn_group_plan with grow): gtable device int64 [B][7] = {dst_node, src_edge,
 * dst_edge, n_edges, src_group, dst_group, n_groups} per batch graph. Copies gsrc (+dst_node),
 * gmask over each graph's edge range and gcnt over its groups, for the forward and the
 * transpose CSR, and writes the batch's grow[G+1] (graph b's group k starts at
 * dst_node + k * group_rows; grow[G] = Nb). */
int bgnn_store_gather_groups(const int64_t* gtable, int32_t B, int32_t group_rows, int64_t Nb, int64_t Gb,
                             int64_t max_edges, int64_t max_groups,
                             const int32_t* gsrc, const uint8_t* gmask, const int32_t* gcnt,
                             const int32_t* gsrc_t, const uint8_t* gmask_t, const int32_t* gcnt_t,
                             int32_t* gsrc_out, uint8_t* gmask_out, int32_t* gcnt_out,
                             int32_t* gsrc_t_out, uint8_t* gmask_t_out, int32_t* gcnt_t_out,
                             int32_t* grow_out, void* stream);
/* Copy each batch graph's node rows (per_edge = 0) or edge rows (per_edge = 1) of a
 * row-major store array (row_bytes per row, a multiple of 4) into the batch array. */
int bgnn_store_gather_rows(const int64_t* table, int32_t B, int32_t per_edge, int64_t max_rows,
                           const void* src, int64_t row_bytes, void* dst, void* stream);

/* ------------------------------------------------------------------------
 * SAGPooling (torch_geometric.nn.SAGPooling as the reference builds it for GraphSAGE_SAG /
 * EAGNN_SAG, Models/BuckGNN.py:203-208,231-236, called at :364,502): PyG's
 * topk(score, ratio, batch) -> x[perm] * score[perm] -> filter_adj(edge_index, perm).
 * `batch` must be non-decreasing (every PyG Batch is); ptr [B+1] = its graph offsets.
 *
 * bgnn_topk_rank: rank[i] = position of node i in its graph's descending score order,
 *   #{j in graph(i) : s_j > s_i or (s_j == s_i and j < i)} (a stable descending sort;
 *   O(n_g^2) compares per graph, staged through LDS).
 * bgnn_topk_select: node i is kept iff rank[i] < k[g] (k[g] = ceil(ratio * n_g), computed by
 *   the caller in fp32 as PyG does); perm[new_ptr[g] + rank[i]] = i, new_id[i] = that position
 *   or -1, batch_out[position] = g (optional). new_ptr [B+1] = running sums of k.
 * bgnn_gather_scale: out[p] = x[perm[p]] * score[perm[p]] ([k, H] rows).
 * bgnn_gather_scale_bwd: over all n input rows: dx[i] = g[new_id[i]] * score[i] and
 *   dscore[i] = <g[new_id[i]], x[i]> (zeros for rows that were not kept; dscore optional).
 * bgnn_filter_edges: the edges whose two ends are kept, in edge_index order, relabelled by
 *   new_id: out_edges[0 .. 2*n_kept) = [src' | dst'] (capacity 2 * num_edges), kept[pos] =
 *   original edge position (optional, for edge_attr), *n_kept (device int64).
 *   Deterministic (no atomics); edges with an end outside [0, num_nodes) are dropped.
 * ---------------------------------------------------------------------- */
int bgnn_topk_rank(const float* score, const int64_t* batch, const int64_t* ptr, int64_t n,
                   int32_t* rank, void* stream);
int bgnn_topk_select(const int32_t* rank, const int64_t* batch, const int64_t* k, const int64_t* new_ptr,
                     int64_t n, int64_t* perm, int32_t* new_id, int64_t* batch_out, void* stream);
int bgnn_gather_scale(const float* x, int64_t ldx, int32_t H, const int64_t* perm, const float* score,
                      int64_t k, float* out, int64_t ldo, void* stream);
int bgnn_gather_scale_bwd(const float* g, int64_t ldg, const float* x, int64_t ldx, int32_t H,
                          const int32_t* new_id, const float* score, int64_t n, float* dx, int64_t lddx,
                          float* dscore, void* stream);
size_t bgnn_filter_edges_ws_bytes(int64_t num_edges);
int bgnn_filter_edges(const int64_t* edge_index, int64_t num_edges, const int32_t* new_id,
                      int64_t num_nodes, int64_t* out_edges, int64_t* kept, int64_t* n_kept,
                      void* ws, size_t ws_bytes, void* stream);

/* ------------------------------------------------------------------------
 * Node-encoder head (Models/BuckGNN.py:67-74, h >= 256): h = ReLU(ReLU(x W1^T + b1) W2^T + b2)
 * for x [N, F] (F = 16), W1 [D1, F] (D1 = 64), W2 [D2, D1] (D2 = 128), row-major fp32, on the
 * VALU with both weights in LDS (the encoder's last Linear is folded into the first SAGE layer).
 * bgnn_mlp2_fwd folds max|h| into *h_amax (f32 bits, atomic max; NULL = off).
 * bgnn_mlp2_bwd: given dh = dL/dh, the weight / bias gradients of both layers (written, not
 * accumulated), deterministic (per-workgroup partials summed in order); x gets no gradient.
 * bgnn_mlp2_supported: whether (F, D1, D2) is built (only 16 x 64 x 128).
 * ---------------------------------------------------------------------- */
int bgnn_mlp2_supported(int32_t F, int32_t D1, int32_t D2);
int bgnn_mlp2_fwd(const float* x, int64_t N, int32_t F, int32_t D1, int32_t D2, const float* W1,
                  const float* b1, const float* W2, const float* b2, float* h, float* h_amax, void* stream);
size_t bgnn_mlp2_bwd_ws_bytes(int64_t N);
int bgnn_mlp2_bwd(const float* x, int64_t N, int32_t F, int32_t D1, int32_t D2, const float* W1,
                  const float* b1, const float* W2, const float* h, const float* dh, float* dW1,
                  float* db1, float* dW2, float* db2, void* ws, size_t ws_bytes, void* stream);

/* ------------------------------------------------------------------------
 * Skip + dropout of the EA_GNN layer loop (Models/BuckGNN.py:382-387): out = drop(a + b) over
 * n floats (b optional: plain dropout; also the backward, drop(g)), with the counter-based
 * mask of the fused SAGE layers (keep_bits4(seed, i / 4), kept values scaled by 1 / (1 - p)).
 * n a multiple of 4, pointers 16-byte aligned; out may alias a.
 * ---------------------------------------------------------------------- */
int bgnn_add_dropout(const float* a, const float* b, int64_t n, float p, uint64_t seed, float* out,
                     void* stream);

/* ------------------------------------------------------------------------
 * ABI 9: BatchNorm1d over a row-major [n_rows, C] fp32 activation (torch.nn.BatchNorm1d, the
 * modules the reference builds after each SAGEConv, Models/BuckGNN.py:133,148,163,179; used by
 * bgnn.nn.BatchNorm1d on the per-module path). C % 4 == 0 with C / 4 a power of two <= 256;
 * 16-byte aligned pointers.
 *   bgnn_bn_stats:     per-block partials [bgnn_bn_slots(n_rows, C), 2, C] of the SHIFTED sums
 *                      sum (x - k), sum (x - k)^2 with k = x's first row (round 5), finished by
 *                      bgnn_bn_finalize_shifted with kshift = x (NOT bgnn_bn_finalize, which
 *                      takes unshifted sums: it would return a mean off by the first row)
 *   bgnn_bn_apply:     y = x * scale + shift
 *   bgnn_bn_bwd_stats: partials of sum g, sum g * (x - mean) * invstd (finished by
 *                      bgnn_reduce_partials into sums[2, C] = dbeta, dgamma)
 *   bgnn_bn_bwd_dx:    train-mode input gradient gamma invstd / N (N g - sums[0] - xhat sums[1])
 *                      (gamma may be NULL: affine=False)
 * ---------------------------------------------------------------------- */
int32_t bgnn_bn_slots(int64_t n_rows, int32_t C);
int bgnn_bn_stats(const float* x, int64_t n_rows, int32_t C, float* partial, void* stream);
/* BatchNorm finalize of bgnn_bn_stats' shifted partials (sums of x - k and (x - k)^2 with k =
 * kshift = the input's first row, which bgnn_bn_stats uses): as bgnn_bn_finalize, mean = k + the
 * shifted mean (round-4 ADVICE: no E[x^2] - E[x]^2 cancellation when |mean| >> std). */
int bgnn_bn_finalize_shifted(const float* bn_partial, int32_t n_slots, int32_t H, int64_t count,
                             const float* kshift, const float* gamma, const float* beta, float eps, float momentum,
                             float* running_mean, float* running_var, float* mean, float* invstd, float* scale,
                             float* shift, void* stream);
int bgnn_bn_apply(const float* x, int64_t n_rows, int32_t C, const float* scale, const float* shift, float* y,
                  void* stream);
int bgnn_bn_bwd_stats(const float* g, const float* x, const float* mean, const float* invstd, int64_t n_rows,
                      int32_t C, float* partial, void* stream);
int bgnn_bn_bwd_dx(const float* g, const float* x, const float* mean, const float* invstd, const float* gamma,
                   const float* sums, int64_t n_rows, int32_t C, float* dx, void* stream);

/* ABI 8: RelativeErrorLoss on denormalised values (Utils/Losses.py:755-761 applied to
 * Normalizer.py:203-215's value * scale + center, TRAIN_FINAL.py:267-270): *loss =
 * mean(|p' - t'| / (|t'| + eps)) with p' = pred * scale + center, t' = y * scale + center over n
 * values (f32, device), and (dpred != NULL) dpred[i] = d loss / d pred[i]
 * = sign(p'_i - t'_i) * scale / ((|t'_i| + eps) * n). One launch, deterministic. */
int bgnn_rel_error_loss(const float* pred, const float* y, int64_t n, float scale, float center, float eps,
                        float* loss, float* dpred, void* stream);

/* ABI 8: small-batch Linear layers (the decoder MLP on the pooled [B = graphs, H] features,
 * Models/BuckGNN.py:94-100): y[B, N] = act(x[B, K] W[N, K]^T + bias) (act = ReLU if relu; bias may
 * be NULL); backward with g = gy masked by y > 0 when y != NULL (the layer's ReLU output):
 * dW = g^T x, db = column sums of g (NULL: skipped), dx = g W (NULL: skipped). K % 4 == 0, x / W /
 * dW / dx 16-B aligned; one wave or thread per output, fixed reduction order (deterministic).
 * Meant for B up to a few hundred rows. */
int bgnn_small_linear_fwd(const float* x, int64_t B, int32_t K, const float* W, const float* bias, int32_t N,
                          int32_t relu, float* y, void* stream);
int bgnn_small_linear_bwd(const float* gy, const float* y, const float* x, int64_t B, int32_t K, const float* W,
                          int32_t N, float* dx, float* dW, float* db, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* BGNN_H */
