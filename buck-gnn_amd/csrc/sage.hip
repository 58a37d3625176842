// Fused element-wise / row-wise pieces of the GraphSAGE layer loop
// (Models/BuckGNN.py:430-444):  BatchNorm1d(train) -> ReLU -> skip -> Dropout,
// and the backward of BatchNorm + the L2 normalize of SAGEConv(normalize=True).
//
// All kernels stream [N, H] fp32 rows with 16-B (float4) accesses. Reductions
// over N (BatchNorm statistics, bias gradient) are per-block partial sums over
// contiguous row ranges, reduced afterwards in fp64 in a fixed order, so results
// do not depend on scheduling.
#include "common.h"
#include "ranges.h"

namespace bgnn {

// ---------------------------------------------------------------------------
// Stage 1 of every partial-slot reduction: [n_slots, 2H] -> kGroups group sums,
// written IN PLACE into the first slot of each group's range (a thread reads its
// whole column range before writing that column, and no other thread touches it).
// Coalesced: a block covers 256 consecutive of the 2H columns for one group.
constexpr int kGroups = 16;

__global__ __launch_bounds__(256) void k_slots_stage1(float* __restrict__ part, int n_slots, int W, int per) {
    const int c = blockIdx.x * 256 + threadIdx.x;
    const int g = blockIdx.y;
    if (c >= W) return;
    const int s0 = g * per, s1 = min(n_slots, s0 + per);
    if (s0 >= s1) return;
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    int s = s0;
    for (; s + 8 <= s1; s += 8) {
#pragma unroll
        for (int u = 0; u < 8; ++u) acc[u] += part[(int64_t)(s + u) * W + c];
    }
    for (; s < s1; ++s) acc[0] += part[(int64_t)s * W + c];
    part[(int64_t)s0 * W + c] = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
}

// Launch stage 1; returns the slot stride the stage-2 kernels must use.
inline int slots_stage1(float* part, int n_slots, int H, hipStream_t s) {
    if (n_slots <= kGroups) return 1;
    const int per = (n_slots + kGroups - 1) / kGroups;
    hipLaunchKernelGGL(k_slots_stage1, dim3((2 * H + 255) / 256, kGroups), dim3(256), 0, s, part, n_slots, 2 * H,
                       per);
    return per;
}

// ---------------------------------------------------------------------------
// Reduce [n_slots, 2, H] partials (slots taken every `stride`); one thread per (channel, slot-phase).
__global__ __launch_bounds__(256) void k_reduce_partials(const float* __restrict__ part, int n_slots, int stride,
                                                         int H, float* __restrict__ out0, float* __restrict__ out1,
                                                         int accumulate) {
    __shared__ double red[4][2][64];
    const int cl = threadIdx.x & 63, ph = threadIdx.x >> 6;
    const int c = blockIdx.x * 64 + cl;
    double s0 = 0.0, s1 = 0.0;
    if (c < H)
        for (int sl = ph * stride; sl < n_slots; sl += 4 * stride) {
            s0 += (double)part[(int64_t)sl * 2 * H + c];
            s1 += (double)part[(int64_t)sl * 2 * H + H + c];
        }
    red[ph][0][cl] = s0;
    red[ph][1][cl] = s1;
    __syncthreads();
    if (ph == 0 && c < H) {
        s0 = (red[0][0][cl] + red[1][0][cl]) + (red[2][0][cl] + red[3][0][cl]);
        s1 = (red[0][1][cl] + red[1][1][cl]) + (red[2][1][cl] + red[3][1][cl]);
        if (out0) out0[c] = accumulate ? out0[c] + (float)s0 : (float)s0;
        if (out1) out1[c] = accumulate ? out1[c] + (float)s1 : (float)s1;
    }
}

// BatchNorm1d finalize (train mode), torch semantics: biased var for
// normalisation, unbiased var for running_var, momentum update.
__global__ __launch_bounds__(256) void k_bn_finalize(const float* __restrict__ part, int n_slots, int stride, int H,
                                                     int64_t count, const float* __restrict__ gamma,
                                                     const float* __restrict__ beta, float eps, float momentum,
                                                     float* __restrict__ rmean, float* __restrict__ rvar,
                                                     float* __restrict__ mean, float* __restrict__ invstd,
                                                     float* __restrict__ scale, float* __restrict__ shift) {
    __shared__ double red[4][2][64];
    const int cl = threadIdx.x & 63, ph = threadIdx.x >> 6;
    const int c = blockIdx.x * 64 + cl;
    double s0 = 0.0, s1 = 0.0;
    if (c < H)
        for (int sl = ph * stride; sl < n_slots; sl += 4 * stride) {
            s0 += (double)part[(int64_t)sl * 2 * H + c];
            s1 += (double)part[(int64_t)sl * 2 * H + H + c];
        }
    red[ph][0][cl] = s0;
    red[ph][1][cl] = s1;
    __syncthreads();
    if (ph == 0 && c < H) {
        s0 = (red[0][0][cl] + red[1][0][cl]) + (red[2][0][cl] + red[3][0][cl]);
        s1 = (red[0][1][cl] + red[1][1][cl]) + (red[2][1][cl] + red[3][1][cl]);
        const double n = (double)count;
        const double mu = s0 / n;
        double var = s1 / n - mu * mu;
        if (var < 0.0) var = 0.0;
        const double is = 1.0 / sqrt(var + (double)eps);
        const float g = gamma ? gamma[c] : 1.f;
        const float b = beta ? beta[c] : 0.f;
        mean[c] = (float)mu;
        invstd[c] = (float)is;
        scale[c] = (float)((double)g * is);
        shift[c] = (float)((double)b - mu * (double)g * is);
        if (rmean && rvar && momentum > 0.f) {
            const double unb = count > 1 ? var * n / (n - 1.0) : var;
            rmean[c] = (float)((1.0 - momentum) * (double)rmean[c] + momentum * mu);
            rvar[c] = (float)((1.0 - momentum) * (double)rvar[c] + momentum * unb);
        }
    }
}

// One-launch reduction of [n_slots, 2, H] partial slots (round 3; replaces k_slots_stage1 + the
// final kernel, one launch fewer per reduction): a block owns 8 channels, its 256 threads are
// 8 channels x 32 slot phases; each thread sums its slots ph, ph + 32, ... of both halves in f64
// (eight loads in flight), then a fixed f64 tree over the 32 phases. MODE 0: out0 / out1 (=, or +=
// with accumulate); MODE 1: the BatchNorm finalize of k_bn_finalize on (sum, sum of squares).
template <int MODE>
__global__ __launch_bounds__(256) void k_reduce_slots(const float* __restrict__ part, int n_slots, int H,
                                                      float* __restrict__ out0, float* __restrict__ out1,
                                                      int accumulate, int64_t count, const float* __restrict__ gamma,
                                                      const float* __restrict__ beta, float eps, float momentum,
                                                      float* __restrict__ rmean, float* __restrict__ rvar,
                                                      float* __restrict__ mean, float* __restrict__ invstd,
                                                      float* __restrict__ scale, float* __restrict__ shift,
                                                      const float* __restrict__ kshift) {
    constexpr int CPB = 8, NPH = 256 / CPB;   // channels per block, slot phases
    __shared__ double red[2][NPH][CPB];
    const int cl = threadIdx.x % CPB, ph = threadIdx.x / CPB;
    const int c = blockIdx.x * CPB + cl;
    const int64_t W = 2 * (int64_t)H;
    double s0 = 0.0, s1 = 0.0;
    if (c < H) {
        int sl = ph;
        for (; sl + 7 * NPH < n_slots; sl += 8 * NPH) {
            float a[8], b[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                a[u] = part[(int64_t)(sl + u * NPH) * W + c];
                b[u] = part[(int64_t)(sl + u * NPH) * W + H + c];
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                s0 += (double)a[u];
                s1 += (double)b[u];
            }
        }
        for (; sl < n_slots; sl += NPH) {
            s0 += (double)part[(int64_t)sl * W + c];
            s1 += (double)part[(int64_t)sl * W + H + c];
        }
    }
    red[0][ph][cl] = s0;
    red[1][ph][cl] = s1;
    __syncthreads();
    for (int o = NPH / 2; o > 0; o >>= 1) {
        if (ph < o) {
            red[0][ph][cl] += red[0][ph + o][cl];
            red[1][ph][cl] += red[1][ph + o][cl];
        }
        __syncthreads();
    }
    if (ph != 0 || c >= H) return;
    s0 = red[0][0][cl];
    s1 = red[1][0][cl];
    if constexpr (MODE == 0) {
        if (out0) out0[c] = accumulate ? out0[c] + (float)s0 : (float)s0;
        if (out1) out1[c] = accumulate ? out1[c] + (float)s1 : (float)s1;
    } else {
        // (kshift: the partials are sums of x - k and (x - k)^2, mean = k + their mean)
        const double n = (double)count;
        const double mu0 = s0 / n;
        double var = s1 / n - mu0 * mu0;
        if (var < 0.0) var = 0.0;
        const double mu = kshift ? (double)kshift[c] + mu0 : mu0;
        const double is = 1.0 / sqrt(var + (double)eps);
        const float g = gamma ? gamma[c] : 1.f;
        const float b = beta ? beta[c] : 0.f;
        mean[c] = (float)mu;
        invstd[c] = (float)is;
        scale[c] = (float)((double)g * is);
        shift[c] = (float)((double)b - mu * (double)g * is);
        if (rmean && rvar && momentum > 0.f) {
            const double unb = count > 1 ? var * n / (n - 1.0) : var;
            rmean[c] = (float)((1.0 - momentum) * (double)rmean[c] + momentum * mu);
            rvar[c] = (float)((1.0 - momentum) * (double)rvar[c] + momentum * unb);
        }
    }
}

// one-launch reductions (k_reduce_slots) instead of stage 1 + final kernel (A/B switch)
static int g_one_pass_reduce = 1;

__global__ void k_bn_eval(int H, const float* __restrict__ gamma, const float* __restrict__ beta, float eps,
                          const float* __restrict__ rmean, const float* __restrict__ rvar,
                          float* __restrict__ scale, float* __restrict__ shift) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= H) return;
    const double is = 1.0 / sqrt((double)rvar[c] + (double)eps);
    const double g = gamma ? gamma[c] : 1.0;
    const double b = beta ? beta[c] : 0.0;
    scale[c] = (float)(g * is);
    shift[c] = (float)(b - (double)rmean[c] * g * is);
}

// ---------------------------------------------------------------------------
// Fold a thread's running max |value| (f32 bits) into *amax: block max over 256 threads,
// then one atomic per block. Must be reached by every thread of the block.
__device__ __forceinline__ void block_amax(uint32_t* amax, uint32_t m) {
    for (int o = 32; o > 0; o >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, o, kWave));
    __shared__ uint32_t red[4];
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        m = max(max(red[0], red[1]), max(red[2], red[3]));
        if (m) atomicMax(amax, m);
    }
}

// x_next = drop(relu(o*scale+shift) + skip*x_prev). Grid-stride over float4s.
__global__ __launch_bounds__(256) void k_sage_apply(const float4* __restrict__ o, const float* __restrict__ scale,
                                                    const float* __restrict__ shift,
                                                    const float4* __restrict__ xprev, int skip, uint32_t thr,
                                                    float inv_keep, uint64_t seed, int64_t n4, int H4,
                                                    float4* __restrict__ xn, uint32_t* __restrict__ amax, int nt,
                                                    int rev) {
    uint32_t m = 0;
    // rev = 1 (grid a multiple of 8): block b sweeps the eighth (b & 7) of the rows from its last
    // element down, so each eighth starts on the rows the aggregation (which sweeps the same
    // eighths upward, one per XCD) wrote last and are still in the Infinity Cache. Element-wise:
    // the result does not depend on the order.
    int64_t lo = 0, hi = n4, i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, st = (int64_t)gridDim.x * blockDim.x;
    if (rev) {
        const int64_t nr = n4 / H4, x = blockIdx.x & 7;
        lo = (nr * x / 8) * H4;
        hi = (nr * (x + 1) / 8) * H4;
        i0 = (int64_t)(blockIdx.x >> 3) * blockDim.x + threadIdx.x;
        st = (int64_t)(gridDim.x >> 3) * blockDim.x;
    }
    for (int64_t q = i0; q < hi - lo; q += st) {
        const int64_t i = rev ? hi - 1 - q : q;
        const int c = (int)(i % H4) * 4;
        float4 v = o[i];
        float y[4] = {v.x, v.y, v.z, v.w};
        if (scale) {
            const float4 sc = *reinterpret_cast<const float4*>(scale + c);
            const float4 sh = *reinterpret_cast<const float4*>(shift + c);
            y[0] = y[0] * sc.x + sh.x; y[1] = y[1] * sc.y + sh.y;
            y[2] = y[2] * sc.z + sh.z; y[3] = y[3] * sc.w + sh.w;
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) y[k] = fmaxf(y[k], 0.f);
        if (skip) {
            const float4 p = xprev[i];
            y[0] += p.x; y[1] += p.y; y[2] += p.z; y[3] += p.w;
        }
        if (thr) {
            const uint32_t keep = keep_bits4(seed, (uint64_t)i, thr);
#pragma unroll
            for (int k = 0; k < 4; ++k) y[k] = ((keep >> k) & 1u) ? y[k] * inv_keep : 0.f;
        }
        store4(reinterpret_cast<float*>(xn + i), y[0], y[1], y[2], y[3], nt);
#pragma unroll
        for (int k = 0; k < 4; ++k) m = max(m, __float_as_uint(y[k]) & 0x7fffffffu);
    }
    if (amax) block_amax(amax, m);
}

// Row-blocked form of k_sage_apply with the range partials of x_next (bgnn_sage_apply given a
// `ranges` buffer; ranges.hip): block lb owns rows [lb rpb, (lb+1) rpb) of the bgnn_rows_slots
// partition, one wave per row (two rows in flight). The element-wise arithmetic, the dropout mask
// index and the store are k_sage_apply's, so x_next has the same bits. Like k_sage_apply's `rev`
// sweep, each XCD takes its share of the row blocks from the last one down and each block its rows
// from the last one down, so the first rows read are the ones the aggregation on that XCD wrote last
// (still in the Infinity Cache). Each wave adds its rows' x_next into its own LDS sum per range
// slot (BlockRanges; the slot is wave-uniform, so no register array is indexed); the 4 waves' sums
// are added in wave order into rpart[lb][slot][H] (every slot written, 0 when unused).
template <int NV>
__global__ __launch_bounds__(256) void k_sage_apply_rows(const float* __restrict__ o, const float* __restrict__ scale,
                                                         const float* __restrict__ shift,
                                                         const float* __restrict__ xprev, int skip, uint32_t thr,
                                                         float inv_keep, uint64_t seed, int64_t n_rows, int H,
                                                         int64_t rpb, float* __restrict__ xn,
                                                         uint32_t* __restrict__ amax, int nt,
                                                         const int32_t* __restrict__ ranges,
                                                         float* __restrict__ rpart) {
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lb = xcd_remap_rev(blockIdx.x, gridDim.x);
    const int64_t r0 = (int64_t)lb * rpb;
    const int64_t r1 = min(n_rows, r0 + rpb);
    const int H4 = H / 4;
    BlockRanges br;
    br.load(ranges, r0, r1);
    __shared__ float4 racc[4][kRangeSlots][128];
    int c4[NV];
    bool cok[NV];
    float4 sc[NV], sh[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        c4[v] = lane + 64 * v;
        cok[v] = c4[v] < H4;
        const int c = cok[v] ? 4 * c4[v] : 0;
        sc[v] = scale ? *reinterpret_cast<const float4*>(scale + c) : make_float4(1.f, 1.f, 1.f, 1.f);
        sh[v] = shift ? *reinterpret_cast<const float4*>(shift + c) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int q = 0; q < kRangeSlots; ++q)
            if (cok[v]) racc[wave][q][c4[v]] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    uint32_t m = 0;
    auto row = [&](int64_t r) {
        const int sl = br.slot(r);
#pragma unroll
        for (int v = 0; v < NV; ++v) {
            if (!cok[v]) continue;
            const int64_t i = r * H4 + c4[v];
            const float4 ov = reinterpret_cast<const float4*>(o)[i];
            float y[4] = {ov.x, ov.y, ov.z, ov.w};
            if (scale) {
                y[0] = y[0] * sc[v].x + sh[v].x; y[1] = y[1] * sc[v].y + sh[v].y;
                y[2] = y[2] * sc[v].z + sh[v].z; y[3] = y[3] * sc[v].w + sh[v].w;
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) y[k] = fmaxf(y[k], 0.f);
            if (skip) {
                const float4 p = reinterpret_cast<const float4*>(xprev)[i];
                y[0] += p.x; y[1] += p.y; y[2] += p.z; y[3] += p.w;
            }
            if (thr) {
                const uint32_t keep = keep_bits4(seed, (uint64_t)i, thr);
#pragma unroll
                for (int k = 0; k < 4; ++k) y[k] = ((keep >> k) & 1u) ? y[k] * inv_keep : 0.f;
            }
            store4(xn + 4 * i, y[0], y[1], y[2], y[3], nt);
#pragma unroll
            for (int k = 0; k < 4; ++k) m = max(m, __float_as_uint(y[k]) & 0x7fffffffu);
            if (sl >= 0) {
                float4 t = racc[wave][sl][c4[v]];
                t.x += y[0]; t.y += y[1]; t.z += y[2]; t.w += y[3];
                racc[wave][sl][c4[v]] = t;
            }
        }
    };
    int64_t r = r1 - 1 - wave;
    for (; r - 4 >= r0; r -= 8) {
        row(r);
        row(r - 4);
    }
    if (r >= r0) row(r);
    if (amax) block_amax(amax, m);
    __syncthreads();
    float4* dst = reinterpret_cast<float4*>(rpart + (int64_t)lb * kRangeSlots * H);
    for (int c = threadIdx.x; c < kRangeSlots * H4; c += 256) {
        const int q = c / H4, cc = c % H4;
        const float4 a0 = racc[0][q][cc], a1 = racc[1][q][cc], a2 = racc[2][q][cc], a3 = racc[3][q][cc];
        dst[c] = make_float4((a0.x + a1.x) + (a2.x + a3.x), (a0.y + a1.y) + (a2.y + a3.y),
                             (a0.z + a1.z) + (a2.z + a3.z), (a0.w + a1.w) + (a2.w + a3.w));
    }
}

// Backward pass 1: partial sums over rows of g2 and g2*xhat per channel.
// Thread layout: H4 = H/4 threads per row, 256/H4 rows per step.
__global__ __launch_bounds__(256) void k_sage_bwd_stats(const float* __restrict__ g,
                                                        const int64_t* __restrict__ g_rows,
                                                        const float* __restrict__ o,
                                                        const float* __restrict__ scale,
                                                        const float* __restrict__ shift,
                                                        const float* __restrict__ mean,
                                                        const float* __restrict__ invstd, uint32_t thr,
                                                        float inv_keep, uint64_t seed, int64_t n_rows, int H,
                                                        int64_t rows_per_block, float* __restrict__ part) {
    __shared__ __attribute__((aligned(16))) float red[2][2][512];
    const int H4 = H / 4;
    const int rpi = 256 / H4;                 // rows per iteration
    const int t = threadIdx.x;
    const int c4 = t % H4, ph = t / H4;
    const int lb = xcd_remap(blockIdx.x, gridDim.x);
    const int64_t r0 = (int64_t)lb * rows_per_block;
    const int64_t r1 = min(n_rows, r0 + rows_per_block);
    float s0[4] = {0, 0, 0, 0}, s1[4] = {0, 0, 0, 0};
    const int c = c4 * 4;
    if (ph < rpi) {
        const float4 sc = *reinterpret_cast<const float4*>(scale + c);
        const float4 sh = *reinterpret_cast<const float4*>(shift + c);
        const float4 mu = *reinterpret_cast<const float4*>(mean + c);
        const float4 is = *reinterpret_cast<const float4*>(invstd + c);
        const float scv[4] = {sc.x, sc.y, sc.z, sc.w}, shv[4] = {sh.x, sh.y, sh.z, sh.w};
        const float muv[4] = {mu.x, mu.y, mu.z, mu.w}, isv[4] = {is.x, is.y, is.z, is.w};
        for (int64_t r = r0 + ph; r < r1; r += rpi) {
            const int64_t i4 = r * H4 + c4;
            const float4 gv = reinterpret_cast<const float4*>(g)[(g_rows ? g_rows[r] : r) * H4 + c4];
            const float4 ov = reinterpret_cast<const float4*>(o)[i4];
            float gg[4] = {gv.x, gv.y, gv.z, gv.w}, oo[4] = {ov.x, ov.y, ov.z, ov.w};
            uint32_t m = 0xF;
            if (thr) m = keep_bits4(seed, (uint64_t)i4, thr);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                float g1 = ((m >> k) & 1u) ? gg[k] * (thr ? inv_keep : 1.f) : 0.f;
                const float yp = oo[k] * scv[k] + shv[k];
                const float g2 = yp > 0.f ? g1 : 0.f;
                const float xh = (oo[k] - muv[k]) * isv[k];
                s0[k] += g2;
                s1[k] += g2 * xh;
            }
        }
    }
    // reduce over row phases (rpi ≤ 2 for H = 512; general rpi via loop)
    __shared__ __attribute__((aligned(16))) float red_all[256][8];
#pragma unroll
    for (int k = 0; k < 4; ++k) { red_all[t][k] = s0[k]; red_all[t][4 + k] = s1[k]; }
    __syncthreads();
    (void)red;
    if (t < H4) {
        float a0[4] = {0, 0, 0, 0}, a1[4] = {0, 0, 0, 0};
        for (int q = 0; q < rpi; ++q)
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                a0[k] += red_all[q * H4 + t][k];
                a1[k] += red_all[q * H4 + t][4 + k];
            }
        float* dst = part + (int64_t)lb * 2 * H;
        *reinterpret_cast<float4*>(dst + c) = make_float4(a0[0], a0[1], a0[2], a0[3]);
        *reinterpret_cast<float4*>(dst + H + c) = make_float4(a1[0], a1[1], a1[2], a1[3]);
    }
}

// Backward pass 2: one wave per row (H <= 512, NV float4 per lane). RELU = false: the layer
// is the bare SAGEConv(normalize=True) of the per-op path (g is dL/do; no ReLU mask, no BN,
// no dropout), i.e. only the L2-normalize backward.
template <int NV, bool RELU = true, bool RANGES = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void k_sage_bwd_rows(
    const float* __restrict__ g, const int64_t* __restrict__ g_rows, const float* __restrict__ o,
    const float* __restrict__ nrm, const float* __restrict__ scale, const float* __restrict__ shift, const float* __restrict__ gamma,
    const float* __restrict__ mean, const float* __restrict__ invstd, const float* __restrict__ sum_g2,
    const float* __restrict__ sum_g2xhat, uint32_t thr, float inv_keep, uint64_t seed, int skip,
    int64_t n_rows, int H, int64_t rows_per_block, float* __restrict__ dh, int64_t lddh,
    float* __restrict__ gskip, float* __restrict__ part, uint32_t* __restrict__ amax, int nt,
    const int32_t* __restrict__ w_rowptr, int w_mode, int rev, const int32_t* __restrict__ ranges,
    const int32_t* __restrict__ rw_rowptr, float* __restrict__ rpart) {
    const int lane = threadIdx.x & 63;
    uint32_t tmax = 0;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lb = xcd_remap(blockIdx.x, gridDim.x);
    const int64_t r0 = (int64_t)lb * rows_per_block;
    const int64_t r1 = min(n_rows, r0 + rows_per_block);
    const int H4 = H / 4;
    const bool bn = (mean != nullptr);
    const float invn = 1.f / (float)(n_rows > 0 ? n_rows : 1);
    int cpos[NV];
    bool cok[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        cpos[v] = (lane + 64 * v) * 4;
        cok[v] = cpos[v] < H;
    }
    // per-channel constants in LDS (read back per row as float4), not VGPRs: 56 registers
    // fewer keep 4 waves per SIMD with two rows in flight per wave.
    // cst[0..6][c] = scale, shift, kA, kB, kC, mean, invstd with
    // do = gamma*invstd/N * (N*g2 - sum_g2 - xhat*sum_g2xhat) = kA g2 - kB - xhat kC
    __shared__ __attribute__((aligned(16))) float cst[7][512];
    for (int c = threadIdx.x; c < H; c += 256) {
        cst[0][c] = scale ? scale[c] : 1.f;
        cst[1][c] = shift ? shift[c] : 0.f;
        if (bn) {
            const float gi = (gamma ? gamma[c] : 1.f) * invstd[c];
            cst[2][c] = gi;
            cst[3][c] = gi * sum_g2[c] * invn;
            cst[4][c] = gi * sum_g2xhat[c] * invn;
            cst[5][c] = mean[c];
            cst[6][c] = invstd[c];
        } else {
            cst[2][c] = 1.f; cst[3][c] = 0.f; cst[4][c] = 0.f; cst[5][c] = 0.f; cst[6][c] = 0.f;
        }
    }
    __syncthreads();
    float db[NV][4], dw[NV][4];   // sums of dh and of w_r * dh (w_mode: row weights from w_rowptr)
#pragma unroll
    for (int v = 0; v < NV; ++v)
#pragma unroll
        for (int k = 0; k < 4; ++k) db[v][k] = dw[v][k] = 0.f;
    // end-of-block reductions; RANGES: first each wave's own sums of rw * dh per range slot
    // (ranges.h; the transposed aggregation of range rows: a super node's dz_l row; rw = 1 or
    // 1 / max(deg_fwd, 1)), kept in LDS rather than registers (the slot is wave-uniform; a register
    // array per slot would cost this kernel a wave per SIMD)
    __shared__ __attribute__((aligned(16))) float red[4][RANGES ? kRangeSlots : 2][512];
    BlockRanges br;
    if constexpr (RANGES) {
        br.load(ranges, r0, r1);
#pragma unroll
        for (int q = 0; q < kRangeSlots; ++q)
#pragma unroll
            for (int v = 0; v < NV; ++v)
                if (cok[v]) *reinterpret_cast<float4*>(&red[wave][q][cpos[v]]) = make_float4(0.f, 0.f, 0.f, 0.f);
    }

    // the next row's g and o rows are loaded one row ahead (two rows in flight per wave: the
    // kernel is latency-bound on these loads, not bandwidth-bound); same rows, same order
    float4 gn[NV], on[NV];
    auto fetch = [&](int64_t rr) {
        const int64_t gr = g_rows ? g_rows[rr] : rr;   // (g_rows: row rr's gradient is row g_rows[rr] of g)
#pragma unroll
        for (int v = 0; v < NV; ++v) {
            const int64_t i4 = rr * H4 + (cok[v] ? (cpos[v] >> 2) : 0);
            gn[v] = reinterpret_cast<const float4*>(g)[gr * H4 + (cok[v] ? (cpos[v] >> 2) : 0)];
            on[v] = reinterpret_cast<const float4*>(o)[i4];
        }
    };
    // rev = 1: the block's rows are walked from its last row down (wave w takes r1-1-w, r1-5-w, ...),
    // so the first rows read are the ones bgnn_sage_bwd_stats read last over the same block ranges
    // and that are still in the Infinity Cache. Only the summation order of the dh partials changes.
    const int64_t nr = r1 - r0 - wave;
    const int64_t cnt = nr > 0 ? (nr + 3) / 4 : 0;
    const int64_t rfirst = rev ? r1 - 1 - wave : r0 + wave;
    const int64_t rstep = rev ? -4 : 4;
    if (cnt > 0) fetch(rfirst);
    for (int64_t j = 0; j < cnt; ++j) {
        const int64_t r = rfirst + j * rstep;
        float ov[NV][4], dov[NV][4], g1v[NV][4];
        float4 gc[NV], oc[NV];
#pragma unroll
        for (int v = 0; v < NV; ++v) { gc[v] = gn[v]; oc[v] = on[v]; }
        if (j + 1 < cnt) fetch(r + rstep);
        float dot = 0.f;
#pragma unroll
        for (int v = 0; v < NV; ++v) {
            if (!cok[v]) {
#pragma unroll
                for (int k = 0; k < 4; ++k) ov[v][k] = dov[v][k] = g1v[v][k] = 0.f;
                continue;
            }
            const int64_t i4 = r * H4 + (cpos[v] >> 2);
            const float4 gv = gc[v];
            const float4 o4 = oc[v];
            const float gg[4] = {gv.x, gv.y, gv.z, gv.w};
            ov[v][0] = o4.x; ov[v][1] = o4.y; ov[v][2] = o4.z; ov[v][3] = o4.w;
            uint32_t m = 0xF;
            if (thr) m = keep_bits4(seed, (uint64_t)i4, thr);
            float cv[7][4];
#pragma unroll
            for (int q = 0; q < 7; ++q) {
                const float4 t4 = *reinterpret_cast<const float4*>(&cst[q][cpos[v]]);
                cv[q][0] = t4.x; cv[q][1] = t4.y; cv[q][2] = t4.z; cv[q][3] = t4.w;
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const float g1 = ((m >> k) & 1u) ? gg[k] * (thr ? inv_keep : 1.f) : 0.f;
                g1v[v][k] = g1;
                const float yp = ov[v][k] * cv[0][k] + cv[1][k];
                const float g2 = (!RELU || yp > 0.f) ? g1 : 0.f;
                float d;
                if (bn) {
                    const float xh = (ov[v][k] - cv[5][k]) * cv[6][k];
                    d = cv[2][k] * g2 - cv[3][k] - xh * cv[4][k];
                } else {
                    d = g2;
                }
                dov[v][k] = d;
                dot += ov[v][k] * d;
            }
        }
        dot = group_sum(dot, kWave);
        const float n = nrm[r];
        const bool through = n >= 1e-12f;
        const float rn = through ? 1.f / n : 1e12f;
        float wr = 0.f;
        if (w_mode) {
            const int32_t d = w_rowptr[r + 1] - w_rowptr[r];
            wr = (w_mode == 1) ? (float)d : (d > 0 ? 1.f : 0.f);
        }
        int sl = -1;
        float rw = 1.f;
        if constexpr (RANGES) {
            sl = br.slot(r);
            if (rw_rowptr) {   // (spmm.hip inv_deg: the MEAN transposed weight)
                const int32_t d = rw_rowptr[r + 1] - rw_rowptr[r];
                rw = __frcp_rn((float)(d > 0 ? d : 1));
            }
        }
#pragma unroll
        for (int v = 0; v < NV; ++v) {
            if (!cok[v]) continue;
            float out[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                out[k] = through ? (dov[v][k] - ov[v][k] * dot) * rn : dov[v][k] * rn;
                db[v][k] += out[k];
                dw[v][k] = fmaf(wr, out[k], dw[v][k]);
                tmax = max(tmax, __float_as_uint(out[k]) & 0x7fffffffu);
            }
            if constexpr (RANGES) {
                if (sl >= 0) {
                    float4* a = reinterpret_cast<float4*>(&red[wave][sl][cpos[v]]);
                    float4 t = *a;
                    t.x += rw_rowptr ? __fmul_rn(out[0], rw) : out[0];
                    t.y += rw_rowptr ? __fmul_rn(out[1], rw) : out[1];
                    t.z += rw_rowptr ? __fmul_rn(out[2], rw) : out[2];
                    t.w += rw_rowptr ? __fmul_rn(out[3], rw) : out[3];
                    *a = t;
                }
            }
            store4(dh + r * lddh + cpos[v], out[0], out[1], out[2], out[3], nt);
            if (skip)
                store4(gskip + r * H + cpos[v], g1v[v][0], g1v[v][1], g1v[v][2], g1v[v][3], nt);
        }
    }
    if (amax) block_amax(amax, tmax);
    if constexpr (RANGES) {   // the range slots first; then the same LDS for db / dw
        __syncthreads();
        float* rd = rpart + (int64_t)lb * kRangeSlots * H;
        for (int c = threadIdx.x; c < kRangeSlots * H; c += 256) {
            const int q = c / H, cc = c % H;
            rd[c] = (red[0][q][cc] + red[1][q][cc]) + (red[2][q][cc] + red[3][q][cc]);
        }
        __syncthreads();
    }
#pragma unroll
    for (int v = 0; v < NV; ++v)
        if (cok[v])
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                red[wave][0][cpos[v] + k] = db[v][k];
                red[wave][1][cpos[v] + k] = dw[v][k];
            }
    __syncthreads();
    float* dst = part + (int64_t)lb * 2 * H;
    for (int c = threadIdx.x; c < H; c += 256) {
        dst[c] = (red[0][0][c] + red[1][0][c]) + (red[2][0][c] + red[3][0][c]);
        dst[H + c] = (red[0][1][c] + red[1][1][c]) + (red[2][1][c] + red[3][1][c]);
    }
}

inline bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

static int g_rows_nt = 0;
void set_rows_nt(int on) { g_rows_nt = on ? 1 : 0; }
int rows_nt() { return g_rows_nt; }
static int g_rows_rev = 1;   // bit 0 on: bwd_rows 107.5 -> 92.9 us in the cfg2 step (profiles/r03_ab_rows_rev.txt)
void set_rows_rev(int on) { g_rows_rev = on & 15; }
int rows_rev() { return g_rows_rev; }

}  // namespace bgnn

using namespace bgnn;

// ---------------------------------------------------------------------------
// Output-gradient prep of a dense Linear (the encoder MLP's LinearFn.backward,
// Models/BuckGNN.py:67-74) in one pass over g [N, C]: the fused ReLU's mask
// (g_out = y > 0 ? g : 0; y = NULL: no mask, g_out = NULL: not written), per-block column sums for the bias gradient
// (part[blk][0][c], the layout bgnn_reduce_partials reads) and max|g_out| folded into *amax.
// C4 = C / 4 threads per row (a power of two dividing 256), 256 / C4 rows per block step; the
// column sums are reduced over the block's threads in a fixed order.
constexpr int kPrepBlocks = 512;

__global__ __launch_bounds__(256) void k_linear_bwd_prep(const float4* __restrict__ g, const float4* __restrict__ y,
                                                         int64_t N, int C4, float4* __restrict__ gout,
                                                         float* __restrict__ part, uint32_t* __restrict__ amax) {
    __shared__ float4 red[256];
    const int t = threadIdx.x;
    const int rpi = 256 / C4;
    const int c4 = t % C4;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    uint32_t m = 0;
    // UR rows per iteration with their loads issued together (one load per row in flight left
    // this pass latency-bound on tall inputs: EA_GNN's node-level [N, 512] gradients)
    constexpr int UR = 4;
    const int64_t stride = (int64_t)gridDim.x * rpi;
    for (int64_t r0 = (int64_t)blockIdx.x * rpi + t / C4; r0 < N; r0 += UR * stride) {
        float4 vv[UR], qq[UR];
#pragma unroll
        for (int u = 0; u < UR; ++u) {
            const int64_t r = r0 + u * stride;
            vv[u] = r < N ? g[r * C4 + c4] : make_float4(0.f, 0.f, 0.f, 0.f);
            if (y) qq[u] = r < N ? y[r * C4 + c4] : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int u = 0; u < UR; ++u) {
            const int64_t r = r0 + u * stride;
            float4 v = vv[u];
            if (y) {
                const float4 q = qq[u];
                v.x = q.x > 0.f ? v.x : 0.f;
                v.y = q.y > 0.f ? v.y : 0.f;
                v.z = q.z > 0.f ? v.z : 0.f;
                v.w = q.w > 0.f ? v.w : 0.f;
            }
            if (gout && r < N) gout[r * C4 + c4] = v;
            acc.x += v.x;
            acc.y += v.y;
            acc.z += v.z;
            acc.w += v.w;
            m = max(m, max(max(__float_as_uint(v.x) & 0x7fffffffu, __float_as_uint(v.y) & 0x7fffffffu),
                           max(__float_as_uint(v.z) & 0x7fffffffu, __float_as_uint(v.w) & 0x7fffffffu)));
        }
    }
    red[t] = acc;
    // one atomic per block (same-address atomics serialise in L2)
    __shared__ uint32_t wmax[4];
    for (int o = 32; o > 0; o >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, o, kWave));
    if ((t & 63) == 0) wmax[t >> 6] = m;
    __syncthreads();
    if (t == 0) {
        m = max(max(wmax[0], wmax[1]), max(wmax[2], wmax[3]));
        if (m) atomicMax(amax, m);
    }
    if (t < C4) {
        float4 s4 = red[t];
        for (int k = 1; k < rpi; ++k) {
            const float4 q = red[t + k * C4];
            s4.x += q.x;
            s4.y += q.y;
            s4.z += q.z;
            s4.w += q.w;
        }
        reinterpret_cast<float4*>(part + (int64_t)blockIdx.x * 2 * (4 * C4))[t] = s4;
    }
}

// bf16 form (EA_GNN's bf16 configuration, bgnn.fused.LinearBf16Fn / bgnn.ea's gathered Linear):
// g, y, g_out bf16 [N, C] (8 elements per 16-B access, C8 = C / 8 threads per row), column sums
// in f32 (each bf16 value is exact in f32), no max|g| (the bf16 GEMMs need no operand scale).
// Replaces torch's threshold_backward + sum(g, 0, dtype=float32): one pass instead of three.
__device__ __forceinline__ float bf16_lo(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float bf16_hi(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }

__global__ __launch_bounds__(256) void k_linear_bwd_prep_bf16(const uint4* __restrict__ g, const uint4* __restrict__ y,
                                                              int64_t N, int C8, uint4* __restrict__ gout,
                                                              float* __restrict__ part) {
    __shared__ float red[256][8];
    const int t = threadIdx.x;
    const int rpi = 256 / C8;
    const int c8 = t % C8;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    // UR rows per iteration, their loads issued together: one 16-B load per row and a grid of
    // 512 blocks left a bias-only pass (no y) latency-bound at ~2 TB/s
    constexpr int UR = 4;
    const int64_t stride = (int64_t)gridDim.x * rpi;
    for (int64_t r0 = (int64_t)blockIdx.x * rpi + t / C8; r0 < N; r0 += UR * stride) {
        uint4 v[UR], q[UR];
#pragma unroll
        for (int u = 0; u < UR; ++u) {
            const int64_t r = r0 + u * stride;
            v[u] = r < N ? g[r * C8 + c8] : make_uint4(0u, 0u, 0u, 0u);
            if (y) q[u] = r < N ? y[r * C8 + c8] : make_uint4(0u, 0u, 0u, 0u);
        }
#pragma unroll
        for (int u = 0; u < UR; ++u) {
            const int64_t r = r0 + u * stride;
            uint32_t w[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
            if (y) {
                const uint32_t qy[4] = {q[u].x, q[u].y, q[u].z, q[u].w};
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const uint32_t lo = bf16_lo(qy[k]) > 0.f ? 0x0000ffffu : 0u;
                    const uint32_t hi = bf16_hi(qy[k]) > 0.f ? 0xffff0000u : 0u;
                    w[k] &= lo | hi;
                }
                if (gout && r < N) gout[r * C8 + c8] = make_uint4(w[0], w[1], w[2], w[3]);
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                acc[2 * k] += bf16_lo(w[k]);
                acc[2 * k + 1] += bf16_hi(w[k]);
            }
        }
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) red[t][k] = acc[k];
    __syncthreads();
    if (t < C8) {
        float s8[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) s8[k] = red[t][k];
        for (int q = 1; q < rpi; ++q)
#pragma unroll
            for (int k = 0; k < 8; ++k) s8[k] += red[t + q * C8][k];
        float4* dst = reinterpret_cast<float4*>(part + (int64_t)blockIdx.x * 2 * (8 * C8)) + 2 * t;
        dst[0] = make_float4(s8[0], s8[1], s8[2], s8[3]);
        dst[1] = make_float4(s8[4], s8[5], s8[6], s8[7]);
    }
}

extern "C" int bgnn_linear_bwd_prep_bf16(const void* g, const void* y, int64_t N, int32_t C, void* g_out,
                                         float* partial, void* stream) {
    BGNN_REQUIRE(g && partial && N >= 0, "linear_bwd_prep_bf16: null pointer or negative size");
    BGNN_REQUIRE(y == nullptr || g_out != nullptr, "linear_bwd_prep_bf16: a ReLU mask needs g_out");
    BGNN_REQUIRE(C >= 8 && C <= 2048 && C % 8 == 0 && (256 % (C / 8)) == 0,
                 "linear_bwd_prep_bf16: C = %d must be 8 * a power of two <= 2048", C);
    BGNN_REQUIRE((((uintptr_t)g | (uintptr_t)(g_out ? g_out : g) | (uintptr_t)partial | (uintptr_t)(y ? y : g)) & 15) == 0,
                 "linear_bwd_prep_bf16: pointers must be 16-B aligned");
    hipStream_t s = as_stream(stream);
    hipLaunchKernelGGL(k_linear_bwd_prep_bf16, dim3(kPrepBlocks), dim3(256), 0, s, reinterpret_cast<const uint4*>(g),
                       reinterpret_cast<const uint4*>(y), N, C / 8, reinterpret_cast<uint4*>(g_out), partial);
    BGNN_CHECK_LAUNCH();
    return BGNN_OK;
}

extern "C" int32_t bgnn_linear_bwd_prep_slots(void) { return kPrepBlocks; }

extern "C" int bgnn_linear_bwd_prep(const float* g, const float* y, int64_t N, int32_t C, float* g_out,
                                    float* partial, float* amax, void* stream) {
    BGNN_REQUIRE(g && partial && amax && N >= 0, "linear_bwd_prep: null pointer or negative size");
    BGNN_REQUIRE(y == nullptr || g_out != nullptr, "linear_bwd_prep: a ReLU mask needs g_out");
    BGNN_REQUIRE(C >= 4 && C <= 1024 && C % 4 == 0 && (256 % (C / 4)) == 0,
                 "linear_bwd_prep: C = %d must be 4 * a power of two <= 1024", C);
    BGNN_REQUIRE((((uintptr_t)g | (uintptr_t)(g_out ? g_out : g) | (uintptr_t)partial | (uintptr_t)(y ? y : g)) & 15) == 0,
                 "linear_bwd_prep: pointers must be 16-B aligned");
    hipStream_t s = as_stream(stream);
    hipLaunchKernelGGL(k_linear_bwd_prep, dim3(kPrepBlocks), dim3(256), 0, s, reinterpret_cast<const float4*>(g),
                       reinterpret_cast<const float4*>(y), N, C / 4, reinterpret_cast<float4*>(g_out), partial,
                       reinterpret_cast<uint32_t*>(amax));
    BGNN_CHECK_LAUNCH();
    return BGNN_OK;
}

extern "C" int bgnn_reduce_partials(const float* partial, int32_t n_slots, int32_t H, float* out0, float* out1,
                                    int32_t accumulate, void* stream) {
    BGNN_REQUIRE(partial && H > 0 && n_slots >= 0, "reduce_partials: bad args");
    hipStream_t s = as_stream(stream);
    if (g_one_pass_reduce) {
        hipLaunchKernelGGL(k_reduce_slots<0>, dim3((H + 7) / 8), dim3(256), 0, s, partial, n_slots, H, out0, out1,
                           accumulate, (int64_t)0, nullptr, nullptr, 0.f, 0.f, nullptr, nullptr, nullptr, nullptr,
                           nullptr, nullptr, nullptr);
        BGNN_CHECK_LAUNCH();
        return BGNN_OK;
    }
    const int stride = slots_stage1(const_cast<float*>(partial), n_slots, H, s);
    BGNN_CHECK_LAUNCH();
    hipLaunchKernelGGL(k_reduce_partials, dim3((H + 63) / 64), dim3(256), 0, s, partial, n_slots, stride, H, out0,
                       out1, accumulate);
    BGNN_CHECK_LAUNCH();
    return BGNN_OK;
}

extern "C" int bgnn_bn_finalize(const float* bn_partial, int32_t n_slots, int32_t H, int64_t count,
                                const float* gamma, const float* beta, float eps, float momentum,
                                float* running_mean, float* running_var, float* mean, float* invstd, float* scale,
                                float* shift, void* stream) {
    BGNN_REQUIRE(bn_partial && H > 0 && count > 0 && mean && invstd && scale && shift, "bn_finalize: bad args");
    hipStream_t s = as_stream(stream);
    if (g_one_pass_reduce) {
        hipLaunchKernelGGL(k_reduce_slots<1>, dim3((H + 7) / 8), dim3(256), 0, s, bn_partial, n_slots, H, nullptr,
                           nullptr, 0, count, gamma, beta, eps, momentum, running_mean, running_var, mean, invstd,
                           scale, shift, nullptr);
        BGNN_CHECK_LAUNCH();
        return BGNN_OK;
    }
    const int stride = slots_stage1(const_cast<float*>(bn_partial), n_slots, H, s);
    BGNN_CHECK_LAUNCH();
    hipLaunchKernelGGL(k_bn_finalize, dim3((H + 63) / 64), dim3(256), 0, s, bn_partial, n_slots, stride, H, count,
                       gamma, beta, eps, momentum, running_mean, running_var, mean, invstd, scale, shift);
    BGNN_CHECK_LAUNCH();
    return BGNN_OK;
}

extern "C" int bgnn_bn_finalize_shifted(const float* bn_partial, int32_t n_slots, int32_t H, int64_t count,
                                        const float* kshift, const float* gamma, const float* beta, float eps,
                                        float momentum, float* running_mean, float* running_var, float* mean,
                                        float* invstd, float* scale, float* shift, void* stream) {
    BGNN_REQUIRE(bn_partial && kshift && H > 0 && count > 0 && mean && invstd && scale && shift,
                 "bn_finalize_shifted: bad args");
    hipLaunchKernelGGL(k_reduce_slots<1>, dim3((H + 7) / 8), dim3(256), 0, as_stream(stream), bn_partial, n_slots, H,
                       nullptr, nullptr, 0, count, gamma, beta, eps, momentum, running_mean, running_var, mean, invstd,
                       scale, shift, kshift);
    BGNN_CHECK_LAUNCH();
    return BGNN_OK;
}

extern "C" int bgnn_bn_eval_coeffs(int32_t H, const float* gamma, const float* beta, float eps,
                                   const float* running_mean, const float* running_var, float* scale, float* shift,
                                   void* stream) {
    BGNN_REQUIRE(H > 0 && running_mean && running_var && scale && shift, "bn_eval_coeffs: bad args");
    hipStream_t s = as_stream(stream);
    hipLaunchKernelGGL(k_bn_eval, dim3((H + 255) / 256), dim3(256), 0, s, H, gamma, beta, eps, running_mean,
                       running_var, scale, shift);
    BGNN_CHECK_LAUNCH();
    return BGNN_OK;
}

extern "C" int bgnn_sage_apply(const float* o, const float* scale, const float* shift, const float* x_prev,
                               int32_t skip, float p, uint64_t seed, int64_t n_rows, int32_t H, float* x_next,
                               float* amax, const int32_t* ranges, float* range_partial, void* stream) {
    BGNN_REQUIRE(H > 0 && H % 4 == 0, "sage_apply: H must be a multiple of 4");
    BGNN_REQUIRE(p >= 0.f && p < 1.f, "sage_apply: dropout p must be in [0, 1)");
    BGNN_REQUIRE((scale == nullptr) == (shift == nullptr), "sage_apply: scale/shift must both be set or NULL");
    BGNN_REQUIRE(!skip || x_prev, "sage_apply: skip requires x_prev");
    BGNN_REQUIRE(al16(o) && al16(x_next) && (!x_prev || al16(x_prev)) && (!scale || (al16(scale) && al16(shift))),
                 "sage_apply: pointers must be 16-byte aligned");
    BGNN_REQUIRE(!ranges || (range_partial && ((uintptr_t)range_partial & 15) == 0 && H <= 512),
                 "sage_apply: ranges need a 16-B aligned range_partial and H <= 512");
    if (n_rows == 0) return BGNN_OK;
    hipStream_t s = as_stream(stream);
    if (ranges) {   // row-blocked form with the range partials (the same x_next)
        const uint32_t thr = dropout_threshold(p);
        const float inv_keep = thr ? 1.f / (1.f - p) : 1.f;
        int64_t rpb = 0;
        const int64_t blocks = rows_slots_of(n_rows, &rpb);
        if (H > 256)
            hipLaunchKernelGGL(k_sage_apply_rows<2>, dim3((unsigned)blocks), dim3(256), 0, s, o, scale, shift, x_prev,
                               skip, thr, inv_keep, seed, n_rows, H, rpb, x_next, reinterpret_cast<uint32_t*>(amax),
                               rows_nt(), ranges, range_partial);
        else
            hipLaunchKernelGGL(k_sage_apply_rows<1>, dim3((unsigned)blocks), dim3(256), 0, s, o, scale, shift, x_prev,
                               skip, thr, inv_keep, seed, n_rows, H, rpb, x_next, reinterpret_cast<uint32_t*>(amax),
                               rows_nt(), ranges, range_partial);
        BGNN_CHECK_LAUNCH();
        return BGNN_OK;
    }
    const int64_t n4 = n_rows * (H / 4);
    int64_t blocks = (n4 + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    const int rev = (rows_rev() & 2) ? 1 : 0;
    if (rev) blocks = (blocks + 7) / 8 * 8;
    const uint32_t thr = dropout_threshold(p);
    const float inv_keep = thr ? 1.f / (1.f - p) : 1.f;
    hipLaunchKernelGGL(k_sage_apply, dim3((unsigned)blocks), dim3(256), 0, s, (const float4*)o, scale, shift,
                       (const float4*)x_prev, skip, thr, inv_keep, seed, n4, H / 4, (float4*)x_next,
                       reinterpret_cast<uint32_t*>(amax), rows_nt(), rev);
    BGNN_CHECK_LAUNCH();
    return BGNN_OK;
}

extern "C" int32_t bgnn_rows_slots(int64_t n_rows) {
    int64_t rpb = 0;
    return (int32_t)rows_grid(n_rows, 4, &rpb);
}

extern "C" int bgnn_sage_bwd_stats(const float* g, const int64_t* g_rows, const float* o, const float* scale,
                                   const float* shift,
                                   const float* mean, const float* invstd, float p, uint64_t seed, int64_t n_rows,
                                   int32_t H, float* partial2, void* stream) {
    BGNN_REQUIRE(H > 0 && H % 4 == 0 && H <= 1024, "sage_bwd_stats: H=%d unsupported", H);
    BGNN_REQUIRE(g && o && scale && shift && mean && invstd && partial2, "sage_bwd_stats: null pointer");
    BGNN_REQUIRE(al16(g) && al16(o) && al16(scale) && al16(shift) && al16(mean) && al16(invstd) && al16(partial2),
                 "sage_bwd_stats: pointers must be 16-byte aligned");
    hipStream_t s = as_stream(stream);
    int64_t rpb = 0;
    const int64_t blocks = rows_grid(n_rows, 4, &rpb);
    const uint32_t thr = dropout_threshold(p);
    const float inv_keep = thr ? 1.f / (1.f - p) : 1.f;
    hipLaunchKernelGGL(k_sage_bwd_stats, dim3((unsigned)blocks), dim3(256), 0, s, g, g_rows, o, scale, shift, mean, invstd,
                       thr, inv_keep, seed, n_rows, H, rpb, partial2);
    BGNN_CHECK_LAUNCH();
    return BGNN_OK;
}

extern "C" int bgnn_sage_bwd_rows(const float* g, const int64_t* g_rows, const float* o, const float* nrm,
                                  const float* scale,
                                  const float* shift, const float* gamma, const float* mean, const float* invstd,
                                  const float* sum_g2, const float* sum_g2xhat, float p, uint64_t seed,
                                  int32_t skip, int64_t n_rows, int32_t H, float* dh, int64_t lddh, float* gskip,
                                  float* partial_db, float* amax, const int32_t* w_rowptr, int32_t w_mode,
                                  const int32_t* ranges, const int32_t* range_w_rowptr, float* range_partial,
                                  void* stream) {
    BGNN_REQUIRE(H > 0 && H % 4 == 0 && H <= 512, "sage_bwd_rows: H=%d unsupported", H);
    BGNN_REQUIRE(w_mode >= 0 && w_mode <= 2 && (w_mode == 0 || w_rowptr), "sage_bwd_rows: bad row weights");
    BGNN_REQUIRE(lddh >= H && lddh % 4 == 0, "sage_bwd_rows: bad lddh");
    BGNN_REQUIRE(!skip || gskip, "sage_bwd_rows: skip requires gskip");
    BGNN_REQUIRE(!mean || (invstd && sum_g2 && sum_g2xhat), "sage_bwd_rows: BN stats incomplete");
    BGNN_REQUIRE(al16(g) && al16(o) && al16(dh) && (!gskip || al16(gskip)) && al16(partial_db),
                 "sage_bwd_rows: pointers must be 16-byte aligned");
    BGNN_REQUIRE(!ranges || (range_partial && al16(range_partial)), "sage_bwd_rows: ranges need range_partial");
    hipStream_t s = as_stream(stream);
    int64_t rpb = 0;
    const int64_t blocks = rows_grid(n_rows, 4, &rpb);
    const uint32_t thr = dropout_threshold(p);
    const float inv_keep = thr ? 1.f / (1.f - p) : 1.f;
#define BGNN_ROWS(NV, R)                                                                                              \
    hipLaunchKernelGGL((k_sage_bwd_rows<NV, true, R>), dim3((unsigned)blocks), dim3(256), 0, s, g, g_rows, o, nrm,   \
                       scale,                                                                                       \
                       shift, gamma, mean, invstd, sum_g2, sum_g2xhat, thr, inv_keep, seed, skip, n_rows, H, rpb,    \
                       dh, lddh, gskip, partial_db, reinterpret_cast<uint32_t*>(amax), rows_nt(), w_rowptr, w_mode,  \
                       rows_rev() & 1, ranges, range_w_rowptr, range_partial)
    if (ranges) {
        if (H > 256) BGNN_ROWS(2, true);
        else BGNN_ROWS(1, true);
    } else {
        if (H > 256) BGNN_ROWS(2, false);
        else BGNN_ROWS(1, false);
    }
#undef BGNN_ROWS
    BGNN_CHECK_LAUNCH();
    return BGNN_OK;
}

// The L2-normalize backward of SAGEConv(normalize=True) on its own (bgnn.nn.SAGEConv's fused
// per-module path, Models/BuckGNN.py:434 under the PyG shim): dh = (g - o <o, g>) / ||h|| per
// row (rows with ||h|| < 1e-12 get g * 1e12: F.normalize's clamped denominator), written at dh (row stride lddh), per-block column sums of dh into partial_db (the bias
// gradient, bgnn_reduce_partials layout) and max |dh| folded into *amax.
extern "C" int bgnn_l2norm_bwd(const float* g, const float* o, const float* nrm, int64_t n_rows, int32_t H,
                               float* dh, int64_t lddh, float* partial_db, float* amax, void* stream) {
    BGNN_REQUIRE(H > 0 && H % 4 == 0 && H <= 512, "l2norm_bwd: H=%d unsupported", H);
    BGNN_REQUIRE(g && o && nrm && dh && partial_db && amax, "l2norm_bwd: null pointer");
    BGNN_REQUIRE(lddh >= H && lddh % 4 == 0, "l2norm_bwd: bad lddh");
    BGNN_REQUIRE(al16(g) && al16(o) && al16(dh) && al16(partial_db), "l2norm_bwd: pointers must be 16-byte aligned");
    hipStream_t s = as_stream(stream);
    int64_t rpb = 0;
    const int64_t blocks = rows_grid(n_rows, 4, &rpb);
    if (H > 256)
        hipLaunchKernelGGL((k_sage_bwd_rows<2, false>), dim3((unsigned)blocks), dim3(256), 0, s, g, nullptr, o, nrm, nullptr,
                           nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 0u, 1.f, (uint64_t)0, 0, n_rows, H,
                           rpb, dh, lddh, nullptr, partial_db, reinterpret_cast<uint32_t*>(amax), rows_nt(), nullptr,
                           0, rows_rev() & 1, nullptr, nullptr, nullptr);
    else
        hipLaunchKernelGGL((k_sage_bwd_rows<1, false>), dim3((unsigned)blocks), dim3(256), 0, s, g, nullptr, o, nrm, nullptr,
                           nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 0u, 1.f, (uint64_t)0, 0, n_rows, H,
                           rpb, dh, lddh, nullptr, partial_db, reinterpret_cast<uint32_t*>(amax), rows_nt(), nullptr,
                           0, rows_rev() & 1, nullptr, nullptr, nullptr);
    BGNN_CHECK_LAUNCH();
    return BGNN_OK;
}
