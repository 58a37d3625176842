// Per-CU operand ingest microbenchmark: how many bytes per cycle one CU pulls from L2 (buffer
// resident in L2) or from HBM (buffer far larger than the caches) with float4 register loads,
// at 1 or 2 workgroups of 256/512 threads per CU. Decides whether the f16x3 GEMMs (~10-11 B/cyc
// per CU of operand traffic) sit at a per-CU ingest ceiling.
//   hipcc --offload-arch=gfx950 -O3 tools/proto/l2bw.hip -o /tmp/l2bw && /tmp/l2bw
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

template <int UNROLL>
__global__ void k_read(const float4* __restrict__ buf, long n4, long per_wg, int iters, float* __restrict__ out) {
    // WG b reads [start, start + per_wg) float4s of buf (wrapping), iters times
    const long start = (long)blockIdx.x * per_wg % n4;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int it = 0; it < iters; ++it) {
        for (long i = threadIdx.x; i < per_wg; i += (long)blockDim.x * UNROLL) {
            float4 v[UNROLL];
#pragma unroll
            for (int u = 0; u < UNROLL; ++u) {
                long j = start + i + (long)u * blockDim.x;
                if (j >= n4) j -= n4;
                v[u] = buf[j];
            }
#pragma unroll
            for (int u = 0; u < UNROLL; ++u) {
                acc.x += v[u].x; acc.y += v[u].y; acc.z += v[u].z; acc.w += v[u].w;
            }
        }
    }
    const float s = acc.x + acc.y + acc.z + acc.w;
    if (s == 1234.5f) out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
    int dev = 0, clk = 0, cus = 0;
    hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, dev);
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const double ghz = clk / 1e6;
    printf("CUs %d, nominal clock %.2f GHz\n", cus, ghz);
    const long big = 1L << 31;   // 8 GiB of floats... 2^31 floats = 8 GiB
    float4* buf;
    hipMalloc(&buf, big * 4);
    hipMemset(buf, 0, big * 4);
    float* out;
    hipMalloc(&out, 1 << 24);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    struct Case { const char* name; long footprint_bytes; long per_wg_bytes; int wgs_per_cu; int threads; int iters; };
    std::vector<Case> cases = {
        {"L2-resident 1 MiB, 1 WG/CU x 512 thr", 1L << 20, 1L << 20, 1, 512, 8},
        {"L2-resident 1 MiB, 1 WG/CU x 256 thr", 1L << 20, 1L << 20, 1, 256, 8},
        {"L2-resident 1 MiB, 2 WG/CU x 256 thr", 1L << 20, 1L << 20, 2, 256, 8},
        {"L2-resident 1 MiB, 4 WG/CU x 256 thr", 1L << 20, 1L << 20, 4, 256, 8},
        {"HBM streaming 4 GiB, 1 WG/CU x 512 thr", 4L << 30, (4L << 30) / 256, 1, 512, 1},
        {"HBM streaming 4 GiB, 4 WG/CU x 256 thr", 4L << 30, (4L << 30) / 1024, 4, 256, 1},
    };
    for (const Case& c : cases) {
        const long n4 = c.footprint_bytes / 16, per_wg = c.per_wg_bytes / 16;
        const int grid = cus * c.wgs_per_cu;
        for (int rep = 0; rep < 3; ++rep) {
            hipEventRecord(e0);
            hipLaunchKernelGGL(k_read<8>, dim3(grid), dim3(c.threads), 0, 0, buf, n4, per_wg, c.iters, out);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            const double bytes = (double)grid * per_wg * 16 * c.iters;
            const double tbs = bytes / (ms * 1e-3) / 1e12;
            if (rep == 2)
                printf("%-44s %8.3f ms  %7.2f TB/s  %6.2f B/cyc/CU at %.2f GHz (%.2f at 2.0)\n", c.name, ms, tbs,
                       tbs * 1e12 / cus / (ghz * 1e9), ghz, tbs * 1e12 / cus / 2.0e9);
        }
    }
    hipFree(buf);
    hipFree(out);
    return 0;
}
