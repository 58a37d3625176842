// Timing ablations of the f16x3 C = A B^T GEMM (bgnn_gemm_set_cfg(100 * abl + cfg); measurement
// only, wrong results): 1 no split arithmetic, 2 no global loads, 3 no staging, 4 MFMA + barriers,
// 5 no C stores, 6 cached C stores, 7 prefetch distance 1, 9 no A loads, 10 no B loads, 11 no
// MFMAs (see k_gemm_x6 in gemm_x6_kernel.h).
#include "gemm_x6_kernel.h"

namespace bgnn {

void launch_x6_nt_abl(int cfg, int abl, dim3 grid, hipStream_t s, const GemmArgs& g) {
    switch (abl) {
        case 1: launch_x6_a<1, 0, 1, 1>(cfg, grid, s, g); break;
        case 2: launch_x6_a<1, 0, 1, 2>(cfg, grid, s, g); break;
        case 3: launch_x6_a<1, 0, 1, 3>(cfg, grid, s, g); break;
        case 4: launch_x6_a<1, 0, 1, 4>(cfg, grid, s, g); break;
        case 5: launch_x6_a<1, 0, 1, 5>(cfg, grid, s, g); break;
        case 6: launch_x6_a<1, 0, 1, 6>(cfg, grid, s, g); break;
        case 9: launch_x6_a<1, 0, 1, 9>(cfg, grid, s, g); break;
        case 10: launch_x6_a<1, 0, 1, 10>(cfg, grid, s, g); break;
        case 11: launch_x6_a<1, 0, 1, 11>(cfg, grid, s, g); break;
        default: launch_x6_a<1, 0, 1, 7>(cfg, grid, s, g); break;
    }
}

}  // namespace bgnn
