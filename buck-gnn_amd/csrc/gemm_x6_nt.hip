// f16x3 GEMM C = A B^T with K-contiguous operands (the SAGE forward z = x [W_l;W_r]^T and input
// gradient dx = [dz_l | dh] [W_l;W_r], plus the drop-add epilogue of bgnn_gemm_f32_dropadd):
// the instantiations of gemm_x6_kernel.h with the plain (0) and the drop-add (8) epilogue.
#include "gemm_x6_kernel.h"

namespace bgnn {

void launch_x6_nt_main(int cfg, int abl, dim3 grid, hipStream_t s, const GemmArgs& g) {
    if (abl == 8) launch_x6_a<1, 0, 1, 8>(cfg, grid, s, g);
    else launch_x6_a<1, 0, 1, 0>(cfg, grid, s, g);
}

}  // namespace bgnn
