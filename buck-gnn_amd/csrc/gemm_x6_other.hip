// f16x3 GEMMs with a k-major operand: the SAGE weight gradient d[W_l;W_r] = [dz_l | dh]^T x
// (TA = 1, TB = 0; k-major quad staging, split-K) and the remaining transpose combinations.
#include "gemm_x6_kernel.h"

namespace bgnn {

void launch_x6_h3_other(int ta, int tb, int cfg, dim3 grid, hipStream_t s, const GemmArgs& g) {
    if (ta == 1 && tb == 0) launch_x6_a<1, 1, 0, 0>(cfg, grid, s, g);
    else if (ta == 0 && tb == 0) launch_x6_a<1, 0, 0, 0>(cfg, grid, s, g);
    else launch_x6_a<1, 1, 1, 0>(cfg, grid, s, g);
}

}  // namespace bgnn
