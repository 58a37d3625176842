// The bf16-operand family of gemm_x6_kernel.h (PREC 2: one bf16 product, f32 accumulation; the
// bf16 configuration of EA_GNN, BASELINE configs[4]), with f32 or bf16 storage of A / B / C.
#include "gemm_x6_kernel.h"

namespace bgnn {

void launch_x6_prec2(int ta, int tb, int cfg, dim3 grid, hipStream_t s, const GemmArgs& g) {
    if (ta == 0 && tb == 0) launch_x6_a<2, 0, 0, 0>(cfg, grid, s, g);
    else if (ta == 0 && tb == 1) launch_x6_a<2, 0, 1, 0>(cfg, grid, s, g);
    else if (ta == 1 && tb == 0) launch_x6_a<2, 1, 0, 0>(cfg, grid, s, g);
    else launch_x6_a<2, 1, 1, 0>(cfg, grid, s, g);
}

// bf16 storage (PREC 2): st = bit 0 A, bit 1 B, bit 2 C; the combinations EA_GNN uses
void launch_x6_bf16_storage(int ta, int tb, int cfg, int st, dim3 grid, hipStream_t s, const GemmArgs& g) {
    if (ta == 0 && tb == 1 && st == 7) launch_x6_a<2, 0, 1, 16 + 7>(cfg, grid, s, g);        // (gemm_b16.hip when K % 64 == 0)
    else if (ta == 0 && tb == 1 && st == 3) launch_x6_a<2, 0, 1, 16 + 3>(cfg, grid, s, g);
    else if (ta == 0 && tb == 1 && st == 5) launch_x6_a<2, 0, 1, 16 + 5>(cfg, grid, s, g);   // edge fwd / dgrad
    else if (ta == 0 && tb == 1 && st == 4) launch_x6_a<2, 0, 1, 16 + 4>(cfg, grid, s, g);   // f32 in, bf16 out
    else if (ta == 0 && tb == 1 && st == 1) launch_x6_a<2, 0, 1, 16 + 1>(cfg, grid, s, g);   // bf16 in, f32 out
    else if (ta == 1 && tb == 0 && st == 3) launch_x6_a<2, 1, 0, 16 + 3>(cfg, grid, s, g);   // wgrad g^T e
    else if (ta == 1 && tb == 0 && st == 1) launch_x6_a<2, 1, 0, 16 + 1>(cfg, grid, s, g);
    else if (ta == 1 && tb == 0 && st == 2) launch_x6_a<2, 1, 0, 16 + 2>(cfg, grid, s, g);
    else launch_x6_a<2, 0, 1, 16 + 5>(cfg, grid, s, g);   // (not reached: bgnn_gemm_bf16 validates st)
}

}  // namespace bgnn
