// Probe of the gfx950 16-bit MFMAs' accumulation arithmetic ("MFMA shape and
// rounding"): what D = A B + C does with bits below the f32 result's ulp, for
// v_mfma_f32_16x16x32_{f16,bf16} and v_mfma_f32_32x32x16_{f16,bf16}.
//
// Part 1, crafted cases on the (0, 0) output: C and a handful of A[0][k] * B[k][0] products chosen
// so that round-to-nearest-even, truncation (round toward zero) and a limited-width internal sum
// give different f32 results.
// Part 2, chains: S MFMAs accumulate into one D (a K = 32 S or 16 S dot product, as a GEMM's main
// loop does), random operands (positive, or signed), every output against the exact (fp64) sum
// and against an f32 round-to-nearest fmaf chain over the same products in the same k order: the
// mean signed error (bias) and the RMS error, both relative to sum |a b|.
//
//   hipcc --offload-arch=gfx950 -O3 tools/proto/mfma_round.hip -o /tmp/mfma_round && /tmp/mfma_round
#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>
#include <cmath>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <random>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

// SHAPE 0 = 16x16x32, 1 = 32x32x16; BF = bf16 operands. A / B: [steps][64 lanes][8] 16-bit
// patterns, C / D: [64 lanes][16] f32 (16x16x32 uses the first 4).
template <int SHAPE, bool BF>
__global__ void k_chain(const uint16_t* __restrict__ A, const uint16_t* __restrict__ B, const float* __restrict__ C,
                        float* __restrict__ D, int steps) {
    const int l = threadIdx.x;
    floatx16 acc16;
    floatx4 acc4;
    for (int r = 0; r < 16; ++r) acc16[r] = C[l * 16 + r];
    for (int r = 0; r < 4; ++r) acc4[r] = C[l * 16 + r];
    for (int s = 0; s < steps; ++s) {
        uint16_t av[8], bv[8];
        for (int j = 0; j < 8; ++j) { av[j] = A[(s * 64 + l) * 8 + j]; bv[j] = B[(s * 64 + l) * 8 + j]; }
        if constexpr (BF) {
            bf16x8 a, b;
            memcpy(&a, av, 16); memcpy(&b, bv, 16);
            if constexpr (SHAPE == 0) acc4 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc4, 0, 0, 0);
            else acc16 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc16, 0, 0, 0);
        } else {
            half8 a, b;
            memcpy(&a, av, 16); memcpy(&b, bv, 16);
            if constexpr (SHAPE == 0) acc4 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, acc4, 0, 0, 0);
            else acc16 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc16, 0, 0, 0);
        }
    }
    for (int r = 0; r < 16; ++r) D[l * 16 + r] = SHAPE == 0 ? (r < 4 ? acc4[r] : 0.f) : acc16[r];
}

// ---------------------------------------------------------------- host side: layouts
struct Shape {
    int mn, kstep;   // output tile mn x mn, k per MFMA
};
static const Shape kShapes[2] = {{16, 32}, {32, 16}};

// lane and element of A[row][k] (A operand) / B[k][col] (B operand) within one MFMA step
static void ab_pos(int shape, int rc, int k, int& lane, int& elem) {
    const Shape& s = kShapes[shape];
    lane = (k / 8) * s.mn + rc;
    elem = k % 8;
}
// lane and register of D[row][col]
static void d_pos(int shape, int row, int col, int& lane, int& reg) {
    if (shape == 0) {   // 16x16: D[4 (l >> 4) + i][l & 15]
        lane = (row / 4) * 16 + col;
        reg = row % 4;
    } else {            // 32x32: row = (r & 3) + 8 (r >> 2) + 4 (l >> 5), col = l & 31
        lane = ((row / 4) % 2) * 32 + col;
        reg = (row % 4) + 4 * (row / 8);
    }
}

static uint16_t to16(double v, bool bf) {
    if (bf) {
        float f = (float)v;
        uint32_t u;
        memcpy(&u, &f, 4);
        u += 0x7fff + ((u >> 16) & 1);
        return (uint16_t)(u >> 16);
    }
    _Float16 h = (_Float16)(float)v;
    uint16_t u;
    memcpy(&u, &h, 2);
    return u;
}
static double from16(uint16_t u, bool bf) {
    if (bf) {
        uint32_t w = (uint32_t)u << 16;
        float f;
        memcpy(&f, &w, 4);
        return f;
    }
    _Float16 h;
    memcpy(&h, &u, 2);
    return (double)(float)h;
}

struct Dev {
    uint16_t *A, *B;
    float *C, *D;
};

static int run(int shape, bool bf, const std::vector<uint16_t>& A, const std::vector<uint16_t>& B,
               const std::vector<float>& C, std::vector<float>& D, int steps, Dev& d) {
    CK(hipMemcpy(d.A, A.data(), A.size() * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(d.B, B.data(), B.size() * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(d.C, C.data(), C.size() * 4, hipMemcpyHostToDevice));
    if (shape == 0 && !bf) hipLaunchKernelGGL((k_chain<0, false>), dim3(1), dim3(64), 0, 0, d.A, d.B, d.C, d.D, steps);
    if (shape == 0 && bf) hipLaunchKernelGGL((k_chain<0, true>), dim3(1), dim3(64), 0, 0, d.A, d.B, d.C, d.D, steps);
    if (shape == 1 && !bf) hipLaunchKernelGGL((k_chain<1, false>), dim3(1), dim3(64), 0, 0, d.A, d.B, d.C, d.D, steps);
    if (shape == 1 && bf) hipLaunchKernelGGL((k_chain<1, true>), dim3(1), dim3(64), 0, 0, d.A, d.B, d.C, d.D, steps);
    CK(hipGetLastError());
    D.assign(64 * 16, 0.f);
    CK(hipMemcpy(D.data(), d.D, D.size() * 4, hipMemcpyDeviceToHost));
    return 0;
}

// one crafted case: C00 and products (k, a, b) on the (0, 0) output of one MFMA
struct Case {
    const char* what;
    double c;
    std::vector<std::tuple<int, double, double>> p;
};

static const char* name(int shape, bool bf) {
    return shape == 0 ? (bf ? "16x16x32_bf16" : "16x16x32_f16") : (bf ? "32x32x16_bf16" : "32x32x16_f16");
}

int main() {
    Dev d;
    const int kMaxSteps = 256;
    CK(hipMalloc(&d.A, (size_t)kMaxSteps * 64 * 8 * 2));
    CK(hipMalloc(&d.B, (size_t)kMaxSteps * 64 * 8 * 2));
    CK(hipMalloc(&d.C, 64 * 16 * 4));
    CK(hipMalloc(&d.D, 64 * 16 * 4));
    const double u = std::ldexp(1.0, -23);   // ulp(1.0f)
    std::vector<Case> cases = {
        {"C=1, p=+0.75ulp (RNE -> 1+ulp; RZ -> 1)", 1.0, {{0, std::ldexp(1.0, -12), 0.75 * std::ldexp(1.0, -11)}}},
        {"C=1, p=+0.5ulp tie (RNE -> 1; RZ -> 1)", 1.0, {{0, std::ldexp(1.0, -12), std::ldexp(1.0, -12)}}},
        {"C=1, p=-0.25ulp(below 1) (RNE -> 1; RZ -> 1-ulp/2)", 1.0, {{0, -std::ldexp(1.0, -13), std::ldexp(1.0, -13)}}},
        {"C=0, p0=1, p1=1.5*2^-24 (RNE -> 1+ulp; drop -> 1)", 0.0,
         {{0, 1.0, 1.0}, {1, std::ldexp(1.0, -12), 1.5 * std::ldexp(1.0, -12)}}},
        {"C=0, p0=1, 15 x 2^-26 (exact 1+1.875ulp; RNE -> 1+2ulp)", 0.0, {}},
        {"C=0, p0=1, p1=-1, p2=2^-30 (exact 2^-30)", 0.0,
         {{0, 1.0, 1.0}, {1, -1.0, 1.0}, {2, std::ldexp(1.0, -15), std::ldexp(1.0, -15)}}},
        {"C=2^-30, p0=1, p1=-1 (exact 2^-30)", std::ldexp(1.0, -30), {{0, 1.0, 1.0}, {1, -1.0, 1.0}}},
        {"C=1, p0=2^-24, p1=2^-24 (exact 1+ulp; per-product RZ -> 1)", 1.0,
         {{0, std::ldexp(1.0, -12), std::ldexp(1.0, -12)}, {1, std::ldexp(1.0, -12), std::ldexp(1.0, -12)}}},
    };
    for (int k = 1; k <= 15; ++k) cases[4].p.push_back({k, std::ldexp(1.0, -13), std::ldexp(1.0, -13)});
    cases[4].p.push_back({0, 1.0, 1.0});
    printf("Part 1: D(0,0) of one MFMA, crafted (exact value; each shape's result as (D - exact) / ulp(exact))\n");
    for (const Case& cs : cases) {
        double exact = cs.c;
        for (auto& t : cs.p) exact += std::get<1>(t) * std::get<2>(t);
        printf("  %-58s exact %.17g\n", cs.what, exact);
        for (int bfi = 0; bfi < 2; ++bfi)
            for (int shape = 0; shape < 2; ++shape) {
                const bool bf = bfi == 1;
                std::vector<uint16_t> A(64 * 8, 0), B(64 * 8, 0);
                std::vector<float> C(64 * 16, 0.f), D;
                bool ok = true;
                double q = cs.c;
                for (auto& t : cs.p) {
                    const int k = std::get<0>(t);
                    if (k >= kShapes[shape].kstep) { ok = false; break; }
                    int la, ea;
                    ab_pos(shape, 0, k, la, ea);
                    A[la * 8 + ea] = to16(std::get<1>(t), bf);
                    B[la * 8 + ea] = to16(std::get<2>(t), bf);
                    q += from16(A[la * 8 + ea], bf) * from16(B[la * 8 + ea], bf);
                }
                if (!ok) continue;
                int ld, rd;
                d_pos(shape, 0, 0, ld, rd);
                C[ld * 16 + rd] = (float)cs.c;
                if (run(shape, bf, A, B, C, D, 1, d)) return 1;
                const double got = D[ld * 16 + rd];
                const double ulp = q != 0 ? std::ldexp(1.0, std::ilogb(q) - 23) : 1e-45;
                printf("    %-14s D = %.17g  (D - exact(operands)) / ulp = %+.3f%s\n", name(shape, bf), got,
                       (got - q) / ulp, q != exact ? "  (operands rounded)" : "");
            }
    }

    printf("\nPart 2: chained MFMAs into one accumulator (K = steps * k per MFMA), all outputs, 16 trials\n");
    printf("  errors relative to sum|a b| per output: mean signed (bias), RMS; 'fmaf' = an f32 RNE fmaf chain "
           "over the same products in k order\n");
    std::mt19937_64 rng(12345);
    for (int sign = 0; sign < 2; ++sign)
        for (int K : {512, 1024, 4096})
            for (int bfi = 0; bfi < 2; ++bfi)
                for (int shape = 0; shape < 2; ++shape) {
                    const bool bf = bfi == 1;
                    const Shape& s = kShapes[shape];
                    const int steps = K / s.kstep;
                    double sb = 0, s2 = 0, fb = 0, f2 = 0;
                    long n = 0;
                    for (int trial = 0; trial < 16; ++trial) {
                        std::normal_distribution<double> nd(0.0, 1.0);
                        // logical A [mn][K], B [K][mn], pieces as 16-bit values
                        std::vector<double> Am(s.mn * (size_t)K), Bm((size_t)K * s.mn);
                        std::vector<uint16_t> A((size_t)steps * 64 * 8), B((size_t)steps * 64 * 8);
                        for (int r = 0; r < s.mn; ++r)
                            for (int k = 0; k < K; ++k) {
                                double a = nd(rng), b = nd(rng);
                                if (!sign) { a = std::fabs(a); b = std::fabs(b); }
                                const uint16_t ua = to16(a, bf), ub = to16(b, bf);
                                Am[r * (size_t)K + k] = from16(ua, bf);
                                Bm[(size_t)k * s.mn + r] = from16(ub, bf);
                                int la, ea;
                                ab_pos(shape, r, k % s.kstep, la, ea);
                                A[((size_t)(k / s.kstep) * 64 + la) * 8 + ea] = ua;
                                B[((size_t)(k / s.kstep) * 64 + la) * 8 + ea] = ub;
                            }
                        std::vector<float> C(64 * 16, 0.f), D;
                        if (run(shape, bf, A, B, C, D, steps, d)) return 1;
                        for (int r = 0; r < s.mn; ++r)
                            for (int c = 0; c < s.mn; ++c) {
                                double ex = 0, mag = 0;
                                float f = 0.f;
                                for (int k = 0; k < K; ++k) {
                                    const double p = Am[r * (size_t)K + k] * Bm[(size_t)k * s.mn + c];
                                    ex += p;
                                    mag += std::fabs(p);
                                    f = std::fmaf((float)Am[r * (size_t)K + k], (float)Bm[(size_t)k * s.mn + c], f);
                                }
                                int ld, rd;
                                d_pos(shape, r, c, ld, rd);
                                const double e = (D[ld * 16 + rd] - ex) / mag, ef = (f - ex) / mag;
                                sb += e; s2 += e * e; fb += ef; f2 += ef * ef;
                                ++n;
                            }
                    }
                    printf("  %-8s K=%-5d %-14s bias %+.3e  rms %.3e   | fmaf bias %+.3e  rms %.3e\n",
                           sign ? "signed" : "positive", K, name(shape, bf), sb / n, std::sqrt(s2 / n), fb / n,
                           std::sqrt(f2 / n));
                }
    return 0;
}
