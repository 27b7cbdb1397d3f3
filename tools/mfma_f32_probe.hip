// Does v_mfma_f32_32x32x2f32 compute a sequential fma chain?  For random operands with a
// wide exponent spread, one MFMA step D = C + A(32x2) B(2x32) is compared per element with
//   H1 fma(a1, b1, fma(a0, b0, c))   H2 fma(a0, b0, fma(a1, b1, c))
//   H3 c + (a0 b0 + a1 b1) rounded once (double)   H4 (a0 b0 + a1 b1 rounded) + c
// Build: hipcc -O3 --offload-arch=gfx950 tools/mfma_f32_probe.hip -o tools/mfma_f32_probe
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>
typedef float f32x16 __attribute__((ext_vector_type(16)));

// one wave: A[32][2], B[2][32], C[32][32] -> D (row-major 32x32).  Lane l: A row l%32,
// k l/32; B col l%32, k l/32; accumulator element i: row 8(i/4) + 4(l/32) + i%4, col l%32.
__global__ void k_probe(const float* A, const float* B, const float* C, float* D, int steps) {
    const int l = threadIdx.x, col = l & 31, hk = l >> 5;
    f32x16 acc;
    for (int i = 0; i < 16; ++i) acc[i] = C[(8 * (i / 4) + 4 * hk + (i & 3)) * 32 + col];
    for (int s = 0; s < steps; ++s) {
        const float a = A[s * 64 + col * 2 + hk];   // A_s[row col][k hk]
        const float b = B[s * 64 + hk * 32 + col];  // B_s[k hk][col]
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
    }
    for (int i = 0; i < 16; ++i) D[(8 * (i / 4) + 4 * hk + (i & 3)) * 32 + col] = acc[i];
}

int main() {
    const int steps = 4, trials = 200;
    std::mt19937 g(7);
    std::uniform_real_distribution<float> u(-1.f, 1.f);
    std::uniform_int_distribution<int> e(-30, 30);
    long n = 0, h1 = 0, h2 = 0, h3 = 0, h4 = 0;
    float *dA, *dB, *dC, *dD;
    hipMalloc(&dA, steps * 64 * 4); hipMalloc(&dB, steps * 64 * 4); hipMalloc(&dC, 1024 * 4); hipMalloc(&dD, 1024 * 4);
    for (int t = 0; t < trials; ++t) {
        std::vector<float> A(steps * 64), B(steps * 64), C(1024), D(1024);
        for (auto& x : A) x = std::ldexp(u(g), e(g) / 6);
        for (auto& x : B) x = std::ldexp(u(g), e(g) / 6);
        for (auto& x : C) x = std::ldexp(u(g), e(g) / 3);
        hipMemcpy(dA, A.data(), A.size() * 4, hipMemcpyHostToDevice);
        hipMemcpy(dB, B.data(), B.size() * 4, hipMemcpyHostToDevice);
        hipMemcpy(dC, C.data(), C.size() * 4, hipMemcpyHostToDevice);
        hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, 0, dA, dB, dC, dD, steps);
        hipMemcpy(D.data(), dD, D.size() * 4, hipMemcpyDeviceToHost);
        for (int r = 0; r < 32; ++r)
            for (int c = 0; c < 32; ++c) {
                float x1 = C[r * 32 + c], x2 = x1, x3 = x1, x4 = x1;
                for (int s = 0; s < steps; ++s) {
                    const float a0 = A[s * 64 + r * 2], a1 = A[s * 64 + r * 2 + 1];
                    const float b0 = B[s * 64 + c], b1 = B[s * 64 + 32 + c];
                    x1 = std::fmaf(a1, b1, std::fmaf(a0, b0, x1));
                    x2 = std::fmaf(a0, b0, std::fmaf(a1, b1, x2));
                    x3 = (float)((double)x3 + ((double)a0 * b0 + (double)a1 * b1));
                    x4 = (float)((float)((double)a0 * b0 + (double)a1 * b1) + x4);
                }
                const float d = D[r * 32 + c];
                ++n; h1 += d == x1; h2 += d == x2; h3 += d == x3; h4 += d == x4;
            }
    }
    std::printf("{\"elements\": %ld, \"seq_fma_k0_first\": %ld, \"seq_fma_k1_first\": %ld, \"one_rounding\": %ld, \"dot2_then_add\": %ld}\n",
                n, h1, h2, h3, h4);
    return 0;
}
