// Time the engine's fp16-weight GEMM (gsv::gemm_nt) on the shapes the engine runs:
// T2S prefill (N0 = 225 rows), batched decode (B = 64), RoBERTa (40 tokens), CN-HuBERT
// (300 frames), the packed prefill of 64 sentences (22848 rows).  Prints per-shape microseconds (hipEvents over 200 launches), the max
// error against a double-precision host GEMM on sampled entries, and a bit hash of C
// (identical hashes under GENIE_GEMM_X3=0 / 1 = bit-identical kernels).
// Build: hipcc -O3 --offload-arch=gfx950 tools/gemm_bench.cpp -Igenie_tts_amd/csrc
//        -Lgenie_tts_amd/_lib -lgenie_engine -Wl,-rpath,$PWD/genie_tts_amd/_lib -o tools/gemm_bench
#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include "kernels.h"

// sw: split fp32 weights (hi + lo planes); ps: A given as its fp16 hi / lo planes (pre-split, the
// large-M kernel only) -- its hash must equal the same shape's f32-A hash
struct Shape { const char* name; int M, N, K, mode, ksplit; int sw = 0; int ps = 0; };

static unsigned long long rng_state = 7;   // private LCG: the HIP runtime may draw from rand()
static float frand() {
    rng_state = rng_state * 6364136223846793005ull + 1442695040888963407ull;
    return (float)((rng_state >> 40) & 0xffffff) / (float)0x1000000;
}
static int irand(int n) { return (int)(frand() * n) % n; }

int main() {
    const Shape shapes[] = {
        {"prefill qkv     ", 225, 1536, 512, gsv::EPI_STORE, 1},
        {"prefill out slab", 225, 512, 512, gsv::EPI_SLAB, 4},
        {"prefill ffn1    ", 225, 2048, 512, gsv::EPI_RELU, 1},
        {"prefill ffn2 slb", 225, 512, 2048, gsv::EPI_SLAB, 8},
        {"b64 qkv slab    ", 64, 1536, 512, gsv::EPI_SLAB, 4},
        {"b64 out slab    ", 64, 512, 512, gsv::EPI_SLAB, 4},
        {"b64 ffn1 slab   ", 64, 2048, 512, gsv::EPI_SLAB, 4},
        {"roberta qkv     ", 40, 3072, 1024, gsv::EPI_STORE, 1},
        {"roberta ffn1    ", 40, 4096, 1024, gsv::EPI_GELU, 1},
        {"roberta ffn2    ", 40, 1024, 4096, gsv::EPI_STORE, 1},
        {"hubert ffn1     ", 300, 3072, 768, gsv::EPI_GELU, 1},
        {"mixed prefill   ", 2400, 1536, 512, gsv::EPI_STORE, 1},
        {"pk64 qkv        ", 22848, 1536, 512, gsv::EPI_STORE, 1},
        {"pk64 out slab   ", 22848, 512, 512, gsv::EPI_SLAB, 4},
        {"pk64 ffn1       ", 22848, 2048, 512, gsv::EPI_RELU, 1},
        {"pk64 ffn2 slab  ", 22848, 512, 2048, gsv::EPI_SLAB, 8},
        {"pk64 qkv    PS  ", 22848, 1536, 512, gsv::EPI_STORE, 1, 0, 1},
        {"pk64 ffn1   PS  ", 22848, 2048, 512, gsv::EPI_RELU, 1, 0, 1},
        {"pk64 ffn2 slb PS", 22848, 512, 2048, gsv::EPI_SLAB, 8, 0, 1},
        {"rob pk qkv  W16 ", 1100, 3072, 1024, gsv::EPI_STORE, 1, 1},
        {"rob pk ffn1 W16 ", 1100, 4096, 1024, gsv::EPI_GELU, 1, 1},
        {"rob pk ffn2 W16 ", 1100, 1024, 4096, gsv::EPI_SLAB, 8, 1},
        {"rob 22 ffn1 W16 ", 22, 4096, 1024, gsv::EPI_GELU, 1, 1},
    };
    for (const Shape& sh : shapes) {
        const int M = sh.M, N = sh.N, K = sh.K;
        // seed per shape (not per position in the list): a PS / W16 row draws the same A, W, bias
        // as the plain row of the same shape, so their hashes are comparable
        rng_state = 7ull + 1000003ull * M + 8191ull * N + 131ull * K + 17ull * sh.mode + sh.ksplit;
        std::vector<float> A((size_t)M * K), bias(N);
        std::vector<__half> W((size_t)N * K);
        for (auto& v : A) v = (frand() - 0.5f) * 2.f;
        for (auto& v : W) v = __float2half((frand() - 0.5f) * 0.1f);
        for (auto& v : bias) v = (frand() - 0.5f);
        float *dA, *dB, *dC;
        __half *dW, *dWl = nullptr;
        const size_t cElems = (size_t)M * N * sh.ksplit;
        (void)hipMalloc(&dA, A.size() * 4);
        (void)hipMalloc(&dW, W.size() * 2);
        (void)hipMalloc(&dB, N * 4);
        (void)hipMalloc(&dC, cElems * 4);
        (void)hipMemcpy(dA, A.data(), A.size() * 4, hipMemcpyHostToDevice);
        (void)hipMemcpy(dW, W.data(), W.size() * 2, hipMemcpyHostToDevice);
        std::vector<__half> Wl;
        if (sh.sw) {   // a lo plane of small values (w = hi + lo 2^-11)
            Wl.resize(W.size());
            for (auto& v : Wl) v = __float2half((frand() - 0.5f) * 0.1f);
            (void)hipMalloc(&dWl, Wl.size() * 2);
            (void)hipMemcpy(dWl, Wl.data(), Wl.size() * 2, hipMemcpyHostToDevice);
        }
        (void)hipMemcpy(dB, bias.data(), N * 4, hipMemcpyHostToDevice);
        gsv::GemmArgs g{};
        g.M = M; g.N = N; g.K = K; g.A = dA; g.lda = K; g.W = dW; g.ldw = K; g.w_f16 = 1;
        g.bias = sh.mode == gsv::EPI_SLAB ? nullptr : dB; g.C = dC; g.ldc = N; g.mode = sh.mode;
        g.ksplit = sh.ksplit; g.slab_stride = (long)M * N;
        g.Wl = dWl;
        __half *dAh = nullptr, *dAl = nullptr;
        if (sh.ps) {   // the planes the producers write: hi = fp16(a), lo = fp16(a - hi), round to nearest even
            std::vector<__half> ah(A.size()), al(A.size());
            for (size_t i = 0; i < A.size(); ++i) {
                ah[i] = __float2half(A[i]);
                al[i] = __float2half(A[i] - __half2float(ah[i]));
            }
            (void)hipMalloc(&dAh, A.size() * 2);
            (void)hipMalloc(&dAl, A.size() * 2);
            (void)hipMemcpy(dAh, ah.data(), A.size() * 2, hipMemcpyHostToDevice);
            (void)hipMemcpy(dAl, al.data(), A.size() * 2, hipMemcpyHostToDevice);
            g.Ah = dAh; g.Al = dAl;
        }
        gsv::gemm_nt(g, 0);
        (void)hipDeviceSynchronize();
        hipEvent_t e0, e1;
        (void)hipEventCreate(&e0);
        (void)hipEventCreate(&e1);
        const int iters = M > 4096 ? 20 : 200;
        (void)hipEventRecord(e0, 0);
        for (int i = 0; i < iters; ++i) gsv::gemm_nt(g, 0);
        (void)hipEventRecord(e1, 0);
        (void)hipEventSynchronize(e1);
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, e0, e1);
        std::vector<float> C(cElems);
        (void)hipMemcpy(C.data(), dC, cElems * 4, hipMemcpyDeviceToHost);
        // sampled check against a double-precision host GEMM
        double maxerr = 0.0;
        for (int t = 0; t < 256; ++t) {
            const int m = irand(M), n = irand(N);
            double ref = 0.0;
            for (int k = 0; k < K; ++k) {
                double wv = (double)__half2float(W[(size_t)n * K + k]);
                if (sh.sw) wv += (double)__half2float(Wl[(size_t)n * K + k]) / 2048.0;
                ref += (double)A[(size_t)m * K + k] * wv;
            }
            double got = 0.0;
            if (sh.mode == gsv::EPI_SLAB) {
                for (int z = 0; z < sh.ksplit; ++z) got += C[(size_t)z * M * N + (size_t)m * N + n];
            } else {
                ref += bias[n];
                if (sh.mode == gsv::EPI_RELU) ref = ref > 0 ? ref : 0;
                if (sh.mode == gsv::EPI_GELU) ref = 0.5 * ref * (1.0 + erf(ref / sqrt(2.0)));
                got = C[(size_t)m * N + n];
            }
            maxerr = fmax(maxerr, fabs(got - ref));
        }
        unsigned long long hsh = 1469598103934665603ull;
        for (size_t i = 0; i < cElems; ++i) {
            unsigned u;
            memcpy(&u, &C[i], 4);
            hsh = (hsh ^ u) * 1099511628211ull;
        }
        const double wbytes = (double)N * K * 2, abytes = (double)M * K * 4;
        const double us = ms * 1000.0 / iters;
        printf("%s M=%5d N=%5d K=%5d split=%2d: %8.2f us  (%6.0f GB/s of W+A)  maxerr %.2e  hash %016llx\n", sh.name,
               M, N, K, sh.ksplit, us, (wbytes + abytes) / (us * 1e3), maxerr, hsh);
        (void)hipFree(dA); (void)hipFree(dW); (void)hipFree(dB); (void)hipFree(dC);
        if (dWl) (void)hipFree(dWl);
        if (dAh) { (void)hipFree(dAh); (void)hipFree(dAl); }
    }
    return 0;
}
