// XCD-local vs cross-XCD all-to-all hand-off (the decode's hop A / hop B shape):
// 16 producer workgroups publish 512 tagged 8-byte granules each; 16 consumer
// workgroups sweep them (thread t polls granule t of every producer, 16 loads), then
// publish their own 512 granules, which the producers sweep: one iteration = 2 hops.
//   config 0: the 32 workgroups on ONE XCD (blocks b % 8 == 0), sc1 stores + sc1 loads
//   config 1: the same workgroups, PLAIN stores + sc1 loads (lines kept in the XCD L2)
//   config 2: 32 workgroups spread over the 8 XCDs (blocks 0..31), sc1 stores (today's decode)
// Build: hipcc -O3 --offload-arch=gfx950 tools/xcd_handoff.hip -o tools/xcd_handoff
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef unsigned long long u64;
constexpr int NP = 16, PT = 512;

__device__ __forceinline__ u64 ld_sc1(const u64* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ void st_sc1(u64* p, u64 v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ void st_plain(u64* p, u64 v) { *(volatile u64*)p = v; }

__device__ __forceinline__ int xcc_id() {
    return __builtin_amdgcn_s_getreg((3 << 11) | 20) & 0xf;   // HW_REG_XCC_ID bits [3:0]
}

__device__ bool sweep(const u64* base, unsigned tag) {   // thread t: granule t of 16 rows of 512
    u64 g[NP];
    const int t = threadIdx.x;
#pragma unroll
    for (int k = 0; k < NP; ++k) g[k] = ld_sc1(base + k * PT + t);
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
        bool all = true;
#pragma unroll
        for (int k = 0; k < NP; ++k) all &= (unsigned)(g[k] >> 32) == tag;
        if (all) return true;
        __builtin_amdgcn_s_sleep(1);
#pragma unroll
        for (int k = 0; k < NP; ++k)
            if ((unsigned)(g[k] >> 32) != tag) g[k] = ld_sc1(base + k * PT + t);
        if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) return false;
    }
}

__global__ __launch_bounds__(PT) void k_hop(u64* A, u64* B, int iters, int config, unsigned long long* out, int* xcc,
                                            int* fail) {
    const int b = blockIdx.x, t = threadIdx.x;
    if (t == 0) xcc[b] = xcc_id();
    int member;
    if (config < 2) {
        if (b % 8 != 0) return;
        member = b / 8;            // 0..31
    } else {
        if (b >= 32) return;
        member = b;
    }
    const bool prod = member < NP;
    const int idx = member % NP;
    const bool plain = config == 1;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 1; i <= iters; ++i) {
        const u64 v = ((u64)(unsigned)i << 32) | (unsigned)(t + idx);
        if (prod) {
            if (plain) st_plain(A + idx * PT + t, v); else st_sc1(A + idx * PT + t, v);
            if (!sweep(B, i)) { *fail = 1; return; }
            __syncthreads();
        } else {
            if (!sweep(A, i)) { *fail = 1; return; }
            __syncthreads();
            if (plain) st_plain(B + idx * PT + t, v); else st_sc1(B + idx * PT + t, v);
        }
    }
    if (member == 0 && t == 0) out[config] = __builtin_amdgcn_s_memrealtime() - t0;
}

int main() {
    u64 *A, *B;
    unsigned long long* out;
    int *xcc, *fail;
    hipMalloc(&A, NP * PT * 8 * 2);
    hipMalloc(&B, NP * PT * 8 * 2);
    hipMalloc(&out, 64);
    hipMalloc(&xcc, 256 * 4);
    hipMalloc(&fail, 4);
    const int iters = 2000;
    const char* names[3] = {"one XCD, sc1 stores  ", "one XCD, plain stores", "8 XCDs,  sc1 stores  "};
    for (int rep = 0; rep < 2; ++rep)
        for (int c = 0; c < 3; ++c) {
            hipMemset(A, 0, NP * PT * 8 * 2);
            hipMemset(B, 0, NP * PT * 8 * 2);
            hipMemset(fail, 0, 4);
            hipLaunchKernelGGL(k_hop, dim3(256), dim3(PT), 0, 0, A, B, iters, c, out, xcc, fail);
            if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); return 1; }
            unsigned long long h[4];
            int f, x[256];
            hipMemcpy(h, out, 32, hipMemcpyDeviceToHost);
            hipMemcpy(&f, fail, 4, hipMemcpyDeviceToHost);
            hipMemcpy(x, xcc, 1024, hipMemcpyDeviceToHost);
            int same = 1;
            for (int m = 0; m < 32; ++m) same &= x[8 * m] == x[0];
            printf("%s: %.3f us per hop%s  (blocks b%%8==0 on one XCC: %s, xcc[0..7] = %d %d %d %d %d %d %d %d)\n",
                   names[c], h[c] * 10e-3 / (2.0 * iters), f ? "  TIMEOUT" : "", same ? "yes" : "no", x[0], x[1],
                   x[2], x[3], x[4], x[5], x[6], x[7]);
        }
    return 0;
}
