// XCD-local vs cross-XCD all-to-all hand-off (the decode's hop A / hop B shape):
// 16 producer workgroups publish 512 tagged 8-byte granules each; 16 consumer
// workgroups sweep them (thread t polls granule t of every producer, 16 loads), then
// publish their own 512 granules, which the producers sweep: one iteration = 2 hops.
//   config 0: the 32 workgroups on ONE XCD (blocks b % 8 == 0), sc1 stores + sc1 loads
//   config 1: the same workgroups, volatile stores (which compile to sc0 sc1) + sc1 loads
//   config 2: 32 workgroups spread over the 8 XCDs (blocks 0..31), sc1 stores (today's decode)
//   config 3: the config-0 workgroups, stores with no cache bits + sc0 loads (TIMES OUT: an sc0
//             load is workgroup scope and keeps hitting the CU's stale L1 line)
//   config 4: no-bit stores + "buffer_inv sc0" (drop the CU's L1) before every poll round + loads
//             with no cache bits: served by the XCD's own L2
//   config 5: no-bit stores + sc1 loads (does an agent-scope load see the XCD L2's dirty line?)
// Build: hipcc -O3 --offload-arch=gfx950 tools/xcd_handoff.hip -o tools/xcd_handoff
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef unsigned long long u64;
constexpr int NP = 16, PT = 512;

__device__ __forceinline__ u64 ld_sc1(const u64* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ void st_sc1(u64* p, u64 v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ void st_plain(u64* p, u64 v) { *(volatile u64*)p = v; }   // (emits sc0 sc1)
__device__ __forceinline__ void st_l2(u64* p, u64 v) {   // buffer_store_dwordx2, no cache bits: stays in the XCD L2
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, 8, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(__attribute__((ext_vector_type(2))) unsigned, v), r, 0, 0, 0);
}

__device__ __forceinline__ int xcc_id() {
    return __builtin_amdgcn_s_getreg((3 << 11) | 20) & 0xf;   // HW_REG_XCC_ID bits [3:0]
}

// load mode: 0 sc1 (agent scope), 1 sc0, 2 no cache bits (after a buffer_inv sc0 of the poll round)
__device__ __forceinline__ u64 ld_mode(const u64* p, int l2) {
    if (l2 == 0) return ld_sc1(p);
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, 8, 0x00020000);
    if (l2 == 1) return __builtin_bit_cast(u64, __builtin_amdgcn_raw_buffer_load_b64(r, 0, 0, 1));
    return __builtin_bit_cast(u64, __builtin_amdgcn_raw_buffer_load_b64(r, 0, 0, 0));
}
__device__ bool sweep(const u64* base, unsigned tag, int G, int l2 = 0) {   // thread t < G: granule t of 16 rows
    u64 g[NP];
    const int t = threadIdx.x;
    if (t >= G) return true;
#pragma unroll
    for (int k = 0; k < NP; ++k) g[k] = ld_mode(base + k * PT + t, l2);
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
        bool all = true;
#pragma unroll
        for (int k = 0; k < NP; ++k) all &= (unsigned)(g[k] >> 32) == tag;
        if (all) return true;
        __builtin_amdgcn_s_sleep(1);
        if (l2 == 2) asm volatile("buffer_inv sc0" ::: "memory");
#pragma unroll
        for (int k = 0; k < NP; ++k)
            if ((unsigned)(g[k] >> 32) != tag) g[k] = ld_mode(base + k * PT + t, l2);
        if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) return false;
    }
}

__global__ __launch_bounds__(PT) void k_hop(u64* A, u64* B, int iters, int config, unsigned long long* out, int* xcc,
                                            int* fail, int G) {
    const int b = blockIdx.x, t = threadIdx.x;
    if (t == 0) xcc[b] = xcc_id();
    int member;
    if (config != 2) {
        if (b % 8 != 0) return;
        member = b / 8;            // 0..31
    } else {
        if (b >= 32) return;
        member = b;
    }
    const bool prod = member < NP;
    const int idx = member % NP;
    const bool plain = config == 1, nobit = config >= 3;
    const int l2 = config == 3 ? 1 : config == 4 ? 2 : 0;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 1; i <= iters; ++i) {
        const u64 v = ((u64)(unsigned)i << 32) | (unsigned)(t + idx);
        if (prod) {
            if (t < G) { if (nobit) st_l2(A + idx * PT + t, v); else if (plain) st_plain(A + idx * PT + t, v); else st_sc1(A + idx * PT + t, v); }
            if (!sweep(B, i, G, l2)) { *fail = 1; return; }
            __syncthreads();
        } else {
            if (!sweep(A, i, G, l2)) { *fail = 1; return; }
            __syncthreads();
            if (t < G) { if (nobit) st_l2(B + idx * PT + t, v); else if (plain) st_plain(B + idx * PT + t, v); else st_sc1(B + idx * PT + t, v); }
        }
    }
    if (member == 0 && t == 0) out[config] = __builtin_amdgcn_s_memrealtime() - t0;
}

// 16-byte granules {tag, v0, v1, v2}: thread t < G polls granule t of every producer
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ u32x4 ld16(__amdgpu_buffer_rsrc_t r, int off) {   // buffer_load_dwordx4 ... sc1 (aux bit 4)
    return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off * 16, 0, 16));
}
__device__ __forceinline__ void st16(u32x4* p, u32x4 v) {
    asm volatile("global_store_dwordx4 %0, %1, off sc1" :: "v"(p), "v"(v) : "memory");
}
__device__ bool sweep16(const u32x4* base, unsigned tag, int G) {
    const int t = threadIdx.x;
    if (t >= G) return true;
    u32x4 g[NP];
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, 0x7fffffff, 0x00020000);
#pragma unroll
    for (int k = 0; k < NP; ++k) g[k] = ld16(r, k * PT + t);
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
        bool all = true;
#pragma unroll
        for (int k = 0; k < NP; ++k) all &= g[k].x == tag;
        if (all) return true;
        __builtin_amdgcn_s_sleep(1);
#pragma unroll
        for (int k = 0; k < NP; ++k)
            if (g[k].x != tag) g[k] = ld16(r, k * PT + t);
        if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) return false;
    }
}
__global__ __launch_bounds__(PT) void k_hop16(u32x4* A, u32x4* B, int iters, unsigned long long* out, int* fail, int G) {
    const int b = blockIdx.x, t = threadIdx.x;
    if (b >= 32) return;
    const bool prod = b < NP;
    const int idx = b % NP;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 1; i <= iters; ++i) {
        const u32x4 v = {(unsigned)i, (unsigned)t, (unsigned)idx, 7u};
        if (prod) {
            if (t < G) st16(A + idx * PT + t, v);
            if (!sweep16(B, i, G)) { *fail = 1; return; }
            __syncthreads();
        } else {
            if (!sweep16(A, i, G)) { *fail = 1; return; }
            __syncthreads();
            if (t < G) st16(B + idx * PT + t, v);
        }
    }
    if (b == 0 && t == 0) out[3] = __builtin_amdgcn_s_memrealtime() - t0;
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
    const char* names[6] = {"one XCD, sc1 stores  ", "one XCD, volatile st ", "8 XCDs,  sc1 stores  ",
                            "one XCD, no-bit st + sc0 ld", "one XCD, no-bit st + L1 inv + no-bit ld",
                            "one XCD, no-bit st + sc1 ld"};
    for (int G : {512, 256, 32, 1})
        for (int c = 0; c < 6; ++c) {
            if (c == 3) continue;   // times out (see the header)
            hipMemset(A, 0, NP * PT * 8 * 2);
            hipMemset(B, 0, NP * PT * 8 * 2);
            hipMemset(fail, 0, 4);
            hipLaunchKernelGGL(k_hop, dim3(256), dim3(PT), 0, 0, A, B, iters, c, out, xcc, fail, G);
            if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); return 1; }
            unsigned long long h[8];
            int f, x[256];
            hipMemcpy(h, out, 64, hipMemcpyDeviceToHost);
            hipMemcpy(&f, fail, 4, hipMemcpyDeviceToHost);
            hipMemcpy(x, xcc, 1024, hipMemcpyDeviceToHost);
            int same = 1;
            for (int m = 0; m < 32; ++m) same &= x[8 * m] == x[0];
            printf("G=%3d granules/producer (%5.1f KB swept per consumer) %s: %.3f us per hop%s%s\n", G,
                   G * 16 * 8 / 1024.0, names[c], h[c] * 10e-3 / (2.0 * iters), f ? "  TIMEOUT" : "",
                   same ? "" : "  (placement not XCD-grouped)");
        }
    u32x4 *A16, *B16;
    hipMalloc(&A16, NP * PT * 16 * 2);
    hipMalloc(&B16, NP * PT * 16 * 2);
    for (int G : {171, 128, 64}) {
        hipMemset(A16, 0, NP * PT * 16 * 2);
        hipMemset(B16, 0, NP * PT * 16 * 2);
        hipMemset(fail, 0, 4);
        hipLaunchKernelGGL(k_hop16, dim3(256), dim3(PT), 0, 0, A16, B16, iters, out, fail, G);
        if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); return 1; }
        unsigned long long h[4];
        int f;
        hipMemcpy(h, out, 32, hipMemcpyDeviceToHost);
        hipMemcpy(&f, fail, 4, hipMemcpyDeviceToHost);
        printf("16-B granules G=%3d per producer (%5.1f KB swept per consumer) 8 XCDs sc1: %.3f us per hop%s\n", G,
               G * 16 * 16 / 1024.0, h[3] * 10e-3 / (2.0 * iters), f ? "  TIMEOUT" : "");
    }
    return 0;
}
