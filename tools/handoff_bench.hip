// Hand-off latency microbenchmark (MI355X): ping-pong of a tagged 8-byte granule
// between two workgroups (placed on different XCDs by blockIdx round-robin), and a
// 1 -> N broadcast / N -> 1 gather, for the granule protocol t2s_persist.hip uses.
// Build: hipcc -O3 --offload-arch=gfx950 tools/handoff_bench.hip -o tools/handoff_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef unsigned long long u64;

__device__ __forceinline__ u64 ld_rlx(const u64* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ void st_rlx(u64* p, u64 v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

template <int SLEEP>
__device__ __forceinline__ bool wait_tag(const u64* p, unsigned tag) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (unsigned it = 0;; ++it) {
        if ((unsigned)(ld_rlx(p) >> 32) == tag) return true;
        if (SLEEP) __builtin_amdgcn_s_sleep(SLEEP);
        if ((it & 255) == 255 && __builtin_amdgcn_s_memrealtime() - t0 > 100000000ull) return false;
    }
}

// mode 0: ping-pong between block 0 and block `peer` (one lane each)
template <int SLEEP>
__global__ void k_pingpong(u64* buf, int iters, int peer, unsigned long long* out, int* fail) {
    if (threadIdx.x != 0) return;
    const int b = blockIdx.x;
    if (b != 0 && b != peer) return;
    u64* ping = buf;        // written by 0
    u64* pong = buf + 16;   // written by peer
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 1; i <= iters; ++i) {
        if (b == 0) {
            st_rlx(ping, ((u64)i << 32) | i);
            if (!wait_tag<SLEEP>(pong, i)) { *fail = 1; return; }
        } else {
            if (!wait_tag<SLEEP>(ping, i)) { *fail = 1; return; }
            st_rlx(pong, ((u64)i << 32) | i);
        }
    }
    if (b == 0) out[0] = __builtin_amdgcn_s_memrealtime() - t0;
}

// mode 1: round of a 512-granule vector: block 0 publishes 512 granules (one per
// thread), every other block (nblk-1) sweeps them all (one per thread) and then
// publishes its own ack granule; block 0 sweeps the acks.  Per iteration time.
__global__ void k_bcast(u64* vec, u64* acks, int iters, unsigned long long* out, int* fail) {
    const int b = blockIdx.x, t = threadIdx.x, nb = gridDim.x;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 1; i <= iters; ++i) {
        if (b == 0) {
            st_rlx(vec + t, ((u64)i << 32) | t);
            for (int k = t + 1; k < nb; k += blockDim.x)
                if (!wait_tag<1>(acks + k * 16, i)) { *fail = 1; return; }
            __syncthreads();
        } else {
            if (!wait_tag<1>(vec + t, i)) { *fail = 1; return; }
            __syncthreads();
            if (t == 0) st_rlx(acks + b * 16, ((u64)i << 32));
        }
    }
    if (b == 0 && t == 0) out[0] = __builtin_amdgcn_s_memrealtime() - t0;
}

int main() {
    u64* buf;
    unsigned long long* out;
    int* fail;
    hipMalloc(&buf, 1 << 20);
    hipMalloc(&out, 64);
    hipMalloc(&fail, 4);
    const int iters = 2000;
    for (int peer : {1, 8, 3}) {
        for (int sleep : {0, 1}) {
            hipMemset(buf, 0, 1 << 20);
            hipMemset(fail, 0, 4);
            if (sleep) hipLaunchKernelGGL(k_pingpong<1>, dim3(16), dim3(64), 0, 0, buf, iters, peer, out, fail);
            else hipLaunchKernelGGL(k_pingpong<0>, dim3(16), dim3(64), 0, 0, buf, iters, peer, out, fail);
            unsigned long long t = 0;
            int f = 0;
            hipMemcpy(&t, out, 8, hipMemcpyDeviceToHost);
            hipMemcpy(&f, fail, 4, hipMemcpyDeviceToHost);
            printf("pingpong peer=%d (xcd %s) sleep=%d: %.3f us per round trip%s\n", peer,
                   peer % 8 == 0 ? "same" : "other", sleep, t * 10e-3 / iters, f ? " FAILED" : "");
        }
    }
    for (int nblk : {2, 17, 65, 241}) {
        hipMemset(buf, 0, 1 << 20);
        hipMemset(fail, 0, 4);
        hipLaunchKernelGGL(k_bcast, dim3(nblk), dim3(512), 0, 0, buf, buf + 4096, 500, out, fail);
        unsigned long long t = 0;
        int f = 0;
        hipMemcpy(&t, out, 8, hipMemcpyDeviceToHost);
        hipMemcpy(&f, fail, 4, hipMemcpyDeviceToHost);
        printf("512-granule broadcast + ack gather, %d consumers: %.3f us per round%s\n", nblk - 1, t * 10e-3 / 500,
               f ? " FAILED" : "");
    }
    return 0;
}
