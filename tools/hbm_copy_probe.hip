// Sweep of device-copy shapes for the achievable-HBM probe (gsv_debug_hbm_copy): float4
// grid-stride, U float4 per thread in flight, optional non-temporal loads / stores, G blocks
// per CU.  Prints GB/s of read + write bytes for a 1 GiB copy (mean of 10 after a warm-up).
// Build: hipcc -O3 --offload-arch=gfx950 tools/hbm_copy_probe.hip -o /tmp/hbm_copy_probe
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f4 __attribute__((ext_vector_type(4)));

template <int U, bool NT>
__global__ __launch_bounds__(256) void k_copy(const f4* __restrict__ src, f4* __restrict__ dst, long n) {
    const long stride = (long)gridDim.x * 256 * U;
    for (long base = (long)blockIdx.x * 256 * U + threadIdx.x; base < n; base += stride) {
        f4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long i = base + (long)u * 256;
            if (i < n) v[u] = NT ? __builtin_nontemporal_load(src + i) : src[i];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long i = base + (long)u * 256;
            if (i < n) {
                if (NT) __builtin_nontemporal_store(v[u], dst + i);
                else dst[i] = v[u];
            }
        }
    }
}

template <int U, bool NT>
static void run(const f4* s, f4* d, long n, int cus, int g) {
    const dim3 grid(cus * g);
    hipLaunchKernelGGL((k_copy<U, NT>), grid, dim3(256), 0, 0, s, d, n);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0, 0);
    for (int i = 0; i < 10; ++i) hipLaunchKernelGGL((k_copy<U, NT>), grid, dim3(256), 0, 0, s, d, n);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    printf("U=%d NT=%d blocks/CU=%2d: %7.0f GB/s\n", U, (int)NT, g, 2.0 * n * 16 * 10 / (ms * 1e-3) / 1e9);
}

int main() {
    const long bytes = 1L << 30, n = bytes / 16;
    f4 *s, *d;
    if (hipMalloc(&s, bytes) != hipSuccess || hipMalloc(&d, bytes) != hipSuccess) return 1;
    hipMemset(s, 0, bytes);
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    for (int g : {4, 8, 16, 32}) {
        run<1, false>(s, d, n, cus, g);
        run<4, false>(s, d, n, cus, g);
        run<4, true>(s, d, n, cus, g);
        run<8, true>(s, d, n, cus, g);
    }
    hipFree(s);
    hipFree(d);
    return 0;
}
