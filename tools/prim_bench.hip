// Latency of the primitives the persistent decode chains (MI355X, one 512-thread
// workgroup per CU): barrier, LDS round trip, DPP reductions, global loads.
// Cycles of the shader clock (s_memtime), averaged over a loop.
// Build: hipcc -O3 --offload-arch=gfx950 tools/prim_bench.hip -o tools/prim_bench
#include <hip/hip_runtime.h>
#include <cstdio>

template <int CTRL, int ROW_MASK>
__device__ __forceinline__ float dpp_f(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(v), __float_as_int(v), CTRL, ROW_MASK, 0xF, false));
}
__device__ __forceinline__ float wsum(float v) {
    v += dpp_f<0xB1, 0xF>(v); v += dpp_f<0x4E, 0xF>(v); v += dpp_f<0x141, 0xF>(v);
    v += dpp_f<0x140, 0xF>(v); v += dpp_f<0x142, 0xA>(v); v += dpp_f<0x143, 0xC>(v);
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}

__global__ __launch_bounds__(512) void k_prims(float* g, unsigned long long* out, int iters) {
    __shared__ float lds[4096];
    const int tid = threadIdx.x;
    float acc = tid;
    unsigned long long t0, t1;
    // 1. barrier
    __syncthreads();
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) __syncthreads();
    t1 = __builtin_amdgcn_s_memtime();
    if (tid == 0) out[0] = (t1 - t0) / iters;
    // 2. LDS write -> barrier -> dependent read of another wave's value
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) {
        lds[tid] = acc;
        __syncthreads();
        acc += lds[(tid + 64) & 511];
        __syncthreads();
    }
    t1 = __builtin_amdgcn_s_memtime();
    if (tid == 0) out[1] = (t1 - t0) / iters;
    // 3. one DPP wave sum (dependent chain)
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) acc = wsum(acc) * 1e-3f;
    t1 = __builtin_amdgcn_s_memtime();
    if (tid == 0) out[2] = (t1 - t0) / iters;
    // 4. 12 interleaved DPP wave sums
    float v[12];
    for (int q = 0; q < 12; ++q) v[q] = acc + q;
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int q = 0; q < 12; ++q) v[q] += dpp_f<0xB1, 0xF>(v[q]);
#pragma unroll
        for (int q = 0; q < 12; ++q) v[q] += dpp_f<0x4E, 0xF>(v[q]);
#pragma unroll
        for (int q = 0; q < 12; ++q) v[q] += dpp_f<0x141, 0xF>(v[q]);
#pragma unroll
        for (int q = 0; q < 12; ++q) v[q] += dpp_f<0x140, 0xF>(v[q]);
#pragma unroll
        for (int q = 0; q < 12; ++q) v[q] += dpp_f<0x142, 0xA>(v[q]);
#pragma unroll
        for (int q = 0; q < 12; ++q) v[q] = (v[q] + dpp_f<0x143, 0xC>(v[q])) * 1e-3f;
    }
    t1 = __builtin_amdgcn_s_memtime();
    if (tid == 0) out[3] = (t1 - t0) / iters;
    for (int q = 0; q < 12; ++q) acc += v[q];
    // 5. dependent LDS read chain (ds_read_b32)
    lds[tid] = (float)((tid * 7) & 511);
    __syncthreads();
    int idx = tid;
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) idx = (int)lds[idx];
    t1 = __builtin_amdgcn_s_memtime();
    if (tid == 0) out[4] = (t1 - t0) / iters;
    acc += idx;
    // 6. dependent global load chain, L2-resident 16 KB
    int gi = tid;
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) gi = __float_as_int(__builtin_nontemporal_load(g + gi)) & 4095;
    t1 = __builtin_amdgcn_s_memtime();
    if (tid == 0) out[5] = (t1 - t0) / iters;
    acc += gi;
    // 7. dependent sc1 (agent) load chain on the same 16 KB
    gi = tid;
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i)
        gi = (int)(__hip_atomic_load((const unsigned*)(g + gi), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 4095u);
    t1 = __builtin_amdgcn_s_memtime();
    if (tid == 0) out[6] = (t1 - t0) / iters;
    acc += gi;
    // 8. expf
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) acc = expf(acc * -1e-3f);
    t1 = __builtin_amdgcn_s_memtime();
    if (tid == 0) out[7] = (t1 - t0) / iters;
    // 9. __syncthreads_or
    t0 = __builtin_amdgcn_s_memtime();
    int o = 0;
    for (int i = 0; i < iters; ++i) o += __syncthreads_or(acc > 1e30f);
    t1 = __builtin_amdgcn_s_memtime();
    if (tid == 0) out[8] = (t1 - t0) / iters;
    if (acc == 12345.f || o == 77) g[0] = acc;
}

int main() {
    float* g;
    unsigned long long* out;
    hipMalloc(&g, 16384 * 4);
    hipMalloc(&out, 64 * 8);
    float h[16384];
    for (int i = 0; i < 16384; ++i) { unsigned u = (unsigned)((i * 2654435761u) >> 20) & 4095u; h[i] = *reinterpret_cast<float*>(&u); }
    hipMemcpy(g, h, sizeof(h), hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_prims, dim3(1), dim3(512), 0, 0, g, out, 200);
    hipLaunchKernelGGL(k_prims, dim3(1), dim3(512), 0, 0, g, out, 200);
    unsigned long long o[16];
    hipMemcpy(o, out, sizeof(o), hipMemcpyDeviceToHost);
    const char* names[] = {"__syncthreads (8 waves)", "LDS write+barrier+read+barrier", "DPP wave sum (1 chain)",
                           "12 interleaved DPP wave sums", "dependent ds_read_b32", "dependent global load (L2)",
                           "dependent sc1 load (L2)", "expf", "__syncthreads_or"};
    for (int i = 0; i < 9; ++i) printf("%-34s %6llu cycles (%.3f us at 2.4 GHz)\n", names[i], o[i], o[i] / 2400.0);
    return 0;
}
