// Where do the workgroups of a CU-masked stream run?  Launches 256 one-per-CU
// workgroups (LDS-sized so no two share a CU) on streams masked to CU bits [0, 64),
// [64, 256) and [0, 256), and counts the distinct XCDs (HW_REG_XCC_ID) and CUs
// (HW_REG_HW_ID se/sh/cu) they landed on -- the mask-bit -> XCD mapping decides
// whether a 32-workgroup layer group of the persistent decode can own one XCD.
// Build: hipcc -O3 --offload-arch=gfx950 tools/cu_mask_probe.hip -o tools/cu_mask_probe
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>
#include <map>
#include <vector>

__global__ __launch_bounds__(64) void k_where(int* out) {
    __shared__ float pad[40000];   // 160 KB: one workgroup per CU
    const unsigned hw = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));   // HW_REG_HW_ID, bits [31:0]
    const unsigned xcc = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (3 << 11)) & 0xf;   // HW_REG_XCC_ID [3:0]
    pad[threadIdx.x] = (float)hw;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < 2000) __builtin_amdgcn_s_sleep(8);   // ~20 us
    if (threadIdx.x == 0) {
        out[2 * blockIdx.x] = (int)xcc;
        out[2 * blockIdx.x + 1] = (int)((hw >> 8) & 0xff);   // cu[11:8], sh[12], se[15:13]
        if (pad[1] == -1.f) out[0] = -2;                     // (keeps the LDS pad allocated)
    }
}

int main() {
    int* d;
    (void)hipMalloc(&d, 512 * 4);
    // (no XCD-exclusive masks: block b runs on XCD b % 8, so a mask leaving an XCD without
    // CUs could strand that XCD's blocks)
    struct M { const char* name; int lo, hi; };
    for (M m : {M{"bits [0,64)", 0, 64}, M{"bits [64,256)", 64, 256}, M{"bits [0,256)", 0, 256},
                M{"bits [0,32)", 0, 32}, M{"bits [224,256)", 224, 256}}) {
        std::vector<uint32_t> mask(8, 0u);
        int nb = 0;
        for (int i = 0; i < 256; ++i) {
            const bool on = m.lo >= 0 ? (i >= m.lo && i < m.hi) : (i % 8 >= -m.lo - 1 && i % 8 < m.hi);
            if (on) { mask[i / 32] |= 1u << (i % 32); ++nb; }
        }
        hipStream_t s;
        if (hipExtStreamCreateWithCUMask(&s, 8, mask.data()) != hipSuccess) { printf("mask stream failed\n"); return 1; }
        (void)hipMemset(d, 0xff, 512 * 4);
        hipLaunchKernelGGL(k_where, dim3(nb), dim3(64), 0, s, d);
        if (hipStreamSynchronize(s) != hipSuccess) { printf("launch failed\n"); return 1; }
        std::vector<int> h(512);
        (void)hipMemcpy(h.data(), d, 512 * 4, hipMemcpyDeviceToHost);
        std::map<int, int> per_xcc;
        std::map<std::pair<int, int>, int> cus;
        for (int b = 0; b < nb; ++b) {
            per_xcc[h[2 * b]]++;
            cus[{h[2 * b], h[2 * b + 1]}]++;
        }
        printf("%-16s %3d blocks: %zu distinct (xcc, se/sh/cu), per XCC:", m.name, nb, cus.size());
        for (auto& kv : per_xcc) printf(" %d:%d", kv.first, kv.second);
        printf("\n   block -> xcc (first 64):");
        for (int b = 0; b < nb && b < 64; ++b) printf(" %d", h[2 * b]);
        printf("\n");
        (void)hipStreamDestroy(s);
    }
    return 0;
}
