// Probe for the k_conv_h<1,32,1,1,4> corruption (r05): does a packed-FP32 VALU op that
// takes its low result from the HIGH half of a 64-bit source pair (op_sel:[0,1]) read
// that half correctly right after the s_waitcnt that completes the VMEM load of the pair?
//
// Each thread, per iteration: v = (0, 0); global_load_dwordx2 v <- src[i];
// s_waitcnt vmcnt(0); [s_nop NOP]; r = v_pk_mul_f32(a, v) with op_sel (mode 1) or
// without (mode 0: r = (a.x*v.x, a.y*v.y)); the result is checked against the
// host-known product and mismatches are counted (lane quarter, which half).
// Several streams run it at once, as the concurrent vocoder lanes did.
//
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/pk_opsel_probe.hip -o tools/pk_opsel_probe
// Run:   tools/pk_opsel_probe <mode 0|1> <nops 0..2> <streams> <reps>
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));   \
            exit(2);                                                                            \
        }                                                                                       \
    } while (0)

typedef float f2 __attribute__((ext_vector_type(2)));

// MFMA-heavy filler: dependent 32x32x16 f16 chains on every SIMD (the MRF convs' pipe use)
__global__ __launch_bounds__(256) void k_mfma_noise(float* out, int iters) {
    typedef _Float16 h8 __attribute__((ext_vector_type(8)));
    typedef float f16v __attribute__((ext_vector_type(16)));
    h8 a, b;
    for (int i = 0; i < 8; ++i) { a[i] = (_Float16)(threadIdx.x * 0.001f + i); b[i] = (_Float16)(1.0f / (1 + i)); }
    f16v c0 = {}, c1 = {};
    for (int it = 0; it < iters; ++it) {
        c0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(b, a, c1, 0, 0, 0);
    }
    float s = 0.f;
    for (int i = 0; i < 16; ++i) s += c0[i] + c1[i];
    if (s == 12345.f) out[threadIdx.x] = s;
}

template <int MODE, int NOPS>
__global__ __launch_bounds__(256) void k_probe(const f2* __restrict__ src, int n, int iters, unsigned* bad) {
    const int tid = blockIdx.x * 256 + threadIdx.x, lane = threadIdx.x & 63;
    f2 a;
    a.x = 1.0f + (tid & 7);
    a.y = 3.0f + (tid & 3);
    unsigned nb_lo = 0, nb_hi = 0;
    for (int it = 0; it < iters; ++it) {
        const int i = (tid * 7 + it * 131) % n;
        const f2* p = src + i;
        f2 v = {0.f, 0.f}, r;   // the load's destination holds zeros before it
        if (MODE == 5) {   // the pair comes from VALU moves, not a load
            const float sx0 = (float)(i + 1), sy0 = -(float)(i + 1);
            asm volatile("v_mov_b32 %0, %3\n\tv_mov_b32 %1, %4\n\t"
                         "v_pk_mul_f32 %2, %5, %6 op_sel:[0,1] op_sel_hi:[1,0]\n\ts_nop 2"
                         : "=&v"(v.x), "=&v"(v.y), "=&v"(r) : "v"(sx0), "v"(sy0), "v"(a), "v"(v) : "memory");
            (void)p;
            // %6 is v's old value (zeros): recompute with the real pair below
            asm volatile("v_pk_mul_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0]\n\ts_nop 2" : "=&v"(r) : "v"(a), "v"(v));
        } else if (MODE == 1) {
            if (NOPS == 0)
                asm volatile("global_load_dwordx2 %0, %1, off\n\ts_waitcnt vmcnt(0)\n\t"
                             "v_pk_mul_f32 %2, %3, %0 op_sel:[0,1] op_sel_hi:[1,0]\n\ts_nop 2"
                             : "+v"(v), "+v"(p), "=&v"(r) : "v"(a) : "memory");
            else
                asm volatile("global_load_dwordx2 %0, %1, off\n\ts_waitcnt vmcnt(0)\n\t"
                             "s_nop 1\n\tv_pk_mul_f32 %2, %3, %0 op_sel:[0,1] op_sel_hi:[1,0]\n\ts_nop 2"
                             : "+v"(v), "+v"(p), "=&v"(r) : "v"(a) : "memory");
        } else {
            if (NOPS == 0)
                asm volatile("global_load_dwordx2 %0, %1, off\n\ts_waitcnt vmcnt(0)\n\t"
                             "v_pk_mul_f32 %2, %3, %0\n\ts_nop 2"
                             : "+v"(v), "+v"(p), "=&v"(r) : "v"(a) : "memory");
            else
                asm volatile("global_load_dwordx2 %0, %1, off\n\ts_waitcnt vmcnt(0)\n\t"
                             "s_nop 1\n\tv_pk_mul_f32 %2, %3, %0\n\ts_nop 2"
                             : "+v"(v), "+v"(p), "=&v"(r) : "v"(a) : "memory");
        }
        // the source values are i + 1 (x) and -(i + 1) (y), exact in f32
        const float sx = (float)(i + 1), sy = -(float)(i + 1);
        const float want_lo = MODE != 0 ? a.x * sy : a.x * sx;
        const float want_hi = MODE != 0 ? a.y * sx : a.y * sy;
        nb_lo += r.x != want_lo;
        nb_hi += r.y != want_hi;
    }
    if (nb_lo) atomicAdd(&bad[(lane >> 4) * 2 + 0], nb_lo);
    if (nb_hi) atomicAdd(&bad[(lane >> 4) * 2 + 1], nb_hi);
}

template <int MODE, int NOPS>
void run(int streams, int reps, int noise) {
    const int n = 1 << 20;
    std::vector<f2> h(n);
    for (int i = 0; i < n; ++i) { h[i].x = (float)(i + 1); h[i].y = -(float)(i + 1); }
    f2* src;
    unsigned* bad;
    CK(hipMalloc(&src, n * sizeof(f2)));
    CK(hipMemcpy(src, h.data(), n * sizeof(f2), hipMemcpyHostToDevice));
    CK(hipMalloc(&bad, 64));
    CK(hipMemset(bad, 0, 64));
    std::vector<hipStream_t> ss(streams);
    for (auto& s : ss) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    std::vector<hipStream_t> ns(noise);
    for (auto& s : ns) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    for (int r = 0; r < reps; ++r) {
        for (auto& s : ns) hipLaunchKernelGGL(k_mfma_noise, dim3(512), dim3(256), 0, s, (float*)src, 4000);
        for (auto& s : ss) hipLaunchKernelGGL((k_probe<MODE, NOPS>), dim3(1024), dim3(256), 0, s, src, n, 64, bad);
    }
    CK(hipDeviceSynchronize());
    unsigned hb[8];
    CK(hipMemcpy(hb, bad, 32, hipMemcpyDeviceToHost));
    const double total = (double)reps * streams * 1024 * 256 * 64;
    printf("mode %d (%s) nops %d streams %d noise %d: %.3g products; wrong low/high per lane quarter:", MODE,
           MODE == 1 ? "op_sel:[0,1] op_sel_hi:[1,0]" : MODE == 5 ? "op_sel, register operand" : "plain", NOPS, streams,
           noise, total);
    for (int q = 0; q < 4; ++q) printf(" q%d %u/%u", q, hb[2 * q], hb[2 * q + 1]);
    printf("\n");
    fflush(stdout);
    CK(hipFree(src));
    CK(hipFree(bad));
    for (auto& s : ss) CK(hipStreamDestroy(s));
}


// Mode 2: the exact instruction block of k_conv_h<1,32,1,1,4>'s staging (hipcc ROCm 7.2, gfx950),
// on the same physical registers: eight x loads, leaky relu through v_pk_mul_f32 into v[4:5],
// then the input-scale loads into v[4:7] / v[8:11] (the second overlapping its address
// v[8:9]), s_waitcnt vmcnt(1) and the op_sel'd in-place v_pk_mul_f32.  Checks every x_j.
template <int CONSUMER>
__global__ __launch_bounds__(256) void k_probe_block(const float* __restrict__ xs, const float* __restrict__ isc,
                                                     int n, int iters, unsigned* bad) {
    const int tid = blockIdx.x * 256 + threadIdx.x, lane = threadIdx.x & 63;
    const unsigned long long slope = (unsigned long long)__float_as_uint(0.1f);   // s[12:13] = {slope, 0}
    unsigned nb[8] = {};
    for (int it = 0; it < iters; ++it) {
        const int i = (tid * 5 + it * 977) % n;
        const float* xp = xs + i;                       // x_j at xp + 64 j
        const int c8 = (tid >> 6) & 3;                  // the wave's channel group: scale isc[8 c8 + j]
        const unsigned long long off8 = (unsigned long long)(c8 * 8);
        float o[8];
        asm volatile(
            "v_mov_b64 v[36:37], %[off8]\n\t"
            "v_mov_b64 v[40:41], 0\n\t"
            "v_mov_b64 v[38:39], 0\n\t"
            "v_mov_b64 v[42:43], 0\n\t"
            "v_mov_b64 v[44:45], 0\n\t"
            "global_load_dword v41, %[xp], off\n\t"
            "global_load_dword v40, %[xp], off offset:256\n\t"
            "global_load_dword v38, %[xp], off offset:512\n\t"
            "global_load_dword v39, %[xp], off offset:768\n\t"
            "global_load_dword v42, %[xp], off offset:1024\n\t"
            "global_load_dword v43, %[xp], off offset:1280\n\t"
            "global_load_dword v44, %[xp], off offset:1536\n\t"
            "global_load_dword v45, %[xp], off offset:1792\n\t"
            "s_waitcnt vmcnt(0)\n\t"
            "v_pk_mul_f32 v[4:5], %[sl], v[40:41] op_sel_hi:[0,1]\n\t"
            "v_cmp_nle_f32_e32 vcc, 0, v41\n\t"
            "s_nop 1\n\t"
            "v_cndmask_b32_e32 v41, v41, v5, vcc\n\t"
            "v_cmp_nle_f32_e32 vcc, 0, v40\n\t"
            "s_nop 1\n\t"
            "v_cndmask_b32_e32 v40, v40, v4, vcc\n\t"
            "v_pk_mul_f32 v[4:5], %[sl], v[38:39] op_sel_hi:[0,1]\n\t"
            "v_cmp_nle_f32_e32 vcc, 0, v39\n\t"
            "s_nop 1\n\t"
            "v_cndmask_b32_e32 v39, v39, v5, vcc\n\t"
            "v_cmp_nle_f32_e32 vcc, 0, v38\n\t"
            "s_nop 1\n\t"
            "v_cndmask_b32_e32 v38, v38, v4, vcc\n\t"
            "v_pk_mul_f32 v[4:5], %[sl], v[42:43] op_sel_hi:[0,1]\n\t"
            "v_cmp_nle_f32_e32 vcc, 0, v43\n\t"
            "s_nop 1\n\t"
            "v_cndmask_b32_e32 v43, v43, v5, vcc\n\t"
            "v_cmp_nle_f32_e32 vcc, 0, v42\n\t"
            "s_nop 1\n\t"
            "v_cndmask_b32_e32 v42, v42, v4, vcc\n\t"
            "v_pk_mul_f32 v[4:5], %[sl], v[44:45] op_sel_hi:[0,1]\n\t"
            "v_cmp_nle_f32_e32 vcc, 0, v45\n\t"
            "s_nop 1\n\t"
            "v_cndmask_b32_e32 v45, v45, v5, vcc\n\t"
            "v_cmp_nle_f32_e32 vcc, 0, v44\n\t"
            "s_nop 1\n\t"
            "v_cndmask_b32_e32 v44, v44, v4, vcc\n\t"
            "v_lshl_add_u64 v[8:9], v[36:37], 2, %[isc]\n\t"
            "global_load_dwordx4 v[4:7], v[8:9], off\n\t"
            "s_nop 0\n\t"
            "global_load_dwordx4 v[8:11], v[8:9], off offset:16\n\t"
            "s_waitcnt vmcnt(1)\n\t"
            "v_pk_mul_f32 v[40:41], v[40:41], v[4:5] op_sel:[0,1] op_sel_hi:[1,0]\n\t"
            "v_pk_mul_f32 v[38:39], v[38:39], v[6:7]\n\t"
            "s_waitcnt vmcnt(0)\n\t"
            "v_pk_mul_f32 v[42:43], v[42:43], v[8:9]\n\t"
            "v_pk_mul_f32 v[44:45], v[44:45], v[10:11]\n\t"
            "s_waitcnt vmcnt(0)\n\t"
            "s_nop %[pad]\n\t"
            "s_cmp_eq_u32 %[cons], 0\n\t"
            "s_cbranch_scc1 1f\n\t"
            "v_max3_f32 v4, |v41|, 0, |v40|\n\t"
            "v_max3_f32 v4, v4, |v38|, |v39|\n\t"
            "v_max3_f32 v4, v4, |v42|, |v43|\n\t"
            "v_max3_f32 v4, v4, |v44|, |v45|\n\t"
            "v_cvt_f16_f32_e32 v4, v41\n\t"
            "v_cvt_f16_f32_e32 v5, v40\n\t"
            "v_cvt_f16_f32_e32 v6, v38\n\t"
            "v_cvt_f16_f32_e32 v7, v39\n\t"
            "1:\n\t"
            "s_nop 2\n\t"
            "v_mov_b32 %[o0], v41\n\tv_mov_b32 %[o1], v40\n\tv_mov_b32 %[o2], v38\n\tv_mov_b32 %[o3], v39\n\t"
            "v_mov_b32 %[o4], v42\n\tv_mov_b32 %[o5], v43\n\tv_mov_b32 %[o6], v44\n\tv_mov_b32 %[o7], v45"
            : [o0] "=&v"(o[0]), [o1] "=&v"(o[1]), [o2] "=&v"(o[2]), [o3] "=&v"(o[3]), [o4] "=&v"(o[4]),
              [o5] "=&v"(o[5]), [o6] "=&v"(o[6]), [o7] "=&v"(o[7])
            : [xp] "v"(xp), [sl] "s"(slope), [isc] "s"(isc), [off8] "v"(off8), [cons] "s"(CONSUMER > 0 ? 1 : 0),
              [pad] "i"(CONSUMER == 2 ? 7 : 0)
            : "v4", "v5", "v6", "v7", "v8", "v9", "v10", "v11", "v36", "v37", "v38", "v39", "v40", "v41",
              "v42", "v43", "v44", "v45", "vcc", "memory");
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            float x = xs[i + 64 * j];
            x = x >= 0.f ? x : x * 0.1f;
            const float want = x * isc[c8 * 8 + j];
            if (o[j] != want) {
                ++nb[j];
                if (atomicAdd(&bad[32], 1u) == 0) {   // the first wrong value: got, want, the x, lane, channel
                    bad[33] = __float_as_uint(o[j]); bad[34] = __float_as_uint(want);
                    bad[35] = __float_as_uint(x); bad[36] = lane; bad[37] = j;
                }
            }
        }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j)
        if (nb[j]) atomicAdd(&bad[(lane >> 4) * 8 + j], nb[j]);
}

template <int CONSUMER>
void run_block(int streams, int reps, int noise) {
    const int n = 1 << 20;
    std::vector<float> hx(n + 64 * 8), hs(32);
    for (size_t i = 0; i < hx.size(); ++i) hx[i] = (float)((int)(i * 2654435761u % 2001) - 1000) / 997.f;
    for (int i = 0; i < 32; ++i) hs[i] = 0.5f + i / 31.f;
    float *x, *sc;
    unsigned* bad;
    CK(hipMalloc(&x, hx.size() * 4));
    CK(hipMemcpy(x, hx.data(), hx.size() * 4, hipMemcpyHostToDevice));
    CK(hipMalloc(&sc, 32 * 4));
    CK(hipMemcpy(sc, hs.data(), 32 * 4, hipMemcpyHostToDevice));
    CK(hipMalloc(&bad, 64 * 4));
    CK(hipMemset(bad, 0, 64 * 4));
    std::vector<hipStream_t> ss(streams);
    for (auto& s : ss) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    std::vector<hipStream_t> ns(noise);
    for (auto& s : ns) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    for (int r = 0; r < reps; ++r) {
        for (auto& s : ns) hipLaunchKernelGGL(k_mfma_noise, dim3(512), dim3(256), 0, s, x, 4000);
        for (auto& s : ss) hipLaunchKernelGGL(k_probe_block<CONSUMER>, dim3(1024), dim3(256), 0, s, x, sc, n, 32, bad);
    }
    CK(hipDeviceSynchronize());
    unsigned hb[64];
    CK(hipMemcpy(hb, bad, 64 * 4, hipMemcpyDeviceToHost));
    printf("block probe, consumer %d, streams %d, MFMA noise streams %d: %.3g staged values; wrong per lane quarter x channel:",
           CONSUMER, streams, noise,
           (double)reps * streams * 1024 * 256 * 32 * 8);
    for (int q = 0; q < 4; ++q) {
        printf(" q%d [", q);
        for (int j = 0; j < 8; ++j) printf("%u%s", hb[q * 8 + j], j < 7 ? " " : "]");
    }
    if (hb[32]) {
        float g, w, xv;
        memcpy(&g, &hb[33], 4); memcpy(&w, &hb[34], 4); memcpy(&xv, &hb[35], 4);
        printf("\n   first wrong: lane %u channel %u got %g (bits %08x) want %g x %g", hb[36], hb[37], g, hb[33], w, xv);
    }
    printf("\n");
    fflush(stdout);
    CK(hipFree(x));
    CK(hipFree(sc));
    CK(hipFree(bad));
    for (auto& s : ss) CK(hipStreamDestroy(s));
    for (auto& s : ns) CK(hipStreamDestroy(s));
}

int main(int argc, char** argv) {
    const int mode = argc > 1 ? atoi(argv[1]) : 1, nops = argc > 2 ? atoi(argv[2]) : 0;
    const int streams = argc > 3 ? atoi(argv[3]) : 4, reps = argc > 4 ? atoi(argv[4]) : 20;
    // modes 2/3/4: the staging block without / with the kernel's consumer sequence / with it after 8 wait
    // states; the second argument is then the number of MFMA noise streams
    if (mode == 2) run_block<0>(streams, reps, nops);
    else if (mode == 3) run_block<1>(streams, reps, nops);
    else if (mode == 4) run_block<2>(streams, reps, nops);
    // modes 0/1/5: the second argument is the number of MFMA noise streams (no extra nops)
    else if (mode == 1) run<1, 0>(streams, reps, nops);
    else if (mode == 5) run<5, 0>(streams, reps, nops);
    else run<0, 0>(streams, reps, nops);
    return 0;
}
