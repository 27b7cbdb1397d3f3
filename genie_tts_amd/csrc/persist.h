// Device helpers of the persistent decode kernel (t2s_persist1.hip, B = 1 and its
// multi-sequence form): tagged-granule hand-offs, global-address-space loads,
// ILP DPP reductions and the graph-order LayerNorm statistics.
//
// Hand-offs are 8-byte {tag, value} granules written by ONE write-through (sc1)
// store and read by relaxed agent-scope (sc1) loads that re-poll until the tag
// matches (MI355X_MICROARCH.md, hand-offs R2: the data is the flag; no fence, no
// counter, one round trip).
#pragma once
#include "common.h"

namespace gsv {
namespace pk {

typedef unsigned long long u64;
constexpr unsigned long long SPIN_TICKS = 300000000ull;   // 3 s of the 100 MHz clock

__device__ __forceinline__ int ld_rlx(const int* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// The engine's stop word (gsv_request_stop): host-coherent pinned memory, read at system
// scope (a PCIe round trip, so the decode kernels read it off their critical path)
__device__ __forceinline__ int ld_stop(const int* p) {
    return p ? __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) : 0;
}
__device__ __forceinline__ u64 ld_rlxu64(const u64* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// one write-through store of {tag, value}
__device__ __forceinline__ void st_gran(u64* p, unsigned tag, float v) {
    __hip_atomic_store(p, ((u64)tag << 32) | __float_as_uint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Loads through global (address space 1) pointers: the layer table holds generic
// pointers, which would otherwise become flat loads (counted in lgkmcnt too).
#define GPTR(T, p) ((const __attribute__((address_space(1))) T*)(p))
template <typename T>
__device__ __forceinline__ T ldg(const T* base, long idx) { return GPTR(T, base)[idx]; }
__device__ __forceinline__ float ldg_h(const __half* base, long idx) {
    return __half2float(__ushort_as_half(*GPTR(unsigned short, base + idx)));
}
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 ldg16(const __half* base, long idx) {   // 8 halves at base[idx]
    const u32x4_t v = *GPTR(u32x4_t, base + idx);   // native vector: no generic-ref copy constructor
    return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ float4 ldg16f(const float* base, long idx) {
    const f32x4_t v = *GPTR(f32x4_t, base + idx);
    return make_float4(v.x, v.y, v.z, v.w);
}

// One lane waits for its granule.  ok := false on timeout or when another
// workgroup failed (the caller leaves after a block-wide check).
__device__ __forceinline__ float wait_gran(const u64* p, unsigned tag, int* err, bool& ok,
                                           unsigned long long ticks = SPIN_TICKS) {
    u64 g = ld_rlxu64(p);
    if ((unsigned)(g >> 32) == tag) return __uint_as_float((unsigned)g);
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (unsigned it = 1;; ++it) {
        __builtin_amdgcn_s_sleep(1);
        g = ld_rlxu64(p);
        if ((unsigned)(g >> 32) == tag) return __uint_as_float((unsigned)g);
        if ((it & 63) == 0) {
            if (ld_rlx(err) != 0) { ok = false; return 0.f; }
            if (__builtin_amdgcn_s_memrealtime() - t0 > ticks) {
                atomicCAS(err, 0, 1);
                ok = false;
                return 0.f;
            }
        }
    }
}

// One lane waits for the TAG of a granule only (a wake-up sentinel: its value is
// never used), sleeping longer between polls -- cheap for the memory queues.
__device__ __forceinline__ void wait_tag_slow(const u64* p, unsigned tag, int* err, bool& ok,
                                              unsigned long long ticks = SPIN_TICKS) {
    if ((unsigned)(ld_rlxu64(p) >> 32) == tag) return;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (unsigned it = 1;; ++it) {
        __builtin_amdgcn_s_sleep(8);
        if ((unsigned)(ld_rlxu64(p) >> 32) == tag) return;
        if ((it & 15) == 0) {
            if (ld_rlx(err) != 0) { ok = false; return; }
            if (__builtin_amdgcn_s_memrealtime() - t0 > ticks) {
                atomicCAS(err, 0, 1);
                ok = false;
                return;
            }
        }
    }
}

// One lane waits for N granules p + k*stride (k < N), all N loads in flight at
// once; re-polls only the ones whose tag is still stale.
template <int N>
__device__ __forceinline__ void wait_gran_n(const u64* p, long stride, unsigned tag, float (&out)[N], int* err,
                                            bool& ok, unsigned long long ticks = SPIN_TICKS) {
    u64 g[N];
#pragma unroll
    for (int k = 0; k < N; ++k) g[k] = ld_rlxu64(p + k * stride);
    unsigned long long t0 = 0;
    for (unsigned it = 0;; ++it) {
        bool all = true;
#pragma unroll
        for (int k = 0; k < N; ++k) all &= (unsigned)(g[k] >> 32) == tag;
        if (all) break;
        if (it == 0) t0 = __builtin_amdgcn_s_memrealtime();
        __builtin_amdgcn_s_sleep(1);
#pragma unroll
        for (int k = 0; k < N; ++k)
            if ((unsigned)(g[k] >> 32) != tag) g[k] = ld_rlxu64(p + k * stride);
        if ((it & 63) == 63) {
            if (ld_rlx(err) != 0) { ok = false; break; }
            if (__builtin_amdgcn_s_memrealtime() - t0 > ticks) {
                atomicCAS(err, 0, 1);
                ok = false;
                break;
            }
        }
    }
#pragma unroll
    for (int k = 0; k < N; ++k) out[k] = __uint_as_float((unsigned)g[k]);
}

// N independent wave sums on the DPP path, interleaved (ILP); lane 63 holds the sums.
template <int N>
__device__ __forceinline__ void wave_sum_n(float (&v)[N]) {
#pragma unroll
    for (int q = 0; q < N; ++q) v[q] += dpp_f<0xB1, 0xF>(v[q]);
#pragma unroll
    for (int q = 0; q < N; ++q) v[q] += dpp_f<0x4E, 0xF>(v[q]);
#pragma unroll
    for (int q = 0; q < N; ++q) v[q] += dpp_f<0x141, 0xF>(v[q]);
#pragma unroll
    for (int q = 0; q < N; ++q) v[q] += dpp_f<0x140, 0xF>(v[q]);
#pragma unroll
    for (int q = 0; q < N; ++q) v[q] += dpp_f<0x142, 0xA>(v[q]);
#pragma unroll
    for (int q = 0; q < N; ++q) v[q] += dpp_f<0x143, 0xC>(v[q]);
}

// LayerNorm statistics of NB rows of 512 values held one per thread (PT = 512
// threads), as the graph computes them (LayerNormalization: mean, then mean of
// squared deviations): DPP wave sums (folded into v_add_f32_dpp), one LDS
// exchange per pass.  red: 2 * 8 * NB floats of LDS.
template <int NB>
__device__ __forceinline__ void ln_stats(const float (&v)[NB], float (&mean)[NB], float (&den)[NB], float* red) {
    constexpr int PWV = 8;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    float t[NB];
#pragma unroll
    for (int b = 0; b < NB; ++b) t[b] = v[b];
    wave_sum_n<NB>(t);
    if (lane == 63) {
#pragma unroll
        for (int b = 0; b < NB; ++b) red[w * NB + b] = t[b];
    }
    __syncthreads();
#pragma unroll
    for (int b = 0; b < NB; ++b) {
        float s0 = 0.f;
#pragma unroll
        for (int ww = 0; ww < PWV; ++ww) s0 += red[ww * NB + b];
        mean[b] = s0 * (1.0f / 512.0f);
        const float d = v[b] - mean[b];
        t[b] = d * d;
    }
    wave_sum_n<NB>(t);
    if (lane == 63) {
#pragma unroll
        for (int b = 0; b < NB; ++b) red[PWV * NB + w * NB + b] = t[b];
    }
    __syncthreads();
#pragma unroll
    for (int b = 0; b < NB; ++b) {
        float s1 = 0.f;
#pragma unroll
        for (int ww = 0; ww < PWV; ++ww) s1 += red[PWV * NB + ww * NB + b];
        den[b] = sqrtf(s1 * (1.0f / 512.0f) + 1e-5f);
    }
}

__device__ __forceinline__ float dot8(const uint4 w, const float4 x0, const float4 x1) {
    float wf[8];
    h8_to_f8(w, wf);
    float s = 0.f;
    s += wf[0] * x0.x; s += wf[1] * x0.y; s += wf[2] * x0.z; s += wf[3] * x0.w;
    s += wf[4] * x1.x; s += wf[5] * x1.y; s += wf[6] * x1.z; s += wf[7] * x1.w;
    return s;
}

}  // namespace pk
}  // namespace gsv
