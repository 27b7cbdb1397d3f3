// Shared device helpers for the gfx950 engine kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>
#include <stdint.h>

#define GSV_WAVE 64

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}

// Deterministic cross-block accumulation: partial sums converted to int64 fixed
// point (2^-32 resolution) and added with device-scope integer atomics, which
// are associative -- the sum is independent of arrival order.
__device__ __forceinline__ long long to_fx(float v) { return __double2ll_rn((double)v * 4294967296.0); }
__device__ __forceinline__ float from_fx(long long v) { return (float)((double)v * (1.0 / 4294967296.0)); }
__device__ __forceinline__ void fx_add(long long* p, float v) {
    atomicAdd(reinterpret_cast<unsigned long long*>(p), (unsigned long long)to_fx(v));
}

// Phase timestamp (100 MHz realtime counter) of block blockIdx.x, slot i (diagnostics).
#define GSV_STAMP(tr, i)                                                              \
    do {                                                                              \
        if ((tr) && threadIdx.x == 0) (tr)[blockIdx.x * 8 + (i)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)

// DPP wave reductions (VALU latency, no LDS crossbar): quad swaps, half-row and
// row mirrors, then row_bcast15 / row_bcast31; lane 63 holds the result, read
// back as a wave-uniform value.
// mov_dpp with bound_ctrl: the compiler folds it into the consuming VALU op
// (v_add_f32_dpp ...), one instruction per reduction step instead of three.
// Lanes of rows outside ROW_MASK are undefined: callers read lane 63 only.
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ float dpp_f(float v) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, ROW_MASK, 0xF, true));
}
template <typename Op>
__device__ __forceinline__ float wave_reduce_dpp(float v, Op op) {
    v = op(v, dpp_f<0xB1, 0xF>(v));    // quad_perm [1,0,3,2]
    v = op(v, dpp_f<0x4E, 0xF>(v));    // quad_perm [2,3,0,1]
    v = op(v, dpp_f<0x141, 0xF>(v));   // row_half_mirror
    v = op(v, dpp_f<0x140, 0xF>(v));   // row_mirror
    v = op(v, dpp_f<0x142, 0xA>(v));   // row_bcast:15 -> rows 1, 3
    v = op(v, dpp_f<0x143, 0xC>(v));   // row_bcast:31 -> rows 2, 3
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}
__device__ __forceinline__ float wave_max_dpp(float v) {
    return wave_reduce_dpp(v, [](float a, float b) { return fmaxf(a, b); });
}
__device__ __forceinline__ float wave_sum_dpp(float v) {
    return wave_reduce_dpp(v, [](float a, float b) { return a + b; });
}

template <int CTRL, int ROW_MASK>
__device__ __forceinline__ int dpp_i(int v) {
    return __builtin_amdgcn_update_dpp(v, v, CTRL, ROW_MASK, 0xF, false);
}
__device__ __forceinline__ int wave_min_dpp(int v) {
    v = min(v, dpp_i<0xB1, 0xF>(v));
    v = min(v, dpp_i<0x4E, 0xF>(v));
    v = min(v, dpp_i<0x141, 0xF>(v));
    v = min(v, dpp_i<0x140, 0xF>(v));
    v = min(v, dpp_i<0x142, 0xA>(v));
    v = min(v, dpp_i<0x143, 0xC>(v));
    return __builtin_amdgcn_readlane(v, 63);
}

// Block (<= 16 waves) reductions on the DPP wave forms: one LDS exchange.
__device__ __forceinline__ float block_max_dpp(float v, float* red) {
    const int w = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
    v = wave_max_dpp(v);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[w] = v;
    __syncthreads();
    float r = red[0];
    for (int i = 1; i < nw; ++i) r = fmaxf(r, red[i]);
    return r;
}
__device__ __forceinline__ float block_sum_dpp(float v, float* red) {
    const int w = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
    v = wave_sum_dpp(v);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[w] = v;
    __syncthreads();
    float r = red[0];
    for (int i = 1; i < nw; ++i) r += red[i];
    return r;
}

// Block-wide sum for blockDim.x <= 1024; `red` needs >= 16 floats of LDS.
__device__ __forceinline__ float block_sum(float v, float* red) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
    v = wave_sum(v);
    __syncthreads();
    if (lane == 0) red[w] = v;
    __syncthreads();
    float r = 0.f;
    for (int i = 0; i < nw; ++i) r += red[i];
    return r;
}

__device__ __forceinline__ float block_max(float v, float* red) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
    v = wave_max(v);
    __syncthreads();
    if (lane == 0) red[w] = v;
    __syncthreads();
    float r = -INFINITY;
    for (int i = 0; i < nw; ++i) r = fmaxf(r, red[i]);
    return r;
}

// 8 fp16 (16 B) -> 8 fp32
__device__ __forceinline__ void h8_to_f8(const uint4 u, float* f) {
    const __half2* h = reinterpret_cast<const __half2*>(&u);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        float2 t = __half22float2(h[i]);
        f[2 * i] = t.x;
        f[2 * i + 1] = t.y;
    }
}

// Philox4x32-10 (Salmon et al. 2011) for the sampler's N(0,1) draws.
__device__ __forceinline__ uint4 philox4x32(uint4 ctr, uint2 key) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint32_t hi0 = __umulhi(0xD2511F53u, ctr.x), lo0 = 0xD2511F53u * ctr.x;
        const uint32_t hi1 = __umulhi(0xCD9E8D57u, ctr.z), lo1 = 0xCD9E8D57u * ctr.z;
        ctr = make_uint4(hi1 ^ ctr.y ^ key.x, lo1, hi0 ^ ctr.w ^ key.y, lo0);
        key.x += 0x9E3779B9u;
        key.y += 0xBB67AE85u;
    }
    return ctr;
}

// (k + 1/2) / 2^23 for the top 23 bits k, exact in f32 and strictly inside (0, 1)
// (largest 1 - 2^-24): the Box-Muller radius sqrt(-2 ln u1) is never 0 and
// cos(2 pi u2) never exactly 0 (u2 != 1/4, 3/4), so q ~ N(0,1) is never +-0 and
// argmax(p / q) never meets 0/0.
__device__ __forceinline__ float u01_open(uint32_t x) {
    return ((float)(x >> 9) + 0.5f) * (1.0f / 8388608.0f);
}

// ----------------------------------------------------------------------
// LayerNorm statistics over 512 values held 2 per thread, single reduction
// (Chan et al. pairwise merge of (mean, M2)), for up to NB rows at once.
// ----------------------------------------------------------------------
template <int NB>
__device__ __forceinline__ void block_meanvar512(const float (&v0)[NB], const float (&v1)[NB], int B,
                                                 float (&mean)[NB], float (&rstd_den)[NB],
                                                 float* red /* >= 4*NB*2 */) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int b = 0; b < NB; ++b) {
        if (b >= B) break;
        float mu = 0.5f * (v0[b] + v1[b]);
        const float d = v0[b] - v1[b];
        float m2 = 0.5f * d * d;
        float n = 2.f;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const float mu_o = __shfl_xor(mu, o, 64);
            const float m2_o = __shfl_xor(m2, o, 64);
            const float dl = mu_o - mu;
            m2 = m2 + m2_o + dl * dl * (n * 0.5f);   // equal counts: nA nB / (nA+nB) = n/2
            mu = mu + dl * 0.5f;
            n *= 2.f;
        }
        if (lane == 0) { red[(w * NB + b) * 2] = mu; red[(w * NB + b) * 2 + 1] = m2; }
    }
    __syncthreads();
#pragma unroll
    for (int b = 0; b < NB; ++b) {
        if (b >= B) break;
        float mu = red[b * 2], m2 = red[b * 2 + 1], n = 128.f;
#pragma unroll
        for (int ww = 1; ww < 4; ++ww) {
            const float mo = red[(ww * NB + b) * 2], m2o = red[(ww * NB + b) * 2 + 1];
            const float dl = mo - mu;
            // merge (n, mu, m2) with (128, mo, m2o)
            const float nt = n + 128.f;
            mu = mu + dl * (128.f / nt);
            m2 = m2 + m2o + dl * dl * (n * 128.f / nt);
            n = nt;
        }
        mean[b] = mu;
        rstd_den[b] = sqrtf(m2 * (1.0f / 512.0f) + 1e-5f);
    }
}

