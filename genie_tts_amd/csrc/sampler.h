// Sampler device body shared by the per-step sampler kernel (t2s.hip) and the
// persistent decode kernel (t2s_persist1.hip).
#pragma once
#include "common.h"
#include "kernels.h"

namespace gsv {

// =====================================================================
// Sampler (t2s_stage_decoder_fp32.onnx#1775-1821, first-stage #1789-1820):
// repetition penalty over the history set, /temperature, top-k threshold
// (k-th largest with multiplicity, wave extraction), softmax, argmax(p / q) with
// q = 1 (greedy) or q ~ N(0,1) (Philox + Box-Muller), stop = argmax(raw)==EOS || tok==EOS.
// =====================================================================
__device__ __forceinline__ uint32_t f2key(float f) {
    const uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float key2f(uint32_t k) {
    const uint32_t u = (k & 0x80000000u) ? (k & 0x7fffffffu) : ~k;
    return __uint_as_float(u);
}

__device__ __forceinline__ void argmax_merge(float& v, int& i, float ov, int oi) {
    if (ov > v || (ov == v && oi < i) || (v != v && ov == ov)) { v = ov; i = oi; }
}

__device__ __forceinline__ void block_argmax(float& v, int& i, float* sv, int* si) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        const float ov = __shfl_xor(v, o, 64);
        const int oi = __shfl_xor(i, o, 64);
        argmax_merge(v, i, ov, oi);
    }
    const int w = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) { sv[w] = v; si[w] = i; }
    __syncthreads();
    v = sv[0];
    i = si[0];
    const int nw = blockDim.x >> 6;
    for (int k = 1; k < nw; ++k) argmax_merge(v, i, sv[k], si[k]);
}

// Block argmax on DPP reductions: value max, then the smallest index holding it.
__device__ __forceinline__ void block_argmax_dpp(float& v, int& i, float* sv, int* si) {
    const float m = wave_max_dpp(v);
    const int mi = wave_min_dpp(v == m ? i : 0x7fffffff);
    const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) { sv[w] = m; si[w] = mi; }
    __syncthreads();
    v = sv[0];
    i = si[0];
    for (int k = 1; k < nw; ++k) argmax_merge(v, i, sv[k], si[k]);
}

// Append the token and advance the sequence state (thread 0; state read at entry).
__device__ __forceinline__ void sample_commit(const SampleArgs& a, int b, int tok, int raw_arg, int n,
                                              int steps, int kv, const uint32_t* seen_s) {
    a.y[(long)b * a.ldy + n] = tok;
    a.ny[b] = n + 1;
    a.seen[(long)b * 33 + (tok >> 5)] = seen_s[tok >> 5] | (1u << (tok & 31));
    if (!a.prefill) {
        const bool stop = raw_arg == 1024 || tok == 1024;
        if (a.stop_out) a.stop_out[b] = stop ? 1 : 0;
        const int st = steps + 1;
        a.steps[b] = st;
        a.kvlen[b] = kv + 1;
        const bool fin = seq_finished(a.force_b, b, a.force_steps, a.max_steps, st, stop);
        if (fin) a.done[b] = 1;
    }
}

#define VOCAB 1025
#define SAMPLE_MAXK 64

// One round of "extract the wave maximum, removing ONE instance": each lane holds
// a descending list h[0..n) with head index hp; returns the maximum (uniform).
template <int N>
__device__ __forceinline__ float wave_extract(const float (&h)[N], int& hp) {
    const int lane = threadIdx.x & 63;
    float head = -INFINITY;
#pragma unroll
    for (int j = 0; j < N; ++j)
        if (j == hp) head = h[j];
    const float m = wave_max_dpp(head);
    const unsigned long long hit = __ballot(head == m && hp < N);
    if (hit && lane == __ffsll((long long)hit) - 1) ++hp;
    return m;
}

template <int N>
__device__ __forceinline__ void sort_desc(float (&h)[N]) {
#pragma unroll
    for (int i = 1; i < N; ++i)
#pragma unroll
        for (int j = i; j > 0; --j)
            if (h[j] > h[j - 1]) { const float t = h[j]; h[j] = h[j - 1]; h[j - 1] = t; }
}

// Shared LDS of one block-sampler invocation (NT threads).
template <int NT>
struct SampleLds {
    float cand[NT / 64][SAMPLE_MAXK];
    float sv[16];
    int si[16];
    float thr;
};

// One sequence's sampling decision on NT threads (the whole block participates).
// ld(i) returns logit i (i < VOCAB); seen_s is the presence bitmap (33 words, LDS);
// step is the 1-based loop step fed to Philox (0 for the first stage).  Returns the
// token (uniform); *raw_out = argmax of the raw logits (stop rule).
template <int NT, typename LoadF>
__device__ int sample_block(LoadF ld, const uint32_t* seen_s, int b, int step, int top_k, float temperature,
                            float rep_penalty, int greedy, uint64_t seed, int ablate, float* logits_out,
                            int* raw_out, SampleLds<NT>& sh) {
    constexpr int SLOTS = (VOCAB + NT - 1) / NT;
    constexpr int NW = NT / 64;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    float l[SLOTS];
#pragma unroll
    for (int j = 0; j < SLOTS; ++j) {
        const int i = tid + NT * j;
        l[j] = i < VOCAB ? ld(i) : -INFINITY;
    }
    __syncthreads();   // seen_s written by the caller
    float v[SLOTS];
    float rv = -INFINITY;
    int ri = 0x7fffffff;
#pragma unroll
    for (int j = 0; j < SLOTS; ++j) {
        const int i = tid + NT * j;
        v[j] = -INFINITY;
        if (i < VOCAB) {
            if (logits_out) logits_out[i] = l[j];
            argmax_merge(rv, ri, l[j], i);
            float pen = l[j];
            if ((seen_s[i >> 5] >> (i & 31)) & 1u) pen = l[j] < 0.f ? l[j] * rep_penalty : l[j] / rep_penalty;
            v[j] = pen / temperature;
        }
    }
    block_argmax_dpp(rv, ri, sh.sv, sh.si);
    *raw_out = ri;
    if (greedy) {
        // q := 1 and softmax is monotone: argmax(p / q) is the first index of the
        // largest penalised logit; the top-k mask cannot remove the maximum.
        float gv = -INFINITY;
        int gi = 0x7fffffff;
#pragma unroll
        for (int j = 0; j < SLOTS; ++j) {
            const int i = tid + NT * j;
            if (i < VOCAB) argmax_merge(gv, gi, v[j], i);
        }
        block_argmax_dpp(gv, gi, sh.sv, sh.si);
        return gi;
    }
    if (ablate == 3) return ri;
    const int K = top_k;
    // ---- k-th largest with multiplicity: every wave extracts its own k largest (one
    // instance per round), then wave 0 extracts the k-th largest of the NW*k candidates.
    if (ablate == 0) {
        float h[SLOTS];
#pragma unroll
        for (int j = 0; j < SLOTS; ++j) h[j] = v[j];
        sort_desc(h);
        int hp = 0;
        for (int r = 0; r < K; ++r) {
            const float m = wave_extract(h, hp);
            if (lane == 0) sh.cand[w][r] = m;
        }
    }
    __syncthreads();
    if (w == 0 && ablate == 0) {
        float h[NW];
#pragma unroll
        for (int j = 0; j < NW; ++j) h[j] = lane < K ? sh.cand[j][lane] : -INFINITY;
        sort_desc(h);
        int hp = 0;
        float m = -INFINITY;
        for (int r = 0; r < K; ++r) m = wave_extract(h, hp);
        if (lane == 0) sh.thr = m;
    }
    if (ablate && tid == 0) sh.thr = -INFINITY;
    __syncthreads();
    const float thr = sh.thr;
    // ---- softmax over kept entries, then argmax(p / q)
    float lmax = -INFINITY;
#pragma unroll
    for (int j = 0; j < SLOTS; ++j) {
        v[j] = v[j] < thr ? -INFINITY : v[j];
        lmax = fmaxf(lmax, v[j]);
    }
    const float m = ablate == 2 ? 0.f : block_max_dpp(lmax, sh.sv);
    float lsum = 0.f;
#pragma unroll
    for (int j = 0; j < SLOTS; ++j) {
        v[j] = expf(v[j] - m);
        lsum += v[j];
    }
    const float sum = ablate == 2 ? 1.f : block_sum_dpp(lsum, sh.sv);
    float bv = -INFINITY;
    int bi = 0x7fffffff;
#pragma unroll
    for (int j = 0; j < SLOTS; ++j) {
        const int i = tid + NT * j;
        if (i >= VOCAB) continue;
        const float p = v[j] / sum;
        const uint4 r = philox4x32(make_uint4((uint32_t)i, (uint32_t)step, (uint32_t)b, 0x51u),
                                   make_uint2((uint32_t)seed, (uint32_t)(seed >> 32)));
        const float u1 = u01_open(r.x), u2 = u01_open(r.y);
        const float q = sqrtf(-2.0f * logf(u1)) * cospif(2.0f * u2);
        argmax_merge(bv, bi, p / q, i);
    }
    block_argmax_dpp(bv, bi, sh.sv, sh.si);
    return bi;
}

}  // namespace gsv
