// Persistent decode: the whole AR loop of the stage decoder
// (t2s_stage_decoder_fp32.onnx, loop Inference.py:95-106) in ONE launch.
//
// Why: at batch 1 a decode step is ~150 MB of fp16 weights (≈25 µs of HBM time)
// spread over 24 layers of tiny dependent GEMVs.  As separate launches every
// layer pays three kernel boundaries plus each kernel's own dependent prologue
// (measured: 15.4 µs per layer).  Here every workgroup keeps a FIXED role for the
// whole generation and the two all-reduces a post-norm layer needs are
// hand-offs inside the launch:
//
//   attention role (16·B workgroups, one per (head, sequence)):
//     x_l = LN2_{l-1}(h1_{l-1} + b2 + ΣFFN_{l-1})   (layer 0: E_audio[tok] + α·pe[n])
//     q,k,v of the head (stage#43-51 per layer) -> K/V row appended to the cache
//     -> attention over [0, kv] (stage#84-96) -> out-proj slice (WoT rows of the head)
//     -> int64 fixed-point atomic adds into accA[s][l][b] -> arrival counter
//   FFN role (64 workgroups, 32 hidden units each):
//     h1_l = LN1_l(x_l + bo + ΣaccA) -> relu(W1 slice) -> W2 split-K slice
//     -> fixed-point adds into accF[s][l][b] -> arrival counter
//   after layer 23 the FFN role computes x_24 and the logits (ar_predict_layer,
//   16 rows per workgroup, write-through stores) -> counter; the attention
//   workgroup (head 0, b) runs the sampler (sampler.h, K10) and publishes the token
//   as a tagged 8-byte granule that every workgroup polls.
//
// Each role also computes the other role's LayerNorm for itself (from the same
// immutable hand-off buffers), so no residual vector is ever published: the only
// cross-workgroup data are the fixed-point accumulators, the logits and the token
// granules.  Every hand-off buffer has a unique address per (step, layer) and is
// zeroed by a memset before the launch, so a consumer can never hit a stale line;
// counters are polled with relaxed agent-scope (sc1) loads and payloads read with
// sc1 loads after a workgroup barrier (MI355X_MICROARCH.md hand-off table, row 3;
// producers drain with s_waitcnt vmcnt(0) before their counter add).  Integer
// accumulation is associative, so results do not depend on arrival order.
//
// Weights of the NEXT layer (and the K/V rows already in the cache) are loaded
// into registers right after a phase's output is published, i.e. while the
// workgroup waits for its next input: the weight stream is off the critical path.
//
// Every spin is bounded (s_memrealtime); a timeout sets the error word and every
// workgroup leaves.  The grid (16·B + 64 ≤ 192 workgroups, one per CU by LDS) is
// checked against the CU count on the host.
#include "common.h"
#include "kernels.h"
#include "sampler.h"
#include <hip/hip_ext.h>

namespace gsv {

namespace {
constexpr int PT = 512;            // threads per workgroup (8 waves)
constexpr int PWV = PT / 64;
constexpr int KU = 6;              // K/V rows per 8-lane group per pass: 64 groups -> 384 keys
constexpr int KVL = 64 * KU;       // K/V rows staged in LDS (LDS-DMA) ahead of the hand-off
constexpr int NFB = 64;            // FFN workgroups (32 hidden units each)
constexpr unsigned long long SPIN_TICKS = 300000000ull;   // 3 s of the 100 MHz clock

__device__ __forceinline__ int ld_rlx(const int* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ long long ld_rlx64(const long long* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long ld_rlxu64(const unsigned long long* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_rlxf(const float* p) {
    return __uint_as_float(__hip_atomic_load(reinterpret_cast<const unsigned*>(p), __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ void st_wt(float* p, float v) {   // write-through (sc1) store
    __hip_atomic_store(reinterpret_cast<unsigned*>(p), __float_as_uint(v), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// Loads through global (address space 1) pointers: the layer table holds generic
// pointers, which would otherwise become flat loads (counted in lgkmcnt too, so
// every LDS wait would also drain the weight prefetch).
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

// One lane: wait until *p >= target.  False on timeout or when another workgroup failed.
__device__ bool spin_ge(const int* p, int target, int* err, int code) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (unsigned it = 0;; ++it) {
        if (ld_rlx(p) >= target) return true;
        if ((it & 63) == 63) {
            if (ld_rlx(err) != 0) return false;
            if (__builtin_amdgcn_s_memrealtime() - t0 > SPIN_TICKS) {
                atomicCAS(err, 0, code);
                return false;
            }
        }
        __builtin_amdgcn_s_sleep(1);
    }
}

struct Ws {   // hand-off workspace addressing (all zeroed before the launch)
    long long* accA; long long* accF; float* lg; int* cnt; unsigned long long* gran;
    int B;
    __device__ long long* A(int s, int l, int b) const { return accA + ((long)(s * 24 + l) * B + b) * 512; }
    __device__ long long* F(int s, int l, int b) const { return accF + ((long)(s * 24 + l) * B + b) * 512; }
    __device__ float* L(int s, int b) const { return lg + ((long)s * B + b) * PERSIST_LGS; }
    __device__ int* cA(int s, int l) const { return cnt + ((long)s * PERSIST_CNT_LINES + 2 * l) * 32; }
    __device__ int* cF(int s, int l) const { return cnt + ((long)s * PERSIST_CNT_LINES + 2 * l + 1) * 32; }
    __device__ int* cL(int s) const { return cnt + ((long)s * PERSIST_CNT_LINES + 48) * 32; }
    __device__ unsigned long long* G(int s, int b) const { return gran + (long)s * 16 + b; }
};

// LayerNorm statistics of NB rows of 512 values, one value per thread per row
// (Chan et al. pairwise merge of (mean, M2)), one LDS exchange.
template <int NB>
__device__ __forceinline__ void ln_stats(const float (&v)[NB], float (&mean)[NB], float (&den)[NB], float* red) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int b = 0; b < NB; ++b) {
        float mu = v[b], m2 = 0.f, n = 1.f;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const float mu_o = __shfl_xor(mu, o, 64);
            const float m2_o = __shfl_xor(m2, o, 64);
            const float dl = mu_o - mu;
            m2 = m2 + m2_o + dl * dl * (n * 0.5f);
            mu = mu + dl * 0.5f;
            n *= 2.f;
        }
        if (lane == 0) { red[(w * NB + b) * 2] = mu; red[(w * NB + b) * 2 + 1] = m2; }
    }
    __syncthreads();
#pragma unroll
    for (int b = 0; b < NB; ++b) {
        float mu = red[b * 2], m2 = red[b * 2 + 1], n = 64.f;
#pragma unroll
        for (int ww = 1; ww < PWV; ++ww) {
            const float mo = red[(ww * NB + b) * 2], m2o = red[(ww * NB + b) * 2 + 1];
            const float dl = mo - mu;
            const float nt = n + 64.f;
            mu = mu + dl * (64.f / nt);
            m2 = m2 + m2o + dl * dl * (n * 64.f / nt);
            n = nt;
        }
        mean[b] = mu;
        den[b] = sqrtf(m2 * (1.0f / 512.0f) + 1e-5f);
    }
    __syncthreads();   // red reusable
}

__device__ __forceinline__ float dot8(const uint4 w, const float4 x0, const float4 x1) {
    float wf[8];
    h8_to_f8(w, wf);
    float s = 0.f;
    s += wf[0] * x0.x; s += wf[1] * x0.y; s += wf[2] * x0.z; s += wf[3] * x0.w;
    s += wf[4] * x1.x; s += wf[5] * x1.y; s += wf[6] * x1.z; s += wf[7] * x1.w;
    return s;
}

struct Shared {
    union {
        struct {               // attention role
            float k[KVL * 32]; // K/V rows [0, min(kv, KVL)) of the head, staged by LDS-DMA
            float v[KVL * 32];
            float x[512];      // x_l
            float h1[512];     // LN1 output (residual of the next layer)
            uint4 wo[32 * 64]; // WoT rows of the head (32 x 512 fp16), staged by LDS-DMA
        } at;
        struct {               // FFN role
            float x[8][512];   // x_l per sequence
            float h1[8][512];  // LN1 output per sequence
        } ff;
    };
    float ored[PWV][512];      // cross-wave reduction of 512-wide partials
    float qkv[96];
    float os[32];
    float fs[8][32];
    float red[2 * PWV * 8];
    float redm[PWV];
    float redl[PWV][8];
    float reda[PWV][32];
    uint32_t seen[33];
    int tok[8];
    int act;                   // bit b: sequence b still decoding
    int flag;
    SampleLds<PT> samp;
};

// Token granules of step s+1 for every sequence active in step s: new tokens and
// the active set.  Block-uniform result; false on error.
__device__ bool poll_tokens(const PersistArgs& a, const Ws& ws, int s, Shared& sh) {
    if (threadIdx.x == 0) {
        int act = sh.act, ok = 1;
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        for (int b = 0; b < a.B && ok; ++b) {
            if (!((act >> b) & 1)) continue;
            for (unsigned it = 0;; ++it) {
                const unsigned long long g = ld_rlxu64(ws.G(s + 1, b));
                if ((unsigned)(g >> 32) == (unsigned)(s + 1)) {
                    sh.tok[b] = (int)(g & 0xffff);
                    if ((g >> 16) & 1) act &= ~(1 << b);
                    break;
                }
                if ((it & 63) == 63) {
                    if (ld_rlx(a.err) != 0) { ok = 0; break; }
                    if (__builtin_amdgcn_s_memrealtime() - t0 > SPIN_TICKS) {
                        atomicCAS(a.err, 0, 3);
                        ok = 0;
                        break;
                    }
                }
                __builtin_amdgcn_s_sleep(1);
            }
        }
        sh.act = act;
        sh.flag = ok;
    }
    __syncthreads();
    const bool ok = sh.flag != 0;
    __syncthreads();
    return ok;
}

__device__ bool block_wait(const int* p, int target, int* err, int code, Shared& sh) {
    if (threadIdx.x == 0) sh.flag = spin_ge(p, target, err, code) ? 1 : 0;
    __syncthreads();
    const bool ok = sh.flag != 0;
    __syncthreads();
    return ok;
}

#define STAMP(i)                                                                          \
    do {                                                                                  \
        if (probe && threadIdx.x == 0)                                                    \
            a.trace[blockIdx.x * 8 + (i)] = __builtin_amdgcn_s_memrealtime();              \
    } while (0)

// --------------------------------------------------------------------------
// attention role: head h of sequence b
// --------------------------------------------------------------------------
__device__ void attn_role(const PersistArgs& a, const Ws& ws, int h, int b, Shared& sh) {
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform: row offsets fold into SGPR bases
    const int B = a.B, NA = 16 * B;
    const int c = lane & 7, g = (w << 3) | (lane >> 3);     // 16-B chunk of a K/V row, key group
    const long kvoff = (long)b * a.sstride + (long)h * a.tmax * 32;
    const bool sampler = h == 0;
    // entry state of sequence b
    const int ny0 = a.ny[b], kv0 = a.kvlen[b], st0 = a.steps[b];
    if (tid < 33) sh.seen[tid] = a.seen[(long)b * 33 + tid];
    if (tid == 0) {
        int act = 0;
        for (int bb = 0; bb < B; ++bb) {
            if (!a.done[bb]) act |= 1 << bb;
            sh.tok[bb] = (int)a.y[(long)bb * a.ldy + a.ny[bb] - 1];
        }
        sh.act = act;
    }
    __syncthreads();
    uint4 wq[12];
    float bqv = 0.f;
    float p_bo = 0.f, p_n1w = 0.f, p_n1b = 0.f, p_b2 = 0.f, p_n2w = 0.f, p_n2b = 0.f;
    // loads for layer l of the step whose K/V length is kv
    auto prefetch = [&](int l, int kv) {
        const PLayer& P = a.L[l];
        // wave w: q, k and v rows h*32 + 4w + r (r < 4) -- 1 KB apart, immediate offsets
        const __half* wb = P.w_in + (long)(h * 32 + 4 * w) * 512;
#pragma unroll
        for (int m = 0; m < 3; ++m)
#pragma unroll
            for (int r = 0; r < 4; ++r) wq[m * 4 + r] = ldg16(wb + (long)m * 512 * 512 + r * 512, lane * 8);
        // lane m*4+r (< 12) holds the bias of row (m, r); read back with readlane
        bqv = lane < 12 ? ldg(P.b_in, (lane >> 2) * 512 + h * 32 + 4 * w + (lane & 3)) : 0.f;
        // WoT rows h*32 .. h*32+31 (contiguous 32 KB) -> LDS, one 1 KB row per wave instruction
        const __half* ob = P.woT + (long)(h * 32 + 4 * w) * 512;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            __builtin_amdgcn_global_load_lds(ob + i * 512 + lane * 8, sh.at.wo + (4 * w + i) * 64, 16, 0, 0);
        // K/V rows [0, min(kv, KVL)) -> LDS, 1 KB (8 rows) per wave instruction.  Rows of the
        // last chunk past kv are read (allocated: tmax >= kv + 16) and masked in the math.
        const float* K = a.kc[l] + kvoff;
        const float* V = a.vc[l] + kvoff;
        const int nch = (min(kv, KVL) + 7) >> 3;
        for (int i = w; i < nch; i += PWV) {
            __builtin_amdgcn_global_load_lds(K + (long)i * 256 + lane * 4, sh.at.k + i * 256, 16, 0, 0);
            __builtin_amdgcn_global_load_lds(V + (long)i * 256 + lane * 4, sh.at.v + i * 256, 16, 0, 0);
        }
        p_bo = ldg(P.b_out, tid); p_n1w = ldg(P.n1w, tid); p_n1b = ldg(P.n1b, tid);
        if (l > 0) {
            const PLayer& Q = a.L[l - 1];
            p_b2 = ldg(Q.b2, tid); p_n2w = ldg(Q.n2w, tid); p_n2b = ldg(Q.n2b, tid);
        }
    };
    int n_exec = 0, last_stop = 0;
    bool alive = true;
    int kv = kv0;
    if ((sh.act >> b) & 1) prefetch(0, kv);
    for (int s = 0; s < a.smax && alive; ++s) {
        const int act = sh.act;
        if (act == 0) break;
        const bool mine = (act >> b) & 1;
        if (!mine) {
            // idle sequence: arrive on every attention counter of the step
            if (tid == 0)
                for (int l = 0; l < 24; ++l) __hip_atomic_fetch_add(ws.cA(s, l), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (!poll_tokens(a, ws, s, sh)) { alive = false; break; }
            continue;
        }
        for (int l = 0; l < 24; ++l) {
            const bool probe = a.trace && s == 8 && l == 12;
            const PLayer& P = a.L[l];
            // ---- layer input x_l
            float xv;
            if (l == 0) {
                const int n = ny0 + s;
                xv = ldg_h(a.emb, (long)sh.tok[b] * 512 + tid) + ldg(a.alpha, 0) * ldg(a.pe, (long)n * 512 + tid);
            } else {
                if (!block_wait(ws.cF(s, l - 1), NFB, a.err, 1, sh)) { alive = false; break; }
                STAMP(0);
                const float acc = from_fx(ld_rlx64(ws.F(s, l - 1, b) + tid));
                float v[1] = {sh.at.h1[tid] + (p_b2 + acc)}, mean[1], den[1];
                ln_stats<1>(v, mean, den, sh.red);
                xv = (v[0] - mean[0]) / den[0] * p_n2w + p_n2b;
            }
            sh.at.x[tid] = xv;
            __syncthreads();
            STAMP(1);
            // ---- q, k, v of head h (12 rows per wave)
            {
                const float4 x0 = *reinterpret_cast<const float4*>(&sh.at.x[lane * 8]);
                const float4 x1 = *reinterpret_cast<const float4*>(&sh.at.x[lane * 8 + 4]);
#pragma unroll
                for (int r = 0; r < 12; ++r) {
                    const float sum = wave_sum_dpp(dot8(wq[r], x0, x1));
                    const float bias = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(bqv), r));
                    if (lane == 0) sh.qkv[(r >> 2) * 32 + 4 * w + (r & 3)] = bias + sum;
                }
            }
            __syncthreads();
            STAMP(5);
            // ---- append the new K/V row, attention over [0, kv]
            float* Kw = a.kc[l] + kvoff;
            float* Vw = a.vc[l] + kvoff;
            const float sc = a.scale;
            const float q0 = sh.qkv[4 * c] * sc, q1 = sh.qkv[4 * c + 1] * sc;
            const float q2 = sh.qkv[4 * c + 2] * sc, q3 = sh.qkv[4 * c + 3] * sc;
            const float4 knew = make_float4(sh.qkv[32 + 4 * c], sh.qkv[33 + 4 * c], sh.qkv[34 + 4 * c], sh.qkv[35 + 4 * c]);
            const float4 vnew = make_float4(sh.qkv[64 + 4 * c], sh.qkv[65 + 4 * c], sh.qkv[66 + 4 * c], sh.qkv[67 + 4 * c]);
            const int T = kv + 1;
            float mt = -INFINITY, ls = 0.f, o0 = 0.f, o1 = 0.f, o2 = 0.f, o3 = 0.f;
            for (int base = 0; base < T; base += 64 * KU) {
                float4 kk[KU], vv[KU];
                if (base == 0) {
#pragma unroll
                    for (int u = 0; u < KU; ++u) {
                        const int t = u * 64 + g;
                        kk[u] = *reinterpret_cast<const float4*>(sh.at.k + t * 32 + 4 * c);
                        vv[u] = *reinterpret_cast<const float4*>(sh.at.v + t * 32 + 4 * c);
                    }
                } else {
#pragma unroll
                    for (int u = 0; u < KU; ++u) {
                        const int t = min(base + u * 64 + g, kv - 1);
                        kk[u] = ldg16f(Kw, (long)t * 32 + 4 * c);
                        vv[u] = ldg16f(Vw, (long)t * 32 + 4 * c);
                    }
                }
                float sv[KU];
                float pm = -INFINITY;
#pragma unroll
                for (int u = 0; u < KU; ++u) {
                    const int t = base + u * 64 + g;
                    if (t == kv) { kk[u] = knew; vv[u] = vnew; }
                    float x = q0 * (kk[u].x * sc);
                    x += q1 * (kk[u].y * sc);
                    x += q2 * (kk[u].z * sc);
                    x += q3 * (kk[u].w * sc);
                    x += dpp_f<0xB1, 0xF>(x);
                    x += dpp_f<0x4E, 0xF>(x);
                    x += dpp_f<0x141, 0xF>(x);
                    const bool valid = t < T;
                    sv[u] = valid ? x : -INFINITY;
                    if (!valid) vv[u] = make_float4(0.f, 0.f, 0.f, 0.f);
                    pm = fmaxf(pm, sv[u]);
                }
                if (pm == -INFINITY) continue;
                const float mn = fmaxf(mt, pm);
                const float f = expf(mt - mn);
                float lsum = 0.f, a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
#pragma unroll
                for (int u = 0; u < KU; ++u) {
                    const float p = expf(sv[u] - mn);
                    lsum += p;
                    a0 += p * vv[u].x; a1 += p * vv[u].y; a2 += p * vv[u].z; a3 += p * vv[u].w;
                }
                ls = ls * f + lsum;
                o0 = o0 * f + a0; o1 = o1 * f + a1; o2 = o2 * f + a2; o3 = o3 * f + a3;
                mt = mn;
            }
            STAMP(6);
            {
                const float bm = wave_max(mt);
                if (lane == 0) sh.redm[w] = bm;
                __syncthreads();
                float m = sh.redm[0];
#pragma unroll
                for (int ww = 1; ww < PWV; ++ww) m = fmaxf(m, sh.redm[ww]);
                const float fsc = mt == -INFINITY ? 0.f : expf(mt - m);
                ls *= fsc; o0 *= fsc; o1 *= fsc; o2 *= fsc; o3 *= fsc;
#pragma unroll
                for (int x = 8; x < 64; x <<= 1) {
                    ls += __shfl_xor(ls, x, 64);
                    o0 += __shfl_xor(o0, x, 64);
                    o1 += __shfl_xor(o1, x, 64);
                    o2 += __shfl_xor(o2, x, 64);
                    o3 += __shfl_xor(o3, x, 64);
                }
                if (lane < 8) {
                    sh.reda[w][4 * lane] = o0; sh.reda[w][4 * lane + 1] = o1;
                    sh.reda[w][4 * lane + 2] = o2; sh.reda[w][4 * lane + 3] = o3;
                    sh.redl[w][lane] = ls;
                }
                __syncthreads();
                if (tid < 32) {
                    const float L = ((sh.redl[0][0] + sh.redl[1][0]) + (sh.redl[2][0] + sh.redl[3][0])) +
                                    ((sh.redl[4][0] + sh.redl[5][0]) + (sh.redl[6][0] + sh.redl[7][0]));
                    const float O = ((sh.reda[0][tid] + sh.reda[1][tid]) + (sh.reda[2][tid] + sh.reda[3][tid])) +
                                    ((sh.reda[4][tid] + sh.reda[5][tid]) + (sh.reda[6][tid] + sh.reda[7][tid]));
                    sh.os[tid] = O / L;
                }
                __syncthreads();
            }
            STAMP(2);
            // ---- out-projection slice of this head -> fixed-point hand-off
            {
                float r[8];
#pragma unroll
                for (int k = 0; k < 8; ++k) r[k] = 0.f;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    float wf[8];
                    h8_to_f8(sh.at.wo[(w + 8 * i) * 64 + lane], wf);
                    const float ov = sh.os[w + 8 * i];
#pragma unroll
                    for (int k = 0; k < 8; ++k) r[k] += wf[k] * ov;
                }
#pragma unroll
                for (int k = 0; k < 8; ++k) sh.ored[w][8 * lane + k] = r[k];
                __syncthreads();
                const float val = ((sh.ored[0][tid] + sh.ored[1][tid]) + (sh.ored[2][tid] + sh.ored[3][tid])) +
                                  ((sh.ored[4][tid] + sh.ored[5][tid]) + (sh.ored[6][tid] + sh.ored[7][tid]));
                // the new K/V row (read by this workgroup only, next step), then the hand-off
                if (tid < 32) Kw[(long)kv * 32 + tid] = sh.qkv[32 + tid];
                else if (tid < 64) Vw[(long)kv * 32 + tid - 32] = sh.qkv[64 + tid - 32];
                fx_add(ws.A(s, l, b) + tid, val);
                drain();
                __syncthreads();
                if (tid == 0) __hip_atomic_fetch_add(ws.cA(s, l), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            STAMP(3);
            // ---- next layer's weights and K/V rows while the others finish
            const float bo = p_bo, n1w = p_n1w, n1b = p_n1b;
            if (l < 23) prefetch(l + 1, kv);
            else prefetch(0, kv + 1);
            // ---- h1_l = LN1(x_l + bo + Σ heads) for the next layer's input (not needed after 23)
            if (l < 23) {
                if (!block_wait(ws.cA(s, l), NA, a.err, 2, sh)) { alive = false; break; }
                const float acc = from_fx(ld_rlx64(ws.A(s, l, b) + tid));
                float v[1] = {sh.at.x[tid] + (bo + acc)}, mean[1], den[1];
                ln_stats<1>(v, mean, den, sh.red);
                sh.at.h1[tid] = (v[0] - mean[0]) / den[0] * n1w + n1b;
                STAMP(4);
            }
        }
        if (!alive) break;
        // ---- sampler (head-0 workgroup of the sequence)
        if (sampler) {
            if (!block_wait(ws.cL(s), NFB, a.err, 4, sh)) { alive = false; break; }
            const float* lg = ws.L(s, b);
            const int st = st0 + s;                 // loop steps already executed
            int raw = 0;
            const int tok = sample_block<PT>([&](int i) { return ld_rlxf(lg + i); }, sh.seen, b, st + 1, a.top_k,
                                             a.temperature, a.rep_penalty, a.greedy, a.seed, 0, nullptr, &raw,
                                             sh.samp);
            if (tid == 0) {
                a.y[(long)b * a.ldy + ny0 + s] = tok;
                sh.seen[tok >> 5] |= 1u << (tok & 31);
                const int stop = (raw == 1024 || tok == 1024) ? 1 : 0;
                const int nst = st + 1;
                const bool fin = a.force_steps > 0 ? nst >= a.force_steps : (stop || nst >= a.max_steps);
                last_stop = stop;
                __hip_atomic_store(ws.G(s + 1, b),
                                   ((unsigned long long)(s + 1) << 32) | (unsigned)tok | (fin ? 1u << 16 : 0u),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        ++n_exec;
        ++kv;
        if (!poll_tokens(a, ws, s, sh)) { alive = false; break; }
    }
    // ---- write back the sequence state (head-0 workgroup)
    if (sampler && n_exec > 0) {
        __syncthreads();
        if (tid < 33) a.seen[(long)b * 33 + tid] = sh.seen[tid];
        if (tid == 0) {
            a.ny[b] = ny0 + n_exec;
            a.steps[b] = st0 + n_exec;
            a.kvlen[b] = kv0 + n_exec;
            a.done[b] = ((sh.act >> b) & 1) ? 0 : 1;
            if (a.stop_out) a.stop_out[b] = (uint8_t)last_stop;
        }
    }
}

// --------------------------------------------------------------------------
// FFN role: hidden units [32 j, 32 j + 32) for every sequence; logits rows
// [16 j, 16 j + 16) (+ row 1024 on the last workgroup)
// --------------------------------------------------------------------------
template <int NB>
__device__ void ffn_role(const PersistArgs& a, const Ws& ws, int j, Shared& sh) {
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform: row offsets fold into SGPR bases
    const int B = a.B, NA = 16 * B;
    int ny0[NB];
#pragma unroll
    for (int b = 0; b < NB; ++b) ny0[b] = b < B ? a.ny[b] : 0;
    if (tid == 0) {
        int act = 0;
        for (int bb = 0; bb < B; ++bb) {
            if (!a.done[bb]) act |= 1 << bb;
            sh.tok[bb] = (int)a.y[(long)bb * a.ldy + a.ny[bb] - 1];
        }
        sh.act = act;
    }
    __syncthreads();
    uint4 w1r[4], w2r[4];
    float b1r[4];
    float p_bo = 0.f, p_n1w = 0.f, p_n1b = 0.f, p_b2 = 0.f, p_n2w = 0.f, p_n2b = 0.f;
    auto prefetch = [&](int l) {
        const PLayer& P = a.L[l];
#pragma unroll
        for (int r = 0; r < 4; ++r)
            w1r[r] = ldg16(P.w1, (long)(j * 32 + w * 4 + r) * 512 + lane * 8);
#pragma unroll
        for (int i = 0; i < 4; ++i)
            w2r[i] = ldg16(P.w2T, (long)(j * 32 + w + 8 * i) * 512 + lane * 8);
#pragma unroll
        for (int r = 0; r < 4; ++r) b1r[r] = ldg(P.b1, j * 32 + w * 4 + r);
        p_bo = ldg(P.b_out, tid); p_n1w = ldg(P.n1w, tid); p_n1b = ldg(P.n1b, tid);
        p_b2 = ldg(P.b2, tid); p_n2w = ldg(P.n2w, tid); p_n2b = ldg(P.n2b, tid);
    };
    // logits rows of this workgroup: 2 per wave, + row 1024 on the last workgroup's wave 0
    const int lrow0 = j * 16 + 2 * w;
    const bool extra = (j == NFB - 1) && w == 0;
    bool alive = true;
    if (sh.act) prefetch(0);
    for (int s = 0; s < a.smax && alive; ++s) {
        const int act = sh.act;
        if (act == 0) break;
        // x_0 = E_audio[tok] + alpha * pe[n]
#pragma unroll
        for (int b = 0; b < NB; ++b) {
            if (b >= B || !((act >> b) & 1)) continue;
            sh.ff.x[b][tid] = ldg_h(a.emb, (long)sh.tok[b] * 512 + tid) + ldg(a.alpha, 0) * ldg(a.pe, (long)(ny0[b] + s) * 512 + tid);
        }
        for (int l = 0; l < 24; ++l) {
            const bool probe = a.trace && s == 8 && l == 12;
            // ---- wait for the attention sum of layer l, h1 = LN1(x + bo + Σ)
            if (!block_wait(ws.cA(s, l), NA, a.err, 5, sh)) { alive = false; break; }
            STAMP(0);
            {
                float v[NB], mean[NB], den[NB];
#pragma unroll
                for (int b = 0; b < NB; ++b) {
                    v[b] = 0.f;
                    if (b < B && ((act >> b) & 1)) v[b] = sh.ff.x[b][tid] + (p_bo + from_fx(ld_rlx64(ws.A(s, l, b) + tid)));
                }
                ln_stats<NB>(v, mean, den, sh.red);
#pragma unroll
                for (int b = 0; b < NB; ++b)
                    if (b < B) sh.ff.h1[b][tid] = (v[b] - mean[b]) / den[b] * p_n1w + p_n1b;
            }
            __syncthreads();
            STAMP(1);
            // ---- FFN1 rows of this slice (4 per wave), ReLU
#pragma unroll
            for (int b = 0; b < NB; ++b) {
                if (b >= B || !((act >> b) & 1)) continue;
                const float4 x0 = *reinterpret_cast<const float4*>(&sh.ff.h1[b][lane * 8]);
                const float4 x1 = *reinterpret_cast<const float4*>(&sh.ff.h1[b][lane * 8 + 4]);
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float sum = wave_sum_dpp(dot8(w1r[r], x0, x1));
                    if (lane == 0) sh.fs[b][w * 4 + r] = fmaxf(b1r[r] + sum, 0.f);
                }
            }
            __syncthreads();
            STAMP(2);
            // ---- FFN2 split-K slice -> fixed-point hand-off
            float w2f[4][8];
#pragma unroll
            for (int i = 0; i < 4; ++i) h8_to_f8(w2r[i], w2f[i]);
#pragma unroll
            for (int b = 0; b < NB; ++b) {
                if (b >= B || !((act >> b) & 1)) continue;
                float r8[8];
#pragma unroll
                for (int k = 0; k < 8; ++k) r8[k] = 0.f;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const float fv = sh.fs[b][w + 8 * i];
#pragma unroll
                    for (int k = 0; k < 8; ++k) r8[k] += w2f[i][k] * fv;
                }
#pragma unroll
                for (int k = 0; k < 8; ++k) sh.ored[w][8 * lane + k] = r8[k];
                __syncthreads();
                const float val = ((sh.ored[0][tid] + sh.ored[1][tid]) + (sh.ored[2][tid] + sh.ored[3][tid])) +
                                  ((sh.ored[4][tid] + sh.ored[5][tid]) + (sh.ored[6][tid] + sh.ored[7][tid]));
                fx_add(ws.F(s, l, b) + tid, val);
                __syncthreads();
            }
            drain();
            __syncthreads();
            if (tid == 0) __hip_atomic_fetch_add(ws.cF(s, l), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            STAMP(3);
            const float b2 = p_b2, n2w = p_n2w, n2b = p_n2b;
            uint4 wp[3];
            if (l < 23) {
                prefetch(l + 1);
            } else {
#pragma unroll
                for (int r = 0; r < 2; ++r)
                    wp[r] = ldg16(a.w_pred, (long)(lrow0 + r) * 512 + lane * 8);
                wp[2] = ldg16(a.w_pred, (long)1024 * 512 + lane * 8);
            }
            // ---- x_{l+1} = LN2(h1 + b2 + Σ FFN)
            if (!block_wait(ws.cF(s, l), NFB, a.err, 6, sh)) { alive = false; break; }
            {
                float v[NB], mean[NB], den[NB];
#pragma unroll
                for (int b = 0; b < NB; ++b) {
                    v[b] = 0.f;
                    if (b < B && ((act >> b) & 1)) v[b] = sh.ff.h1[b][tid] + (b2 + from_fx(ld_rlx64(ws.F(s, l, b) + tid)));
                }
                ln_stats<NB>(v, mean, den, sh.red);
#pragma unroll
                for (int b = 0; b < NB; ++b)
                    if (b < B) sh.ff.x[b][tid] = (v[b] - mean[b]) / den[b] * n2w + n2b;
            }
            __syncthreads();
            STAMP(4);
            if (l == 23) {
                // ---- logits rows (ar_predict_layer, no bias), write-through stores
#pragma unroll
                for (int b = 0; b < NB; ++b) {
                    if (b >= B || !((act >> b) & 1)) continue;
                    const float4 x0 = *reinterpret_cast<const float4*>(&sh.ff.x[b][lane * 8]);
                    const float4 x1 = *reinterpret_cast<const float4*>(&sh.ff.x[b][lane * 8 + 4]);
                    float* lg = ws.L(s, b);
#pragma unroll
                    for (int r = 0; r < 2; ++r) {
                        const float sum = wave_sum_dpp(dot8(wp[r], x0, x1));
                        if (lane == 0) st_wt(lg + lrow0 + r, sum);
                    }
                    if (extra) {
                        const float sum = wave_sum_dpp(dot8(wp[2], x0, x1));
                        if (lane == 0) st_wt(lg + 1024, sum);
                    }
                }
                drain();
                __syncthreads();
                if (tid == 0) __hip_atomic_fetch_add(ws.cL(s), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                prefetch(0);
            }
        }
        if (!alive) break;
        if (!poll_tokens(a, ws, s, sh)) { alive = false; break; }
    }
}

template <int NB>
__global__ __launch_bounds__(PT) void k_decode_persist(PersistArgs a) {
    __shared__ Shared sh;
    const Ws ws{a.accA, a.accF, a.lg, a.cnt, a.gran, a.B};
    const int NA = 16 * a.B;
    if ((int)blockIdx.x < NA) attn_role(a, ws, blockIdx.x & 15, blockIdx.x >> 4, sh);
    else ffn_role<NB>(a, ws, blockIdx.x - NA, sh);
}

}  // namespace

int persist_grid(int B) { return 16 * B + NFB; }

size_t persist_ws_bytes(int B, int smax, size_t* zero_bytes) {
    // [counters | granules] (zeroed) then [accA | accF] (zeroed) then logits
    const size_t cnt = (size_t)smax * PERSIST_CNT_LINES * 128;
    const size_t gran = (size_t)(smax + 1) * 16 * 8;
    const size_t acc = (size_t)smax * 24 * B * 512 * 8;
    const size_t lg = (size_t)smax * B * PERSIST_LGS * 4;
    if (zero_bytes) *zero_bytes = cnt + gran + 2 * acc + 4;   // + error word
    return cnt + gran + 2 * acc + 16 + lg;
}

void persist_bind_ws(PersistArgs& a, void* base, int B, int smax) {
    char* p = (char*)base;
    a.cnt = (int*)p;
    p += (size_t)smax * PERSIST_CNT_LINES * 128;
    a.gran = (unsigned long long*)p;
    p += (size_t)(smax + 1) * 16 * 8;
    a.accA = (long long*)p;
    p += (size_t)smax * 24 * B * 512 * 8;
    a.accF = (long long*)p;
    p += (size_t)smax * 24 * B * 512 * 8;
    a.err = (int*)p;
    p += 16;
    a.lg = (float*)p;
    a.smax = smax;
}

hipError_t decode_persist(const PersistArgs& a, hipStream_t s, hipEvent_t start, hipEvent_t stop) {
    const dim3 g(persist_grid(a.B)), blk(PT);
    if (a.B <= 1) hipExtLaunchKernelGGL(k_decode_persist<1>, g, blk, 0, s, start, stop, 0, a);
    else if (a.B <= 2) hipExtLaunchKernelGGL(k_decode_persist<2>, g, blk, 0, s, start, stop, 0, a);
    else if (a.B <= 4) hipExtLaunchKernelGGL(k_decode_persist<4>, g, blk, 0, s, start, stop, 0, a);
    else hipExtLaunchKernelGGL(k_decode_persist<8>, g, blk, 0, s, start, stop, 0, a);
    return hipGetLastError();
}

}  // namespace gsv
