// Persistent decode: the whole AR loop of the stage decoder
// (t2s_stage_decoder_fp32.onnx, loop Inference.py:95-106) in ONE launch.
//
// Why: at batch 1 a decode step is ~150 MB of fp16 weights (≈25 µs of HBM time)
// spread over 24 layers of tiny dependent GEMVs.  As separate launches every
// layer pays kernel boundaries plus each kernel's own dependent prologue
// (measured 15.4 µs per layer).  Here every workgroup keeps a FIXED role for the
// whole generation, and the two all-reduces a post-norm layer needs are
// hand-offs inside the launch.
//
// Grid: G layer groups x (16·B attention + 64 FFN workgroups); group g owns the
// layers l ≡ g (mod G) and streams its next layer's weights (registers + LDS-DMA)
// during the G-1 layers it only tracks.  Per owned layer:
//   attention (head h, sequence b): q,k,v rows of the head (stage#43-51) ->
//     attention over [0, kv] (stage#84-96) -> out-proj slice (WoT rows of the head)
//     -> 512 partial granules PA[l][b][h][*]
//   FFN (slice j = hidden units [32 j, 32 j + 32)):
//     reduce-A: columns [8 j, 8 j + 8) of Σ_h PA (fixed order) -> granules RA
//     h1_l = LN1_l(x_l + bo + RA) -> relu(W1 slice) -> W2 slice -> partials PF[l][b][j][*]
//     reduce-F: columns [8 j, 8 j + 8) of Σ_j' PF (fixed order) -> granules RF
//   every workgroup tracks the residual stream of its sequences from RA / RF:
//     x_l = LN2_{l-1}(h1_{l-1} + b2 + RF_{l-1}),  h1_l = LN1_l(x_l + bo + RA_l)
//   after layer 23 the FFN workgroups of group 23 % G compute x_24 and the logits
//   (ar_predict_layer) as granules LG; the group-0 head-0 attention workgroup of
//   each sequence runs the sampler (sampler.h, K10) and publishes the token
//   granule TK that every workgroup polls.
//
// Hand-offs are 8-byte {tag, value} granules written by ONE write-through (sc1)
// store and read by relaxed agent-scope (sc1) loads that re-poll until the tag
// matches (MI355X_MICROARCH.md, hand-offs R2: the data is the flag; no fence, no
// counter, one round trip).  tag = (launch epoch << 12) | (step + 1), so a ring of
// RING step slots is reused without zeroing; sums are formed by a fixed set of
// lanes in a fixed order, so results do not depend on arrival order.
//
// Every spin is bounded (s_memrealtime); a timeout sets the error word and every
// workgroup leaves.  The grid (<= 256 workgroups, one per CU by LDS) is checked
// against the CU count on the host.
#include "common.h"
#include "kernels.h"
#include "sampler.h"
#include "persist.h"
#include <hip/hip_ext.h>

namespace gsv {

namespace {
using namespace pk;
constexpr int PT = 512;            // threads per workgroup (8 waves)
constexpr int PWV = PT / 64;
constexpr int KVL = 320;           // K/V rows of a head staged in LDS ahead of the hand-off
constexpr int TMAXP = 4096;        // longest key range (pe table)
constexpr int NFB = 64;            // FFN workgroups per group (32 hidden units each)
constexpr int RING = 4;            // granule ring depth (steps)

// Ring of step slots of granules (u64).  Per slot: PA [24][B][16][512],
// RA [24][B][512], PF [24][B][64][512], RF [24][B][512], LG [B][1056], TK [16].
struct Ws {
    u64* ring;
    int B;
    unsigned epoch;
    __device__ long oRA() const { return (long)24 * B * 16 * 512; }
    __device__ long oPF() const { return oRA() + (long)24 * B * 512; }
    __device__ long oRF() const { return oPF() + (long)24 * B * 64 * 512; }
    __device__ long oLG() const { return oRF() + (long)24 * B * 512; }
    __device__ long oTK() const { return oLG() + (long)B * PERSIST_LGS; }
    __device__ long slot_sz() const { return oTK() + 16; }
    __device__ u64* slot(int s) const { return ring + (long)(s % RING) * slot_sz(); }
    __device__ unsigned tag(int s) const { return (epoch << 12) | (unsigned)(s + 1); }
    __device__ u64* PA(int s, int l, int b, int h) const { return slot(s) + ((long)(l * B + b) * 16 + h) * 512; }
    __device__ u64* RA(int s, int l, int b) const { return slot(s) + oRA() + (long)(l * B + b) * 512; }
    __device__ u64* PF(int s, int l, int b, int j) const { return slot(s) + oPF() + ((long)(l * B + b) * 64 + j) * 512; }
    __device__ u64* RF(int s, int l, int b) const { return slot(s) + oRF() + (long)(l * B + b) * 512; }
    __device__ u64* LG(int s, int b) const { return slot(s) + oLG() + (long)b * PERSIST_LGS; }
    __device__ u64* TK(int s, int b) const { return slot(s) + oTK() + b; }
};

struct Shared {
    union {
        struct {                    // attention role
            float k[KVL * 32];      // K/V rows [0, min(kv, KVL)) of the head (LDS-DMA)
            float v[KVL * 32];
            float p[TMAXP];         // scores, then softmax numerators
            float x[512];           // x_l of the sequence
            float h1[512];          // LN1 output of the sequence
            float ov[16][32];       // P·V partial sums of 16 key groups
            float lg[PERSIST_LGS];  // logits (sampler)
        } at;
        struct {                    // FFN role
            float x[8][512];        // x_l per sequence
            float h1[8][512];       // LN1 output per sequence
            float rf[64][8];        // reduce-F operands
        } ff;
    };
    float qkv[96];
    float os[32];
    float fs[8][32];
    float red[2 * PWV * 8];
    int fail;                       // set once by any thread whose hand-off failed
    float wred[2][PWV];
    uint32_t seen[33];
    int tok[8];
    int act;                        // bit b: sequence b still decoding
    int flag;
    unsigned long long stamp[16];   // [0,8) 100 MHz realtime, [8,16) shader clock
    SampleLds<PT> samp;
};

// Phase stamps go to LDS (no vector-memory op that a later vmcnt wait would count)
// and are flushed once per step.
#define STAMP(i)                                                                          \
    do {                                                                                  \
        if (probe && threadIdx.x == 0) {                                                  \
            sh.stamp[i] = __builtin_amdgcn_s_memrealtime();                               \
            sh.stamp[8 + (i)] = __builtin_amdgcn_s_memtime();                             \
        }                                                                                 \
    } while (0)

// Block-wide "every hand-off of this phase arrived": one barrier; a failure is sticky.
__device__ __forceinline__ bool block_ok(bool ok, Shared& sh) {
    if (!ok) sh.fail = 1;
    __syncthreads();
    return sh.fail == 0;
}

// Token granules of step s+1 for every sequence active in step s: new tokens and
// the active set.  Block-uniform result; false on error.
__device__ bool poll_tokens(const PersistArgs& a, const Ws& ws, int s, Shared& sh) {
    if (threadIdx.x == 0) {
        int act = sh.act;
        bool ok = true;
        for (int b = 0; b < a.B && ok; ++b) {
            if (!((act >> b) & 1)) continue;
            const float v = wait_gran(ws.TK(s + 1, b), ws.tag(s + 1), a.err, ok);
            const unsigned u = __float_as_uint(v);
            sh.tok[b] = (int)(u & 0xffff);
            if ((u >> 16) & 1) act &= ~(1 << b);
        }
        sh.act = act;
        sh.flag = ok ? 1 : 0;
    }
    __syncthreads();
    const bool ok = sh.flag != 0;
    __syncthreads();
    return ok;
}

// LayerNorm parameters of one layer, one element per thread (loaded a layer ahead)
struct LnP {
    float bo, n1w, n1b, b2, n2w, n2b;
    __device__ void load(const PLayer& P, int tid) {
        bo = ldg(P.b_out, tid); n1w = ldg(P.n1w, tid); n1b = ldg(P.n1b, tid);
        b2 = ldg(P.b2, tid); n2w = ldg(P.n2w, tid); n2b = ldg(P.n2b, tid);
    }
};

// out[i] = LN(res[i] + (bias + R[b0+i])) for the tracked sequences; R from granules.
template <int NB, typename GranF>
__device__ __forceinline__ bool track_ln(GranF gran, unsigned tag, const float* res, float* out, int b0, int nb,
                                         int act, float bias, float g, float be, int* err, Shared& sh) {
    const int tid = threadIdx.x;
    bool ok = true;
    float v[NB], mean[NB], den[NB];
#pragma unroll
    for (int i = 0; i < NB; ++i) {
        v[i] = 0.f;
        if (i < nb && ((act >> (b0 + i)) & 1)) v[i] = res[i * 512 + tid] + (bias + wait_gran(gran(b0 + i) + tid, tag, err, ok));
    }
    if (!block_ok(ok, sh)) return false;
    ln_stats<NB>(v, mean, den, sh.red);
#pragma unroll
    for (int i = 0; i < NB; ++i)
        if (i < nb) out[i * 512 + tid] = (v[i] - mean[i]) / den[i] * g + be;
    return true;
}

// Scores of the general case (more than 512 keys or rows beyond the LDS stage),
// out of line so the common path keeps its registers.  Returns the lane's max.
__device__ __noinline__ float scores_general(Shared& sh, const float* Kw, int kv, int T, float q0, float q1, float q2,
                                             float q3, float sc, float4 knew, int c8, int g) {
    float lmax = -INFINITY;
    for (int base = 0; base < T; base += 512) {
        float sv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int t = base + 64 * u + g;
            float4 kr;
            if (t < kv && t < KVL) kr = *reinterpret_cast<const float4*>(sh.at.k + t * 32 + 4 * c8);
            else if (t < kv) kr = ldg16f(Kw, (long)t * 32 + 4 * c8);
            else kr = knew;
            float x = q0 * (kr.x * sc);
            x += q1 * (kr.y * sc);
            x += q2 * (kr.z * sc);
            x += q3 * (kr.w * sc);
            sv[u] = x;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) sv[u] += dpp_f<0xB1, 0xF>(sv[u]);
#pragma unroll
        for (int u = 0; u < 8; ++u) sv[u] += dpp_f<0x4E, 0xF>(sv[u]);
#pragma unroll
        for (int u = 0; u < 8; ++u) sv[u] += dpp_f<0x141, 0xF>(sv[u]);
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int t = base + 64 * u + g;
            if (t < T) {
                if (c8 == 0) sh.at.p[t] = sv[u];
                lmax = fmaxf(lmax, sv[u]);
            }
        }
    }
    return lmax;
}

// The sampler body (sampler.h) out of line: it runs once per step and would
// otherwise share the register allocation of the decode loop.
__device__ __forceinline__ int run_sampler(Shared& sh, int b, int step, int top_k, float temperature, float rep_penalty,
                                        int greedy, uint64_t seed, int* raw) {
    return sample_block<PT>([&](int i) { return sh.at.lg[i]; }, sh.seen, b, step, top_k, temperature, rep_penalty,
                            greedy, seed, 0, nullptr, raw, sh.samp);
}

// --------------------------------------------------------------------------
// One workgroup of role ATTN (head h, sequence ab) or FFN (slice j, NB >= B).
// --------------------------------------------------------------------------
template <bool ATTN, int NB>
__device__ void run_block(const PersistArgs& a, const Ws& ws, Shared& sh) {
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform: row offsets fold into SGPR bases
    const int B = a.B, G = a.groups, NA = 16 * B, per = NA + NFB;
    const int grp = blockIdx.x / per, r = blockIdx.x - grp * per;
    const int h = r & 15, ab = r >> 4, j = r - NA;
    const int b0 = ATTN ? ab : 0, nb = ATTN ? 1 : B;
    const bool sampler = ATTN && h == 0 && grp == 0;
    const bool logits_grp = !ATTN && grp == 23 % G;
    float* X = ATTN ? sh.at.x : &sh.ff.x[0][0];
    float* H1 = ATTN ? sh.at.h1 : &sh.ff.h1[0][0];
    // entry state
    int ny0[NB];
#pragma unroll
    for (int i = 0; i < NB; ++i) ny0[i] = i < nb ? a.ny[b0 + i] : 0;
    const int kv0 = ATTN ? a.kvlen[ab] : 0, st0 = ATTN ? a.steps[ab] : 0;
    if (sampler && tid < 33) sh.seen[tid] = a.seen[(long)ab * 33 + tid];
    if (tid == 0) {
        int act = 0;
        for (int bb = 0; bb < B; ++bb) {
            if (!a.done[bb]) act |= 1 << bb;
            sh.tok[bb] = (int)a.y[(long)bb * a.ldy + a.ny[bb] - 1];
        }
        sh.act = act;
        sh.fail = 0;
    }
    __syncthreads();
    const long kvoff = (long)ab * a.sstride + (long)h * a.tmax * 32;
    uint4 wq[12], wo[4];
    float bq[3] = {0.f, 0.f, 0.f};
    uint4 w1r[4], w2r[4], wp[3];
    float b1r[4];
    auto prefetch = [&](int l, int kv) {   // this workgroup's operands of layer l
        const PLayer& P = a.L[l];
        if constexpr (ATTN) {
            // wave w, lane group r4 = lane >> 4: rows (m, h*32 + 4w + r4) of W_in for m = q, k, v;
            // lane i16 = lane & 15 holds columns 8*i16 + 128*c (c < 4) of each: a row is reduced
            // over 16 lanes (4 DPP steps, no cross-row broadcast)
            const int r4 = lane >> 4, i16 = lane & 15;
            const __half* wb = P.w_in + (long)(h * 32 + 4 * w + r4) * 512 + 8 * i16;
#pragma unroll
            for (int m = 0; m < 3; ++m)
#pragma unroll
                for (int c = 0; c < 4; ++c) wq[m * 4 + c] = ldg16(wb + (long)m * 512 * 512 + c * 128, 0);
#pragma unroll
            for (int m = 0; m < 3; ++m) bq[m] = ldg(P.b_in, m * 512 + h * 32 + 4 * w + r4);
            // out-projection: thread tid owns output column tid, W_out[tid][h*32 .. h*32+32)
#pragma unroll
            for (int k = 0; k < 4; ++k) wo[k] = ldg16(P.w_out + (long)tid * 512 + h * 32 + 8 * k, 0);
            // K/V rows [0, min(kv, KVL)) -> LDS, 8 rows (1 KB) per wave instruction.  Rows of the
            // last chunk past kv are read (allocated: tmax >= kv + 16) and never used.
            const float* K = a.kc[l] + kvoff;
            const float* V = a.vc[l] + kvoff;
            const int nch = (min(kv, KVL) + 7) >> 3;
            for (int i = w; i < nch; i += PWV) {
                __builtin_amdgcn_global_load_lds(K + (long)i * 256 + lane * 4, sh.at.k + i * 256, 16, 0, 0);
                __builtin_amdgcn_global_load_lds(V + (long)i * 256 + lane * 4, sh.at.v + i * 256, 16, 0, 0);
            }
        } else {
#pragma unroll
            for (int q = 0; q < 4; ++q) w1r[q] = ldg16(P.w1 + (long)(j * 32 + w * 4 + q) * 512, lane * 8);
#pragma unroll
            for (int q = 0; q < 4; ++q) b1r[q] = ldg(P.b1, j * 32 + w * 4 + q);
            // FFN2: thread tid owns output column tid, W2[tid][j*32 .. j*32+32)
#pragma unroll
            for (int k = 0; k < 4; ++k) w2r[k] = ldg16(P.w2 + (long)tid * 2048 + j * 32 + 8 * k, 0);
        }
    };
    // logits rows (logits group): 2 per wave, + row 1024 on the last FFN workgroup's wave 0
    const int lrow0 = j * 16 + 2 * w;
    const bool extra = (j == NFB - 1) && w == 0;
    const bool mine_seq = !ATTN || ((sh.act >> ab) & 1);
    if (sh.act && mine_seq) prefetch(grp, kv0);
    LnP lp;                                   // layer l's parameters
    float pb2 = 0.f, pn2w = 0.f, pn2b = 0.f;  // layer l-1's LN2
    lp.load(a.L[0], tid);
    int n_exec = 0, last_stop = 0;
    int kv = kv0;
    for (int s = 0; s < a.smax; ++s) {
        const int act = sh.act;
        if (act == 0) break;
        const unsigned tag = ws.tag(s);
        if (ATTN && !((act >> ab) & 1)) {     // finished sequence: nothing to publish (reducers skip it)
            if (!poll_tokens(a, ws, s, sh)) return;
            continue;
        }
        // x_0 = E_audio[tok] + alpha * pe[n]
#pragma unroll
        for (int i = 0; i < NB; ++i) {
            if (i >= nb || !((act >> (b0 + i)) & 1)) continue;
            X[i * 512 + tid] = ldg_h(a.emb, (long)sh.tok[b0 + i] * 512 + tid) +
                               ldg(a.alpha, 0) * ldg(a.pe, (long)(ny0[i] + s) * 512 + tid);
        }
        for (int l = 0; l < 24; ++l) {
            const bool probe = a.trace && s == 8 && l == 12;
            const bool mine = (l - grp) % G == 0;
            // ---- x_l (layer 0: the embedding above)
            if (l > 0) {
                STAMP(0);
                if (!track_ln<NB>([&](int b) { return ws.RF(s, l - 1, b); }, tag, H1, X, b0, nb, act, pb2, pn2w,
                                  pn2b, a.err, sh))
                    return;
            }
            __syncthreads();
            STAMP(1);
            if constexpr (ATTN) if (mine) {
                // ---- q, k, v of head h: 3 rows per lane group, 16 lanes per row
                {
                    const int r4 = lane >> 4, i16 = lane & 15;
                    float acc[3] = {0.f, 0.f, 0.f};
#pragma unroll
                    for (int c = 0; c < 4; ++c) {
                        const float4 x0 = *reinterpret_cast<const float4*>(&X[8 * i16 + 128 * c]);
                        const float4 x1 = *reinterpret_cast<const float4*>(&X[8 * i16 + 128 * c + 4]);
#pragma unroll
                        for (int m = 0; m < 3; ++m) acc[m] += dot8(wq[m * 4 + c], x0, x1);
                    }
#pragma unroll
                    for (int m = 0; m < 3; ++m) acc[m] += dpp_f<0xB1, 0xF>(acc[m]);
#pragma unroll
                    for (int m = 0; m < 3; ++m) acc[m] += dpp_f<0x4E, 0xF>(acc[m]);
#pragma unroll
                    for (int m = 0; m < 3; ++m) acc[m] += dpp_f<0x141, 0xF>(acc[m]);
#pragma unroll
                    for (int m = 0; m < 3; ++m) acc[m] += dpp_f<0x140, 0xF>(acc[m]);
                    if (i16 == 0) {
#pragma unroll
                        for (int m = 0; m < 3; ++m) sh.qkv[m * 32 + 4 * w + r4] = bq[m] + acc[m];
                    }
                }
                __syncthreads();
                STAMP(2);
                // ---- scores (q*s)·(k*s) over [0, kv]: 8 lanes per key row (16 B each, conflict-free
                // LDS reads), keys t = base + 64 u + g
                float* Kw = a.kc[l] + kvoff;
                float* Vw = a.vc[l] + kvoff;
                const float sc = a.scale;
                const int T = kv + 1;
                const int c8 = lane & 7, g = (w << 3) | (lane >> 3);
                const float4 qc = *reinterpret_cast<const float4*>(sh.qkv + 4 * c8);
                const float q0 = qc.x * sc, q1 = qc.y * sc, q2 = qc.z * sc, q3 = qc.w * sc;
                float lmax = -INFINITY;
                const float4 knew = *reinterpret_cast<const float4*>(sh.qkv + 32 + 4 * c8);
                if (T <= 512 && kv <= KVL) {
                    // common case, branch-free: every cached row is in LDS, 8 keys per lane in two halves
#pragma unroll
                    for (int hf = 0; hf < 2; ++hf) {
                        float sv[4];
#pragma unroll
                        for (int u = 0; u < 4; ++u) {
                            const int t = 64 * (4 * hf + u) + g;
                            float4 kr = *reinterpret_cast<const float4*>(sh.at.k + min(t, KVL - 1) * 32 + 4 * c8);
                            if (t == kv) { kr.x = knew.x; kr.y = knew.y; kr.z = knew.z; kr.w = knew.w; }
                            float x = q0 * (kr.x * sc);
                            x += q1 * (kr.y * sc);
                            x += q2 * (kr.z * sc);
                            x += q3 * (kr.w * sc);
                            sv[u] = x;
                        }
#pragma unroll
                        for (int u = 0; u < 4; ++u) sv[u] += dpp_f<0xB1, 0xF>(sv[u]);
#pragma unroll
                        for (int u = 0; u < 4; ++u) sv[u] += dpp_f<0x4E, 0xF>(sv[u]);
#pragma unroll
                        for (int u = 0; u < 4; ++u) sv[u] += dpp_f<0x141, 0xF>(sv[u]);
#pragma unroll
                        for (int u = 0; u < 4; ++u) {
                            const int t = 64 * (4 * hf + u) + g;
                            sv[u] = t < T ? sv[u] : -INFINITY;
                            lmax = fmaxf(lmax, sv[u]);
                        }
                        if (c8 == 0) {
#pragma unroll
                            for (int u = 0; u < 4; ++u) sh.at.p[64 * (4 * hf + u) + g] = sv[u];   // p[t >= T] is never read
                        }
                    }
                } else {
                    lmax = scores_general(sh, Kw, kv, T, q0, q1, q2, q3, sc, knew, c8, g);
                }
                const float wm = wave_max_dpp(lmax);
                if (lane == 0) sh.wred[0][w] = wm;
                __syncthreads();
                float M = sh.wred[0][0];
#pragma unroll
                for (int ww = 1; ww < PWV; ++ww) M = fmaxf(M, sh.wred[0][ww]);
                float lsum = 0.f;
                for (int t = tid; t < T; t += PT) {
                    const float e = expf(sh.at.p[t] - M);
                    sh.at.p[t] = e;
                    lsum += e;
                }
                const float ws_ = wave_sum_dpp(lsum);
                if (lane == 0) sh.wred[1][w] = ws_;
                __syncthreads();
                STAMP(3);
                // ---- P·V: 16 key groups x 32 dims; LDS rows unrolled by 4 with independent sums
                {
                    const int kg = tid >> 5, d = tid & 31;
                    const int tl = min(kv, KVL);
                    float o4[4] = {0.f, 0.f, 0.f, 0.f};
                    int t = kg;
                    for (; t + 48 < tl; t += 64) {
#pragma unroll
                        for (int u = 0; u < 4; ++u) o4[u] += sh.at.p[t + 16 * u] * sh.at.v[(t + 16 * u) * 32 + d];
                    }
                    for (; t < tl; t += 16) o4[0] += sh.at.p[t] * sh.at.v[t * 32 + d];
                    for (; t < kv; t += 16) o4[1] += sh.at.p[t] * ldg(Vw, (long)t * 32 + d);
                    if (t == kv) o4[2] += sh.at.p[t] * sh.qkv[64 + d];
                    sh.at.ov[kg][d] = (o4[0] + o4[1]) + (o4[2] + o4[3]);
                }
                __syncthreads();
                if (tid < 32) {
                    float O = 0.f, L = 0.f;
#pragma unroll
                    for (int kg = 0; kg < 16; ++kg) O += sh.at.ov[kg][tid];
#pragma unroll
                    for (int ww = 0; ww < PWV; ++ww) L += sh.wred[1][ww];
                    sh.os[tid] = O / L;
                }
                __syncthreads();
                STAMP(4);
                // ---- out-projection slice of this head (column tid) -> partial granule
                {
                    float acc = 0.f;
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        const float4 oa = *reinterpret_cast<const float4*>(sh.os + 8 * k);
                        const float4 ob = *reinterpret_cast<const float4*>(sh.os + 8 * k + 4);
                        acc += dot8(wo[k], oa, ob);
                    }
                    st_gran(ws.PA(s, l, ab, h) + tid, tag, acc);
                    // the new K/V row (read by this workgroup only, next step)
                    if (tid < 32) Kw[(long)kv * 32 + tid] = sh.qkv[32 + tid];
                    else if (tid < 64) Vw[(long)kv * 32 + tid - 32] = sh.qkv[64 + tid - 32];
                }
                STAMP(5);
                __syncthreads();   // LDS operands consumed before the next layer's LDS-DMA lands
                // ---- next layer of this group (or of the next step) while the others work
                prefetch(l + G < 24 ? l + G : l + G - 24, l + G < 24 ? kv : kv + 1);
            }
            // ---- h1_l = LN1(x_l + bo + Σ_h attention partials)
            if (!ATTN && mine) {
                // owner FFN workgroups sum the 16 head partials of every column themselves
                // (fixed order, one hop), and publish the sums of their 8 columns (RA) for
                // every other workgroup that tracks the residual stream
                bool ok = true;
                float v[NB], mean[NB], den[NB];
#pragma unroll
                for (int i = 0; i < NB; ++i) {
                    v[i] = 0.f;
                    if (i < nb && ((act >> i) & 1)) {
                        float pa[16];
                        wait_gran_n<16>(ws.PA(s, l, i, 0) + tid, 512, tag, pa, a.err, ok);
                        float sum = 0.f;
#pragma unroll
                        for (int hh = 0; hh < 16; ++hh) sum += pa[hh];
                        if ((tid >> 3) == j) st_gran(ws.RA(s, l, i) + tid, tag, sum);
                        v[i] = X[i * 512 + tid] + (lp.bo + sum);
                    }
                }
                if (!block_ok(ok, sh)) return;
                STAMP(2);
                ln_stats<NB>(v, mean, den, sh.red);
#pragma unroll
                for (int i = 0; i < NB; ++i)
                    if (i < nb) H1[i * 512 + tid] = (v[i] - mean[i]) / den[i] * lp.n1w + lp.n1b;
                __syncthreads();
                STAMP(6);
            } else if (l < 23 || logits_grp) {
                // (not needed after layer 23 unless this workgroup computes the logits)
                if (!track_ln<NB>([&](int b) { return ws.RA(s, l, b); }, tag, X, H1, b0, nb, act, lp.bo, lp.n1w,
                                  lp.n1b, a.err, sh))
                    return;
                __syncthreads();
                STAMP(6);
            }
            pb2 = lp.b2; pn2w = lp.n2w; pn2b = lp.n2b;
            lp.load(a.L[l < 23 ? l + 1 : 0], tid);
            if constexpr (!ATTN) if (mine) {
                // ---- FFN1 rows of this slice (4 per wave), ReLU
#pragma unroll
                for (int i = 0; i < NB; ++i) {
                    if (i >= nb || !((act >> i) & 1)) continue;
                    const float4 x0 = *reinterpret_cast<const float4*>(&H1[i * 512 + lane * 8]);
                    const float4 x1 = *reinterpret_cast<const float4*>(&H1[i * 512 + lane * 8 + 4]);
                    float acc[4];
#pragma unroll
                    for (int q = 0; q < 4; ++q) acc[q] = dot8(w1r[q], x0, x1);
                    wave_sum_n<4>(acc);
                    if (lane == 63) {
#pragma unroll
                        for (int q = 0; q < 4; ++q) sh.fs[i][w * 4 + q] = fmaxf(b1r[q] + acc[q], 0.f);
                    }
                }
                __syncthreads();
                STAMP(3);
                // ---- FFN2 slice (column tid) -> partial granules
                {
#pragma unroll
                    for (int i = 0; i < NB; ++i) {
                        if (i >= nb || !((act >> i) & 1)) continue;
                        float acc = 0.f;
#pragma unroll
                        for (int k = 0; k < 4; ++k) {
                            const float4 fa = *reinterpret_cast<const float4*>(&sh.fs[i][8 * k]);
                            const float4 fb = *reinterpret_cast<const float4*>(&sh.fs[i][8 * k + 4]);
                            acc += dot8(w2r[k], fa, fb);
                        }
                        st_gran(ws.PF(s, l, i, j) + tid, tag, acc);
                    }
                }
                STAMP(4);
                // ---- reduce-F: columns [8j, 8j+8) of Σ_j' PF, fixed order
                {
                    const int jj = tid >> 3, c = tid & 7;
#pragma unroll
                    for (int i = 0; i < NB; ++i) {
                        if (i >= nb || !((act >> i) & 1)) continue;
                        bool ok = true;
                        sh.ff.rf[jj][c] = wait_gran(ws.PF(s, l, i, jj) + 8 * j + c, tag, a.err, ok);
                        if (!block_ok(ok, sh)) return;
                        if (tid < 8) {
                            float s4[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                            for (int q = 0; q < 64; ++q) s4[q & 3] += sh.ff.rf[q][tid];
                            const float sum = (s4[0] + s4[1]) + (s4[2] + s4[3]);
                            st_gran(ws.RF(s, l, i) + 8 * j + tid, tag, sum);
                        }
                        __syncthreads();
                    }
                }
                STAMP(5);
                if (l + G >= 24 && logits_grp) {
#pragma unroll
                    for (int q = 0; q < 2; ++q) wp[q] = ldg16(a.w_pred + (long)(lrow0 + q) * 512, lane * 8);
                    wp[2] = ldg16(a.w_pred + (long)1024 * 512, lane * 8);
                }
                prefetch(l + G < 24 ? l + G : l + G - 24, 0);
            }
        }
        if (logits_grp) {
            // ---- x_24 = LN2_23(h1_23 + b2 + RF_23), logits rows (ar_predict_layer, no bias)
            if (!track_ln<NB>([&](int b) { return ws.RF(s, 23, b); }, tag, H1, X, 0, nb, act, pb2, pn2w, pn2b, a.err,
                              sh))
                return;
            __syncthreads();
#pragma unroll
            for (int i = 0; i < NB; ++i) {
                if (i >= nb || !((act >> i) & 1)) continue;
                const float4 x0 = *reinterpret_cast<const float4*>(&X[i * 512 + lane * 8]);
                const float4 x1 = *reinterpret_cast<const float4*>(&X[i * 512 + lane * 8 + 4]);
                float acc[3];
#pragma unroll
                for (int q = 0; q < 3; ++q) acc[q] = dot8(wp[q], x0, x1);
                wave_sum_n<3>(acc);
                if (lane == 63) {
                    u64* lg = ws.LG(s, i);
                    st_gran(lg + lrow0, tag, acc[0]);
                    st_gran(lg + lrow0 + 1, tag, acc[1]);
                    if (extra) st_gran(lg + 1024, tag, acc[2]);
                }
            }
        }
        // ---- sampler (group 0, head-0 workgroup of the sequence)
        if (sampler) {
            bool ok = true;
            const u64* lgg = ws.LG(s, ab);
            for (int i = tid; i < 1025; i += PT) sh.at.lg[i] = wait_gran(lgg + i, tag, a.err, ok);
            if (!block_ok(ok, sh)) return;
            const int st = st0 + s;                 // loop steps already executed
            int raw = 0;
            const int tok = run_sampler(sh, ab, st + 1, a.top_k, a.temperature, a.rep_penalty, a.greedy, a.seed, &raw);
            if (tid == 0) {
                a.y[(long)ab * a.ldy + ny0[0] + s] = tok;
                sh.seen[tok >> 5] |= 1u << (tok & 31);
                const int stop = (raw == 1024 || tok == 1024) ? 1 : 0;
                const int nst = st + 1;
                const bool fin = seq_finished(a.force_b, ab, a.force_steps, a.max_steps, nst, stop);
                last_stop = stop;
                st_gran(ws.TK(s + 1, ab), ws.tag(s + 1), __uint_as_float((unsigned)tok | (fin ? 1u << 16 : 0u)));
            }
        }
        if (a.trace && s == 8 && tid < 16) a.trace[blockIdx.x * 16 + tid] = sh.stamp[tid];
        ++n_exec;
        ++kv;
        if (!poll_tokens(a, ws, s, sh)) return;
    }
    // ---- write back the sequence state (sampler workgroup)
    if (sampler && n_exec > 0) {
        __syncthreads();
        if (tid < 33) a.seen[(long)ab * 33 + tid] = sh.seen[tid];
        if (tid == 0) {
            a.ny[ab] = ny0[0] + n_exec;
            a.steps[ab] = st0 + n_exec;
            a.kvlen[ab] = kv0 + n_exec;
            a.done[ab] = ((sh.act >> ab) & 1) ? 0 : 1;
            if (a.stop_out) a.stop_out[ab] = (uint8_t)last_stop;
        }
    }
}

template <int NB>
__global__ __launch_bounds__(PT) void k_decode_persist(PersistArgs a) {
    __shared__ Shared sh;
    const Ws ws{a.ring, a.B, a.epoch};
    const int per = 16 * a.B + NFB;
    if ((int)(blockIdx.x % per) < 16 * a.B) run_block<true, 1>(a, ws, sh);
    else run_block<false, NB>(a, ws, sh);
}

}  // namespace

int persist_groups(int B, int n_cu) {
    for (int g = 3; g >= 1; --g)
        if (24 % g == 0 && g * (16 * B + NFB) <= n_cu) return g;
    return 0;
}

int persist_grid(int B, int groups) { return groups * (16 * B + NFB); }

size_t persist_ring_bytes(int B) {
    const size_t slot = (size_t)24 * B * (16 + 1 + 64 + 1) * 512 + (size_t)B * PERSIST_LGS + 16;
    return slot * RING * 8;
}

int persist_max_tokens() { return TMAXP; }

hipError_t decode_persist(const PersistArgs& a, hipStream_t s, hipEvent_t start, hipEvent_t stop) {
    const dim3 g(persist_grid(a.B, a.groups)), blk(PT);
    if (a.B <= 1) hipExtLaunchKernelGGL(k_decode_persist<1>, g, blk, 0, s, start, stop, 0, a);
    else if (a.B <= 2) hipExtLaunchKernelGGL(k_decode_persist<2>, g, blk, 0, s, start, stop, 0, a);
    else if (a.B <= 4) hipExtLaunchKernelGGL(k_decode_persist<4>, g, blk, 0, s, start, stop, 0, a);
    else hipExtLaunchKernelGGL(k_decode_persist<8>, g, blk, 0, s, start, stop, 0, a);
    return hipGetLastError();
}

}  // namespace gsv
