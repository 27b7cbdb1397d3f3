// Persistent decode for ONE sequence (the single-stream case): the whole AR loop
// of the stage decoder (t2s_stage_decoder_fp32.onnx, loop Inference.py:95-106)
// in one launch, with TWO hand-offs per layer.
//
// A post-norm layer (stage#43-120) is a chain  x_l -> q,k,v -> attention -> out-proj
// -> LN1 -> FFN1 -> FFN2 -> LN2 -> x_{l+1}.  Spread over many CUs it needs an
// all-to-all after the out-projection and one after FFN2; nothing else has to
// cross workgroups:
//   attention workgroup (head h, 16 per layer): reads the 16 FFN2 partials of the
//     previous layer plus its LN1 output h1_{l-1}, forms x_l = LN2(h1 + b2 + sum)
//     itself, then q/k/v of head h, attention over the cached keys, and the
//     head's out-projection slice -> 512 partial granules PA[l][h].
//   FFN workgroup (slice j = hidden units [128 j, 128 j + 128), 16 per layer):
//     forms x_l the same way (off the critical path, while attention runs), then
//     h1_l = LN1(x_l + bo + sum_h PA[l][h]), publishes h1_l (32 columns per
//     slice), FFN1 rows of the slice (ReLU), FFN2 partial -> granules PF[l][j].
// So a token costs 2 hand-offs per layer + logits + sampler + token = 50 hops
// (a design in which every workgroup tracks the residual stream needs 3 per
// layer).  Everything else is local.
//
// Grid: G layer groups x 32 workgroups (one per CU; LDS forces it): G = 8 fills
// the chip (256); with the vocoder overlapped on its own CUs (engine option
// "vocoder_cus") G = 6 or 7.  Group g owns layers g, g+G, g+2G, ... and keeps its
// weights of the owned layer it works on next in registers (q/k/v rows 48,
// out-proj column 16; W1 rows 64, W2 column 64 VGPRs) with the head's K/V rows in
// LDS, all loaded during the G-1 layers it waits; a waiting workgroup sleeps on one wake-up granule (the output of the
// layer two before its own) and polls its real inputs only then.  Group 1's FFN
// workgroups also hold the logits rows (ar_predict_layer, 64 + 1 per workgroup)
// in LDS for the whole launch and compute the logits after layer 23.  Greedy
// decoding: each of them also reduces its rows to the first argmax of the
// penalised and of the raw logits and publishes those 4 granules; every group-0
// workgroup polls the 16 x 4 granules and resolves the token (and the stop rule)
// itself -- one hop from the logits to layer 0 -- and group 0's head-0 attention
// workgroup records it (y, seen, the token granule TK the other groups read).
// Sampled decoding: the logits go to group 2's head-0 attention workgroup, which
// runs the sampler (sampler.h, K10) and publishes TK, which group 0 waits on.
//
// Hand-offs: the two per-layer all-to-alls (PA, PFH) travel as 16-byte granules
// {tag, v0, v1, v2} -- three consecutive columns and their tag in one write-through
// store, swept by 16-byte loads (MI355X_MICROARCH.md: 8-byte accesses run at
// 0.54-0.70x the 16-byte rate; tools/xcd_handoff.hip on this pattern: a 16-producer
// row sweep 1.55 us vs 1.98 us with 8-byte {tag, value} granules).  Two threads poll
// each column group (half of the rows each; the second continues the first's sum in
// row order), so the poll registers stay small.  The logits candidates and the token
// keep 8-byte granules (persist.h).  tag = (epoch << 12) | (step + 1) in a ring of
// RING1 step slots.  Every sum is formed in a fixed order, so results do not depend
// on arrival order.  Every spin is bounded; a timeout sets the error word and every
// workgroup leaves.
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
constexpr int NG_MAX = 8;          // layer groups (a.groups, 3..8): layer l -> group l % a.groups
constexpr int GW = 32;             // workgroups per group: 16 attention + 16 FFN
constexpr int NF = 16;             // FFN slices per layer (128 hidden units each)
constexpr int KVL1 = 448;          // K/V rows of a head staged in LDS
constexpr int TMAX1 = 4096;        // longest key range (pe table)
constexpr int RING1 = 4;           // granule ring depth (steps)
constexpr int LOGIT_GRP = 1;       // FFN workgroups of this group compute the logits
constexpr int SAMPLER_GRP = 2;     // head-0 attention workgroup of this group samples
constexpr int LROWS = 64;          // logits rows per FFN workgroup (16 x 64 = 1024, + EOS row)
constexpr long FOLD_LAYER = 2 * 1536 + 2 * 2048;   // PersistArgs::fold floats per layer
constexpr long LOGIT_FOLD = 24 * FOLD_LAYER;        // then [W_pred n2w_23 | W_pred n2b_23] (1025 each)

// A 512-column row as 16-byte granules: column c -> block b = c / 32, granule
// 11 b + (c % 32) / 3, slot (c % 32) % 3 (11 granules per 32-column block, the last
// holding 2 columns): GQ granules per row.
constexpr int GQ = 176;
__device__ __forceinline__ int gq_col(int q, int k) { return 32 * (q / 11) + 3 * (q % 11) + k; }
__device__ __forceinline__ int gq_n(int q) { return q % 11 == 10 ? 2 : 3; }
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// Granule ring.  Per step slot: PA [24][16][GQ], PFH [24][17][GQ] (rows 0..15 FFN2
// partials, row 16 = h1) of 16-byte granules, then LG [PERSIST_LGS], TK [16] of 8-byte
// ones.  The 16-byte rows are addressed as a buffer (byte offsets).
struct Ws1 {
    u64* ring;
    unsigned epoch;
    __amdgpu_buffer_rsrc_t rs;                          // the ring as a buffer resource
    static constexpr long ROW = 2L * GQ;                 // u64 units per 16-byte-granule row
    static constexpr long oPFH = 24L * 16 * ROW;
    static constexpr long oLG = oPFH + 24L * 17 * ROW;
    static constexpr long oTK = oLG + PERSIST_LGS;
    static constexpr long SLOT = oTK + 16;
    __device__ u64* slot(int s) const { return ring + (long)(s % RING1) * SLOT; }
    __device__ unsigned tag(int s) const { return (epoch << 12) | (unsigned)(s + 1); }
    // byte offsets of the 16-byte rows (< 2^31: the ring is ~9 MB)
    __device__ int PA(int s, int l, int h) const {
        return (int)(((long)(s % RING1) * SLOT + ((long)l * 16 + h) * ROW) * 8);
    }
    __device__ int PFH(int s, int l, int j) const {
        return (int)(((long)(s % RING1) * SLOT + oPFH + ((long)l * 17 + j) * ROW) * 8);
    }
    __device__ const u64* at(int byte_off) const { return ring + byte_off / 8; }
    __device__ u64* LG(int s) const { return slot(s) + oLG; }
    __device__ u64* TK(int s) const { return slot(s) + oTK; }
};

// One write-through 16-byte store {tag, v0, v1, v2} (buffer_store_dwordx4 ... sc1).
template <class W>
__device__ __forceinline__ void st_g16(const W& ws, int off, unsigned tag, float v0, float v1, float v2) {
    const u32x4 v = {tag, __float_as_uint(v0), __float_as_uint(v1), __float_as_uint(v2)};
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, v),
                                           ws.rs, off, 0, 16 /* sc1 */);
}
template <class W>
__device__ __forceinline__ u32x4 ld_g16(const W& ws, int off) {   // buffer_load_dwordx4 ... sc1
    return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(ws.rs, off, 0, 16 /* sc1 */));
}

// One lane waits for N 16-byte granules off + k * stride (k < N), all N loads in
// flight; re-polls only the stale ones (persist.h wait_gran_n with 16-byte granules).
template <int N, class W>
__device__ __forceinline__ void wait_g16_n(const W& ws, int off, int stride, unsigned tag, u32x4 (&g)[N], int* err,
                                           bool& ok, unsigned long long ticks) {
#pragma unroll
    for (int k = 0; k < N; ++k) g[k] = ld_g16(ws, off + k * stride);
    unsigned long long t0 = 0;
    for (unsigned it = 0;; ++it) {
        bool all = true;
#pragma unroll
        for (int k = 0; k < N; ++k) all &= g[k].x == tag;
        if (all) break;
        if (it == 0) t0 = __builtin_amdgcn_s_memrealtime();
        __builtin_amdgcn_s_sleep(1);
        asm volatile("" ::: "memory");   // the loads below are re-issued every round
#pragma unroll
        for (int k = 0; k < N; ++k)
            if (g[k].x != tag) g[k] = ld_g16(ws, off + k * stride);
        if ((it & 63) == 63) {
            if (ld_rlx(err) != 0) { ok = false; break; }
            if (__builtin_amdgcn_s_memrealtime() - t0 > ticks) {
                atomicCAS(err, 0, 1);
                ok = false;
                break;
            }
        }
    }
}

// A sleeping lane waits for the TAG of a 16-byte granule (dword 0) only.
__device__ __forceinline__ void wait_tag16_slow(const u64* p, unsigned tag, int* err, bool& ok,
                                                unsigned long long ticks) {
    if ((unsigned)ld_rlxu64(p) == tag) return;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (unsigned it = 1;; ++it) {
        __builtin_amdgcn_s_sleep(8);
        if ((unsigned)ld_rlxu64(p) == tag) return;
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

// Small arrays first: their LDS offsets stay below 64 KB, so an access is the
// lane's tid-based address plus an instruction offset (no extra address
// registers live across the layer loop -- the kernel sits at the 256-VGPR limit).
struct Shared1 {
    float pk[PWV][64];              // per-wave staging of 64 published columns (16-byte granules)
    float hs[3 * GQ];               // partial row sums of the first poll half (hop B / hop A)
    float h1s[32];                  // h1 block j of an FFN workgroup, staged for its 11 granules
    float qkv[96];
    _Float16 osh[PWV][32], osl[PWV][32];   // MFMA row operand: head output split hi + lo (out-projection),
                                           // one copy per wave (each wave merges the head itself)
    float lnb[2][512];              // LayerNorm inputs: [0] x_l (form_x), [1] LN1 (FFN)
    _Float16 xh[512], xl[512];      // MFMA row operand: h1 split hi + lo (FFN1)
    _Float16 fh[128], fl[128];      // MFMA row operand: FFN1 output split hi + lo (FFN2)
    float p2[3][512];               // LN2 of layer l-1 (b2, scale, shift) for form_x (LDS-DMA)
    float red[2 * PWV];
    float wred[2][PWV];
    uint32_t seen[33];
    int tok, fin, fail;
    int stopreq;                    // the stop word as last read (gsv_request_stop; fills the 8-byte padding)
    unsigned long long stamp[16];   // [0,8) 100 MHz realtime, [8,16) shader clock
    SampleLds<PT> samp;
    union {
        struct {                    // FFN role
            uint4 wp[LROWS + 1][65];   // logits rows (group LOGIT_GRP), resident for the launch (rows
                                       // padded by 16 B: the MFMA B reads of 16 rows are conflict-free)
            float lp23[3][512];        // LN2 of layer 23 (b2, scale, shift), logits group
            float lfB[LROWS + 16], lfC[LROWS + 16];   // folded LN2_23 vectors of the rows (fold)
            float xr[512];             // x_l (form_x), read back by the hop-A column owners
            uint32_t seenq[64][33];    // multi-sequence logits workgroups: each sequence's seen bitmap
            float bo[512], n1w[512];   // out-projection bias and LN1 scale of the layer (LDS-DMA)
        } ff;
        struct {                    // attention role
            float k[KVL1 * 32];     // K/V rows [0, min(kv, KVL1)) of the head (LDS-DMA)
            float v[KVL1 * 32];
            float p[TMAX1];         // scores, then softmax numerators
            float ov[16][32];       // P.V partial sums of 16 key groups (general path)
            float ov4[PWV][32];     // P.V partial of each wave (fast path)
            float lg[PERSIST_LGS];  // logits (sampler)
        } at;
    };
    // multi-sequence launch (k_decode_persist1m): per-sequence state (last: the offsets of
    // the arrays above stay as the single-sequence kernel has them)
    struct {
        int tok[64], act[64], ny0[64], kv0[64], st0[64], nexe[64], lstop[64], lfin[64];
        int kstep[64];              // the step whose status of the sequence is known (seq_runs)
        int stop_s;                 // the step the stop word was last read at (resolve_m)
        uint32_t seens[4][33];      // a sampler workgroup's sequences h, h + 16, h + 32, h + 48
    } m;
};

#define STAMP1(i)                                                                         \
    do {                                                                                  \
        if (probe && threadIdx.x == 0) {                                                  \
            sh.stamp[i] = __builtin_amdgcn_s_memrealtime();                               \
            sh.stamp[8 + (i)] = __builtin_amdgcn_s_memtime();                             \
        }                                                                                 \
    } while (0)

// threadIdx.x as a value the compiler cannot see through: the lane-derived LDS / ring
// offsets of a pass are recomputed from it (a few VALU operations) instead
// of hoisted out of the layer / sequence loops and spilled (a chain of dependent scratch reloads
// costs ~1 us per pass)
__device__ __forceinline__ int opaque_tid() {
    int t = threadIdx.x;
    asm volatile("" : "+v"(t));
    return t;
}

// A workgroup barrier without __syncthreads' memory fence: LDS writes are complete
// (lgkmcnt(0)) but in-flight global stores are not waited for.  The multi-sequence
// kernel's waves publish write-through granules and go on with the next sequence; a
// fence there would hold every wave for the stores' ~1 us round trip.
__device__ __forceinline__ void bar_nf() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}
template <bool NF>
__device__ __forceinline__ void bar_t() {
    if (NF) bar_nf();
    else __syncthreads();
}
template <bool NF = false>
__device__ __forceinline__ bool block_ok_t(bool ok, Shared1& sh) {
    if (!ok) sh.fail = 1;
    bar_t<NF>();
    return sh.fail == 0;
}
__device__ __forceinline__ bool block_ok1(bool ok, Shared1& sh) {
    if (!ok) sh.fail = 1;
    __syncthreads();
    return sh.fail == 0;
}

// LayerNorm statistics of a 512-value row already in LDS, computed by EVERY wave
// over the whole row (8 values per lane, the same order in every wave and every
// workgroup), in ONE interleaved DPP reduction of the shifted sum and sum of
// squares: with c = row[0], mean = c + E[v - c] and var = E[(v - c)^2] -
// E[v - c]^2 (the shift keeps the difference well conditioned when |mean| >> std;
// ORT's own LayerNorm kernel is one-pass too); the scale is returned as
// rden = 1 / sqrt(var + eps) (v_rsq_f32, so the normalisation is a multiply).
// One barrier (the caller's, after the row is written) per LayerNorm.
__device__ __forceinline__ void ln_row_stats(const float* buf, float& mean, float& rden) {
    const int lane = threadIdx.x & 63;
    const float4 a = *reinterpret_cast<const float4*>(buf + 8 * lane);
    const float4 b = *reinterpret_cast<const float4*>(buf + 8 * lane + 4);
    const float c = buf[0];
    const float v8[8] = {a.x - c, a.y - c, a.z - c, a.w - c, b.x - c, b.y - c, b.z - c, b.w - c};
    float r[2];
    r[0] = ((v8[0] + v8[1]) + (v8[2] + v8[3])) + ((v8[4] + v8[5]) + (v8[6] + v8[7]));
    r[1] = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) r[1] += v8[k] * v8[k];
    wave_sum_n<2>(r);
    const float d = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(r[0]), 63)) * (1.0f / 512.0f);
    const float q = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(r[1]), 63)) * (1.0f / 512.0f);
    mean = c + d;
    rden = __builtin_amdgcn_rsqf(fmaxf(q - d * d, 0.f) + 1e-5f);   // 1 / sqrt(var + eps), v_rsq_f32
}

__device__ __forceinline__ float ln_apply(float v, float mean, float rden, float w, float b) {
    return (v - mean) * rden * w + b;
}

// Batch-1 GEMV on the 16x16x32 f16 MFMA (v_mfma_f32_16x16x32_f16).  The weights
// are exactly fp16; the f32 activation vector is split x = hi + lo into two fp16
// rows (A rows 0 and 1, rows 2..15 zero), so C row 0 + C row 1 = W.x with the
// dropped residual ~2^-22 |x| (f32-level, as the prefill GEMM).  Lane l holds
// A[row l & 15][k = 8 (l >> 4) + i], B[k = 8 (l >> 4) + i][col l & 15] and
// C[row 4 (l >> 4) + r][col l & 15]: the result of column l (l < 16) is
// c[0] + c[1].  Replaces 2 VALU ops per MAC (cvt + fma) and the DPP row sums.
typedef _Float16 h8v __attribute__((ext_vector_type(8)));
__device__ __forceinline__ h8v bfrag(const uint4 w) { return __builtin_bit_cast(h8v, w); }
// This lane's A-operand base: row 0 reads hi, rows 1..15 lo; chunk c is one
// ds_read_b128 at base + 32 c (an instruction offset).  Rows 2..15 of C are
// never used, so their lanes need no zeroing: they read the lo row again, which
// the LDS serves as a broadcast (128 distinct bytes per fragment either way),
// with no exec-masked branches around the reads.
__device__ __forceinline__ const _Float16* abase(const _Float16* hi, const _Float16* lo, int lane) {
    return ((lane & 15) == 0 ? hi : lo) + 8 * (lane >> 4);
}
__device__ __forceinline__ h8v afrag(const _Float16* base, int k0) {
    return __builtin_bit_cast(h8v, *reinterpret_cast<const uint4*>(base + k0));
}
__device__ __forceinline__ f32x4 mfma16(h8v a, h8v b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}
// fp16 split of an f32 activation; false when |v| is beyond the fp16 range
__device__ __forceinline__ bool split_h(float v, _Float16& hi, _Float16& lo) {
    hi = (_Float16)v;
    lo = (_Float16)(v - (float)hi);
    return fabsf(v) < 65504.f;
}
constexpr int ERR_F16_RANGE = 2;   // error word: an activation left the fp16 range (host re-runs)


// Scores of the general case (more than 512 keys or rows beyond the LDS stage),
// out of line so the common path keeps its registers.  Returns the lane's max.
// (templates on V: each kernel gets its own out-of-line copy, so the multi-sequence
// kernel does not change the single-sequence kernel's register allocation)
template <int V, class SH>
__device__ __noinline__ float scores_general1(SH& sh, const float* Kw, int kv, int T, float q0, float q1,
                                              float q2, float q3, float sc, float4 knew, int c8, int g) {
    float lmax = -INFINITY;
    for (int base = 0; base < T; base += 512) {
        float sv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int t = base + 64 * u + g;
            float4 kr;
            if (t < kv && t < KVL1) kr = *reinterpret_cast<const float4*>(sh.at.k + t * 32 + 4 * c8);
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

// One wave's share of the head's attention (the common case: T <= 512 keys, every
// row [0, kv] in LDS -- the new row kv is written there with the q/k/v results):
// keys t = 64 u + g (u < NU, g = 8 w + lane / 8), 8 lanes x 4 dims per key row
// (conflict-free 16-B LDS reads), every K and V read of the NU rounds issued up
// front.  Rows past kv are read as row kv (finite) and weighted by exp(-inf) = 0,
// so the rounds carry no per-key selects beyond the score mask.  Online softmax within the wave: m_w = max s, p = exp(s -
// m_w), l_w = sum p, o_w = sum p v (rows of 16 lanes summed by row_ror 8) -> LDS
// sh.wred[0/1][w], sh.at.ov4[w][row]; the caller merges the 8 waves after a barrier.
// x + (x of the other 16-lane row of the pair) / (of the other 32-lane half), every lane
__device__ __forceinline__ float swap_sum16(float x) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float swap_sum32(float x) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// Head output from the 8 wave partials (m_w, l_w in sh.wred, o_w in sh.at.ov4),
// merged by EVERY wave into its own operand copy (no barrier after): lane j < 8
// weighs wave j, e_j = exp(m_j - M); O = sum e_j o_j / sum e_j l_j.
template <class SH>
__device__ __forceinline__ void merge_waves1(SH& sh, int w, int lane) {
    const int j = lane & 7;
    const float mj = sh.wred[0][j];
    float M = mj;
    M = fmaxf(M, dpp_f<0xB1, 0xF>(M));
    M = fmaxf(M, dpp_f<0x4E, 0xF>(M));
    M = fmaxf(M, dpp_f<0x141, 0xF>(M));
    const float e = mj == -INFINITY ? 0.f : __expf(mj - M);
    float L = e * sh.wred[1][j];
    L += dpp_f<0xB1, 0xF>(L);
    L += dpp_f<0x4E, 0xF>(L);
    L += dpp_f<0x141, 0xF>(L);
    const int d = lane & 31;
    float O = 0.f;
#pragma unroll
    for (int ww = 0; ww < PWV; ++ww)
        O += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(e), ww)) * sh.at.ov4[ww][d];
    if (lane < 32) split_h(O / L, sh.osh[w][d], sh.osl[w][d]);   // a convex combination of V rows
    __builtin_amdgcn_wave_barrier();
}

template <int NU, class SH>
__device__ __forceinline__ void wave_attn1(SH& sh, float q0, float q1, float q2, float q3, float sc,
                                           int kv, int T, int c8, int g, int w, int lane) {
    float4 kr[NU];
#pragma unroll
    for (int u = 0; u < NU; ++u)
        kr[u] = *reinterpret_cast<const float4*>(sh.at.k + min(64 * u + g, kv) * 32 + 4 * c8);
    // (q s) . (k s) as (q s s) . k: the key's scale folded into the query once per
    // lane instead of once per key element (rounding differs at the ulp level)
    const float p0 = q0 * sc, p1 = q1 * sc, p2 = q2 * sc, p3 = q3 * sc;
    float sv[NU];
#pragma unroll
    for (int u = 0; u < NU; ++u) {
        const float4 k4 = kr[u];
        float x = p0 * k4.x;
        x += p1 * k4.y;
        x += p2 * k4.z;
        x += p3 * k4.w;
        sv[u] = x;
    }
#pragma unroll
    for (int u = 0; u < NU; ++u) sv[u] += dpp_f<0xB1, 0xF>(sv[u]);
#pragma unroll
    for (int u = 0; u < NU; ++u) sv[u] += dpp_f<0x4E, 0xF>(sv[u]);
#pragma unroll
    for (int u = 0; u < NU; ++u) sv[u] += dpp_f<0x141, 0xF>(sv[u]);
    float4 vr[NU];   // V reads in flight during the max reduction
#pragma unroll
    for (int u = 0; u < NU; ++u)
        vr[u] = *reinterpret_cast<const float4*>(sh.at.v + min(64 * u + g, kv) * 32 + 4 * c8);
    float wm = -INFINITY;
#pragma unroll
    for (int u = 0; u < NU; ++u) {
        sv[u] = 64 * u + g < T ? sv[u] : -INFINITY;
        wm = fmaxf(wm, sv[u]);
    }
    const float m_w = wave_max_dpp(wm);
    const float mref = m_w == -INFINITY ? 0.f : m_w;   // (wave-uniform) every key of this wave masked
    float o0 = 0.f, o1 = 0.f, o2 = 0.f, o3 = 0.f, lsum = 0.f;
#pragma unroll
    for (int u = 0; u < NU; ++u) {
        const float pu = __expf(sv[u] - mref);   // v_exp_f32 (ORT's MLAS exp is not libm's either); masked: exp(-inf) = 0
        const float4 v4 = vr[u];
        o0 += pu * v4.x;
        o1 += pu * v4.y;
        o2 += pu * v4.z;
        o3 += pu * v4.w;
        lsum += pu;
    }
    // sum over the wave's 8 key groups (lanes c8 + 8 k): row_ror 8 within each 16-lane
    // row, then the gfx950 row / half swaps (VALU, no LDS round trip)
    o0 += dpp_f<0x128, 0xF>(o0);
    o1 += dpp_f<0x128, 0xF>(o1);
    o2 += dpp_f<0x128, 0xF>(o2);
    o3 += dpp_f<0x128, 0xF>(o3);
    o0 = swap_sum16(o0); o1 = swap_sum16(o1); o2 = swap_sum16(o2); o3 = swap_sum16(o3);
    o0 = swap_sum32(o0); o1 = swap_sum32(o1); o2 = swap_sum32(o2); o3 = swap_sum32(o3);
    const float l_w = wave_sum_dpp(c8 == 0 ? lsum : 0.f);
    if (lane < 8) *reinterpret_cast<float4*>(&sh.at.ov4[w][4 * lane]) = make_float4(o0, o1, o2, o3);
    if (lane == 0) {
        sh.wred[0][w] = m_w;
        sh.wred[1][w] = l_w;
    }
}

// The general case (more than 512 keys or rows beyond the LDS stage): scores into
// sh.at.p, block softmax, P.V over 16 key groups, head output -> sh.osh/osl.  Out
// of line so the common path keeps its registers.
template <int V, class SH>
__device__ __noinline__ void attn_general1(SH& sh, const float* Kw, const float* Vw, int kv, int T, float q0,
                                           float q1, float q2, float q3, float sc, float4 knew, int c8, int g, int w,
                                           int lane, int tid) {
    const float lmax = scores_general1<V>(sh, Kw, kv, T, q0, q1, q2, q3, sc, knew, c8, g);
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
    {
        const int kg = tid >> 5, d = tid & 31;
        const int tl = min(kv, KVL1);
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
    if (lane < 32) {   // every wave its own operand copy
        float O = 0.f, L = 0.f;
#pragma unroll
        for (int kg = 0; kg < 16; ++kg) O += sh.at.ov[kg][lane];
#pragma unroll
        for (int ww = 0; ww < PWV; ++ww) L += sh.wred[1][ww];
        split_h(O / L, sh.osh[w][lane], sh.osl[w][lane]);   // a convex combination of V rows
    }
    __builtin_amdgcn_wave_barrier();
}

// Step start: thread 0 learns the token of step s (s >= 1: granule TK(s), whose
// bit 16 says the previous step finished the sequence).  Group 0 needs the token
// at once (its layer 0 starts from it) and sleeps on the layer-23 output of the
// previous step first; the other groups only need the stop bit and poll slowly.
// Returns false when the loop is over (or on error: sh.fail).

// A stop request (gsv_request_stop, the reference's stop_event checked once per loop
// step, Inference.py:96-97) seen at a token: the launch is abandoned as a timed-out
// one is -- error word 3, so every workgroup leaves at its next wait and no sequence
// state is written back (the host returns GSV_E_STOPPED; the sentence yields None).
// Only a token resolver reads the stop word, and only once per step, so workgroups
// never disagree about a sequence's tokens.
__device__ __forceinline__ void stop_launch(const PersistArgs& a, bool& ok) {
    atomicCAS(a.err, 0, 3);
    ok = false;
}
// Fused greedy step end (group 0, s >= 1): the token of step s - 1 from the logits
// workgroups' local argmaxes (LG(s - 1): candidate q's {penalised max, its index, raw
// max, its index} at 4 q .. 4 q + 3; q = 4 j + w covers rows 64 j + 16 w .. + 16, q =
// 64 the EOS row): the first argmax over all 1025 logits, as sample_block's greedy
// branch (value max, then the smallest index holding it); the stop rule
// (stop_condition_tensor, t2s_stage_decoder_fp32.onnx#1807-1821) and the loop end
// (Inference.py:95-106).  The publisher also appends y, marks seen and publishes TK(s).
__device__ void resolve_greedy(const PersistArgs& a, const Ws1& ws, int s, int ny0, int st0, bool publisher,
                               Shared1& sh, int& last_stop, int& last_fin) {
    const int tid = threadIdx.x;
    bool ok = true;
    if (tid == 0) wait_tag16_slow(ws.at(ws.PFH(s - 1, 23, 0)), ws.tag(s - 1), a.err, ok, a.spin_ticks);
    if (tid == 64) sh.stopreq = ld_stop(a.stop_req);   // wave 1: beside wave 0's (longer) wait
    if (!block_ok1(ok, sh)) return;
    if (tid < 64) {
        // lane q: candidate q's {penalised max, its index, raw max, its index} (16 rows of
        // slice q / 4); lane 0 also the EOS row's (candidate 64, index 1024)
        float f[4];
        wait_gran_n<4>(ws.LG(s - 1) + 4 * tid, 1, ws.tag(s - 1), f, a.err, ok, a.spin_ticks);
        float gv = f[0], rv = f[2];
        int gi = __float_as_int(f[1]), ri = __float_as_int(f[3]);
        if (tid == 0) {
            float e[4];
            wait_gran_n<4>(ws.LG(s - 1) + 256, 1, ws.tag(s - 1), e, a.err, ok, a.spin_ticks);
            argmax_merge(gv, gi, e[0], __float_as_int(e[1]));
            argmax_merge(rv, ri, e[2], __float_as_int(e[3]));
        }
        const float gm = wave_max_dpp(gv), rm = wave_max_dpp(rv);
        const int tok = wave_min_dpp(gv == gm ? gi : 0x7fffffff);
        const int raw = wave_min_dpp(rv == rm ? ri : 0x7fffffff);
        if (tid == 0) {
            const int stop = (raw == 1024 || tok == 1024) ? 1 : 0;
            const bool fin = seq_finished(a.force_b, 0, a.force_steps, a.max_steps, st0 + s, stop);
            if (sh.stopreq) stop_launch(a, ok);
            sh.tok = tok;
            sh.fin = fin ? 1 : 0;
            if (publisher && ok) {
                a.y[ny0 + s - 1] = tok;
                sh.seen[tok >> 5] |= 1u << (tok & 31);
                last_stop = stop;
                last_fin = fin ? 1 : 0;
                st_gran(ws.TK(s), ws.tag(s), __uint_as_float((unsigned)tok | (fin ? 1u << 16 : 0u)));
            }
        }
    }
    if (!ok) sh.fail = 1;
}

// Step start: thread 0 learns the token of step s (s >= 1: granule TK(s), whose
// bit 16 says the previous step finished the sequence).  Group 0 needs the token
// at once (its layer 0 starts from it): with fused greedy it resolves it itself
// (resolve_greedy), else it sleeps on the layer-23 output of the previous step and
// then polls TK; the other groups only need the stop bit and poll slowly (the
// greedy logits workgroups also mark the token in their seen bitmap).
// Returns false when the loop is over (or on error: sh.fail).
__device__ bool step_start(const PersistArgs& a, const Ws1& ws, int s, bool grp0, Shared1& sh, bool fused,
                           bool mark_seen, bool publisher, int ny0, int st0, int& last_stop, int& last_fin) {
    if (fused && grp0 && s > 0) {
        resolve_greedy(a, ws, s, ny0, st0, publisher, sh, last_stop, last_fin);
    } else if (threadIdx.x == 0) {
        bool ok = true;
        if (s > 0) {
            float v;
            if (grp0) {
                wait_tag16_slow(ws.at(ws.PFH(s - 1, 23, 0)), ws.tag(s - 1), a.err, ok, a.spin_ticks);
                v = ok ? wait_gran(ws.TK(s), ws.tag(s), a.err, ok, a.spin_ticks) : 0.f;
            } else {
                wait_tag_slow(ws.TK(s), ws.tag(s), a.err, ok, a.spin_ticks);
                v = ok ? wait_gran(ws.TK(s), ws.tag(s), a.err, ok, a.spin_ticks) : 0.f;
            }
            const unsigned u = __float_as_uint(v);
            sh.tok = (int)(u & 0xffff);
            sh.fin = ok ? (int)((u >> 16) & 1) : 1;
            if (mark_seen && ok) sh.seen[sh.tok >> 5] |= 1u << (sh.tok & 31);
        }
        if (!ok) sh.fail = 1;
    }
    __syncthreads();
    const bool go = sh.fail == 0 && sh.fin == 0;
    __syncthreads();
    return go;
}

// 512 floats src -> LDS dst by LDS-DMA, half h (256 floats, one 1-KB wave
// instruction).  Per-layer vectors travel this way: no registers are held for
// them across the layers a workgroup waits; every reader is behind a barrier.
__device__ __forceinline__ void dma_half(const float* src, float* dst, int h, int lane) {
    __builtin_amdgcn_global_load_lds(src + 256 * h + lane * 4, dst + 256 * h, 16, 0, 0);
}
// Idle a workgroup between publishing a layer's output and streaming the weights
// of its next owned layer (needed 7 layers later): the consumers' gather of the
// hand-off is not queued behind this CU's refill burst (MI355X_MICROARCH.md,
// gather-pass / handoff-1to1 endpoint classes).
__device__ __forceinline__ void pf_wait(int ticks) {
    for (int i = 0; i < ticks; ++i) __builtin_amdgcn_s_sleep(32);
}
// LN2 of layer l - 1 -> sh.p2 (call from every wave; l > 0).  The single-sequence kernel:
// waves 0..5 (its fenced barriers order the DMAs long before the next owned layer reads
// them).  The multi-sequence kernel (POLLERS): waves 0, 1, 2, 4, 5, 6, the hop-B gather's
// polling waves, whose in-order vmcnt waits retire these DMAs before the gather's last
// barrier, after which sh.p2 is read -- waves 3 and 7 never poll and that kernel has no
// fenced barrier between a prefetch and the next gather.  (Hardening found while looking
// for the r05 persist1m deviation, profiles/r05x_persist1m_deviation.txt; it did not
// change that case.  The single-sequence kernel keeps its assignment: moving its DMAs
// cost ~0.25 ms per launch, r05b.)
template <bool POLLERS = false>
__device__ __forceinline__ void dma_ln2(const PLayer& Q, Shared1& sh, int w, int lane) {
    if (POLLERS) {
        if (w < 2) dma_half(Q.b2, sh.p2[0], w & 1, lane);
        else if (w == 2 || w == 4) dma_half(Q.n2w, sh.p2[1], w == 4, lane);
        else if (w == 5 || w == 6) dma_half(Q.n2b, sh.p2[2], w == 6, lane);
    } else {
        if (w < 2) dma_half(Q.b2, sh.p2[0], w & 1, lane);
        else if (w < 4) dma_half(Q.n2w, sh.p2[1], w & 1, lane);
        else if (w < 6) dma_half(Q.n2b, sh.p2[2], w & 1, lane);
    }
}

// Hop B: u = h1_{l-1} + (b2 + sum_j PF[l-1][j]) (l >= 1; the partials summed in
// slice order) -> sh.lnb[0], and with `split` the MFMA operand split of u * n2w ->
// sh.xh / sh.xl; lp2 = LDS rows {b2, scale, shift} of LN2_{l-1}.  A sleeping lane
// waits for the wake-up granule (layer l-2's output); then thread q < GQ polls rows
// 0..7 of granule column q and thread 256 + q rows 8..16, continuing the first
// thread's sums in row order (bit-identical to one thread summing rows 0..15).
// Ends with a block barrier.
template <class W, bool NF = false>
__device__ __forceinline__ bool gather_pfh(const PersistArgs& a, const W& ws, int s, int l, const float* lp2,
                                           Shared1& sh, bool split, bool wake = true) {
    const int tid = threadIdx.x, q = tid & 255;
    const unsigned tag = ws.tag(s);
    constexpr int RB = (int)Ws1::ROW * 8;   // bytes per row
    bool ok = true;
    if (l >= 2 && wake) {   // (a sequence that follows another through this layer polls at once)
        if (tid == 0) wait_tag16_slow(ws.at(ws.PFH(s, l - 2, 0)), tag, a.err, ok, a.spin_ticks);
        if (!block_ok_t<NF>(ok, sh)) return false;
    }
    const int off = ws.PFH(s, l - 1, 0) + 16 * q;
    u32x4 g[9];
    if (tid < GQ) {
        u32x4 h[8];
        wait_g16_n<8>(ws, off, RB, tag, h, a.err, ok, a.spin_ticks);
        float f0 = __uint_as_float(h[0].y), f1 = __uint_as_float(h[0].z), f2 = __uint_as_float(h[0].w);
#pragma unroll
        for (int r = 1; r < 8; ++r) {
            f0 += __uint_as_float(h[r].y);
            f1 += __uint_as_float(h[r].z);
            f2 += __uint_as_float(h[r].w);
        }
        sh.hs[3 * q] = f0; sh.hs[3 * q + 1] = f1; sh.hs[3 * q + 2] = f2;
    } else if (tid >= 256 && q < GQ) {
        wait_g16_n<9>(ws, off + 8 * RB, RB, tag, g, a.err, ok, a.spin_ticks);
    }
    if (!block_ok_t<NF>(ok, sh)) return false;
    if (tid >= 256 && q < GQ) {
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            if (k == 2 && gq_n(q) == 2) break;
            float f = sh.hs[3 * q + k];
#pragma unroll
            for (int r = 0; r < 8; ++r) f += __uint_as_float(g[r][1 + k]);
            const int c = gq_col(q, k);
            const float u = __uint_as_float(g[8][1 + k]) + (lp2[c] + f);
            sh.lnb[0][c] = u;
            if (split) {
                const float un = u * lp2[512 + c];
                if (!split_h(un, sh.xh[c], sh.xl[c]) || !(fabsf(un) < a.f16_limit)) {
                    atomicCAS(a.err, 0, ERR_F16_RANGE);
                    ok = false;
                }
            }
        }
    }
    return block_ok_t<NF>(ok, sh);
}

// x_l for column tid: layer 0 from the token (E_audio[tok] + alpha * pe[n]),
// otherwise LN2_{l-1}(u) with u from the hop-B gather.
template <class W, bool NF = false>
__device__ __forceinline__ bool form_x(const PersistArgs& a, const W& ws, int s, int l, int pos, const float* lp2,
                                       float& xv, Shared1& sh, int tok, bool wake = true) {
    const int tid = threadIdx.x;
    if (l == 0) {
        xv = ldg_h(a.emb, (long)tok * 512 + tid) + ldg(a.alpha, 0) * ldg(a.pe, (long)pos * 512 + tid);
        return true;
    }
    if (!gather_pfh<W, NF>(a, ws, s, l, lp2, sh, false, wake)) return false;
    const float v = sh.lnb[0][tid];
    float mean, rden;
    ln_row_stats(sh.lnb[0], mean, rden);
    xv = ln_apply(v, mean, rden, lp2[512 + tid], lp2[1024 + tid]);
    return true;
}

// The attention role's x_l without waiting for its LayerNorm statistics: u = the
// LN2_{l-1} INPUT (l = 0: x_0 itself) -> sh.lnb[0], and the MFMA operand split of
// u * n2w (l = 0: u) -> sh.xh / sh.xl, then the block barrier.  The q/k/v GEMV
// runs on that operand while the statistics are formed: with x = (u - mean) rden
// n2w + n2b,  W x + b = rden (W (u n2w) - mean W n2w) + (W n2b + b), the two
// constant vectors folded per layer at load time (PersistArgs::fold).
template <class W, bool NF = false>
__device__ __forceinline__ bool form_u(const PersistArgs& a, const W& ws, int s, int l, int pos, const float* lp2,
                                       Shared1& sh, int tok, bool wake = true) {
    const int tid = threadIdx.x;
    if (l > 0) return gather_pfh<W, NF>(a, ws, s, l, lp2, sh, true, wake);
    bool ok = true;
    const float u = ldg_h(a.emb, (long)tok * 512 + tid) + ldg(a.alpha, 0) * ldg(a.pe, (long)pos * 512 + tid);
    sh.lnb[0][tid] = u;
    if (!split_h(u, sh.xh[tid], sh.xl[tid]) || !(fabsf(u) < a.f16_limit)) {
        atomicCAS(a.err, 0, ERR_F16_RANGE);
        ok = false;
    }
    return block_ok_t<NF>(ok, sh);
}

// A wave's 64 published columns [64 w, 64 w + 64) (two 32-column blocks), staged by
// lanes < 16 in sh.pk[w][16 t + lane], leave as the blocks' 22 granules of the row at
// byte offset `row`.  In-wave LDS order needs no fence (LDS ops of a wave complete in
// order; the asm statement keeps the compiler from moving the reads up).
template <class W>
__device__ __forceinline__ void pub64(const W& ws, Shared1& sh, int row, unsigned tag, int w, int lane) {
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
    if (lane < 22) {
        const int b = lane >= 11 ? 1 : 0, r = lane - 11 * b;
        const float* p = sh.pk[w] + 32 * b + 3 * r;
        st_g16(ws, row + 16 * (11 * (2 * w + b) + r), tag, p[0], p[1], r == 10 ? 0.f : p[2]);
    }
}

// --------------------------------------------------------------------------
// Attention workgroup: head h of layers grp, grp + G, grp + 2G, ...
// --------------------------------------------------------------------------
__device__ void run_attn(const PersistArgs& a, const Ws1& ws, Shared1& sh, int grp, int h) {
    const int tid = threadIdx.x, lane = tid & 63, ng = a.groups;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const bool fused = a.greedy && a.knob[0] == 0;   // fused greedy step end (knob0 = 1: the sampler path)
    const bool sampler = !fused && grp == SAMPLER_GRP && h == 0;
    const bool publisher = fused ? (grp == 0 && h == 0) : sampler;   // records y / seen / sequence state
    const int ny0 = a.ny[0], kv0 = a.kvlen[0], st0 = a.steps[0];
    if (tid == 0) {
        sh.tok = (int)a.y[ny0 - 1];
        sh.fin = a.done[0] ? 1 : 0;
        sh.fail = 0;
    }
    if (publisher && tid < 33) sh.seen[tid] = a.seen[tid];
    const long kvoff = (long)h * a.tmax * 32;
    uint4 wq[16], wo[4];
    float qfB = 0.f, qfC = 0.f;   // folded LN2 vectors of this lane's q/k/v row
    auto prefetch = [&](int l, int kv) {
        const PLayer& P = a.L[l];
        // MFMA B fragments (lane: column lane & 15, k 8 (lane >> 4) .. + 8 of each 32-chunk).
        // q/k/v: wave w < 6 -> rows (m = w >> 1, dims 16 (w & 1) + (lane & 15)) of head h, K chunks c < 16
        const int n16 = lane & 15, k8 = 8 * (lane >> 4);
        if (w < 6) {
            const int row = (w >> 1) * 512 + h * 32 + 16 * (w & 1) + n16;
#pragma unroll
            for (int c = 0; c < 16; ++c) wq[c] = ldg16(P.w_in + (long)row * 512 + 32 * c + k8, 0);
            qfB = ldg(a.fold, (long)l * FOLD_LAYER + row);
            qfC = ldg(a.fold, (long)l * FOLD_LAYER + 1536 + row);
        }
        // out-projection: wave w -> output columns 64 w + 16 t + (lane & 15), K = the head's 32 dims
#pragma unroll
        for (int t = 0; t < 4; ++t) wo[t] = ldg16(P.w_out + (long)(64 * w + 16 * t + n16) * 512 + h * 32 + k8, 0);
        if (l > 0) dma_ln2(a.L[l - 1], sh, w, lane);
        // K/V rows [0, min(kv, KVL1)) -> LDS, 8 rows (1 KB) per wave instruction; lanes of
        // the last chunk past row kv - 1 stay idle (row kv is written by the q/k/v epilogue)
        const float* K = a.kc[l] + kvoff;
        const float* V = a.vc[l] + kvoff;
        const int nr = min(kv, KVL1), nch = (nr + 7) >> 3;
        for (int i = w; i < nch; i += PWV) {
            if (8 * i + (lane >> 3) < nr) {
                __builtin_amdgcn_global_load_lds(K + (long)i * 256 + lane * 4, sh.at.k + i * 256, 16, 0, 0);
                __builtin_amdgcn_global_load_lds(V + (long)i * 256 + lane * 4, sh.at.v + i * 256, 16, 0, 0);
            }
        }
    };
    __syncthreads();
    if (sh.fin) return;
    prefetch(grp, kv0);
    int n_exec = 0, last_stop = 0, last_fin = 0;
    for (int s = 0; s < a.smax; ++s) {
        if (!step_start(a, ws, s, grp == 0, sh, fused, false, publisher, ny0, st0, last_stop, last_fin)) break;
        const unsigned tag = ws.tag(s);
        const int kv = kv0 + s;
        for (int l = grp; l < 24; l += ng) {
            const bool probe = a.trace && ((s == 8 && (l == 12 || l == 13 || l == 23)) || (s == 9 && l == 0));
            STAMP1(0);
            if (!form_u(a, ws, s, l, ny0 + s, &sh.p2[0][0], sh, sh.tok)) return;
            STAMP1(1);
            // ---- q, k, v of head h on the MFMA: wave w < 6 -> 16 rows (C row 0 + row 1),
            // the LN2 statistics formed while the MFMAs run
            if (w < 6) {
                const _Float16* ab = abase(sh.xh, sh.xl, lane);
                float mean, rden;
                ln_row_stats(sh.lnb[0], mean, rden);   // first: interleaved with the MFMAs below
                f32x4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int cb = 0; cb < 16; cb += 8) {   // 8 operand reads in flight, then 8 MFMAs
                    h8v af[8];
#pragma unroll
                    for (int i = 0; i < 8; ++i) af[i] = afrag(ab, 32 * (cb + i));
#pragma unroll
                    for (int i = 0; i < 8; i += 2) {
                        c0 = mfma16(af[i], bfrag(wq[cb + i]), c0);
                        c1 = mfma16(af[i + 1], bfrag(wq[cb + i + 1]), c1);
                    }
                }
                mean = l > 0 ? mean : 0.f;   // layer 0: x_0 is not a LayerNorm output
                rden = l > 0 ? rden : 1.f;
                if (lane < 16) {
                    const float val = rden * (((c0[0] + c1[0]) + (c0[1] + c1[1])) - mean * qfB) + qfC;
                    sh.qkv[16 * w + lane] = val;
                    if (kv < KVL1 && w >= 2) {   // the new K / V row into the LDS stage (fast path reads it there)
                        float* row = (w < 4 ? sh.at.k : sh.at.v) + kv * 32 + 16 * (w & 1);
                        row[lane] = val;
                    }
                }
            }
            STAMP1(6);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's K/V LDS-DMA has landed
            STAMP1(7);
            __syncthreads();
            STAMP1(2);
            // ---- scores (q*s).(k*s) over [0, kv]: 8 lanes per key row (16 B each,
            // conflict-free LDS reads), keys t = base + 64 u + g
            float* Kw = a.kc[l] + kvoff;
            float* Vw = a.vc[l] + kvoff;
            const float sc = a.scale;
            const int T = kv + 1;
            const int c8 = lane & 7, g = (w << 3) | (lane >> 3);
            const float4 qc = *reinterpret_cast<const float4*>(sh.qkv + 4 * c8);
            const float q0 = qc.x * sc, q1 = qc.y * sc, q2 = qc.z * sc, q3 = qc.w * sc;
            const float4 knew = *reinterpret_cast<const float4*>(sh.qkv + 32 + 4 * c8);
            if (T <= 512 && kv < KVL1) {
                // common case: every cached row is in LDS (per-wave online softmax,
                // wave_attn1); the round count is specialised so every LDS read of a
                // round is issued up front.
                const int nu = (T + 63) >> 6;
                if (nu <= 2) wave_attn1<2>(sh, q0, q1, q2, q3, sc, kv, T, c8, g, w, lane);
                else if (nu <= 4) wave_attn1<4>(sh, q0, q1, q2, q3, sc, kv, T, c8, g, w, lane);
                else if (nu == 5) wave_attn1<5>(sh, q0, q1, q2, q3, sc, kv, T, c8, g, w, lane);
                else if (nu == 6) wave_attn1<6>(sh, q0, q1, q2, q3, sc, kv, T, c8, g, w, lane);
                else wave_attn1<8>(sh, q0, q1, q2, q3, sc, kv, T, c8, g, w, lane);
                __syncthreads();
                STAMP1(3);
                merge_waves1(sh, w, lane);
            } else {
                attn_general1<0>(sh, Kw, Vw, kv, T, q0, q1, q2, q3, sc, knew, c8, g, w, lane, tid);
            }
            STAMP1(4);
            // ---- out-projection slice of this head (column tid) -> partial granule
            {
                const h8v af = afrag(abase(sh.osh[w], sh.osl[w], lane), 0);
                f32x4 acc[4];
#pragma unroll
                for (int t = 0; t < 4; ++t) acc[t] = mfma16(af, bfrag(wo[t]), f32x4{0.f, 0.f, 0.f, 0.f});
                if (lane < 16) {
#pragma unroll
                    for (int t = 0; t < 4; ++t) sh.pk[w][16 * t + lane] = acc[t][0] + acc[t][1];
                }
                pub64(ws, sh, ws.PA(s, l, h), tag, w, lane);
                // the new K/V row (read by this workgroup only, next step)
                if (tid < 32) Kw[(long)kv * 32 + tid] = sh.qkv[32 + tid];
                else if (tid < 64) Vw[(long)kv * 32 + tid - 32] = sh.qkv[64 + tid - 32];
            }
            STAMP1(5);
            __syncthreads();   // LDS operands consumed before the next layer's LDS-DMA lands
            // ---- next owned layer (this step) or the first one of the next step
            const int ln = l + ng < 24 ? l + ng : grp;
            pf_wait(a.pf_delay);   // let the hand-off leave before this CU streams again
            prefetch(ln, l + ng < 24 ? kv : kv + 1);
            if (probe && tid < 16) a.trace[blockIdx.x * 16 + tid] = sh.stamp[tid];
        }
        // ---- sampler: logits granules of this step -> token -> TK(s + 1)
        if (sampler) {
            const bool probe = a.trace && s == 8;   // step-end trace (tools/knob_sweep.py)
            bool ok = true;
            if (tid == 0) wait_tag16_slow(ws.at(ws.PFH(s, 23, 0)), tag, a.err, ok, a.spin_ticks);
            if (tid == 64) sh.stopreq = ld_stop(a.stop_req);
            if (!block_ok1(ok, sh)) return;
            STAMP1(0);
            const u64* lgg = ws.LG(s);
            const int st = st0 + s;   // loop steps already executed
            int raw = 0, tok = 0;
            if (a.greedy) {
                // greedy (RandomNormalLike := 1): the token is the first argmax of the penalised
                // logits (sample_block's greedy branch), raw the first argmax of the raw ones.
                // Logits polled straight into registers, both argmaxes reduced together: one
                // barrier instead of sample_block's LDS staging and two block reductions.
                float g[2];
                wait_gran_n<2>(lgg + tid, PT, tag, g, a.err, ok, a.spin_ticks);
                float rv = -INFINITY, gv = -INFINITY;
                int ri = 0x7fffffff, gi = 0x7fffffff;
#pragma unroll
                for (int j = 0; j < 3; ++j) {
                    const int i = tid + PT * j;
                    float lj;
                    if (j < 2) lj = g[j];
                    else if (tid == 0) lj = wait_gran(lgg + 1024, tag, a.err, ok, a.spin_ticks);
                    else continue;
                    argmax_merge(rv, ri, lj, i);
                    float pen = lj;
                    if ((sh.seen[i >> 5] >> (i & 31)) & 1u) pen = lj < 0.f ? lj * a.rep_penalty : lj / a.rep_penalty;
                    argmax_merge(gv, gi, pen / a.temperature, i);
                }
                const float rm = wave_max_dpp(rv), gm = wave_max_dpp(gv);
                const int rmi = wave_min_dpp(rv == rm ? ri : 0x7fffffff);
                const int gmi = wave_min_dpp(gv == gm ? gi : 0x7fffffff);
                if (lane == 0) {   // (the previous readers of these slots passed many barriers ago)
                    sh.samp.sv[w] = rm; sh.samp.si[w] = rmi;
                    sh.samp.sv[8 + w] = gm; sh.samp.si[8 + w] = gmi;
                }
                if (!block_ok1(ok, sh)) return;
                rv = sh.samp.sv[0]; ri = sh.samp.si[0];
                gv = sh.samp.sv[8]; gi = sh.samp.si[8];
#pragma unroll
                for (int k = 1; k < PWV; ++k) {
                    argmax_merge(rv, ri, sh.samp.sv[k], sh.samp.si[k]);
                    argmax_merge(gv, gi, sh.samp.sv[8 + k], sh.samp.si[8 + k]);
                }
                raw = ri;
                tok = gi;
                STAMP1(1);
            } else {
                for (int i = tid; i < 1025; i += PT) sh.at.lg[i] = wait_gran(lgg + i, tag, a.err, ok, a.spin_ticks);
                if (!block_ok1(ok, sh)) return;
                STAMP1(1);
                tok = sample_block<PT>([&](int i) { return sh.at.lg[i]; }, sh.seen, 0, st + 1, a.top_k,
                                       a.temperature, a.rep_penalty, a.greedy, a.seed, 0, nullptr, &raw, sh.samp);
            }
            if (tid == 0) {
                a.y[ny0 + s] = tok;
                sh.seen[tok >> 5] |= 1u << (tok & 31);
                const int stop = (raw == 1024 || tok == 1024) ? 1 : 0;
                const int nst = st + 1;
                const bool fin = seq_finished(a.force_b, 0, a.force_steps, a.max_steps, nst, stop);
                last_stop = stop;
                last_fin = fin ? 1 : 0;
                bool go = true;
                if (sh.stopreq) stop_launch(a, go);   // no token: every waiting workgroup sees the error word
                else st_gran(ws.TK(s + 1), ws.tag(s + 1), __uint_as_float((unsigned)tok | (fin ? 1u << 16 : 0u)));
            }
            STAMP1(2);
            if (probe && tid < 16) a.trace[blockIdx.x * 16 + tid] = sh.stamp[tid];
        }
        ++n_exec;
    }
    // fused greedy at the launch's step cap: the last executed step's token is still unresolved
    if (fused && grp == 0 && n_exec == a.smax && n_exec > 0 && sh.fail == 0 && sh.fin == 0) {
        resolve_greedy(a, ws, n_exec, ny0, st0, publisher, sh, last_stop, last_fin);
        __syncthreads();
    }
    // ---- sequence state write-back (the workgroup that recorded the tokens)
    if (publisher && n_exec > 0 && sh.fail == 0) {
        __syncthreads();
        if (tid < 33) a.seen[tid] = sh.seen[tid];
        if (tid == 0) {
            a.ny[0] = ny0 + n_exec;
            a.steps[0] = st0 + n_exec;
            a.kvlen[0] = kv0 + n_exec;
            a.done[0] = (uint8_t)last_fin;
            if (a.stop_out) a.stop_out[0] = (uint8_t)last_stop;
        }
    }
}

// --------------------------------------------------------------------------
// FFN workgroup: hidden slice j of layers grp, grp + 8, grp + 16 (+ logits rows
// [64 j, 64 j + 64) in group LOGIT_GRP).
// --------------------------------------------------------------------------
__device__ void run_ffn(const PersistArgs& a, const Ws1& ws, Shared1& sh, int grp, int j) {
    const int tid = threadIdx.x, lane = tid & 63, ng = a.groups;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const bool logits = grp == LOGIT_GRP;
    const bool fused = a.greedy && a.knob[0] == 0;
    const int ny0 = a.ny[0], st0 = a.steps[0];
    int last_stop = 0, last_fin = 0;   // (unused by FFN workgroups)
    if (tid == 0) {
        sh.tok = (int)a.y[ny0 - 1];
        sh.fin = a.done[0] ? 1 : 0;
        sh.fail = 0;
    }
    if (logits && fused && tid < 33) sh.seen[tid] = a.seen[tid];   // the repetition penalty of its rows
    if (logits) {
        // rows 64 j + r (r < 64) and, on the last slice, the EOS row 1024 -- resident for the launch
        for (int e = tid; e < (LROWS + 1) * 64; e += PT) {
            const int r = e >> 6, c = e & 63;
            const int row = r < LROWS ? j * LROWS + r : 1024;
            sh.ff.wp[r][c] = (r < LROWS || j == NF - 1) ? ldg16(a.w_pred, (long)row * 512 + 8 * c)
                                                        : make_uint4(0u, 0u, 0u, 0u);
        }
        if (tid < LROWS + 16) {
            const int row = tid < LROWS ? j * LROWS + tid : 1024;
            const bool live = tid < LROWS || (tid == LROWS && j == NF - 1);
            sh.ff.lfB[tid] = live ? ldg(a.fold, LOGIT_FOLD + row) : 0.f;
            sh.ff.lfC[tid] = live ? ldg(a.fold, LOGIT_FOLD + 1025 + row) : 0.f;
        }
        sh.ff.lp23[0][tid] = ldg(a.L[23].b2, tid);
        sh.ff.lp23[1][tid] = ldg(a.L[23].n2w, tid);
        sh.ff.lp23[2][tid] = ldg(a.L[23].n2b, tid);
    }
    uint4 w1r[16], w2r[16];
    float bo = 0.f, n1w = 0.f, n1b = 0.f;    // out-proj bias and LN1 of layer l
    float ffB = 0.f, ffC = 0.f;              // folded LN1 vectors of this lane's FFN1 row
    auto prefetch = [&](int l) {
        const PLayer& P = a.L[l];
        // MFMA B fragments (lane: column lane & 15, k 8 (lane >> 4) .. + 8 of each 32-chunk)
        // FFN1: wave w -> hidden rows 128 j + 16 w + (lane & 15), K chunks c < 16
        const int n16 = lane & 15, k8 = 8 * (lane >> 4);
#pragma unroll
        for (int c = 0; c < 16; ++c) w1r[c] = ldg16(P.w1 + (long)(j * 128 + w * 16 + n16) * 512 + 32 * c + k8, 0);
        // FFN2: wave w -> output columns 64 w + 16 t + (lane & 15), hidden chunks 128 j + 32 c
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int c = 0; c < 4; ++c)
                w2r[4 * t + c] = ldg16(P.w2 + (long)(64 * w + 16 * t + n16) * 2048 + j * 128 + 32 * c + k8, 0);
        ffB = ldg(a.fold, (long)l * FOLD_LAYER + 3072 + j * 128 + w * 16 + n16);
        ffC = ldg(a.fold, (long)l * FOLD_LAYER + 5120 + j * 128 + w * 16 + n16);
        bo = ldg(P.b_out, tid); n1w = ldg(P.n1w, tid); n1b = ldg(P.n1b, tid);
        if (l > 0) dma_ln2(a.L[l - 1], sh, w, lane);
    };
    __syncthreads();
    if (sh.fin) return;
    prefetch(grp);
    for (int s = 0; s < a.smax; ++s) {
        if (!step_start(a, ws, s, grp == 0, sh, fused, logits && fused, false, ny0, st0, last_stop, last_fin))
            break;
        const unsigned tag = ws.tag(s);
        for (int l = grp; l < 24; l += ng) {
            const bool probe = a.trace && ((s == 8 && (l == 12 || l == 13 || l == 23)) || (s == 9 && l == 0));
            STAMP1(0);
            float xv;
            if (!form_x(a, ws, s, l, ny0 + s, &sh.p2[0][0], xv, sh, sh.tok)) return;
            STAMP1(1);
            // ---- v = x_l + (bo + sum_h PA[l][h]) (heads summed in order) -> lnb[1], and the
            // MFMA operand split of v * n1w: FFN1 runs on it while the LN1 statistics are
            // formed (W1 h1 + b1 = rden (W1 (v n1w) - mean W1 n1w) + (W1 n1b + b1), the
            // constant vectors folded at load time, as form_u)
            // (hop A: thread q < GQ sums heads 0..7 of granule column q, thread 256 + q
            // continues with heads 8..15 and forms the column group's v / operand split)
            {
                bool ok = true;
                constexpr int RB = (int)Ws1::ROW * 8;
                const int q = tid & 255, off = ws.PA(s, l, 0) + 16 * q;
                sh.ff.xr[tid] = xv;
                sh.ff.bo[tid] = bo;
                sh.ff.n1w[tid] = n1w;
                u32x4 g[8];
                if (tid < GQ) {
                    wait_g16_n<8>(ws, off, RB, tag, g, a.err, ok, a.spin_ticks);
                    float f0 = __uint_as_float(g[0].y), f1 = __uint_as_float(g[0].z), f2 = __uint_as_float(g[0].w);
#pragma unroll
                    for (int r = 1; r < 8; ++r) {
                        f0 += __uint_as_float(g[r].y);
                        f1 += __uint_as_float(g[r].z);
                        f2 += __uint_as_float(g[r].w);
                    }
                    sh.hs[3 * q] = f0; sh.hs[3 * q + 1] = f1; sh.hs[3 * q + 2] = f2;
                } else if (tid >= 256 && q < GQ) {
                    wait_g16_n<8>(ws, off + 8 * RB, RB, tag, g, a.err, ok, a.spin_ticks);
                }
                if (!block_ok1(ok, sh)) return;
                if (tid >= 256 && q < GQ) {
#pragma unroll
                    for (int k = 0; k < 3; ++k) {
                        if (k == 2 && gq_n(q) == 2) break;
                        float sum = sh.hs[3 * q + k];
#pragma unroll
                        for (int r = 0; r < 8; ++r) sum += __uint_as_float(g[r][1 + k]);
                        const int c = gq_col(q, k);
                        const float vc = sh.ff.xr[c] + (sh.ff.bo[c] + sum);
                        sh.lnb[1][c] = vc;
                        const float un = vc * sh.ff.n1w[c];
                        if (!split_h(un, sh.xh[c], sh.xl[c]) || !(fabsf(un) < a.f16_limit)) {
                            atomicCAS(a.err, 0, ERR_F16_RANGE);
                            ok = false;
                        }
                    }
                }
                if (!block_ok1(ok, sh)) return;
            }
            const float v = sh.lnb[1][tid];
            STAMP1(2);
            // ---- FFN1 rows of this slice on the MFMA (16 per wave), ReLU -> fh/fl.  The LN1
            // statistics come first in program order so the scheduler interleaves their
            // VALU work with the MFMAs (two waves per SIMD share its matrix pipe: the
            // MFMAs set the pace, the VALU slots are free)
            {
                const _Float16* ab = abase(sh.xh, sh.xl, lane);
                float mean, rden;
                ln_row_stats(sh.lnb[1], mean, rden);
                f32x4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int cb = 0; cb < 16; cb += 8) {   // 8 operand reads in flight, then 8 MFMAs
                    h8v af[8];
#pragma unroll
                    for (int i = 0; i < 8; ++i) af[i] = afrag(ab, 32 * (cb + i));
#pragma unroll
                    for (int i = 0; i < 8; i += 2) {
                        c0 = mfma16(af[i], bfrag(w1r[cb + i]), c0);
                        c1 = mfma16(af[i + 1], bfrag(w1r[cb + i + 1]), c1);
                    }
                }
                const float h1_pub = (v - mean) * rden * n1w + n1b;   // h1_l, published after the FFN2 partials
                if ((tid >> 5) == j) sh.h1s[tid & 31] = h1_pub;
                if (lane < 16) {
                    const float f = fmaxf(rden * (((c0[0] + c1[0]) + (c0[1] + c1[1])) - mean * ffB) + ffC, 0.f);
                    split_h(f, sh.fh[w * 16 + lane], sh.fl[w * 16 + lane]);
                    if (!(fabsf(f) < a.f16_limit)) {
                        atomicCAS(a.err, 0, ERR_F16_RANGE);
                        sh.fail = 1;
                    }
                }
            }
            STAMP1(6);
            __syncthreads();
            if (sh.fail) return;
            STAMP1(3);
            // ---- FFN2 slice on the MFMA (64 output columns per wave) -> partial granules
            {
                f32x4 acc[4];
#pragma unroll
                for (int t = 0; t < 4; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
                const _Float16* ab = abase(sh.fh, sh.fl, lane);
                h8v af[4];
#pragma unroll
                for (int c = 0; c < 4; ++c) af[c] = afrag(ab, 32 * c);
#pragma unroll
                for (int c = 0; c < 4; ++c)
#pragma unroll
                    for (int t = 0; t < 4; ++t) acc[t] = mfma16(af[c], bfrag(w2r[4 * t + c]), acc[t]);
                if (lane < 16) {
#pragma unroll
                    for (int t = 0; t < 4; ++t) sh.pk[w][16 * t + lane] = acc[t][0] + acc[t][1];
                }
                pub64(ws, sh, ws.PFH(s, l, j), tag, w, lane);
            }
            // h1 block j of this workgroup (the next layer's residual input: 11 granules),
            // after the partials: a store in flight stalls every later vmcnt(0)
            // (staged before the FFN1 barrier; the lane index is re-formed here so no
            // hoisted address waits in a spill slot: a reload's vmcnt(0) would wait for the
            // partials' write-through stores)
            if (w == 0) {
                int ln = lane;
                asm volatile("" : "+v"(ln));
                if (ln < 11) {
                    const float* p = sh.h1s + 3 * ln;
                    st_g16(ws, ws.PFH(s, l, 16) + 16 * (11 * j + ln), tag, p[0], p[1], ln == 10 ? 0.f : p[2]);
                }
            }
            STAMP1(4);
            __syncthreads();   // fs / b1 consumed before the next prefetch lands
            pf_wait(a.pf_delay);
            prefetch(l + ng < 24 ? l + ng : grp);
            if (probe && tid < 16) a.trace[blockIdx.x * 16 + tid] = sh.stamp[tid];
        }
        if (logits) {
            const bool probe = a.trace && s == 8;   // step-end trace (tools/knob_sweep.py)
            const int lane = opaque_tid() & 63;   // (the row / LDS offsets below: no spilled copies)
            STAMP1(0);
            // ---- logits rows (ar_predict_layer, no bias) of x_24 = LN2_23(h1_23 + b2 + sum PF_23)
            // on the MFMA, the LN2 folded through the rows as in form_u: wave w < 4 -> rows
            // 16 w .. + 16 of this slice, wave 4 of the last slice -> the EOS row
            if (!form_u(a, ws, s, 24, 0, &sh.ff.lp23[0][0], sh, 0)) return;
            STAMP1(1);
            if (w < 4 || (w == 4 && j == NF - 1)) {
                const _Float16* ab = abase(sh.xh, sh.xl, lane);
                float mean, rden;
                ln_row_stats(sh.lnb[0], mean, rden);   // first: interleaved with the MFMAs below
                const uint4* wb = &sh.ff.wp[min(16 * w + (lane & 15), LROWS)][lane >> 4];
                f32x4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int cb = 0; cb < 16; cb += 2) {   // few operands live: the FFN weights stay in registers
                    c0 = mfma16(afrag(ab, 32 * cb), bfrag(wb[4 * cb]), c0);
                    c1 = mfma16(afrag(ab, 32 * (cb + 1)), bfrag(wb[4 * (cb + 1)]), c1);
                }
                const int rl = 16 * w + lane;   // LROWS: the EOS row
                const float v = rden * (((c0[0] + c1[0]) + (c0[1] + c1[1])) - mean * sh.ff.lfB[min(rl, LROWS)]) +
                                sh.ff.lfC[min(rl, LROWS)];
                if (!fused) {
                    if (lane < 16 && (w < 4 || lane == 0)) st_gran(ws.LG(s) + (w < 4 ? j * LROWS + rl : 1024), tag, v);
                } else {
                    // greedy: this wave's 16 rows (wave 4: the EOS row alone) reduced to the first
                    // argmax of the penalised logits (K10 penalty over the seen tokens,
                    // / temperature) and of the raw ones: 4 granules of candidate q = 4 j + w
                    // (q = 64: the EOS row), no barrier
                    const int i = w < 4 ? j * LROWS + rl : 1024;
                    const bool live = w < 4 ? lane < 16 : lane == 0;
                    float pv = ((sh.seen[i >> 5] >> (i & 31)) & 1u) ? (v < 0.f ? v * a.rep_penalty : v / a.rep_penalty)
                                                                   : v;
                    pv = pv / a.temperature;
                    float gv = live ? pv : -INFINITY, rv = live ? v : -INFINITY;
                    int gi = live ? i : 0x7fffffff, ri = gi;
                    // 16-lane row reductions (row 0 holds the live lanes): value max, then the
                    // smallest index holding it
                    gv = fmaxf(gv, dpp_f<0xB1, 0xF>(gv)); rv = fmaxf(rv, dpp_f<0xB1, 0xF>(rv));
                    gv = fmaxf(gv, dpp_f<0x4E, 0xF>(gv)); rv = fmaxf(rv, dpp_f<0x4E, 0xF>(rv));
                    gv = fmaxf(gv, dpp_f<0x141, 0xF>(gv)); rv = fmaxf(rv, dpp_f<0x141, 0xF>(rv));
                    gv = fmaxf(gv, dpp_f<0x140, 0xF>(gv)); rv = fmaxf(rv, dpp_f<0x140, 0xF>(rv));
                    const float gm = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(gv)));
                    const float rm = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(rv)));
                    int gmi = (live && pv == gm) ? i : 0x7fffffff, rmi = (live && v == rm) ? i : 0x7fffffff;
                    gmi = min(gmi, dpp_i<0xB1, 0xF>(gmi)); rmi = min(rmi, dpp_i<0xB1, 0xF>(rmi));
                    gmi = min(gmi, dpp_i<0x4E, 0xF>(gmi)); rmi = min(rmi, dpp_i<0x4E, 0xF>(rmi));
                    gmi = min(gmi, dpp_i<0x141, 0xF>(gmi)); rmi = min(rmi, dpp_i<0x141, 0xF>(rmi));
                    gmi = min(gmi, dpp_i<0x140, 0xF>(gmi)); rmi = min(rmi, dpp_i<0x140, 0xF>(rmi));
                    if (lane < 4) {
                        const float out = lane == 0 ? gm : lane == 1 ? __int_as_float(gmi)
                                        : lane == 2 ? rm : __int_as_float(rmi);
                        st_gran(ws.LG(s) + 4 * (w < 4 ? 4 * j + w : 64) + lane, tag, out);
                    }
                }
            }
            STAMP1(2);
            if (probe && tid < 16) a.trace[blockIdx.x * 16 + tid] = sh.stamp[tid];
            __syncthreads();   // operands consumed before the next step's writes
        }
    }
}

#ifdef PERSIST1_MULTI
// ==========================================================================
// Several sequences in one launch (k_decode_persist1m, B = 2..MB): the same layer
// groups, two hand-offs per layer and weights in registers as the single-sequence
// kernel.  Each workgroup runs its owned layer for the live sequences one after
// another with the weights it loaded once: sequence b's hand-off is in flight while
// the workgroup works on sequence b + 1, so a step of B sequences costs about one
// sequence's chain plus (B - 1) workgroup passes -- not B chains.  The head's K/V
// rows of the next sequence are staged in LDS by LDS-DMA as soon as the current
// one's attention has read them.  Every per-sequence computation is the
// single-sequence kernel's (same code, same order), so each sequence's tokens are
// the ones a launch of its own gives.  Granule rows are per sequence (WsSeq), the
// token granules TK(s, b) carry each sequence's token and finished bit, and a
// finished sequence is skipped by every workgroup from the next step on.
// ==========================================================================
constexpr int MB = 64;   // sequences per multi-sequence launch (Shared1::m)
typedef unsigned long long u64m;

struct WsSeq {   // one sequence's view of the multi-sequence ring: Ws1's interface
    u64* ring;
    unsigned epoch;
    __amdgpu_buffer_rsrc_t rs;
    long slot_u64, oPFH, oLG, oTK;
    int nb, b;
    __device__ u64* slot(int s) const { return ring + (long)(s % RING1) * slot_u64; }
    __device__ unsigned tag(int s) const { return (epoch << 12) | (unsigned)(s + 1); }
    __device__ int PA(int s, int l, int h) const {   // rows 0..15: head partials; 16: x_l
        return (int)(((long)(s % RING1) * slot_u64 + ((long)(l * nb + b) * 17 + h) * Ws1::ROW) * 8);
    }
    __device__ int PFH(int s, int l, int j) const {
        return (int)(((long)(s % RING1) * slot_u64 + oPFH + ((long)(l * nb + b) * 17 + j) * Ws1::ROW) * 8);
    }
    __device__ const u64* at(int byte_off) const { return ring + byte_off / 8; }
    __device__ u64* LG(int s) const { return slot(s) + oLG + (long)b * PERSIST_LGS; }
    __device__ u64* TK(int s) const { return slot(s) + oTK + b; }
    __device__ WsSeq seq(int bb) const { WsSeq r = *this; r.b = bb; return r; }
};
// ring layout per step slot for nb sequences: PA [24][nb][17][GQ] (16 head partials + x_l),
// PFH [24][nb][17][GQ] (16-byte granules), LG [nb][PERSIST_LGS], TK [64] (8-byte granules);
// < 2^31 bytes at nb = 64
__host__ __device__ inline long wsm_oPFH(int nb) { return 24L * nb * 17 * Ws1::ROW; }
__host__ __device__ inline long wsm_oLG(int nb) { return wsm_oPFH(nb) + 24L * nb * 17 * Ws1::ROW; }
__host__ __device__ inline long wsm_oTK(int nb) { return wsm_oLG(nb) + (long)nb * PERSIST_LGS; }
__host__ __device__ inline long wsm_slot(int nb) { return wsm_oTK(nb) + MB; }

// Per-sequence state into LDS (thread b < nb).
__device__ __forceinline__ void init_m(const PersistArgs& a, Shared1& sh) {
    const int tid = threadIdx.x, nb = a.B;
    if (tid < nb) {
        const int b = tid, ny0 = a.ny[b];
        sh.m.ny0[b] = ny0;
        sh.m.kv0[b] = a.kvlen[b];
        sh.m.st0[b] = a.steps[b];
        sh.m.tok[b] = (int)a.y[(long)b * a.ldy + ny0 - 1];
        sh.m.act[b] = a.done[b] ? 0 : 1;
        sh.m.nexe[b] = 0;
        sh.m.lstop[b] = 0;
        sh.m.lfin[b] = a.done[b] ? 1 : 0;
        sh.m.kstep[b] = 0;
    }
    if (tid == 0) {
        sh.fail = 0;
        sh.stopreq = 0;
        sh.m.stop_s = -1;
    }
}
__device__ __forceinline__ u64m live_mask(const Shared1& sh, int nb) {
    u64m m = 0;
    for (int b = 0; b < nb; ++b) m |= sh.m.act[b] ? 1ull << b : 0ull;
    return m;
}

// Waves 3 and 7 issue every write-through store of the multi-sequence kernel (the
// granules, the K/V rows); the other six poll the hand-offs and run the LDS-DMA.  On
// CDNA a wave's vmcnt covers its stores and its loads in issue order, so a wave that
// polls next sequence's inputs right after publishing would wait for its stores'
// write-through round trip (~1 us) on every sequence.
__device__ __forceinline__ bool is_pub_wave(int w) { return w == 3 || w == 7; }


// The 512 partial columns the 8 waves staged in sh.pk (column c at flat index c) leave
// as the row's GQ granules at byte offset `row`, stored by waves 3 and 7 (88 each: two
// stores per lane); wave 7's idle lanes 40..50 of the second store carry the 11
// granules of the 32-column block in sh.h1s to byte offset blk (the FFN: its h1 block;
// attention: its block of x_l).  Every operand is read and held in registers before
// the first store: a spill reload after an sc1 store waits for it (~1 us).
template <class W>
__device__ __forceinline__ void pub_all(const W& ws, Shared1& sh, int row, unsigned tag, int w, int lane, int blk) {
    bar_nf();
    if (is_pub_wave(w)) {
        const float* pk = &sh.pk[0][0];
        const int q0 = (w == 3 ? 0 : 88) + lane, q1 = q0 + 64;
        const int c0 = gq_col(q0, 0);
        float a0 = pk[c0], a1 = pk[c0 + 1], a2 = gq_n(q0) == 2 ? 0.f : pk[c0 + 2];
        float b0 = 0.f, b1 = 0.f, b2 = 0.f;
        int o0 = row + 16 * q0, o1 = row + 16 * q1;
        bool second = lane < 24;
        if (second) {
            const int c1 = gq_col(q1, 0);
            b0 = pk[c1]; b1 = pk[c1 + 1]; b2 = gq_n(q1) == 2 ? 0.f : pk[c1 + 2];
        }
        if (w == 7 && lane >= 40 && lane < 51) {
            const int r = lane - 40;
            const float* p = sh.h1s + 3 * r;
            b0 = p[0]; b1 = p[1]; b2 = r == 10 ? 0.f : p[2];
            o1 = blk + 16 * r;
            second = true;
        }
        asm volatile("" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(b0), "+v"(b1), "+v"(b2), "+v"(o0), "+v"(o1));
        st_g16(ws, o0, tag, a0, a1, a2);
        if (second) st_g16(ws, o1, tag, b0, b1, b2);
    }
}

// The head's K/V rows [0, min(kv, KVL1)) of sequence b, layer l -> the LDS stage
// (LDS-DMA by the six non-publishing waves)
template <class SH>
__device__ __forceinline__ void stage_kv(const PersistArgs& a, SH& sh, int l, int b, int h, int kv, int w,
                                         int lane) {
    if (is_pub_wave(w)) return;
    const int wi = w < 3 ? w : w - 1;   // 0..5
    const long off = (long)b * a.sstride + (long)h * a.tmax * 32;
    const float* K = a.kc[l] + off;
    const float* V = a.vc[l] + off;
    const int nr = min(kv, KVL1), nch = (nr + 7) >> 3;
    for (int i = wi; i < nch; i += 6) {
        if (8 * i + (lane >> 3) < nr) {
            __builtin_amdgcn_global_load_lds(K + (long)i * 256 + lane * 4, sh.at.k + i * 256, 16, 0, 0);
            __builtin_amdgcn_global_load_lds(V + (long)i * 256 + lane * 4, sh.at.v + i * 256, 16, 0, 0);
        }
    }
}

// Fused greedy token of sequence b for step s - 1 (resolve_greedy's arithmetic on its
// own candidate granules LG(s - 1, b), polled directly: in the multi-sequence pipeline
// they are usually there already); the publisher appends it and publishes TK(s, b).
// Sets sh.m.tok[b] and sh.m.act[b]; ends with a barrier.
__device__ void resolve_m(const PersistArgs& a, const WsSeq& ws, int s, int b, bool publisher, Shared1& sh) {
    const int tid = threadIdx.x;
    bool ok = true;
    // the stop word, once per step (wave 1; tid 0 below may still see the previous step's
    // value: a stop takes effect within two steps)
    if (tid == 64 && sh.m.stop_s != s) {
        sh.stopreq = ld_stop(a.stop_req);
        sh.m.stop_s = s;
    }
    if (tid < 64) {
        float f[4];
        wait_gran_n<4>(ws.LG(s - 1) + 4 * tid, 1, ws.tag(s - 1), f, a.err, ok, a.spin_ticks);
        float gv = f[0], rv = f[2];
        int gi = __float_as_int(f[1]), ri = __float_as_int(f[3]);
        if (tid == 0) {
            float e[4];
            wait_gran_n<4>(ws.LG(s - 1) + 256, 1, ws.tag(s - 1), e, a.err, ok, a.spin_ticks);
            argmax_merge(gv, gi, e[0], __float_as_int(e[1]));
            argmax_merge(rv, ri, e[2], __float_as_int(e[3]));
        }
        const float gm = wave_max_dpp(gv), rm = wave_max_dpp(rv);
        const int tok = wave_min_dpp(gv == gm ? gi : 0x7fffffff);
        const int raw = wave_min_dpp(rv == rm ? ri : 0x7fffffff);
        if (tid == 0) {
            const int stop = (raw == 1024 || tok == 1024) ? 1 : 0;
            const bool fin = seq_finished(a.force_b, b, a.force_steps, a.max_steps, sh.m.st0[b] + s, stop);
            if (sh.stopreq) stop_launch(a, ok);
            sh.m.tok[b] = tok;
            sh.m.act[b] = fin ? 0 : 1;
            if (publisher && ok) {
                a.y[(long)b * a.ldy + sh.m.ny0[b] + s - 1] = tok;
                sh.m.lstop[b] = stop;
                sh.m.lfin[b] = fin ? 1 : 0;
                sh.m.nexe[b] = s;
                st_gran(ws.TK(s), ws.tag(s), __uint_as_float((unsigned)tok | (fin ? 1u << 16 : 0u)));
            }
        }
    }
    if (!ok) sh.fail = 1;
    bar_nf();
}

// Does sequence b run step s (s >= 1)?  Learned lazily, just before a workgroup's first
// owned layer of step s touches sequence b, so step s of one sequence starts while the
// others still finish step s - 1: group 0 with fused greedy resolves the token itself,
// every other workgroup reads the token granule TK(s, b) (sleeping on it).  The logits
// workgroups (`seenq`) mark the token in that sequence's seen bitmap.  Returns the
// block-uniform answer (false also on error).
__device__ __forceinline__ void take_tk(unsigned u, int b, int s, uint32_t (*seenq)[33], Shared1& sh) {
    const int tok = (int)(u & 0xffff);
    if (seenq) seenq[b][tok >> 5] |= 1u << (tok & 31);
    sh.m.tok[b] = tok;
    sh.m.act[b] = ((u >> 16) & 1) ? 0 : 1;
    sh.m.kstep[b] = s;
}
__device__ bool seq_runs(const PersistArgs& a, const WsSeq& base, int s, int b, unsigned long long live, bool grp0,
                         bool fused, bool publisher, uint32_t (*seenq)[33], Shared1& sh) {
    const int tid = threadIdx.x;
    if (fused && grp0) {
        resolve_m(a, base.seq(b), s, b, publisher, sh);
    } else if (sh.m.kstep[b] != s) {
        // one look at the token granules of every later live sequence whose status is
        // unknown (one round trip for many), then wait for sequence b's if it was not there
        if (tid >= b && tid < a.B && ((live >> tid) & 1ull) && sh.m.kstep[tid] != s) {
            const WsSeq ws = base.seq(tid);
            const u64 g = ld_rlxu64(ws.TK(s));
            if ((unsigned)g == ws.tag(s)) take_tk((unsigned)(g >> 32), tid, s, seenq, sh);   // {tag, value}
        }
        bar_nf();
        if (sh.m.kstep[b] != s) {
            if (tid == 0) {
                bool ok = true;
                const WsSeq ws = base.seq(b);
                wait_tag_slow(ws.TK(s), ws.tag(s), a.err, ok, a.spin_ticks);
                const float v = ok ? wait_gran(ws.TK(s), ws.tag(s), a.err, ok, a.spin_ticks) : 0.f;
                if (ok) take_tk(__float_as_uint(v), b, s, seenq, sh);
                else sh.fail = 1;
            }
            bar_nf();
        }
    }
    return sh.fail == 0 && sh.m.act[b] != 0;
}

__device__ void run_attn_m(const PersistArgs& a, const WsSeq& base, Shared1& sh, int grp, int h) {
    const int tid = threadIdx.x, lane = tid & 63, ng = a.groups, nb = a.B;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const bool fused = a.greedy && a.knob[0] == 0;
    // sampled decoding: head h's workgroup of group SAMPLER_GRP samples sequences h, h + 16, ...
    const bool sampler = !fused && grp == SAMPLER_GRP && h < nb;
    const bool publisher = fused && grp == 0 && h == 0;
    init_m(a, sh);
    if (sampler)
        for (int i = tid; i < 4 * 33; i += PT)
            if (h + 16 * (i / 33) < nb) sh.m.seens[i / 33][i % 33] = a.seen[(long)(h + 16 * (i / 33)) * 33 + i % 33];
    uint4 wq[16], wo[4];
    float qfB = 0.f, qfC = 0.f;
    auto prefetch = [&](int l) {   // the weights of owned layer l (as run_attn; no K/V)
        const PLayer& P = a.L[l];
        const int n16 = lane & 15, k8 = 8 * (lane >> 4);
        if (w < 6) {
            const int row = (w >> 1) * 512 + h * 32 + 16 * (w & 1) + n16;
#pragma unroll
            for (int c = 0; c < 16; ++c) wq[c] = ldg16(P.w_in + (long)row * 512 + 32 * c + k8, 0);
            qfB = ldg(a.fold, (long)l * FOLD_LAYER + row);
            qfC = ldg(a.fold, (long)l * FOLD_LAYER + 1536 + row);
        }
#pragma unroll
        for (int t = 0; t < 4; ++t) wo[t] = ldg16(P.w_out + (long)(64 * w + 16 * t + n16) * 512 + h * 32 + k8, 0);
        if (l > 0) dma_ln2<true>(a.L[l - 1], sh, w, lane);
    };
    auto next_live = [&](u64m live, int from) {   // the next live sequence at or after `from`, else -1
        const u64m m = from < 64 ? live >> from : 0ull;
        return m ? from + (int)__builtin_ctzll(m) : -1;
    };
    __syncthreads();
    u64m live = live_mask(sh, nb);
    __syncthreads();
    if (!live) return;
    int staged = -1;   // (layer, sequence) whose K/V rows are in the LDS stage: l * MB + b
    prefetch(grp);
    {
        const int b0 = next_live(live, 0);
        stage_kv(a, sh, grp, b0, h, sh.m.kv0[b0], w, lane);
        staged = grp * MB + b0;
    }
    int n_exec = 0;
    for (int s = 0; s < a.smax && live && sh.fail == 0; ++s) {
        const unsigned tag = base.tag(s);
        for (int l = grp; l < 24; l += ng) {
            for (int b = next_live(live, 0); b >= 0; b = next_live(live, b + 1)) {
                const WsSeq ws = base.seq(b);
                const int tid = opaque_tid(), lane = tid & 63;
                if (l == grp && s > 0 && !seq_runs(a, base, s, b, live, grp == 0, fused, publisher, nullptr, sh)) {
                    if (sh.fail) return;
                    live &= ~(1ull << b);   // finished: skipped from here on (by every workgroup)
                    continue;
                }
                const bool probe = a.trace && s == 8 && l == grp && b < 4;   // tools/ptrace_multi.py
                const bool pd = probe && b == 1;
#define MSTAMP(k) if (pd && tid == 0) sh.stamp[k] = __builtin_amdgcn_s_memrealtime()
                const unsigned long long t_in = probe ? __builtin_amdgcn_s_memrealtime() : 0ull;
                const int kv = sh.m.kv0[b] + s;
                if (staged != l * MB + b) {   // (a sequence that finished took the stage's turn)
                    stage_kv(a, sh, l, b, h, kv, w, lane);
                    staged = l * MB + b;
                }
                MSTAMP(0);
                if (!form_u<WsSeq, true>(a, ws, s, l, sh.m.ny0[b] + s, &sh.p2[0][0], sh, sh.m.tok[b],
                                         b == next_live(live, 0)))
                    return;
                if (w < 6) {
                    const _Float16* ab = abase(sh.xh, sh.xl, lane);
                    float mean, rden;
                    ln_row_stats(sh.lnb[0], mean, rden);
                    f32x4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                    for (int cb = 0; cb < 16; cb += 8) {
                        h8v af[8];
#pragma unroll
                        for (int i = 0; i < 8; ++i) af[i] = afrag(ab, 32 * (cb + i));
#pragma unroll
                        for (int i = 0; i < 8; i += 2) {
                            c0 = mfma16(af[i], bfrag(wq[cb + i]), c0);
                            c1 = mfma16(af[i + 1], bfrag(wq[cb + i + 1]), c1);
                        }
                    }
                    if (w == 0 && lane < 32) {   // x_l block h (form_x's arithmetic) for the FFN's PA row 16
                        const int c = 32 * h + lane;
                        sh.h1s[lane] = l > 0 ? ln_apply(sh.lnb[0][c], mean, rden, sh.p2[1][c], sh.p2[2][c])
                                             : sh.lnb[0][c];
                    }
                    mean = l > 0 ? mean : 0.f;
                    rden = l > 0 ? rden : 1.f;
                    if (lane < 16) {
                        const float val = rden * (((c0[0] + c1[0]) + (c0[1] + c1[1])) - mean * qfB) + qfC;
                        sh.qkv[16 * w + lane] = val;
                        if (kv < KVL1 && w >= 2) {
                            float* row = (w < 4 ? sh.at.k : sh.at.v) + kv * 32 + 16 * (w & 1);
                            row[lane] = val;
                        }
                    }
                }
                MSTAMP(1);
                if (!is_pub_wave(w)) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // its K/V LDS-DMA landed
                bar_nf();
                MSTAMP(2);
                const long kvoff = (long)b * a.sstride + (long)h * a.tmax * 32;
                float* Kw = a.kc[l] + kvoff;
                float* Vw = a.vc[l] + kvoff;
                const float sc = a.scale;
                const int T = kv + 1;
                const int c8 = lane & 7, g = (w << 3) | (lane >> 3);
                const float4 qc = *reinterpret_cast<const float4*>(sh.qkv + 4 * c8);
                const float q0 = qc.x * sc, q1 = qc.y * sc, q2 = qc.z * sc, q3 = qc.w * sc;
                const float4 knew = *reinterpret_cast<const float4*>(sh.qkv + 32 + 4 * c8);
                // the next sequence whose K/V this layer stages (at the first owned layer of
                // a step its status is not known yet: staged anyway, re-staged if it changed)
                const int bn = next_live(live, b + 1);
                if (T <= 512 && kv < KVL1) {
                    const int nu = (T + 63) >> 6;
                    if (nu <= 2) wave_attn1<2>(sh, q0, q1, q2, q3, sc, kv, T, c8, g, w, lane);
                    else if (nu <= 4) wave_attn1<4>(sh, q0, q1, q2, q3, sc, kv, T, c8, g, w, lane);
                    else if (nu == 5) wave_attn1<5>(sh, q0, q1, q2, q3, sc, kv, T, c8, g, w, lane);
                    else if (nu == 6) wave_attn1<6>(sh, q0, q1, q2, q3, sc, kv, T, c8, g, w, lane);
                    else wave_attn1<8>(sh, q0, q1, q2, q3, sc, kv, T, c8, g, w, lane);
                    bar_nf();   // the stage is read: the next sequence's K/V may land
                    if (bn >= 0) {
                        stage_kv(a, sh, l, bn, h, sh.m.kv0[bn] + s, w, lane);
                        staged = l * MB + bn;
                    }
                    merge_waves1(sh, w, lane);
                    MSTAMP(3);
                } else {
                    MSTAMP(3);
                    attn_general1<1>(sh, Kw, Vw, kv, T, q0, q1, q2, q3, sc, knew, c8, g, w, lane, tid);
                    bar_nf();
                    if (bn >= 0) {
                        stage_kv(a, sh, l, bn, h, sh.m.kv0[bn] + s, w, lane);
                        staged = l * MB + bn;
                    }
                }
                {
                    const h8v af = afrag(abase(sh.osh[w], sh.osl[w], lane), 0);
                    f32x4 acc[4];
#pragma unroll
                    for (int t = 0; t < 4; ++t) acc[t] = mfma16(af, bfrag(wo[t]), f32x4{0.f, 0.f, 0.f, 0.f});
                    if (lane < 16) {
#pragma unroll
                        for (int t = 0; t < 4; ++t) sh.pk[w][16 * t + lane] = acc[t][0] + acc[t][1];
                    }
                    MSTAMP(4);
                    pub_all(ws, sh, ws.PA(s, l, h), tag, w, lane, ws.PA(s, l, 16) + 16 * 11 * h);
                    MSTAMP(5);
                    if (w == 7) {   // the new K/V row (read by this workgroup only, next step)
                        if (lane < 32) Kw[(long)kv * 32 + lane] = sh.qkv[32 + lane];
                        else Vw[(long)kv * 32 + lane - 32] = sh.qkv[64 + lane - 32];
                    }
                }
                bar_nf();   // operands consumed before the next sequence writes them
                if (probe && tid == 0) {
                    a.trace[blockIdx.x * 16 + 2 * b] = t_in;
                    a.trace[blockIdx.x * 16 + 2 * b + 1] = __builtin_amdgcn_s_memrealtime();
                    if (pd)
                        for (int k = 0; k < 8; ++k) a.trace[blockIdx.x * 16 + 8 + k] = sh.stamp[k];
                }
            }
            // ---- next owned layer (this step) or the first one of the next step
            const int ln = l + ng < 24 ? l + ng : grp;
            pf_wait(a.pf_delay);
            prefetch(ln);
            const int b0 = next_live(live, 0);
            if (b0 >= 0 && staged != ln * MB + b0) {
                stage_kv(a, sh, ln, b0, h, sh.m.kv0[b0] + (l + ng < 24 ? s : s + 1), w, lane);
                staged = ln * MB + b0;
            }
        }
        // ---- sampler (sampled decoding): each of this workgroup's live sequences' logits of
        // this step -> token -> TK(s + 1, b)
        if (sampler) {
            for (int b = h; b < nb; b += 16) {
                if (!((live >> b) & 1ull)) continue;
                const WsSeq ws = base.seq(b);
                bool ok = true;
                if (tid == 0) wait_tag16_slow(ws.at(ws.PFH(s, 23, 0)), tag, a.err, ok, a.spin_ticks);
                if (tid == 64) sh.stopreq = ld_stop(a.stop_req);
                if (!block_ok1(ok, sh)) return;
                const u64* lgg = ws.LG(s);
                for (int i = tid; i < 1025; i += PT) sh.at.lg[i] = wait_gran(lgg + i, tag, a.err, ok, a.spin_ticks);
                if (!block_ok1(ok, sh)) return;
                const int st = sh.m.st0[b] + s;
                uint32_t* seen = sh.m.seens[b >> 4];
                int raw = 0;
                const int tok = sample_block<PT>([&](int i) { return sh.at.lg[i]; }, seen, b, st + 1, a.top_k,
                                                 a.temperature, a.rep_penalty, a.greedy, a.seed, 0, nullptr, &raw,
                                                 sh.samp);
                if (tid == 0) {
                    const int stop = (raw == 1024 || tok == 1024) ? 1 : 0;
                    const int fin = seq_finished(a.force_b, b, a.force_steps, a.max_steps, st + 1, stop) ? 1 : 0;
                    a.y[(long)b * a.ldy + sh.m.ny0[b] + s] = tok;
                    seen[tok >> 5] |= 1u << (tok & 31);
                    sh.m.lstop[b] = stop;
                    sh.m.lfin[b] = fin;
                    sh.m.nexe[b] = s + 1;
                    bool go = true;
                    if (sh.stopreq) stop_launch(a, go);
                    else st_gran(ws.TK(s + 1), ws.tag(s + 1), __uint_as_float((unsigned)tok | (fin ? 1u << 16 : 0u)));
                }
                __syncthreads();   // sh.at.lg / sh.samp consumed before the next sequence's
            }
        }
        ++n_exec;
    }
    // fused greedy at the launch's step cap: the live sequences' last tokens are unresolved
    if (fused && grp == 0 && n_exec == a.smax && n_exec > 0 && sh.fail == 0) {
        for (int b = next_live(live, 0); b >= 0; b = next_live(live, b + 1))
            resolve_m(a, base.seq(b), n_exec, b, publisher, sh);
    }
    // ---- sequence state write-back.  Fused: the publisher, every sequence (seen = the
    // launch's input bitmap | the tokens it appended, read back from y); sampled: each
    // sampler workgroup, its sequences (their bitmaps).
    if ((publisher || sampler) && sh.fail == 0) {
        if (tid == 0) __threadfence();   // the y stores of thread 0 have reached L2
        __syncthreads();
        for (int b = 0; b < nb; ++b) {
            if (sampler && (b & 15) != h) continue;
            const int ne = sh.m.nexe[b];
            if (ne <= 0) continue;
            if (tid < 33) {
                uint32_t word;
                if (sampler) {
                    word = sh.m.seens[b >> 4][tid];
                } else {
                    word = a.seen[(long)b * 33 + tid];
                    const int64_t* yb = a.y + (long)b * a.ldy + sh.m.ny0[b];
                    for (int i = 0; i < ne; ++i) {
                        const int t = (int)__hip_atomic_load(yb + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        if ((t >> 5) == tid) word |= 1u << (t & 31);
                    }
                }
                a.seen[(long)b * 33 + tid] = word;
            }
            if (tid == 0) {
                a.ny[b] = sh.m.ny0[b] + ne;
                a.steps[b] = sh.m.st0[b] + ne;
                a.kvlen[b] = sh.m.kv0[b] + ne;
                a.done[b] = (uint8_t)sh.m.lfin[b];
                if (a.stop_out) a.stop_out[b] = (uint8_t)sh.m.lstop[b];
            }
        }
    }
}

__device__ void run_ffn_m(const PersistArgs& a, const WsSeq& base, Shared1& sh, int grp, int j) {
    const int tid = threadIdx.x, lane = tid & 63, ng = a.groups, nb = a.B;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const bool logits = grp == LOGIT_GRP;
    const bool fused = a.greedy && a.knob[0] == 0;
    init_m(a, sh);
    if (logits && fused)
        for (int i = tid; i < nb * 33; i += PT) sh.ff.seenq[i / 33][i % 33] = a.seen[i];
    if (logits) {
        for (int e = tid; e < (LROWS + 1) * 64; e += PT) {
            const int r = e >> 6, c = e & 63;
            const int row = r < LROWS ? j * LROWS + r : 1024;
            sh.ff.wp[r][c] = (r < LROWS || j == NF - 1) ? ldg16(a.w_pred, (long)row * 512 + 8 * c)
                                                        : make_uint4(0u, 0u, 0u, 0u);
        }
        if (tid < LROWS + 16) {
            const int row = tid < LROWS ? j * LROWS + tid : 1024;
            const bool live = tid < LROWS || (tid == LROWS && j == NF - 1);
            sh.ff.lfB[tid] = live ? ldg(a.fold, LOGIT_FOLD + row) : 0.f;
            sh.ff.lfC[tid] = live ? ldg(a.fold, LOGIT_FOLD + 1025 + row) : 0.f;
        }
        sh.ff.lp23[0][tid] = ldg(a.L[23].b2, tid);
        sh.ff.lp23[1][tid] = ldg(a.L[23].n2w, tid);
        sh.ff.lp23[2][tid] = ldg(a.L[23].n2b, tid);
    }
    uint4 w1r[16], w2r[16];
    float bo = 0.f, n1w = 0.f, n1b = 0.f;
    float ffB = 0.f, ffC = 0.f;
    auto prefetch = [&](int l) {
        const PLayer& P = a.L[l];
        const int n16 = lane & 15, k8 = 8 * (lane >> 4);
#pragma unroll
        for (int c = 0; c < 16; ++c) w1r[c] = ldg16(P.w1 + (long)(j * 128 + w * 16 + n16) * 512 + 32 * c + k8, 0);
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int c = 0; c < 4; ++c)
                w2r[4 * t + c] = ldg16(P.w2 + (long)(64 * w + 16 * t + n16) * 2048 + j * 128 + 32 * c + k8, 0);
        ffB = ldg(a.fold, (long)l * FOLD_LAYER + 3072 + j * 128 + w * 16 + n16);
        ffC = ldg(a.fold, (long)l * FOLD_LAYER + 5120 + j * 128 + w * 16 + n16);
        bo = ldg(P.b_out, tid); n1w = ldg(P.n1w, tid); n1b = ldg(P.n1b, tid);
        if (l > 0) dma_ln2<true>(a.L[l - 1], sh, w, lane);
    };
    auto next_live = [&](u64m live, int from) {
        const u64m m = from < 64 ? live >> from : 0ull;
        return m ? from + (int)__builtin_ctzll(m) : -1;
    };
    __syncthreads();
    u64m live = live_mask(sh, nb);
    __syncthreads();
    if (!live) return;
    prefetch(grp);
    for (int s = 0; s < a.smax && live && sh.fail == 0; ++s) {
        const unsigned tag = base.tag(s);
        for (int l = grp; l < 24; l += ng) {
            for (int b = next_live(live, 0); b >= 0; b = next_live(live, b + 1)) {
                const WsSeq ws = base.seq(b);
                const int tid = opaque_tid(), lane = tid & 63;
                if (l == grp && s > 0 &&
                    !seq_runs(a, base, s, b, live, grp == 0, fused, false, logits && fused ? sh.ff.seenq : nullptr, sh)) {
                    if (sh.fail) return;
                    live &= ~(1ull << b);
                    continue;
                }
                const bool probe = a.trace && s == 8 && l == grp && b < 4;   // tools/ptrace_multi.py
                const bool pd = probe && b == 1;
                const unsigned long long t_in = probe ? __builtin_amdgcn_s_memrealtime() : 0ull;
                {
                    bool ok = true;
                    // the first live sequence: a sleeping lane waits for the layer's attention
                    // input (the head partials follow about one pass later), then all poll
                    if (b == next_live(live, 0)) {
                        if (tid == 0) wait_tag16_slow(ws.at(l > 0 ? ws.PFH(s, l - 1, 0) : ws.PA(s, 0, 0)), tag, a.err,
                                                      ok, a.spin_ticks);
                        if (!block_ok_t<true>(ok, sh)) return;
                    }
                    MSTAMP(0);
                    constexpr int RB = (int)Ws1::ROW * 8;
                    const int q = tid & 255, off = ws.PA(s, l, 0) + 16 * q;
                    sh.ff.bo[tid] = bo;
                    sh.ff.n1w[tid] = n1w;
                    u32x4 g[9];   // (second half: rows 8..15 and x_l)
                    if (tid < GQ) {
                        u32x4 h8[8];
                        wait_g16_n<8>(ws, off, RB, tag, h8, a.err, ok, a.spin_ticks);
                        float f0 = __uint_as_float(h8[0].y), f1 = __uint_as_float(h8[0].z), f2 = __uint_as_float(h8[0].w);
#pragma unroll
                        for (int r = 1; r < 8; ++r) {
                            f0 += __uint_as_float(h8[r].y);
                            f1 += __uint_as_float(h8[r].z);
                            f2 += __uint_as_float(h8[r].w);
                        }
                        sh.hs[3 * q] = f0; sh.hs[3 * q + 1] = f1; sh.hs[3 * q + 2] = f2;
                    } else if (tid >= 256 && q < GQ) {
                        wait_g16_n<9>(ws, off + 8 * RB, RB, tag, g, a.err, ok, a.spin_ticks);
                    }
                    if (!block_ok_t<true>(ok, sh)) return;
                    MSTAMP(1);
                    if (tid >= 256 && q < GQ) {
#pragma unroll
                        for (int k = 0; k < 3; ++k) {
                            if (k == 2 && gq_n(q) == 2) break;
                            float sum = sh.hs[3 * q + k];
#pragma unroll
                            for (int r = 0; r < 8; ++r) sum += __uint_as_float(g[r][1 + k]);
                            const int c = gq_col(q, k);
                            const float vc = __uint_as_float(g[8][1 + k]) + (sh.ff.bo[c] + sum);
                            sh.lnb[1][c] = vc;
                            const float un = vc * sh.ff.n1w[c];
                            if (!split_h(un, sh.xh[c], sh.xl[c]) || !(fabsf(un) < a.f16_limit)) {
                                atomicCAS(a.err, 0, ERR_F16_RANGE);
                                ok = false;
                            }
                        }
                    }
                    if (!block_ok_t<true>(ok, sh)) return;
                }
                MSTAMP(6);
                const float v = sh.lnb[1][tid];
                {
                    const _Float16* ab = abase(sh.xh, sh.xl, lane);
                    float mean, rden;
                    ln_row_stats(sh.lnb[1], mean, rden);
                    f32x4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                    for (int cb = 0; cb < 16; cb += 8) {
                        h8v af[8];
#pragma unroll
                        for (int i = 0; i < 8; ++i) af[i] = afrag(ab, 32 * (cb + i));
#pragma unroll
                        for (int i = 0; i < 8; i += 2) {
                            c0 = mfma16(af[i], bfrag(w1r[cb + i]), c0);
                            c1 = mfma16(af[i + 1], bfrag(w1r[cb + i + 1]), c1);
                        }
                    }
                    MSTAMP(7);
                    const float h1_pub = (v - mean) * rden * n1w + n1b;
                    if ((tid >> 5) == j) sh.h1s[tid & 31] = h1_pub;
                    if (lane < 16) {
                        const float f = fmaxf(rden * (((c0[0] + c1[0]) + (c0[1] + c1[1])) - mean * ffB) + ffC, 0.f);
                        split_h(f, sh.fh[w * 16 + lane], sh.fl[w * 16 + lane]);
                        if (!(fabsf(f) < a.f16_limit)) {
                            atomicCAS(a.err, 0, ERR_F16_RANGE);
                            sh.fail = 1;
                        }
                    }
                }
                bar_nf();
                MSTAMP(2);
                if (sh.fail) return;
                {
                    f32x4 acc[4];
#pragma unroll
                    for (int t = 0; t < 4; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
                    const _Float16* ab = abase(sh.fh, sh.fl, lane);
                    h8v af[4];
#pragma unroll
                    for (int c = 0; c < 4; ++c) af[c] = afrag(ab, 32 * c);
#pragma unroll
                    for (int c = 0; c < 4; ++c)
#pragma unroll
                        for (int t = 0; t < 4; ++t) acc[t] = mfma16(af[c], bfrag(w2r[4 * t + c]), acc[t]);
                    if (lane < 16) {
#pragma unroll
                        for (int t = 0; t < 4; ++t) sh.pk[w][16 * t + lane] = acc[t][0] + acc[t][1];
                    }
                    MSTAMP(3);
                    // with h1 block j (11 granules; staged before FFN1's barrier)
                    pub_all(ws, sh, ws.PFH(s, l, j), tag, w, lane, ws.PFH(s, l, 16) + 16 * 11 * j);
                    MSTAMP(4);
                }
                bar_nf();   // operands consumed before the next sequence writes them
                MSTAMP(5);
                if (probe && tid == 0) {
                    a.trace[blockIdx.x * 16 + 2 * b] = t_in;
                    a.trace[blockIdx.x * 16 + 2 * b + 1] = __builtin_amdgcn_s_memrealtime();
                    if (pd)
                        for (int k = 0; k < 8; ++k) a.trace[blockIdx.x * 16 + 8 + k] = sh.stamp[k];
                }
#undef MSTAMP
            }
            pf_wait(a.pf_delay);
            prefetch(l + ng < 24 ? l + ng : grp);
        }
        if (logits) {
            for (int b = next_live(live, 0); b >= 0; b = next_live(live, b + 1)) {
                const WsSeq ws = base.seq(b);
                if (!form_u<WsSeq, true>(a, ws, s, 24, 0, &sh.ff.lp23[0][0], sh, 0, b == next_live(live, 0))) return;
                if (w < 4 || (w == 4 && j == NF - 1)) {
                    const _Float16* ab = abase(sh.xh, sh.xl, lane);
                    float mean, rden;
                    ln_row_stats(sh.lnb[0], mean, rden);
                    const uint4* wb = &sh.ff.wp[min(16 * w + (lane & 15), LROWS)][lane >> 4];
                    f32x4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                    for (int cb = 0; cb < 16; cb += 2) {
                        c0 = mfma16(afrag(ab, 32 * cb), bfrag(wb[4 * cb]), c0);
                        c1 = mfma16(afrag(ab, 32 * (cb + 1)), bfrag(wb[4 * (cb + 1)]), c1);
                    }
                    const int rl = 16 * w + lane;
                    const float v = rden * (((c0[0] + c1[0]) + (c0[1] + c1[1])) - mean * sh.ff.lfB[min(rl, LROWS)]) +
                                    sh.ff.lfC[min(rl, LROWS)];
                    if (!fused) {
                        if (lane < 16 && (w < 4 || lane == 0)) sh.pk[w][lane] = v;   // (published by wave 7)
                    } else {
                        const int i = w < 4 ? j * LROWS + rl : 1024;
                        const bool lv = w < 4 ? lane < 16 : lane == 0;
                        const uint32_t* seen = sh.ff.seenq[b];
                        float pv = ((seen[i >> 5] >> (i & 31)) & 1u) ? (v < 0.f ? v * a.rep_penalty : v / a.rep_penalty) : v;
                        pv = pv / a.temperature;
                        float gv = lv ? pv : -INFINITY, rv = lv ? v : -INFINITY;
                        gv = fmaxf(gv, dpp_f<0xB1, 0xF>(gv)); rv = fmaxf(rv, dpp_f<0xB1, 0xF>(rv));
                        gv = fmaxf(gv, dpp_f<0x4E, 0xF>(gv)); rv = fmaxf(rv, dpp_f<0x4E, 0xF>(rv));
                        gv = fmaxf(gv, dpp_f<0x141, 0xF>(gv)); rv = fmaxf(rv, dpp_f<0x141, 0xF>(rv));
                        gv = fmaxf(gv, dpp_f<0x140, 0xF>(gv)); rv = fmaxf(rv, dpp_f<0x140, 0xF>(rv));
                        const float gm = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(gv)));
                        const float rm = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(rv)));
                        int gmi = (lv && pv == gm) ? i : 0x7fffffff, rmi = (lv && v == rm) ? i : 0x7fffffff;
                        gmi = min(gmi, dpp_i<0xB1, 0xF>(gmi)); rmi = min(rmi, dpp_i<0xB1, 0xF>(rmi));
                        gmi = min(gmi, dpp_i<0x4E, 0xF>(gmi)); rmi = min(rmi, dpp_i<0x4E, 0xF>(rmi));
                        gmi = min(gmi, dpp_i<0x141, 0xF>(gmi)); rmi = min(rmi, dpp_i<0x141, 0xF>(rmi));
                        gmi = min(gmi, dpp_i<0x140, 0xF>(gmi)); rmi = min(rmi, dpp_i<0x140, 0xF>(rmi));
                        if (lane < 4) {
                            const float out = lane == 0 ? gm : lane == 1 ? __int_as_float(gmi)
                                            : lane == 2 ? rm : __int_as_float(rmi);
                            sh.pk[w][lane] = out;   // (published by wave 7)
                        }
                    }
                }
                bar_nf();
                if (w == 7) {   // this slice's logits granules: 16 x 4 rows (+ the EOS row on the last slice)
                    const bool eos = j == NF - 1;
                    if (!fused) {
                        if (lane < 16) {
#pragma unroll
                            for (int ww = 0; ww < 4; ++ww) st_gran(ws.LG(s) + j * LROWS + 16 * ww + lane, tag, sh.pk[ww][lane]);
                        } else if (lane == 16 && eos) {
                            st_gran(ws.LG(s) + 1024, tag, sh.pk[4][0]);
                        }
                    } else if (lane < 16 || (lane < 20 && eos)) {
                        const int ww = lane >> 2, k = lane & 3;
                        st_gran(ws.LG(s) + 4 * (ww < 4 ? 4 * j + ww : 64) + k, tag, sh.pk[ww][k]);
                    }
                }
                bar_nf();   // operands consumed before the next sequence writes them
            }
        }
    }
}

#ifndef PERSIST1_NO_ENTRY   // (t2s_persistm.hip reuses the helpers above, not this kernel)
__global__ __launch_bounds__(PT) void k_decode_persist1m(PersistArgs a) {
    __shared__ Shared1 sh;
    WsSeq ws;
    ws.ring = a.ring;
    ws.epoch = a.epoch;
    ws.rs = __builtin_amdgcn_make_buffer_rsrc(a.ring, 0, 0x7fffffff, 0x00020000);
    ws.nb = a.B;
    ws.b = 0;
    ws.oPFH = wsm_oPFH(a.B);
    ws.oLG = wsm_oLG(a.B);
    ws.oTK = wsm_oTK(a.B);
    ws.slot_u64 = wsm_slot(a.B);
    const int grp = blockIdx.x / GW, r = blockIdx.x - grp * GW;
    if (r < 16) run_attn_m(a, ws, sh, grp, r);
    else run_ffn_m(a, ws, sh, grp, r - 16);
}
#endif

#else   // the single-sequence kernel

__global__ __launch_bounds__(PT) void k_decode_persist1(PersistArgs a) {
    __shared__ Shared1 sh;
    const Ws1 ws{a.ring, a.epoch, __builtin_amdgcn_make_buffer_rsrc(a.ring, 0, 0x7fffffff, 0x00020000)};
    const int grp = blockIdx.x / GW, r = blockIdx.x - grp * GW;
    if (r < 16) run_attn(a, ws, sh, grp, r);
    else run_ffn(a, ws, sh, grp, r - 16);
}
#endif

}  // namespace

#if defined(PERSIST1_MULTI) && defined(PERSIST1_NO_ENTRY)
#elif defined(PERSIST1_MULTI)
int persist1m_max_batch() { return MB; }
size_t persist1m_ring_bytes(int B) { return (size_t)wsm_slot(B) * RING1 * 8; }

hipError_t decode_persist1m(const PersistArgs& a, hipStream_t s, hipEvent_t start, hipEvent_t stop) {
    if (a.groups < 3 || a.groups > NG_MAX || a.B < 2 || a.B > MB) return hipErrorInvalidValue;
    hipExtLaunchKernelGGL(k_decode_persist1m, dim3(a.groups * GW), dim3(PT), 0, s, start, stop, 0, a);
    return hipGetLastError();
}

#else
int persist1_grid(int groups) { return groups * GW; }
int persist1_max_groups() { return NG_MAX; }

size_t persist1_ring_bytes() { return (size_t)Ws1::SLOT * RING1 * 8; }
hipError_t decode_persist1(const PersistArgs& a, hipStream_t s, hipEvent_t start, hipEvent_t stop) {
    if (a.groups < 3 || a.groups > NG_MAX) return hipErrorInvalidValue;   // groups 1, 2 own the logits, sampler
    hipExtLaunchKernelGGL(k_decode_persist1, dim3(a.groups * GW), dim3(PT), 0, s, start, stop, 0, a);
    return hipGetLastError();
}

#endif

}  // namespace gsv
