// Batched persistent decode (k_decode_persistm): the AR loop of the stage decoder
// (t2s_stage_decoder_fp32.onnx#43-114, loop Inference.py:95-106) for B sequences with
// the batch on the MFMA M dimension.
//
// The multi-sequence kernel k_decode_persist1m keeps each layer's weights in registers
// and runs the live sequences one after another through every workgroup: a step costs
// ~B workgroup passes of ~6 us (a hand-off round trip plus one sequence's compute), and
// at B = 64 the decode runs at 1.28 ms per step, ~18 % of its K/V-streaming bound.
// Here the chip is split into sequence GROUPS instead of layer groups:
//   group g (up to 16 of 16 workgroups each) decodes sequences b = g, g + G, g + 2G, ...
//   (at most MG = 4) through ALL 24 layers; workgroup r of the group is attention head r
//   AND FFN slice r (hidden units [128 r, 128 r + 128)).
// A layer is the single-sequence kernel's two hand-offs (head partials -> FFN, FFN2
// partials -> next layer), but every pass serves the group's sequences together:
//   - one gather round trip for all of them (one thread sums a granule column's 16 rows
//     in row order -- the arithmetic of gather_pfh's two threads);
//   - q/k/v, out-projection, FFN1, FFN2 and the logits as 16x16x32 MFMAs whose A rows
//     2i / 2i + 1 are sequence i's hi / lo split (t2s_persist1.hip puts one sequence's
//     hi / lo in rows 0 / 1; an MFMA output row depends on its own A row only, and the
//     K chains, folds and sums are the single-sequence kernel's, so every sequence's
//     values -- and tokens -- are bit-identical to its own launch);
//   - the weights stream from L2 once per pass (blocks r of every group sit on XCD r % 8,
//     so one XCD's L2 serves two heads' slices to 16 groups) instead of living in VGPRs.
// Attention stays per (sequence, head) with the single-sequence kernel's code (K/V rows
// staged in LDS by LDS-DMA, the new row from the q/k/v epilogue).  Greedy: every
// workgroup resolves its group's tokens from the logits candidates itself (one hop);
// sampled: workgroup i of the group samples sequence i.  Ring, tags, error word, stop
// word and sequence state are persist1m's (WsSeq), so the host treats both alike.
#define PERSIST1_MULTI
#define PERSIST1_NO_ENTRY
#include "t2s_persist1.hip"

namespace gsv {
namespace {

#ifndef PERSISTM_LATE_W
#define PERSISTM_LATE_W 0
#endif
constexpr int MG = 4;           // sequences per group
constexpr int NSG_MAX = 16;     // groups (x 16 workgroups: the whole chip)
constexpr int GWM = 16;         // workgroups per group
constexpr int AST = 512 + 8;    // A-tile row strides (halves; 16-B pad)
constexpr int FST = 128 + 8;
constexpr int OST = 32 + 8;

struct SharedM {
    struct {                                  // names as Shared1::at (the shared attention helpers)
        float k[KVL1 * 32];                   // K/V rows [0, min(kv, KVL1)) of (layer, sequence, head r)
        float v[KVL1 * 32];
        float ov[16][32];
        float ov4[PWV][32];
        union {
            float p[TMAX1];                   // general-path scores
            struct {
                _Float16 A[2 * MG][AST];      // MFMA A tile: rows 2i / 2i + 1 = hi / lo of sequence i's input
                float lnb[MG][512];           // the input rows (LayerNorm statistics)
            } g;
            float pk[MG][512];                // the rows a pass publishes
            float lg[1056];                   // sampler: one sequence's logits
        };
    } at;
    _Float16 F[2 * MG][FST];                  // FFN2's A tile (FFN1 outputs)
    _Float16 O[2 * MG][OST];                  // the out-projection's A tile (head outputs)
    float qkvs[MG][96];                       // head r's q, k, v per sequence
    float qkv[96];                            // ... of the sequence in attention (the helpers' operand)
    _Float16 osh[PWV][32], osl[PWV][32];      // merge_waves1's per-wave head output
    float h1s[MG][32];                        // block r of the published x_l / h1 rows
    float ovm[MG][PWV][32];                   // concurrent attention: wave w's partial o of sequence i
    float wredm[MG][2][PWV];                  // ... and its m_w, l_w
    float cand[MG][5][4];                     // greedy candidates of this slice's 4 waves + EOS
    float wred[2][PWV];
    uint32_t seenq[MG][33];
    int tok[MG], act[MG], ny0[MG], kv0[MG], st0[MG], nexe[MG], lstop[MG], lfin[MG];
    int fail, stopreq;
    SampleLds<PT> samp;
};

__device__ __forceinline__ int nth_bit(unsigned m, int n) {   // index of the n-th set bit of m
    for (int k = 0; k < n; ++k) m &= m - 1;
    return __builtin_ctz(m);
}
// lane's A-operand base in a tile of 2 MG rows (rows 8..15 of the MFMA repeat 0..7; unused)
__device__ __forceinline__ const _Float16* abase_m(const _Float16* tile, int stride, int lane) {
    return tile + (lane & 7) * stride + 8 * (lane >> 4);
}
// hi + lo split of the product u m, as the single-sequence kernel's compiled split of
// `un = u * m; split_h(un, ...)` computes it: hipcc contracts the product into the
// conversions there, hi = f16(u m) and lo = f16(u m - hi) with the product exact (two
// v_fma_mixlo_f16), which differs from converting the f32-rounded product when u m
// sits at an f16 rounding tie.  Written out here so every sequence's operands -- and
// values -- are the single kernel's bit for bit (profiles/r05x_persist1m_deviation.txt).
__device__ __forceinline__ void split_mul_h(float u, float m, _Float16& hi, _Float16& lo) {
    unsigned h, l;
    asm("v_fma_mixlo_f16 %0, %1, %2, 0" : "=v"(h) : "v"(u), "v"(m));
    asm("v_fma_mixlo_f16 %0, %1, %2, -%3 op_sel_hi:[0,0,1]" : "=v"(l) : "v"(u), "v"(m), "v"(h));
    hi = __builtin_bit_cast(_Float16, (unsigned short)(h & 0xffffu));
    lo = __builtin_bit_cast(_Float16, (unsigned short)(l & 0xffffu));
}

// wait_g16_n (t2s_persist1.hip) with the error word and the wait bound checked every 4th poll:
// the group-wide gathers resolve within a few dozen polls, so a check every 64th (the
// single-sequence kernel's) never fired and a forced timeout could not be tested
template <int N>
__device__ __forceinline__ void wait_g16_m(const WsSeq& ws, int off, int stride, unsigned tag, u32x4 (&g)[N],
                                           int* err, bool& ok, unsigned long long ticks) {
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
        if ((it & 3) == 3) {
            if (ld_rlx(err) != 0) { ok = false; break; }
            if (__builtin_amdgcn_s_memrealtime() - t0 > ticks) {
                atomicCAS(err, 0, 1);
                ok = false;
                break;
            }
        }
    }
}

__device__ __forceinline__ bool ok_all(bool ok, SharedM& sh) {
    if (!ok) sh.fail = 1;
    bar_nf();
    return sh.fail == 0;
}

// tools/ptrace_pm.py: phase stamps of step 8 (layer 12 and the step's ends), slot k of this
// workgroup's 16, 100 MHz clock
#define PMSTAMP(cond, k)                                                                        \
    do {                                                                                        \
        if (a.trace && s == 8 && (cond) && threadIdx.x == 0)                                    \
            a.trace[blockIdx.x * 16 + (k)] = __builtin_amdgcn_s_memrealtime();                  \
    } while (0)

// The 17-row granule blocks of the live sequences (byte offsets blk(i) of row 0; rows
// 0..15 partials, row 16 the residual row) -> u = row16 + (vec[c] + sum of rows 0..15
// in row order) into lnb[i], the fp16 split of u * mul[c] into A rows 2i, 2i + 1.  One
// thread per (sequence, granule column) in two round trips (rows 0..8, then 9..16: 17
// granules in flight make hipcc spill the whole array); vec / mul are loaded first.
// Ends with a barrier.
template <class Blk>
__device__ __forceinline__ bool gather_m(const PersistArgs& a, const WsSeq& ws, SharedM& sh, unsigned live,
                                         unsigned tag, Blk blk, const float* vec, const float* mul, bool dbg_ffn = false) {
    constexpr int RB = (int)Ws1::ROW * 8;
    const int nl = __builtin_popcount(live);
    bool ok = true;
    for (int it = opaque_tid(); it < nl * GQ; it += PT) {
        const int n = it / GQ, q = it - n * GQ;
        const int i = nth_bit(live, n);
        const int off = blk(i) + 16 * q;
        float vv[3], mm[3];   // in flight beside the granules
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const int c = gq_col(q, min(k, gq_n(q) - 1));
            vv[k] = ldg(vec, c);
            mm[k] = ldg(mul, c);
        }
        float f[3];
        {
            u32x4 g[9];
            wait_g16_m<9>(ws, off, RB, tag, g, a.err, ok, a.spin_ticks);
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                f[k] = __uint_as_float(g[0][1 + k]);
#pragma unroll
                for (int r = 1; r < 9; ++r) f[k] += __uint_as_float(g[r][1 + k]);
            }
        }
        if (!ok) break;
        u32x4 g[8];
        wait_g16_m<8>(ws, off + 9 * RB, RB, tag, g, a.err, ok, a.spin_ticks);
        if (!ok) break;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            if (k == 2 && gq_n(q) == 2) break;
#pragma unroll
            for (int r = 0; r < 7; ++r) f[k] += __uint_as_float(g[r][1 + k]);
            const int c = gq_col(q, k);
            const float u = __uint_as_float(g[7][1 + k]) + (vv[k] + f[k]);
            sh.at.g.lnb[i][c] = u;
            const float un = u * mm[k];
            _Float16 hi, lo;
            split_mul_h(u, mm[k], hi, lo);
            if (!(fabsf(un) < 65504.f) || !(fabsf(un) < a.f16_limit)) {   // (split_h's range test)
                atomicCAS(a.err, 0, ERR_F16_RANGE);
                ok = false;
            }
#ifdef PERSIST_DBG
            if (a.knob[3] == 12 && dbg_ffn && i == 0) {
                float* tf = reinterpret_cast<float*>(a.trace);
                tf[3000 + c] = un; tf[3512 + c] = (float)hi; tf[4024 + c] = u; tf[4536 + c] = mm[k];
            }
#endif
            sh.at.g.A[2 * i][c] = hi;
            sh.at.g.A[2 * i + 1][c] = lo;
        }
    }
    return ok_all(ok, sh);
}

// LayerNorm statistics of the live sequences' rows (every wave, the same order)
__device__ __forceinline__ void stats_m(const SharedM& sh, unsigned live, float (&mean)[MG], float (&rden)[MG]) {
#pragma unroll
    for (int i = 0; i < MG; ++i) {
        mean[i] = 0.f;
        rden[i] = 1.f;
        if ((live >> i) & 1u) ln_row_stats(sh.at.g.lnb[i], mean[i], rden[i]);
    }
}

// Sequence i's row of 512 published columns (pk[i]) as its GQ granules at byte offset
// `row`, and its 32-column block h1s[i] (11 granules) at `blk`; waves 3 and 7 store
// (persist1m's pub_all layout).  Every operand is in registers before the first store.
__device__ __forceinline__ void pub_m(const WsSeq& ws, SharedM& sh, int i, int row, int blk, unsigned tag, int w,
                                      int lane) {
    if (!is_pub_wave(w)) return;
    const float* pk = sh.at.pk[i];
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
        const float* p = sh.h1s[i] + 3 * r;
        b0 = p[0]; b1 = p[1]; b2 = r == 10 ? 0.f : p[2];
        o1 = blk + 16 * r;
        second = true;
    }
    asm volatile("" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(b0), "+v"(b1), "+v"(b2), "+v"(o0), "+v"(o1));
    st_g16(ws, o0, tag, a0, a1, a2);
    if (second) st_g16(ws, o1, tag, b0, b1, b2);
}

// ---- attention with a double-buffered K stage: the K rows of the next sequence land in one
// LDS buffer while this sequence's attention reads the other; V rows are read from memory
// by the lanes that weigh them (issued first, in flight during the scores).  The arithmetic
// is wave_attn1's / attn_general1's (t2s_persist1.hip) operation for operation: only where
// the operands come from differs, so every value is the single-sequence kernel's.

// K rows [0, min(kv, KVL1)) of (layer l, sequence b, head h) -> LDS buffer dst by LDS-DMA
// (the six non-publishing waves)
__device__ __forceinline__ void stage_k(const PersistArgs& a, float* dst, int l, int b, int h, int kv, int w,
                                        int lane) {
    if (is_pub_wave(w)) return;
    const int wi = w < 3 ? w : w - 1;
    const float* K = a.kc[l] + (long)b * a.sstride + (long)h * a.tmax * 32;
    const int nr = min(kv, KVL1), nch = (nr + 7) >> 3;
    for (int i = wi; i < nch; i += 6) {
        if (8 * i + (lane >> 3) < nr) {
            // from inline asm: the waitcnt pass would put a vmcnt(0) before every LDS read of
            // the attention running beside this DMA (it cannot tell the two K buffers apart),
            // i.e. wait for the next sequence's rows; the wait is the explicit one before use
            const unsigned la = __builtin_amdgcn_readfirstlane(
                (unsigned)(size_t)(__attribute__((address_space(3))) char*)(dst + i * 256));
            // (M0 bound as an operand, so the compiler sets and tracks it)
            asm volatile("global_load_lds_dwordx4 %1, off" ::"{m0}"(la), "v"(K + (long)i * 256 + lane * 4) : "memory");
        }
    }
}

// This lane's V rows t = min(64 u + g, kv) (u < 8) of one sequence: rows < kv from memory,
// row kv (and the clamped ones past it) the new row -- the values the LDS stage held.
__device__ __forceinline__ void load_v8(float4 (&vr)[8], const float* Vw, float4 vnew, int kv, int c8, int g) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
        const int t = min(64 * u + g, kv);
        vr[u] = t < kv ? ldg16f(Vw, (long)t * 32 + 4 * c8) : vnew;
    }
}

template <int NU>
__device__ __forceinline__ void wave_attn_m(SharedM& sh, const float* Ks, const float4 (&vr)[8], float q0,
                                            float q1, float q2, float q3, float sc, int kv, int T, int c8, int g,
                                            int w, int lane) {
    float4 kr[NU];
#pragma unroll
    for (int u = 0; u < NU; ++u) kr[u] = *reinterpret_cast<const float4*>(Ks + min(64 * u + g, kv) * 32 + 4 * c8);
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
    float wm = -INFINITY;
#pragma unroll
    for (int u = 0; u < NU; ++u) {
        sv[u] = 64 * u + g < T ? sv[u] : -INFINITY;
        wm = fmaxf(wm, sv[u]);
    }
    const float m_w = wave_max_dpp(wm);
    const float mref = m_w == -INFINITY ? 0.f : m_w;
    float o0 = 0.f, o1 = 0.f, o2 = 0.f, o3 = 0.f, lsum = 0.f;
#pragma unroll
    for (int u = 0; u < NU; ++u) {
        const float pu = __expf(sv[u] - mref);
        const float4 v4 = vr[u];
        o0 += pu * v4.x;
        o1 += pu * v4.y;
        o2 += pu * v4.z;
        o3 += pu * v4.w;
        lsum += pu;
    }
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

__device__ __noinline__ float scores_general_m(SharedM& sh, const float* Ks, const float* Kw, int kv, int T, float q0,
                                               float q1, float q2, float q3, float sc, float4 knew, int c8, int g) {
    float lmax = -INFINITY;
    for (int base = 0; base < T; base += 512) {
        float sv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int t = base + 64 * u + g;
            float4 kr;
            if (t < kv && t < KVL1) kr = *reinterpret_cast<const float4*>(Ks + t * 32 + 4 * c8);
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

__device__ __noinline__ void attn_general_m(SharedM& sh, const float* Ks, const float* Kw, const float* Vw, int kv,
                                            int T, float q0, float q1, float q2, float q3, float sc, float4 knew,
                                            int c8, int g, int w, int lane, int tid) {
    const float lmax = scores_general_m(sh, Ks, Kw, kv, T, q0, q1, q2, q3, sc, knew, c8, g);
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
            for (int u = 0; u < 4; ++u) o4[u] += sh.at.p[t + 16 * u] * ldg(Vw, (long)(t + 16 * u) * 32 + d);
        }
        for (; t < tl; t += 16) o4[0] += sh.at.p[t] * ldg(Vw, (long)t * 32 + d);
        for (; t < kv; t += 16) o4[1] += sh.at.p[t] * ldg(Vw, (long)t * 32 + d);
        if (t == kv) o4[2] += sh.at.p[t] * sh.qkv[64 + d];
        sh.at.ov[kg][d] = (o4[0] + o4[1]) + (o4[2] + o4[3]);
    }
    __syncthreads();
    if (lane < 32) {
        float O = 0.f, L = 0.f;
#pragma unroll
        for (int kg = 0; kg < 16; ++kg) O += sh.at.ov[kg][lane];
#pragma unroll
        for (int ww = 0; ww < PWV; ++ww) L += sh.wred[1][ww];
        split_h(O / L, sh.osh[w][lane], sh.osl[w][lane]);
    }
    __builtin_amdgcn_wave_barrier();
}

// Greedy token of step s - 1 of group sequence i (global b), resolved by ONE wave from
// the logits candidates LG(s - 1) (resolve_m's arithmetic).  Lane 0 updates the state.
__device__ void resolve_w(const PersistArgs& a, const WsSeq& ws, int s, int i, int b, bool publisher, SharedM& sh,
                          bool& ok) {
    const int lane = threadIdx.x & 63;
    float f[4];
    wait_gran_n<4>(ws.LG(s - 1) + 4 * lane, 1, ws.tag(s - 1), f, a.err, ok, a.spin_ticks);
    float gv = f[0], rv = f[2];
    int gi = __float_as_int(f[1]), ri = __float_as_int(f[3]);
    if (lane == 0) {
        float e[4];
        wait_gran_n<4>(ws.LG(s - 1) + 256, 1, ws.tag(s - 1), e, a.err, ok, a.spin_ticks);
        argmax_merge(gv, gi, e[0], __float_as_int(e[1]));
        argmax_merge(rv, ri, e[2], __float_as_int(e[3]));
    }
    const float gm = wave_max_dpp(gv), rm = wave_max_dpp(rv);
    const int tok = wave_min_dpp(gv == gm ? gi : 0x7fffffff);
    const int raw = wave_min_dpp(rv == rm ? ri : 0x7fffffff);
    if (lane == 0) {
        const int stop = (raw == 1024 || tok == 1024) ? 1 : 0;
        const bool fin = seq_finished(a.force_b, b, a.force_steps, a.max_steps, sh.st0[i] + s, stop);
        if (sh.stopreq) stop_launch(a, ok);
        sh.tok[i] = tok;
        sh.act[i] = fin ? 0 : 1;
        sh.seenq[i][tok >> 5] |= 1u << (tok & 31);
        if (publisher && ok) {
            a.y[(long)b * a.ldy + sh.ny0[i] + s - 1] = tok;
            sh.lstop[i] = stop;
            sh.lfin[i] = fin ? 1 : 0;
            sh.nexe[i] = s;
            st_gran(ws.TK(s), ws.tag(s), __uint_as_float((unsigned)tok | (fin ? 1u << 16 : 0u)));
        }
    }
}

// ---- concurrent attention (every live sequence of the group at once): wave w computes its
// share -- keys t = 64 u + 8 w + lane / 8, wave_attn1's partition -- of EVERY live sequence's
// head-r attention, K and V rows straight from memory into registers (row kv, the new one, from
// the q/k/v results; rows past it read row kv and weigh 0), the next sequence's rows in flight
// while this one is computed; then one barrier and one wave per sequence merges the 8 partials.
// wave_part_m / merge_m are wave_attn_m / merge_waves1 operation for operation (operands from
// registers instead of the LDS stage), so every value is the single-sequence kernel's.  The
// serial loop paid a K stage, two barriers and a merge per sequence (~2.6 us each, four per
// layer, profiles/r05t_persistm_trace64.json).  Rounds u >= ceil(T / 64) are masked to
// exp(-inf) = 0 and add exact zeros, so one NU serves every live sequence.
template <int NU>
__device__ __forceinline__ void load_kv_m(float4 (&kr)[NU], float4 (&vr)[NU], const float* Kw, const float* Vw,
                                          float4 knew, float4 vnew, int kv, int c8, int g) {
#pragma unroll
    for (int u = 0; u < NU; ++u) {
        const int t = min(64 * u + g, kv);
        kr[u] = t < kv ? ldg16f(Kw, (long)t * 32 + 4 * c8) : knew;
        vr[u] = t < kv ? ldg16f(Vw, (long)t * 32 + 4 * c8) : vnew;
    }
}

template <int NU>
__device__ __forceinline__ void wave_part_m(SharedM& sh, int i, const float4 (&kr)[NU], const float4 (&vr)[NU],
                                            float q0, float q1, float q2, float q3, float sc, int T, int c8, int g,
                                            int w, int lane) {
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
    float wm = -INFINITY;
#pragma unroll
    for (int u = 0; u < NU; ++u) {
        sv[u] = 64 * u + g < T ? sv[u] : -INFINITY;
        wm = fmaxf(wm, sv[u]);
    }
    const float m_w = wave_max_dpp(wm);
    const float mref = m_w == -INFINITY ? 0.f : m_w;
    float o0 = 0.f, o1 = 0.f, o2 = 0.f, o3 = 0.f, lsum = 0.f;
#pragma unroll
    for (int u = 0; u < NU; ++u) {
        const float pu = __expf(sv[u] - mref);
        const float4 v4 = vr[u];
        o0 += pu * v4.x;
        o1 += pu * v4.y;
        o2 += pu * v4.z;
        o3 += pu * v4.w;
        lsum += pu;
    }
    o0 += dpp_f<0x128, 0xF>(o0);
    o1 += dpp_f<0x128, 0xF>(o1);
    o2 += dpp_f<0x128, 0xF>(o2);
    o3 += dpp_f<0x128, 0xF>(o3);
    o0 = swap_sum16(o0); o1 = swap_sum16(o1); o2 = swap_sum16(o2); o3 = swap_sum16(o3);
    o0 = swap_sum32(o0); o1 = swap_sum32(o1); o2 = swap_sum32(o2); o3 = swap_sum32(o3);
    const float l_w = wave_sum_dpp(c8 == 0 ? lsum : 0.f);
    if (lane < 8) *reinterpret_cast<float4*>(&sh.ovm[i][w][4 * lane]) = make_float4(o0, o1, o2, o3);
    if (lane == 0) {
        sh.wredm[i][0][w] = m_w;
        sh.wredm[i][1][w] = l_w;
    }
}

// PF: the next sequence's rows in flight during this one's share (NU <= 4; at NU = 7 the two
// register sets spilled, so longer rows are loaded one sequence at a time)
template <int NU, bool PF = (NU <= 4)>
__device__ void attn_conc_m(const PersistArgs& a, SharedM& sh, unsigned live, int g, int nsg, int r, int l, int s,
                            int w, int lane) {
    const int c8 = lane & 7, gk = (w << 3) | (lane >> 3);
    const float sc = a.scale;
    constexpr int NB = PF ? NU : 1;
    float4 kA[NU], vA[NU], kB[NB], vB[NB];
    auto ld = [&](int i, float4 (&kk)[NU], float4 (&vv)[NU]) {
        const long off = (long)(g + i * nsg) * a.sstride + (long)r * a.tmax * 32;
        load_kv_m<NU>(kk, vv, a.kc[l] + off, a.vc[l] + off, *reinterpret_cast<const float4*>(&sh.qkvs[i][32 + 4 * c8]),
                      *reinterpret_cast<const float4*>(&sh.qkvs[i][64 + 4 * c8]), sh.kv0[i] + s, c8, gk);
    };
    unsigned m = live;
    int i = __builtin_ctz(m);
    ld(i, kA, vA);
    for (;;) {
        const unsigned nx = m & (m - 1);
        if constexpr (PF)
            if (nx) ld(__builtin_ctz(nx), kB, vB);   // in flight during this sequence's share
        const float4 qc = *reinterpret_cast<const float4*>(&sh.qkvs[i][4 * c8]);
        wave_part_m<NU>(sh, i, kA, vA, qc.x * sc, qc.y * sc, qc.z * sc, qc.w * sc, sc, sh.kv0[i] + s + 1, c8, gk, w,
                        lane);
        if (!nx) break;
        m = nx;
        i = __builtin_ctz(m);
        if constexpr (PF) {
#pragma unroll
            for (int u = 0; u < NU; ++u) {
                kA[u] = kB[u];
                vA[u] = vB[u];
            }
        } else {
            ld(i, kA, vA);
        }
    }
}

// merge_waves1's arithmetic for sequence i, by one wave, into the out-projection's A tile
// (rows 2 i / 2 i + 1 = hi / lo of the head output)
__device__ __forceinline__ void merge_m(SharedM& sh, int i, int lane) {
    const int j = lane & 7;
    const float mj = sh.wredm[i][0][j];
    float M = mj;
    M = fmaxf(M, dpp_f<0xB1, 0xF>(M));
    M = fmaxf(M, dpp_f<0x4E, 0xF>(M));
    M = fmaxf(M, dpp_f<0x141, 0xF>(M));
    const float e = mj == -INFINITY ? 0.f : __expf(mj - M);
    float L = e * sh.wredm[i][1][j];
    L += dpp_f<0xB1, 0xF>(L);
    L += dpp_f<0x4E, 0xF>(L);
    L += dpp_f<0x141, 0xF>(L);
    const int d = lane & 31;
    float O = 0.f;
#pragma unroll
    for (int ww = 0; ww < PWV; ++ww)
        O += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(e), ww)) * sh.ovm[i][ww][d];
    if (lane < 32) split_h(O / L, sh.O[2 * i][d], sh.O[2 * i + 1][d]);
}

__device__ void run_group(const PersistArgs& a, const WsSeq& base, SharedM& sh, int g, int r) {
    const int nsg = a.groups, nb = a.B;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nloc = g < nb ? (nb - g + nsg - 1) / nsg : 0;   // this group's sequences: b = g + i nsg
    const bool fused = a.greedy && a.knob[0] == 0;
    const bool publisher = fused && r == 0;
    const bool sampler = !fused && r < nloc;                 // samples sequence i = r
    {
        const int tid = threadIdx.x;
        if (tid < nloc) {
            const int i = tid, b = g + i * nsg, ny0 = a.ny[b];
            sh.ny0[i] = ny0;
            sh.kv0[i] = a.kvlen[b];
            sh.st0[i] = a.steps[b];
            sh.tok[i] = (int)a.y[(long)b * a.ldy + ny0 - 1];
            sh.act[i] = a.done[b] ? 0 : 1;
            sh.nexe[i] = 0;
            sh.lstop[i] = 0;
            sh.lfin[i] = a.done[b] ? 1 : 0;
        }
        for (int e = tid; e < nloc * 33; e += PT) sh.seenq[e / 33][e % 33] = a.seen[(long)(g + (e / 33) * nsg) * 33 + e % 33];
        if (tid == 0) {
            sh.fail = 0;
            sh.stopreq = 0;
        }
    }
    __syncthreads();
    unsigned live = 0;
    for (int i = 0; i < nloc; ++i) live |= sh.act[i] ? 1u << i : 0u;
    // the two K stage buffers (sh.at.k, sh.at.v) and the (step, layer, sequence) each holds / receives
    int skey0 = -1, skey1 = -1, cur = 0;
    auto kbuf = [&](int bsel) { return bsel ? sh.at.v : sh.at.k; };
    int n_exec = 0;
    for (int s = 0; s < a.smax && live && sh.fail == 0; ++s) {
        const unsigned tag = base.tag(s);
        PMSTAMP(true, 12);
        if (s > 0) {   // ---- the tokens of step s - 1
            if (fused) {
                bool ok = true;
                if (w < MG && ((live >> w) & 1u)) resolve_w(a, base.seq(g + w * nsg), s, w, g + w * nsg, publisher, sh, ok);
                if (!ok_all(ok, sh)) return;
            } else {
                bool ok = true;
                const int tid = threadIdx.x;
                if (tid < MG && ((live >> tid) & 1u)) {
                    const WsSeq ws = base.seq(g + tid * nsg);
                    const float v = wait_gran(ws.TK(s), ws.tag(s), a.err, ok, a.spin_ticks);
                    if (ok) {
                        const unsigned u = __float_as_uint(v);
                        sh.tok[tid] = (int)(u & 0xffff);
                        sh.act[tid] = ((u >> 16) & 1) ? 0 : 1;
                    }
                }
                if (!ok_all(ok, sh)) return;
            }
            unsigned nl = 0;
            for (int i = 0; i < nloc; ++i) nl |= ((live >> i) & 1u) && sh.act[i] ? 1u << i : 0u;
            live = nl;
            bar_nf();
            if (!live) break;
        }
        PMSTAMP(true, 13);
        // this step's attention: every live sequence at once when all of them are on the
        // single kernel's LDS path (T <= 512 keys, kv < KVL1), else one after another
        // (knob2 = 1 forces the serial loop: A/B)
        bool conc = a.knob[2] == 0;
        int nu_max = 1;
        for (unsigned m = live; m; m &= m - 1) {
            const int kv = sh.kv0[__builtin_ctz(m)] + s;
            conc = conc && kv + 1 <= 512 && kv < KVL1;
            nu_max = max(nu_max, (kv + 1 + 63) >> 6);
        }
        if (!conc) {
            const int i0 = __builtin_ctz(live);
            const int key = (s * 24 + 0) * MG + i0;
            if ((cur ? skey1 : skey0) != key) {   // layer 0's first K stage (the step's first layer)
                stage_k(a, kbuf(cur), 0, g + i0 * nsg, r, sh.kv0[i0] + s, w, threadIdx.x & 63);
                (cur ? skey1 : skey0) = key;
            }
        }
        for (int l = 0; l < 24; ++l) {
            const PLayer& P = a.L[l];
            const int tid = opaque_tid(), lane = tid & 63;
            const int n16 = lane & 15, k8 = 8 * (lane >> 4);
            const bool up = lane >= 16;   // lanes 0..15: sequences 0, 1; 16..31: 2, 3 (MFMA rows 0..3 / 4..7)
            // ================= attention role: head r =================
            PMSTAMP(l == 12, 0);
            uint4 wq[16], wo[4];
            float qfB = 0.f, qfC = 0.f;
            float xw = 0.f, xb = 0.f;   // LN2_{l-1} scale / shift of column 32 r + lane (x_l block r)
            if (l > 0 && w == 0 && lane < 32) {
                xw = ldg(a.L[l - 1].n2w, 32 * r + lane);
                xb = ldg(a.L[l - 1].n2b, 32 * r + lane);
            }
            auto load_wq = [&]() {
                if (w < 6) {
                    const int row = (w >> 1) * 512 + r * 32 + 16 * (w & 1) + n16;
#pragma unroll
                    for (int c = 0; c < 16; ++c) wq[c] = ldg16(P.w_in + (long)row * 512 + 32 * c + k8, 0);
                    qfB = ldg(a.fold, (long)l * FOLD_LAYER + row);
                    qfC = ldg(a.fold, (long)l * FOLD_LAYER + 1536 + row);
                }
#pragma unroll
                for (int t = 0; t < 4; ++t) wo[t] = ldg16(P.w_out + (long)(64 * w + 16 * t + n16) * 512 + r * 32 + k8, 0);
            };
            // PERSISTM_LATE_W (A/B build, tools/r06g_late_w.hip): the layer's weight loads after
            // its gathers, so no gather polls behind ~128 KB of weight loads in its own wave's queue
            constexpr bool late_w = PERSISTM_LATE_W != 0;
            if constexpr (!late_w) load_wq();
            if (l == 0) {   // x_0 = E_audio[tok] + alpha pe[n]
                bool ok = true;
                const int nl = __builtin_popcount(live);
                for (int it = tid; it < nl * 512; it += PT) {
                    const int i = nth_bit(live, it >> 9), c = it & 511;
                    const float u = ldg_h(a.emb, (long)sh.tok[i] * 512 + c) +
                                    ldg(a.alpha, 0) * ldg(a.pe, (long)(sh.ny0[i] + s) * 512 + c);
                    sh.at.g.lnb[i][c] = u;
                    _Float16 hi, lo;
                    if (!split_h(u, hi, lo) || !(fabsf(u) < a.f16_limit)) {
                        atomicCAS(a.err, 0, ERR_F16_RANGE);
                        ok = false;
                    }
                    sh.at.g.A[2 * i][c] = hi;
                    sh.at.g.A[2 * i + 1][c] = lo;
                }
                if (!ok_all(ok, sh)) return;
            } else {
                const PLayer& Q = a.L[l - 1];
                if (!gather_m(a, base, sh, live, tag, [&](int i) { return base.seq(g + i * nsg).PFH(s, l - 1, 0); },
                              Q.b2, Q.n2w))
                    return;
            }
            if constexpr (late_w) load_wq();
            PMSTAMP(l == 12, 1);
            {
                float mean[MG], rden[MG];
                stats_m(sh, live, mean, rden);
                if (w == 0 && lane < 32) {   // block r of x_l (form_x's arithmetic) for the FFN's PA row 16
                    const int c = 32 * r + lane;
#pragma unroll
                    for (int i = 0; i < MG; ++i)
                        if ((live >> i) & 1u)
                            sh.h1s[i][lane] = l > 0 ? ln_apply(sh.at.g.lnb[i][c], mean[i], rden[i], xw, xb)
                                                    : sh.at.g.lnb[i][c];
                }
                if (w < 6) {
                    const _Float16* ab = abase_m(&sh.at.g.A[0][0], AST, lane);
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
                    if (lane < 32) {
#pragma unroll
                        for (int k = 0; k < 2; ++k) {
                            const int i = (up ? 2 : 0) + k;
                            if ((live >> i) & 1u) {
                                const float mn = l > 0 ? (up ? mean[2 + k] : mean[k]) : 0.f;
                                const float rd = l > 0 ? (up ? rden[2 + k] : rden[k]) : 1.f;
                                sh.qkvs[i][16 * w + n16] =
                                    rd * (((c0[2 * k] + c1[2 * k]) + (c0[2 * k + 1] + c1[2 * k + 1])) - mn * qfB) + qfC;
                            }
                        }
                    }
                }
            }
            bar_nf();   // q/k/v of every sequence; the A tile / lnb are free (the general path's scores)
            PMSTAMP(l == 12, 2);
            if (conc) {
                if (nu_max <= 2) attn_conc_m<2>(a, sh, live, g, nsg, r, l, s, w, lane);
                else if (nu_max <= 4) attn_conc_m<4>(a, sh, live, g, nsg, r, l, s, w, lane);
                else if (nu_max <= 6) attn_conc_m<6>(a, sh, live, g, nsg, r, l, s, w, lane);
                else attn_conc_m<7>(a, sh, live, g, nsg, r, l, s, w, lane);   // (kv < KVL1 = 448: T <= 448)
                bar_nf();   // every wave's partials of every sequence in LDS
                if (w < __builtin_popcount(live)) merge_m(sh, nth_bit(live, w), lane);
                if (w == 7) {   // the new K/V rows (read by this workgroup only, next step)
                    for (unsigned m = live; m; m &= m - 1) {
                        const int i = __builtin_ctz(m), kv = sh.kv0[i] + s;
                        const long kvoff = (long)(g + i * nsg) * a.sstride + (long)r * a.tmax * 32;
                        float* dst = (lane < 32 ? a.kc[l] + kvoff : a.vc[l] + kvoff - 32) + (long)kv * 32 + lane;
                        *dst = sh.qkvs[i][32 + lane];
                    }
                }
            } else {
            // V rows of the next sequence in registers, loaded while this one's attention runs
            float4 vpre[8];
            auto v_of = [&](int ii) {   // (after the q/k/v barrier: qkvs holds every sequence's new row)
                const int c8 = lane & 7, gk = (w << 3) | (lane >> 3);
                const float* Vw = a.vc[l] + (long)(g + ii * nsg) * a.sstride + (long)r * a.tmax * 32;
                load_v8(vpre, Vw, *reinterpret_cast<const float4*>(&sh.qkvs[ii][64 + 4 * c8]), sh.kv0[ii] + s, c8, gk);
            };
            v_of(__builtin_ctz(live));
            for (unsigned m = live; m; m &= m - 1) {
                const int i = __builtin_ctz(m), b = g + i * nsg;
                const int kv = sh.kv0[i] + s, T = kv + 1;
                const int key = (s * 24 + l) * MG + i;
                if ((cur ? skey1 : skey0) != key) {
                    stage_k(a, kbuf(cur), l, b, r, kv, w, lane);
                    (cur ? skey1 : skey0) = key;
                }
                float* Ks = kbuf(cur);
                if (!is_pub_wave(w)) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // its K LDS-DMA landed
                if (kv < KVL1 && (w == 2 || w == 3) && lane < 16) (Ks + kv * 32 + 16 * (w & 1))[lane] = sh.qkvs[i][16 * w + lane];
                if (tid < 96) sh.qkv[tid] = sh.qkvs[i][tid];
                bar_nf();
                PMSTAMP(l == 12 && a.knob[1] == 1, 8 + i);   // (knob1 = 1: per-sequence attention stamps)
                // this sequence's V rows (loaded one iteration ago) passed through an asm barrier
                // after the wait: their uses below do not wait for the prefetch issued next
                float4 vcur[8];
                // (wave 7's one K/V row store of the previous sequence may stay in flight)
                if (w == 7) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
                else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    vcur[u] = vpre[u];
                    asm volatile("" : "+v"(vcur[u].x), "+v"(vcur[u].y), "+v"(vcur[u].z), "+v"(vcur[u].w));
                }
                {
                    const unsigned nx = m & (m - 1);
                    if (nx) {   // the next sequence's K rows land in the other buffer, its V rows in
                                // registers, during this attention
                        const int i2 = __builtin_ctz(nx);
                        stage_k(a, kbuf(cur ^ 1), l, g + i2 * nsg, r, sh.kv0[i2] + s, w, lane);
                        (cur ? skey0 : skey1) = (s * 24 + l) * MG + i2;
                        v_of(i2);
                    }
                }
                const long kvoff = (long)b * a.sstride + (long)r * a.tmax * 32;
                const float* Kw = a.kc[l] + kvoff;
                const float* Vw = a.vc[l] + kvoff;
                const float sc = a.scale;
                const int c8 = lane & 7, gk = (w << 3) | (lane >> 3);
                const float4 qc = *reinterpret_cast<const float4*>(sh.qkv + 4 * c8);
                const float q0 = qc.x * sc, q1 = qc.y * sc, q2 = qc.z * sc, q3 = qc.w * sc;
                const float4 knew = *reinterpret_cast<const float4*>(sh.qkv + 32 + 4 * c8);
                if (T <= 512 && kv < KVL1) {
                    const int nu = (T + 63) >> 6;
                    if (nu <= 2) wave_attn_m<2>(sh, Ks, vcur, q0, q1, q2, q3, sc, kv, T, c8, gk, w, lane);
                    else if (nu <= 4) wave_attn_m<4>(sh, Ks, vcur, q0, q1, q2, q3, sc, kv, T, c8, gk, w, lane);
                    else if (nu == 5) wave_attn_m<5>(sh, Ks, vcur, q0, q1, q2, q3, sc, kv, T, c8, gk, w, lane);
                    else if (nu == 6) wave_attn_m<6>(sh, Ks, vcur, q0, q1, q2, q3, sc, kv, T, c8, gk, w, lane);
                    else wave_attn_m<8>(sh, Ks, vcur, q0, q1, q2, q3, sc, kv, T, c8, gk, w, lane);
                    bar_nf();   // the stage is read; every wave's partials are in LDS
                    merge_waves1(sh, w, lane);
                } else {
                    attn_general_m(sh, Ks, Kw, Vw, kv, T, q0, q1, q2, q3, sc, knew, c8, gk, w, lane, tid);
                    bar_nf();
                }
                cur ^= 1;
                if (w == 0 && lane < 32) {
                    sh.O[2 * i][lane] = sh.osh[0][lane];
                    sh.O[2 * i + 1][lane] = sh.osl[0][lane];
                }
#ifdef PERSIST_DBG   // tools/persist_dbg.py (debug build only)
                if (a.knob[3] == 7 && s == 1 && l < 8 && w == 0 && b == 0)
                    reinterpret_cast<float*>(a.trace)[(l * 16 + r) * 64 + lane] =
                        lane < 32 ? sh.qkv[lane] : (float)sh.osh[0][lane - 32] + (float)sh.osl[0][lane - 32];
#endif
                if (w == 7) {   // the new K/V row (read by this workgroup only, next step): one store
                    float* dst = (lane < 32 ? a.kc[l] + kvoff : a.vc[l] + kvoff - 32) + (long)kv * 32 + lane;
                    *dst = sh.qkvs[i][32 + lane];
                }
            }
            }
            bar_nf();   // O complete
            PMSTAMP(l == 12, 3);
            {
                const h8v af = afrag(abase_m(&sh.O[0][0], OST, lane), 0);
                f32x4 acc[4];
#pragma unroll
                for (int t = 0; t < 4; ++t) acc[t] = mfma16(af, bfrag(wo[t]), f32x4{0.f, 0.f, 0.f, 0.f});
                if (lane < 32) {
#pragma unroll
                    for (int k = 0; k < 2; ++k) {
                        const int i = (up ? 2 : 0) + k;
                        if ((live >> i) & 1u) {
#pragma unroll
                            for (int t = 0; t < 4; ++t) sh.at.pk[i][64 * w + 16 * t + n16] = acc[t][2 * k] + acc[t][2 * k + 1];
#ifdef PERSIST_DBG
                            if (a.knob[3] == 9 && s == 1 && l == 0 && g == 0 && i == 0)
                                for (int t = 0; t < 4; ++t)
                                    reinterpret_cast<float*>(a.trace)[r * 512 + 64 * w + 16 * t + n16] = acc[t][2 * k] + acc[t][2 * k + 1];
#endif
                        }
                    }
                }
            }
            bar_nf();
            for (unsigned m = live; m; m &= m - 1) {
                const int i = __builtin_ctz(m);
                const WsSeq ws = base.seq(g + i * nsg);
                pub_m(ws, sh, i, ws.PA(s, l, r), ws.PA(s, l, 16) + 16 * 11 * r, tag, w, lane);
            }
            bar_nf();   // pk consumed
            PMSTAMP(l == 12, 4);
            // ================= FFN role: slice r =================
            uint4 w1r[16], w2r[16];   // W2's columns are loaded once FFN1 has consumed W1's rows
            float ffB, ffC, n1w_t, n1b_t;
            auto load_w1 = [&]() {
                const int tid2 = opaque_tid(), lane2 = tid2 & 63, m16 = lane2 & 15, q8 = 8 * (lane2 >> 4);
#pragma unroll
                for (int c = 0; c < 16; ++c) w1r[c] = ldg16(P.w1 + (long)(r * 128 + w * 16 + m16) * 512 + 32 * c + q8, 0);
                n1w_t = ldg(P.n1w, tid2);
                n1b_t = ldg(P.n1b, tid2);
                ffB = ldg(a.fold, (long)l * FOLD_LAYER + 3072 + r * 128 + w * 16 + m16);
                ffC = ldg(a.fold, (long)l * FOLD_LAYER + 5120 + r * 128 + w * 16 + m16);
            };
            if constexpr (!late_w) load_w1();
            if (!gather_m(a, base, sh, live, tag, [&](int i) { return base.seq(g + i * nsg).PA(s, l, 0); }, P.b_out,
                          P.n1w, s == 1 && l == 0 && g == 0 && r == 0))
                return;
            if constexpr (late_w) load_w1();
            PMSTAMP(l == 12, 5);
            {
                const int tid2 = opaque_tid(), lane2 = tid2 & 63;
                float mean[MG], rden[MG];
                stats_m(sh, live, mean, rden);
#ifdef PERSIST_DBG   // knob3 = 11: FFN1's A rows as the single-sequence kernel lays them out (row 0 hi, 1..15 lo)
                const _Float16* ab = a.knob[3] == 11 ? ((lane2 & 15) == 0 ? &sh.at.g.A[0][0] : &sh.at.g.A[1][0]) + 8 * (lane2 >> 4)
                                                     : abase_m(&sh.at.g.A[0][0], AST, lane2);
#else
                const _Float16* ab = abase_m(&sh.at.g.A[0][0], AST, lane2);
#endif
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
                PMSTAMP(l == 12 && a.knob[1] == 2, 8);
                {
                    const int m16 = lane2 & 15, q8 = 8 * (lane2 >> 4);
#pragma unroll
                    for (int t = 0; t < 4; ++t)
#pragma unroll
                        for (int c = 0; c < 4; ++c)
                            w2r[4 * t + c] = ldg16(P.w2 + (long)(64 * w + 16 * t + m16) * 2048 + r * 128 + 32 * c + q8, 0);
                }
                PMSTAMP(l == 12 && a.knob[1] == 2, 9);
#ifdef PERSIST_DBG
                if (a.knob[3] == 12 && s == 1 && l == 0 && g == 0 && r == 0) {
                    float* tf = reinterpret_cast<float*>(a.trace);
                    if (w == 0 && lane2 < 16) {
                        tf[lane2 * 4 + 0] = c0[0]; tf[lane2 * 4 + 1] = c1[0]; tf[lane2 * 4 + 2] = c0[1]; tf[lane2 * 4 + 3] = c1[1];
                    }
                    tf[64 + tid2] = sh.at.g.lnb[0][tid2];
                    tf[576 + tid2] = (float)sh.at.g.A[0][tid2] + (float)sh.at.g.A[1][tid2];
                    tf[1088 + tid2] = ffB;
                    tf[1600 + tid2] = sh.at.g.lnb[0][tid2] * ldg(P.n1w, tid2);
                    tf[2112 + tid2] = (float)sh.at.g.A[0][tid2];
                }
#endif
                if ((tid2 >> 5) == r) {   // block r of h1 = LN1(v) for the next layer's PFH row 16
                    const float n1w = n1w_t, n1b = n1b_t;
#pragma unroll
                    for (int i = 0; i < MG; ++i)
                        if ((live >> i) & 1u) sh.h1s[i][tid2 & 31] = (sh.at.g.lnb[i][tid2] - mean[i]) * rden[i] * n1w + n1b;
                }
                bool ok = true;
                if (lane2 < 32) {
                    const bool up2 = lane2 >= 16;
#pragma unroll
                    for (int k = 0; k < 2; ++k) {
                        const int i = (up2 ? 2 : 0) + k;
                        if ((live >> i) & 1u) {
                            const float mn = up2 ? mean[2 + k] : mean[k], rd = up2 ? rden[2 + k] : rden[k];
                            const float f =
                                fmaxf(rd * (((c0[2 * k] + c1[2 * k]) + (c0[2 * k + 1] + c1[2 * k + 1])) - mn * ffB) + ffC, 0.f);
                            split_h(f, sh.F[2 * i][w * 16 + (lane2 & 15)], sh.F[2 * i + 1][w * 16 + (lane2 & 15)]);
#ifdef PERSIST_DBG
                            if ((a.knob[3] == 10 || a.knob[3] == 11) && s == 1 && l == 0 && g == 0 && i == 0) {
                                float* tf = reinterpret_cast<float*>(a.trace);
                                tf[r * 128 + w * 16 + (lane2 & 15)] = f;
                                if (w == 0 && lane2 == 0) { tf[2048 + 2 * r] = mn; tf[2049 + 2 * r] = rd; }
                            }
#endif
                            if (!(fabsf(f) < a.f16_limit)) {
                                atomicCAS(a.err, 0, ERR_F16_RANGE);
                                ok = false;
                            }
                        }
                    }
                }
                PMSTAMP(l == 12 && a.knob[1] == 2, 10);
                if (!ok_all(ok, sh)) return;   // F complete; lnb / A free
            }
            PMSTAMP(l == 12, 6);
            {
                const int tid2 = opaque_tid(), lane2 = tid2 & 63;
                const _Float16* ab = abase_m(&sh.F[0][0], FST, lane2);
                h8v af[4];
#pragma unroll
                for (int c = 0; c < 4; ++c) af[c] = afrag(ab, 32 * c);
                f32x4 acc[4];
#pragma unroll
                for (int t = 0; t < 4; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int c = 0; c < 4; ++c)
#pragma unroll
                    for (int t = 0; t < 4; ++t) acc[t] = mfma16(af[c], bfrag(w2r[4 * t + c]), acc[t]);
                if (lane2 < 32) {
                    const bool up2 = lane2 >= 16;
#pragma unroll
                    for (int k = 0; k < 2; ++k) {
                        const int i = (up2 ? 2 : 0) + k;
                        if ((live >> i) & 1u) {
#pragma unroll
                            for (int t = 0; t < 4; ++t)
                                sh.at.pk[i][64 * w + 16 * t + (lane2 & 15)] = acc[t][2 * k] + acc[t][2 * k + 1];
#ifdef PERSIST_DBG
                            if (a.knob[3] == 8 && s == 1 && l == 0 && g == 0 && i == 0)
                                for (int t = 0; t < 4; ++t)
                                    reinterpret_cast<float*>(a.trace)[r * 512 + 64 * w + 16 * t + (lane2 & 15)] = acc[t][2 * k] + acc[t][2 * k + 1];
#endif
                        }
                    }
                }
            }
            bar_nf();
            {
                const int lane2 = opaque_tid() & 63;
                for (unsigned m = live; m; m &= m - 1) {
                    const int i = __builtin_ctz(m);
                    const WsSeq ws = base.seq(g + i * nsg);
                    pub_m(ws, sh, i, ws.PFH(s, l, r), ws.PFH(s, l, 16) + 16 * 11 * r, tag, w, lane2);
                }
                if (l < 23 && !conc) {   // the next layer's first K stage lands during the hop
                    const int i0 = __builtin_ctz(live);
                    stage_k(a, kbuf(cur), l + 1, g + i0 * nsg, r, sh.kv0[i0] + s, w, lane2);
                    (cur ? skey1 : skey0) = (s * 24 + l + 1) * MG + i0;
                }
            }
            bar_nf();   // pk consumed
            PMSTAMP(l == 12, 7);
            PMSTAMP(l == 23, 14);
        }
        // ================= logits of step s: rows 64 r .. 64 r + 63 (+ EOS on r = 15) =================
        {
            // the stop word (host memory: a PCIe read that took ~30 us under this kernel's load,
            // profiles/r05r_stop_read.txt) every 4th step, for the next resolve: a stop takes
            // effect within 5 steps
            if ((s & 3) == 0 && threadIdx.x == 64) sh.stopreq = ld_stop(a.stop_req);
            const int tid0 = opaque_tid(), lane0 = tid0 & 63;
            const int row = w < 4 ? 64 * r + 16 * w + (lane0 & 15) : 1024;
            const bool lrow = w < 4 || (w == 4 && r == NF - 1);
            // this slice's w_pred rows -> the (free) K stage by LDS-DMA during the gather, rows
            // padded by 16 B (conflict-free B-fragment reads); (64 r + rr, or the EOS row 1024)
            float* wpl = sh.at.k;
            for (int rr = w; rr < (r == NF - 1 ? LROWS + 1 : LROWS); rr += PWV) {
                const int grow = rr < LROWS ? LROWS * r + rr : 1024;
                __builtin_amdgcn_global_load_lds(reinterpret_cast<const float*>(a.w_pred) + (long)grow * 256 + lane0 * 4,
                                                 wpl + rr * 260, 16, 0, 0);
            }
            float lfB = 0.f, lfC = 0.f;
            if (lrow) {
                lfB = ldg(a.fold, LOGIT_FOLD + row);
                lfC = ldg(a.fold, LOGIT_FOLD + 1025 + row);
            }
            if (!gather_m(a, base, sh, live, tag, [&](int i) { return base.seq(g + i * nsg).PFH(s, 23, 0); },
                          a.L[23].b2, a.L[23].n2w))
                return;
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's w_pred rows landed
            bar_nf();
            PMSTAMP(a.knob[1] == 0, 8);
            const int tid = opaque_tid(), lane = tid & 63, n16 = lane & 15, k8 = 8 * (lane >> 4);
            const bool up = lane >= 16;
            float mean[MG], rden[MG];
            stats_m(sh, live, mean, rden);
            if (lrow) {
                const _Float16* ab = abase_m(&sh.at.g.A[0][0], AST, lane);
                const _Float16* wb = reinterpret_cast<const _Float16*>(wpl + (w < 4 ? 16 * w + n16 : LROWS) * 260) + k8;
                f32x4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int cb = 0; cb < 16; cb += 2) {
                    c0 = mfma16(afrag(ab, 32 * cb), bfrag(*reinterpret_cast<const uint4*>(wb + 32 * cb)), c0);
                    c1 = mfma16(afrag(ab, 32 * (cb + 1)), bfrag(*reinterpret_cast<const uint4*>(wb + 32 * (cb + 1))), c1);
                }
                const bool lv = w < 4 || n16 == 0;
#pragma unroll
                for (int k = 0; k < 2; ++k) {
                    const int i = (up ? 2 : 0) + k;
                    const float mn = up ? mean[2 + k] : mean[k], rd = up ? rden[2 + k] : rden[k];
                    const float v = rd * (((c0[2 * k] + c1[2 * k]) + (c0[2 * k + 1] + c1[2 * k + 1])) - mn * lfB) + lfC;
                    const bool mine = lane < 32 && ((live >> i) & 1u);
                    if (!fused) {
                        if (mine && lv) {
                            const WsSeq ws = base.seq(g + i * nsg);
                            st_gran(ws.LG(s) + row, tag, v);
                        }
                    } else {
                        // (rows 2, 3 of lanes 32..63 reduce garbage and are never read)
                        const uint32_t* seen = sh.seenq[i & (MG - 1)];
                        float pv = ((seen[row >> 5] >> (row & 31)) & 1u) ? (v < 0.f ? v * a.rep_penalty : v / a.rep_penalty)
                                                                         : v;
                        pv = pv / a.temperature;
                        float gv = lv ? pv : -INFINITY, rv = lv ? v : -INFINITY;
                        gv = fmaxf(gv, dpp_f<0xB1, 0xF>(gv)); rv = fmaxf(rv, dpp_f<0xB1, 0xF>(rv));
                        gv = fmaxf(gv, dpp_f<0x4E, 0xF>(gv)); rv = fmaxf(rv, dpp_f<0x4E, 0xF>(rv));
                        gv = fmaxf(gv, dpp_f<0x141, 0xF>(gv)); rv = fmaxf(rv, dpp_f<0x141, 0xF>(rv));
                        gv = fmaxf(gv, dpp_f<0x140, 0xF>(gv)); rv = fmaxf(rv, dpp_f<0x140, 0xF>(rv));
                        int gmi = (lv && pv == gv) ? row : 0x7fffffff, rmi = (lv && v == rv) ? row : 0x7fffffff;
                        gmi = min(gmi, dpp_i<0xB1, 0xF>(gmi)); rmi = min(rmi, dpp_i<0xB1, 0xF>(rmi));
                        gmi = min(gmi, dpp_i<0x4E, 0xF>(gmi)); rmi = min(rmi, dpp_i<0x4E, 0xF>(rmi));
                        gmi = min(gmi, dpp_i<0x141, 0xF>(gmi)); rmi = min(rmi, dpp_i<0x141, 0xF>(rmi));
                        gmi = min(gmi, dpp_i<0x140, 0xF>(gmi)); rmi = min(rmi, dpp_i<0x140, 0xF>(rmi));
                        if (mine && n16 < 4)
                            sh.cand[i][w][n16] = n16 == 0 ? gv : n16 == 1 ? __int_as_float(gmi) : n16 == 2 ? rv
                                                                                                    : __int_as_float(rmi);
                    }
                }
            }
            bar_nf();
            PMSTAMP(a.knob[1] == 0, 9);
            if (fused && w == 7) {   // this slice's candidates: 16 granules per sequence (+ 4 EOS on r = 15)
                const bool eos = r == NF - 1;
                for (unsigned m = live; m; m &= m - 1) {
                    const int i = __builtin_ctz(m);
                    const WsSeq ws = base.seq(g + i * nsg);
                    if (lane < 16 || (lane < 20 && eos)) {
                        const int ww = lane >> 2, k = lane & 3;
                        st_gran(ws.LG(s) + 4 * (ww < 4 ? 4 * r + ww : 64) + k, tag, sh.cand[i][ww][k]);
                    }
                }
            }
            bar_nf();   // A / lnb consumed
            PMSTAMP(a.knob[1] == 0, 10);
            skey0 = skey1 = -1;   // (the w_pred rows overwrote both K buffers)
        }
        // ---- sampler (sampled decoding): sequence i = r of the group
        if (sampler && ((live >> r) & 1u)) {
            const int tid = threadIdx.x, i = r, b = g + i * nsg;
            const WsSeq ws = base.seq(b);
            bool ok = true;
            const u64* lgg = ws.LG(s);
            for (int k = tid; k < 1025; k += PT) sh.at.lg[k] = wait_gran(lgg + k, tag, a.err, ok, a.spin_ticks);
            if (!ok) sh.fail = 1;
            __syncthreads();
            if (sh.fail) return;
            const int st = sh.st0[i] + s;
            uint32_t* seen = sh.seenq[i];
            int raw = 0;
            const int tok = sample_block<PT>([&](int k) { return sh.at.lg[k]; }, seen, b, st + 1, a.top_k,
                                             a.temperature, a.rep_penalty, a.greedy, a.seed, 0, nullptr, &raw, sh.samp);
            if (tid == 0) {
                const int stop = (raw == 1024 || tok == 1024) ? 1 : 0;
                const int fin = seq_finished(a.force_b, b, a.force_steps, a.max_steps, st + 1, stop) ? 1 : 0;
                a.y[(long)b * a.ldy + sh.ny0[i] + s] = tok;
                seen[tok >> 5] |= 1u << (tok & 31);
                sh.lstop[i] = stop;
                sh.lfin[i] = fin;
                sh.nexe[i] = s + 1;
                bool go = true;
                if ((s & 3) == 0 && ld_stop(a.stop_req)) stop_launch(a, go);
                else st_gran(ws.TK(s + 1), ws.tag(s + 1), __uint_as_float((unsigned)tok | (fin ? 1u << 16 : 0u)));
            }
            __syncthreads();   // sh.at.lg / sh.samp consumed
        }
        PMSTAMP(true, 15);
        ++n_exec;
    }
    // fused greedy at the launch's step cap: the live sequences' last tokens are unresolved
    if (fused && n_exec == a.smax && n_exec > 0 && sh.fail == 0) {
        bool ok = true;
        if (w < MG && ((live >> w) & 1u)) resolve_w(a, base.seq(g + w * nsg), n_exec, w, g + w * nsg, publisher, sh, ok);
        if (!ok_all(ok, sh)) return;
    }
    // ---- sequence state write-back (the publisher: every sequence of the group; a sampler:
    // its sequence), only when no workgroup failed
    __syncthreads();
    if ((publisher || sampler) && sh.fail == 0) {
        if (threadIdx.x == 0) __threadfence();   // thread 0's y stores have reached L2
        __syncthreads();
        if (ld_rlx(a.err) != 0) return;
        const int tid = threadIdx.x;
        for (int i = 0; i < nloc; ++i) {
            if (sampler && i != r) continue;
            const int ne = sh.nexe[i], b = g + i * nsg;
            if (ne <= 0) continue;
            if (tid < 33) a.seen[(long)b * 33 + tid] = sh.seenq[i][tid];
            if (tid == 0) {
                a.ny[b] = sh.ny0[i] + ne;
                a.steps[b] = sh.st0[i] + ne;
                a.kvlen[b] = sh.kv0[i] + ne;
                a.done[b] = (uint8_t)sh.lfin[i];
                if (a.stop_out) a.stop_out[b] = (uint8_t)sh.lstop[i];
            }
        }
    }
}

__global__ __launch_bounds__(PT) void k_decode_persistm(PersistArgs a) {
    __shared__ SharedM sh;
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
    // block = 16 g + r: block b runs on XCD b % 8, so head / slice r of every group shares XCD r % 8
    run_group(a, ws, sh, blockIdx.x / GWM, blockIdx.x % GWM);
}

}  // namespace

int persistm_groups(int B) { return (B + MG - 1) / MG; }
int persistm_max_groups() { return NSG_MAX; }
int persistm_grid(int groups) { return groups * GWM; }

hipError_t decode_persistm(const PersistArgs& a, hipStream_t s, hipEvent_t start, hipEvent_t stop) {
    if (a.groups < 1 || a.groups > NSG_MAX || a.B < 1 || a.B > MB || a.B > MG * a.groups) return hipErrorInvalidValue;
    hipExtLaunchKernelGGL(k_decode_persistm, dim3(a.groups * GWM), dim3(PT), 0, s, start, stop, 0, a);
    return hipGetLastError();
}

}  // namespace gsv
