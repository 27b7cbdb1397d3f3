// VITS kernels for gfx950 (SoVITS TextEncoder/MRTE/flow + HiFi-GAN generator +
// MelStyleEncoder).  Reference graph: src/genie_tts/Data/{v2,v2ProPlus}/Models/vits_fp32.onnx.
//
// The generator's dilated residual convs are >95 % of the FLOPs (SURVEY §8a:
// 130 GFLOP per 3.2 s utterance).  They run as an implicit GEMM on
// v_mfma_f32_32x32x2_f32 (exact fp32 FMA chain: the reference is fp32 and the
// parity bar is waveform RMS <= 1e-4): M = Cout, N = time, K = Cin x taps, with
// the LeakyReLU pre-activation fused into the LDS staging of the input and the
// residual / MRF-mean / tanh fused into the epilogue.  ConvTranspose1d runs as
// `stride` polyphase convs of the same kernel (blockIdx.z = phase).
#include "common.h"
#include "vits.h"
#include "vits_epi.h"
#include <algorithm>
#include <cstdlib>

namespace gsv {

template <int KT> struct ConvCfg {
    static constexpr int CI = KT == 1 ? 32 : KT == 2 ? 32 : KT <= 4 ? 16 : KT <= 7 ? 8 : 4;
    static constexpr int KC = CI * KT;            // K-chunk per pipeline stage (multiple of 4)
};

#define CONV_BN 64
#define CONV_BM 64
#define CONV_XW_MAX 128

// Software pipeline: the next K-chunk (input halo tile + weight tile) is loaded
// into registers while the MFMAs consume the current chunk from LDS; LDS is
// double-buffered so each chunk costs one barrier.
template <int KT, bool V4>
__global__ __launch_bounds__(256) void k_conv1d(ConvArgs a) {
    constexpr int CI = ConvCfg<KT>::CI, KC = ConvCfg<KT>::KC;
    constexpr int NX = (CI * CONV_XW_MAX + 255) / 256;     // input elements per thread (max)
    constexpr int NW = (CONV_BM * KC / 4 + 255) / 256;     // weight float4 per thread
    __shared__ float Xs[2][CI * CONV_XW_MAX];
    __shared__ float Ws[2][CONV_BM][KC + 1];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int wm = w >> 1, wn = w & 1;
    const int t0 = blockIdx.x * CONV_BN, co0 = blockIdx.y * CONV_BM;
    const bool split = a.phases <= 1 && gridDim.z > 1;
    const int ph = split ? 0 : blockIdx.z;
    const float* W = a.w + (long)ph * a.w_phase_stride;
    const int dil = a.dil;
    const int XW = CONV_BN + (KT - 1) * dil;
    const long wrow = (long)a.Cin * KT;
    const int nch_all = (a.Cin + CI - 1) / CI;
    // split-K: this block reduces Cin chunks [c_lo, c_hi)
    const int c_lo = split ? (int)((long)blockIdx.z * nch_all / gridDim.z) : 0;
    const int c_hi = split ? (int)((long)(blockIdx.z + 1) * nch_all / gridDim.z) : nch_all;
    const int nch = c_hi - c_lo;
    float xr[NX];
    float4 wr[NW];

    auto load = [&](int ci0) {
#pragma unroll
        for (int i = 0; i < NX; ++i) {
            const int e = tid + i * 256;
            float v = 0.f;
            if (e < CI * XW) {
                const int ci = e / XW, u = e - ci * XW;
                const int tin = t0 - a.pad + u;
                if (ci0 + ci < a.Cin && tin >= 0 && tin < a.Tin)
                    v = a.x[(long)(ci0 + ci) * a.x_cs + (long)tin * a.x_ts];   // pre-activation in store()
            }
            xr[i] = v;
        }
#pragma unroll
        for (int i = 0; i < NW; ++i) {
            const int e = tid + i * 256;          // float4 index in the 64 x KC tile
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if (e < CONV_BM * KC / 4) {
                const int r = e / (KC / 4), kc = (e - r * (KC / 4)) * 4;
                const int co = co0 + r;
                const long kabs = (long)ci0 * KT + kc;
                if (co < a.Cout) {
                    if (V4) {
                        if (kabs < wrow) v = *reinterpret_cast<const float4*>(W + co * wrow + kabs);
                    } else {
                        const float* src = W + co * wrow + kabs;
                        if (kabs < wrow) v.x = src[0];
                        if (kabs + 1 < wrow) v.y = src[1];
                        if (kabs + 2 < wrow) v.z = src[2];
                        if (kabs + 3 < wrow) v.w = src[3];
                    }
                }
            }
            wr[i] = v;
        }
    };
    auto store = [&](int buf) {
#pragma unroll
        for (int i = 0; i < NX; ++i) {
            const int e = tid + i * 256;
            const float v = a.in_act && xr[i] < 0.f ? xr[i] * a.in_slope : xr[i];
            if (e < CI * XW) Xs[buf][e] = v;
        }
#pragma unroll
        for (int i = 0; i < NW; ++i) {
            const int e = tid + i * 256;
            if (e < CONV_BM * KC / 4) {
                const int r = e / (KC / 4), kc = (e - r * (KC / 4)) * 4;
                Ws[buf][r][kc] = wr[i].x;
                Ws[buf][r][kc + 1] = wr[i].y;
                Ws[buf][r][kc + 2] = wr[i].z;
                Ws[buf][r][kc + 3] = wr[i].w;
            }
        }
    };

    f32x16 acc;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = 0.f;
    const int ncol = wn * 32 + (lane & 31);
    const int h = lane >> 5;
    const int arow = wm * 32 + (lane & 31);
    load(c_lo * CI);
    store(0);
    __syncthreads();
    for (int c = 0; c < nch; ++c) {
        const int buf = c & 1;
        if (c + 1 < nch) load((c_lo + c + 1) * CI);
        const float* xs = Xs[buf];
#pragma unroll
        for (int kp = 0; kp < KC / 2; ++kp) {
            const int k0 = 2 * kp, k1 = 2 * kp + 1;
            const int off0 = (k0 / KT) * XW + (k0 % KT) * dil;
            const int off1 = (k1 / KT) * XW + (k1 % KT) * dil;
            const float av = Ws[buf][arow][h ? k1 : k0];
            const float bv = xs[(h ? off1 : off0) + ncol];
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc, 0, 0, 0);
        }
        if (c + 1 < nch) store(buf ^ 1);
        __syncthreads();
    }
    const int t = t0 + ncol;
    if (t >= a.n_t) return;
    if (split) {
        float* P = a.part + (long)blockIdx.z * a.Cout * a.n_t;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int co = co0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
            if (co < a.Cout) P[(long)co * a.n_t + t] = acc[r];
        }
        return;
    }
    float v[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] = acc[r];
    conv_epilogue16(a, co0 + wm * 32 + 4 * h, t, ph, v);
}

// Fixed-order sum of the split-K slabs + the conv epilogue (one thread per output).
__global__ __launch_bounds__(256) void k_conv_reduce(ConvArgs a, int nsplit) {
    const long i = (long)blockIdx.x * 256 + threadIdx.x;
    const long n = (long)a.Cout * a.n_t;
    if (i >= n) return;
    const int co = (int)(i / a.n_t), t = (int)(i - (long)co * a.n_t);
    // slabs loaded 8 at a time (independent loads in flight), summed in slab order
    float v = 0.f;
    for (int s0 = 0; s0 < nsplit; s0 += 8) {
        float p[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) p[j] = s0 + j < nsplit ? a.part[(long)(s0 + j) * n + i] : 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j)
            if (s0 + j < nsplit) v = (s0 + j == 0) ? p[j] : v + p[j];
    }
    conv_epilogue(a, co, t, 0, v);
}

template <int KT>
static void launch_conv(const ConvArgs& a, dim3 grid, hipStream_t s) {
    const bool v4 = ((a.Cin * KT) % 4 == 0) && ((reinterpret_cast<uintptr_t>(a.w) & 15) == 0) &&
                    ((a.w_phase_stride % 4) == 0);
    if (v4) hipLaunchKernelGGL((k_conv1d<KT, true>), grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((k_conv1d<KT, false>), grid, dim3(256), 0, s, a);
}

static int conv_ci(int K) {
    switch (K) {
        case 1: return ConvCfg<1>::CI;
        case 2: return ConvCfg<2>::CI;
        case 3: return ConvCfg<3>::CI;
        case 4: return ConvCfg<4>::CI;
        case 5: return ConvCfg<5>::CI;
        case 7: return ConvCfg<7>::CI;
        default: return ConvCfg<11>::CI;
    }
}

void conv1d(const ConvArgs& a, hipStream_t s) {
    if (a.wh && conv1d_h(a, s)) return;
    dim3 grid((a.n_t + CONV_BN - 1) / CONV_BN, (a.Cout + CONV_BM - 1) / CONV_BM,
              a.phases > 0 ? a.phases : 1);
    // Under-filled grids (the T=2G / S-frame encoder, MRTE and flow convs) split
    // the Cin reduction so the launch covers the chip.
    int nsplit = 1;
    const int blocks = (int)(grid.x * grid.y);
    if (a.part && a.phases <= 1 && blocks < 128) {
        const int nch = (a.Cin + conv_ci(a.K) - 1) / conv_ci(a.K);
        nsplit = std::min(nch, (256 + blocks - 1) / blocks);
        while (nsplit > 1 && (long)nsplit * a.Cout * a.n_t > a.part_cap) --nsplit;
    }
    if (nsplit > 1) grid.z = nsplit;
    switch (a.K) {
        case 1: launch_conv<1>(a, grid, s); break;
        case 2: launch_conv<2>(a, grid, s); break;
        case 3: launch_conv<3>(a, grid, s); break;
        case 4: launch_conv<4>(a, grid, s); break;
        case 5: launch_conv<5>(a, grid, s); break;
        case 7: launch_conv<7>(a, grid, s); break;
        case 11: launch_conv<11>(a, grid, s); break;
        default: return;   // host validates K
    }
    if (nsplit > 1) {
        const long n = (long)a.Cout * a.n_t;
        hipLaunchKernelGGL(k_conv_reduce, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, a, nsplit);
    }
}

__global__ __launch_bounds__(256) void k_mean3(const float4* __restrict__ a, const float4* __restrict__ b,
                                                const float4* __restrict__ c, float4* __restrict__ o, long n4,
                                                float div) {
    const long i = (long)blockIdx.x * 256 + threadIdx.x;
    if (i >= n4) return;
    const float4 x = a[i], y = b[i], z = c[i];
    o[i] = make_float4(((x.x + y.x) + z.x) / div, ((x.y + y.y) + z.y) / div, ((x.z + y.z) + z.z) / div,
                       ((x.w + y.w) + z.w) / div);
}
__global__ __launch_bounds__(256) void k_mean3_tail(const float* a, const float* b, const float* c, float* o, long lo,
                                                     long n, float div) {
    const long i = lo + (long)blockIdx.x * 256 + threadIdx.x;
    if (i < n) o[i] = ((a[i] + b[i]) + c[i]) / div;
}

void mean3(const float* a, const float* b, const float* c, float* out, long n, float div, hipStream_t s) {
    const bool v4 = ((reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(b) |
                      reinterpret_cast<uintptr_t>(c) | reinterpret_cast<uintptr_t>(out)) & 15) == 0;
    const long n4 = v4 ? n / 4 : 0;
    if (n4 > 0)
        hipLaunchKernelGGL(k_mean3, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, s,
                           (const float4*)a, (const float4*)b, (const float4*)c, (float4*)out, n4, div);
    if (4 * n4 < n)
        hipLaunchKernelGGL(k_mean3_tail, dim3((unsigned)((n - 4 * n4 + 255) / 256)), dim3(256), 0, s, a, b, c, out,
                           4 * n4, n, div);
}

// ------------------------------------------------------------ segment table
__global__ __launch_bounds__(256) void k_seg_fill(int* seg, long n, const int* off, const int* len, int nseg,
                                                   int f) {
    const long t = (long)blockIdx.x * 256 + threadIdx.x;
    if (t >= n) return;
    int lo = 0, hi = nseg - 1;   // last segment with off * f <= t
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if ((long)off[mid] * f <= t) lo = mid;
        else hi = mid - 1;
    }
    const long a = (long)off[lo] * f;
    seg[t] = (t >= a && t < a + (long)len[lo] * f) ? lo : -1;
}

void seg_fill(int* seg, long n, const int* off, const int* len, int nseg, int f, hipStream_t s) {
    hipLaunchKernelGGL(k_seg_fill, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, seg, n, off, len, nseg, f);
}

// ----------------------------------------------------------------- LN over C
// modules.LayerNorm: transpose -> layer_norm(channels, eps 1e-5) -> transpose.
// Block = 64 time columns x 4 channel groups; each thread keeps its channel
// slice in registers (C <= 4*LNC_MAX), coalesced along t.
#define LNC_MAX 64
__global__ __launch_bounds__(256) void k_ln_channels(const float* x, const float* y, float* out,
                                                     int C, int T, const float* g, const float* b) {
    __shared__ float red[4][64];
    const int tl = threadIdx.x & 63, cg = threadIdx.x >> 6;
    const int t = blockIdx.x * 64 + tl;
    const bool ok = t < T;
    float v[LNC_MAX];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < LNC_MAX; ++i) {
        const int c = cg + 4 * i;
        float xv = 0.f;
        if (c < C && ok) {
            xv = x[(long)c * T + t];
            if (y) xv = xv + y[(long)c * T + t];
        }
        v[i] = xv;
        s += xv;
    }
    red[cg][tl] = s;
    __syncthreads();
    const float mean = (red[0][tl] + red[1][tl] + red[2][tl] + red[3][tl]) / (float)C;
    __syncthreads();
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < LNC_MAX; ++i) {
        const int c = cg + 4 * i;
        if (c < C) {
            const float d = v[i] - mean;
            q += d * d;
        }
    }
    red[cg][tl] = q;
    __syncthreads();
    const float den = sqrtf((red[0][tl] + red[1][tl] + red[2][tl] + red[3][tl]) / (float)C + 1e-5f);
    if (!ok) return;
#pragma unroll
    for (int i = 0; i < LNC_MAX; ++i) {
        const int c = cg + 4 * i;
        if (c < C) out[(long)c * T + t] = (v[i] - mean) / den * g[c] + b[c];
    }
}

// Narrow form for C <= 256, C % 16 == 0 (the 192-channel encoders): one wave per
// 4 time columns, lane = (t & 3) + 4 * channel group; reductions by shuffles over
// the 16 groups, so short sequences still spread over T/4 waves.
__global__ __launch_bounds__(64) void k_ln_channels_w(const float* x, const float* y, float* out,
                                                     int C, int T, const float* g, const float* b,
                                                     const int* seg) {
    const int lane = threadIdx.x, tl = lane & 3, cg = lane >> 2;
    const int t = blockIdx.x * 4 + tl;
    const bool ok = t < T;
    const bool gap = ok && seg && seg[t] < 0;
    const int nc = C >> 4;
    float v[16];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        float xv = 0.f;
        if (i < nc && ok) {
            const long o = (long)(cg + 16 * i) * T + t;
            xv = x[o];
            if (y) xv = xv + y[o];
        }
        v[i] = xv;
        s += xv;
    }
#pragma unroll
    for (int o = 4; o < 64; o <<= 1) s += __shfl_xor(s, o, 64);
    const float mean = s / (float)C;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i)
        if (i < nc) {
            const float d = v[i] - mean;
            q += d * d;
        }
#pragma unroll
    for (int o = 4; o < 64; o <<= 1) q += __shfl_xor(q, o, 64);
    const float den = sqrtf(q / (float)C + 1e-5f);
    if (!ok) return;
#pragma unroll
    for (int i = 0; i < 16; ++i)
        if (i < nc) {
            const int c = cg + 16 * i;
            out[(long)c * T + t] = gap ? 0.f : (v[i] - mean) / den * g[c] + b[c];
        }
}

void ln_channels(const float* x, const float* y, float* out, int C, int T, const float* g,
                 const float* b, hipStream_t s, const int* seg) {
    if (C % 16 == 0 && C <= 256)
        hipLaunchKernelGGL(k_ln_channels_w, dim3((T + 3) / 4), dim3(64), 0, s, x, y, out, C, T, g, b, seg);
    else if (!seg)
        hipLaunchKernelGGL(k_ln_channels, dim3((T + 63) / 64), dim3(256), 0, s, x, y, out, C, T, g, b);
    else
        std::abort();   // the segmented front's LayerNorms are all 192-channel
}

// ----------------------------------------------------------------- attention
// One block per (head, query row).  attentions.MultiHeadAttention (rel-pos,
// window 4; (v2)#308-...) and MelStyleEncoder's ScaledDotProductAttention.
#define MHA_MAXK 2048
#define MHA_MAXD 128
#define MHA_MAXW 8      // largest rel-pos window
__global__ __launch_bounds__(256) void k_mha(MhaArgs a) {
    __shared__ float qs[MHA_MAXD];
    __shared__ float p[MHA_MAXK];
    __shared__ float red[16];
    __shared__ float part[2][MHA_MAXD];
    __shared__ float qe[2 * MHA_MAXW + 1];
    const int hd = blockIdx.x, i = blockIdx.y, tid = threadIdx.x;
    const int dk = a.dk, c0 = hd * dk;
    int nk = a.nk;
    const float* kb = a.k;
    const float* vb = a.v;
    int ir = i;        // the row's index in its own sequence (rel-pos offsets)
    if (a.row_seg) {   // packed sequences: this row's keys are rows [seg0, seg0 + nk)
        const int seg0 = a.row_seg[2 * i];
        nk = a.row_seg[2 * i + 1];
        kb += (long)seg0 * a.k_ts;
        vb += (long)seg0 * a.v_ts;
        ir = i - seg0;
    }
    for (int d = tid; d < dk; d += 256) {
        const float qv = a.q[(long)i * a.q_ts + (long)(c0 + d) * a.q_cs];
        qs[d] = a.postdiv ? qv : qv / a.scale;
    }
    __syncthreads();
    if (a.ek) {   // rel-pos key terms q . ek[r] of the window, one wave per r, lanes over d
        const int lane = tid & 63, w = tid >> 6;
        for (int r = w; r <= 2 * a.window; r += 4) {
            float sl = 0.f;
            for (int d = lane; d < dk; d += 64) sl += qs[d] * a.ek[(long)r * dk + d];
            sl = wave_sum(sl);
            if (lane == 0) qe[r] = sl;
        }
        __syncthreads();
    }
    float lmax = -INFINITY;
    for (int j = tid; j < nk; j += 256) {
        // 32 key loads in flight per step (the d order of the single sum is kept)
        const float* kp = kb + (long)j * a.k_ts + (long)c0 * a.k_cs;
        float s = 0.f;
        int d = 0;
        for (; d + 32 <= dk; d += 32) {
            float kv[32];
#pragma unroll
            for (int u = 0; u < 32; ++u) kv[u] = kp[(long)(d + u) * a.k_cs];
#pragma unroll
            for (int u = 0; u < 32; ++u) s += qs[d + u] * kv[u];
        }
        for (; d < dk; ++d) s += qs[d] * kp[(long)d * a.k_cs];
        if (a.postdiv) s = s / a.scale;
        if (a.ek) {
            const int r = j - ir;
            if (r >= -a.window && r <= a.window) s = s + qe[r + a.window];
        }
        p[j] = s;
        lmax = fmaxf(lmax, s);
    }
    const float m = block_max(lmax, red);
    float lsum = 0.f;
    for (int j = tid; j < nk; j += 256) {
        const float e = expf(p[j] - m);
        p[j] = e;
        lsum += e;
    }
    const float sum = block_sum(lsum, red);
    for (int j = tid; j < nk; j += 256) p[j] = p[j] / sum;
    __syncthreads();
    // out[d] = sum_j p_j v[j][d]  (+ sum_{|j-i|<=W} p_j ev[j-i+W][d])
    const int half = tid >> 7, dd = tid & 127;
    for (int d = dd; d < dk; d += 128) {
        const float* vp = vb + (long)(c0 + d) * a.v_cs;
        float o = 0.f;
        int j = half;
        for (; j + 30 < nk; j += 32) {   // 16 value loads in flight per step, j order kept
            float vv[16];
#pragma unroll
            for (int u = 0; u < 16; ++u) vv[u] = vp[(long)(j + 2 * u) * a.v_ts];
#pragma unroll
            for (int u = 0; u < 16; ++u) o += p[j + 2 * u] * vv[u];
        }
        for (; j < nk; j += 2) o += p[j] * vp[(long)j * a.v_ts];
        part[half][d] = o;
    }
    __syncthreads();
    for (int d = tid; d < dk; d += 256) {
        float o = part[0][d] + part[1][d];
        if (a.ev) {   // every ev load of the window in flight at once, summed in r order
            float evv[2 * MHA_MAXW + 1];
#pragma unroll
            for (int r = 0; r <= 2 * MHA_MAXW; ++r) evv[r] = r <= 2 * a.window ? a.ev[(long)r * dk + d] : 0.f;
            float ol = 0.f;
#pragma unroll
            for (int r = 0; r <= 2 * MHA_MAXW; ++r) {
                const int j = ir + r - a.window;
                if (r <= 2 * a.window && j >= 0 && j < nk) ol += p[j] * evv[r];
            }
            o = o + ol;
        }
        a.out[(long)i * a.o_ts + (long)(c0 + d) * a.o_cs] = o;
    }
}

void mha(const MhaArgs& a, hipStream_t s) {
    if ((a.ek || a.ev) && a.window > MHA_MAXW) return;   // window 4, checked when the weights load
    hipLaunchKernelGGL(k_mha, dim3(a.heads, a.nq), dim3(256), 0, s, a);
}

// ----------------------------------------------------------------- elementwise
// quantizer.decode + x2 nearest (torch.cat([q, q]).permute(1,2,0).view): out[c][2t+r] = cb[sem[t]][c]
__global__ void k_cb_up2(const int64_t* sem, int G, const float* cb, float* out) {
    const int c = blockIdx.y, t2 = blockIdx.x * blockDim.x + threadIdx.x;
    if (t2 >= 2 * G) return;
    out[(long)c * 2 * G + t2] = cb[sem[t2 >> 1] * 768 + c];
}
void codebook_upsample2(const int64_t* sem, int G, const float* cb, float* out, hipStream_t s) {
    hipLaunchKernelGGL(k_cb_up2, dim3((2 * G + 127) / 128, 768), dim3(128), 0, s, sem, G, cb, out);
}

__global__ void k_embed_ch(const int64_t* ids, int n, const float* emb, int C, float* out) {
    const int c = blockIdx.y, t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    out[(long)c * n + t] = emb[ids[t] * C + c];
}
void embed_channels(const int64_t* ids, int n, const float* emb, int C, float* out, hipStream_t s) {
    hipLaunchKernelGGL(k_embed_ch, dim3((n + 127) / 128, C), dim3(128), 0, s, ids, n, emb, C, out);
}

// commons.fused_add_tanh_sigmoid_multiply (cond already added by the conv epilogue)
__global__ void k_wn_gate(const float* xin, float* acts, int H, int T) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (long)H * T) return;
    const float a = xin[i], b = xin[i + (long)H * T];
    acts[i] = tanhf(a) * (1.0f / (1.0f + expf(-b)));
}
void wn_gate(const float* xin, float* acts, int H, int T, hipStream_t s) {
    const long n = (long)H * T;
    hipLaunchKernelGGL(k_wn_gate, dim3((n + 255) / 256), dim3(256), 0, s, xin, acts, H, T);
}

// Conv1dGLU: out = x + a * sigmoid(b), h = [a; b] channel-major [2C][T]
__global__ void k_glu(const float* h, const float* x, float* out, int C, int T, long x_cs, long x_ts) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (long)C * T) return;
    const int c = (int)(i / T), t = (int)(i - (long)c * T);
    const float a = h[i], b = h[i + (long)C * T];
    const long xi = (long)c * x_cs + (long)t * x_ts;
    out[xi] = x[xi] + a * (1.0f / (1.0f + expf(-b)));
}
void glu_resid(const float* h, const float* x, float* out, int C, int T, long x_cs, long x_ts,
               hipStream_t s) {
    const long n = (long)C * T;
    hipLaunchKernelGGL(k_glu, dim3((n + 255) / 256), dim3(256), 0, s, h, x, out, C, T, x_cs, x_ts);
}

// z_p = m_p + (eps * exp(logs_p)) * noise_scale   ((v2)#6490-6495)
__global__ void k_noise(const float* m, const float* logs, const float* eps, float sc, float* z, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float e = eps ? eps[i] : 0.f;
    z[i] = m[i] + (e * expf(logs[i])) * sc;
}
void noise_zp(const float* m, const float* logs, const float* eps, float scale, float* z, int n,
              hipStream_t s) {
    hipLaunchKernelGGL(k_noise, dim3((n + 255) / 256), dim3(256), 0, s, m, logs, eps, scale, z, n);
}
// Same with eps = the engine's Philox N(0,1): element i <- Philox4x32-10(counter
// (i, 0, 0, 0x7A), key seed), Box-Muller on the first two words (tests/philox.py
// restates it), standing in for onnxruntime's RandomNormalLike draw.
__global__ void k_noise_philox(const float* m, const float* logs, uint64_t seed, float sc, float* z, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint4 r = philox4x32(make_uint4((uint32_t)i, 0u, 0u, 0x7Au), make_uint2((uint32_t)seed, (uint32_t)(seed >> 32)));
    const float e = sqrtf(-2.0f * logf(u01_open(r.x))) * cospif(2.0f * u01_open(r.y));
    z[i] = m[i] + (e * expf(logs[i])) * sc;
}
void noise_zp_philox(const float* m, const float* logs, uint64_t seed, float scale, float* z, int n, hipStream_t s) {
    hipLaunchKernelGGL(k_noise_philox, dim3((n + 255) / 256), dim3(256), 0, s, m, logs, seed, scale, z, n);
}

__global__ void k_flip(const float* in, float* out, int C, int T) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (long)C * T) return;
    const int c = (int)(i / T), t = (int)(i - (long)c * T);
    out[i] = in[(long)(C - 1 - c) * T + t];
}
void flip_channels(const float* in, float* out, int C, int T, hipStream_t s) {
    const long n = (long)C * T;
    hipLaunchKernelGGL(k_flip, dim3((n + 255) / 256), dim3(256), 0, s, in, out, C, T);
}

// ---- segmented-batch forms of the front's per-utterance kernels
__global__ void k_cb_up2_seg(const int64_t* const* sems, const int* seg, const int* off, int T, const float* cb,
                             float* out) {
    const int c = blockIdx.y, t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= T) return;
    const int sg = seg[t];
    out[(long)c * T + t] = sg < 0 ? 0.f : cb[sems[sg][(t - off[sg]) >> 1] * 768 + c];
}
void codebook_upsample2_seg(const int64_t* const* sems, const int* seg, const int* off, int T, const float* cb,
                            float* out, hipStream_t s) {
    hipLaunchKernelGGL(k_cb_up2_seg, dim3((T + 127) / 128, 768), dim3(128), 0, s, sems, seg, off, T, cb, out);
}

__global__ void k_embed_seg(const int64_t* const* ids, const int* seg, const int* off, int n, const float* emb,
                            int C, float* out) {
    const int c = blockIdx.y, t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    const int sg = seg[t];
    out[(long)c * n + t] = sg < 0 ? 0.f : emb[ids[sg][t - off[sg]] * C + c];
}
void embed_channels_seg(const int64_t* const* ids, const int* seg, const int* off, int n, const float* emb, int C,
                        float* out, hipStream_t s) {
    hipLaunchKernelGGL(k_embed_seg, dim3((n + 127) / 128, C), dim3(128), 0, s, ids, seg, off, n, emb, C, out);
}

__global__ void k_noise_philox_seg(const float* m, const float* logs, const uint64_t* seeds, const int* seg,
                                   const int* off, const int* len, float sc, float* z, int C, int T) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (long)C * T) return;
    const int c = (int)(i / T), t = (int)(i - (long)c * T);
    const int sg = seg[t];
    if (sg < 0) {
        z[i] = 0.f;
        return;
    }
    const uint64_t seed = seeds[sg];
    float e = 0.f;   // seed 0: noise_zp without eps
    if (seed != 0) {
        const uint32_t k = (uint32_t)c * (uint32_t)len[sg] + (uint32_t)(t - off[sg]);
        const uint4 r = philox4x32(make_uint4(k, 0u, 0u, 0x7Au), make_uint2((uint32_t)seed, (uint32_t)(seed >> 32)));
        e = sqrtf(-2.0f * logf(u01_open(r.x))) * cospif(2.0f * u01_open(r.y));
    }
    z[i] = m[i] + (e * expf(logs[i])) * sc;
}
void noise_zp_philox_seg(const float* m, const float* logs, const uint64_t* seeds, const int* seg, const int* off,
                         const int* len, float scale, float* z, int C, int T, hipStream_t s) {
    const long n = (long)C * T;
    hipLaunchKernelGGL(k_noise_philox_seg, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, m, logs, seeds, seg,
                       off, len, scale, z, C, T);
}

__global__ void k_gather_vecs(const float* const* ptrs, int dim, float* out) {
    const int i = blockIdx.x;
    for (int d = threadIdx.x; d < dim; d += blockDim.x) out[(long)i * dim + d] = ptrs[i][d];
}
void gather_vecs(const float* const* ptrs, int n, int dim, float* out, hipStream_t s) {
    if (n > 0) hipLaunchKernelGGL(k_gather_vecs, dim3(n), dim3(256), 0, s, ptrs, dim, out);
}

__global__ void k_reflect_pad(const float* x, int n, int pad, float* out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int m = n + 2 * pad;
    if (i >= m) return;
    int j = i - pad;
    if (j < 0) j = -j;
    if (j >= n) j = 2 * (n - 1) - j;
    out[i] = x[j];
}
void reflect_pad(const float* x, int n, int pad, float* out, hipStream_t s) {
    const int m = n + 2 * pad;
    hipLaunchKernelGGL(k_reflect_pad, dim3((m + 255) / 256), dim3(256), 0, s, x, n, pad, out);
}

// sqrt(re^2 + im^2 + 1e-6)  ((v2)#40-45), reim rows interleaved [re0, im0, re1, im1, ...]
__global__ void k_stft_mag(const float* reim, int frames, int bins, float* spec) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= frames * bins) return;
    const int f = i / bins, b = i - f * bins;
    const float re = reim[(long)f * 2 * bins + 2 * b], im = reim[(long)f * 2 * bins + 2 * b + 1];
    spec[i] = sqrtf((re * re + im * im) + 1e-6f);
}
void stft_mag(const float* reim, int frames, int bins, float* spec, hipStream_t s) {
    const int n = frames * bins;
    hipLaunchKernelGGL(k_stft_mag, dim3((n + 255) / 256), dim3(256), 0, s, reim, frames, bins, spec);
}

// temporal_avg_pool: sum over time / T (the mask is all ones at batch 1).  Block =
// 64 channels x 4 time phases (t = phase mod 4, 8 loads in flight per thread),
// the 4 phase sums added in phase order.
__global__ __launch_bounds__(256) void k_time_mean(const float* x, int T, int C, float* out) {
    __shared__ float part[4][64];
    const int cl = threadIdx.x & 63, ph = threadIdx.x >> 6;
    const int c = blockIdx.x * 64 + cl;
    float s = 0.f;
    if (c < C) {
        int t = ph;
        for (; t + 28 < T; t += 32) {
            float v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = x[(long)(t + 4 * u) * C + c];
#pragma unroll
            for (int u = 0; u < 8; ++u) s += v[u];
        }
        for (; t < T; t += 4) s += x[(long)t * C + c];
    }
    part[ph][cl] = s;
    __syncthreads();
    if (ph == 0 && c < C) out[c] = (((part[0][cl] + part[1][cl]) + part[2][cl]) + part[3][cl]) / (float)T;
}
void time_mean(const float* x, int T, int C, float* out, hipStream_t s) {
    hipLaunchKernelGGL(k_time_mean, dim3((C + 63) / 64), dim3(256), 0, s, x, T, C, out);
}

__global__ void k_prelu(const float* x, const float* a, float* out, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    out[i] = x[i] >= 0.f ? x[i] : x[i] * a[i];
}
void prelu_vec(const float* x, const float* a, float* out, int n, hipStream_t s) {
    hipLaunchKernelGGL(k_prelu, dim3((n + 255) / 256), dim3(256), 0, s, x, a, out, n);
}

__global__ void k_add(const float* a, const float* b, float* out, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = a[i] + b[i];
}
void add_vec(const float* a, const float* b, float* out, int n, hipStream_t s) {
    hipLaunchKernelGGL(k_add, dim3((n + 255) / 256), dim3(256), 0, s, a, b, out, n);
}

}  // namespace gsv
