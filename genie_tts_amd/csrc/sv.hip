// V2ProPlus speaker-verification embedding: the reference runs, once per reference clip,
//   sv_emb = model_manager.speaker_verification_model.run(None, {'waveform': audio_16k})[0]
// (src/genie_tts/Audio/ReferenceAudio.py:68-76; session loaded at ModelManager.py:155-170)
// and feeds it to the prompt encoder (prompt_encoder_fp32.onnx#269, Gemm 20480 -> 1024).
// speaker_encoder.onnx is absent here; the model is GPT-SoVITS's v2Pro SV
// (SV.compute_embedding3): Kaldi fbank (80 mel, 16 kHz, dither 0) -> ERes2NetV2
// (baseWidth 24, scale 4, expansion 4).forward3 -> [2048 x 10] channel-major mean over
// time.  Restated op by op in oracle/sv.py, which the GPU tests hold this file to.
//
// Layout: a feature map (C channels over F x T) is position-major [F][T][C] in HBM
// (C innermost), so a 1x1 conv is a GEMM over positions and a 3x3 / stride-2 conv is
// an implicit GEMM whose A rows gather the tap's input position -- no im2col.
// Every conv is k_sv_conv: 64 positions x 64 output channels per block, K = taps x Cin
// in steps of 32 staged through LDS, on the f16 MFMA with both operands split into fp16
// hi + lo (the weights are arbitrary fp32 with BatchNorm folded in at load, so they are
// split too: three MFMAs per product, f32-level accuracy); an activation beyond the fp16
// range re-runs the call on the f32 MFMA (v_mfma_f32_32x32x2f32).  The
// Res2Net pieces fold into the A gather (sp + spx[i]; cat(x, y) of the AFF convs) and
// into the epilogue (bias, residual, ReLU / Hardtanh(0, 20) / SiLU, the AFF mix
// x (1 + tanh v) + y (1 - tanh v)), so each block is its convs and nothing else.
#include <cmath>

#include "common.h"
#include "engine_internal.h"

namespace gsv {
namespace {

constexpr int SV_NMEL = 80, SV_FRAME = 400, SV_SHIFT = 160, SV_NFFT = 512, SV_NBIN = 257;
constexpr int SV_STAGE_PLANES[4] = {64, 128, 256, 512};
constexpr int SV_STAGE_BLOCKS[4] = {3, 4, 6, 3};
constexpr int SV_STAGE_STRIDE[4] = {1, 2, 2, 2};
constexpr bool SV_STAGE_AFF[4] = {false, false, true, true};

enum { SV_ACT_NONE = 0, SV_ACT_RELU = 1, SV_ACT_RELU20 = 2, SV_ACT_SILU = 3 };
enum { SV_A_PLAIN = 0, SV_A_ADD = 1, SV_A_CAT = 2 };

struct SvConvArgs {
    // geometry: input F x T (position-major), output Fo x To, kernel k (1 or 3), stride, pad
    int Fi, Ti, Fo, To, k, stride, pad;
    int cin, cout, K;          // K = k * k * cin (weights [cout][tap][cin])
    // A: channels [0, cin) of src (row stride lda) -- plus src2 (ADD: same channels; CAT:
    // channels [csplit, cin) come from src2's [0, cin - csplit))
    const float* src; long lda;
    const float* src2; long lda2;
    int amode, csplit;
    const float* w;            // [cout][K] fp32, BatchNorm folded
    const __half *wh, *wl;     // the same split into fp16 hi + lo (non-null: the f16 MFMA path)
    int* ovf;                  // f16 path: set when an activation is beyond the fp16 range
    float lim;                 // f16 path: largest |activation| it accepts (65000; tests lower it)
    const float* bias;         // [cout] (folded)
    const float* res; long ldr;     // optional residual added before the activation
    int act;
    const float* ax; long ldx;      // AFF mix: out = ax (1 + tanh v) + ay (1 - tanh v)
    const float* ay; long ldy;
    float* out; long ldo;
    int ksplit;                // > 1: K split over blockIdx.z, raw sums into slab[z][M][cout] (k_sv_reduce)
    float* slab;
};

// The epilogue of one output element: bias (folded BN), residual, activation, AFF mix.
__device__ __forceinline__ void sv_epilogue(const SvConvArgs& a, int row, int col, float acc) {
    float v = acc + (a.bias ? a.bias[col] : 0.f);
    if (a.res) v += a.res[(long)row * a.ldr + col];
    if (a.act == SV_ACT_RELU) v = fmaxf(v, 0.f);
    else if (a.act == SV_ACT_RELU20) v = fminf(fmaxf(v, 0.f), 20.f);
    else if (a.act == SV_ACT_SILU) v = v / (1.f + expf(-v));
    if (a.ax) {
        const float t = tanhf(v);
        v = a.ax[(long)row * a.ldx + col] * (1.f + t) + a.ay[(long)row * a.ldy + col] * (1.f - t);
    }
    a.out[(long)row * a.ldo + col] = v;
}

typedef _Float16 svh8 __attribute__((ext_vector_type(8)));

// H = false: f32 MFMA (v_mfma_f32_32x32x2f32) on f32 tiles.  H = true: the same tiles on
// the f16 MFMA (v_mfma_f32_32x32x16_f16, 16x the f32 rate) with both operands split
// into fp16 hi + lo -- the weights once at load (wh, wl planes), the activations as
// they leave LDS -- and C += Ah Wh + Al Wh + Ah Wl (the dropped Al Wl term is
// ~2^-22 relative, f32-level).  An activation beyond the fp16 range sets *ovf and the
// host runs the model again on the f32 path.
template <bool H>
__global__ __launch_bounds__(256) void k_sv_conv(SvConvArgs a) {
    constexpr int AP = H ? 36 : 33;   // H: 16-byte aligned rows for the fragment reads
    __shared__ __attribute__((aligned(16))) float As[64][AP];
    __shared__ __attribute__((aligned(16))) float Ws[H ? 1 : 64][33];
    __shared__ __attribute__((aligned(16))) _Float16 Wh[H ? 64 : 1][40], Wl[H ? 64 : 1][40];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int wm = wv >> 1, wn = wv & 1;
    const int M = a.Fo * a.To;
    const int m0 = blockIdx.x * 64, n0 = blockIdx.y * 64;   // positions on x: long clips exceed 65535 tiles
    const int sr = tid >> 2, sc = (tid & 3) * 8;
    const int gm = m0 + sr, gn = n0 + sr;
    // this thread's A row: output position (fo, to) -> top-left input position
    int fb = 0, tb = 0;
    if (gm < M) {
        const int fo = gm / a.To, to = gm - fo * a.To;
        fb = fo * a.stride - a.pad;
        tb = to * a.stride - a.pad;
    }
    f32x16 acc;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = 0.f;
    bool big = false;
    // this block's K range: whole 32-k steps, split over blockIdx.z
    const int steps = (a.K + 31) / 32, kz = blockIdx.z, ks = a.ksplit > 1 ? a.ksplit : 1;
    const int k_lo = 32 * (int)((long)steps * kz / ks), k_hi = min(a.K, 32 * (int)((long)steps * (kz + 1) / ks));
    // The next 32-k step's operands are loaded into registers while the current step's
    // MFMAs run (raw values; the Res2Net add is done when they are staged, so the loads
    // stay in flight across the MFMAs)
    float av[8], av2[8], wv8[8];
    uint4 hw, lw;
    auto load = [&](int k0) {
        const int kk = k0 + sc;       // 8 consecutive k of one tap (cin % 8 == 0)
#pragma unroll
        for (int i = 0; i < 8; ++i) av[i] = av2[i] = 0.f;
        if (gm < M && kk < a.K) {
            const int tap = kk / a.cin, ci = kk - tap * a.cin;
            const int dy = tap / a.k, dx = tap - dy * a.k;
            const int fi = fb + dy, ti = tb + dx;
            if (fi >= 0 && fi < a.Fi && ti >= 0 && ti < a.Ti) {
                const long pos = (long)fi * a.Ti + ti;
                const float* p;
                if (a.amode == SV_A_CAT && ci >= a.csplit) p = a.src2 + pos * a.lda2 + (ci - a.csplit);
                else p = a.src + pos * a.lda + ci;
                const float4 x0 = reinterpret_cast<const float4*>(p)[0], x1 = reinterpret_cast<const float4*>(p)[1];
                av[0] = x0.x; av[1] = x0.y; av[2] = x0.z; av[3] = x0.w;
                av[4] = x1.x; av[5] = x1.y; av[6] = x1.z; av[7] = x1.w;
                if (a.amode == SV_A_ADD) {
                    const float4* q = reinterpret_cast<const float4*>(a.src2 + pos * a.lda2 + ci);
                    const float4 y0 = q[0], y1 = q[1];
                    av2[0] = y0.x; av2[1] = y0.y; av2[2] = y0.z; av2[3] = y0.w;
                    av2[4] = y1.x; av2[5] = y1.y; av2[6] = y1.z; av2[7] = y1.w;
                }
            }
        }
        if (H) {
            hw = make_uint4(0u, 0u, 0u, 0u);
            lw = make_uint4(0u, 0u, 0u, 0u);
            if (gn < a.cout && kk < a.K) {
                hw = *reinterpret_cast<const uint4*>(a.wh + (long)gn * a.K + kk);
                lw = *reinterpret_cast<const uint4*>(a.wl + (long)gn * a.K + kk);
            }
        } else {
#pragma unroll
            for (int i = 0; i < 8; ++i) wv8[i] = 0.f;
            if (gn < a.cout && kk < a.K) {
                const float4* p = reinterpret_cast<const float4*>(a.w + (long)gn * a.K + kk);
                const float4 x0 = p[0], x1 = p[1];
                wv8[0] = x0.x; wv8[1] = x0.y; wv8[2] = x0.z; wv8[3] = x0.w;
                wv8[4] = x1.x; wv8[5] = x1.y; wv8[6] = x1.z; wv8[7] = x1.w;
            }
        }
    };
    if (k_lo < k_hi) load(k_lo);
    for (int k0 = k_lo; k0 < k_hi; k0 += 32) {
        if (a.amode == SV_A_ADD) {
#pragma unroll
            for (int i = 0; i < 8; ++i) av[i] += av2[i];
        }
        if (H) {
            *reinterpret_cast<float4*>(&As[sr][sc]) = make_float4(av[0], av[1], av[2], av[3]);
            *reinterpret_cast<float4*>(&As[sr][sc + 4]) = make_float4(av[4], av[5], av[6], av[7]);
            *reinterpret_cast<uint4*>(&Wh[sr][sc]) = hw;
            *reinterpret_cast<uint4*>(&Wl[sr][sc]) = lw;
        } else {
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                As[sr][sc + i] = av[i];
                Ws[sr][sc + i] = wv8[i];
            }
        }
        __syncthreads();
        if (k0 + 32 < k_hi) load(k0 + 32);
        if (H) {
            const int r = lane & 31, hh = lane >> 5;
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) {
                const float* ap = &As[wm * 32 + r][ks * 16 + 8 * hh];
                const float4 x0 = *reinterpret_cast<const float4*>(ap);
                const float4 x1 = *reinterpret_cast<const float4*>(ap + 4);
                const float v[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
                svh8 ahi, alo;
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    big |= !(fabsf(v[j]) < a.lim);
                    const _Float16 hj = (_Float16)v[j];
                    ahi[j] = hj;
                    alo[j] = (_Float16)(v[j] - (float)hj);
                }
                const svh8 bh = *reinterpret_cast<const svh8*>(&Wh[wn * 32 + r][ks * 16 + 8 * hh]);
                const svh8 bl = *reinterpret_cast<const svh8*>(&Wl[wn * 32 + r][ks * 16 + 8 * hh]);
                acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ahi, bh, acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(alo, bh, acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ahi, bl, acc, 0, 0, 0);
            }
        } else {
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                const float x = As[wm * 32 + (lane & 31)][2 * j + (lane >> 5)];
                const float y = Ws[wn * 32 + (lane & 31)][2 * j + (lane >> 5)];
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(x, y, acc, 0, 0, 0);
            }
        }
        __syncthreads();
    }
    if (H && big) atomicOr(a.ovf, 1);
    const int col = n0 + wn * 32 + (lane & 31);
    if (col >= a.cout) return;
    float* slab = ks > 1 ? a.slab + (long)kz * M * a.cout : nullptr;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (row >= M) continue;
        if (slab) slab[(long)row * a.cout + col] = acc[r];
        else sv_epilogue(a, row, col, acc[r]);
    }
}

// Split-K reduce: the slabs summed in z order, then the conv's epilogue.
__global__ __launch_bounds__(256) void k_sv_reduce(SvConvArgs a) {
    const long M = (long)a.Fo * a.To, e = (long)blockIdx.x * 256 + threadIdx.x;
    if (e >= M * a.cout) return;
    const long stride = M * a.cout;
    float v = a.slab[e];
    for (int z = 1; z < a.ksplit; ++z) v += a.slab[z * stride + e];
    sv_epilogue(a, (int)(e / a.cout), (int)(e % a.cout), v);
}

// Kaldi fbank, one block per frame: remove DC, pre-emphasis 0.97, povey window, zero pad
// to 512, power spectrum by a direct DFT over a 512-entry cosine table, 80 mel banks,
// log(max(e, FLT_EPSILON)).  Writes the stem's input x[f][t] (F = 80 rows of T).
__global__ __launch_bounds__(256) void k_sv_fbank(const float* wav, int T, const float* win, const float* cos_tab,
                                                   const float* banks, float* x) {
    __shared__ float fr[SV_FRAME];
    __shared__ float ct[SV_NFFT];
    __shared__ float pw[SV_NBIN + 3];
    __shared__ float red[16];
    const int t = blockIdx.x, tid = threadIdx.x;
    const float* src = wav + (long)t * SV_SHIFT;
    float s = 0.f;
    for (int i = tid; i < SV_FRAME; i += 256) {
        const float v = src[i];
        fr[i] = v;
        s += v;
    }
    for (int i = tid; i < SV_NFFT; i += 256) ct[i] = cos_tab[i];
    const float mean = block_sum(s, red) / (float)SV_FRAME;   // block_sum syncs: fr is complete
    float y[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int i = tid + 256 * j;
        y[j] = 0.f;
        if (i < SV_FRAME) {
            const float cur = fr[i] - mean, prev = fr[i > 0 ? i - 1 : 0] - mean;
            y[j] = (cur - 0.97f * prev) * win[i];
        }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int i = tid + 256 * j;
        if (i < SV_FRAME) fr[i] = y[j];
    }
    __syncthreads();
    for (int b = tid; b < SV_NBIN; b += 256) {
        float re = 0.f, im = 0.f;
        for (int n = 0; n < SV_FRAME; ++n) {
            const int e = (b * n) & (SV_NFFT - 1);
            re += fr[n] * ct[e];
            im += fr[n] * ct[(e + 3 * SV_NFFT / 4) & (SV_NFFT - 1)];   // sin(2 pi e / N) = cos(2 pi (e - N/4) / N)
        }
        pw[b] = re * re + im * im;
    }
    __syncthreads();
    if (tid < SV_NMEL) {
        const float* bk = banks + tid * SV_NBIN;
        float e = 0.f;
        for (int b = 0; b < SV_NBIN; ++b) e += pw[b] * bk[b];
        x[(long)tid * T + t] = logf(fmaxf(e, 1.1920928955078125e-07f));
    }
}

// stem: Conv2d(1 -> 64, 3x3, pad 1) + folded BatchNorm + ReLU on x [80][T] -> [80 T][64]
__global__ __launch_bounds__(256) void k_sv_stem(const float* x, int T, const float* w, const float* b, float* out) {
    const long p = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int c = threadIdx.x & 63;
    if (p >= (long)SV_NMEL * T) return;
    const int f = (int)(p / T), t = (int)(p - (long)f * T);
    float s = b[c];
#pragma unroll
    for (int dy = 0; dy < 3; ++dy)
#pragma unroll
        for (int dx = 0; dx < 3; ++dx) {
            const int fi = f + dy - 1, ti = t + dx - 1;
            if (fi >= 0 && fi < SV_NMEL && ti >= 0 && ti < T) s += w[c * 9 + dy * 3 + dx] * x[(long)fi * T + ti];
        }
    out[p * 64 + c] = fmaxf(s, 0.f);
}

// sv_emb[c * F + f] = mean_t fuse[(f T + t)][c]   (forward3: flatten(1, 2).mean(-1))
__global__ __launch_bounds__(256) void k_sv_pool(const float* x, int F, int T, int C, float* out) {
    const int e = blockIdx.x * 256 + threadIdx.x;
    if (e >= C * F) return;
    const int f = e / C, c = e - f * C;
    const float* p = x + (long)f * T * C + c;
    float s = 0.f;
    for (int t = 0; t < T; ++t) s += p[(long)t * C];
    out[c * F + f] = s / (float)T;
}

int sv_down(int n) { return (n - 1) / 2 + 1; }   // 1x1 stride 2 pad 0 == 3x3 stride 2 pad 1
constexpr size_t SV_SLAB_CAP = (size_t)8 << 20;   // split-K slab floats (32 MB)

}  // namespace

int sv_frames(int n_samples) { return n_samples < SV_FRAME ? 0 : 1 + (n_samples - SV_FRAME) / SV_SHIFT; }

}  // namespace gsv

using namespace gsv;

// Conv weight [co][ci][kh][kw] -> [co][(kh kw) tap][ci] with the BatchNorm `bn` folded:
// W' = W g / sqrt(var + eps), b' = (b - mean) g / sqrt(var + eps) + beta.
int gsv_engine::sv_conv_upload(const std::string& wname, const std::string& bname, const std::string& bn,
                               SvConv* c) {
    const Staged* w = find(wname);
    if (!w || w->dims.size() != 4) return set_error(GSV_E_WEIGHT, "missing/bad SV weight " + wname);
    const int co = (int)w->dims[0], ci = (int)w->dims[1], k = (int)w->dims[2];
    if (w->dims[3] != k || ci % 8) return set_error(GSV_E_WEIGHT, "bad SV conv shape " + wname);
    std::vector<float> scale(co, 1.f), shift(co, 0.f);
    // the conv's own bias (optional: the state-dict layout has none on BatchNorm'd convs;
    // an export that folded the BatchNorm carries it there instead)
    const Staged* b = bname.empty() ? nullptr : find(bname);
    if (b) {
        if ((int)b->data.size() != co) return set_error(GSV_E_WEIGHT, "bad SV weight " + bname);
        for (int o = 0; o < co; ++o) shift[o] = b->data[o];
    }
    const bool has_bn = !bn.empty() && find(bn + ".weight");
    if (!bn.empty() && !has_bn && !b)
        return set_error(GSV_E_WEIGHT, "missing SV BatchNorm " + bn + " (and no folded bias " + bname + ")");
    if (has_bn) {
        const Staged *g = find(bn + ".weight"), *be = find(bn + ".bias"), *mu = find(bn + ".running_mean"),
                     *var = find(bn + ".running_var");
        if (!g || !be || !mu || !var || (int)g->data.size() != co || (int)be->data.size() != co ||
            (int)mu->data.size() != co || (int)var->data.size() != co)
            return set_error(GSV_E_WEIGHT, "missing/bad SV BatchNorm " + bn);
        for (int o = 0; o < co; ++o) {
            const float s = g->data[o] / sqrtf(var->data[o] + 1e-5f);
            shift[o] = (shift[o] - mu->data[o]) * s + be->data[o];
            scale[o] = s;
        }
    }
    const int taps = k * k, K = taps * ci;
    std::vector<float> h((size_t)co * K);
    for (int o = 0; o < co; ++o)
        for (int i = 0; i < ci; ++i)
            for (int t = 0; t < taps; ++t)
                h[(size_t)o * K + t * ci + i] = w->data[((size_t)o * ci + i) * taps + t] * scale[o];
    c->w = (float*)dalloc(h.size() * 4);
    c->b = (float*)dalloc((size_t)co * 4);
    if (!c->w || !c->b) return set_error(GSV_E_HIP, "hipMalloc failed for " + wname);
    hipMemcpy(c->w, h.data(), h.size() * 4, hipMemcpyHostToDevice);
    // fp16 hi + lo planes for the f16 MFMA path, unless a weight is beyond the fp16 range
    bool fits = true;
    for (float v : h) fits = fits && std::fabs(v) < 65000.f;
    if (fits) {
        std::vector<__half> hi(h.size()), lo(h.size());
        for (size_t i = 0; i < h.size(); ++i) {
            hi[i] = __float2half(h[i]);
            lo[i] = __float2half(h[i] - __half2float(hi[i]));
        }
        c->wh = (__half*)dalloc(hi.size() * 2);
        c->wl = (__half*)dalloc(lo.size() * 2);
        if (!c->wh || !c->wl) return set_error(GSV_E_HIP, "hipMalloc failed for " + wname);
        hipMemcpy(c->wh, hi.data(), hi.size() * 2, hipMemcpyHostToDevice);
        hipMemcpy(c->wl, lo.data(), lo.size() * 2, hipMemcpyHostToDevice);
    }
    hipMemcpy(c->b, shift.data(), (size_t)co * 4, hipMemcpyHostToDevice);
    c->cin = ci;
    c->cout = co;
    c->k = k;
    return 0;
}

int gsv_engine::finalize_sv() {
    SvWeights& S = sv;
    {   // stem (cin 1: its own kernel)
        const Staged* w = find("conv1.weight");
        if (!w || w->data.size() != 64 * 9) return set_error(GSV_E_WEIGHT, "missing/bad SV weight conv1.weight");
        const Staged *g = find("bn1.weight"), *be = find("bn1.bias"), *mu = find("bn1.running_mean"),
                     *var = find("bn1.running_var"), *cb = find("conv1.bias");
        if ((!g || !be || !mu || !var) && !cb) return set_error(GSV_E_WEIGHT, "missing SV BatchNorm bn1");
        if (cb && cb->data.size() != 64) return set_error(GSV_E_WEIGHT, "bad SV weight conv1.bias");
        std::vector<float> hw(64 * 9), hb(64);
        for (int o = 0; o < 64; ++o) {
            const float b0 = cb ? cb->data[o] : 0.f;
            if (g && be && mu && var) {
                const float s = g->data[o] / sqrtf(var->data[o] + 1e-5f);
                for (int t = 0; t < 9; ++t) hw[o * 9 + t] = w->data[o * 9 + t] * s;
                hb[o] = (b0 - mu->data[o]) * s + be->data[o];
            } else {   // BatchNorm folded into the conv by the export
                for (int t = 0; t < 9; ++t) hw[o * 9 + t] = w->data[o * 9 + t];
                hb[o] = b0;
            }
        }
        S.stem_w = (float*)dalloc(hw.size() * 4);
        S.stem_b = (float*)dalloc(hb.size() * 4);
        hipMemcpy(S.stem_w, hw.data(), hw.size() * 4, hipMemcpyHostToDevice);
        hipMemcpy(S.stem_b, hb.data(), hb.size() * 4, hipMemcpyHostToDevice);
    }
    S.blocks.clear();
    int cin = 64;
    for (int s = 0; s < 4; ++s) {
        const int planes = SV_STAGE_PLANES[s], width = planes * 24 / 64;
        for (int b = 0; b < SV_STAGE_BLOCKS[s]; ++b) {
            SvBlock B;
            B.width = width;
            B.stride = b == 0 ? SV_STAGE_STRIDE[s] : 1;
            B.aff = SV_STAGE_AFF[s];
            const std::string p = "layer" + std::to_string(s + 1) + "." + std::to_string(b);
            if (int e = sv_conv_upload(p + ".conv1.weight", p + ".conv1.bias", p + ".bn1", &B.conv1)) return e;
            for (int i = 0; i < 4; ++i)
                if (int e = sv_conv_upload(p + ".convs." + std::to_string(i) + ".weight",
                                           p + ".convs." + std::to_string(i) + ".bias",
                                           p + ".bns." + std::to_string(i), &B.convs[i]))
                    return e;
            if (B.aff)
                for (int i = 0; i < 3; ++i) {
                    const std::string q = p + ".fuse_models." + std::to_string(i) + ".local_att.";
                    if (int e = sv_conv_upload(q + "0.weight", q + "0.bias", q + "1", &B.aff_a[i])) return e;
                    if (int e = sv_conv_upload(q + "3.weight", q + "3.bias", q + "4", &B.aff_b[i])) return e;
                }
            if (int e = sv_conv_upload(p + ".conv3.weight", p + ".conv3.bias", p + ".bn3", &B.conv3)) return e;
            B.has_sc = find(p + ".shortcut.0.weight") != nullptr;
            if (B.has_sc)
                if (int e = sv_conv_upload(p + ".shortcut.0.weight", p + ".shortcut.0.bias", p + ".shortcut.1", &B.sc)) return e;
            if (B.conv1.cin != cin || B.conv3.cout != planes * 4 || (!B.has_sc && (B.stride != 1 || cin != planes * 4)))
                return set_error(GSV_E_WEIGHT, "SV block " + p + " shape mismatch");
            S.blocks.push_back(B);
            cin = planes * 4;
        }
    }
    if (int e = sv_conv_upload("layer3_ds.weight", "layer3_ds.bias", "", &S.ds34)) return e;
    if (int e = sv_conv_upload("fuse34.local_att.0.weight", "fuse34.local_att.0.bias", "fuse34.local_att.1", &S.fuse_a))
        return e;
    if (int e = sv_conv_upload("fuse34.local_att.3.weight", "fuse34.local_att.3.bias", "fuse34.local_att.4", &S.fuse_b))
        return e;
    // fbank tables (torchaudio.compliance.kaldi semantics; computed in double, stored f32)
    std::vector<float> win(SV_FRAME), ct(SV_NFFT), banks((size_t)SV_NMEL * SV_NBIN, 0.f);
    for (int i = 0; i < SV_FRAME; ++i)
        win[i] = (float)pow(0.5 - 0.5 * cos(2.0 * M_PI * i / (SV_FRAME - 1)), 0.85);
    for (int i = 0; i < SV_NFFT; ++i) ct[i] = (float)cos(2.0 * M_PI * i / SV_NFFT);
    auto mel = [](double f) { return 1127.0 * log(1.0 + f / 700.0); };
    const double lo = mel(20.0), hi = mel(8000.0), delta = (hi - lo) / (SV_NMEL + 1);
    for (int m = 0; m < SV_NMEL; ++m) {
        const double l = lo + m * delta, c = lo + (m + 1) * delta, r = lo + (m + 2) * delta;
        for (int k = 0; k < SV_NFFT / 2; ++k) {
            const double v = mel(k * 16000.0 / SV_NFFT);
            const double up = (v - l) / (c - l), down = (r - v) / (r - c);
            banks[(size_t)m * SV_NBIN + k] = (float)std::max(0.0, std::min(up, down));
        }
    }
    S.win = (float*)dalloc(win.size() * 4);
    S.cos_tab = (float*)dalloc(ct.size() * 4);
    S.banks = (float*)dalloc(banks.size() * 4);
    hipMemcpy(S.win, win.data(), win.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(S.cos_tab, ct.data(), ct.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(S.banks, banks.data(), banks.size() * 4, hipMemcpyHostToDevice);
    S.ready = true;
    return 0;
}

namespace {
struct SvMap {   // a feature map in the workspace
    float* p;
    int F, T, C;
    long ld;     // row stride (channels of the buffer it lives in)
};

SvConvArgs sv_args(const SvConv& c, const SvMap& in, int stride, int pad, float* out, long ldo, int* ovf,
                   float lim) {
    SvConvArgs a{};
    a.Fi = in.F; a.Ti = in.T;
    a.k = c.k; a.stride = stride; a.pad = pad;
    a.Fo = (in.F + 2 * pad - c.k) / stride + 1;
    a.To = (in.T + 2 * pad - c.k) / stride + 1;
    a.cin = c.cin; a.cout = c.cout; a.K = c.k * c.k * c.cin;
    a.src = in.p; a.lda = in.ld;
    a.amode = SV_A_PLAIN;
    a.w = c.w; a.bias = c.b;
    if (ovf && c.wh) {   // the split-fp16 path (ovf: its range flag)
        a.wh = c.wh; a.wl = c.wl; a.ovf = ovf; a.lim = lim;
    }
    a.act = SV_ACT_NONE;
    a.out = out; a.ldo = ldo;
    return a;
}

// A conv with few blocks (stages 3-4: 33-352 for 256 CUs) waits out a memory round trip
// per 32-k step on few CUs; it splits K over up to 8 blocks (>= 4 steps each, up to ~512
// blocks) when the slabs fit (slab_cap floats), and k_sv_reduce applies the epilogue.
void sv_conv(SvConvArgs a, hipStream_t st, float* slab, size_t slab_cap) {
    const int M = a.Fo * a.To;
    const int blocks = ((M + 63) / 64) * ((a.cout + 63) / 64), steps = (a.K + 31) / 32;
    int ks = 1;
    while (ks < 8 && blocks * ks < 512 && steps / (2 * ks) >= 4 && (size_t)2 * ks * M * a.cout <= slab_cap) ks *= 2;
    a.ksplit = ks;
    a.slab = slab;
    const dim3 grid((M + 63) / 64, (a.cout + 63) / 64, ks);
    if (a.wh) hipLaunchKernelGGL(k_sv_conv<true>, grid, dim3(256), 0, st, a);
    else hipLaunchKernelGGL(k_sv_conv<false>, grid, dim3(256), 0, st, a);
    if (ks > 1)
        hipLaunchKernelGGL(k_sv_reduce, dim3((unsigned)(((long)M * a.cout + 255) / 256)), dim3(256), 0, st, a);
}
}  // namespace

size_t gsv_engine::sv_ws_floats(int T) {
    const size_t P1 = (size_t)SV_NMEL * T;
    // x (fbank) + 3 block buffers [P1][256] + H, O [P1][96] + Z [P1][24] + AFF tmp + ds / fuse maps
    const int T4 = sv_down(sv_down(sv_down(T)));
    return P1 + 3 * P1 * 256 + 2 * P1 * 96 + P1 * 24 + P1 * 24 + 2 * (size_t)10 * T4 * 2048 + (size_t)10 * T4 * 512 + 64 +
           SV_SLAB_CAP;
}

int gsv_engine::sv_forward(const float* wav, int n, float* out, hipStream_t st, int* ovf, float lim) {
    const SvWeights& S = sv;
    const int T = sv_frames(n);
    const size_t P1 = (size_t)SV_NMEL * T;
    const size_t need = sv_ws_floats(T);
    if (need > sv_ws_n) {
        const size_t cap = grow_cap(need, sv_ws_n);
        retire(sv_ws);
        sv_ws = nullptr;
        sv_ws_n = 0;
        reclaim();
        if (hipMalloc(&sv_ws, cap * 4) != hipSuccess) return set_error(GSV_E_HIP, "SV workspace");
        sv_ws_n = cap;
    }
    float* x = sv_ws;
    float* big[3] = {x + P1, x + P1 + P1 * 256, x + P1 + 2 * P1 * 256};
    float* H = big[2] + P1 * 256;
    float* O = H + P1 * 96;
    float* Z = O + P1 * 96;
    float* A = Z + P1 * 24;
    const int T4 = sv_down(sv_down(sv_down(T)));
    float* ds = A + P1 * 24;
    float* fuse = ds + (size_t)10 * T4 * 2048;
    float* fa = fuse + (size_t)10 * T4 * 2048;
    float* slab = fa + (size_t)10 * T4 * 512 + 64;
    auto conv = [&](const SvConvArgs& c) { sv_conv(c, st, slab, SV_SLAB_CAP); };

    hipLaunchKernelGGL(k_sv_fbank, dim3(T), dim3(256), 0, st, wav, T, S.win, S.cos_tab, S.banks, x);
    hipLaunchKernelGGL(k_sv_stem, dim3((unsigned)((P1 + 3) / 4)), dim3(256), 0, st, x, T, S.stem_w, S.stem_b, big[0]);
    SvMap cur{big[0], SV_NMEL, T, 64, 64};
    int cur_buf = 0, keep_buf = -1;
    SvMap out3{};
    size_t bi = 0;
    for (int s = 0; s < 4; ++s) {
        for (int b = 0; b < SV_STAGE_BLOCKS[s]; ++b, ++bi) {
            const SvBlock& B = S.blocks[bi];
            const int w = B.width, w4 = 4 * w;
            int ob = 0;
            while (ob == cur_buf || ob == keep_buf) ++ob;
            // conv1 (1x1, stride) + BN + Hardtanh -> H [P][4w]
            SvConvArgs c1 = sv_args(B.conv1, cur, B.stride, 0, H, w4, ovf, lim);
            c1.act = SV_ACT_RELU20;
            conv(c1);
            const SvMap hmap{H, c1.Fo, c1.To, w4, w4};
            // the split chain: sp_0 = conv(spx_0); sp_i = conv(sp_{i-1} + spx_i) or conv(AFF(sp_{i-1}, spx_i))
            for (int i = 0; i < 4; ++i) {
                SvMap in{H + i * w, hmap.F, hmap.T, w, w4};
                SvConvArgs c = sv_args(B.convs[i], in, 1, 1, O + i * w, w4, ovf, lim);
                if (i > 0 && !B.aff) {
                    c.amode = SV_A_ADD;
                    c.src = O + (i - 1) * w; c.lda = w4;
                    c.src2 = H + i * w; c.lda2 = w4;
                } else if (i > 0) {
                    // AFF: t = SiLU(conv_a(cat(sp, spx_i))), z = sp (1 + tanh conv_b(t)) + spx_i (1 - tanh ...)
                    SvMap cat{O + (i - 1) * w, hmap.F, hmap.T, 2 * w, w4};
                    SvConvArgs ca = sv_args(B.aff_a[i - 1], cat, 1, 0, A, w / 4, ovf, lim);
                    ca.amode = SV_A_CAT;
                    ca.src2 = H + i * w; ca.lda2 = w4; ca.csplit = w;
                    ca.act = SV_ACT_SILU;
                    conv(ca);
                    SvMap tm{A, hmap.F, hmap.T, w / 4, w / 4};
                    SvConvArgs cb = sv_args(B.aff_b[i - 1], tm, 1, 0, Z, w, ovf, lim);
                    cb.ax = O + (i - 1) * w; cb.ldx = w4;
                    cb.ay = H + i * w; cb.ldy = w4;
                    conv(cb);
                    c.src = Z; c.lda = w;
                }
                c.act = SV_ACT_RELU20;
                conv(c);
            }
            // shortcut (1x1 conv + BN, or identity) and conv3 + BN + residual + Hardtanh
            float* y = big[ob];
            const long cout = B.conv3.cout;
            const float* res = cur.p;
            long ldr = cur.ld;
            if (B.has_sc) {
                SvConvArgs sc = sv_args(B.sc, cur, B.stride, 0, y, cout, ovf, lim);
                conv(sc);
                res = y;
                ldr = cout;
            }
            const SvMap omap{O, hmap.F, hmap.T, w4, w4};
            SvConvArgs c3 = sv_args(B.conv3, omap, 1, 0, y, cout, ovf, lim);
            c3.res = res; c3.ldr = ldr;
            c3.act = SV_ACT_RELU20;
            conv(c3);
            cur = SvMap{y, hmap.F, hmap.T, (int)cout, cout};
            cur_buf = ob;
        }
        if (s == 2) {
            out3 = cur;
            keep_buf = cur_buf;
        }
    }
    // layer3_ds (3x3 stride 2, no BN) and fuse34 = AFF(out4, out3_ds)
    SvConvArgs d = sv_args(S.ds34, out3, 2, 1, ds, 2048, ovf, lim);
    conv(d);
    if (d.Fo != cur.F || d.To != cur.T) return set_error(GSV_E_ARG, "SV layer3_ds / layer4 shape mismatch");
    SvMap cat{cur.p, cur.F, cur.T, 4096, cur.ld};
    SvConvArgs fa_ = sv_args(S.fuse_a, cat, 1, 0, fa, 512, ovf, lim);
    fa_.amode = SV_A_CAT;
    fa_.src2 = ds; fa_.lda2 = 2048; fa_.csplit = 2048;
    fa_.act = SV_ACT_SILU;
    conv(fa_);
    SvMap tm{fa, cur.F, cur.T, 512, 512};
    SvConvArgs fb = sv_args(S.fuse_b, tm, 1, 0, fuse, 2048, ovf, lim);
    fb.ax = cur.p; fb.ldx = cur.ld;
    fb.ay = ds; fb.ldy = 2048;
    conv(fb);
    hipLaunchKernelGGL(k_sv_pool, dim3((2048 * cur.F + 255) / 256), dim3(256), 0, st, fuse, cur.F, cur.T, 2048, out);
    return hipGetLastError() == hipSuccess ? 0 : set_error(GSV_E_HIP, "SV launch");
}

extern "C" int gsv_sv_frames(int n_samples) { return sv_frames(n_samples); }

extern "C" int gsv_sv(gsv_engine* eng, const float* audio_16k, int n_samples, float* sv_emb, void* stream) {
    if (!eng) return set_error(GSV_E_ARG, "null engine");
    if (!audio_16k || !sv_emb) return set_error(GSV_E_ARG, "null arg");
    if (!eng->finalized || !eng->sv.ready) return set_error(GSV_E_STATE, "SV weights not loaded");
    if (sv_frames(n_samples) < 1) return set_error(GSV_E_ARG, "audio too short for the SV fbank (< 400 samples)");
    hipSetDevice(eng->device);
    StreamScope sc(eng, stream);
    if (!eng->sv_f16) return eng->sv_forward(audio_16k, n_samples, sv_emb, sc.st(), nullptr, 0.f);
    if (!eng->sv_ovf) {
        if (hipMalloc((void**)&eng->sv_ovf, 4) != hipSuccess ||
            hipHostMalloc((void**)&eng->sv_ovf_host, 4, hipHostMallocDefault) != hipSuccess)
            return set_error(GSV_E_HIP, "SV overflow flag");
    }
    hipMemsetAsync(eng->sv_ovf, 0, 4, sc.st());
    if (int r = eng->sv_forward(audio_16k, n_samples, sv_emb, sc.st(), eng->sv_ovf, eng->sv_f16_limit)) return r;
    hipMemcpyAsync(eng->sv_ovf_host, eng->sv_ovf, 4, hipMemcpyDeviceToHost, sc.st());
    if (hipStreamSynchronize(sc.st()) != hipSuccess) return set_error(GSV_E_HIP, "SV sync");
    if (*eng->sv_ovf_host == 0) return 0;
    // an activation beyond the fp16 range: the same call on the f32 MFMA path
    ++eng->sv_f32_reruns;
    return eng->sv_forward(audio_16k, n_samples, sv_emb, sc.st(), nullptr, 0.f);
}
