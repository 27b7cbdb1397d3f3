// CN-HuBERT SSL extractor (chinese-hubert-base): the reference runs
//   ssl_content = model_manager.cn_hubert.run(None, {'input_values': audio_16k})[0]
// (src/genie_tts/Audio/ReferenceAudio.py:48-52, session loaded at
// ModelManager.py:172-195).  The graph is GPT-SoVITS's export of transformers'
// HubertModel(raw 16 kHz audio)["last_hidden_state"].transpose(1, 2); its file is
// not in this container, so the op order below follows the published model
// (transformers HubertModel, feat_extract_norm="group", post-norm encoder):
//
//   conv0 (1 -> 512, k10 s5, no bias) -> GroupNorm(512 groups) -> GELU
//   conv1..6 (512 -> 512, k3 s2 x4, k2 s2 x2, no bias) -> GELU
//   LayerNorm(512) -> Linear 512 -> 768
//   h += GELU(pos_conv(h))   (Conv1d 768, k128, pad 64, 16 groups, last frame dropped)
//   LayerNorm(768); 12 x [MHA(12 x 64) + residual -> LN -> FFN 3072 GELU + residual -> LN]
//   out [768][T] (channel-major, the graph's transposed output)
//
// Layout: activations time-major [T][C] in HBM.  A stride-s conv over a
// time-major input is a plain GEMM with no im2col: output row t reads the k
// consecutive input rows starting at s t, i.e. A = X with lda = s C and K = k C
// (weights re-ordered to [co][tap][ci] at load).  Every GEMM is gemm_nt (t2s.hip):
// split-fp16 activations on the f16 MFMA, weights as W16 planes -- the fp16 bin's
// exact values as one plane, an fp32 export's values as hi + lo; attention is k_mha
// (vits.hip).
// The grouped positional conv is 16 GEMMs over per-group im2col rows (K = 6144)
// split over K into slabs, reduced with bias + GELU + the residual add.
#include "common.h"
#include "engine_internal.h"

#include <algorithm>

namespace gsv {
namespace {

__device__ __forceinline__ float gelu_erf(float v) { return 0.5f * v * (1.f + erff(v * 0.70710678118654752f)); }

// conv0: out[t][c] = sum_j w[c][j] x[5 t + j]  (no bias), one block per time step
__global__ __launch_bounds__(512) void k_hb_conv0(const float* x, const float* w, int T0, float* out) {
    const int t = blockIdx.x, c = threadIdx.x;
    __shared__ float xs[10];
    if (c < 10) xs[c] = x[(long)5 * t + c];
    __syncthreads();
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < 10; ++j) s += w[c * 10 + j] * xs[j];
    out[(long)t * 512 + c] = s;
}

// GroupNorm(num_groups = C): per-channel statistics over time of a time-major
// [T][C] tensor.  Pass 1: partial sums of (x - shift_c) per time slice; the
// finaliser forms mean_c; pass 2 the same for (x - mean_c)^2 (two-pass, exact
// mean as torch's group_norm computes it up to summation order).
__global__ __launch_bounds__(512) void k_hb_colsum(const float* x, int T, int C, const float* center, int sq,
                                                    float* part) {
    const int c = threadIdx.x, z = blockIdx.x, nz = gridDim.x;
    const int t0 = (int)((long)T * z / nz), t1 = (int)((long)T * (z + 1) / nz);
    const float m = center ? center[c] : 0.f;
    float s = 0.f;
    for (int t = t0; t < t1; ++t) {
        const float d = x[(long)t * C + c] - m;
        s += sq ? d * d : d;
    }
    part[(long)z * C + c] = s;
}
__global__ __launch_bounds__(512) void k_hb_colfin(const float* part, int nz, int T, int C, int sq, float* mean,
                                                    float* rstd) {
    const int c = threadIdx.x;
    float s = 0.f;
    for (int z = 0; z < nz; ++z) s += part[(long)z * C + c];
    if (!sq) mean[c] = s / (float)T;
    else rstd[c] = 1.f / sqrtf(s / (float)T + 1e-5f);
}
__global__ __launch_bounds__(512) void k_hb_gn_gelu(float* x, int C, const float* mean, const float* rstd,
                                                     const float* g, const float* b) {
    const int t = blockIdx.x, c = threadIdx.x;
    float* p = x + (long)t * C + c;
    *p = gelu_erf((*p - mean[c]) * rstd[c] * g[c] + b[c]);
}

// im2col of the positional conv, all groups: A[g][t][j * 48 + i] = h[t - 64 + j][48 g + i]
__global__ __launch_bounds__(256) void k_hb_pos_im2col(const float* h, int T, float* A) {
    const int t = blockIdx.x, g = blockIdx.y;
    float* dst = A + ((long)g * T + t) * 6144;
    for (int e = threadIdx.x; e < 6144; e += 256) {
        const int j = e / 48, i = e - j * 48, ts = t - 64 + j;
        dst[e] = (ts >= 0 && ts < T) ? h[(long)ts * 768 + 48 * g + i] : 0.f;
    }
}
// h[t][c] += GELU(bias[c] + sum_z slab[z][t][c])  (slabs summed in z order)
__global__ __launch_bounds__(256) void k_hb_pos_reduce(const float* slabs, int nz, long zstride, const float* bias,
                                                        float* h, int n) {
    const int e = blockIdx.x * 256 + threadIdx.x;
    if (e >= n) return;
    float s = slabs[e];
    for (int z = 1; z < nz; ++z) s += slabs[(long)z * zstride + e];
    h[e] = h[e] + gelu_erf(bias[e % 768] + s);
}
// [T][768] -> [768][T]
__global__ __launch_bounds__(256) void k_hb_transpose(const float* h, int T, float* out) {
    __shared__ float tile[32][33];
    const int t0 = blockIdx.x * 32, c0 = blockIdx.y * 32;
    const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
    for (int r = ty; r < 32; r += 8) {
        const int t = t0 + r;
        tile[r][tx] = t < T ? h[(long)t * 768 + c0 + tx] : 0.f;
    }
    __syncthreads();
    for (int r = ty; r < 32; r += 8) {
        const int t = t0 + tx;
        if (t < T) out[(long)(c0 + r) * T + t] = tile[tx][r];
    }
}

constexpr int HB_KS[7] = {10, 3, 3, 3, 3, 2, 2};
constexpr int HB_SS[7] = {5, 2, 2, 2, 2, 2, 2};

}  // namespace

// LayerNorm over rows of D (<= 1024) values, two-pass (mean, then mean of squared
// deviations), one block per row (CN-HuBERT eps 1e-5, RoBERTa eps 1e-12).
// With slabs: the input row is res + (bias + sum_z slab_z) (split-K GEMM partials
// summed in slab order: EPI_RESID's res + (bias + acc) with acc formed in slices).
__global__ __launch_bounds__(256) void k_ln_rows_d(const float* in, float* out, int D, const float* g, const float* b,
                                                    float eps, int nslab, long sstride, const float* bias,
                                                    const float* res) {
    __shared__ float red[16];
    const long r = blockIdx.x;
    const float* x = in + r * D;
    float v[4];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int d = threadIdx.x + 256 * i;
        if (nslab == 0) {
            v[i] = d < D ? x[d] : 0.f;
        } else if (d < D) {
            float acc = x[d];
            for (int z = 1; z < nslab; ++z) acc += x[z * sstride + d];
            v[i] = res[r * D + d] + (bias[d] + acc);
        } else {
            v[i] = 0.f;
        }
        s += v[i];
    }
    const float mean = block_sum(s, red) / (float)D;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int d = threadIdx.x + 256 * i;
        if (d < D) q += (v[i] - mean) * (v[i] - mean);
    }
    const float den = sqrtf(block_sum(q, red) / (float)D + eps);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int d = threadIdx.x + 256 * i;
        if (d < D) out[r * D + d] = (v[i] - mean) / den * g[d] + b[d];
    }
}

GemmArgs gemm_f16(int M, int N, int K, const float* A, long lda, const void* W, const float* bias, float* C,
                  long ldc, int mode, const float* res, long ldr) {
    GemmArgs a{};
    a.M = M; a.N = N; a.K = K;
    a.A = A; a.lda = lda;
    a.W = W; a.ldw = K; a.w_f16 = 1;
    a.bias = bias;
    a.C = C; a.ldc = ldc;
    a.mode = mode;
    a.res = res; a.ldr = ldr;
    return a;
}

GemmArgs gemm_w16(int M, int N, int K, const float* A, long lda, const W16& W, const float* bias, float* C,
                  long ldc, int mode, const float* res, long ldr) {
    GemmArgs a = gemm_f16(M, N, K, A, lda, W.hi, bias, C, ldc, mode, res, ldr);
    a.Wl = W.lo;
    return a;
}

void layernorm_rows_d(const float* in, float* out, int rows, int D, const float* g, const float* b, float eps,
                      hipStream_t s) {
    hipLaunchKernelGGL(k_ln_rows_d, dim3(rows), dim3(256), 0, s, in, out, D, g, b, eps, 0, 0L, nullptr, nullptr);
}

void layernorm_rows_d_slabs(const float* slabs, int nslab, long slab_stride, const float* bias, const float* res,
                            float* out, int rows, int D, const float* g, const float* b, float eps, hipStream_t s) {
    hipLaunchKernelGGL(k_ln_rows_d, dim3(rows), dim3(256), 0, s, slabs, out, D, g, b, eps, nslab, slab_stride, bias,
                       res);
}

int hubert_frames(int n) {
    int T = n;
    for (int i = 0; i < 7; ++i) {
        if (T < HB_KS[i]) return 0;
        T = (T - HB_KS[i]) / HB_SS[i] + 1;
    }
    return T;
}

}  // namespace gsv

using namespace gsv;

// Weights (transformers HubertModel names; encoder.pos_conv_embed.conv.weight is
// the weight-normed kernel g v / ||v|| as an exported graph stores it).
int gsv_engine::finalize_hubert() {
    int err = 0;
    HubertWeights& H = hubert;
    H.conv0_w = up_f32("feature_extractor.conv_layers.0.conv.weight", &err);
    H.gn_w = up_f32("feature_extractor.conv_layers.0.layer_norm.weight", &err);
    H.gn_b = up_f32("feature_extractor.conv_layers.0.layer_norm.bias", &err);
    for (int i = 1; i < 7; ++i) {
        // [co][ci][k] -> [co][k][ci]: one output row reads k consecutive time-major rows
        const std::string n = "feature_extractor.conv_layers." + std::to_string(i) + ".conv.weight";
        const Staged* s = find(n);
        const int k = HB_KS[i];
        if (!s || s->data.size() != (size_t)512 * 512 * k) return set_error(GSV_E_WEIGHT, "missing/bad weight " + n);
        std::vector<float> h((size_t)512 * 512 * k);
        for (int co = 0; co < 512; ++co)
            for (int ci = 0; ci < 512; ++ci)
                for (int j = 0; j < k; ++j) h[((size_t)co * k + j) * 512 + ci] = s->data[((size_t)co * 512 + ci) * k + j];
        H.conv_w[i] = upload_w16(n, h, &err);
    }
    H.fp_ln_w = up_f32("feature_projection.layer_norm.weight", &err);
    H.fp_ln_b = up_f32("feature_projection.layer_norm.bias", &err);
    H.fp_w = up_w16("feature_projection.projection.weight", &err);
    H.fp_b = up_f32("feature_projection.projection.bias", &err);
    {
        // [768][48][128] -> per group g: [48 o][128 j][48 i] (im2col K order j, i)
        const std::string n = "encoder.pos_conv_embed.conv.weight";
        const Staged* s = find(n);
        if (!s || s->data.size() != (size_t)768 * 48 * 128) return set_error(GSV_E_WEIGHT, "missing/bad weight " + n);
        std::vector<float> h((size_t)768 * 6144);
        for (int co = 0; co < 768; ++co)
            for (int i = 0; i < 48; ++i)
                for (int j = 0; j < 128; ++j) h[(size_t)co * 6144 + j * 48 + i] = s->data[((size_t)co * 48 + i) * 128 + j];
        H.pos_w = upload_w16(n, h, &err);
    }
    H.pos_b = up_f32("encoder.pos_conv_embed.conv.bias", &err);
    H.enc_ln_w = up_f32("encoder.layer_norm.weight", &err);
    H.enc_ln_b = up_f32("encoder.layer_norm.bias", &err);
    for (int l = 0; l < 12; ++l) {
        const std::string p = "encoder.layers." + std::to_string(l) + ".";
        HubertLayerW& L = H.L[l];
        // q, k, v projections fused into one [2304][768] weight
        std::vector<float> wqkv((size_t)2304 * 768);
        std::vector<float> bqkv(2304);
        const char* nm[3] = {"q_proj", "k_proj", "v_proj"};
        for (int m = 0; m < 3; ++m) {
            const Staged* w = find(p + "attention." + nm[m] + ".weight");
            const Staged* b = find(p + "attention." + nm[m] + ".bias");
            if (!w || !b || w->data.size() != (size_t)768 * 768 || b->data.size() != 768)
                return set_error(GSV_E_WEIGHT, "missing/bad weight " + p + "attention." + nm[m]);
            std::copy(w->data.begin(), w->data.end(), wqkv.begin() + (size_t)m * 768 * 768);
            for (int e = 0; e < 768; ++e) bqkv[m * 768 + e] = b->data[e];
        }
        L.wqkv = upload_w16(p + "attention.{q,k,v}_proj.weight", wqkv, &err);
        L.bqkv = (float*)dalloc(bqkv.size() * 4);
        hipMemcpy(L.bqkv, bqkv.data(), bqkv.size() * 4, hipMemcpyHostToDevice);
        L.wo = up_w16(p + "attention.out_proj.weight", &err);
        L.bo = up_f32(p + "attention.out_proj.bias", &err);
        L.ln1w = up_f32(p + "layer_norm.weight", &err);
        L.ln1b = up_f32(p + "layer_norm.bias", &err);
        L.w1 = up_w16(p + "feed_forward.intermediate_dense.weight", &err);
        L.b1 = up_f32(p + "feed_forward.intermediate_dense.bias", &err);
        L.w2 = up_w16(p + "feed_forward.output_dense.weight", &err);
        L.b2 = up_f32(p + "feed_forward.output_dense.bias", &err);
        L.ln2w = up_f32(p + "final_layer_norm.weight", &err);
        L.ln2b = up_f32(p + "final_layer_norm.bias", &err);
    }
    if (err) return err;
    H.ready = true;
    return 0;
}

float* gsv_engine::hubert_ws(size_t floats) {
    if (floats > hubert.ws_floats) {
        const size_t cap = grow_cap(floats, hubert.ws_floats);
        retire(hubert.ws);
        hubert.ws = nullptr;
        hubert.ws_floats = 0;
        reclaim();
        if (hipMalloc(&hubert.ws, cap * 4) != hipSuccess) return nullptr;
        hubert.ws_floats = cap;
    }
    return hubert.ws;
}

int gsv_engine::hubert_forward(const float* audio, int n, float* out, hipStream_t st) {
    const HubertWeights& H = hubert;
    int Ts[8];
    Ts[0] = n;
    for (int i = 0; i < 7; ++i) Ts[i + 1] = (Ts[i] - HB_KS[i]) / HB_SS[i] + 1;
    const int T0 = Ts[1], T = Ts[7];
    constexpr int NZ_GN = 64, NZ_POS = 8;
    // workspace: two conv ping-pong buffers [T0][512], then the encoder buffers
    const size_t conv_buf = (size_t)T0 * 512;
    const size_t enc = (size_t)T * (768 * 4 + 2304 + 3072) + (size_t)16 * T * 6144 + (size_t)NZ_POS * T * 768;
    float* ws = hubert_ws(2 * conv_buf + enc + (size_t)NZ_GN * 512 + 1024);
    if (!ws) return set_error(GSV_E_HIP, "hubert workspace");
    float *cA = ws, *cB = ws + conv_buf;
    float* e0 = ws + 2 * conv_buf;
    float *h = e0, *tmp = h + (size_t)T * 768, *att = tmp + (size_t)T * 768, *xproj = att + (size_t)T * 768;
    float* qkv = xproj + (size_t)T * 768;
    float* f = qkv + (size_t)T * 2304;
    float* im = f + (size_t)T * 3072;
    float* slabs = im + (size_t)16 * T * 6144;
    float* gpart = slabs + (size_t)NZ_POS * T * 768;
    float *gmean = gpart + (size_t)NZ_GN * 512, *grstd = gmean + 512;

    // ---- feature extractor
    hipLaunchKernelGGL(k_hb_conv0, dim3(T0), dim3(512), 0, st, audio, H.conv0_w, T0, cA);
    hipLaunchKernelGGL(k_hb_colsum, dim3(NZ_GN), dim3(512), 0, st, cA, T0, 512, (const float*)nullptr, 0, gpart);
    hipLaunchKernelGGL(k_hb_colfin, dim3(1), dim3(512), 0, st, gpart, NZ_GN, T0, 512, 0, gmean, grstd);
    hipLaunchKernelGGL(k_hb_colsum, dim3(NZ_GN), dim3(512), 0, st, cA, T0, 512, (const float*)gmean, 1, gpart);
    hipLaunchKernelGGL(k_hb_colfin, dim3(1), dim3(512), 0, st, gpart, NZ_GN, T0, 512, 1, gmean, grstd);
    hipLaunchKernelGGL(k_hb_gn_gelu, dim3(T0), dim3(512), 0, st, cA, 512, gmean, grstd, H.gn_w, H.gn_b);
    float *src = cA, *dst = cB;
    for (int i = 1; i < 7; ++i) {
        gemm_nt(gemm_w16(Ts[i + 1], 512, HB_KS[i] * 512, src, (long)HB_SS[i] * 512, H.conv_w[i], nullptr, dst, 512,
                        EPI_GELU),
                st);
        std::swap(src, dst);
    }
    // ---- feature projection: LayerNorm(512) -> Linear(512 -> 768)
    layernorm_rows_d(src, dst, T, 512, H.fp_ln_w, H.fp_ln_b, 1e-5f, st);
    gemm_nt(gemm_w16(T, 768, 512, dst, 512, H.fp_w, H.fp_b, xproj, 768, EPI_STORE), st);
    // ---- positional conv embedding: h = x + GELU(conv(x)), then LayerNorm(768)
    hipLaunchKernelGGL(k_hb_pos_im2col, dim3(T, 16), dim3(256), 0, st, xproj, T, im);
    for (int g = 0; g < 16; ++g) {
        GemmArgs a = gemm_w16(T, 48, 6144, im + (size_t)g * T * 6144, 6144, H.pos_w.at((size_t)g * 48 * 6144),
                             nullptr, slabs + 48 * g, 768, EPI_SLAB);
        a.ksplit = NZ_POS;
        a.slab_stride = (long)T * 768;
        gemm_nt(a, st);
    }
    hipMemcpyAsync(tmp, xproj, (size_t)T * 768 * 4, hipMemcpyDeviceToDevice, st);
    hipLaunchKernelGGL(k_hb_pos_reduce, dim3((T * 768 + 255) / 256), dim3(256), 0, st, slabs, NZ_POS,
                       (long)T * 768, H.pos_b, tmp, T * 768);
    layernorm_rows_d(tmp, h, T, 768, H.enc_ln_w, H.enc_ln_b, 1e-5f, st);
    // ---- 12 post-norm encoder layers
    // h = LN(h + A W^T + b).  A short clip's out-projection / FFN2 (768 outputs: 12 column
    // tiles x ceil(T / 64) row tiles, < 256 blocks) splits K into slabs that the LayerNorm
    // reduces in order (as RoBERTa's), so the GEMM covers the chip.
    const bool split = ((T + 63) / 64) * 12 < 256;
    auto resid_ln = [&](const float* A, int K, const W16& W, const float* bias, int z, const float* lw,
                        const float* lb) {
        if (split) {
            GemmArgs g = gemm_w16(T, 768, K, A, K, W, nullptr, slabs, 768, EPI_SLAB);
            g.ksplit = z;
            g.slab_stride = (long)T * 768;
            gemm_nt(g, st);
            layernorm_rows_d_slabs(slabs, z, (long)T * 768, bias, h, h, T, 768, lw, lb, 1e-5f, st);
        } else {
            gemm_nt(gemm_w16(T, 768, K, A, K, W, bias, tmp, 768, EPI_RESID, h, 768), st);
            layernorm_rows_d(tmp, h, T, 768, lw, lb, 1e-5f, st);
        }
    };
    for (int l = 0; l < 12; ++l) {
        const HubertLayerW& L = H.L[l];
        gemm_nt(gemm_w16(T, 2304, 768, h, 768, L.wqkv, L.bqkv, qkv, 2304, EPI_STORE), st);
        MhaArgs m{};
        m.q = qkv; m.q_ts = 2304; m.q_cs = 1;
        m.k = qkv + 768; m.k_ts = 2304; m.k_cs = 1;
        m.v = qkv + 1536; m.v_ts = 2304; m.v_cs = 1;
        m.out = att; m.o_ts = 768; m.o_cs = 1;
        m.nq = T; m.nk = T; m.heads = 12; m.dk = 64;
        m.postdiv = 0; m.scale = 8.f;   // q * 64^-0.5 (exact: a power of two)
        mha(m, st);
        resid_ln(att, 768, L.wo, L.bo, 4, L.ln1w, L.ln1b);
        gemm_nt(gemm_w16(T, 3072, 768, h, 768, L.w1, L.b1, f, 3072, EPI_GELU), st);
        resid_ln(f, 3072, L.w2, L.b2, NZ_POS, L.ln2w, L.ln2b);
    }
    hipLaunchKernelGGL(k_hb_transpose, dim3((T + 31) / 32, 24), dim3(256), 0, st, h, T, out);
    return hipGetLastError() == hipSuccess ? 0 : set_error(GSV_E_HIP, "hubert launch");
}

extern "C" int gsv_hubert_frames(int n_samples) { return hubert_frames(n_samples); }

extern "C" int gsv_hubert(gsv_engine* eng, const float* audio_16k, int n_samples, float* ssl_content, void* stream) {
    if (!eng) return set_error(GSV_E_ARG, "null engine");
    if (!audio_16k || !ssl_content) return set_error(GSV_E_ARG, "null arg");
    if (!eng->finalized || !eng->hubert.ready) return set_error(GSV_E_STATE, "CN-HuBERT weights not loaded");
    if (hubert_frames(n_samples) < 1) return set_error(GSV_E_ARG, "audio too short for CN-HuBERT");
    hipSetDevice(eng->device);
    StreamScope sc(eng, stream);
    return eng->hubert_forward(audio_16k, n_samples, ssl_content, sc.st());
}
