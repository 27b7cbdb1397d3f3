// VITS orchestration: restates vits_fp32.onnx (V2 / V2ProPlus) and
// prompt_encoder_fp32.onnx on the engine's kernels.  Called from
// gsv_vits_decode / gsv_prompt_encode (reference call sites:
// src/genie_tts/Core/Inference.py:47-60, src/genie_tts/Audio/ReferenceAudio.py:68-76).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>
#include <cstdlib>
#include <string>
#include <vector>

#include "engine_internal.h"

#include <thread>

using namespace gsv;

namespace {

std::vector<float> fold_wn(const Staged* v, const Staged* g) {
    // w = (v / ||v||_2 over dims 1..) * g  (ReduceL2 -> Div -> Mul in the graph)
    const long o = v->dims[0];
    const long per = (long)v->data.size() / o;
    std::vector<float> w(v->data.size());
    for (long i = 0; i < o; ++i) {
        double s = 0;
        for (long j = 0; j < per; ++j) s += (double)v->data[i * per + j] * v->data[i * per + j];
        const float nrm = (float)std::sqrt(s);
        const float gg = g->data[i];
        for (long j = 0; j < per; ++j) w[i * per + j] = (v->data[i * per + j] / nrm) * gg;
    }
    return w;
}

}  // namespace

// upload helpers ------------------------------------------------------------
static float* up_vec(gsv_engine* e, const std::vector<float>& v) {
    float* d = (float*)e->dalloc(v.size() * 4);
    if (d) hipMemcpy(d, v.data(), v.size() * 4, hipMemcpyHostToDevice);
    return d;
}

// fp16 copy [Cout][K][Cin] of a conv weight [Cout][Cin][K] for the f16-split path
// (vits_convh.hip), or nullptr when some value is not fp16-exact (then the conv
// stays on the f32 path).  scale[co] = g/||v|| (weight norm) or 1.
static bool upload_f16(gsv_engine* e, const std::vector<float>& v, int cout, int cin, int k,
                       const std::vector<float>& scale, Conv& c) {
    std::vector<__half> h((size_t)cout * cin * k);
    for (int co = 0; co < cout; ++co)
        for (int ci = 0; ci < cin; ++ci)
            for (int j = 0; j < k; ++j) {
                const float x = v[((size_t)co * cin + ci) * k + j];
                const __half hx = __float2half(x);
                if (__half2float(hx) != x) return false;
                h[((size_t)co * k + j) * cin + ci] = hx;
            }
    c.wh = (__half*)e->dalloc(h.size() * 2);
    c.wscale = (float*)e->dalloc((size_t)cout * 4);
    if (!c.wh || !c.wscale) return false;
    hipMemcpy(c.wh, h.data(), h.size() * 2, hipMemcpyHostToDevice);
    hipMemcpy(c.wscale, scale.data(), (size_t)cout * 4, hipMemcpyHostToDevice);
    return true;
}

static int load_conv(gsv_engine* e, const std::string& base, Conv& c, bool wn, bool bias = true,
                     bool f16 = false) {
    std::vector<float> w;
    const Staged* s = nullptr;
    if (wn) {
        const Staged* v = e->find(base + ".weight_v");
        const Staged* g = e->find(base + ".weight_g");
        if (!v || !g) return set_error(GSV_E_WEIGHT, "missing weight " + base + ".weight_v/g");
        w = fold_wn(v, g);
        s = v;
        if (f16) {
            // the same g/||v|| as fold_wn, applied to the f32 sums instead of the weights
            const long o = v->dims[0], per = (long)v->data.size() / o;
            std::vector<float> sc(o);
            for (long i = 0; i < o; ++i) {
                double q = 0;
                for (long j = 0; j < per; ++j) q += (double)v->data[i * per + j] * v->data[i * per + j];
                sc[i] = g->data[i] / (float)std::sqrt(q);
            }
            upload_f16(e, v->data, (int)v->dims[0], (int)v->dims[1], v->dims.size() > 2 ? (int)v->dims[2] : 1,
                       sc, c);
        }
    } else {
        s = e->find(base + ".weight");
        if (!s) return set_error(GSV_E_WEIGHT, "missing weight " + base + ".weight");
        w = s->data;
        if (f16)   // no weight norm: unit scale
            upload_f16(e, s->data, (int)s->dims[0], (int)s->dims[1], s->dims.size() > 2 ? (int)s->dims[2] : 1,
                       std::vector<float>((size_t)s->dims[0], 1.f), c);
    }
    c.cout = (int)s->dims[0];
    c.cin = (int)s->dims[1];
    c.k = s->dims.size() > 2 ? (int)s->dims[2] : 1;
    c.w = up_vec(e, w);
    if (bias) {
        const Staged* b = e->find(base + ".bias");
        if (!b) return set_error(GSV_E_WEIGHT, "missing weight " + base + ".bias");
        c.b = up_vec(e, b->data);
    }
    return 0;
}

// ConvTranspose1d(Cin, Cout, k, stride u, pad (k-u)/2), weight [Cin][Cout][k] (WN over dim 0)
// -> u polyphase convs of M = ceil(k/u) taps: W_r[co][ci][j] = w[ci][co][r + (M-1-j)*u]
static int load_convT(gsv_engine* e, const std::string& base, int u, Conv& c) {
    const Staged* v = e->find(base + ".weight_v");
    const Staged* g = e->find(base + ".weight_g");
    const Staged* b = e->find(base + ".bias");
    if (!v || !g || !b) return set_error(GSV_E_WEIGHT, "missing weight " + base);
    std::vector<float> w = fold_wn(v, g);
    const int cin = (int)v->dims[0], cout = (int)v->dims[1], k = (int)v->dims[2];
    const int M = (k + u - 1) / u;
    std::vector<float> pw((size_t)u * cout * cin * M, 0.f);
    for (int r = 0; r < u; ++r)
        for (int co = 0; co < cout; ++co)
            for (int ci = 0; ci < cin; ++ci)
                for (int j = 0; j < M; ++j) {
                    const int kk = r + (M - 1 - j) * u;
                    if (kk < k)
                        pw[(((size_t)r * cout + co) * cin + ci) * M + j] = w[((size_t)ci * cout + co) * k + kk];
                }
    c.w = up_vec(e, pw);
    c.b = up_vec(e, b->data);
    c.cout = cout;
    c.cin = cin;
    c.k = M;
    c.phases = u;
    // the split-fp16 path's copy: the unfolded weight_v values (fp16 in the Genie bins)
    // as [phase][Cout][M][Cin], the weight norm g/||v|| (over dim 0 = Cin) as a per-input-
    // channel scale; absent when some value is not fp16-exact (the f32 path stays)
    std::vector<__half> ph((size_t)u * cout * M * cin, __float2half(0.f));
    bool exact = true;
    for (int r = 0; r < u && exact; ++r)
        for (int co = 0; co < cout && exact; ++co)
            for (int j = 0; j < M && exact; ++j) {
                const int kk = r + (M - 1 - j) * u;
                if (kk >= k) continue;
                for (int ci = 0; ci < cin; ++ci) {
                    const float x = v->data[((size_t)ci * cout + co) * k + kk];
                    const __half hx = __float2half(x);
                    if (__half2float(hx) != x) { exact = false; break; }
                    ph[(((size_t)r * cout + co) * M + j) * cin + ci] = hx;
                }
            }
    if (exact) {
        std::vector<float> isc(cin), one(cout, 1.f);
        const long per = (long)cout * k;
        for (int ci = 0; ci < cin; ++ci) {
            double q = 0;
            for (long t = 0; t < per; ++t) q += (double)v->data[ci * per + t] * v->data[ci * per + t];
            isc[ci] = g->data[ci] / (float)std::sqrt(q);
        }
        c.wh = (__half*)e->dalloc(ph.size() * 2);
        c.wscale = up_vec(e, one);
        c.in_scale = up_vec(e, isc);
        if (!c.wh || !c.wscale || !c.in_scale) return set_error(GSV_E_HIP, "ConvTranspose fp16 upload failed");
        hipMemcpy(c.wh, ph.data(), ph.size() * 2, hipMemcpyHostToDevice);
    }
    return 0;
}

static int load_concat(gsv_engine* e, const std::vector<std::string>& bases, Conv& c) {
    std::vector<float> w, b;
    int cin = 0, cout = 0;
    for (const auto& n : bases) {
        const Staged* s = e->find(n + ".weight");
        const Staged* sb = e->find(n + ".bias");
        if (!s || !sb) return set_error(GSV_E_WEIGHT, "missing weight " + n);
        w.insert(w.end(), s->data.begin(), s->data.end());
        b.insert(b.end(), sb->data.begin(), sb->data.end());
        cout += (int)s->dims[0];
        cin = (int)s->dims[1];
    }
    c.w = up_vec(e, w);
    c.b = up_vec(e, b);
    c.cout = cout;
    c.cin = cin;
    c.k = 1;
    return 0;
}

static float* up_named(gsv_engine* e, const std::string& n, int* err) { return e->up_f32(n, err); }

static int load_attn_layers(gsv_engine* e, const std::string& pre, int n, std::vector<AttnLayer>& out) {
    out.resize(n);
    int err = 0;
    for (int i = 0; i < n; ++i) {
        const std::string a = pre + ".attn_layers." + std::to_string(i) + ".";
        AttnLayer& L = out[i];
        if (int r = load_concat(e, {a + "conv_q", a + "conv_k", a + "conv_v"}, L.qkv)) return r;
        if (int r = load_conv(e, a + "conv_o", L.o, false)) return r;
        if (int r = load_conv(e, pre + ".ffn_layers." + std::to_string(i) + ".conv_1", L.ffn1, false)) return r;
        if (int r = load_conv(e, pre + ".ffn_layers." + std::to_string(i) + ".conv_2", L.ffn2, false)) return r;
        for (const char* nm : {"emb_rel_k", "emb_rel_v"}) {   // k_mha's rel-pos terms: window 4 (<= MHA_MAXW)
            const auto* st = e->find(a + nm);
            if (st && st->data.size() != (size_t)(2 * 4 + 1) * 96)
                return set_error(GSV_E_WEIGHT, a + nm + ": expected [1, 9, 96] (relative window 4)");
        }
        L.ek = up_named(e, a + "emb_rel_k", &err);
        L.ev = up_named(e, a + "emb_rel_v", &err);
        L.g1 = up_named(e, pre + ".norm_layers_1." + std::to_string(i) + ".gamma", &err);
        L.b1 = up_named(e, pre + ".norm_layers_1." + std::to_string(i) + ".beta", &err);
        L.g2 = up_named(e, pre + ".norm_layers_2." + std::to_string(i) + ".gamma", &err);
        L.b2 = up_named(e, pre + ".norm_layers_2." + std::to_string(i) + ".beta", &err);
        if (err) return err;
    }
    return 0;
}

static int load_ref_enc(gsv_engine* e, const std::string& p, RefEnc& r) {
    int err = 0;
    r.fc0_w = e->up_f32(p + "spectral.0.fc.weight", &err);
    r.fc0_b = e->up_f32(p + "spectral.0.fc.bias", &err);
    r.fc3_w = e->up_f32(p + "spectral.3.fc.weight", &err);
    r.fc3_b = e->up_f32(p + "spectral.3.fc.bias", &err);
    if (err) return err;
    for (int i = 0; i < 2; ++i)
        if (int x = load_conv(e, p + "temporal." + std::to_string(i) + ".conv1.conv", r.temporal[i], false)) return x;
    Conv qkv;
    if (int x = load_concat(e, {p + "slf_attn.w_qs", p + "slf_attn.w_ks", p + "slf_attn.w_vs"}, qkv)) return x;
    r.wqkv = qkv.w;
    r.bqkv = qkv.b;
    r.fcw = e->up_f32(p + "slf_attn.fc.weight", &err);
    r.fcb = e->up_f32(p + "slf_attn.fc.bias", &err);
    r.out_w = e->up_f32(p + "fc.fc.weight", &err);
    r.out_b = e->up_f32(p + "fc.fc.bias", &err);
    if (err) return err;
    r.out_dim = (int)e->find(p + "fc.fc.weight")->dims[0];
    // windowed one-sided DFT basis for STFT(n_fft 2048), bins [0, 704), periodic Hann
    std::vector<float> basis((size_t)1408 * 2048);
    for (int b = 0; b < 704; ++b)
        for (int n = 0; n < 2048; ++n) {
            const double win = 0.5 - 0.5 * std::cos(2.0 * M_PI * n / 2048.0);
            const double ang = 2.0 * M_PI * (double)((long)b * n % 2048) / 2048.0;
            basis[(size_t)(2 * b) * 2048 + n] = (float)(win * std::cos(ang));
            basis[(size_t)(2 * b + 1) * 2048 + n] = (float)(-win * std::sin(ang));
        }
    r.dft = up_vec(e, basis);
    return r.dft ? 0 : set_error(GSV_E_HIP, "dft alloc");
}

int gsv_engine::finalize_vits() {
    VitsWeights& V = vits;
    const bool pp = version == GSV_V2PP;
    V.gin = pp ? 1024 : 512;
    V.upc = pp ? 768 : 512;
    const int rates[5] = {10, 8, 2, 2, 2};
    const int ks_v2[5] = {16, 16, 8, 2, 2}, ks_pp[5] = {20, 16, 8, 2, 2};
    for (int i = 0; i < 5; ++i) { V.up_rate[i] = rates[i]; V.up_k[i] = pp ? ks_pp[i] : ks_v2[i]; }
    int err = 0;
    const std::string P = "vq_model.enc_p.";
    V.codebook = up_f32("vq_model.quantizer.vq.layers.0._codebook.embed", &err);
    V.text_emb = up_f32(P + "text_embedding.weight", &err);
    if (err) return err;
    if (int r = load_conv(this, P + "ssl_proj", V.ssl_proj, false)) return r;
    if (int r = load_attn_layers(this, P + "encoder_ssl", 3, V.enc_ssl)) return r;
    if (int r = load_attn_layers(this, P + "encoder_text", 6, V.enc_text)) return r;
    if (int r = load_attn_layers(this, P + "encoder2", 3, V.enc2)) return r;
    const std::string M = P + "mrte.";
    if (int r = load_conv(this, M + "c_pre", V.c_pre, false)) return r;
    if (int r = load_conv(this, M + "text_pre", V.text_pre, false)) return r;
    if (int r = load_conv(this, M + "c_post", V.c_post, false)) return r;
    if (int r = load_conv(this, M + "cross_attention.conv_q", V.mrte_qkv_q, false)) return r;
    if (int r = load_concat(this, {M + "cross_attention.conv_k", M + "cross_attention.conv_v"}, V.mrte_kv)) return r;
    if (int r = load_conv(this, M + "cross_attention.conv_o", V.mrte_o, false)) return r;
    if (int r = load_conv(this, P + "proj", V.proj, false)) return r;
    for (int f = 0; f < 4; ++f) {
        const std::string F = "vq_model.flow.flows." + std::to_string(2 * f) + ".";
        auto& fl = V.flows[f];
        if (int r = load_conv(this, F + "pre", fl.pre, false)) return r;
        if (int r = load_conv(this, F + "post", fl.post, false)) return r;
        if (int r = load_conv(this, F + "enc.cond_layer", fl.cond, true)) return r;
        for (int l = 0; l < 4; ++l) {
            if (int r = load_conv(this, F + "enc.in_layers." + std::to_string(l), fl.in_l[l], true)) return r;
            if (int r = load_conv(this, F + "enc.res_skip_layers." + std::to_string(l), fl.rs[l], true)) return r;
        }
    }
    const std::string D = "vq_model.dec.";
    // (f32 path: on the split-fp16 kernel the flows' output z of the synthetic weights leaves
    // the fp16 range and every batch re-ran its generator on f32 -- r04k, 62.6 -> 77.8 ms)
    if (int r = load_conv(this, D + "conv_pre", V.conv_pre, false)) return r;
    if (int r = load_conv(this, D + "cond", V.cond, false)) return r;
    if (int r = load_conv(this, D + "conv_post", V.conv_post, false, false)) return r;
    for (int i = 0; i < 5; ++i)
        if (int r = load_convT(this, D + "ups." + std::to_string(i), V.up_rate[i], V.ups[i])) return r;
    for (int j = 0; j < 15; ++j)
        for (int c = 0; c < 2; ++c)
            for (int m = 0; m < 3; ++m) {
                const std::string n = D + "resblocks." + std::to_string(j) + (c == 0 ? ".convs1." : ".convs2.") +
                                      std::to_string(m);
                if (int r = load_conv(this, n, V.rb[j][c][m], true, true, true)) return r;
            }
    if (!pp)
        if (int r = load_ref_enc(this, "vq_model.ref_enc.", V.ref)) return r;
    V.ready = true;
    return hipDeviceSynchronize() == hipSuccess ? 0 : set_error(GSV_E_HIP, "finalize_vits");
}

int gsv_engine::finalize_prompt_encoder() {
    int err = 0;
    if (int r = load_ref_enc(this, "ref_enc.", penc.ref)) return r;
    penc.sv_w = up_f16("sv_emb.weight", &err);
    penc.sv_b = up_f32("sv_emb.bias", &err);
    penc.to512_w = up_f32("ge_to512.weight", &err);
    penc.to512_b = up_f32("ge_to512.bias", &err);
    penc.prelu = up_f32("prelu.weight", &err);
    if (err) return err;
    penc.ready = true;
    return 0;
}

// ---------------------------------------------------------------- helpers
// Split-K workspace of the engine whose VITS/prompt-encoder call is running on
// this thread (set by SplitkScope; conv1d splits only when it is set).
static thread_local float* tls_splitk = nullptr;
static thread_local long tls_splitk_cap = 0;
static thread_local int* tls_ovf = nullptr;   // set while the f16-split MRF path is enabled
static thread_local int tls_convh_tile = 0;    // the running engine's option "convh_tile"
static thread_local bool tls_convt_f16 = false;   // ... and "convt_f16" (the ConvTransposes on the split path)
static thread_local bool tls_mrf_fused = false;   // ... and "mrf_fused" (narrow stages' conv pairs as one kernel)
static thread_local int tls_convh_ws = 0;        // ... CUs of the pass's stream under "convh_ws" (0: off)
static thread_local int tls_convh_persist = 0;   // ... CUs of the pass's stream under "convh_persist" (0: off)
// The per-pass thread-local state of one vocoder pass (split-fp16 flag word, tile, ConvT path).
struct ConvhScope {
    ConvhScope(int* ovf, int tile, bool convt, bool fused, int persist_cus = 0, int ws_cus = 0) {
        tls_ovf = ovf; tls_convh_tile = tile; tls_convt_f16 = convt; tls_mrf_fused = fused;
        tls_convh_persist = persist_cus;
        tls_convh_ws = ws_cus;
    }
    ~ConvhScope() {
        tls_ovf = nullptr; tls_convh_tile = 0; tls_convt_f16 = false; tls_mrf_fused = false; tls_convh_persist = 0;
        tls_convh_ws = 0;
    }
};
struct SplitkScope {
    SplitkScope(float* p, long cap) { tls_splitk = p; tls_splitk_cap = cap; }
    ~SplitkScope() { tls_splitk = nullptr; tls_splitk_cap = 0; }
};
// A nested split-K scratch (the front's text branch on the side stream), the outer one restored.
struct SplitkSwap {
    float* p;
    long c;
    SplitkSwap(float* np, long nc) : p(tls_splitk), c(tls_splitk_cap) { tls_splitk = np; tls_splitk_cap = nc; }
    ~SplitkSwap() { tls_splitk = p; tls_splitk_cap = c; }
};

static ConvArgs cargs(const Conv& c, const float* x, int T, float* out, int mode = CV_STORE,
                      const int* seg = nullptr) {
    ConvArgs a{};
    a.seg = seg;
    a.part = tls_splitk; a.part_cap = tls_splitk_cap;
    a.x = x; a.x_cs = T; a.x_ts = 1; a.Cin = c.cin; a.Tin = T;
    a.w = c.w; a.Cout = c.cout; a.K = c.k; a.dil = 1; a.pad = (c.k - 1) / 2;
    a.bias = c.b;
    a.out = out; a.o_cs = T; a.o_ts = 1; a.n_t = T; a.o_tstride = 1; a.o_toff = 0; a.o_len = T;
    a.mode = mode; a.r_cs = T; a.r_ts = 1;
    a.phases = 1;
    a.tile_force = tls_convh_tile;
    a.persist = tls_convh_persist;
    a.ws = tls_convh_ws;
    if (tls_ovf && c.wh) { a.wh = c.wh; a.wscale = c.wscale; a.ovf = tls_ovf; }
    return a;
}

// seg / rows: a segmented batch (ConvArgs::seg of the T columns, MhaArgs::row_seg), else null
static void attn_encoder(gsv_engine* e, const std::vector<AttnLayer>& Ls, float* x, int T, float* qkv,
                         float* att, float* tmp, float* ffn, hipStream_t s, const int* seg = nullptr,
                         const int* rows = nullptr) {
    for (const AttnLayer& L : Ls) {
        conv1d(cargs(L.qkv, x, T, qkv, CV_STORE, seg), s);
        MhaArgs m{};
        m.q = qkv; m.q_ts = 1; m.q_cs = T;
        m.k = qkv + (size_t)192 * T; m.k_ts = 1; m.k_cs = T;
        m.v = qkv + (size_t)384 * T; m.v_ts = 1; m.v_cs = T;
        m.out = att; m.o_ts = 1; m.o_cs = T;
        m.nq = T; m.nk = T; m.heads = 2; m.dk = 96; m.postdiv = 0; m.scale = std::sqrt(96.0f);
        m.ek = L.ek; m.ev = L.ev; m.window = 4;
        m.row_seg = rows;
        mha(m, s);
        conv1d(cargs(L.o, att, T, tmp, CV_STORE, seg), s);
        ln_channels(x, tmp, x, 192, T, L.g1, L.b1, s, seg);
        conv1d(cargs(L.ffn1, x, T, ffn, CV_RELU, seg), s);
        conv1d(cargs(L.ffn2, ffn, T, tmp, CV_STORE, seg), s);
        ln_channels(x, tmp, x, 192, T, L.g2, L.b2, s, seg);
    }
}

// MelStyleEncoder on an STFT magnitude [F][704] -> ge [out_dim] (vits(v2)#79-271)
static void run_ref_enc(VitsWorkspace& W, const RefEnc& R, const float* audio, int n, float* ge,
                        hipStream_t s) {
    const int padded = n + 2 * 704;
    const int F = (padded - 2048) / 640 + 1;
    reflect_pad(audio, n, 704, W.pad, s);
    GemmArgs g{};
    g.M = F; g.N = 1408; g.K = 2048; g.A = W.pad; g.lda = 640;
    g.W = R.dft; g.ldw = 2048; g.w_f16 = 0; g.C = W.reim; g.ldc = 1408; g.mode = EPI_STORE;
    gemm_nt(g, s);
    stft_mag(W.reim, F, 704, W.spec, s);
    GemmArgs l0{};
    l0.M = F; l0.N = 128; l0.K = 704; l0.A = W.spec; l0.lda = 704;
    l0.W = R.fc0_w; l0.ldw = 704; l0.bias = R.fc0_b; l0.C = W.r0; l0.ldc = 128; l0.mode = EPI_MISH;
    gemm_nt(l0, s);
    GemmArgs l1 = l0;
    l1.K = 128; l1.A = W.r0; l1.lda = 128; l1.W = R.fc3_w; l1.ldw = 128; l1.bias = R.fc3_b; l1.C = W.r1;
    gemm_nt(l1, s);
    // temporal Conv1dGLU x2 on the [F][128] rows viewed channel-major via strides
    float* xin = W.r1;
    float* xout = W.r2;
    for (int i = 0; i < 2; ++i) {
        ConvArgs c = cargs(R.temporal[i], xin, F, W.r3);
        c.x_cs = 1; c.x_ts = 128;               // x(ci, t) = rows[t][ci]
        conv1d(c, s);                            // -> [256][F] channel-major
        glu_resid(W.r3, xin, xout, 128, F, 1, 128, s);
        float* t = xin; xin = xout; xout = (i == 0 ? W.r1 : t);
    }
    // xin: [F][128] rows.  Self-attention (2 heads x 64, temperature sqrt(128)) + residual
    GemmArgs q{};
    q.M = F; q.N = 384; q.K = 128; q.A = xin; q.lda = 128; q.W = R.wqkv; q.ldw = 128;
    q.bias = R.bqkv; q.C = W.rq; q.ldc = 384; q.mode = EPI_STORE;
    gemm_nt(q, s);
    MhaArgs m{};
    m.q = W.rq; m.q_ts = 384; m.q_cs = 1;
    m.k = W.rq + 128; m.k_ts = 384; m.k_cs = 1;
    m.v = W.rq + 256; m.v_ts = 384; m.v_cs = 1;
    m.out = W.ratt; m.o_ts = 128; m.o_cs = 1;
    m.nq = F; m.nk = F; m.heads = 2; m.dk = 64; m.postdiv = 1; m.scale = std::sqrt(128.0f);
    mha(m, s);
    GemmArgs fc{};
    fc.M = F; fc.N = 128; fc.K = 128; fc.A = W.ratt; fc.lda = 128; fc.W = R.fcw; fc.ldw = 128;
    fc.bias = R.fcb; fc.C = W.r3; fc.ldc = 128; fc.mode = EPI_RESID; fc.res = xin; fc.ldr = 128;
    gemm_nt(fc, s);
    GemmArgs o{};
    o.M = F; o.N = R.out_dim; o.K = 128; o.A = W.r3; o.lda = 128; o.W = R.out_w; o.ldw = 128;
    o.bias = R.out_b; o.C = W.r0; o.ldc = R.out_dim; o.mode = EPI_STORE;
    gemm_nt(o, s);
    time_mean(W.r0, F, R.out_dim, ge, s);
}

// with_gen = false: the front part's buffers only (the packed front of a segmented batch)
static int ensure_vits_ws(gsv_engine* e, VitsWorkspace& W, int T, int S, int n_audio, bool with_gen = true) {
    const VitsWeights& V = e->vits;
    const size_t gen = with_gen ? (size_t)V.upc * T * 20 : 0;   // max C*T over generator stages: upc/2^(i+1) * T*prod(u)
    const int F = n_audio > 0 ? (n_audio + 1408 - 2048) / 640 + 1 : 0;
    if ((size_t)T <= W.cap_t && S <= W.cap_text && gen <= W.cap_gen && F <= W.cap_spec) return 0;
    // 1.25x headroom on every dimension that grows; the old buffers are retired (freed by
    // reclaim once nothing queued reads them), so a ramp of utterance lengths does not accumulate
    const size_t t = grow_cap((size_t)T, W.cap_t);
    const int sT = (int)grow_cap(S, W.cap_text);
    const size_t g = gen > W.cap_gen ? grow_cap(gen, W.cap_gen) : W.cap_gen;
    const int f = (int)grow_cap(F, W.cap_spec);
    for (void* p : W.owned) e->retire(p);
    W.owned.clear();
    for (float*& p : W.gx) p = nullptr;
    W.cap_t = W.cap_gen = 0;
    W.cap_text = W.cap_spec = 0;
    e->reclaim();   // a no-op on a lane thread (vb_active): the next growth on the issuing thread frees them
    auto A = [&](size_t n) -> float* {
        void* p = nullptr;
        if (hipMalloc(&p, ((n * 4) + 255) & ~(size_t)255) != hipSuccess) return nullptr;
        W.owned.push_back(p);
        return (float*)p;
    };
    W.q = A(768 * t); W.y = A(192 * t); W.te = A(192 * (size_t)sT);
    W.qkv = A(576 * t); W.att = A(192 * t); W.a = A(512 * t); W.ffn = A(768 * t);
    W.tqkv = A(576 * (size_t)sT); W.tatt = A(192 * (size_t)sT); W.ta = A(192 * (size_t)sT);
    W.tffn = A(768 * (size_t)sT);
    W.ssl_enc = A(512 * t); W.text_enc = A(512 * (size_t)sT); W.mq = A(512 * t);
    W.mkv = A(1024 * (size_t)sT); W.mo = A(512 * t);
    W.stats = A(384 * t); W.z = A(192 * t); W.z2 = A(192 * t); W.fh = A(192 * t);
    W.fx = A(384 * t); W.fa = A(192 * t); W.fskip = A(192 * t); W.fm = A(96 * t);
    W.gcond = A(4 * 1536); W.dcond = A(1024); W.ge = A(1024); W.pe_ge = A(1024); W.sv = A(1024);
    if (g > 0) { W.g0 = A(g); W.g1 = A(g); W.g2 = A(g); W.g3 = A(g); W.g4 = A(g); }
    if (f > 0) {
        W.pad = A((size_t)f * 640 + 2048 + 1408);
        W.reim = A((size_t)f * 1408); W.spec = A((size_t)f * 704);
        W.r0 = A((size_t)f * 1024); W.r1 = A((size_t)f * 128); W.r2 = A((size_t)f * 128);
        W.r3 = A((size_t)f * 256); W.rq = A((size_t)f * 384); W.ratt = A((size_t)f * 128);
    }
    if (!W.splitk) {
        W.splitk_cap = 2L << 20;   // 8 MB: >= 384 tiles of 64 x 64 (never re-sized: engine lifetime)
        W.splitk = (float*)e->dalloc((size_t)W.splitk_cap * 4);
        W.splitk2 = (float*)e->dalloc((size_t)W.splitk_cap * 4);
    }
    if ((g > 0 && !W.g4) || !W.splitk || !W.splitk2 || !W.fm) return set_error(GSV_E_HIP, "VITS workspace allocation failed");
    W.cap_t = t; W.cap_text = sT; W.cap_gen = g; W.cap_spec = f;
    return 0;
}

// The MRF convs run on the f16-split MFMA path when enabled; an activation too
// large for fp16 sets the overflow flag, and the utterance is then decoded again
// on the f32 path (same kernels otherwise), so the output never depends on the
// fp16 range.  The flag check is a host sync on the caller's stream.
int gsv_engine::vits_decode(const int64_t* text_seq, int n_text, const int64_t* sem, int G,
                            const float* ref_audio, int n_audio, const float* ge_in,
                            const float* ge_adv_in, const float* eps, uint64_t noise_seed, float noise_scale,
                            float* audio, hipStream_t s) {
    if (use_convh && !vovf) {   // stream-ordered zeroing: no null-stream call beside running lanes / captures
        if (hipMalloc(&vovf, 64) != hipSuccess || hipHostMalloc((void**)&vovf_host, 64, hipHostMallocDefault) != hipSuccess)
            return set_error(GSV_E_HIP, "overflow flag alloc");
        hipMemsetAsync(vovf, 0, 64, s);
    }
    if (vpending || vqueued)   // the overlapped vocoder call shares the workspace: finish it first
        if (int r = vits_wait(nullptr)) return r;
    if (vb_active)
        if (int r = vits_batch_finish(nullptr)) return r;
    if (!use_convh) {
        if (int r = vits_decode_pass(vws, text_seq, n_text, sem, G, ref_audio, n_audio, ge_in, ge_adv_in, eps,
                                     noise_seed, noise_scale, audio, s, nullptr, timing))
            return r;
        return vits_read_ms();
    }
    if (int r = vits_decode_pass(vws, text_seq, n_text, sem, G, ref_audio, n_audio, ge_in, ge_adv_in, eps, noise_seed,
                                 noise_scale, audio, s, vovf, timing))
        return r;
    hipMemcpyAsync(vovf_host, vovf, 4, hipMemcpyDeviceToHost, s);
    if (hipStreamSynchronize(s) != hipSuccess) return set_error(GSV_E_HIP, "vits sync");
    if (*vovf_host == 0) return vits_read_ms();
    hipMemsetAsync(vovf, 0, 4, s);
    ++vits_f32_reruns;
    if (int r = vits_decode_pass(vws, text_seq, n_text, sem, G, ref_audio, n_audio, ge_in, ge_adv_in, eps, noise_seed,
                                 noise_scale, audio, s, nullptr, timing))
        return r;
    return vits_read_ms();
}

// Phase time of the last timed vocoder pass (events ev[4], ev[5] around it).
int gsv_engine::vits_read_ms() {
    if (!timing) return 0;
    if (hipEventSynchronize(ev[5]) != hipSuccess) return set_error(GSV_E_HIP, "vits timing");
    hipEventElapsedTime(&ms[3], ev[4], ev[5]);
    return 0;
}

// ---------------------------------------------------------------- overlapped vocoder
// Option "vocoder_cus" = K splits the CUs: the engine stream (T2S: encoder,
// prefill, the persistent decode with (n_cu - K) / 32 layer groups) is masked to
// n_cu - K of them and the vocoder stream to the other K, so the vocoder of
// utterance i runs beside the T2S of utterance i + 1 -- the persistent decode
// needs all its workgroups resident, and disjoint masks guarantee it.  (An
// unmasked engine stream with only the decode kernel on a masked one measured
// slower: its prefill ran at the speed of 64-192 CUs, the HW queues -- 4 per
// process -- being shared with the masked streams.)  The mask bits number the CUs
// XCD-interleaved (bit i: XCD i % 8; measured -- a mask balanced under the
// XCD-major reading left XCDs short and the decode timed out for K = 32, 96), so
// bits [0, K) give the vocoder K / 8 CUs of every XCD and every XCD keeps the
// (n_cu - K) / 8 CUs its share of the decode grid needs (workgroups go to the
// XCDs round robin).
// Lane streams re-created after a change of vocoder_cus / lane_priority (workspaces kept).
int gsv_engine::remake_lane_streams() {
    drop_sides();
    for (auto& L : vlanes) {
        hipStream_t ns = nullptr;
        if (make_lane_stream(&ns) != hipSuccess) return set_error(GSV_E_HIP, "lane stream");
        hipStreamDestroy(L.st);
        L.st = ns;
    }
    return 0;
}

// A vocoder lane's stream: on the vocoder CUs when option vocoder_cus splits the chip
// (bits [0, vocoder_cus), as the overlapped single vocoder), else on every CU.  Option
// lanes_all_cus keeps the lanes on every CU under the split: the T2S stream leaves the
// vocoder CUs free during the persistent decode, the lanes use the whole chip otherwise.
// CUs a stream of this engine runs on (its CU mask): the persistent conv grid's size.
int gsv_engine::stream_cus(hipStream_t st) const {
    if (vocoder_cus == 0) return n_cu;
    if (st == vstream) return vocoder_cus;
    if (st == stream) return decode_cus();
    for (const VitsLane& L : vlanes)
        if (st == L.st) return lanes_all_cus ? n_cu : vocoder_cus;
    return n_cu;
}

gsv_engine::SideStream* gsv_engine::side_of(hipStream_t s) {
    bool own = s && (s == stream || s == vstream);
    for (const VitsLane& L : vlanes) own = own || s == L.st;
    if (!own) return nullptr;   // a caller's stream: its lifetime is not the engine's to track
    std::lock_guard<std::mutex> lk(side_mu);
    for (auto& p : sides)
        if (p->main == s) return p.get();
    auto sd = std::make_unique<SideStream>();
    sd->main = s;
    const int words = (n_cu + 31) / 32;
    std::vector<uint32_t> mask(words, 0u);
    if (hipExtStreamGetCUMask(s, (uint32_t)words, mask.data()) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;   // mask unknown: a side stream might land on the decode's CUs
    }
    bool all = true;
    for (int i = 0; i < n_cu; ++i) all = all && ((mask[i / 32] >> (i % 32)) & 1u);
    // CU-masked streams (the vocoder's K CUs beside a decode) keep the front in order: on 64 CUs the
    // two branches only contend (r06w: 5.66 vs 5.16 ms per VITS beside the decode)
    if (!all) return nullptr;
    bool ok = true;
    for (int k = 0; k < 2; ++k)
        ok = ok && hipStreamCreateWithFlags(&sd->st[k], hipStreamNonBlocking) == hipSuccess &&
             hipEventCreateWithFlags(&sd->join[k], hipEventDisableTiming) == hipSuccess;
    ok = ok && hipEventCreateWithFlags(&sd->fork, hipEventDisableTiming) == hipSuccess;
    if (!ok) {
        for (int k = 0; k < 2; ++k) {
            if (sd->st[k]) hipStreamDestroy(sd->st[k]);
            if (sd->join[k]) hipEventDestroy(sd->join[k]);
        }
        if (sd->fork) hipEventDestroy(sd->fork);
        (void)hipGetLastError();
        return nullptr;   // the front / generator then run their branches in order on s
    }
    sides.push_back(std::move(sd));
    return sides.back().get();
}

// Before one of the engine's streams is destroyed or re-made: the side streams go with them.
void gsv_engine::drop_sides() {
    std::lock_guard<std::mutex> lk(side_mu);
    for (auto& p : sides) {
        for (int k = 0; k < 2; ++k) {
            hipStreamSynchronize(p->st[k]);
            hipStreamDestroy(p->st[k]);
            hipEventDestroy(p->join[k]);
        }
        hipEventDestroy(p->fork);
    }
    sides.clear();
}

hipError_t gsv_engine::make_lane_stream(hipStream_t* st) {
    if (vocoder_cus == 0 || lanes_all_cus) return hipStreamCreateWithPriority(st, hipStreamNonBlocking, lane_priority);
    const int words = (n_cu + 31) / 32;
    std::vector<uint32_t> mv(words, 0u);
    for (int i = 0; i < vocoder_cus; ++i) mv[i / 32] |= 1u << (i % 32);
    return hipExtStreamCreateWithCUMask(st, (uint32_t)words, mv.data());
}

int gsv_engine::set_vocoder_cus(int K) {
    if (K != 0 && (K % 8 != 0 || K < 8 || n_cu - K < 3 * persist1_grid(1) || n_cu % 32 != 0))
        return set_error(GSV_E_ARG, "vocoder_cus: a multiple of 8 leaving >= 96 CUs for the decode");
    const int D = dec_cus_opt > 0 ? dec_cus_opt : n_cu - K - dec_cu_off;
    if (K != 0 && (dec_cu_off % 8 != 0 || D % 32 != 0 || D < 3 * persist1_grid(1) || K + dec_cu_off + D > n_cu))
        return set_error(GSV_E_ARG, "decode_cus / decode_cu_offset: a multiple of 32 (>= 96) CUs at a multiple "
                                    "of 8 past the vocoder CUs, within the chip");
    if (gq_n) return set_error(GSV_E_STATE, "vocoder_cus: finish the started generates first");
    if (int r = vits_wait(nullptr)) return r;
    if (int r = vits_batch_finish(nullptr)) return r;
    if (int r = pf_drop()) return r;   // a launched prefetch runs on the vocoder stream
    if (sync_own_streams() != hipSuccess) return set_error(GSV_E_HIP, "vocoder_cus sync");
    hipStream_t ns = nullptr, nv = nullptr;
    if (K == 0) {
        if (hipStreamCreateWithFlags(&ns, hipStreamNonBlocking) != hipSuccess) return set_error(GSV_E_HIP, "stream");
    } else {
        const int words = (n_cu + 31) / 32;
        std::vector<uint32_t> mt(words, 0u), mv(words, 0u);
        for (int i = 0; i < n_cu; ++i) {
            if (i < K) mv[i / 32] |= 1u << (i % 32);
            else if (i >= K + dec_cu_off && i < K + dec_cu_off + D) mt[i / 32] |= 1u << (i % 32);
        }
        if (hipExtStreamCreateWithCUMask(&ns, (uint32_t)words, mt.data()) != hipSuccess ||
            hipExtStreamCreateWithCUMask(&nv, (uint32_t)words, mv.data()) != hipSuccess)
            return set_error(GSV_E_HIP, "CU-masked stream");
        for (hipEvent_t* e : {&vev_in, &vev_done})
            if (!*e && hipEventCreateWithFlags(e, hipEventDisableTiming) != hipSuccess)
                return set_error(GSV_E_HIP, "vocoder events");
    }
    drop_sides();
    if (own_stream && stream) hipStreamDestroy(stream);
    if (vstream) hipStreamDestroy(vstream);
    stream = ns;
    own_stream = true;
    vstream = nv;
    vocoder_cus = K;
    return remake_lane_streams();
}

// The call is queued, not launched: its ~400 launches are issued by the next
// T2S generate right after the persistent decode kernel (vits_launch_queued), so
// the host enqueues them while the GPU decodes instead of delaying that T2S.
int gsv_engine::vits_async(const gsv_vits_item& u, float noise_scale, hipStream_t caller) {
    if (!vstream) return set_error(GSV_E_STATE, "overlapped vocoder: set option vocoder_cus first");
    if (int r = vits_wait(nullptr)) return r;
    if (vb_active)
        if (int r = vits_batch_finish(nullptr)) return r;
    if (use_convh && !vovf) {
        if (hipMalloc(&vovf, 64) != hipSuccess || hipHostMalloc((void**)&vovf_host, 64, hipHostMallocDefault) != hipSuccess)
            return set_error(GSV_E_HIP, "overflow flag alloc");
        hipMemsetAsync(vovf, 0, 64, caller);   // ordered before the call by vev_in
    }
    hipEventRecord(vev_in, caller);   // the inputs are ready in the caller's stream order here
    vcall = u;
    vcall_scale = noise_scale;
    vqueued = true;
    return 0;
}

// s: the vocoder stream (beside a decode), or the engine stream when no T2S work is
// queued behind (the last sentence of a stream: its n_cu - K CUs are idle then).
int gsv_engine::vits_launch_queued(hipStream_t s) {
    if (!vqueued) return 0;
    vqueued = false;
    if (!s) s = vstream;
    const gsv_vits_item& u = vcall;
    hipStreamWaitEvent(s, vev_in, 0);
    if (int r = vits_decode_pass(vws, u.text_seq, u.n_text, u.sem, u.n_sem, u.ref_audio, u.n_audio, u.ge, u.ge_adv,
                                 u.noise_mode == 1 ? u.eps : nullptr, u.noise_mode == 2 ? u.noise_seed : 0,
                                 vcall_scale, u.audio, s, use_convh ? vovf : nullptr, timing))
        return r;
    if (use_convh) hipMemcpyAsync(vovf_host, vovf, 4, hipMemcpyDeviceToHost, s);
    hipEventRecord(vev_done, s);
    vpending = true;
    vlast = s;
    return 0;
}

int gsv_engine::vits_wait(hipStream_t caller) {
    // still queued (no decode launched since): nothing runs on the engine stream unless
    // a started generate does, so the call takes the T2S CUs
    if (int r = vits_launch_queued(gq_n == 0 ? stream : vstream)) return r;
    if (!vpending) return 0;
    vpending = false;
    if (hipEventSynchronize(vev_done) != hipSuccess) return set_error(GSV_E_HIP, "overlapped vocoder");
    if (use_convh && *vovf_host) {   // fp16-range overflow: the same utterance again on the f32 path
        const gsv_vits_item& u = vcall;
        hipMemsetAsync(vovf, 0, 4, vlast);
        ++vits_f32_reruns;
        if (int r = vits_decode_pass(vws, u.text_seq, u.n_text, u.sem, u.n_sem, u.ref_audio, u.n_audio, u.ge,
                                     u.ge_adv, u.noise_mode == 1 ? u.eps : nullptr,
                                     u.noise_mode == 2 ? u.noise_seed : 0, vcall_scale, u.audio, vlast, nullptr,
                                     timing))
            return r;
        hipEventRecord(vev_done, vlast);
        if (hipEventSynchronize(vev_done) != hipSuccess) return set_error(GSV_E_HIP, "overlapped vocoder re-run");
    }
    if (int r = vits_read_ms()) return r;
    if (caller) hipStreamWaitEvent(caller, vev_done, 0);
    return 0;
}

// The HiFi-GAN generator (vits_fp32.onnx dec.*) on z [192][T]: conv_pre + the
// conditioning vector dcond, 5 x (ConvTranspose1d up + 3 MRF resblocks), conv_post + tanh
// -> audio [T * prod(up_rate)].  gb: five buffers of >= upc * T * 20 floats.  seg
// (segmented batch, else null): the time tables of the 6 rates (T, T u0, ...), and
// dcond holds one vector per utterance (stride dcond_sstride); gaps stay zero.
static void vits_generator(const VitsWeights& V, float* const (&gb)[5], const float* z, int T, const float* dcond,
                           long dcond_sstride, const int* const* seg, float* audio, hipStream_t s,
                           gsv_engine::SideStream* sd = nullptr, float* const* gx = nullptr) {
    float* x = gb[0];
    // x = conv_pre(z) + cond(ge)   (dec#: Conv -> Add(cond))
    ConvArgs c2 = cargs(V.conv_pre, z, T, x, CV_VEC);
    c2.vec = dcond;
    if (seg) { c2.seg = seg[0]; c2.vec_sstride = dcond_sstride; }
    conv1d(c2, s);
    int C = V.upc, Tc = T;
    float* const* bufs = gb + 1;
    for (int i = 0; i < 5; ++i) {
        const Conv& up = V.ups[i];
        const int u = V.up_rate[i], kfull = V.up_k[i], padT = (kfull - u) / 2;
        const int Tn = (Tc - 1) * u - 2 * padT + kfull;
        const int* sg = seg ? seg[i + 1] : nullptr;
        float* yb = bufs[0];
        ConvArgs ct{};
        ct.x = x; ct.x_cs = Tc; ct.x_ts = 1; ct.Cin = C; ct.Tin = Tc;
        ct.w = up.w; ct.Cout = up.cout; ct.K = up.k; ct.dil = 1; ct.pad = up.k - 1;
        ct.bias = up.b; ct.out = yb; ct.o_cs = Tn; ct.o_ts = 1;
        ct.n_t = (Tn + padT + u - 1) / u; ct.o_tstride = u; ct.o_toff = -padT; ct.o_len = Tn;
        ct.in_act = 1; ct.in_slope = 0.1f; ct.mode = CV_STORE;
        ct.phases = u; ct.w_phase_stride = (long)up.cout * up.cin * up.k;
        ct.seg = sg;
        ct.tile_force = tls_convh_tile;
        ct.persist = tls_convh_persist;
        if (tls_ovf && up.wh && tls_convt_f16) {   // the split-fp16 path (polyphase weights, input-channel weight norm)
            ct.wh = up.wh; ct.wscale = up.wscale; ct.ovf = tls_ovf; ct.in_scale = up.in_scale;
            ct.wh_phase_stride = (long)up.cout * up.k * up.cin;
        }
        conv1d(ct, s);
        C = up.cout;
        Tc = Tn;
        float* rbuf = bufs[1];
        float* xt = bufs[2];
        float* accb = bufs[3];
        // the narrow stages (C <= 32, byte-bound): each conv1 + conv2 pair as one kernel with
        // xt in LDS (vits_mrf.hip); its output ping-pongs between rbuf and xt (no in-place update:
        // neighbouring blocks read the input's halo)
        // One utterance (sd, gx): the stage's three resblocks are independent given yb, so they run
        // on three streams -- resblock j's steps on its own rbuf / xt, its last step a plain
        // residual into out_j -- and x = ((out_0 + out_1) + out_2) / 3 afterwards: the arithmetic
        // and order of the ACC_FIRST / ACC_ADD / ACC_MEAN chain below, so the audio is identical.
        // Only on the split-fp16 path (no split-K scratch shared between the streams).
        bool par = sd && gx && tls_ovf;
        for (int j = 0; j < 3 && par; ++j)
            for (int mi = 0; mi < 3; ++mi)
                par = par && V.rb[i * 3 + j][0][mi].wh && V.rb[i * 3 + j][1][mi].wh;
        if (par) {
            hipEventRecord(sd->fork, s);
            for (int k = 0; k < 2; ++k) hipStreamWaitEvent(sd->st[k], sd->fork, 0);
            float* outs[3] = {accb, gx[2], gx[5]};
            for (int j = 0; j < 3; ++j) {
                const hipStream_t js = j == 0 ? s : sd->st[j - 1];
                float* jr = j == 0 ? rbuf : gx[3 * (j - 1)];
                float* jx = j == 0 ? xt : gx[3 * (j - 1) + 1];
                const int kk = V.rb_k[j];
                const float* rcur = yb;
                const bool fj = tls_mrf_fused && C <= 32;
                for (int mi = 0; mi < 3; ++mi) {
                    const Conv& c1 = V.rb[i * 3 + j][0][mi];
                    const Conv& c2w = V.rb[i * 3 + j][1][mi];
                    // fused: ping-pong yb -> jr -> jx -> out (the pair reads its input's halo); unfused:
                    // conv1 into jx, conv2's residual update in place in jr, the last into out
                    float* dst = mi == 2 ? outs[j] : (fj ? (mi == 0 ? jr : jx) : jr);
                    float* scratch = !fj ? jx : (mi == 0 ? jx : mi == 1 ? outs[j] : jr);
                    bool done = false;
                    if (fj) {
                        MrfPairArgs m{};
                        m.r = rcur; m.T = Tc; m.C = C; m.K = kk; m.dil = V.rb_d[mi];
                        m.w1 = c1.wh; m.s1 = c1.wscale; m.b1 = c1.b;
                        m.w2 = c2w.wh; m.s2 = c2w.wscale; m.ovf = tls_ovf;
                        m.e = cargs(c2w, rcur, Tc, dst);
                        m.e.res = rcur;
                        m.e.seg = sg;
                        m.e.mode = CV_RESID;
                        done = mrf_pair(m, js);
                    }
                    if (!done) {
                        ConvArgs a1 = cargs(c1, rcur, Tc, scratch);
                        a1.dil = V.rb_d[mi]; a1.pad = (kk * V.rb_d[mi] - V.rb_d[mi]) / 2; a1.in_act = 1; a1.in_slope = 0.1f;
                        a1.seg = sg;
                        conv1d(a1, js);
                        ConvArgs a2 = cargs(c2w, scratch, Tc, dst);
                        a2.in_act = 1; a2.in_slope = 0.1f; a2.res = rcur; a2.mode = CV_RESID;
                        a2.seg = sg;
                        conv1d(a2, js);
                    }
                    rcur = dst;
                }
                if (j > 0) hipEventRecord(sd->join[j - 1], js);
            }
            for (int k = 0; k < 2; ++k) hipStreamWaitEvent(s, sd->join[k], 0);
            mean3(outs[0], outs[1], outs[2], x, (long)C * Tc, 3.0f, s);
            continue;
        }
        const bool fuse = tls_ovf && tls_mrf_fused && C <= 32;
        for (int j = 0; j < 3 && fuse; ++j) {
            const int kk = V.rb_k[j];
            const float* rcur = yb;
            for (int mi = 0; mi < 3; ++mi) {
                const Conv& c1 = V.rb[i * 3 + j][0][mi];
                const Conv& c2w = V.rb[i * 3 + j][1][mi];
                MrfPairArgs m{};
                m.r = rcur; m.T = Tc; m.C = C; m.K = kk; m.dil = V.rb_d[mi];
                m.w1 = c1.wh; m.s1 = c1.wscale; m.b1 = c1.b;
                m.w2 = c2w.wh; m.s2 = c2w.wscale; m.ovf = tls_ovf;
                m.e = cargs(c2w, rcur, Tc, mi == 0 ? rbuf : xt);
                m.e.res = rcur;
                m.e.seg = sg;
                if (mi < 2) {
                    m.e.mode = CV_RESID;
                } else if (j == 0) {
                    m.e.mode = CV_ACC_FIRST; m.e.acc = accb;
                } else if (j == 1) {
                    m.e.mode = CV_ACC_ADD; m.e.acc = accb;
                } else {
                    m.e.mode = CV_ACC_MEAN; m.e.acc = accb; m.e.div = 3.0f; m.e.out = x;
                }
                if (!mrf_pair(m, s)) {   // not covered (weights off the fp16 path): the two convs, xt in
                    // a buffer free at this point (x is rewritten only by the last MEAN step)
                    float* scratch = mi == 2 ? rbuf : x;
                    ConvArgs a1 = cargs(c1, rcur, Tc, scratch);
                    a1.dil = V.rb_d[mi]; a1.pad = (kk * V.rb_d[mi] - V.rb_d[mi]) / 2; a1.in_act = 1; a1.in_slope = 0.1f;
                    a1.seg = sg;
                    conv1d(a1, s);
                    ConvArgs a2 = m.e;
                    a2.x = scratch; a2.in_act = 1; a2.in_slope = 0.1f;
                    conv1d(a2, s);
                }
                rcur = mi == 0 ? rbuf : xt;
            }
        }
        for (int j = 0; j < 3 && !fuse; ++j) {
            const int kk = V.rb_k[j];
            const float* rcur = yb;
            for (int mi = 0; mi < 3; ++mi) {
                const int d = V.rb_d[mi];
                const Conv& c1 = V.rb[i * 3 + j][0][mi];
                const Conv& c2w = V.rb[i * 3 + j][1][mi];
                ConvArgs a1 = cargs(c1, rcur, Tc, xt);
                a1.dil = d; a1.pad = (kk * d - d) / 2; a1.in_act = 1; a1.in_slope = 0.1f;
                a1.seg = sg;
                conv1d(a1, s);
                ConvArgs a2 = cargs(c2w, xt, Tc, rbuf);
                a2.in_act = 1; a2.in_slope = 0.1f; a2.res = rcur;
                a2.seg = sg;
                if (mi < 2) {
                    a2.mode = CV_RESID;
                } else if (j == 0) {
                    a2.mode = CV_ACC_FIRST; a2.acc = accb;
                } else if (j == 1) {
                    a2.mode = CV_ACC_ADD; a2.acc = accb;
                } else {
                    a2.mode = CV_ACC_MEAN; a2.acc = accb; a2.div = 3.0f; a2.out = x;
                }
                conv1d(a2, s);
                rcur = rbuf;
            }
        }
    }
    ConvArgs cp = cargs(V.conv_post, x, Tc, audio, CV_TANH);
    cp.in_act = 1; cp.in_slope = 0.01f;
    cp.seg = seg ? seg[5] : nullptr;
    conv1d(cp, s);
}

// One utterance on stream s with workspace W.  ovf != NULL: the MRF convs run on
// the f16-split path and OR 1 into *ovf on an fp16-range overflow.  noise: eps
// (device [192, 2G]) if given, else Philox N(0,1) keyed by noise_seed when it is
// non-zero, else zeros.  timed: phase events (ms[3]) around the pass.
int gsv_engine::vits_decode_pass(VitsWorkspace& W, const int64_t* text_seq, int n_text, const int64_t* sem, int G,
                                 const float* ref_audio, int n_audio, const float* ge_in,
                                 const float* ge_adv_in, const float* eps, uint64_t noise_seed, float noise_scale,
                                 float* audio, hipStream_t s, int* ovf, bool timed) {
    if (!vits.ready) return set_error(GSV_E_STATE, "VITS weights not loaded");
    if (G <= 0 || n_text <= 0) return set_error(GSV_E_ARG, "empty VITS input");
    if (2 * G > MHA_MAXK_HOST || n_text > MHA_MAXK_HOST) return set_error(GSV_E_CAPACITY, "sequence too long");
    if (int r = ensure_vits_ws(this, W, 2 * G, n_text, version == GSV_V2PP ? 0 : n_audio)) return r;
    SplitkScope sk(W.splitk, W.splitk_cap);
    ConvhScope cs(ovf, convh_tile, convt_f16, mrf_fused, convh_persist ? stream_cus(s) : 0,
                  convh_ws == 1 ? stream_cus(s) : 0);
    (void)hipGetLastError();   // the launches below are checked as one batch at the end
    if (timed) hipEventRecord(ev[4], s);
    if (int r = vits_front(W, text_seq, n_text, sem, G, ref_audio, n_audio, ge_in, ge_adv_in, eps, noise_seed,
                           noise_scale, W.dcond, s))
        return r;
    float* const gb[5] = {W.g0, W.g1, W.g2, W.g3, W.g4};
    // the three resblocks of a stage on three streams (vits_fork, an unmasked engine stream)
    SideStream* sd = vits_fork && ovf && s == stream ? side_of(s) : nullptr;
    if (sd && !W.gx[0]) {
        for (float*& p : W.gx) {
            void* q = nullptr;
            if (hipMalloc(&q, ((W.cap_gen * 4) + 255) & ~(size_t)255) != hipSuccess) {
                sd = nullptr;
                break;
            }
            W.owned.push_back(q);   // retired with the workspace's other buffers when it grows
            p = (float*)q;
        }
        if (!sd) {
            (void)hipGetLastError();
            for (float*& p : W.gx) p = nullptr;   // (allocated ones stay in W.owned)
        }
    }
    vits_generator(vits, gb, W.z, 2 * G, W.dcond, 0, nullptr, audio, s, sd, sd ? W.gx : nullptr);
    if (timed) hipEventRecord(ev[5], s);   // read by vits_read_ms once the pass is known to be final
    return hipGetLastError() == hipSuccess ? 0 : set_error(GSV_E_HIP, "vits launch");
}

// Everything of vits_fp32.onnx before the generator, for one utterance: conditioning,
// enc_p (codebook decode, ssl_proj, encoder_ssl, text encoder), MRTE, z_p, the reverse
// flow -> z in W.z [192][2G]; and the generator's conditioning vector dcond_out [upc] =
// dec.cond(ge).  The caller set the split-K scope.
// fs (a segmented batch): every utterance of it at once, laid out back to back along the
// frame axis (fs->Tt columns) and the text axis (fs->St), zero gaps (the convs' seg
// epilogue, seg-aware LayerNorm / noise / embedding kernels), attention within each
// utterance (row_seg); ge / ge_m per utterance (vec_sstride); z [192][Tt] in W.z and
// dcond_out [n][upc].  The per-utterance arguments are unused then.
int gsv_engine::vits_front(VitsWorkspace& W, const int64_t* text_seq, int n_text, const int64_t* sem, int G,
                           const float* ref_audio, int n_audio, const float* ge_in, const float* ge_adv_in,
                           const float* eps, uint64_t noise_seed, float noise_scale, float* dcond_out,
                           hipStream_t s, const FrontSeg* fs) {
    const VitsWeights& V = vits;
    if (!V.ready) return set_error(GSV_E_STATE, "VITS weights not loaded");
    const bool pp = version == GSV_V2PP;
    const int* sT = fs ? fs->segT : nullptr;
    const int* sS = fs ? fs->segS : nullptr;
    int T, S;
    if (fs) {
        T = fs->Tt;
        S = fs->St;
        if (int r = ensure_vits_ws(this, W, T, S, 0, false)) return r;
    } else {
        if (G <= 0 || n_text <= 0) return set_error(GSV_E_ARG, "empty VITS input");
        if (pp ? (!ge_in || !ge_adv_in) : (!ref_audio && !ge_in))
            return set_error(GSV_E_ARG, "missing conditioning input");
        T = 2 * G;
        S = n_text;
        if (T > MHA_MAXK_HOST || S > MHA_MAXK_HOST) return set_error(GSV_E_CAPACITY, "sequence too long");
        if (int r = ensure_vits_ws(this, W, T, S, pp ? 0 : n_audio)) return r;
    }
    // ---- conditioning: ge (flow cond / dec.cond) and MRTE vector
    const float* ge;
    const float* ge_m;
    if (fs) {   // one vector per utterance
        ge = fs->ge;
        ge_m = fs->gem;
    } else if (!pp && ge_in) {   // V2 with the reference's ge from gsv_ref_encode (once per reference)
        ge = ge_in;
        ge_m = ge_in;
    } else if (!pp) {
        run_ref_enc(W, V.ref, ref_audio, n_audio, W.ge, s);
        ge = W.ge;
        ge_m = W.ge;
    } else {
        ge = ge_in;
        ge_m = ge_adv_in;
    }
    // ---- the text branch (text embedding, encoder_text, MRTE's text_pre and k/v projection) needs
    // only the phones: it runs on the side stream beside the SSL branch below (both are chains of
    // small latency-bound kernels; r06w) and joins before MRTE's attention.  Its buffers (te, t*,
    // text_enc, mkv) and split-K scratch (splitk2) are its own; same kernels, same results.
    // only a single call on the engine stream (the single-request path): beside the next batch's T2S
    // the batched fronts' second stream only adds contention (r06fin: mixed100 320 vs 325 utt/s)
    SideStream* sd = vits_fork && !fs && s == stream ? side_of(s) : nullptr;
    const hipStream_t ts = sd ? sd->st[0] : s;
    if (sd) {
        hipEventRecord(sd->fork, s);
        hipStreamWaitEvent(ts, sd->fork, 0);
    }
    {
        SplitkSwap sk2(W.splitk2, W.splitk_cap);
        if (fs) embed_channels_seg(fs->texts, sS, fs->offS, S, V.text_emb, 192, W.te, ts);
        else embed_channels(text_seq, S, V.text_emb, 192, W.te, ts);
        attn_encoder(this, V.enc_text, W.te, S, W.tqkv, W.tatt, W.ta, W.tffn, ts, sS, fs ? fs->rowS : nullptr);
        conv1d(cargs(V.text_pre, W.te, S, W.text_enc, CV_STORE, sS), ts);
        conv1d(cargs(V.mrte_kv, W.text_enc, S, W.mkv, CV_STORE, sS), ts);
    }
    if (sd) hipEventRecord(sd->join[0], ts);
    // ---- enc_p: codebook decode x2, ssl_proj, encoder_ssl
    if (fs) codebook_upsample2_seg(fs->sems, sT, fs->offT, T, V.codebook, W.q, s);
    else codebook_upsample2(sem, G, V.codebook, W.q, s);
    conv1d(cargs(V.ssl_proj, W.q, T, W.y, CV_STORE, sT), s);
    attn_encoder(this, V.enc_ssl, W.y, T, W.qkv, W.att, W.a, W.ffn, s, sT, fs ? fs->rowT : nullptr);
    // ---- MRTE
    conv1d(cargs(V.c_pre, W.y, T, W.ssl_enc, CV_STORE, sT), s);
    conv1d(cargs(V.mrte_qkv_q, W.ssl_enc, T, W.mq, CV_STORE, sT), s);
    if (sd) hipStreamWaitEvent(s, sd->join[0], 0);
    MhaArgs m{};
    m.q = W.mq; m.q_ts = 1; m.q_cs = T;
    m.k = W.mkv; m.k_ts = 1; m.k_cs = S;
    m.v = W.mkv + (size_t)512 * S; m.v_ts = 1; m.v_cs = S;
    m.out = W.mo; m.o_ts = 1; m.o_cs = T;
    m.nq = T; m.nk = S; m.heads = 4; m.dk = 128; m.postdiv = 0; m.scale = std::sqrt(128.0f);
    m.row_seg = fs ? fs->rowX : nullptr;   // a frame attends to its own utterance's text
    mha(m, s);
    ConvArgs co = cargs(V.mrte_o, W.mo, T, W.a, CV_RESID_VEC, sT);
    co.res = W.ssl_enc; co.vec = ge_m;
    if (fs) co.vec_sstride = V.mrte_o.cout;
    conv1d(co, s);
    conv1d(cargs(V.c_post, W.a, T, W.y, CV_STORE, sT), s);
    attn_encoder(this, V.enc2, W.y, T, W.qkv, W.att, W.a, W.ffn, s, sT, fs ? fs->rowT : nullptr);
    conv1d(cargs(V.proj, W.y, T, W.stats, CV_STORE, sT), s);
    // ---- z_p = m_p + eps*exp(logs_p)*noise_scale
    if (fs)
        noise_zp_philox_seg(W.stats, W.stats + (size_t)192 * T, fs->seeds, sT, fs->offT, fs->lenT, noise_scale, W.z,
                            192, T, s);
    else if (!eps && noise_seed != 0)
        noise_zp_philox(W.stats, W.stats + (size_t)192 * T, noise_seed, noise_scale, W.z, 192 * T, s);
    else
        noise_zp(W.stats, W.stats + (size_t)192 * T, eps, noise_scale, W.z, 192 * T, s);
    // conditioning convs of the whole batch: the n vectors [n][cin] as n time columns,
    // results utterance-major [n][cout] (one CV_VEC row per utterance)
    const int nv = fs ? fs->n : 1;
    auto vec_conv = [&](const Conv& c, const float* x, float* out) {
        ConvArgs a = cargs(c, x, nv, out);
        a.x_cs = 1; a.x_ts = c.cin;
        a.o_cs = 1; a.o_ts = c.cout;
        conv1d(a, s);
    };
    float* gcond = fs ? fs->gcond : W.gcond;
    // ---- reverse flow: for f = 6,4,2,0: flip, coupling (mean-only)
    for (int fi = 3; fi >= 0; --fi) {
        const auto& fl = V.flows[fi];
        flip_channels(W.z, W.z2, 192, T, s);
        vec_conv(fl.cond, ge, gcond);                                    // g = cond_layer(ge) [1536]
        conv1d(cargs(fl.pre, W.z2, T, W.fh, CV_STORE, sT), s);           // h = pre(x0)   (x0 = first 96 ch)
        hipMemsetAsync(W.fskip, 0, (size_t)192 * T * 4, s);
        for (int l = 0; l < 4; ++l) {
            ConvArgs ci = cargs(fl.in_l[l], W.fh, T, W.fx, CV_VEC, sT);
            ci.vec = gcond + l * 384;
            ci.vec_sstride = fl.cond.cout;
            conv1d(ci, s);
            wn_gate(W.fx, W.fa, 192, T, s);
            if (l < 3) {
                ConvArgs rs = cargs(fl.rs[l], W.fa, T, W.fh, CV_SPLIT_RESID, sT);
                rs.res = W.fh; rs.split = 192; rs.out2 = W.fskip; rs.res2 = W.fskip;
                conv1d(rs, s);
            } else {
                ConvArgs rs = cargs(fl.rs[l], W.fa, T, W.fskip, CV_RESID, sT);
                rs.res = W.fskip;
                conv1d(rs, s);
            }
        }
        // x1 = x1 - post(skip); z = cat(x0, x1)
        ConvArgs po = cargs(fl.post, W.fskip, T, W.z2 + (size_t)96 * T, CV_SUB, sT);
        po.res = W.z2 + (size_t)96 * T;
        conv1d(po, s);
        float* t = W.z; W.z = W.z2; W.z2 = t;
    }
    vec_conv(V.cond, ge, dcond_out);
    return 0;
}

// Several utterances at once: utterance i runs on lane i % K (its own stream and
// workspace), so up to K vocoder chains -- each a few hundred small launches that
// under-fill the chip -- overlap on the GPU.  Each utterance has its own overflow
// flag; after the join, flagged utterances are decoded again on the f32 path.
int gsv_engine::vits_decode_batch(int n, const gsv_vits_item* it, float noise_scale, hipStream_t s) {
    if (n <= 0) return 0;
    if (vb_active)   // an overlapped batch shares the lanes: finish it first
        if (int r = vits_batch_finish(nullptr)) return r;
    if (n > 1 && (vpending || vqueued))
        if (int r = vits_wait(nullptr)) return r;
    if (n == 1) {   // one utterance: the engine stream itself, no lane fork/join
        const gsv_vits_item& u = it[0];
        return vits_decode(u.text_seq, u.n_text, u.sem, u.n_sem, u.ref_audio, u.n_audio, u.ge, u.ge_adv,
                           u.noise_mode == 1 ? u.eps : nullptr, u.noise_mode == 2 ? u.noise_seed : 0, noise_scale,
                           u.audio, s);
    }
    vb_items.assign(it, it + n);
    if (int r = vits_batch_launch(noise_scale, s, true)) return r;
    return vits_batch_finish(s);
}

// ---------------------------------------------------------------- segmented batch
// Buffers for n utterances of T frames in total (gaps included).
int gsv_engine::seg_reserve(int n, int T) {
    SegBatch& B = sgb;
    const VitsWeights& V = vits;
    if ((size_t)T > B.cap_t) {
        const size_t t = std::max((size_t)T, B.cap_t + B.cap_t / 4);
        for (float** p : {&B.z, &B.audio}) {
            retire(*p);
            *p = nullptr;
        }
        for (auto& g : B.g) { retire(g); g = nullptr; }
        for (auto& q : B.seg) { retire(q); q = nullptr; }
        B.cap_t = 0;
        reclaim();
        long f = 1;
        for (int i = 0; i < 5; ++i) f *= V.up_rate[i];
        bool ok = hipMalloc(&B.z, (size_t)192 * t * 4) == hipSuccess &&
                  hipMalloc(&B.audio, (size_t)f * t * 4) == hipSuccess;
        for (auto& g : B.g) ok = ok && hipMalloc(&g, (size_t)V.upc * t * 20 * 4) == hipSuccess;
        long fs = 1;
        for (int i = 0; i < 6; ++i) {
            ok = ok && hipMalloc(&B.seg[i], (size_t)fs * t * 4) == hipSuccess;
            if (i < 5) fs *= V.up_rate[i];
        }
        if (!ok) return set_error(GSV_E_HIP, "segmented vocoder buffers");
        B.cap_t = t;
    }
    if (n > B.cap_n) {
        const int cn = (int)grow_cap(n, B.cap_n);
        for (float** p : {&B.dcond}) { retire(*p); *p = nullptr; }
        for (int** p : {&B.off, &B.len, &B.ovf}) { retire(*p); *p = nullptr; }
        retire_host(B.ovf_host);
        retire_host(B.h_pin);
        B.ovf_host = nullptr;
        B.h_pin = nullptr;
        B.cap_n = 0;
        for (float** p : {&B.ge, &B.gem, &B.gcond}) { retire(*p); *p = nullptr; }
        const int gin = V.flows[0].cond.cin, gcn = V.flows[0].cond.cout;
        reclaim();
        if (hipMalloc(&B.ge, (size_t)cn * gin * 4) != hipSuccess || hipMalloc(&B.gem, (size_t)cn * 512 * 4) != hipSuccess ||
            hipMalloc(&B.gcond, (size_t)cn * gcn * 4) != hipSuccess)
            return set_error(GSV_E_HIP, "segmented vocoder conditioning");
        if (hipMalloc(&B.dcond, (size_t)cn * V.upc * 4) != hipSuccess || hipMalloc(&B.off, (size_t)cn * 4) != hipSuccess ||
            hipMalloc(&B.len, (size_t)cn * 4) != hipSuccess || hipMalloc(&B.ovf, 64) != hipSuccess ||
            hipHostMalloc((void**)&B.ovf_host, 64, hipHostMallocDefault) != hipSuccess ||
            hipHostMalloc((void**)&B.h_pin, (size_t)cn * 8, hipHostMallocDefault) != hipSuccess)
            return set_error(GSV_E_HIP, "segmented vocoder tables");
        B.cap_n = cn;
    }
    if (!B.done && hipEventCreateWithFlags(&B.done, hipEventDisableTiming) != hipSuccess)
        return set_error(GSV_E_HIP, "segmented vocoder event");
    return 0;
}

// The packed front's tables (FrontSeg) for vb_items, built on the host and copied to the
// device on stream s with one copy: text layout, per-column utterance / key-range tables,
// per-utterance input pointers and Philox keys.  The frame layout is sgb's (h_off, h_len,
// seg[0]).
int gsv_engine::seg_front_tables(hipStream_t s) {
    SegBatch& B = sgb;
    const int n = (int)vb_items.size(), Tt = B.T;
    std::vector<int> offS(n);
    int St = 0;
    for (int i = 0; i < n; ++i) {
        offS[i] = St;
        St += vb_items[i].n_text + (i + 1 < n ? SEG_GAP : 0);
    }
    B.St = St;
    auto al = [](size_t x) { return (x + 15) & ~(size_t)15; };
    size_t o = 0;
    const size_t o_segS = o; o = al(o + (size_t)St * 4);
    const size_t o_rowT = o; o = al(o + (size_t)Tt * 8);
    const size_t o_rowS = o; o = al(o + (size_t)St * 8);
    const size_t o_rowX = o; o = al(o + (size_t)Tt * 8);
    const size_t o_offS = o; o = al(o + (size_t)n * 4);
    const size_t o_sems = o; o = al(o + (size_t)n * 8);
    const size_t o_texts = o; o = al(o + (size_t)n * 8);
    const size_t o_seeds = o; o = al(o + (size_t)n * 8);
    const size_t o_gep = o; o = al(o + (size_t)n * 8);
    const size_t o_gemp = o; o = al(o + (size_t)n * 8);
    // the previous batch's copy out of the pinned staging (and its reads of tab_dev) may still
    // be queued: wait for that copy alone
    if (B.tab_ev && hipEventSynchronize(B.tab_ev) != hipSuccess) return set_error(GSV_E_HIP, "vocoder table sync");
    if (!B.tab_ev && hipEventCreateWithFlags(&B.tab_ev, hipEventDisableTiming) != hipSuccess)
        return set_error(GSV_E_HIP, "vocoder table event");
    if (o > B.tab_cap) {
        retire(B.tab_dev);   // a queued batch may still read the old table / staging: retired, not freed
        retire_host(B.tab_pin);
        B.tab_dev = B.tab_pin = nullptr;
        B.tab_cap = 0;
        const size_t cap = o + o / 4;
        if (hipMalloc((void**)&B.tab_dev, cap) != hipSuccess ||
            hipHostMalloc((void**)&B.tab_pin, cap, hipHostMallocDefault) != hipSuccess)
            return set_error(GSV_E_HIP, "segmented vocoder front tables");
        B.tab_cap = cap;
    }
    char* h = B.tab_pin;
    int* segS = reinterpret_cast<int*>(h + o_segS);
    int* rowT = reinterpret_cast<int*>(h + o_rowT);
    int* rowS = reinterpret_cast<int*>(h + o_rowS);
    int* rowX = reinterpret_cast<int*>(h + o_rowX);
    std::fill(segS, segS + St, -1);
    std::fill(rowT, rowT + 2 * (size_t)Tt, 0);
    std::fill(rowS, rowS + 2 * (size_t)St, 0);
    std::fill(rowX, rowX + 2 * (size_t)Tt, 0);
    const bool pp = version == GSV_V2PP;
    for (int i = 0; i < n; ++i) {
        const gsv_vits_item& u = vb_items[i];
        const int t0 = B.h_off[i], tl = B.h_len[i], s0 = offS[i], sl = u.n_text;
        for (int t = t0; t < t0 + tl; ++t) {
            rowT[2 * t] = t0; rowT[2 * t + 1] = tl;
            rowX[2 * t] = s0; rowX[2 * t + 1] = sl;
        }
        for (int c = s0; c < s0 + sl; ++c) {
            segS[c] = i;
            rowS[2 * c] = s0; rowS[2 * c + 1] = sl;
        }
        reinterpret_cast<int*>(h + o_offS)[i] = s0;
        reinterpret_cast<const int64_t**>(h + o_sems)[i] = u.sem;
        reinterpret_cast<const int64_t**>(h + o_texts)[i] = u.text_seq;
        reinterpret_cast<uint64_t*>(h + o_seeds)[i] = u.noise_mode == 2 ? u.noise_seed : 0;
        reinterpret_cast<const float**>(h + o_gep)[i] = u.ge;
        reinterpret_cast<const float**>(h + o_gemp)[i] = pp ? u.ge_adv : u.ge;
    }
    hipMemcpyAsync(B.tab_dev, B.tab_pin, o, hipMemcpyHostToDevice, s);
    hipEventRecord(B.tab_ev, s);
    char* d = B.tab_dev;
    FrontSeg& f = B.fs;
    f.n = n; f.Tt = Tt; f.St = St;
    f.segT = B.seg[0];
    f.segS = reinterpret_cast<const int*>(d + o_segS);
    f.rowT = reinterpret_cast<const int*>(d + o_rowT);
    f.rowS = reinterpret_cast<const int*>(d + o_rowS);
    f.rowX = reinterpret_cast<const int*>(d + o_rowX);
    f.offT = B.off; f.lenT = B.len;
    f.offS = reinterpret_cast<const int*>(d + o_offS);
    f.sems = reinterpret_cast<const int64_t* const*>(d + o_sems);
    f.texts = reinterpret_cast<const int64_t* const*>(d + o_texts);
    f.seeds = reinterpret_cast<const uint64_t*>(d + o_seeds);
    f.ge = B.ge; f.gem = B.gem; f.gcond = B.gcond;
    B.ge_ptrs = reinterpret_cast<const float* const*>(d + o_gep);
    B.gem_ptrs = reinterpret_cast<const float* const*>(d + o_gemp);
    return 0;
}

// The packed front of the batch on stream st: z into sgb.z, dec.cond(ge) into sgb.dcond.
int gsv_engine::seg_front(hipStream_t st) {
    SegBatch& B = sgb;
    const int n = (int)vb_items.size();
    gather_vecs(B.ge_ptrs, n, vits.flows[0].cond.cin, B.ge, st);
    gather_vecs(B.gem_ptrs, n, vits.mrte_o.cout, B.gem, st);
    if (int r = ensure_vits_ws(this, B.fw, B.T, B.St, 0, false)) return r;
    SplitkScope sk(B.fw.splitk, B.fw.splitk_cap);
    if (int r = vits_front(B.fw, nullptr, 0, nullptr, 0, nullptr, 0, nullptr, nullptr, nullptr, 0, vb_scale, B.dcond,
                           st, &B.fs))
        return r;
    hipMemcpyAsync(B.z, B.fw.z, (size_t)192 * B.T * 4, hipMemcpyDeviceToDevice, st);
    return 0;
}

// One generator pass over the batch on stream st (f16: the MRF convs on the split-fp16
// path, flagging an fp16-range input in sgb.ovf).
int gsv_engine::seg_generate(hipStream_t st, bool f16) {
    SegBatch& B = sgb;
    ConvhScope cs(f16 ? B.ovf : nullptr, convh_tile, convt_f16, mrf_fused, convh_persist ? stream_cus(st) : 0,
                  convh_ws == 1 || (convh_ws == 2 && vb_alone) ? stream_cus(st) : 0);
    const int* seg[6] = {B.seg[0], B.seg[1], B.seg[2], B.seg[3], B.seg[4], B.seg[5]};
    float* const gb[5] = {B.g[0], B.g[1], B.g[2], B.g[3], B.g[4]};
    vits_generator(vits, gb, B.z, B.T, B.dcond, vits.upc, seg, B.audio, st);
    return 0;
}

// Each utterance's audio out of the batch buffer (stream st).
void gsv_engine::seg_copy_out(hipStream_t st) {
    long f = 1;
    for (int i = 0; i < 5; ++i) f *= vits.up_rate[i];
    for (size_t i = 0; i < vb_items.size(); ++i)
        hipMemcpyAsync(vb_items[i].audio, sgb.audio + f * sgb.h_off[i], (size_t)f * sgb.h_len[i] * 4,
                       hipMemcpyDeviceToDevice, st);
}

// Fork the batch in vb_items over the lanes (ordered after stream s) and issue it:
// each lane's launches by a host thread of its own (a vocoder pass is a few hundred
// launches, and one thread issuing every lane's would pace the lanes; the per-pass
// host state -- split-K workspace, overflow flag -- is thread-local).  join: wait
// for the issuing threads here; otherwise vits_batch_finish joins them.
int gsv_engine::vits_batch_launch(float noise_scale, hipStream_t s, bool join) {
    const int n = (int)vb_items.size();
    vb_alone = join;
    const int K = std::min(n, vits_lanes);
    for (int l = (int)vlanes.size(); l < K; ++l) {
        VitsLane L;
        if (make_lane_stream(&L.st) != hipSuccess ||
            hipEventCreateWithFlags(&L.join, hipEventDisableTiming) != hipSuccess)
            return set_error(GSV_E_HIP, "vocoder lane stream");
        vlanes.push_back(L);
    }
    if (!vfork && hipEventCreateWithFlags(&vfork, hipEventDisableTiming) != hipSuccess)
        return set_error(GSV_E_HIP, "vocoder fork event");
    // Stream s resets buffers the previous batch may still read on the lanes (the flags,
    // sgb's offsets / segment tables / z, the packed front's tables): order it after that
    // batch's lane work and generator.  vits_batch_finish joined the issuing threads, so
    // the events are recorded (an event never recorded is a no-op wait).
    for (const VitsLane& L : vlanes) hipStreamWaitEvent(s, L.join, 0);
    if (sgb.done) hipStreamWaitEvent(s, sgb.done, 0);
    if (n > vflag_cap) {
        retire(vflags);
        retire_host(vflags_host);
        vflags = nullptr;
        vflags_host = nullptr;
        vflag_cap = 0;
        if (hipMalloc((void**)&vflags, (size_t)n * 4) != hipSuccess ||
            hipHostMalloc((void**)&vflags_host, (size_t)n * 4, hipHostMallocDefault) != hipSuccess)
            return set_error(GSV_E_HIP, "vocoder flags");
        vflag_cap = n;
    }
    // segmented: utterances back to back along time (zero gaps), one generator pass
    const VitsWeights& V = vits;
    bool seg = seg_vocoder && n > 1;
    for (int i = 0; i < 5 && seg; ++i) seg = (V.up_k[i] - V.up_rate[i]) % 2 == 0;   // output = u x input
    if (seg) {
        sgb.h_off.resize(n);
        sgb.h_len.resize(n);
        int T = 0;
        for (int i = 0; i < n; ++i) {
            if (vb_items[i].n_sem <= 0) return set_error(GSV_E_ARG, "empty VITS input");
            sgb.h_off[i] = T;
            sgb.h_len[i] = 2 * vb_items[i].n_sem;
            T += sgb.h_len[i] + (i + 1 < n ? SEG_GAP : 0);
        }
        if (int r = seg_reserve(n, T)) return r;
        sgb.T = T;
        std::memcpy(sgb.h_pin, sgb.h_off.data(), (size_t)n * 4);   // pinned staging: the copies stay async
        std::memcpy(sgb.h_pin + n, sgb.h_len.data(), (size_t)n * 4);
        hipMemcpyAsync(sgb.off, sgb.h_pin, (size_t)n * 4, hipMemcpyHostToDevice, s);
        hipMemcpyAsync(sgb.len, sgb.h_pin + n, (size_t)n * 4, hipMemcpyHostToDevice, s);
        hipMemsetAsync(sgb.z, 0, (size_t)192 * T * 4, s);
        hipMemsetAsync(sgb.ovf, 0, 4, s);
        long f = 1;
        for (int i = 0; i < 6; ++i) {
            seg_fill(sgb.seg[i], f * T, sgb.off, sgb.len, n, (int)f, s);
            if (i < 5) f *= V.up_rate[i];
        }
        // the front part packed too when every item carries its conditioning vectors and
        // draws no explicit eps (else: each item's front on a lane)
        bool packed = seg_front_on;
        const bool pp = version == GSV_V2PP;
        for (int i = 0; i < n && packed; ++i) {
            const gsv_vits_item& u = vb_items[i];
            packed = u.noise_mode != 1 && u.n_text > 0 && 2 * u.n_sem <= MHA_MAXK_HOST &&
                     u.n_text <= MHA_MAXK_HOST && u.ge != nullptr && (!pp || u.ge_adv != nullptr);
        }
        if (packed) {
            if (int r = seg_front_tables(s)) return r;
            ++vits_packed_fronts;
        }
        vb_packed = packed;
    } else {
        vb_packed = false;
    }
    // Every workspace the lanes will use is sized here, on the issuing thread: no lane thread
    // allocates (a hipMalloc beside another thread's stream capture or launches is avoided).
    for (int l = 0; l < K; ++l) {
        if (seg && vb_packed) break;   // the packed front: one workspace, sized below
        int T = 0, S = 0, A = 0;
        for (int i = l; i < n; i += K) {
            T = std::max(T, 2 * vb_items[i].n_sem);
            S = std::max(S, vb_items[i].n_text);
            A = std::max(A, version == GSV_V2PP ? 0 : vb_items[i].n_audio);
        }
        if (T > MHA_MAXK_HOST || S > MHA_MAXK_HOST) continue;   // the lane reports the capacity error
        // with the generator buffers, as the lanes' own ensure_vits_ws calls ask (vits_front, the pass)
        if (int r = ensure_vits_ws(this, vlanes[l].ws, std::max(T, 2), std::max(S, 2), A)) return r;
    }
    if (seg && vb_packed)
        if (int r = ensure_vits_ws(this, sgb.fw, sgb.T, sgb.St, 0, false)) return r;
    if (timing) hipEventRecord(ev[4], s);
    hipMemsetAsync(vflags, 0, (size_t)n * 4, s);
    hipEventRecord(vfork, s);
    for (int l = 0; l < K; ++l) hipStreamWaitEvent(vlanes[l].st, vfork, 0);
    vb_k = K;
    vb_seg = seg;
    vb_scale = noise_scale;
    vb_rcs.assign(K + 1, 0);
    vb_errs.assign(K + 1, std::string());
    auto lane_work = [this, K, n, seg](int l) {
        hipSetDevice(device);
        VitsLane& L = vlanes[l];
        for (int i = l; i < n; i += K) {
            const gsv_vits_item& u = vb_items[i];
            int r = 0;
            if (seg && vb_packed) {   // every utterance's front part in one pass, on lane 0
                if (l == 0) r = seg_front(L.st);
                if (r) {
                    vb_rcs[l] = r;
                    vb_errs[l] = gsv_last_error();
                    return;
                }
                break;
            } else if (seg) {   // the front part; z and dec.cond(ge) into the batch buffers
                VitsWorkspace& W = L.ws;
                r = ensure_vits_ws(this, W, 2 * u.n_sem, u.n_text, version == GSV_V2PP ? 0 : u.n_audio);
                if (!r) {
                    SplitkScope sk(W.splitk, W.splitk_cap);
                    r = vits_front(W, u.text_seq, u.n_text, u.sem, u.n_sem, u.ref_audio, u.n_audio, u.ge, u.ge_adv,
                                   u.noise_mode == 1 ? u.eps : nullptr, u.noise_mode == 2 ? u.noise_seed : 0,
                                   vb_scale, sgb.dcond + (size_t)i * vits.upc, L.st);
                }
                if (!r)
                    hipMemcpy2DAsync(sgb.z + sgb.h_off[i], (size_t)sgb.T * 4, W.z, (size_t)sgb.h_len[i] * 4,
                                     (size_t)sgb.h_len[i] * 4, 192, hipMemcpyDeviceToDevice, L.st);
            } else {
                r = vits_decode_pass(L.ws, u.text_seq, u.n_text, u.sem, u.n_sem, u.ref_audio, u.n_audio, u.ge,
                                     u.ge_adv, u.noise_mode == 1 ? u.eps : nullptr,
                                     u.noise_mode == 2 ? u.noise_seed : 0, vb_scale, u.audio, L.st,
                                     use_convh ? vflags + i : nullptr, false);
            }
            if (r) {
                vb_rcs[l] = r;
                vb_errs[l] = gsv_last_error();   // g_err is thread-local: keep the lane thread's text
                return;
            }
        }
        hipEventRecord(L.join, L.st);
    };
    // the generator of a segmented batch: on lane 0's stream after every lane's front part
    auto gen_work = [this, K]() {
        hipSetDevice(device);
        for (int l = 0; l < K; ++l)
            if (vb_rcs[l]) return;
        hipStream_t gs = vlanes[0].st;
        for (int l = 1; l < K; ++l) hipStreamWaitEvent(gs, vlanes[l].join, 0);
        (void)hipGetLastError();
        seg_generate(gs, use_convh);
        if (use_convh) hipMemcpyAsync(sgb.ovf_host, sgb.ovf, 4, hipMemcpyDeviceToHost, gs);
        seg_copy_out(gs);
        sgb.st = gs;
        hipEventRecord(sgb.done, gs);
        if (hipGetLastError() != hipSuccess) {
            vb_rcs[K] = set_error(GSV_E_HIP, "segmented generator launch");
            vb_errs[K] = gsv_last_error();
        }
    };
    vb_active = true;
    if (!vits_threads) {
        for (int l = 0; l < K; ++l) lane_work(l);
        if (seg) gen_work();
    } else if (seg) {
        // one coordinating thread: lane threads issue the front parts, then it issues the generator
        vb_threads.emplace_back([this, K, lane_work, gen_work]() {
            std::vector<std::thread> lanes;
            for (int l = 0; l < K; ++l) lanes.emplace_back(lane_work, l);
            for (auto& t : lanes) t.join();
            gen_work();
        });
        if (join) {
            for (auto& t : vb_threads) t.join();
            vb_threads.clear();
        }
    } else {
        for (int l = 0; l < K; ++l) vb_threads.emplace_back(lane_work, l);
        if (join) {
            for (auto& t : vb_threads) t.join();
            vb_threads.clear();
        }
    }
    return 0;
}

// Order stream s after the running batch's lanes and generator without finishing it: the
// issuing threads are joined (their events recorded), the results stay for vits_batch_finish.
void gsv_engine::vits_batch_order(hipStream_t s) {
    if (!vb_active) return;
    for (auto& t : vb_threads) t.join();
    vb_threads.clear();
    for (int l = 0; l < vb_k; ++l) hipStreamWaitEvent(s, vlanes[l].join, 0);
    if (vb_seg) hipStreamWaitEvent(s, sgb.done, 0);
}

// Join the batch: lanes -> stream s (NULL: the engine stream), f32 re-runs of the
// utterances that met the fp16 range, phase time.
int gsv_engine::vits_batch_finish(hipStream_t s) {
    if (!vb_active) return 0;
    vb_active = false;
    for (auto& t : vb_threads) t.join();
    vb_threads.clear();
    if (!s) s = stream;
    const int n = (int)vb_items.size(), K = vb_k;
    for (int l = 0; l < K; ++l) hipStreamWaitEvent(s, vlanes[l].join, 0);
    if (vb_seg) hipStreamWaitEvent(s, sgb.done, 0);
    for (int l = 0; l <= K; ++l)
        if (l < (int)vb_rcs.size() && vb_rcs[l]) {   // the other lanes may still write: drain them before reporting
            hipStreamSynchronize(s);
            for (int k = 0; k < K; ++k) hipStreamSynchronize(vlanes[k].st);
            return set_error(vb_rcs[l], (l < K ? "vocoder lane " + std::to_string(l) : std::string("generator")) +
                                            ": " + vb_errs[l]);
        }
    if (vb_seg) {
        if (use_convh) {
            if (hipStreamSynchronize(s) != hipSuccess) return set_error(GSV_E_HIP, "vocoder batch sync");
            if (*sgb.ovf_host) {   // an fp16-range input: the generator again on the f32 path
                ++vits_f32_reruns;
                seg_generate(s, false);
                seg_copy_out(s);
            }
        }
    } else if (use_convh) {
        hipMemcpyAsync(vflags_host, vflags, (size_t)n * 4, hipMemcpyDeviceToHost, s);
        if (hipStreamSynchronize(s) != hipSuccess) return set_error(GSV_E_HIP, "vocoder batch sync");
        for (int i = 0; i < n; ++i) {
            if (!vflags_host[i]) continue;
            ++vits_f32_reruns;
            const gsv_vits_item& u = vb_items[i];
            if (int r = vits_decode_pass(vws, u.text_seq, u.n_text, u.sem, u.n_sem, u.ref_audio, u.n_audio, u.ge,
                                         u.ge_adv, u.noise_mode == 1 ? u.eps : nullptr,
                                         u.noise_mode == 2 ? u.noise_seed : 0, vb_scale, u.audio, s, nullptr,
                                         false))
                return r;
        }
    }
    if (timing) {
        hipEventRecord(ev[5], s);
        hipEventSynchronize(ev[5]);
        hipEventElapsedTime(&ms[3], ev[4], ev[5]);
    }
    return hipGetLastError() == hipSuccess ? 0 : set_error(GSV_E_HIP, "vocoder batch");
}

// V2: the reference encoder alone (vits(v2)#79-271: ref spectrogram -> MelStyleEncoder ->
// ge [512]); it depends on the reference audio only, so a caller synthesising many
// sentences against one reference computes it once and passes it as gsv_vits_item.ge.
int gsv_engine::ref_encode(const float* ref_audio, int n_audio, float* ge, hipStream_t s) {
    if (!vits.ready) return set_error(GSV_E_STATE, "VITS weights not loaded");
    if (version == GSV_V2PP) return set_error(GSV_E_STATE, "V2ProPlus: use gsv_prompt_encode");
    if (n_audio < 2048) return set_error(GSV_E_ARG, "reference audio too short");
    if (int r = ensure_vits_ws(this, vws, 2, 2, n_audio)) return r;
    SplitkScope sk(vws.splitk, vws.splitk_cap);
    (void)hipGetLastError();
    run_ref_enc(vws, vits.ref, ref_audio, n_audio, ge, s);
    return hipGetLastError() == hipSuccess ? 0 : set_error(GSV_E_HIP, "reference encoder launch");
}

int gsv_engine::prompt_encode(const float* ref_audio, int n_audio, const float* sv_emb, float* ge,
                              float* ge_adv, hipStream_t s) {
    if (!penc.ready) return set_error(GSV_E_STATE, "prompt encoder weights not loaded");
    if (n_audio < 2048) return set_error(GSV_E_ARG, "reference audio too short");
    if (int r = ensure_vits_ws(this, vws, 2, 2, n_audio)) return r;
    VitsWorkspace& W = vws;
    SplitkScope sk(W.splitk, W.splitk_cap);
    (void)hipGetLastError();
    run_ref_enc(W, penc.ref, ref_audio, n_audio, W.pe_ge, s);
    // ge = PReLU(ref_enc + (sv_emb @ W^T + b)); ge_adv = ge @ W512^T + b  (prompt_encoder#269-280)
    GemmArgs g{};
    g.M = 1; g.N = 1024; g.K = 20480; g.A = sv_emb; g.lda = 20480;
    g.W = penc.sv_w; g.ldw = 20480; g.w_f16 = 1; g.bias = penc.sv_b; g.C = W.sv; g.ldc = 1024;
    g.mode = EPI_STORE;
    gemm_nt(g, s);
    add_vec(W.pe_ge, W.sv, W.pe_ge, 1024, s);
    prelu_vec(W.pe_ge, penc.prelu, ge, 1024, s);
    GemmArgs a{};
    a.M = 1; a.N = 512; a.K = 1024; a.A = ge; a.lda = 1024; a.W = penc.to512_w; a.ldw = 1024;
    a.bias = penc.to512_b; a.C = ge_adv; a.ldc = 512; a.mode = EPI_STORE;
    gemm_nt(a, s);
    return hipGetLastError() == hipSuccess ? 0 : set_error(GSV_E_HIP, "prompt encoder launch");
}

extern "C" int gsv_vits_decode(gsv_engine* eng, const int64_t* text_seq, int32_t n_text,
                               const int64_t* sem, int32_t n_sem, const float* ref_audio,
                               int32_t n_audio, const float* ge, const float* ge_adv,
                               const float* eps, float noise_scale, float* audio, void* stream) {
    if (!eng) return set_error(GSV_E_ARG, "null engine");
    hipSetDevice(eng->device);
    if (!eng->finalized) return set_error(GSV_E_STATE, "weights not finalized");
    StreamScope sc(eng, stream);
    return eng->vits_decode(text_seq, n_text, sem, n_sem, ref_audio, n_audio, ge, ge_adv, eps, 0,
                            noise_scale, audio, sc.st());
}

extern "C" int gsv_vits_decode_batch(gsv_engine* eng, int32_t n, const gsv_vits_item* items, float noise_scale,
                                     void* stream) {
    if (!eng) return set_error(GSV_E_ARG, "null engine");
    if (n < 0 || (n > 0 && !items)) return set_error(GSV_E_ARG, "bad args");
    hipSetDevice(eng->device);
    if (!eng->finalized) return set_error(GSV_E_STATE, "weights not finalized");
    for (int i = 0; i < n; ++i)
        if (items[i].noise_mode < 0 || items[i].noise_mode > 2 || (items[i].noise_mode == 1 && !items[i].eps) ||
            !items[i].audio)
            return set_error(GSV_E_ARG, "bad vocoder item " + std::to_string(i));
    StreamScope sc(eng, stream);
    return eng->vits_decode_batch(n, items, noise_scale, sc.st());
}

extern "C" int gsv_vits_decode_async(gsv_engine* eng, const gsv_vits_item* item, float noise_scale, void* stream) {
    if (!eng) return set_error(GSV_E_ARG, "null engine");
    if (!item || item->noise_mode < 0 || item->noise_mode > 2 || (item->noise_mode == 1 && !item->eps) || !item->audio)
        return set_error(GSV_E_ARG, "bad vocoder item");
    hipSetDevice(eng->device);
    if (!eng->finalized) return set_error(GSV_E_STATE, "weights not finalized");
    return eng->vits_async(*item, noise_scale, (hipStream_t)stream);
}

extern "C" int gsv_vits_wait(gsv_engine* eng, void* stream) {
    if (!eng) return set_error(GSV_E_ARG, "null engine");
    hipSetDevice(eng->device);
    return eng->vits_wait((hipStream_t)stream);
}

extern "C" int gsv_vits_decode_batch_async(gsv_engine* eng, int32_t n, const gsv_vits_item* items,
                                           float noise_scale, void* stream) {
    if (!eng) return set_error(GSV_E_ARG, "null engine");
    if (n <= 0 || !items) return set_error(GSV_E_ARG, "bad args");
    hipSetDevice(eng->device);
    if (!eng->finalized) return set_error(GSV_E_STATE, "weights not finalized");
    for (int i = 0; i < n; ++i)
        if (items[i].noise_mode < 0 || items[i].noise_mode > 2 || (items[i].noise_mode == 1 && !items[i].eps) ||
            !items[i].audio)
            return set_error(GSV_E_ARG, "bad vocoder item " + std::to_string(i));
    if (int r = eng->vits_batch_finish(nullptr)) return r;
    if (int r = eng->vits_wait(nullptr)) return r;
    eng->vb_items.assign(items, items + n);
    // ordered after the caller's stream only: the engine stream stays free for the T2S
    // of the next batch, which runs beside this one
    return eng->vits_batch_launch(noise_scale, (hipStream_t)stream, false);
}

extern "C" int gsv_vits_batch_wait(gsv_engine* eng, void* stream) {
    if (!eng) return set_error(GSV_E_ARG, "null engine");
    hipSetDevice(eng->device);
    return eng->vits_batch_finish((hipStream_t)stream);
}

extern "C" int gsv_ref_encode(gsv_engine* eng, const float* ref_audio, int32_t n_audio, float* ge, void* stream) {
    if (!eng) return set_error(GSV_E_ARG, "null engine");
    if (!ref_audio || !ge) return set_error(GSV_E_ARG, "bad args");
    hipSetDevice(eng->device);
    if (!eng->finalized) return set_error(GSV_E_STATE, "weights not finalized");
    if (int r = eng->vits_wait(nullptr)) return r;   // shares the vocoder workspace
    if (int r = eng->vits_batch_finish(nullptr)) return r;
    StreamScope sc(eng, stream);
    return eng->ref_encode(ref_audio, n_audio, ge, sc.st());
}

extern "C" int gsv_prompt_encode(gsv_engine* eng, const float* ref_audio, int32_t n_audio,
                                 const float* sv_emb, float* ge, float* ge_adv, void* stream) {
    if (!eng) return set_error(GSV_E_ARG, "null engine");
    hipSetDevice(eng->device);
    if (!eng->finalized) return set_error(GSV_E_STATE, "weights not finalized");
    if (int r = eng->vits_wait(nullptr)) return r;   // shares the vocoder workspace
    if (int r = eng->vits_batch_finish(nullptr)) return r;
    StreamScope sc(eng, stream);
    return eng->prompt_encode(ref_audio, n_audio, sv_emb, ge, ge_adv, sc.st());
}

// ---------------------------------------------------------------- debug hooks
extern "C" int gsv_debug_copy(gsv_engine* eng, const char* name, float* dst, int64_t n, void* stream) {
    if (!eng || !name || !dst) return set_error(GSV_E_ARG, "null arg");
    const VitsWorkspace& W = eng->vws;
    const std::string nm(name);
    const float* src = nm == "ge" ? W.ge : nm == "stats" ? W.stats : nm == "z" ? W.z
                     : nm == "y" ? W.y : nm == "q" ? W.q : nm == "te" ? W.te : nm == "g0" ? W.g0
                     : nm == "g1" ? W.g1 : nm == "spec" ? W.spec : nm == "a" ? W.a : nullptr;
    if (!src) return set_error(GSV_E_ARG, "unknown debug buffer " + nm);
    StreamScope sc(eng, stream);
    return hipMemcpyAsync(dst, src, (size_t)n * 4, hipMemcpyDeviceToDevice, sc.st()) == hipSuccess
               ? 0 : set_error(GSV_E_HIP, "debug copy");
}

extern "C" int gsv_debug_conv1d(const float* x, int cin, int tin, const float* w, int cout, int k,
                                int dil, int pad, const float* bias, float* out, int tout,
                                int in_act, float slope, float* splitk_ws, int64_t splitk_cap,
                                void* stream) {
    ConvArgs a{};
    a.x = x; a.x_cs = tin; a.x_ts = 1; a.Cin = cin; a.Tin = tin;
    a.w = w; a.Cout = cout; a.K = k; a.dil = dil; a.pad = pad; a.bias = bias;
    a.out = out; a.o_cs = tout; a.o_ts = 1; a.n_t = tout; a.o_tstride = 1; a.o_toff = 0; a.o_len = tout;
    a.in_act = in_act; a.in_slope = slope; a.mode = CV_STORE; a.phases = 1;
    a.part = splitk_ws; a.part_cap = splitk_cap;
    conv1d(a, (hipStream_t)stream);
    return hipGetLastError() == hipSuccess ? 0 : set_error(GSV_E_HIP, "debug conv");
}

extern "C" int gsv_debug_conv1d_h(const float* x, int cin, int tin, const void* wh, const float* scale,
                                  int cout, int k, int dil, int pad, const float* bias, float* out, int tout,
                                  int in_act, float slope, int* ovf, void* stream) {
    ConvArgs a{};
    a.x = x; a.x_cs = tin; a.x_ts = 1; a.Cin = cin; a.Tin = tin;
    a.Cout = cout; a.K = k; a.dil = dil; a.pad = pad; a.bias = bias;
    a.out = out; a.o_cs = tout; a.o_ts = 1; a.n_t = tout; a.o_tstride = 1; a.o_toff = 0; a.o_len = tout;
    a.in_act = in_act; a.in_slope = slope; a.mode = CV_STORE; a.phases = 1;
    a.wh = (const __half*)wh; a.wscale = scale; a.ovf = ovf;
    if (!conv1d_h(a, (hipStream_t)stream)) return set_error(GSV_E_ARG, "conv shape not covered by the f16 path");
    return hipGetLastError() == hipSuccess ? 0 : set_error(GSV_E_HIP, "debug conv h");
}
