// Host side of the MI355X GPT-SoVITS engine: weight staging/upload, device
// state, and the C ABI declared in include/genie_engine.h.
//
// T2S orchestration restates GENIE.t2s_cpu (src/genie_tts/Core/Inference.py:63-109):
// encoder -> first-stage decoder -> <=500 stage-decoder steps -> trim; the step
// loop runs on the device as a replayed hipGraph (state lives in HBM, the host
// only polls the per-sequence done flags between graph chunks).
#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "../../include/genie_engine.h"
#include "engine_internal.h"
#include "kernels.h"
#include "prefill_attn.h"

using namespace gsv;

static thread_local std::string g_err;

const char* gsv_last_error(void) { return g_err.c_str(); }
// The build marks its flags in the version string: the Python loader refuses a library built
// with the packed-FP32 target feature on (the gfx950 op_sel fault; build.py).
#if GSV_NO_PACKED_FP32
const char* gsv_version(void) { return "genie-mi355x 0.1 (gfx950, no packed-fp32)"; }
#else
const char* gsv_version(void) { return "genie-mi355x 0.1 (gfx950, packed-fp32)"; }
#endif

namespace gsv {
int set_error(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

int hip_error(const std::string& what, hipError_t e) {
    return set_error(GSV_E_HIP, what + ": " + hipGetErrorName(e));
}
}  // namespace gsv

// ------------------------------------------------------------ allocation
std::shared_mutex gsv::capture_mu;

static int64_t alloc_bytes(void* p) {
    size_t n = 0;
    return p && hipMemPtrGetInfo(p, &n) == hipSuccess ? (int64_t)n : 0;
}

void gsv_engine::retire(void* p) {
    if (!p) return;
    const int64_t n = alloc_bytes(p);
    std::lock_guard<std::mutex> g(alloc_mu);
    retired.push_back(p);
    retired_bytes += n;
}

void gsv_engine::retire_host(void* p) {
    if (!p) return;
    std::lock_guard<std::mutex> g(alloc_mu);
    retired_host.push_back(p);
}

// Free the retired buffers.  Skipped while a vocoder batch's lane threads may still be issuing
// work (they are joined by vits_batch_finish; the next growth reclaims).  This engine's streams
// are drained first, so no queued kernel still reads a retired buffer, and no capture runs in
// the process while hipFree synchronises the device.
void gsv_engine::reclaim() {
    if (vb_active) return;
    std::vector<void*> d, h;
    int64_t nb = 0;
    {
        std::lock_guard<std::mutex> g(alloc_mu);
        if (retired.empty() && retired_host.empty()) return;
        d.swap(retired);
        h.swap(retired_host);
        nb = retired_bytes;
        retired_bytes = 0;
    }
    std::unique_lock<std::shared_mutex> cl(gsv::capture_mu);
    if (sync_own_streams() != hipSuccess) {   // keep them: a later pass (or the destructor) frees them
        (void)hipGetLastError();
        std::lock_guard<std::mutex> g(alloc_mu);
        retired.insert(retired.end(), d.begin(), d.end());
        retired_host.insert(retired_host.end(), h.begin(), h.end());
        retired_bytes += nb;
        return;
    }
    for (void* p : d) hipFree(p);
    for (void* p : h) hipHostFree(p);
    reclaimed_bytes += nb;
    ++reclaims;
}

void* gsv_engine::dalloc(size_t bytes) {
    void* p = nullptr;
    if (bytes == 0) bytes = 16;
    if (hipMalloc(&p, (bytes + 255) & ~(size_t)255) != hipSuccess) return nullptr;
    std::lock_guard<std::mutex> g(alloc_mu);   // vocoder lane threads grow their workspaces
    allocs.push_back(p);
    return p;
}

void gsv_engine::release_all() {
    for (auto& kv : graphs) hipGraphExecDestroy(kv.second);
    graphs.clear();
    for (void* p : allocs) hipFree(p);
    allocs.clear();
}

gsv_engine::~gsv_engine() {
    for (auto& t : vb_threads) t.join();
    std::unique_lock<std::shared_mutex> cl(gsv::capture_mu);   // hipFree below synchronises the device
    release_all();
    for (void* p : pk_allocs) hipFree(p);
    pk_allocs.clear();
    if (pk_tiles) hipFree(pk_tiles);
    drop_sides();
    if (own_stream && stream) hipStreamDestroy(stream);
    if (vstream) hipStreamDestroy(vstream);
    for (hipEvent_t e : {vev_in, vev_done, pf_in, pf_done, pf_copied, pf_fork, pf_ev[0], pf_ev[1], pf_ev[2]})
        if (e) hipEventDestroy(e);
    if (done_host) hipHostFree(done_host);
    for (auto& e : kev) if (e) hipEventDestroy(e);
    if (ktrace) hipFree(ktrace);
    if (ptrace) hipFree(ptrace);
    if (pws) hipFree(pws);
    if (hubert.ws) hipFree(hubert.ws);
    if (bert.ws) hipFree(bert.ws);
    if (sv_ws) hipFree(sv_ws);
    if (sv_ovf) hipFree(sv_ovf);
    if (sv_ovf_host) hipHostFree(sv_ovf_host);
    if (perr_host) hipHostFree(perr_host);
    if (stop_word) hipHostFree(stop_word);
    if (res_pin) hipHostFree(res_pin);
    for (GenSlot& g : gq) {
        if (g.res) hipHostFree(g.res);
        if (g.perr_h) hipHostFree(g.perr_h);
        for (hipEvent_t e : {g.d0, g.done, g.k0, g.k1})
            if (e) hipEventDestroy(e);
    }
    for (float* p : {sgb.z, sgb.dcond, sgb.audio, sgb.g[0], sgb.g[1], sgb.g[2], sgb.g[3], sgb.g[4]})
        if (p) hipFree(p);
    for (int* p : {sgb.seg[0], sgb.seg[1], sgb.seg[2], sgb.seg[3], sgb.seg[4], sgb.seg[5], sgb.off, sgb.len, sgb.ovf})
        if (p) hipFree(p);
    for (float* p : {sgb.ge, sgb.gem, sgb.gcond})
        if (p) hipFree(p);
    if (sgb.tab_dev) hipFree(sgb.tab_dev);
    if (sgb.tab_pin) hipHostFree(sgb.tab_pin);
    if (sgb.tab_ev) hipEventDestroy(sgb.tab_ev);
    if (sgb.ovf_host) hipHostFree(sgb.ovf_host);
    if (sgb.h_pin) hipHostFree(sgb.h_pin);
    if (sgb.done) hipEventDestroy(sgb.done);
    if (vovf_host) hipHostFree(vovf_host);
    if (vovf) hipFree(vovf);
    for (auto& L : vlanes) {
        if (L.st) hipStreamDestroy(L.st);
        if (L.join) hipEventDestroy(L.join);
    }
    if (vfork) hipEventDestroy(vfork);
    if (vflags) hipFree(vflags);
    if (vflags_host) hipHostFree(vflags_host);
    if (perr) hipFree(perr);
    for (void* p : state_allocs) hipFree(p);
    state_allocs.clear();
    for (void* p : enc_allocs) hipFree(p);
    for (auto& e : poll_ev) if (e) hipEventDestroy(e);
    for (auto& e : ev) if (e) hipEventDestroy(e);
    if (ev_in) hipEventDestroy(ev_in);
    if (ev_out) hipEventDestroy(ev_out);
    for (void* p : retired) hipFree(p);
    for (void* p : retired_host) hipHostFree(p);
}

hipError_t gsv_engine::sync_own_streams() {
    hipError_t r = hipSuccess;
    for (hipStream_t s : {stream, vstream})
        if (s && r == hipSuccess) r = hipStreamSynchronize(s);
    {
        std::lock_guard<std::mutex> lk(side_mu);
        for (auto& p : sides)
            for (hipStream_t q : p->st)
                if (r == hipSuccess) r = hipStreamSynchronize(q);
    }
    for (auto& L : vlanes)
        if (L.st && r == hipSuccess) r = hipStreamSynchronize(L.st);
    return r;
}

// ------------------------------------------------------------ weights
const Staged* gsv_engine::find(const std::string& n) const {
    auto it = staged.find(n);
    return it == staged.end() ? nullptr : &it->second;
}

float* gsv_engine::up_f32(const std::string& n, int* err) {
    const Staged* s = find(n);
    if (!s) { *err = set_error(GSV_E_WEIGHT, "missing weight " + n); return nullptr; }
    float* d = (float*)dalloc(s->data.size() * 4);
    if (!d) { *err = set_error(GSV_E_HIP, "hipMalloc failed for " + n); return nullptr; }
    hipMemcpy(d, s->data.data(), s->data.size() * 4, hipMemcpyHostToDevice);
    return d;
}

// fp16 copies never round: a tensor bound for an fp16-only path must be fp16-exact (the
// Genie fp16 bins are); an fp32 tensor of a split-weight path goes through up_w16.
static int64_t first_non_f16(const float* v, size_t n) {
    for (size_t i = 0; i < n; ++i)
        if (__half2float(__float2half(v[i])) != v[i] && !(v[i] != v[i])) return (int64_t)i;
    return -1;
}

extern "C" int gsv_f16_exact(const float* v, int64_t n, int64_t* first_bad) {
    if (!v && n > 0) return set_error(GSV_E_ARG, "null values");
    const int64_t b = n > 0 ? first_non_f16(v, (size_t)n) : -1;
    if (first_bad) *first_bad = b;
    return b < 0 ? 1 : 0;
}

int gsv::f16_inexact_error(const std::string& n, const float* v, int64_t i) {
    char buf[96];
    std::snprintf(buf, sizeof buf, " is not fp16-exact (element %lld = %.9g)", (long long)i, (double)v[i]);
    return set_error(GSV_E_WEIGHT, "weight " + n + buf + "; its path takes fp16 weights only");
}

__half* gsv_engine::up_f16(const std::string& n, int* err) {
    const Staged* s = find(n);
    if (!s) { *err = set_error(GSV_E_WEIGHT, "missing weight " + n); return nullptr; }
    const int64_t bad = first_non_f16(s->data.data(), s->data.size());
    if (bad >= 0) { *err = f16_inexact_error(n, s->data.data(), bad); return nullptr; }
    std::vector<__half> h(s->data.size());
    for (size_t i = 0; i < h.size(); ++i) h[i] = __float2half(s->data[i]);
    __half* d = (__half*)dalloc(h.size() * 2);
    if (!d) { *err = set_error(GSV_E_HIP, "hipMalloc failed for " + n); return nullptr; }
    hipMemcpy(d, h.data(), h.size() * 2, hipMemcpyHostToDevice);
    return d;
}

__half* gsv_engine::up_f16_t(const std::string& n, int* err) {
    const Staged* s = find(n);
    if (!s || s->dims.size() != 2) { *err = set_error(GSV_E_WEIGHT, "missing 2-D weight " + n); return nullptr; }
    const int64_t bad = first_non_f16(s->data.data(), s->data.size());
    if (bad >= 0) { *err = f16_inexact_error(n, s->data.data(), bad); return nullptr; }
    const size_t R = s->dims[0], C = s->dims[1];
    std::vector<__half> h(R * C);
    for (size_t r = 0; r < R; ++r)
        for (size_t c = 0; c < C; ++c) h[c * R + r] = __float2half(s->data[r * C + c]);
    __half* d = (__half*)dalloc(h.size() * 2);
    if (!d) { *err = set_error(GSV_E_HIP, "hipMalloc failed for " + n); return nullptr; }
    hipMemcpy(d, h.data(), h.size() * 2, hipMemcpyHostToDevice);
    return d;
}

// W16 planes of v (already in the kernel's layout): hi only when every value is fp16-exact,
// else hi = fp16(w) and lo = fp16((w - hi) 2^11).  |w| beyond the fp16 range has no split.
W16 gsv_engine::upload_w16(const std::string& n, const std::vector<float>& v, int* err) {
    W16 w;
    if (*err) return w;
    std::vector<__half> hi(v.size()), lo;
    const bool exact = first_non_f16(v.data(), v.size()) < 0;
    if (!exact) lo.resize(v.size());
    for (size_t i = 0; i < v.size(); ++i) {
        if (!(std::fabs(v[i]) <= 65504.f)) {
            *err = set_error(GSV_E_WEIGHT, "weight " + n + " has a value beyond the fp16 range");
            return w;
        }
        hi[i] = __float2half(v[i]);
        if (!exact) lo[i] = __float2half((v[i] - __half2float(hi[i])) * W16_LO_SCALE);
    }
    w.hi = (__half*)dalloc(hi.size() * 2);
    if (!exact) w.lo = (__half*)dalloc(lo.size() * 2);
    if (!w.hi || (!exact && !w.lo)) { *err = set_error(GSV_E_HIP, "hipMalloc failed for " + n); return W16{}; }
    hipMemcpy(w.hi, hi.data(), hi.size() * 2, hipMemcpyHostToDevice);
    if (!exact) hipMemcpy(w.lo, lo.data(), lo.size() * 2, hipMemcpyHostToDevice);
    if (!exact) ++w16_split_tensors;
    return w;
}

W16 gsv_engine::up_w16(const std::string& n, int* err) {
    const Staged* s = find(n);
    if (!s) { *err = set_error(GSV_E_WEIGHT, "missing weight " + n); return W16{}; }
    return upload_w16(n, s->data, err);
}

static std::vector<float> default_div_term() {
    // exp(-2i ln(1e4)/512) in fp32; a character directory may override it with
    // the exact constant of its own graph ("pe.div_term").
    std::vector<float> d(256);
    const float c = (float)(-(std::log(10000.0) / 512.0));
    for (int i = 0; i < 256; ++i) d[i] = std::exp((float)(2 * i) * c);
    return d;
}

int gsv_engine::finalize_t2s() {
    int err = 0;
    // PE table rows 0..pe_max-1 at 1-based positions (row p = position p).
    std::vector<float> div = default_div_term();
    if (const Staged* s = find("pe.div_term"))
        if (s->data.size() == 256) div = s->data;
    pe_max = 4096;
    if (const char* e = std::getenv("GENIE_FFN_SLICES")) ffn_slices = std::atoi(e) == 32 ? 32 : 64;
    if (const char* e = std::getenv("GENIE_DECODE_FUSE")) fuse_qkv = std::atoi(e) == 2;
    if (const char* e = std::getenv("GENIE_ACC")) use_acc = std::atoi(e) != 0;
    if (const char* e = std::getenv("GENIE_PERSIST")) use_persist = std::atoi(e) != 0;
    if (const char* e = std::getenv("GENIE_PERSIST1")) use_persist1 = std::atoi(e) != 0;
    if (const char* e = std::getenv("GENIE_PERSIST1M")) use_persist1m = std::atoi(e) != 0;
    if (const char* e = std::getenv("GENIE_PERSISTM")) use_persistm = std::atoi(e) != 0;
    if (const char* e = std::getenv("GENIE_PRESPLIT")) use_presplit = std::atoi(e) != 0;
    if (const char* e = std::getenv("GENIE_CONVH")) use_convh = std::atoi(e) != 0;
    if (const char* e = std::getenv("GENIE_CONVH_WS")) convh_ws = std::max(0, std::min(2, std::atoi(e)));
    if (const char* e = std::getenv("GENIE_VITS_FORK")) vits_fork = std::atoi(e) != 0;
    if (const char* e = std::getenv("GENIE_PF_DELAY")) persist1_pf_delay = std::max(0, std::atoi(e));
    if (const char* e = std::getenv("GENIE_KTRACE"))
        if (std::atoi(e) == 1 && !ktrace) {
            hipMalloc(&ktrace, (size_t)3 * 256 * 8 * 8);
            hipMemset(ktrace, 0, (size_t)3 * 256 * 8 * 8);
        }
    std::vector<float> pe((size_t)pe_max * 512);
    for (int p = 0; p < pe_max; ++p)
        for (int i = 0; i < 256; ++i) {
            const float ang = (float)p * div[i];
            pe[(size_t)p * 512 + 2 * i] = std::sin(ang);
            pe[(size_t)p * 512 + 2 * i + 1] = std::cos(ang);
        }
    pe_tab = (float*)dalloc(pe.size() * 4);
    hipMemcpy(pe_tab, pe.data(), pe.size() * 4, hipMemcpyHostToDevice);

    // ar_audio_position alpha etc.
    emb_audio = up_f16("ar_audio_embedding.word_embeddings.weight", &err);
    alpha_audio = up_f32("ar_audio_position.alpha", &err);
    w_pred = up_f16("ar_predict_layer.weight", &err);
    for (int l = 0; l < 24 && !err; ++l) {
        const std::string p = "transformer_encoder.layers." + std::to_string(l) + ".";
        T2SLayerW& L = layers[l];
        L.w_in = up_f16(p + "self_attn.in_proj_weight", &err);
        L.b_in = up_f32(p + "self_attn.in_proj_bias", &err);
        L.w_out = up_f16(p + "self_attn.out_proj.weight", &err);
        L.b_out = up_f32(p + "self_attn.out_proj.bias", &err);
        L.w1 = up_f16(p + "linear1.weight", &err);
        L.b1 = up_f32(p + "linear1.bias", &err);
        L.w2 = up_f16(p + "linear2.weight", &err);
        L.woT = up_f16_t(p + "self_attn.out_proj.weight", &err);
        L.w2T = up_f16_t(p + "linear2.weight", &err);
        L.b2 = up_f32(p + "linear2.bias", &err);
        L.n1w = up_f32(p + "norm1.weight", &err);
        L.n1b = up_f32(p + "norm1.bias", &err);
        L.n2w = up_f32(p + "norm2.weight", &err);
        L.n2b = up_f32(p + "norm2.bias", &err);
    }
    if (err) return err;
    // LayerNorm affine folded through the GEMV that consumes it (PersistArgs::fold), in
    // double from the staged fp16-valued weights
    {
        constexpr size_t FL = 2 * 1536 + 2 * 2048;
        std::vector<float> fold(24 * FL + 2 * 1025, 0.f);
        auto fw = [&](const std::string& n) { return find(n); };
        for (int l = 0; l < 24; ++l) {
            const std::string p = "transformer_encoder.layers." + std::to_string(l) + ".";
            const std::string q = "transformer_encoder.layers." + std::to_string(l - 1) + ".";
            const Staged *win = fw(p + "self_attn.in_proj_weight"), *bin = fw(p + "self_attn.in_proj_bias");
            const Staged *w1 = fw(p + "linear1.weight"), *b1 = fw(p + "linear1.bias");
            const Staged *n1w = fw(p + "norm1.weight"), *n1b = fw(p + "norm1.bias");
            const Staged* n2w = l > 0 ? fw(q + "norm2.weight") : nullptr;
            const Staged* n2b = l > 0 ? fw(q + "norm2.bias") : nullptr;
            float* F = fold.data() + l * FL;
            for (int r = 0; r < 1536; ++r) {
                double sb = 0.0, sc = 0.0;
                if (l > 0)
                    for (int k = 0; k < 512; ++k) {
                        const double wv = win->data[(size_t)r * 512 + k];
                        sb += wv * n2w->data[k];
                        sc += wv * n2b->data[k];
                    }
                F[r] = (float)sb;
                F[1536 + r] = (float)(sc + bin->data[r]);
            }
            for (int r = 0; r < 2048; ++r) {
                double sb = 0.0, sc = 0.0;
                for (int k = 0; k < 512; ++k) {
                    const double wv = w1->data[(size_t)r * 512 + k];
                    sb += wv * n1w->data[k];
                    sc += wv * n1b->data[k];
                }
                F[3072 + r] = (float)sb;
                F[5120 + r] = (float)(sc + b1->data[r]);
            }
        }
        {   // logits head: LN2 of layer 23 folded through ar_predict_layer (no bias)
            const Staged* wp = fw("ar_predict_layer.weight");
            const Staged* n2w = fw("transformer_encoder.layers.23.norm2.weight");
            const Staged* n2b = fw("transformer_encoder.layers.23.norm2.bias");
            float* F = fold.data() + 24 * FL;
            for (int r = 0; r < 1025; ++r) {
                double sb = 0.0, sc = 0.0;
                for (int k = 0; k < 512; ++k) {
                    const double wv = wp->data[(size_t)r * 512 + k];
                    sb += wv * n2w->data[k];
                    sc += wv * n2b->data[k];
                }
                F[r] = (float)sb;
                F[1025 + r] = (float)sc;
            }
        }
        ln_fold = (float*)dalloc(fold.size() * 4);
        if (!ln_fold) return set_error(GSV_E_HIP, "LayerNorm fold");
        hipMemcpy(ln_fold, fold.data(), fold.size() * 4, hipMemcpyHostToDevice);
    }
    hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, device);
    text_emb = up_f32("encoder.ar_text_embedding.word_embeddings.weight", &err);
    bert_w = up_f32("encoder.bert_proj.weight", &err);
    bert_b = up_f32("encoder.bert_proj.bias", &err);
    alpha_text = up_f32("encoder.ar_text_position.alpha", &err);
    ssl_w = up_f32("vits.ssl_proj.weight", &err);
    ssl_b = up_f32("vits.ssl_proj.bias", &err);
    codebook = up_f32("vits.quantizer.vq.layers.0._codebook.embed", &err);
    if (err) return err;
    cb_sumsq = (float*)dalloc(1024 * 4);
    sumsq_rows(codebook, 768, 1024, 768, cb_sumsq, nullptr);
    // qk scale exactly as the graph: Sqrt(Div(1, Sqrt(Cast(32))))  (stage#84-90)
    qk_scale = std::sqrt(1.0f / std::sqrt(32.0f));
    return hipDeviceSynchronize() == hipSuccess ? 0 : set_error(GSV_E_HIP, "finalize_t2s sync");
}

// ------------------------------------------------------------ capacity
int gsv_engine::reserve(int batch, int tokens) {
    if (batch <= max_batch && tokens <= tmax) return 0;
    if (batch > 64) return set_error(GSV_E_CAPACITY, "batch > 64 not supported");
    if (tokens > pe_max - 1) return set_error(GSV_E_CAPACITY, "tokens exceed PE table");
    // graphs capture buffer addresses: drop them before reallocating
    for (auto& kv : graphs) hipGraphExecDestroy(kv.second);
    graphs.clear();
    // quantised growth: batch to a power of two (<= 64), tokens to a multiple of 256 (<= the
    // PE table), so a server's load ramp re-allocates a few times, not once per new maximum
    int pb = 1;
    while (pb < batch) pb <<= 1;
    const int nb = std::max(max_batch, std::min(64, pb));
    const int nt = std::max(tmax, std::min(pe_max - 1, (tokens + 255) / 256 * 256));
    for (void* p : state_allocs) retire(p);
    state_allocs.clear();
    max_batch = tmax = 0;   // nothing is allocated until the new state is complete
    reclaim();              // the old state's memory goes back before the new state is allocated
    auto A = [&](size_t bytes) -> void* {
        void* p = nullptr;
        if (hipMalloc(&p, (bytes + 255) & ~(size_t)255) != hipSuccess) return nullptr;
        state_allocs.push_back(p);
        return p;
    };
    const size_t kv_layer = (size_t)nb * 16 * nt * 32;
    for (int l = 0; l < 24; ++l) {
        kcache[l] = (float*)A(kv_layer * 4);
        vcache[l] = (float*)A(kv_layer * 4);
        if (!kcache[l] || !vcache[l]) return set_error(GSV_E_HIP, "KV cache allocation failed");
    }
    y = (int64_t*)A((size_t)nb * nt * 8);
    ny = (int*)A(nb * 4);
    kvlen = (int*)A(nb * 4);
    steps = (int*)A(nb * 4);
    done = (uint8_t*)A(nb);
    stopf = (uint8_t*)A(nb);
    seen = (uint32_t*)A((size_t)nb * 33 * 4);
    forceb = (int*)A(nb * 4);
    dslab = (float*)A((size_t)8 * nb * 2048 * 4);   // batched-decode split-K slabs (2 regions)
    h = (float*)A((size_t)nb * 512 * 4);
    h1 = (float*)A((size_t)nb * 512 * 4);
    s1 = (float*)A((size_t)nb * 512 * 4);
    s2 = (float*)A((size_t)nb * 512 * 4);
    q = (float*)A((size_t)nb * 512 * 4);
    o = (float*)A((size_t)nb * 512 * 4);
    f = (float*)A((size_t)nb * 2048 * 4);
    logits = (float*)A((size_t)nb * 1025 * 4);
    attn_part = (float*)A((size_t)16 * nb * 512 * 4);
    ffn_part = (float*)A((size_t)64 * nb * 512 * 4);
    ident = (int*)A(nb * 4);
    pH = (float*)A((size_t)nt * 512 * 4);
    pQ = (float*)A((size_t)nt * 512 * 4);
    pO = (float*)A((size_t)nt * 512 * 4);
    pS = (float*)A((size_t)nt * 512 * 4);
    pH1 = (float*)A((size_t)nt * 512 * 4);
    pF = (float*)A((size_t)nt * 2048 * 4);
    prow_len = (int*)A((size_t)nt * 4);
    prompts_buf = (int64_t*)A((size_t)nt * 8);
    acc64 = (long long*)A((size_t)nb * ACC_SEQ * 8);
    pSlab = (float*)A((size_t)8 * nt * 512 * 4);
    if (!pF || !prompts_buf || !acc64 || !pSlab) return set_error(GSV_E_HIP, "state allocation failed");
    // stream-ordered (no null-stream call while another thread may be capturing), then waited
    // for: id lives on this frame
    hipMemsetAsync(acc64, 0, (size_t)nb * ACC_SEQ * 8, stream);
    std::vector<int> id(nb);
    for (int i = 0; i < nb; ++i) id[i] = i;
    hipMemcpyAsync(ident, id.data(), nb * 4, hipMemcpyHostToDevice, stream);
    hipMemsetAsync(done, 1, nb, stream);
    hipMemsetAsync(forceb, 0, nb * 4, stream);
    if (hipStreamSynchronize(stream) != hipSuccess) return set_error(GSV_E_HIP, "state init");
    max_batch = nb;
    tmax = nt;
    return 0;
}

// ------------------------------------------------------------ encoder
static __global__ void k_fill_row_len(int* rl, int L, int N0) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r < N0) rl[r] = r < L ? L : r + 1;
}

int gsv_engine::ensure_enc_ws(int P, int L) {
    if (P <= enc_cap_p && L <= enc_cap_l) return 0;
    const int cp = (int)grow_cap(P, enc_cap_p), cl = (int)grow_cap(L, enc_cap_l);
    for (void* p : enc_allocs) retire(p);
    enc_allocs.clear();
    enc_cap_p = enc_cap_l = 0;
    reclaim();
    auto A = [&](size_t bytes) -> float* {
        void* p = nullptr;
        if (hipMalloc(&p, (bytes + 255) & ~(size_t)255) != hipSuccess) return nullptr;
        enc_allocs.push_back(p);
        return (float*)p;
    };
    e_im2col = A((size_t)cp * 1536 * 4);
    e_h = A((size_t)cp * 768 * 4);
    e_hh = A((size_t)cp * 4);
    e_dist = A((size_t)cp * 1024 * 4);
    e_bproj = A((size_t)cl * 512 * 4);
    e_bert = A((size_t)cl * 1024 * 4);
    if (!e_im2col || !e_h || !e_hh || !e_dist || !e_bproj || !e_bert) return set_error(GSV_E_HIP, "encoder workspace");
    enc_cap_p = cp;
    enc_cap_l = cl;
    return 0;
}

int gsv_engine::encode(const gsv_utt* u, float* x, int64_t* prompts, hipStream_t st, bool do_prompts) {
    const int L = u->n_ref + u->n_text, P = u->n_ssl / 2;
    if (L <= 0 || P <= 0) return set_error(GSV_E_ARG, "empty utterance");
    if (int e = ensure_enc_ws(P, L)) return e;
    if (do_prompts) {
    // K2: ssl_proj Conv1d(768,768,k2,s2) as GEMM over im2col, then VQ argmin (#2-48)
    ssl_im2col(u->ssl, u->n_ssl, e_im2col, st);
    GemmArgs g{};
    g.M = P; g.N = 768; g.K = 1536;
    g.A = e_im2col; g.lda = 1536;
    g.W = ssl_w; g.ldw = 1536; g.w_f16 = 0;
    g.bias = ssl_b; g.C = e_h; g.ldc = 768; g.mode = EPI_STORE;
    gemm_nt(g, st);
    sumsq_rows(e_h, 768, P, 768, e_hh, st);
    GemmArgs d{};
    d.M = P; d.N = 1024; d.K = 768;
    d.A = e_h; d.lda = 768; d.W = codebook; d.ldw = 768; d.w_f16 = 0;
    d.C = e_dist; d.ldc = 1024; d.mode = EPI_VQDIST; d.rowsq = e_hh; d.colsq = cb_sumsq;
    gemm_nt(d, st);
    argmin_dist_rows(e_dist, P, 1024, prompts, st);
    }
    // K1: text embedding + bert projection + PE (#49-83)
    const float* bproj = nullptr;
    if (u->ref_bert || u->text_bert) {
        if (u->ref_bert)
            hipMemcpyAsync(e_bert, u->ref_bert, (size_t)u->n_ref * 1024 * 4, hipMemcpyDeviceToDevice, st);
        else
            hipMemsetAsync(e_bert, 0, (size_t)u->n_ref * 1024 * 4, st);
        if (u->text_bert)
            hipMemcpyAsync(e_bert + (size_t)u->n_ref * 1024, u->text_bert, (size_t)u->n_text * 1024 * 4,
                           hipMemcpyDeviceToDevice, st);
        else
            hipMemsetAsync(e_bert + (size_t)u->n_ref * 1024, 0, (size_t)u->n_text * 1024 * 4, st);
        GemmArgs b{};
        b.M = L; b.N = 512; b.K = 1024;
        b.A = e_bert; b.lda = 1024; b.W = bert_w; b.ldw = 1024; b.w_f16 = 0;
        b.C = e_bproj; b.ldc = 512; b.mode = EPI_STORE;
        gemm_nt(b, st);
        bproj = e_bproj;
    }
    text_embed(u->ref_seq, u->n_ref, u->text_seq, u->n_text, text_emb, bproj, bert_b, alpha_text,
               pe_tab, x, st);
    const hipError_t le = hipGetLastError();
    return le == hipSuccess ? 0 : hip_error("encode launch", le);
}

// ------------------------------------------------------------ prefill
int gsv_engine::prefill_slot(int b, const float* x, int L, const int64_t* pr, int P,
                             const gsv_sampler* sp, float* logits_out, hipStream_t st, int noise_b) {
    const int N0 = L + P;
    if (N0 + 1 > tmax) return set_error(GSV_E_CAPACITY, "prefill exceeds reserved tokens");
    if (x != pH) hipMemcpyAsync(pH, x, (size_t)L * 512 * 4, hipMemcpyDeviceToDevice, st);
    seq_state_init(b, pr, P, L, y, tmax, ny, kvlen, steps, done, seen, st);
    audio_embed_prompts(pr, P, emb_audio, alpha_audio, pe_tab, pH + (size_t)L * 512, st);
    hipLaunchKernelGGL(k_fill_row_len, dim3((N0 + 255) / 256), dim3(256), 0, st, prow_len, L, N0);
    const long sstride = (long)16 * tmax * 32;
    for (int l = 0; l < 24; ++l) {
        const T2SLayerW& W = layers[l];
        GemmArgs g{};
        g.M = N0; g.N = 1536; g.K = 512; g.A = pH; g.lda = 512;
        g.W = W.w_in; g.ldw = 512; g.w_f16 = 1; g.bias = W.b_in;
        g.C = pQ; g.ldc = 512; g.mode = EPI_QKV;
        g.kv.k = kcache[l] + b * sstride; g.kv.v = vcache[l] + b * sstride;
        g.kv.tmax = tmax; g.kv.pos0 = 0; g.kv.seq_stride = sstride;
        gemm_nt(g, st);
        AttnArgs at{};
        at.q = pQ; at.ldq = 512; at.k = kcache[l] + b * sstride; at.v = vcache[l] + b * sstride;
        at.seq_stride = sstride; at.tmax = tmax; at.row_len = prow_len; at.out = pO; at.ldo = 512;
        at.rows = N0; at.scale = qk_scale;
        if (use_attn_mf32 && prefill_mf32_on()) attn_rows_mf32_seq(at, st);   // the f32 MFMA, k_attn_flash's arithmetic
        else attn_rows(at, st);
        // out-proj and FFN2 have 32 output tiles: split K over 4 / 8 blocks into slabs,
        // reduced in fixed order (+ bias + residual) by the LayerNorm that follows
        const bool slabs = gemm_slabs_supported(512, 512, 512) && gemm_slabs_supported(2048, 2048, 2048);
        const long slab_stride = (long)tmax * 512;
        GemmArgs go{};
        go.M = N0; go.N = 512; go.K = 512; go.A = pO; go.lda = 512;
        go.W = W.w_out; go.ldw = 512; go.w_f16 = 1; go.bias = W.b_out;
        if (slabs) {
            go.C = pSlab; go.ldc = 512; go.mode = EPI_SLAB; go.ksplit = 4; go.slab_stride = slab_stride;
            gemm_nt(go, st);
            layernorm_rows_slabs(pSlab, 4, slab_stride, W.b_out, pH, pH1, N0, W.n1w, W.n1b, st);
        } else {
            go.C = pS; go.ldc = 512; go.mode = EPI_RESID; go.res = pH; go.ldr = 512;
            gemm_nt(go, st);
            layernorm_rows(pS, pH1, N0, W.n1w, W.n1b, st);
        }
        GemmArgs g1{};
        g1.M = N0; g1.N = 2048; g1.K = 512; g1.A = pH1; g1.lda = 512;
        g1.W = W.w1; g1.ldw = 512; g1.w_f16 = 1; g1.bias = W.b1;
        g1.C = pF; g1.ldc = 2048; g1.mode = EPI_RELU;
        gemm_nt(g1, st);
        GemmArgs g2{};
        g2.M = N0; g2.N = 512; g2.K = 2048; g2.A = pF; g2.lda = 2048;
        g2.W = W.w2; g2.ldw = 2048; g2.w_f16 = 1; g2.bias = W.b2;
        if (slabs) {
            g2.C = pSlab; g2.ldc = 512; g2.mode = EPI_SLAB; g2.ksplit = 8; g2.slab_stride = slab_stride;
            gemm_nt(g2, st);
            layernorm_rows_slabs(pSlab, 8, slab_stride, W.b2, pH1, pH, N0, W.n2w, W.n2b, st);
        } else {
            g2.C = pS; g2.ldc = 512; g2.mode = EPI_RESID; g2.res = pH1; g2.ldr = 512;
            gemm_nt(g2, st);
            layernorm_rows(pS, pH, N0, W.n2w, W.n2b, st);
        }
    }
    // logits of the last row (#1785-1788), first-stage sampler on prompts (#1789-1815)
    GemvArgs lg{};
    lg.B = 1; lg.N = 1025; lg.K = 512; lg.src = pH + (size_t)(N0 - 1) * 512; lg.lds = 512;
    lg.W = w_pred; lg.C = logits + (size_t)b * 1025; lg.ldc = 1025; lg.mode = EPI_STORE;
    gemv_f16(lg, st);
    SampleArgs sa = sampler_args(sp, 1);
    sa.logits = logits + (size_t)b * 1025;
    sa.y = y + (size_t)b * tmax; sa.ny = ny + b; sa.seen = seen + (size_t)b * 33;
    sa.done = done + b; sa.stop_out = nullptr; sa.steps = steps + b; sa.kvlen = kvlen + b;
    sa.prefill = 1; sa.logits_out = logits_out; sa.ldlo = 1025;
    sa.b0 = noise_b >= 0 ? noise_b : b;   // Philox counter: the slot's own noise for its first-stage token
                                          // (a prefetch into slot 1 draws slot 0's: it is decoded there)
    sample_tokens(sa, st);
    return hipGetLastError() == hipSuccess ? 0 : set_error(GSV_E_HIP, "prefill launch");
}

// ------------------------------------------------------------ packed prefill
// Prefill of a whole batch as ONE row set: the N0_b = L_b + P_b rows of every
// utterance are packed back to back (row r -> sequence row_seq[r], position
// row_pos[r]), so each layer is one GEMM per weight over sum_b N0_b rows (the
// weights are read once per layer, not once per utterance), the QKV epilogue
// scatters K/V into each sequence's own cache slot, and attention rows see
// their own sequence's keys [0, row_len[r]) with the first-stage prefix-LM mask
// (t2s_first_stage_decoder_fp32.onnx#29-56: x rows see the L x keys, prompt
// row j sees L + j + 1).  Arithmetic per row is the single-sequence path's.
static __global__ void k_gather_rows512(const float* src, const int* rows, float* dst, int n) {
    const int b = blockIdx.x;
    if (b >= n) return;
    const float* s = src + (long)rows[b] * 512;
    for (int i = threadIdx.x; i < 512; i += blockDim.x) dst[(long)b * 512 + i] = s[i];
}

int gsv_engine::ensure_packed(int rows, int B) {
    if (rows <= pk_rows && B <= pk_batch) return 0;
    const int nr = (int)grow_cap(rows, pk_rows), nb = (int)grow_cap(B, pk_batch);
    for (void* p : pk_allocs) retire(p);
    pk_allocs.clear();
    pk_rows = pk_batch = 0;
    reclaim();
    auto A = [&](size_t bytes) -> void* {
        void* p = nullptr;
        if (hipMalloc(&p, (bytes + 255) & ~(size_t)255) != hipSuccess) return nullptr;
        pk_allocs.push_back(p);
        return p;
    };
    pk_H = (float*)A((size_t)nr * 512 * 4);
    pk_Q = (float*)A((size_t)nr * 512 * 4);
    pk_O = (float*)A((size_t)nr * 512 * 4);
    pk_S = (float*)A((size_t)nr * 512 * 4);
    pk_H1 = (float*)A((size_t)nr * 512 * 4);
    pk_F = (float*)A((size_t)nr * 2048 * 4);
    pk_slab = (float*)A((size_t)8 * nr * 512 * 4);
    pk_rowinfo = (int*)A((size_t)3 * nr * 4);
    pk_prompts = (int64_t*)A((size_t)nr * 8);
    pk_last = (int*)A((size_t)nb * 4);
    pk_xlast = (float*)A((size_t)nb * 512 * 4);
    pk_Hh = (__half*)A((size_t)nr * 512 * 2);
    pk_Hl = (__half*)A((size_t)nr * 512 * 2);
    pk_H1h = (__half*)A((size_t)nr * 512 * 2);
    pk_H1l = (__half*)A((size_t)nr * 512 * 2);
    pk_Fh = (__half*)A((size_t)nr * 2048 * 2);
    pk_Fl = (__half*)A((size_t)nr * 2048 * 2);
    if (!pk_H || !pk_F || !pk_slab || !pk_rowinfo || !pk_prompts || !pk_last || !pk_xlast || !pk_Hh || !pk_Hl ||
        !pk_H1h || !pk_H1l || !pk_Fh || !pk_Fl) {
        pk_rows = pk_batch = 0;
        return set_error(GSV_E_HIP, "packed prefill allocation failed");
    }
    pk_rows = nr;
    pk_batch = nb;
    return 0;
}

int gsv_engine::prefill_packed(int B, const gsv_utt* utts, const gsv_sampler* sp, hipStream_t st) {
    std::vector<int> off(B + 1, 0), Ls(B), Ps(B), poff(B + 1, 0);
    for (int b = 0; b < B; ++b) {
        Ls[b] = utts[b].n_ref + utts[b].n_text;
        Ps[b] = utts[b].n_ssl / 2;
        if (Ls[b] <= 0 || Ps[b] <= 0) return set_error(GSV_E_ARG, "empty utterance");
        if (Ls[b] + Ps[b] + 1 > tmax) return set_error(GSV_E_CAPACITY, "prefill exceeds reserved tokens");
        off[b + 1] = off[b] + Ls[b] + Ps[b];
        poff[b + 1] = poff[b] + Ps[b];
    }
    const int R = off[B];
    if (int e = ensure_packed(R, B)) return e;
    // host row tables: sequence, position, visible keys; last row of each sequence
    // tiles of <= TR rows of one sequence for the attention: 128 on the MFMA kernel, else
    // 16 for the LDS-staged f32 kernels
    const bool mfma_attn = attn_mfma_on();
    // the row-per-lane f32 kernel (k_attn_rowlane; GENIE_PACKED_ROWLANE=0: k_attn_flash
    // over 16-row tiles, the same results)
    static const bool rowlane_opt = [] { const char* e = std::getenv("GENIE_PACKED_ROWLANE"); return !(e && std::atoi(e) == 0); }();
    // the same arithmetic on the f32 MFMA (k_attn_mf32; GENIE_PACKED_MF32=0: k_attn_rowlane)
    static const bool mf32_opt = [] { const char* e = std::getenv("GENIE_PACKED_MF32"); return !(e && std::atoi(e) == 0); }();
    const bool mf32 = !mfma_attn && mf32_opt && use_attn_mf32;
    const bool rowlane = !mfma_attn && !mf32 && rowlane_opt;
    const int TR = mfma_attn ? 128 : mf32 ? 32 * MF32_NW : rowlane ? 64 * ROWLANE_NW : 16;
    int ntiles = 0, maxn0 = 0;
    for (int b = 0; b < B; ++b) {
        ntiles += (off[b + 1] - off[b] + TR - 1) / TR;
        maxn0 = std::max(maxn0, off[b + 1] - off[b]);
    }
    pk_host.resize((size_t)3 * R + B + 3 * (size_t)ntiles);
    int* hs = pk_host.data();
    int* hp = hs + R;
    int* hl = hs + 2 * R;
    int* hlast = hs + 3 * R;
    int* htile = hlast + B;
    int ti = 0;
    for (int b = 0; b < B; ++b) {
        for (int j = 0; j < Ls[b] + Ps[b]; ++j) {
            const int r = off[b] + j;
            hs[r] = b;
            hp[r] = j;
            hl[r] = j < Ls[b] ? Ls[b] : j + 1;
        }
        hlast[b] = off[b + 1] - 1;
        for (int r0 = off[b]; r0 < off[b + 1]; r0 += TR, ++ti) {
            htile[3 * ti] = b;
            htile[3 * ti + 1] = r0;
            htile[3 * ti + 2] = std::min(TR, off[b + 1] - r0);
        }
    }
    hipMemcpyAsync(pk_rowinfo, hs, (size_t)3 * R * 4, hipMemcpyHostToDevice, st);
    hipMemcpyAsync(pk_last, hlast, (size_t)B * 4, hipMemcpyHostToDevice, st);
    if (ntiles > pk_tile_cap) {
        const int cap = (int)grow_cap(ntiles, pk_tile_cap);
        retire(pk_tiles);
        pk_tiles = nullptr;
        pk_tile_cap = 0;
        reclaim();
        if (hipMalloc((void**)&pk_tiles, (size_t)3 * cap * 4) != hipSuccess)
            return set_error(GSV_E_HIP, "packed prefill tile table");
        pk_tile_cap = cap;
    }
    hipMemcpyAsync(pk_tiles, htile, (size_t)3 * ntiles * 4, hipMemcpyHostToDevice, st);
    // the LDS-staged tile kernel measured slower here (prefill 62.5 vs 45.4 ms at B=64):
    // kept behind GENIE_PACKED_TILE for A/B
    static const bool tile_opt = [] { const char* e = std::getenv("GENIE_PACKED_TILE"); return e && std::atoi(e); }();
    const bool tiled = !mfma_attn && !mf32 && !rowlane && tile_opt && maxn0 <= ATTN_TILE_MAXK;
    // the online-softmax kernel over the same tiles (GENIE_PACKED_FLASH=0: the per-row kernel)
    static const bool flash_opt = [] { const char* e = std::getenv("GENIE_PACKED_FLASH"); return !(e && std::atoi(e) == 0); }();
    const bool flash_tiles = flash_opt;
    const int* row_seq = pk_rowinfo;
    const int* row_pos = pk_rowinfo + R;
    const int* row_len = pk_rowinfo + 2 * R;
    // encoder per utterance (prompts computed once per distinct ssl_content buffer)
    for (int b = 0; b < B; ++b) {
        const gsv_utt& u = utts[b];
        int64_t* pr = pk_prompts + poff[b];
        int src = -1;
        for (int c = 0; c < b && src < 0; ++c)
            if (utts[c].ssl == u.ssl && utts[c].n_ssl == u.n_ssl) src = c;
        if (int e = encode(&u, pk_H + (size_t)off[b] * 512, pr, st, src < 0)) return e;
        if (src >= 0) hipMemcpyAsync(pr, pk_prompts + poff[src], (size_t)Ps[b] * 8, hipMemcpyDeviceToDevice, st);
        if (timing && b == 0) hipEventRecord(ev[1], st);
        seq_state_init(b, pr, Ps[b], Ls[b], y, tmax, ny, kvlen, steps, done, seen, st);
        audio_embed_prompts(pr, Ps[b], emb_audio, alpha_audio, pe_tab, pk_H + (size_t)(off[b] + Ls[b]) * 512, st);
    }
    const long sstride = (long)16 * tmax * 32;
    const long slab_stride = (long)R * 512;
    const bool slabs = gemm_slabs_supported(512, 512, 512) && gemm_slabs_supported(2048, 2048, 2048);
    // pre-split A (r06): the LayerNorms and FFN1's epilogue write the fp16 hi / lo planes their
    // consumer GEMM would split, where that GEMM runs on the large-M kernel (same values, same
    // MFMA sequence: bit-identical); layer 0's q/k/v reads the encoder's f32 rows
    const bool ps = use_presplit && slabs;
    const bool ps_qkv = ps && gemm_presplit_path(R, 1536, 512, 512);
    const bool ps_ffn1 = ps && gemm_presplit_path(R, 2048, 512, 512);
    const bool ps_ffn2 = ps && gemm_presplit_path(R, 512, 2048, 2048);
    for (int l = 0; l < 24; ++l) {
        const T2SLayerW& W = layers[l];
        GemmArgs g{};
        g.M = R; g.N = 1536; g.K = 512; g.A = pk_H; g.lda = 512;
        g.W = W.w_in; g.ldw = 512; g.w_f16 = 1; g.bias = W.b_in;
        g.C = pk_Q; g.ldc = 512; g.mode = EPI_QKV;
        g.kv.k = kcache[l]; g.kv.v = vcache[l]; g.kv.tmax = tmax; g.kv.seq_stride = sstride;
        g.kv.row_seq = row_seq; g.kv.row_pos = row_pos;
        if (ps_qkv && l > 0) { g.Ah = pk_Hh; g.Al = pk_Hl; }   // written by the previous layer's LN2
        gemm_nt(g, st);
        AttnArgs at{};
        at.q = pk_Q; at.ldq = 512; at.k = kcache[l]; at.v = vcache[l];
        at.seq_stride = sstride; at.tmax = tmax; at.row_len = row_len; at.row_seq = row_seq;
        at.out = pk_O; at.ldo = 512; at.rows = R; at.scale = qk_scale;
        if (mfma_attn) {   // 128-row tiles of one sequence on the split-fp16 MFMA
            at.tiles = pk_tiles;
            at.ntiles = ntiles;
            attn_rows_mfma(at, 128, st);
        } else if (mf32) {   // tiles of 32 MF32_NW rows on the f32 MFMA
            at.tiles = pk_tiles;
            at.ntiles = ntiles;
            attn_rows_mf32(at, st);
        } else if (rowlane) {   // tiles of 64 ROWLANE_NW rows, one row per lane
            at.tiles = pk_tiles;
            at.ntiles = ntiles;
            attn_rows_rowlane(at, st);
        } else if (tiled) {
            at.tiles = pk_tiles;
            at.ntiles = ntiles;
            attn_rows_tiled(at, st);
        } else if (flash_tiles) {   // 16-row tiles of one sequence, K/V staged once per tile
            at.tiles = pk_tiles;
            at.ntiles = ntiles;
            attn_rows_flash_tiled(at, st);
        } else {
            attn_rows(at, st);
        }
        GemmArgs go{};
        go.M = R; go.N = 512; go.K = 512; go.A = pk_O; go.lda = 512;
        go.W = W.w_out; go.ldw = 512; go.w_f16 = 1; go.bias = W.b_out;
        GemmArgs g1{};
        g1.M = R; g1.N = 2048; g1.K = 512; g1.A = pk_H1; g1.lda = 512;
        g1.W = W.w1; g1.ldw = 512; g1.w_f16 = 1; g1.bias = W.b1;
        g1.C = pk_F; g1.ldc = 2048; g1.mode = EPI_RELU;
        GemmArgs g2{};
        g2.M = R; g2.N = 512; g2.K = 2048; g2.A = pk_F; g2.lda = 2048;
        g2.W = W.w2; g2.ldw = 2048; g2.w_f16 = 1; g2.bias = W.b2;
        if (slabs) {
            go.C = pk_slab; go.ldc = 512; go.mode = EPI_SLAB; go.ksplit = 4; go.slab_stride = slab_stride;
            gemm_nt(go, st);
            layernorm_rows_slabs(pk_slab, 4, slab_stride, W.b_out, pk_H, pk_H1, R, W.n1w, W.n1b, st,
                                 ps_ffn1 ? pk_H1h : nullptr, ps_ffn1 ? pk_H1l : nullptr);
            if (ps_ffn1) { g1.Ah = pk_H1h; g1.Al = pk_H1l; }
            if (ps_ffn2) { g1.mode = EPI_RELU_SPLIT; g1.Ch = pk_Fh; g1.Cl = pk_Fl; g1.ldc = 2048; }
            gemm_nt(g1, st);
            g2.C = pk_slab; g2.ldc = 512; g2.mode = EPI_SLAB; g2.ksplit = 8; g2.slab_stride = slab_stride;
            if (ps_ffn2) { g2.Ah = pk_Fh; g2.Al = pk_Fl; }
            gemm_nt(g2, st);
            const bool next_ps = ps_qkv && l < 23;   // the next layer's q/k/v A planes
            layernorm_rows_slabs(pk_slab, 8, slab_stride, W.b2, pk_H1, pk_H, R, W.n2w, W.n2b, st,
                                 next_ps ? pk_Hh : nullptr, next_ps ? pk_Hl : nullptr);
        } else {
            go.C = pk_S; go.ldc = 512; go.mode = EPI_RESID; go.res = pk_H; go.ldr = 512;
            gemm_nt(go, st);
            layernorm_rows(pk_S, pk_H1, R, W.n1w, W.n1b, st);
            gemm_nt(g1, st);
            g2.C = pk_S; g2.ldc = 512; g2.mode = EPI_RESID; g2.res = pk_H1; g2.ldr = 512;
            gemm_nt(g2, st);
            layernorm_rows(pk_S, pk_H, R, W.n2w, W.n2b, st);
        }
    }
    // logits of each sequence's last row (#1785-1788), first-stage sampler (#1789-1815)
    hipLaunchKernelGGL(k_gather_rows512, dim3(B), dim3(256), 0, st, pk_H, pk_last, pk_xlast, B);
    GemmArgs lg{};
    lg.M = B; lg.N = 1025; lg.K = 512; lg.A = pk_xlast; lg.lda = 512; lg.W = w_pred; lg.ldw = 512;
    lg.w_f16 = 1; lg.C = logits; lg.ldc = 1025; lg.mode = EPI_STORE;
    gemm_nt(lg, st);
    SampleArgs sa = sampler_args(sp, B);
    sa.prefill = 1;
    sample_tokens(sa, st);
    return hipGetLastError() == hipSuccess ? 0 : set_error(GSV_E_HIP, "packed prefill launch");
}

SampleArgs gsv_engine::sampler_args(const gsv_sampler* sp, int B) {
    SampleArgs sa{};
    sa.B = B;
    sa.logits = logits; sa.ldl = 1025;
    sa.y = y; sa.ldy = tmax; sa.ny = ny; sa.seen = seen;
    sa.done = done; sa.stop_out = stopf; sa.steps = steps; sa.kvlen = kvlen;
    sa.top_k = sp ? sp->top_k : 15;
    sa.temperature = sp ? sp->temperature : 1.0f;
    sa.rep_penalty = sp ? sp->repetition_penalty : 1.35f;
    sa.greedy = sp ? sp->greedy : 1;
    sa.seed = sp ? sp->seed : 0;
    sa.max_steps = sp ? sp->max_steps : 500;
    sa.force_steps = sp ? sp->force_steps : 0;
    sa.force_b = forceb;
    sa.prefill = 0;
    sa.stop_req = stop_word;
    sa.stop_hit = stop_word + 1;
    return sa;
}

// ------------------------------------------------------------ decode step
void gsv_engine::decode_step(int B, const gsv_sampler* sp, float* logits_out, hipStream_t st) {
    const long sstride = (long)16 * tmax * 32;
    // fixed-point hand-off slices of layer l (fused path): FFN output, attention output
    const bool acc = use_acc && !fuse_qkv && B <= 8 && tmax <= 1024;
    auto accF = [&](int l) { return acc ? acc64 + (long)(2 * l) * 512 : nullptr; };
    auto accA = [&](int l) { return acc ? acc64 + (long)(2 * l + 1) * 512 : nullptr; };
    decode_embed(B, y, tmax, ny, emb_audio, alpha_audio, pe_tab, h, done, st);
    if (B <= 8 && tmax <= 1024) {
        // fused path: 2 launches per layer (QKV+attention+out-proj | FFN1+FFN2)
        for (int l = 0; l < 24; ++l) {
            const T2SLayerW& W = layers[l];
            if (fuse_qkv) {
                QkvAttnArgs qa{};
                qa.B = B;
                if (l == 0) {
                    qa.src = h;
                } else {
                    qa.part = ffn_part; qa.n_part = ffn_slices; qa.part_stride = (long)B * 512;
                    qa.part_bias = layers[l - 1].b2; qa.part_res = h1;
                    qa.ln_g = layers[l - 1].n2w; qa.ln_b = layers[l - 1].n2b; qa.ln_out = h;
                }
                qa.W_in = W.w_in; qa.b_in = W.b_in; qa.k = kcache[l]; qa.v = vcache[l];
                qa.seq_stride = sstride; qa.tmax = tmax; qa.kvlen = kvlen; qa.done = done;
                qa.scale = qk_scale; qa.WoT = W.woT; qa.attn_part = attn_part;
                qkv_attn_outproj(qa, st);
            } else {
                GemvArgs a{};
                a.B = B; a.N = 1536; a.K = 512;
                if (l == 0) {
                    a.src = h; a.lds = 512;
                } else {
                    a.part = ffn_part; a.n_part = ffn_slices; a.part_stride = (long)B * 512;
                    a.part_bias = layers[l - 1].b2; a.part_res = h1;
                    a.ln_g = layers[l - 1].n2w; a.ln_b = layers[l - 1].n2b; a.ln_out = h;
                }
                a.W = W.w_in; a.bias = W.b_in; a.C = q; a.ldc = 512; a.mode = EPI_QKV;
                a.kv.k = kcache[l]; a.kv.v = vcache[l]; a.kv.tmax = tmax; a.kv.row_pos = kvlen;
                a.kv.seq_stride = sstride; a.kv.row_skip = done;
                if (l > 0) { a.acc_in = accF(l - 1); a.acc_bstride = ACC_SEQ; }
                if (l == probe_layer) a.trace = ktrace;
                gemv_f16(a, st);
                AttnOutArgs ao{};
                ao.B = B; ao.q = q; ao.k = kcache[l]; ao.v = vcache[l]; ao.seq_stride = sstride;
                ao.tmax = tmax; ao.kvlen = kvlen; ao.done = done; ao.scale = qk_scale;
                ao.WoT = W.woT; ao.part = attn_part;
                ao.acc_out = accA(l); ao.acc_bstride = ACC_SEQ;
                if (l == probe_layer && ktrace) ao.trace = ktrace + 256 * 8;
                attn_outproj(ao, st);
            }
            FfnArgs fa{};
            fa.B = B; fa.nslices = ffn_slices; fa.h = h; fa.bo = W.b_out; fa.attn_part = attn_part;
            fa.ln_g = W.n1w; fa.ln_b = W.n1b; fa.h1 = h1;
            fa.W1 = W.w1; fa.b1 = W.b1; fa.W2T = W.w2T; fa.part = ffn_part;
            if (!fuse_qkv) { fa.acc_attn = accA(l); fa.acc_out = accF(l); fa.acc_bstride = ACC_SEQ; }
            if (l == probe_layer && ktrace) fa.trace = ktrace + 2 * 256 * 8;
            if (probe_now && l == probe_layer) ffn_fused(fa, st, kev[0], kev[1]);
            else ffn_fused(fa, st);
        }
        GemvArgs lg{};
        lg.B = B; lg.N = 1025; lg.K = 512;
        lg.part = ffn_part; lg.n_part = ffn_slices; lg.part_stride = (long)B * 512;
        lg.part_bias = layers[23].b2; lg.part_res = h1;
        lg.ln_g = layers[23].n2w; lg.ln_b = layers[23].n2b;
        lg.W = w_pred; lg.C = logits; lg.ldc = 1025; lg.mode = EPI_STORE;
        lg.acc_in = accF(23); lg.acc_bstride = ACC_SEQ;
        gemv_f16(lg, st);
    } else {
        // batched path (B > 8): split-fp16 MFMA GEMMs over the B rows with the K
        // dimension split over grid.z into f32 slabs (>= 96 workgroups per GEMM at
        // B = 64 instead of N / 64), each reduction fused into its consumer: the
        // attention prologue sums the QKV slabs (+ bias, K/V row append), the
        // LayerNorms sum the out-projection / FFN2 slabs (+ bias + residual), and
        // FFN2's operand load sums the FFN1 slabs (+ bias, ReLU).  Slab sums run in
        // a fixed order: results do not depend on scheduling.
        const long sq = (long)B * 1536, sf = (long)B * 2048, so = (long)B * 512;
        float* slabA = dslab;                       // QKV slabs, then FFN1 slabs
        float* slabB = dslab + (long)4 * max_batch * 2048;   // out-proj slabs, then FFN2 slabs
        for (int l = 0; l < 24; ++l) {
            const T2SLayerW& W = layers[l];
            GemmArgs g{};
            g.M = B; g.N = 1536; g.K = 512; g.A = h; g.lda = 512;
            g.W = W.w_in; g.ldw = 512; g.w_f16 = 1;
            g.C = slabA; g.ldc = 1536; g.mode = EPI_SLAB; g.ksplit = 4; g.slab_stride = sq;
            gemm_nt(g, st);
            AttnDecArgs at{};
            at.slabs = slabA; at.nslab = 4; at.slab_stride = sq; at.b_in = W.b_in;
            at.k = kcache[l]; at.v = vcache[l]; at.seq_stride = sstride; at.tmax = tmax;
            at.kvlen = kvlen; at.done = done; at.out = o; at.B = B; at.scale = qk_scale;
            attn_decode_slabs(at, st);
            GemmArgs go{};
            go.M = B; go.N = 512; go.K = 512; go.A = o; go.lda = 512; go.W = W.w_out; go.ldw = 512;
            go.w_f16 = 1; go.C = slabB; go.ldc = 512; go.mode = EPI_SLAB; go.ksplit = 4; go.slab_stride = so;
            gemm_nt(go, st);
            layernorm_rows_slabs(slabB, 4, so, W.b_out, h, h1, B, W.n1w, W.n1b, st);
            GemmArgs g1{};
            g1.M = B; g1.N = 2048; g1.K = 512; g1.A = h1; g1.lda = 512; g1.W = W.w1; g1.ldw = 512;
            g1.w_f16 = 1; g1.C = slabA; g1.ldc = 2048; g1.mode = EPI_SLAB; g1.ksplit = 4; g1.slab_stride = sf;
            gemm_nt(g1, st);
            GemmArgs g2{};
            g2.M = B; g2.N = 512; g2.K = 2048; g2.A = slabA; g2.lda = 2048;
            g2.a_nslab = 4; g2.a_slab_stride = sf; g2.a_bias = W.b1; g2.a_relu = 1;
            g2.W = W.w2; g2.ldw = 2048; g2.w_f16 = 1;
            g2.C = slabB; g2.ldc = 512; g2.mode = EPI_SLAB; g2.ksplit = 16; g2.slab_stride = so;
            gemm_nt(g2, st);
            layernorm_rows_slabs(slabB, 16, so, W.b2, h1, h, B, W.n2w, W.n2b, st);
        }
        GemmArgs lg{};
        lg.M = B; lg.N = 1025; lg.K = 512; lg.A = h; lg.lda = 512; lg.W = w_pred; lg.ldw = 512;
        lg.w_f16 = 1; lg.C = logits; lg.ldc = 1025; lg.mode = EPI_STORE;
        gemm_nt(lg, st);
    }
    SampleArgs sa = sampler_args(sp, B);
    sa.logits_out = logits_out; sa.ldlo = 1025;
    if (acc) { sa.acc_zero = acc64; sa.acc_n = ACC_SEQ; }
    sample_tokens(sa, st);
}

hipGraphExec_t gsv_engine::step_graph(int B, const gsv_sampler* sp, int chunk, hipStream_t st) {
    const std::string key = std::to_string(B) + ":" + std::to_string(chunk) + ":" +
                            std::to_string(sp->top_k) + ":" + std::to_string(sp->greedy) + ":" +
                            std::to_string(sp->seed) + ":" + std::to_string(sp->max_steps) + ":" +
                            std::to_string(sp->force_steps) + ":" +
                            std::to_string(sp->temperature) + ":" +
                            std::to_string(sp->repetition_penalty);
    auto it = graphs.find(key);
    if (it != graphs.end()) return it->second;
    hipGraph_t g = nullptr;
    std::shared_lock<std::shared_mutex> cl(gsv::capture_mu);   // no device-synchronising free meanwhile
    if ((graph_err = hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal)) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    for (int i = 0; i < chunk; ++i) decode_step(B, sp, nullptr, st);
    if ((graph_err = hipStreamEndCapture(st, &g)) != hipSuccess) {
        if (g) hipGraphDestroy(g);
        // an invalidated capture can leave the stream in capture mode: end it, or every later
        // launch on the stream fails with hipErrorStreamCaptureInvalidated (r05k)
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        if (hipStreamIsCapturing(st, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone) {
            hipGraph_t g2 = nullptr;
            hipStreamEndCapture(st, &g2);
            if (g2) hipGraphDestroy(g2);
        }
        (void)hipGetLastError();
        return nullptr;
    }
    hipGraphExec_t ex = nullptr;
    if ((graph_err = hipGraphInstantiate(&ex, g, nullptr, nullptr, 0)) != hipSuccess) {
        ex = nullptr;
        (void)hipGetLastError();
    }
    hipGraphDestroy(g);
    if (ex) graphs[key] = ex;
    return ex;
}

int gsv_engine::decode_loop(int B, const gsv_sampler* sp, hipStream_t st, bool allow_persist) {
    // Steps are launched as replayed hipGraphs (chunk of 8 steps, tail by 1-step
    // graphs so forced lengths run no extra step).  The host polls the done flags
    // of chunk k while chunk k+1 already runs, so the GPU never waits on the host.
    const int limit = loop_limit > 0 ? loop_limit : sp->force_steps > 0 ? sp->force_steps : sp->max_steps;
    if (stop_requested()) return stopped_error();
    if (allow_persist && use_persist && persist_family(B) && persist_admit()) return decode_persistent(B, sp, st);
    __atomic_store_n(stop_word + 1, 0, __ATOMIC_RELEASE);   // no kernel of this engine runs: the loops are synchronous
    const int chunk = 8;
    hipGraphExec_t ex8 = step_graph(B, sp, chunk, st);
    hipGraphExec_t ex1 = ex8 ? step_graph(B, sp, 1, st) : nullptr;
    // A capture that fails (another host thread's device-wide synchronisation -- hipFree,
    // hipDeviceSynchronize -- can invalidate it) leaves this loop on eager launches of the
    // same kernels: same results, more launch overhead; the next loop tries to capture again.
    const bool eager = !ex8 || !ex1;
    if (eager) {
        ++graph_fallbacks;
        static const bool log = std::getenv("GENIE_LOG_GRAPH") != nullptr;
        if (log) fprintf(stderr, "[genie] step-graph capture failed (%s): eager decode steps\n", hipGetErrorName(graph_err));
    }
    auto run_steps = [&](hipGraphExec_t ex, int n) -> int {
        if (eager) {
            for (int i = 0; i < n; ++i) decode_step(B, sp, nullptr, st);
            const hipError_t le = hipGetLastError();
            return le == hipSuccess ? 0 : hip_error("decode step launch", le);
        }
        if (const hipError_t ge = hipGraphLaunch(ex, st)) return hip_error("graph launch", ge);
        return 0;
    };
    if (!done_host) {
        if (hipHostMalloc((void**)&done_host, 2 * 64, hipHostMallocDefault) != hipSuccess)
            return set_error(GSV_E_HIP, "pinned alloc");
        for (auto& e : poll_ev) hipEventCreateWithFlags(&e, hipEventDisableTiming);
    }
    int launched = 0, k = 0, checked = 0;
    bool finished = false, probed = false;
    // Live kernel timing: the step after the first chunk runs eagerly (same kernels as the
    // graph) so the probed FFN launch can carry start/stop events -- graph event nodes are
    // not timing events on HIP.  The host is ahead of the GPU then, so the eager launches
    // queue behind the running chunk and execute back to back, as inside the graph.
    bool probe_pending = timing && kev[0] != nullptr;
    while (launched < limit && !finished) {
        if (stop_requested()) break;   // the queued chunks finish their sequences at the sampler
        int n = std::min(chunk, limit - launched);
        if (probe_pending && launched == chunk) {
            n = 1;
            probe_now = true;
            decode_step(B, sp, nullptr, st);
            probe_now = false;
            probe_pending = false;
            probed = true;
        } else if (n == chunk) {
            if (int r = run_steps(ex8, chunk)) return r;
        } else {
            for (int i = 0; i < n; ++i)
                if (int r = run_steps(ex1, 1)) return r;
        }
        launched += n;
        const int slot = k & 1;
        hipMemcpyAsync(done_host + 64 * slot, done, B, hipMemcpyDeviceToHost, st);
        hipEventRecord(poll_ev[slot], st);
        ++k;
        if (k - checked >= 2) {   // inspect the older chunk while the newer one runs
            const int cs = checked & 1;
            if (hipEventSynchronize(poll_ev[cs]) != hipSuccess) return set_error(GSV_E_HIP, "poll");
            bool all = true;
            for (int b = 0; b < B; ++b) all = all && done_host[64 * cs + b];
            ++checked;
            if (all) finished = true;
        }
    }
    if (hipStreamSynchronize(st) != hipSuccess) return set_error(GSV_E_HIP, "decode sync");
    // the word itself, or a sampler that ended sequences on it (the word may be cleared since)
    if (stop_requested() || __atomic_load_n(stop_word + 1, __ATOMIC_ACQUIRE) != 0) return stopped_error();
    if (probed) {
        // one sample per decode loop: the probed step's layer-`probe_layer` FFN launch
        float ms = 0.f;
        const hipError_t e = hipEventElapsedTime(&ms, kev[0], kev[1]);
        if (e == hipSuccess && ms > 0.f) {
            kern_us_sum += ms * 1000.0;
            ++kern_n;
        } else {
            kern_err = e == hipSuccess ? -1 : (int)e;
            (void)hipGetLastError();
        }
    }
    return 0;
}

// B = 1: the single-sequence kernel; B = 2..64: its multi-sequence form (the live
// sequences one after another through each layer's workgroups), faster than the
// per-step graphs at every batch size (tools/batch_sweep.py --compare,
// profiles/r03i_batch_sweep.json).
constexpr int PERSIST1M_MAX_B = 64;
bool gsv_engine::persist_family(int B) const {
    return use_persist1 && decode_cus() >= persist1_grid(3) &&
           (B == 1 || (use_persist1m && B <= std::min(PERSIST1M_MAX_B, persist1m_max_batch())));
}

int gsv_engine::decode_persistent(int B, const gsv_sampler* sp, hipStream_t st) {
    return decode_persistent_as(B, sp, st);
}

// Enqueue one persistent decode launch on st (no host wait): the error word is
// copied to perr_dst and, when res_dst is given, the results of res_b sequences
// (enqueue_results layout) behind it; queued vocoder / prefetch work is launched
// on the vocoder CUs right after the kernel.  one: the single-sequence kernel
// (t2s_persist1.hip) instead of the general one.
int gsv_engine::persist_enqueue(int B, const gsv_sampler* sp, hipStream_t st, int* perr_dst,
                                hipEvent_t k0, hipEvent_t k1, char* res_dst, int res_b) {
    // One launch runs every loop step (t2s_persist1.hip).  Hand-offs are tagged
    // granules in a ring; the launch epoch in the tag makes the ring reusable
    // without zeroing (re-zeroed when the epoch wraps or the layout changes).
    const int limit = loop_limit > 0 ? loop_limit : sp->force_steps > 0 ? sp->force_steps : sp->max_steps;
    if (tmax > PERSIST_TMAX) return set_error(GSV_E_CAPACITY, "persistent decode: tokens exceed 4096");
    // one: the persist1 family (B = 1 single-sequence kernel, B > 1 its multi-sequence form)
    const size_t need = B == 1 ? persist1_ring_bytes() : persist1m_ring_bytes(B);
    const int layout = B == 1 ? -1 : -100 - B;   // ring layout key: the kernels slot the ring differently
    if (need > pws_bytes || layout != pws_batch) {
        if (need > pws_bytes) {
            // sized for the next power-of-two batch (<= 64): a ramp of B re-allocates log2 times
            int pb = 2;
            while (pb < B) pb <<= 1;
            const size_t cap = B == 1 ? need : std::max(need, persist1m_ring_bytes(std::min(pb, 64)));
            retire(pws);
            pws = nullptr;
            pws_bytes = 0;
            reclaim();
            if (hipMalloc(&pws, cap) != hipSuccess) return set_error(GSV_E_HIP, "persistent ring");
            pws_bytes = cap;
        }
        hipMemsetAsync(pws, 0, pws_bytes, st);
        pws_batch = layout;
        pepoch = 0;
    }
    if (++pepoch >= (1u << 20)) {
        hipMemsetAsync(pws, 0, pws_bytes, st);
        pepoch = 1;
    }
    if (!perr && hipMalloc((void**)&perr, 64) != hipSuccess) return set_error(GSV_E_HIP, "error word");
    PersistArgs a{};
    a.B = B;
    // layer groups: as many as the engine stream's CUs hold (all of them unless the
    // vocoder is overlapped on its own CUs)
    a.groups = std::min(persist1_max_groups(), decode_cus() / persist1_grid(1));
    if (const char* e = std::getenv("GENIE_PERSIST_GROUPS")) a.groups = std::max(3, std::min(a.groups, std::atoi(e)));
    for (int l = 0; l < 24; ++l) {
        const T2SLayerW& W = layers[l];
        a.L[l] = PLayer{W.w_in, W.w_out, W.w1, W.w2, W.b_in, W.b_out, W.b1, W.b2, W.n1w, W.n1b, W.n2w, W.n2b};
    }
    a.emb = emb_audio; a.alpha = alpha_audio; a.pe = pe_tab; a.w_pred = w_pred;
    for (int l = 0; l < 24; ++l) { a.kc[l] = kcache[l]; a.vc[l] = vcache[l]; }
    a.sstride = (long)16 * tmax * 32; a.tmax = tmax; a.scale = qk_scale;
    a.y = y; a.ldy = tmax; a.ny = ny; a.kvlen = kvlen; a.steps = steps; a.done = done; a.stop_out = stopf;
    a.seen = seen;
    a.top_k = sp->top_k; a.temperature = sp->temperature; a.rep_penalty = sp->repetition_penalty;
    a.greedy = sp->greedy; a.seed = sp->seed; a.max_steps = sp->max_steps; a.force_steps = sp->force_steps;
    a.force_b = forceb;
    a.ring = (unsigned long long*)pws;
    a.epoch = pepoch;
    a.err = perr;
    a.stop_req = stop_word;
    a.smax = std::max(1, std::min(limit, 4000));
    a.trace = ptrace;
    a.pf_delay = B == 1 ? persist1_pf_delay : 0;   // (the multi-sequence forms: measured only at 0)
    for (int i = 0; i < 4; ++i) a.knob[i] = persist1_knob[i];
    a.fold = ln_fold;
    a.spin_ticks = persist_spin_ticks;
    a.f16_limit = persist1_f16_limit > 0 ? (float)persist1_f16_limit : 65504.f;
    if (!perr_zeroed) hipMemsetAsync(perr, 0, 4, st);   // (a prefetched slot's copy launch zeroes it)
    perr_zeroed = false;
    // a queued prefetch starts once this stream's prefill (same workspaces) is done
    if (pf_queued && !pf_pending) hipEventRecord(pf_fork, st);
    // B >= persistm_min_b: the batched kernel, one group of <= 4 sequences per 16 CUs
    const int pm_groups = std::min({persistm_max_groups(), decode_cus() / persistm_grid(1), B});
    const bool pm = B > 1 && use_persistm && B >= persistm_min_b && pm_groups >= persistm_groups(B);
    if (pm) a.groups = pm_groups;
    const hipError_t le = B == 1 ? decode_persist1(a, st, k0, k1)
                          : pm   ? decode_persistm(a, st, k0, k1)
                                 : decode_persist1m(a, st, k0, k1);
    if (le != hipSuccess)
        return set_error(GSV_E_HIP, "persistent decode launch");
    ++persist_launches;
    hipMemcpyAsync(perr_dst, perr, 4, hipMemcpyDeviceToHost, st);
    if (res_dst) enqueue_results(res_b, st, res_dst);   // valid if this launch succeeds
    // a queued overlapped vocoder call and T2S prefetch: enqueue them now (vocoder
    // CUs, in that order), while the GPU decodes
    if (int r = vits_launch_queued()) return r;
    if (int r = pf_launch_queued()) return r;
    return 0;
}

void gsv_engine::probe_sample(hipEvent_t k0, hipEvent_t k1) {
    float ms = 0.f;
    const hipError_t e = hipEventElapsedTime(&ms, k0, k1);
    if (e == hipSuccess && ms > 0.f) {
        kern_us_sum += ms * 1000.0;
        ++kern_n;
    } else {
        kern_err = e == hipSuccess ? -1 : (int)e;
        (void)hipGetLastError();
    }
}

// A persistent launch whose hand-off outwaited its bound: its grid was not all resident
// (placement, other work on the CUs) and the steps re-run as per-step graphs.  Two in a
// row mean the condition persists: a hold begins -- the next persist_backoff generates
// (or persist_backoff_s seconds, whichever ends first) run on the graphs, then the
// persistent path is probed again.  A probe that times out again starts a hold twice as
// long; a launch that completes ends the back-off.
static double steady_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

void gsv_engine::note_persist_timeout() {
    ++persist_timeouts;
    if (++persist_timeout_run >= 2) {
        const int n = persist_backoff > 0 ? persist_backoff : persist_backoff_base;
        const double sec = persist_backoff_s * n / std::max(1, persist_backoff_base);
        persist_hold = n;
        persist_hold_end = steady_s() + std::min(60.0, sec);
        persist_backoff = std::min(4096, 2 * n);
        ++persist_disabled;
        std::fprintf(stderr,
                     "[genie] persistent decode timed out %d times in a row: per-step graphs for the next %d "
                     "generates (%.1f s at most)\n",
                     persist_timeout_run, n, std::min(60.0, sec));
    }
}

void gsv_engine::note_persist_ok() {
    persist_timeout_run = 0;
    persist_backoff = 0;
}

bool gsv_engine::persist_admit() {
    if (persist_hold <= 0) return true;
    if (--persist_hold <= 0 || steady_s() >= persist_hold_end) {
        persist_hold = 0;   // probe the persistent path again
        return true;
    }
    return false;
}

int gsv_engine::stopped_error() {
    ++stops;
    return set_error(GSV_E_STOPPED, "stopped by gsv_request_stop");
}

int gsv_engine::decode_persistent_as(int B, const gsv_sampler* sp, hipStream_t st) {
    if (!perr_host && hipHostMalloc((void**)&perr_host, 64, hipHostMallocDefault) != hipSuccess)
        return set_error(GSV_E_HIP, "pinned alloc");
    const bool probe = timing && kev[0] != nullptr;
    if (int r = persist_enqueue(B, sp, st, perr_host, probe ? kev[0] : nullptr, probe ? kev[1] : nullptr,
                                res_batch ? res_pin : nullptr, res_batch))
        return r;
    if (const hipError_t we = host_wait(st)) return hip_error("persistent decode sync", we);
    // code 3 (or any code under a pending stop): a stop request abandoned the launch
    if (*perr_host == 3 || (*perr_host != 0 && stop_requested())) return stopped_error();
    // code 2: the kernel met an activation beyond the fp16 range of its split-operand
    // MFMA GEMVs.  It stopped before writing the sequence state back (KV rows and
    // tokens of the partial run are rewritten), so the same steps run again as
    // per-step graphs (t2s_decode.hip: f32 activations on the VALU, no fp16 operand).
    if (*perr_host == 2) {
        ++persist1_f16_reruns;
        return decode_loop(B, sp, st, false);
    }
    // code 1: a hand-off waited past its bound -- the launch's workgroups were not
    // all resident (other work on the device) or stalled.  Every workgroup left
    // before the sequence state was written back, so the same steps run again as
    // per-step graphs, which need no co-residency.
    if (*perr_host == 1) {
        note_persist_timeout();
        return decode_loop(B, sp, st, false);
    }
    if (*perr_host != 0)
        return set_error(GSV_E_HIP, "persistent decode failed (code " + std::to_string(*perr_host) + ")");
    note_persist_ok();
    if (stop_requested()) return stopped_error();
    res_ready = res_batch > 0;
    if (probe) probe_sample(kev[0], kev[1]);
    return 0;
}

// ============================================================ T2S prefetch
// The next utterance of a stream is encoded and prefilled ahead, on the vocoder
// CUs (after the overlapped vocoder call queued before it), into slot 1 while
// slot 0 decodes; the generate it was made for copies slot 1 into slot 0 (KV rows
// [0, N0) of every layer and head + the sequence state, one launch) and decodes
// there, so every decode path keeps working on slot 0 and the tokens are the
// ones the plain path gives (the prefill samples with slot 0's Philox counter).
namespace {
struct SlotCopyArgs {
    float* kc[24];
    float* vc[24];
    long sstride;
    int tmax, n0;
    int64_t* y;
    int *ny, *kvlen, *steps;
    uint8_t* done;
    uint32_t* seen;
    int* forceb;
    int force0;
    int* err;
};
// block (head h, layer l, k|v): rows [0, n0) of the head, contiguous n0 x 32 floats
__global__ __launch_bounds__(256) void k_slot_copy(SlotCopyArgs a) {
    const int h = blockIdx.x, l = blockIdx.y;
    float* base = (blockIdx.z ? a.vc[l] : a.kc[l]) + (long)h * a.tmax * 32;
    const float4* src = reinterpret_cast<const float4*>(base + a.sstride);
    float4* dst = reinterpret_cast<float4*>(base);
    for (int i = threadIdx.x; i < a.n0 * 8; i += 256) dst[i] = src[i];
    if (h == 0 && l == 0 && blockIdx.z == 0) {
        for (int i = threadIdx.x; i < a.tmax; i += 256) a.y[i] = a.y[a.tmax + i];
        if (threadIdx.x < 33) a.seen[threadIdx.x] = a.seen[33 + threadIdx.x];
        if (threadIdx.x == 0) {
            a.ny[0] = a.ny[1];
            a.kvlen[0] = a.kvlen[1];
            a.steps[0] = a.steps[1];
            a.done[0] = a.done[1];
            a.forceb[0] = a.force0;
            if (a.err) a.err[0] = 0;
        }
    }
}

bool same_utt(const gsv_utt& a, const gsv_utt& b) {
    return a.ref_seq == b.ref_seq && a.n_ref == b.n_ref && a.text_seq == b.text_seq && a.n_text == b.n_text &&
           a.ref_bert == b.ref_bert && a.text_bert == b.text_bert && a.ssl == b.ssl && a.n_ssl == b.n_ssl &&
           a.force_steps == b.force_steps;
}
bool same_sampler(const gsv_sampler& a, const gsv_sampler& b) {
    return a.top_k == b.top_k && a.temperature == b.temperature && a.repetition_penalty == b.repetition_penalty &&
           a.greedy == b.greedy && a.seed == b.seed && a.max_steps == b.max_steps && a.force_steps == b.force_steps;
}
// the sampler generate runs with (defaults of the reference graphs)
int norm_sampler(const gsv_sampler* s, gsv_sampler& sp) {
    sp = s ? *s : gsv_sampler{15, 1.0f, 1.35f, 1, 0, 500, 0};
    if (sp.top_k < 1 || sp.top_k > 64) return set_error(GSV_E_ARG, "top_k must be in [1, 64]");
    if (sp.max_steps <= 0) sp.max_steps = 500;
    return 0;
}
}  // namespace

// Launch the queued prefetch into slot 1 (vocoder stream) unless slot 1 still
// holds a launched one that no generate has taken yet.
int gsv_engine::pf_launch_queued() {
    if (!pf_queued || pf_pending) return 0;
    pf_queued = false;
    pf_p = pf_q;
    const gsv_utt& u = pf_p.u;
    const int L = u.n_ref + u.n_text, P = u.n_ssl / 2;
    hipStreamWaitEvent(vstream, pf_in, 0);
    hipStreamWaitEvent(vstream, pf_fork, 0);   // the engine stream's encoder / prefill work (same workspaces)
    if (pf_copied_valid) hipStreamWaitEvent(vstream, pf_copied, 0);   // slot 1 taken by the last generate
    if (timing) hipEventRecord(pf_ev[0], vstream);
    if (int e = encode(&u, pH, prompts_buf, vstream)) return e;
    if (timing) hipEventRecord(pf_ev[1], vstream);
    if (int e = prefill_slot(1, pH, L, prompts_buf, P, &pf_p.sp, nullptr, vstream, 0)) return e;
    if (timing) hipEventRecord(pf_ev[2], vstream);
    hipEventRecord(pf_done, vstream);
    pf_pending = true;
    return 0;
}

// Finish a launched prefetch (it writes the T2S workspaces) and forget a queued
// one (unless keep_queued).
int gsv_engine::pf_drop(bool keep_queued) {
    if (!keep_queued) pf_queued = false;
    if (!pf_pending) return 0;
    pf_pending = false;
    return hipEventSynchronize(pf_done) == hipSuccess ? 0 : set_error(GSV_E_HIP, "T2S prefetch");
}

// Also sets slot 0's forced step count and zeroes the decode error word (two
// stream operations fewer before the decode launch).
void gsv_engine::pf_take(hipStream_t st, int force0) {
    hipStreamWaitEvent(st, pf_done, 0);
    if (!perr && hipMalloc((void**)&perr, 64) != hipSuccess) perr = nullptr;
    SlotCopyArgs a{};
    for (int l = 0; l < 24; ++l) { a.kc[l] = kcache[l]; a.vc[l] = vcache[l]; }
    a.sstride = (long)16 * tmax * 32; a.tmax = tmax; a.n0 = pf_p.n0;
    a.y = y; a.ny = ny; a.kvlen = kvlen; a.steps = steps; a.done = done; a.seen = seen;
    a.forceb = forceb; a.force0 = force0; a.err = perr;
    perr_zeroed = perr != nullptr;
    hipLaunchKernelGGL(k_slot_copy, dim3(16, 24, 2), dim3(256), 0, st, a);
    hipEventRecord(pf_copied, st);
    pf_copied_valid = true;
    pf_pending = false;
}

// ============================================================ host wait
// The host thread waits for a decode by polling the stream (and yielding) rather
// than sleeping in hipStreamSynchronize: the wake-up after a blocking sync costs
// tens of microseconds per utterance (option "spin_wait", default on).
hipError_t gsv_engine::host_wait(hipStream_t st) {
    if (!spin_wait) return hipStreamSynchronize(st);
    for (;;) {
        const hipError_t e = hipStreamQuery(st);
        if (e == hipSuccess) return hipSuccess;
        if (e != hipErrorNotReady) return e;
        std::this_thread::yield();
    }
}

// ============================================================ generate results
int gsv_engine::ensure_res_pin(int batch) {
    const size_t need = (size_t)batch * 8 + (size_t)batch * tmax * 8;
    if (need <= res_pin_bytes) return 0;
    const size_t cap = grow_cap(need, res_pin_bytes);
    retire_host(res_pin);
    res_pin = nullptr;
    res_pin_bytes = 0;
    if (hipHostMalloc((void**)&res_pin, cap, hipHostMallocDefault) != hipSuccess)
        return set_error(GSV_E_HIP, "pinned result buffer");
    res_pin_bytes = cap;
    return 0;
}

// [ny: batch int][steps: batch int][y: batch x tmax int64] -> dst (pinned)
void gsv_engine::enqueue_results(int batch, hipStream_t st, char* dst) {
    int* h = reinterpret_cast<int*>(dst);
    hipMemcpyAsync(h, ny, (size_t)batch * 4, hipMemcpyDeviceToHost, st);
    hipMemcpyAsync(h + batch, steps, (size_t)batch * 4, hipMemcpyDeviceToHost, st);
    hipMemcpyAsync(dst + (size_t)batch * 8, y, (size_t)batch * tmax * 8, hipMemcpyDeviceToHost, st);
}

// Inference.py:108-109 then :41-44 on the copied results: y[:, -idx:] with the last
// token zeroed, cut at the first id >= 1024.
int gsv_engine::trim_results(const char* res, int batch, int64_t* out_tokens, int out_stride, int32_t* out_len) {
    const int* hny = reinterpret_cast<const int*>(res);
    const int* hsteps = hny + batch;
    const int64_t* hy = reinterpret_cast<const int64_t*>(res + (size_t)batch * 8);
    for (int b = 0; b < batch; ++b) {
        const int n = hny[b];
        const int64_t* yy = hy + (size_t)b * tmax;
        const int idx = hsteps[b] - 1;
        const int start = idx > 0 ? n - idx : 0;      // y[:, -idx:] ; idx == 0 -> whole y
        int cnt = n - start;
        for (int i = 0; i < cnt; ++i)
            if ((start + i == n - 1 ? 0 : yy[start + i]) >= 1024) { cnt = i; break; }
        if (cnt > out_stride) return set_error(GSV_E_CAPACITY, "out_stride too small");
        std::memcpy(out_tokens + (size_t)b * out_stride, yy + start, (size_t)cnt * 8);
        if (cnt > 0 && start + cnt == n) out_tokens[(size_t)b * out_stride + cnt - 1] = 0;   // y[0, -1] = 0
        out_len[b] = cnt;
    }
    return 0;
}

// ============================================================ C ABI
#define ENG_CHECK(e) \
    if (!(e)) return set_error(GSV_E_ARG, "null engine")

extern "C" int gsv_engine_create(int device, int version, gsv_engine** out) {
    if (!out) return set_error(GSV_E_ARG, "out is null");
    if (hipSetDevice(device) != hipSuccess) return set_error(GSV_E_HIP, "hipSetDevice failed");
    auto* e = new gsv_engine();
    e->device = device;
    e->version = version;
    if (hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess) {
        delete e;
        return set_error(GSV_E_HIP, "stream create failed");
    }
    e->own_stream = true;
    if (hipHostMalloc((void**)&e->stop_word, 64, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess) {
        hipStreamDestroy(e->stream);
        delete e;
        return set_error(GSV_E_HIP, "stop word alloc failed");
    }
    *e->stop_word = 0;
    for (auto& x : e->ev) hipEventCreate(&x);
    hipEventCreateWithFlags(&e->ev_in, hipEventDisableTiming);
    hipEventCreateWithFlags(&e->ev_out, hipEventDisableTiming);
    *out = e;
    return 0;
}

extern "C" int gsv_engine_destroy(gsv_engine* eng) {
    ENG_CHECK(eng);
    hipSetDevice(eng->device);
    for (auto& t : eng->vb_threads) t.join();   // lane threads of an unfinished async batch
    eng->vb_threads.clear();
    eng->sync_own_streams();   // not a device-wide sync: other engines of the process keep running
    delete eng;
    return 0;
}

extern "C" int gsv_set_weight(gsv_engine* eng, const char* name, const void* host, int dtype,
                              const int64_t* dims, int ndim) {
    ENG_CHECK(eng);
    if (!name || !host || ndim < 0 || (ndim > 0 && !dims)) return set_error(GSV_E_ARG, "bad weight args");
    Staged s;
    size_t n = 1;
    for (int i = 0; i < ndim; ++i) { s.dims.push_back(dims[i]); n *= (size_t)dims[i]; }
    s.data.resize(n);
    if (dtype == GSV_F32) {
        std::memcpy(s.data.data(), host, n * 4);
    } else if (dtype == GSV_F16) {
        const __half* hp = (const __half*)host;
        for (size_t i = 0; i < n; ++i) s.data[i] = __half2float(hp[i]);
    } else {
        return set_error(GSV_E_ARG, "unknown dtype");
    }
    eng->staged[name] = std::move(s);
    return 0;
}

extern "C" int gsv_finalize_weights(gsv_engine* eng) {
    ENG_CHECK(eng);
    hipSetDevice(eng->device);
    if (eng->finalized) return set_error(GSV_E_STATE, "already finalized");
    // the uploads are synchronous null-stream copies: no other thread's capture may run meanwhile
    std::unique_lock<std::shared_mutex> cl(gsv::capture_mu);
    const bool has_hubert = eng->find("feature_extractor.conv_layers.0.conv.weight") != nullptr;
    const bool has_roberta = eng->find("embeddings.word_embeddings.weight") != nullptr;
    const bool has_sv = eng->find("layer3_ds.weight") != nullptr;
    if (!(has_hubert || has_roberta || has_sv) || eng->find("ar_audio_embedding.word_embeddings.weight")) {
        if (int e = eng->finalize_t2s()) return e;
    }
    if (has_hubert) {   // CN-HuBERT (a GenieData model, usually an engine of its own)
        if (int e = eng->finalize_hubert()) return e;
    }
    if (has_roberta) {  // RoBERTa (GenieData, Chinese BERT features)
        if (int e = eng->finalize_roberta()) return e;
    }
    if (has_sv) {       // speaker verification (GenieData speaker_encoder, V2ProPlus sv_emb)
        if (int e = eng->finalize_sv()) return e;
    }
    if (eng->find("vq_model.dec.conv_pre.weight")) {
        if (int e = eng->finalize_vits()) return e;
    }
    if (eng->find("sv_emb.weight")) {
        if (int e = eng->finalize_prompt_encoder()) return e;
    }
    eng->staged.clear();
    eng->finalized = true;
    return 0;
}

extern "C" int gsv_reserve(gsv_engine* eng, int max_batch, int max_tokens) {
    ENG_CHECK(eng);
    hipSetDevice(eng->device);
    if (int e = eng->gen_drain()) return e;   // started generates finish first (results stay queued)
    if (int e = eng->pf_drop()) return e;   // a prefetch writes the T2S workspaces and slot 1
    if (!eng->finalized) return set_error(GSV_E_STATE, "weights not finalized");
    return eng->reserve(max_batch, max_tokens);
}


extern "C" int gsv_t2s_encode(gsv_engine* eng, const gsv_utt* u, float* x, int64_t* prompts,
                              void* stream) {
    ENG_CHECK(eng);
    if (!u || !x || !prompts) return set_error(GSV_E_ARG, "null arg");
    if (!eng->finalized) return set_error(GSV_E_STATE, "weights not finalized");
    hipSetDevice(eng->device);
    if (int e = eng->gen_drain()) return e;
    if (int e = eng->pf_drop()) return e;
    StreamScope sc(eng, stream);
    return eng->encode(u, x, prompts, sc.st());
}

extern "C" int gsv_t2s_prefill(gsv_engine* eng, int seq, const float* x, int32_t n_x,
                               const int64_t* prompts, int32_t n_prompts, const gsv_sampler* s,
                               int64_t* yout, float* logits_out, void* stream) {
    ENG_CHECK(eng);
    hipSetDevice(eng->device);
    if (int e = eng->gen_drain()) return e;   // started generates finish first (results stay queued)
    if (int e = eng->pf_drop()) return e;   // a prefetch writes the T2S workspaces and slot 1
    if (!eng->finalized) return set_error(GSV_E_STATE, "weights not finalized");
    if (seq < 0 || seq >= eng->max_batch) return set_error(GSV_E_CAPACITY, "slot out of range");
    if (s && (s->top_k < 1 || s->top_k > 64)) return set_error(GSV_E_ARG, "top_k must be in [1, 64]");
    StreamScope sc(eng, stream);
    hipStream_t st = sc.st();
    if (int e = eng->prefill_slot(seq, x, n_x, prompts, n_prompts, s, logits_out, st)) return e;
    if (yout)
        hipMemcpyAsync(yout, eng->y + (size_t)seq * eng->tmax, (size_t)(n_prompts + 1) * 8,
                       hipMemcpyDeviceToDevice, st);
    return hipGetLastError() == hipSuccess ? 0 : set_error(GSV_E_HIP, "prefill");
}

// Steps on slot `seq` only: temporarily view the batch as that single slot.
extern "C" int gsv_t2s_decode_steps(gsv_engine* eng, int seq, int nsteps, const gsv_sampler* s,
                                    int64_t* yout, uint8_t* stop, float* logits_out, void* stream) {
    ENG_CHECK(eng);
    hipSetDevice(eng->device);
    if (int e = eng->gen_drain()) return e;   // started generates finish first (results stay queued)
    if (int e = eng->pf_drop()) return e;   // a prefetch writes the T2S workspaces and slot 1
    if (seq != 0) return set_error(GSV_E_ARG, "decode_steps supports slot 0");
    StreamScope sc(eng, stream);
    hipStream_t st = sc.st();
    gsv_sampler sp = s ? *s : gsv_sampler{15, 1.0f, 1.35f, 1, 0, 500, 0};
    if (sp.top_k < 1 || sp.top_k > 64) return set_error(GSV_E_ARG, "top_k must be in [1, 64]");
    sp.force_steps = 1 << 30;   // session semantics: the caller owns the stop decision
    hipMemsetAsync(eng->done, 0, 1, st);
    hipMemsetAsync(eng->forceb, 0, 4, st);
    for (int i = 0; i < nsteps; ++i) {
        eng->decode_step(1, &sp, logits_out ? logits_out + (size_t)i * 1025 : nullptr, st);
        if (stop) hipMemcpyAsync(stop + i, eng->stopf, 1, hipMemcpyDeviceToDevice, st);
    }
    if (yout) {
        int n = 0;
        hipMemcpyAsync(&n, eng->ny, 4, hipMemcpyDeviceToHost, st);
        hipStreamSynchronize(st);
        hipMemcpyAsync(yout, eng->y, (size_t)n * 8, hipMemcpyDeviceToDevice, st);
    }
    return hipGetLastError() == hipSuccess ? 0 : set_error(GSV_E_HIP, "decode_steps");
}

extern "C" int gsv_t2s_read_kv(gsv_engine* eng, int seq, int layer, float* k, float* v, int32_t* n,
                               void* stream) {
    ENG_CHECK(eng);
    hipSetDevice(eng->device);
    if (int e = eng->gen_drain()) return e;   // started generates finish first (results stay queued)
    if (int e = eng->pf_drop()) return e;   // a prefetch writes the T2S workspaces and slot 1
    if (layer < 0 || layer >= 24 || seq < 0 || seq >= eng->max_batch) return set_error(GSV_E_ARG, "range");
    StreamScope sc(eng, stream);
    hipStream_t st = sc.st();
    int len = 0;
    hipMemcpyAsync(&len, eng->kvlen + seq, 4, hipMemcpyDeviceToHost, st);
    hipStreamSynchronize(st);
    if (n) *n = len;
    const long sstride = (long)16 * eng->tmax * 32;
    for (int hh = 0; hh < 16; ++hh) {
        const float* ks = eng->kcache[layer] + seq * sstride + (long)hh * eng->tmax * 32;
        const float* vs = eng->vcache[layer] + seq * sstride + (long)hh * eng->tmax * 32;
        hipMemcpy2DAsync(k + hh * 32, 512 * 4, ks, 32 * 4, 32 * 4, len, hipMemcpyDeviceToDevice, st);
        hipMemcpy2DAsync(v + hh * 32, 512 * 4, vs, 32 * 4, 32 * 4, len, hipMemcpyDeviceToDevice, st);
    }
    return hipStreamSynchronize(st) == hipSuccess ? 0 : set_error(GSV_E_HIP, "read_kv");
}

extern "C" int gsv_t2s_generate(gsv_engine* eng, int batch, const gsv_utt* utts,
                                const gsv_sampler* s, int64_t* out_tokens, int32_t out_stride,
                                int32_t* out_len, void* stream) {
    ENG_CHECK(eng);
    hipSetDevice(eng->device);
    if (!eng->finalized) return set_error(GSV_E_STATE, "weights not finalized");
    if (batch <= 0 || !utts || !out_tokens || !out_len) return set_error(GSV_E_ARG, "bad args");
    gsv_sampler sp;
    if (int e = norm_sampler(s, sp)) return e;
    if (eng->stop_requested()) return eng->stopped_error();   // Inference.py:96-97 at step 0
    if (int e = eng->gen_drain()) return e;   // started generates finish first (results stay queued)
    // prefetched (gsv_t2s_prefetch, launched into slot 1 during the last decode)?  A
    // queued prefetch is for a later call: it stays queued (launched during this
    // decode) unless this is a batch, whose prefill uses slot 1 itself.
    const bool hit = batch == 1 && eng->pf_pending && same_utt(utts[0], eng->pf_p.u) &&
                     same_sampler(sp, eng->pf_p.sp);
    if (!hit)
        if (int e = eng->pf_drop(batch == 1)) return e;
    const int steps_cap = sp.force_steps > 0 ? sp.force_steps : sp.max_steps;
    int need = 0, limit = 0;
    std::vector<int> hforce(batch);
    for (int b = 0; b < batch; ++b) {
        if (utts[b].force_steps < 0) return set_error(GSV_E_ARG, "negative force_steps");
        hforce[b] = utts[b].force_steps;
        const int cap_b = hforce[b] > 0 ? hforce[b] : steps_cap;
        const int n0 = utts[b].n_ref + utts[b].n_text + utts[b].n_ssl / 2;
        need = std::max(need, n0 + cap_b + 16);
        limit = std::max(limit, cap_b);
    }
    if (int e = eng->reserve(batch, need)) return e;
    StreamScope sc(eng, stream);
    hipStream_t st = sc.st();
    if (!hit) hipMemcpyAsync(eng->forceb, hforce.data(), batch * 4, hipMemcpyHostToDevice, st);
    eng->loop_limit = limit;
    if (hit) {   // encoded and prefilled ahead (gsv_t2s_prefetch): slot 1 -> slot 0
        eng->pf_take(st, hforce[0]);
    } else {
    if (eng->timing) hipEventRecord(eng->ev[0], st);
    hipMemsetAsync(eng->done, 1, eng->max_batch, st);
    if (batch > 1 && eng->use_packed) {
        if (int e = eng->prefill_packed(batch, utts, &sp, st)) return e;
    } else {
        for (int b = 0; b < batch; ++b) {
            const gsv_utt& u = utts[b];
            const int L = u.n_ref + u.n_text, P = u.n_ssl / 2;
            if (int e = eng->encode(&u, eng->pH, eng->prompts_buf, st)) return e;
            if (eng->timing && b == 0) hipEventRecord(eng->ev[1], st);
            if (int e = eng->prefill_slot(b, eng->pH, L, eng->prompts_buf, P, &sp, nullptr, st)) return e;
        }
    }
    }
    if (eng->timing) hipEventRecord(eng->ev[2], st);
    if (int e = eng->ensure_res_pin(batch)) return e;
    eng->res_batch = batch;
    eng->res_ready = false;
    // option vocoder_first: the decode waits for the overlapped vocoder batch, so none of that
    // batch's kernels is left pending while the persistent decode holds every CU
    if (eng->vocoder_first && eng->vb_active) eng->vits_batch_order(st);
    const int rc = eng->decode_loop(batch, &sp, st);
    eng->res_batch = 0;
    eng->perr_zeroed = false;
    eng->loop_limit = 0;
    if (rc) return rc;
    if (eng->timing) hipEventRecord(eng->ev[3], st);
    // trim on host (Inference.py:108-109, then :41-44)
    if (!eng->res_ready) {   // not already copied behind a successful persistent launch
        eng->enqueue_results(batch, st, eng->res_pin);
        if (hipStreamSynchronize(st) != hipSuccess) return set_error(GSV_E_HIP, "generate sync");
    } else if (eng->timing && hipEventSynchronize(eng->ev[3]) != hipSuccess) {
        return set_error(GSV_E_HIP, "generate sync");
    }
    if (eng->timing) {   // a prefetched utterance: its encode / prefill phases ran on the vocoder CUs
        hipEventElapsedTime(&eng->ms[0], hit ? eng->pf_ev[0] : eng->ev[0], hit ? eng->pf_ev[1] : eng->ev[1]);
        hipEventElapsedTime(&eng->ms[1], hit ? eng->pf_ev[1] : eng->ev[1], hit ? eng->pf_ev[2] : eng->ev[2]);
        hipEventElapsedTime(&eng->ms[2], eng->ev[2], eng->ev[3]);
    }
    return eng->trim_results(eng->res_pin, batch, out_tokens, out_stride, out_len);
}

// ============================================================ asynchronous generate
int gsv_engine::gen_drain() {
    if (gq_n == 0) return 0;
    return hipStreamSynchronize(stream) == hipSuccess ? 0 : set_error(GSV_E_HIP, "generate drain");
}

int gsv_engine::gen_start(const gsv_utt& u, const gsv_sampler& sp, hipStream_t caller) {
    if (gq_n == 2) return set_error(GSV_E_STATE, "two generates in flight: finish one first");
    if (u.force_steps < 0) return set_error(GSV_E_ARG, "negative force_steps");
    const int L = u.n_ref + u.n_text, P = u.n_ssl / 2;
    if (L <= 0 || P <= 0) return set_error(GSV_E_ARG, "empty utterance");
    const int cap = u.force_steps > 0 ? u.force_steps : sp.force_steps > 0 ? sp.force_steps : sp.max_steps;
    const int need = L + P + cap + 16;
    const bool hit = pf_pending && same_utt(u, pf_p.u) && same_sampler(sp, pf_p.sp);
    if (!hit)
        if (int e = pf_drop(true)) return e;
    if (need > tmax || max_batch < 1) {   // the KV cache is re-allocated: nothing may be in flight
        if (int e = gen_drain()) return e;
        if (int e = pf_drop()) return e;
    }
    if (int e = reserve(1, need)) return e;
    GenSlot& g = gq[(gq_head + gq_n) % 2];
    const size_t rb = 8 + (size_t)tmax * 8;
    if (g.res_bytes < rb) {
        retire_host(g.res);
        g.res = nullptr;
        g.res_bytes = 0;
        if (hipHostMalloc((void**)&g.res, rb, hipHostMallocDefault) != hipSuccess) return set_error(GSV_E_HIP, "pinned results");
        g.res_bytes = rb;
    }
    if (!g.perr_h) {
        if (hipHostMalloc((void**)&g.perr_h, 64, hipHostMallocDefault) != hipSuccess) return set_error(GSV_E_HIP, "pinned alloc");
        for (hipEvent_t* e : {&g.d0, &g.done, &g.k0, &g.k1})
            if (hipEventCreate(e) != hipSuccess) return set_error(GSV_E_HIP, "generate events");
    }
    g.u = u;
    g.sp = sp;
    g.hit = hit;
    g.sync = false;
    g.sync_rc = 0;
    hipStream_t st = stream;
    hipEventRecord(ev_in, caller);   // the caller's inputs are ready here; its stream is NOT made to
    hipStreamWaitEvent(st, ev_in, 0);   // wait for the engine (gen_finish orders it)
    loop_limit = cap;
    if (hit) {
        pf_take(st, u.force_steps);
    } else {
        hipMemsetD32Async(forceb, u.force_steps, 1, st);
        hipMemsetAsync(done, 1, max_batch, st);
        if (timing) hipEventRecord(ev[0], st);
        if (int e = encode(&u, pH, prompts_buf, st)) return e;
        if (timing) hipEventRecord(ev[1], st);
        if (int e = prefill_slot(0, pH, L, prompts_buf, P, &sp, nullptr, st)) return e;
    }
    hipEventRecord(g.d0, st);
    const bool persist_ok = use_persist && use_persist1 && decode_cus() >= persist1_grid(3) && !stop_requested() &&
                            persist_admit();
    int rc = 0;
    if (persist_ok) {
        rc = persist_enqueue(1, &sp, st, g.perr_h, timing ? g.k0 : nullptr, timing ? g.k1 : nullptr, g.res, 1);
    } else {   // no persistent path (or a stop is pending): this one runs to completion now
        res_batch = 1;
        res_ready = false;
        rc = decode_loop(1, &sp, st, false);
        res_batch = 0;
        perr_zeroed = false;
        if (rc == 0) enqueue_results(1, st, g.res);
        *g.perr_h = 0;
        g.sync = true;
        g.sync_rc = rc;
    }
    loop_limit = 0;
    if (rc && !g.sync) return rc;
    hipEventRecord(g.done, st);
    ++gq_n;
    return 0;
}

int gsv_engine::gen_finish(int64_t* out_tokens, int out_stride, int32_t* out_len, hipStream_t caller) {
    if (gq_n == 0) return set_error(GSV_E_STATE, "no generate in flight");
    // A vocoder call still queued here had no later generate to launch it behind (the
    // last sentences of a stream): launch it on the vocoder CUs now, beside the decode
    // this call waits for, instead of after it on the T2S CUs.
    if (vqueued && vstream)
        if (int r = vits_launch_queued(vstream)) return r;
    GenSlot& g = gq[gq_head];
    gq_head = (gq_head + 1) % 2;
    --gq_n;
    if (g.sync && g.sync_rc) return g.sync_rc == GSV_E_STOPPED ? set_error(GSV_E_STOPPED, "stopped by gsv_request_stop")
                                                               : g.sync_rc;
    for (;;) {   // poll, as host_wait
        const hipError_t e = hipEventQuery(g.done);
        if (e == hipSuccess) break;
        if (e != hipErrorNotReady) return set_error(GSV_E_HIP, "generate");
        if (spin_wait) std::this_thread::yield();
        else if (hipEventSynchronize(g.done) != hipSuccess) return set_error(GSV_E_HIP, "generate");
    }
    if (!g.sync && (*g.perr_h == 3 || stop_requested())) return stopped_error();
    if (!g.sync && *g.perr_h == 0) note_persist_ok();
    if (*g.perr_h != 0) {
        // the launch met an fp16-range activation (2) or a hand-off timeout (1): the
        // sequence state was not written back; drain and run this utterance again on
        // the synchronous path, which handles both (its own prefill, slot 0)
        if (*g.perr_h == 2) ++persist1_f16_reruns;
        else if (*g.perr_h == 1) note_persist_timeout();
        if (int e = gen_drain()) return e;
        const int saved_n = gq_n;
        gq_n = 0;   // the synchronous path must not see the queue
        const int r = gsv_t2s_generate(this, 1, &g.u, &g.sp, out_tokens, out_stride, out_len, caller);
        gq_n = saved_n;
        return r;
    }
    if (timing) {
        if (g.hit) {
            hipEventElapsedTime(&ms[0], pf_ev[0], pf_ev[1]);
            hipEventElapsedTime(&ms[1], pf_ev[1], pf_ev[2]);
        } else {
            hipEventElapsedTime(&ms[0], ev[0], ev[1]);
            hipEventElapsedTime(&ms[1], ev[1], g.d0);
        }
        hipEventElapsedTime(&ms[2], g.d0, g.done);
        if (!g.sync) probe_sample(g.k0, g.k1);
    }
    if (caller) hipStreamWaitEvent(caller, g.done, 0);
    return trim_results(g.res, 1, out_tokens, out_stride, out_len);
}

extern "C" int gsv_t2s_generate_start(gsv_engine* eng, const gsv_utt* utt, const gsv_sampler* s, void* stream) {
    ENG_CHECK(eng);
    hipSetDevice(eng->device);
    if (!eng->finalized) return set_error(GSV_E_STATE, "weights not finalized");
    if (!utt) return set_error(GSV_E_ARG, "null utterance");
    gsv_sampler sp;
    if (int e = norm_sampler(s, sp)) return e;
    return eng->gen_start(*utt, sp, (hipStream_t)stream);
}

extern "C" int gsv_t2s_generate_finish(gsv_engine* eng, int64_t* out_tokens, int32_t out_stride, int32_t* out_len,
                                       void* stream) {
    ENG_CHECK(eng);
    hipSetDevice(eng->device);
    if (!out_tokens || !out_len) return set_error(GSV_E_ARG, "null output");
    return eng->gen_finish(out_tokens, out_stride, out_len, (hipStream_t)stream);
}

extern "C" int gsv_t2s_prefetch(gsv_engine* eng, const gsv_utt* utt, const gsv_sampler* s, void* stream) {
    ENG_CHECK(eng);
    hipSetDevice(eng->device);
    if (!eng->finalized) return set_error(GSV_E_STATE, "weights not finalized");
    if (!utt) return set_error(GSV_E_ARG, "null utterance");
    if (!eng->vstream) return set_error(GSV_E_STATE, "T2S prefetch: set option vocoder_cus first");
    if (utt->force_steps < 0) return set_error(GSV_E_ARG, "negative force_steps");
    const int L = utt->n_ref + utt->n_text, P = utt->n_ssl / 2;
    if (L <= 0 || P <= 0) return set_error(GSV_E_ARG, "empty utterance");
    gsv_sampler sp;
    if (int e = norm_sampler(s, sp)) return e;
    const int cap = utt->force_steps > 0 ? utt->force_steps : sp.force_steps > 0 ? sp.force_steps : sp.max_steps;
    const int need = L + P + cap + 16;
    if (eng->max_batch < 2 || need > eng->tmax)   // the KV cache is re-allocated: nothing may be in flight
        if (int e = eng->pf_drop()) return e;
    if (int e = eng->reserve(2, need)) return e;
    if (!eng->pf_in) {
        for (hipEvent_t* e : {&eng->pf_in, &eng->pf_done, &eng->pf_copied, &eng->pf_fork})
            if (hipEventCreateWithFlags(e, hipEventDisableTiming) != hipSuccess) return set_error(GSV_E_HIP, "prefetch events");
        for (hipEvent_t& e : eng->pf_ev)
            if (hipEventCreate(&e) != hipSuccess) return set_error(GSV_E_HIP, "prefetch events");
    }
    hipEventRecord(eng->pf_in, (hipStream_t)stream);   // the inputs are ready in the caller's order here
    eng->pf_q = gsv_engine::Prefetch{*utt, sp, L + P};   // replaces a queued one; a launched one stays
    eng->pf_queued = true;
    return 0;
}

extern "C" int gsv_set_timing(gsv_engine* eng, int enabled) {
    ENG_CHECK(eng);
    eng->timing = enabled != 0;
    if (eng->timing && !eng->kev[0]) {
        hipEventCreate(&eng->kev[0]);
        hipEventCreate(&eng->kev[1]);
    }
    eng->kern_us_sum = 0.0;
    eng->kern_n = 0;
    return 0;
}

extern "C" int gsv_get_kernel_timing(gsv_engine* eng, float* avg_us, int32_t* samples) {
    ENG_CHECK(eng);
    if (avg_us) *avg_us = eng->kern_n ? (float)(eng->kern_us_sum / eng->kern_n) : 0.f;
    if (samples) *samples = eng->kern_n ? eng->kern_n : -eng->kern_err;
    return 0;
}

extern "C" int gsv_get_timing(gsv_engine* eng, float* ms4) {
    ENG_CHECK(eng);
    for (int i = 0; i < 4; ++i) ms4[i] = eng->ms[i];
    return 0;
}

extern "C" int gsv_debug_sample(const float* logits, const uint32_t* seen, int B, const gsv_sampler* s,
                                int step, int64_t* tokens, uint8_t* stop, void* stream) {
    if (!logits || !seen || !s || !tokens || B <= 0 || step < 1) return set_error(GSV_E_ARG, "bad args");
    if (s->top_k < 1 || s->top_k > 64) return set_error(GSV_E_ARG, "top_k must be in [1, 64]");
    hipStream_t st = (hipStream_t)stream;
    // scratch decode state: y[b] (ldy 1), ny = 0, steps = step - 1, done = 0
    char* buf = nullptr;
    const size_t need = (size_t)B * (8 + 4 + 4 + 4 + 1 + 132);
    if (hipMalloc(&buf, need) != hipSuccess) return set_error(GSV_E_HIP, "scratch");
    int64_t* y = (int64_t*)buf;
    int* ny = (int*)(y + B);
    int* steps = ny + B;
    int* kvlen = steps + B;
    uint32_t* seen_c = (uint32_t*)(kvlen + B);
    uint8_t* done = (uint8_t*)(seen_c + 33 * B);
    hipMemsetAsync(buf, 0, need, st);
    hipMemcpyAsync(seen_c, seen, (size_t)B * 33 * 4, hipMemcpyDeviceToDevice, st);
    std::vector<int> hs(B, step - 1);
    hipMemcpyAsync(steps, hs.data(), B * 4, hipMemcpyHostToDevice, st);
    SampleArgs a{};
    a.B = B; a.logits = logits; a.ldl = 1025; a.y = y; a.ldy = 1; a.ny = ny; a.seen = seen_c;
    a.done = done; a.stop_out = stop; a.steps = steps; a.kvlen = kvlen;
    a.top_k = s->top_k; a.temperature = s->temperature; a.rep_penalty = s->repetition_penalty;
    a.greedy = s->greedy; a.seed = s->seed; a.max_steps = 1 << 30; a.force_steps = 0; a.prefill = 0;
    sample_tokens(a, st);
    hipMemcpyAsync(tokens, y, (size_t)B * 8, hipMemcpyDeviceToDevice, st);
    const bool ok = hipStreamSynchronize(st) == hipSuccess;
    hipFree(buf);
    return ok ? 0 : set_error(GSV_E_HIP, "debug sample");
}

extern "C" int gsv_set_option(gsv_engine* eng, const char* name, int value) {
    ENG_CHECK(eng);
    if (!name) return set_error(GSV_E_ARG, "null option name");
    hipSetDevice(eng->device);
    const std::string n(name);
    if (n == "packed") {          // batched generate: one packed prefill over all utterances
        eng->use_packed = value != 0;
    } else if (n == "attn_mf32") {   // prefill attention on the f32 MFMA (0: k_attn_flash; same results)
        eng->use_attn_mf32 = value != 0;
    } else if (n == "persist") {   // also ends a timeout back-off
        eng->use_persist = value != 0;
        eng->persist_hold = 0;
        eng->note_persist_ok();
    } else if (n == "persist_backoff") {   // generates of the first back-off hold (default 64)
        if (value < 1) return set_error(GSV_E_ARG, "persist_backoff: >= 1");
        eng->persist_backoff_base = value;
    } else if (n == "persist_backoff_ms") {   // its time bound (default 5000)
        if (value < 1) return set_error(GSV_E_ARG, "persist_backoff_ms: >= 1");
        eng->persist_backoff_s = value / 1000.0;
    } else if (n == "persist1") {
        eng->use_persist1 = value != 0;
    } else if (n == "persist1m") {   // B = 2..64: the multi-sequence form of persist1 (0: per-step graphs)
        eng->use_persist1m = value != 0;
    } else if (n == "persistm") {    // the batched persistent decode (t2s_persistm.hip) from persistm_min_b on
        eng->use_persistm = value != 0;
    } else if (n == "persistm_min_b") {
        if (value < 2) return set_error(GSV_E_ARG, "persistm_min_b: >= 2");
        eng->persistm_min_b = value;
    } else if (n == "persist_spin_ticks") {   // test hook: bound of a hand-off wait (100 MHz ticks)
        eng->persist_spin_ticks = value > 0 ? (unsigned long long)value : gsv_engine::PERSIST_SPIN_TICKS;
    } else if (n == "persist1_f16_limit") {   // test hook: force the fp16-range fallback
        eng->persist1_f16_limit = value;
    } else if (n == "pf_delay") {   // single-sequence decode: s_sleep(32) ticks before the next-layer prefetch
        eng->persist1_pf_delay = std::max(0, value);
    } else if (n.size() == 5 && n.compare(0, 4, "knob") == 0 && n[4] >= '0' && n[4] <= '3') {
        eng->persist1_knob[n[4] - '0'] = value;   // single-sequence decode tuning variant (0 = default)
    } else if (n == "vits_lanes") {   // concurrent vocoder streams of gsv_vits_decode_batch
        if (value < 1 || value > 16) return set_error(GSV_E_ARG, "vits_lanes: 1..16");
        eng->vits_lanes = value;
    } else if (n == "gemm_presplit") {   // the packed prefill's large GEMMs on pre-split A (same results)
        eng->use_presplit = value != 0;
    } else if (n == "convh_persist") {
        eng->convh_persist = value != 0;
    } else if (n == "convh_ws") {   // 0 off, 1 every batched generator pass, 2 (default) a batch vocoded alone
        eng->convh_ws = std::max(0, std::min(2, value));
    } else if (n == "vits_fork") {
        eng->vits_fork = value != 0;
    } else if (n == "vocoder_first") {
        eng->vocoder_first = value != 0;
    } else if (n == "lanes_all_cus") {
        if (int r = eng->vits_batch_finish(nullptr)) return r;
        eng->sync_own_streams();
        eng->lanes_all_cus = value != 0;
        if (int r = eng->remake_lane_streams()) return r;
    } else if (n == "lane_priority" || n == "t2s_priority") {
        // HIP stream priorities (lower = served first): the overlapped batch vocoder's lanes
        // beside the T2S of the next batch on the engine stream
        int least = 0, greatest = 0;
        hipDeviceGetStreamPriorityRange(&least, &greatest);
        const int p = std::min(std::max(value, std::min(least, greatest)), std::max(least, greatest));
        if (int r = eng->vits_batch_finish(nullptr)) return r;
        if (int r = eng->vits_wait(nullptr)) return r;
        eng->sync_own_streams();
        if (n == "lane_priority") {
            eng->lane_priority = p;
            if (int r = eng->remake_lane_streams()) return r;
        } else {
            if (eng->vocoder_cus || eng->gq_n || !eng->own_stream)
                return set_error(GSV_E_STATE, "t2s_priority: needs the engine's own unmasked stream, idle");
            if (int r = eng->pf_drop()) return r;
            hipStream_t ns = nullptr;
            if (hipStreamCreateWithPriority(&ns, hipStreamNonBlocking, p) != hipSuccess)
                return set_error(GSV_E_HIP, "stream");
            eng->drop_sides();
            hipStreamDestroy(eng->stream);
            eng->stream = ns;
            eng->t2s_priority = p;
        }
    } else if (n == "seg_vocoder") {   // batched vocoder: one generator pass over the batch (0: per-lane passes)
        if (int r = eng->vits_batch_finish(nullptr)) return r;
        eng->seg_vocoder = value != 0;
    } else if (n == "seg_front") {   // ... and its front part packed into one pass too (0: per lane)
        if (int r = eng->vits_batch_finish(nullptr)) return r;
        eng->seg_front_on = value != 0;
    } else if (n == "vits_threads") {   // vocoder lanes issued by one host thread each (default 1)
        eng->vits_threads = value != 0;
    } else if (n == "spin_wait") {   // host waits for a decode by polling the stream (default 1)
        eng->spin_wait = value != 0;
    } else if (n == "decode_cus" || n == "decode_cu_offset") {   // see gsv_engine::decode_cus
        if (value < 0) return set_error(GSV_E_ARG, n + ": >= 0");
        const int save_d = eng->dec_cus_opt, save_o = eng->dec_cu_off;
        (n == "decode_cus" ? eng->dec_cus_opt : eng->dec_cu_off) = value;
        if (eng->vocoder_cus)
            if (int r = eng->set_vocoder_cus(eng->vocoder_cus)) {
                eng->dec_cus_opt = save_d;
                eng->dec_cu_off = save_o;
                return r;
            }
    } else if (n == "vocoder_cus") {   // overlapped vocoder: CUs reserved for gsv_vits_decode_async
        return eng->set_vocoder_cus(value);
    } else if (n == "sv_f16") {   // speaker verification on the split-fp16 MFMA convs (0: the f32 MFMA path)
        eng->sv_f16 = value != 0;
    } else if (n == "sv_f16_limit") {   // tests: force the f32 re-run (0: the fp16 range)
        eng->sv_f16_limit = value > 0 ? (float)value : 65000.f;
    } else if (n == "convh" || n == "convt_f16" || n == "convh_tile" || n == "mrf_fused") {
        // a queued or pending vocoder call finishes under the mode it began with
        if (n == "convh_tile" && (value < 0 || value > 4)) return set_error(GSV_E_ARG, "convh_tile: 0..4");
        if (int r = eng->vits_wait(nullptr)) return r;
        if (int r = eng->vits_batch_finish(nullptr)) return r;
        if (n == "convh") eng->use_convh = value != 0;
        else if (n == "convt_f16") eng->convt_f16 = value != 0;
        else if (n == "mrf_fused") eng->mrf_fused = value != 0;
        else eng->convh_tile = value;
    } else if (n == "ptrace") {
        if (value && !eng->ptrace) {
            if (hipMalloc(&eng->ptrace, (size_t)256 * 16 * 8) != hipSuccess) return set_error(GSV_E_HIP, "ptrace alloc");
            hipMemset(eng->ptrace, 0, (size_t)256 * 16 * 8);
        } else if (!value && eng->ptrace) {
            eng->retire(eng->ptrace);
            eng->ptrace = nullptr;
        }
    } else {
        return set_error(GSV_E_ARG, "unknown option " + n);
    }
    return 0;
}

extern "C" int gsv_request_stop(gsv_engine* eng, int32_t on) {
    ENG_CHECK(eng);
    __atomic_store_n(eng->stop_word, on ? 1 : 0, __ATOMIC_RELEASE);
    return 0;
}

extern "C" int gsv_get_counter(gsv_engine* eng, const char* name, int64_t* value) {
    ENG_CHECK(eng);
    if (!name || !value) return set_error(GSV_E_ARG, "null arg");
    const std::string n(name);
    if (n == "persist_timeouts") *value = eng->persist_timeouts;
    else if (n == "persist1_f16_reruns") *value = eng->persist1_f16_reruns;
    else if (n == "vits_f32_reruns") *value = eng->vits_f32_reruns;
    else if (n == "vits_packed_fronts") *value = eng->vits_packed_fronts;
    else if (n == "sv_f32_reruns") *value = eng->sv_f32_reruns;
    else if (n == "w16_split_tensors") *value = eng->w16_split_tensors;
    else if (n == "persist_disabled") *value = eng->persist_disabled;
    else if (n == "persist_launches") *value = eng->persist_launches;
    else if (n == "persist_hold") *value = eng->persist_hold;
    else if (n == "stops") *value = eng->stops;
    else if (n == "graph_fallbacks") *value = eng->graph_fallbacks;
    else if (n == "retired_bytes") { std::lock_guard<std::mutex> g(eng->alloc_mu); *value = eng->retired_bytes; }
    else if (n == "reclaimed_bytes") *value = eng->reclaimed_bytes;
    else if (n == "reclaims") *value = eng->reclaims;
    else return set_error(GSV_E_ARG, "unknown counter " + n);
    return 0;
}

// The achievable HBM rate on this GPU: a grid-stride copy, 4 x 16 B per thread in
// flight with non-temporal loads / stores, 32 workgroups of 256 threads per CU -- the fastest of the
// shapes swept by tools/hbm_copy_probe.hip (6.04 TB/s of read + write bytes; 4.6-5.6 TB/s for one
// plain 16-B load per thread; the guide quotes 6.29 TB/s).
typedef float hc_f4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void k_hbm_copy(const hc_f4* __restrict__ src, hc_f4* __restrict__ dst, long n) {
    const long stride = (long)gridDim.x * 1024;
    for (long base = (long)blockIdx.x * 1024 + threadIdx.x; base < n; base += stride) {
        hc_f4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (base + 256 * u < n) v[u] = __builtin_nontemporal_load(src + base + 256 * u);
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (base + 256 * u < n) __builtin_nontemporal_store(v[u], dst + base + 256 * u);
    }
}

extern "C" int gsv_debug_hbm_copy(const void* src, void* dst, int64_t bytes, int iters, void* stream, float* ms) {
    if (!src || !dst || !ms || bytes < 16 || iters < 1 || (bytes & 15) ||
        (reinterpret_cast<uintptr_t>(src) & 15) || (reinterpret_cast<uintptr_t>(dst) & 15))
        return set_error(GSV_E_ARG, "hbm copy: 16-B aligned buffers and size, iters >= 1");
    hipStream_t s = (hipStream_t)stream;
    int dev = 0, cus = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const long n = bytes / 16;
    const dim3 grid((unsigned)std::max(1, 32 * cus));
    hipLaunchKernelGGL(k_hbm_copy, grid, dim3(256), 0, s, (const hc_f4*)src, (hc_f4*)dst, n);   // warm
    hipEvent_t e0, e1;
    if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess)
        return set_error(GSV_E_HIP, "hbm copy: event");
    hipEventRecord(e0, s);
    for (int i = 0; i < iters; ++i)
        hipLaunchKernelGGL(k_hbm_copy, grid, dim3(256), 0, s, (const hc_f4*)src, (hc_f4*)dst, n);
    hipEventRecord(e1, s);
    const hipError_t r = hipEventSynchronize(e1);
    float t = 0.f;
    if (r == hipSuccess) hipEventElapsedTime(&t, e0, e1);
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    if (r != hipSuccess || hipGetLastError() != hipSuccess) return set_error(GSV_E_HIP, "hbm copy launch");
    *ms = t / iters;
    return 0;
}

extern "C" int gsv_debug_ptrace(gsv_engine* eng, uint64_t* host, int n) {
    ENG_CHECK(eng);
    if (!eng->ptrace) return set_error(GSV_E_STATE, "enable option ptrace first");
    n = std::min(n, 256 * 16);
    return hipMemcpy(host, eng->ptrace, (size_t)n * 8, hipMemcpyDeviceToHost) == hipSuccess
               ? 0 : set_error(GSV_E_HIP, "ptrace copy");
}

extern "C" int gsv_debug_ktrace(gsv_engine* eng, uint64_t* host, int n) {
    ENG_CHECK(eng);
    if (!eng->ktrace) return set_error(GSV_E_STATE, "set GENIE_KTRACE=1 before gsv_finalize_weights");
    n = std::min(n, 3 * 256 * 8);
    return hipMemcpy(host, eng->ktrace, (size_t)n * 8, hipMemcpyDeviceToHost) == hipSuccess
               ? 0 : set_error(GSV_E_HIP, "ktrace copy");
}
