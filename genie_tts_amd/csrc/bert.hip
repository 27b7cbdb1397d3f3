// RoBERTa BERT features for Chinese text (chinese-roberta-wwm-ext-large): the
// reference runs
//   text_bert = model_manager.roberta_model.run(None, {'input_ids', 'attention_mask',
//                                                       'repeats': word2ph})[0]
// (src/genie_tts/GetPhonesAndBert.py:64-74; session ModelManager.py:132-150).
// The graph (RoBERTa.onnx, GenieData) is GPT-SoVITS's get_bert_feature: BertModel
// hidden_states[-3] (the output of layer L - 2 of L), CLS/SEP rows dropped, each
// character's row repeated word2ph[i] times -> [sum(word2ph), 1024].  It is absent
// from this container; the op order follows transformers' BertModel:
//   x = LayerNorm(word[id] + position[t] + token_type[0])            eps 1e-12
//   L - 2 x post-norm layers: MHA (16 x 64) + residual -> LN; FFN 4096 GELU + residual -> LN
// Activations time-major [N][1024]; GEMMs k_gemm_x3 on the f16 MFMA with the f32
// activations split hi + lo and the fp32 weights split hi + lo 2^-11 (W16: three MFMAs
// per product, ~22 significant bits of each weight kept); attention k_mha.
#include "common.h"
#include "engine_internal.h"

#include <algorithm>
#include <numeric>

namespace gsv {
namespace {

// x[t] = LN(word[ids[t]] + pos[p(t)] + type0), D = 1024, one block per token;
// p(t) = row_pos[t] for packed sentences, else t
__global__ __launch_bounds__(256) void k_bert_embed(const int64_t* ids, const float* word, const float* pos,
                                                     const float* type0, const float* g, const float* b, float eps,
                                                     const int* row_pos, float* out) {
    __shared__ float red[16];
    const int t = blockIdx.x;
    const long id = ids[t];
    const long pt = row_pos ? row_pos[t] : t;
    float v[4];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int d = threadIdx.x + 256 * i;
        v[i] = (word[id * 1024 + d] + type0[d]) + pos[pt * 1024 + d];
        s += v[i];
    }
    const float mean = block_sum(s, red) / 1024.f;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) q += (v[i] - mean) * (v[i] - mean);
    const float den = sqrtf(block_sum(q, red) / 1024.f + eps);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int d = threadIdx.x + 256 * i;
        out[(long)t * 1024 + d] = (v[i] - mean) / den * g[d] + b[d];
    }
}

// out[p] = h[rows[p]]  (repeat_interleave of the character rows by word2ph)
__global__ __launch_bounds__(256) void k_bert_repeat(const float* h, const int* rows, float* out) {
    const int p = blockIdx.x;
    const float4* src = reinterpret_cast<const float4*>(h + (long)rows[p] * 1024);
    reinterpret_cast<float4*>(out + (long)p * 1024)[threadIdx.x] = src[threadIdx.x];
}

}  // namespace
}  // namespace gsv

using namespace gsv;

int gsv_engine::finalize_roberta() {
    int err = 0;
    BertWeights& B = bert;
    B.word = up_f32("embeddings.word_embeddings.weight", &err);
    B.pos = up_f32("embeddings.position_embeddings.weight", &err);
    B.type = up_f32("embeddings.token_type_embeddings.weight", &err);
    B.ln_w = up_f32("embeddings.LayerNorm.weight", &err);
    B.ln_b = up_f32("embeddings.LayerNorm.bias", &err);
    if (err) return err;
    if (const Staged* w = find("embeddings.word_embeddings.weight")) B.vocab = (int)w->dims[0];
    if (const Staged* p = find("embeddings.position_embeddings.weight")) B.max_pos = (int)p->dims[0];
    int n = 0;
    while (find("encoder.layer." + std::to_string(n) + ".attention.self.query.weight")) ++n;
    if (n < 3) return set_error(GSV_E_WEIGHT, "RoBERTa: fewer than 3 encoder layers");
    B.n_layers = n;
    B.L.resize(n - 2);   // hidden_states[-3]: only layers 0 .. L-3 are run
    for (int l = 0; l < n - 2; ++l) {
        const std::string p = "encoder.layer." + std::to_string(l) + ".";
        BertLayerW& L = B.L[l];
        // q, k, v fused into one [3072][1024] weight; every projection keeps the
        // initializers' fp32 values (RoBERTa.onnx is fp32, ModelManager.py:139-142):
        // fp16-exact tensors take one plane, others the hi + lo split (W16)
        std::vector<float> wqkv((size_t)3072 * 1024);
        std::vector<float> bqkv(3072);
        const char* nm[3] = {"query", "key", "value"};
        for (int m = 0; m < 3; ++m) {
            const Staged* w = find(p + "attention.self." + nm[m] + ".weight");
            const Staged* b = find(p + "attention.self." + nm[m] + ".bias");
            if (!w || !b || w->data.size() != (size_t)1024 * 1024 || b->data.size() != 1024)
                return set_error(GSV_E_WEIGHT, "missing/bad weight " + p + "attention.self." + nm[m]);
            std::copy(w->data.begin(), w->data.end(), wqkv.begin() + (size_t)m * 1024 * 1024);
            for (int e = 0; e < 1024; ++e) bqkv[m * 1024 + e] = b->data[e];
        }
        L.wqkv = upload_w16(p + "attention.self.{query,key,value}.weight", wqkv, &err);
        L.bqkv = (float*)dalloc(bqkv.size() * 4);
        hipMemcpy(L.bqkv, bqkv.data(), bqkv.size() * 4, hipMemcpyHostToDevice);
        L.wo = up_w16(p + "attention.output.dense.weight", &err);
        L.bo = up_f32(p + "attention.output.dense.bias", &err);
        L.ln1w = up_f32(p + "attention.output.LayerNorm.weight", &err);
        L.ln1b = up_f32(p + "attention.output.LayerNorm.bias", &err);
        L.w1 = up_w16(p + "intermediate.dense.weight", &err);
        L.b1 = up_f32(p + "intermediate.dense.bias", &err);
        L.w2 = up_w16(p + "output.dense.weight", &err);
        L.b2 = up_f32(p + "output.dense.bias", &err);
        L.ln2w = up_f32(p + "output.LayerNorm.weight", &err);
        L.ln2b = up_f32(p + "output.LayerNorm.bias", &err);
    }
    if (err) return err;
    B.ready = true;
    return 0;
}

int gsv_engine::roberta_forward(const int64_t* ids, int N, const int* rows, int n_out, float* out, hipStream_t st,
                                const int* row_pos, const int* row_seg) {
    const BertWeights& B = bert;
    // out-projection / FFN2 of a few rows fill only N / 64 workgroups: K is split into
    // slabs (4 / 8, reduced in slab order by the LayerNorm that follows).  The split does
    // not depend on N, so a packed batch and one call per sentence give identical rows.
    constexpr int zo = 4, z2 = 8, zmax = z2;
    const size_t need = (size_t)N * (1024 * 4 + 3072 + 4096) + (size_t)n_out + 3 * (size_t)N + 64 +
                        (size_t)zmax * N * 1024;
    if (need > bert.ws_floats) {
        const size_t cap = grow_cap(need, bert.ws_floats);
        retire(bert.ws);
        bert.ws = nullptr;
        bert.ws_floats = 0;
        reclaim();
        if (hipMalloc(&bert.ws, cap * 4) != hipSuccess) return set_error(GSV_E_HIP, "RoBERTa workspace");
        bert.ws_floats = cap;
    }
    float* h = bert.ws;
    float *tmp = h + (size_t)N * 1024, *att = tmp + (size_t)N * 1024, *qkv = att + (size_t)N * 1024;
    float* f = qkv + (size_t)N * 3072;
    int* drows = reinterpret_cast<int*>(f + (size_t)N * 4096);
    int* dpos = drows + n_out;
    int* dseg = dpos + N;
    float* slabs = reinterpret_cast<float*>(dseg + 2 * N + 16);   // zmax x [N][1024]
    hipMemcpyAsync(drows, rows, (size_t)n_out * 4, hipMemcpyHostToDevice, st);
    if (row_pos) hipMemcpyAsync(dpos, row_pos, (size_t)N * 4, hipMemcpyHostToDevice, st);
    if (row_seg) hipMemcpyAsync(dseg, row_seg, (size_t)N * 8, hipMemcpyHostToDevice, st);
    constexpr float EPS = 1e-12f;
    hipLaunchKernelGGL(k_bert_embed, dim3(N), dim3(256), 0, st, ids, B.word, B.pos, B.type, B.ln_w, B.ln_b, EPS,
                       row_pos ? dpos : nullptr, h);
    for (const BertLayerW& L : B.L) {
        gemm_nt(gemm_w16(N, 3072, 1024, h, 1024, L.wqkv, L.bqkv, qkv, 3072, EPI_STORE), st);
        MhaArgs m{};
        m.q = qkv; m.q_ts = 3072; m.q_cs = 1;
        m.k = qkv + 1024; m.k_ts = 3072; m.k_cs = 1;
        m.v = qkv + 2048; m.v_ts = 3072; m.v_cs = 1;
        m.out = att; m.o_ts = 1024; m.o_cs = 1;
        m.nq = N; m.nk = N; m.heads = 16; m.dk = 64;
        m.postdiv = 0; m.scale = 8.f;   // scores / sqrt(64) (exact: a power of two)
        m.row_seg = row_seg ? dseg : nullptr;   // packed: each sentence attends within itself
        mha(m, st);
        auto resid_ln = [&](const float* A, int K, const W16& W, const float* bias, int z, const float* lw,
                            const float* lb) {
            if (z > 1) {
                GemmArgs g = gemm_w16(N, 1024, K, A, K, W, nullptr, slabs, 1024, EPI_SLAB);
                g.ksplit = z;
                g.slab_stride = (long)N * 1024;
                gemm_nt(g, st);
                layernorm_rows_d_slabs(slabs, z, (long)N * 1024, bias, h, h, N, 1024, lw, lb, EPS, st);
            } else {
                gemm_nt(gemm_w16(N, 1024, K, A, K, W, bias, tmp, 1024, EPI_RESID, h, 1024), st);
                layernorm_rows_d(tmp, h, N, 1024, lw, lb, EPS, st);
            }
        };
        resid_ln(att, 1024, L.wo, L.bo, zo, L.ln1w, L.ln1b);
        gemm_nt(gemm_w16(N, 4096, 1024, h, 1024, L.w1, L.b1, f, 4096, EPI_GELU), st);
        resid_ln(f, 4096, L.w2, L.b2, z2, L.ln2w, L.ln2b);
    }
    hipLaunchKernelGGL(k_bert_repeat, dim3(n_out), dim3(256), 0, st, h, drows, out);
    // the row tables are read by the kernels above; keep the pageable sources alive until they ran
    if (hipStreamSynchronize(st) != hipSuccess) return set_error(GSV_E_HIP, "RoBERTa");
    return hipGetLastError() == hipSuccess ? 0 : set_error(GSV_E_HIP, "RoBERTa launch");
}

extern "C" int gsv_roberta(gsv_engine* eng, const int64_t* input_ids, const int64_t* attention_mask, int32_t n_tokens,
                           const int64_t* repeats, int32_t n_chars, float* text_bert, void* stream) {
    if (!eng) return set_error(GSV_E_ARG, "null engine");
    if (!input_ids || !text_bert || (n_chars > 0 && !repeats)) return set_error(GSV_E_ARG, "null arg");
    if (!eng->finalized || !eng->bert.ready) return set_error(GSV_E_STATE, "RoBERTa weights not loaded");
    if (n_tokens < 2 || n_tokens > eng->bert.max_pos) return set_error(GSV_E_ARG, "RoBERTa: bad token count");
    if (n_chars < 0 || n_chars > n_tokens - 2) return set_error(GSV_E_ARG, "RoBERTa: more characters than tokens");
    if (attention_mask)
        for (int i = 0; i < n_tokens; ++i)
            if (attention_mask[i] != 1) return set_error(GSV_E_ARG, "RoBERTa: padded batches are not supported");
    std::vector<int> rows;
    for (int i = 0; i < n_chars; ++i) {
        if (repeats[i] < 0) return set_error(GSV_E_ARG, "RoBERTa: negative repeat");
        for (int64_t r = 0; r < repeats[i]; ++r) rows.push_back(1 + i);   // CLS row 0 dropped
    }
    if (rows.empty()) return 0;
    hipSetDevice(eng->device);
    StreamScope sc(eng, stream);
    return eng->roberta_forward(input_ids, n_tokens, rows.data(), (int)rows.size(), text_bert, sc.st());
}

extern "C" int gsv_roberta_batch(gsv_engine* eng, int32_t n_seq, const int64_t* input_ids, const int32_t* n_tokens,
                                 const int64_t* repeats, const int32_t* n_chars, float* text_bert, void* stream) {
    if (!eng) return set_error(GSV_E_ARG, "null engine");
    if (n_seq < 1 || !input_ids || !n_tokens || !n_chars || !text_bert) return set_error(GSV_E_ARG, "null arg");
    if (!eng->finalized || !eng->bert.ready) return set_error(GSV_E_STATE, "RoBERTa weights not loaded");
    std::vector<int> rows, pos, seg;
    int row0 = 0;
    long rep0 = 0;
    for (int s = 0; s < n_seq; ++s) {
        const int nt = n_tokens[s], nc = n_chars[s];
        if (nt < 2 || nt > eng->bert.max_pos) return set_error(GSV_E_ARG, "RoBERTa: bad token count");
        if (nc < 0 || nc > nt - 2) return set_error(GSV_E_ARG, "RoBERTa: more characters than tokens");
        if (nc > 0 && !repeats) return set_error(GSV_E_ARG, "null repeats");
        for (int i = 0; i < nc; ++i) {
            if (repeats[rep0 + i] < 0) return set_error(GSV_E_ARG, "RoBERTa: negative repeat");
            for (int64_t r = 0; r < repeats[rep0 + i]; ++r) rows.push_back(row0 + 1 + i);   // CLS dropped
        }
        for (int t = 0; t < nt; ++t) {
            pos.push_back(t);
            seg.push_back(row0);
            seg.push_back(nt);
        }
        row0 += nt;
        rep0 += nc;
    }
    if (rows.empty()) return 0;
    hipSetDevice(eng->device);
    StreamScope sc(eng, stream);
    return eng->roberta_forward(input_ids, row0, rows.data(), (int)rows.size(), text_bert, sc.st(), pos.data(),
                                seg.data());
}
