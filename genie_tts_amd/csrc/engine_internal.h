// Internal engine state (not part of the C ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>

#include <algorithm>
#include <map>
#include <mutex>
#include <shared_mutex>
#include <memory>
#include <thread>
#include <string>
#include <vector>

#include "../../include/genie_engine.h"
#include "kernels.h"
#include "vits.h"

namespace gsv {
int set_error(int code, const std::string& msg);
int hip_error(const std::string& what, hipError_t e);   // GSV_E_HIP, the message naming the HIP error
int f16_inexact_error(const std::string& weight, const float* v, int64_t index);
struct StreamScope;
// Process-wide: every stream capture of the library holds it shared from begin to end; code
// that synchronises the device (hipFree / hipHostFree of retired buffers, weight upload,
// engine teardown) holds it exclusively, so it never invalidates another thread's capture.
extern std::shared_mutex capture_mu;
// Growth policy of run-time buffers: at least `need`, and at least 1.25x the current capacity,
// so a load ramp re-allocates O(log) times instead of once per new maximum.
inline size_t grow_cap(size_t need, size_t cur) { return need <= cur ? cur : std::max(need, cur + cur / 4); }
constexpr long ACC_SEQ = 24 * 2 * 512;   // fixed-point hand-off accumulators per sequence

struct Staged {
    std::vector<int64_t> dims;
    std::vector<float> data;   // host fp32 copy (fp16 inputs upcast exactly)
};

struct T2SLayerW {
    __half *w_in = nullptr, *w_out = nullptr, *w1 = nullptr, *w2 = nullptr;
    __half *woT = nullptr, *w2T = nullptr;   // transposed copies for the fused decode path
    float *b_in = nullptr, *b_out = nullptr, *b1 = nullptr, *b2 = nullptr;
    float *n1w = nullptr, *n1b = nullptr, *n2w = nullptr, *n2b = nullptr;
};
// CN-HuBERT (hubert.hip): chinese-hubert-base, transformers HubertModel layout
struct HubertLayerW {
    W16 wqkv, wo, w1, w2;
    float *bqkv = nullptr, *bo = nullptr, *b1 = nullptr, *b2 = nullptr;
    float *ln1w = nullptr, *ln1b = nullptr, *ln2w = nullptr, *ln2b = nullptr;
};
struct HubertWeights {
    bool ready = false;
    float *conv0_w = nullptr, *gn_w = nullptr, *gn_b = nullptr;
    W16 conv_w[7];                    // conv 1..6 as [co][tap][ci]
    float *fp_ln_w = nullptr, *fp_ln_b = nullptr, *fp_b = nullptr;
    W16 fp_w;
    W16 pos_w;                        // [768][tap 128][ci 48] (16 groups of 48 rows)
    float *pos_b = nullptr, *enc_ln_w = nullptr, *enc_ln_b = nullptr;
    HubertLayerW L[12];
    float* ws = nullptr;              // workspace (grown per call)
    size_t ws_floats = 0;
};
int hubert_frames(int n_samples);
// RoBERTa (bert.hip): chinese-roberta-wwm-ext-large, transformers BertModel layout
using BertLayerW = HubertLayerW;
struct BertWeights {
    bool ready = false;
    float *word = nullptr, *pos = nullptr, *type = nullptr, *ln_w = nullptr, *ln_b = nullptr;
    int vocab = 0, max_pos = 0, n_layers = 0;
    std::vector<BertLayerW> L;        // layers 0 .. n_layers - 3 (hidden_states[-3])
    float* ws = nullptr;
    size_t ws_floats = 0;
};
// Speaker verification (sv.hip): ERes2NetV2 convs, BatchNorm folded, weights [co][tap][ci] f32
struct SvConv {
    float *w = nullptr, *b = nullptr;
    __half *wh = nullptr, *wl = nullptr;   // w split into fp16 hi + lo (null: |w| beyond the fp16 range)
    int cin = 0, cout = 0, k = 1;
};
struct SvBlock {
    SvConv conv1, convs[4], conv3, sc, aff_a[3], aff_b[3];
    int width = 0, stride = 1;
    bool aff = false, has_sc = false;
};
struct SvWeights {
    bool ready = false;
    float *stem_w = nullptr, *stem_b = nullptr;     // conv1 (1 -> 64, 3x3) + bn1 folded
    std::vector<SvBlock> blocks;                     // layer1..4: 3 + 4 + 6 + 3
    SvConv ds34, fuse_a, fuse_b;                     // layer3_ds, fuse34 local_att convs
    float *win = nullptr, *cos_tab = nullptr, *banks = nullptr;   // fbank tables
};
int sv_frames(int n_samples);
}  // namespace gsv

struct gsv_engine {
    int device = 0, version = GSV_V2;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    bool finalized = false;
    std::map<std::string, gsv::Staged> staged;
    std::vector<void*> allocs;        // weights + workspaces (engine lifetime)
    std::mutex alloc_mu;              // guards allocs (vocoder lane threads)
    std::vector<void*> state_allocs;  // decode capacity (re-sized by reserve)
    std::vector<void*> enc_allocs;    // encoder workspace (re-sized by ensure_enc_ws)

    // ---- T2S weights
    __half* emb_audio = nullptr;
    float* alpha_audio = nullptr;
    __half* w_pred = nullptr;
    gsv::T2SLayerW layers[24];
    float *text_emb = nullptr, *bert_w = nullptr, *bert_b = nullptr, *alpha_text = nullptr;
    float *ssl_w = nullptr, *ssl_b = nullptr, *codebook = nullptr, *cb_sumsq = nullptr;
    float* pe_tab = nullptr;
    float* ln_fold = nullptr;         // PersistArgs::fold (the LayerNorm affine folded through W_in / W1)
    int pe_max = 0;
    float qk_scale = 0.f;

    // ---- decode capacity / state
    int max_batch = 0, tmax = 0;
    float *kcache[24] = {}, *vcache[24] = {};
    int64_t* y = nullptr;
    int *ny = nullptr, *kvlen = nullptr, *steps = nullptr, *ident = nullptr;
    uint8_t *done = nullptr, *stopf = nullptr;
    uint32_t* seen = nullptr;
    float* dslab = nullptr;           // batched decode: [2][4][B][2048] split-K slabs
    int* forceb = nullptr;            // per-slot forced loop length (gsv_utt.force_steps; 0 = sampler rule)
    int loop_limit = 0;               // >0: loop-step bound of the current generate (max over its slots)
    float *h = nullptr, *h1 = nullptr, *s1 = nullptr, *s2 = nullptr, *q = nullptr, *o = nullptr;
    float *f = nullptr, *logits = nullptr;
    float *attn_part = nullptr, *ffn_part = nullptr;
    int ffn_slices = 64;
    bool fuse_qkv = false;  // 3 launches/layer measured faster than 2 (GENIE_DECODE_FUSE=2 to A/B)
    float *pH = nullptr, *pQ = nullptr, *pO = nullptr, *pS = nullptr, *pH1 = nullptr, *pF = nullptr;
    int* prow_len = nullptr;
    int64_t* prompts_buf = nullptr;

    // ---- encoder workspace
    int enc_cap_p = 0, enc_cap_l = 0;
    float *e_im2col = nullptr, *e_h = nullptr, *e_hh = nullptr, *e_dist = nullptr;
    float *e_bproj = nullptr, *e_bert = nullptr;

    // ---- VITS
    gsv::VitsWeights vits;
    gsv::VitsWorkspace vws;
    gsv::PromptEncWeights penc;
    gsv::HubertWeights hubert;
    gsv::BertWeights bert;
    gsv::SvWeights sv;
    float* sv_ws = nullptr;           // SV workspace (grown per call)
    size_t sv_ws_n = 0;
    bool sv_f16 = true;               // option "sv_f16": split-fp16 MFMA convs (else f32 MFMA)
    float sv_f16_limit = 65000.f;     // option "sv_f16_limit" (> 0): largest activation the f16 path takes
    int* sv_ovf = nullptr;            // device flag: an activation beyond the fp16 range
    int* sv_ovf_host = nullptr;       // pinned copy
    int sv_f32_reruns = 0;            // SV calls re-run on the f32 path after an overflow

    std::map<std::string, hipGraphExec_t> graphs;
    hipError_t graph_err = hipSuccess;   // the last step-graph capture's failure
    int64_t graph_fallbacks = 0;         // decode loops run eagerly after a failed capture (counter)
    bool timing = false;
    float ms[4] = {0, 0, 0, 0};
    hipEvent_t ev[6] = {};
    hipEvent_t ev_in = nullptr, ev_out = nullptr;
    uint8_t* done_host = nullptr;       // pinned, 2 slots x 64
    // live kernel timing: event pair captured around layer `probe_layer`'s FFN launch
    hipEvent_t kev[2] = {};
    int probe_layer = 12;
    double kern_us_sum = 0.0;
    int kern_n = 0;
    int kern_err = 0;        // last hipEventElapsedTime failure (reported as -samples)
    bool probe_now = false;  // eager step in flight: time the probed FFN launch
    unsigned long long* ktrace = nullptr;
    float* pSlab = nullptr;       // prefill split-K slabs [8][tmax][512]
    long long* acc64 = nullptr;   // per sequence [24 layers][FFN out, attn out][512] fixed-point hand-offs
    bool use_acc = true;          // GENIE_ACC=0: split-K partial slabs instead   // GENIE_KTRACE: phase stamps [3][256][8] of layer probe_layer
    hipEvent_t poll_ev[2] = {};
    // ---- persistent decode (t2s_persist1.hip)
    void* pws = nullptr;               // granule ring
    size_t pws_bytes = 0;
    int pws_batch = 0;                 // batch the ring is laid out for
    unsigned pepoch = 0;               // launch epoch (granule tags)
    int* perr = nullptr;               // device error word
    int* perr_host = nullptr;          // pinned error word
    bool use_persist1 = true;          // GENIE_PERSIST1=0: per-step graphs at every batch size
    bool use_persist1m = true;         // GENIE_PERSIST1M=0: per-step graphs at B = 2..64
    bool use_persistm = true;          // option "persistm" / GENIE_PERSISTM: the batched kernel from persistm_min_b on
    int persistm_min_b = 32;           // option "persistm_min_b" (B = 32: 62.2 vs 65.0 ms per generate, r05t)
    bool use_persist = true;           // GENIE_PERSIST=0: per-step graphs instead
    bool use_convh = true;             // GENIE_CONVH=0: MRF convs on the f32 MFMA path
    bool convt_f16 = true;             // option "convt_f16": the upsample ConvTransposes on the split-fp16 path too
    int convh_tile = 0;                // option "convh_tile": 0 = cost model, 1..4 = force a k_conv_h tile (tests)
    // option "convh_ws": the wide MRF convs weight-stationary (k_conv_ws) -- 0 off, 1 in every batched
    // generator pass, 2 (default) only in a batch the caller waits for (gsv_vits_decode_batch: the
    // vocoder has the GPU; beside the next batch's T2S its LDS-heavy blocks crowd the prefill out, r06p)
    int convh_ws = 2;
    bool vb_alone = false;             // the batch being issued is a synchronous gsv_vits_decode_batch
    bool mrf_fused = true;             // option "mrf_fused": the C <= 32 stages' conv pairs as one kernel
    bool convh_persist = false;        // option "convh_persist": large split-fp16 convs as a persistent tile loop
    int stream_cus(hipStream_t st) const;
    int* vovf = nullptr;               // f16-split conv overflow flag (device)
    int* vovf_host = nullptr;          // pinned copy
    int vits_f32_reruns = 0;           // utterances re-run on the f32 path after an overflow
    long vits_packed_fronts = 0;       // segmented vocoder batches whose front part ran packed
    int n_cu = 0;
    unsigned long long* ptrace = nullptr;   // option "ptrace": persistent phase stamps [256][8]

    ~gsv_engine();
    void* dalloc(size_t bytes);
    void release_all();
    // Buffers replaced while the engine runs are retired, then freed by reclaim(): hipFree /
    // hipHostFree synchronise the device, which invalidates a hipGraph capture running on
    // another thread (another engine of the process) and fails that thread's call
    // (hipErrorStreamCaptureImplicit, gpurun_out/r05k_*.err).  reclaim() frees them under the
    // exclusive capture_mu after this engine's own streams drained; every growth path calls it
    // between retiring the old buffer and allocating the new one, so the footprint stays the
    // live buffers plus one replacement.
    std::vector<void*> retired, retired_host;
    int64_t retired_bytes = 0;         // retired, not yet freed (counter "retired_bytes")
    int64_t reclaimed_bytes = 0;       // freed by reclaim (counter "reclaimed_bytes")
    int64_t reclaims = 0;              // reclaim passes that freed something (counter "reclaims")
    void retire(void* p);
    void retire_host(void* p);
    void reclaim();
    // Waits for this engine's own streams (engine, vocoder, lanes) -- never a device-wide sync.
    hipError_t sync_own_streams();
    const gsv::Staged* find(const std::string& n) const;
    float* up_f32(const std::string& n, int* err);
    __half* up_f16(const std::string& n, int* err);
    __half* up_f16_t(const std::string& n, int* err);   // transposed 2-D upload
    // up_f16 / up_f16_t refuse a tensor that is not fp16-exact (GSV_E_WEIGHT); the W16
    // uploads split such a tensor into hi + lo planes for the split-weight GEMM
    gsv::W16 upload_w16(const std::string& n, const std::vector<float>& v, int* err);
    gsv::W16 up_w16(const std::string& n, int* err);
    long w16_split_tensors = 0;        // tensors uploaded as hi + lo planes (counter "w16_split_tensors")
    int finalize_t2s();
    int finalize_vits();
    int finalize_prompt_encoder();
    int finalize_hubert();
    float* hubert_ws(size_t floats);
    int hubert_forward(const float* audio, int n, float* out, hipStream_t st);
    int finalize_roberta();
    int finalize_sv();
    int sv_conv_upload(const std::string& wname, const std::string& bname, const std::string& bn, gsv::SvConv* c);
    size_t sv_ws_floats(int frames);
    int sv_forward(const float* wav, int n, float* out, hipStream_t st, int* ovf, float lim);
    // RoBERTa over N token rows; rows[n_out]: the token row of each output row.  Packed
    // sentences: row_pos (host [N], position within its sentence) and row_seg (host [N][2],
    // {first row, rows} of its sentence), else one sentence.
    int roberta_forward(const int64_t* ids, int N, const int* rows, int n_out, float* out, hipStream_t st,
                        const int* row_pos = nullptr, const int* row_seg = nullptr);
    int reserve(int batch, int tokens);
    int ensure_enc_ws(int P, int L);
    int encode(const gsv_utt* u, float* x, int64_t* prompts, hipStream_t st, bool do_prompts = true);
    // packed (multi-utterance) prefill
    bool use_packed = true;            // option "packed"
    bool use_attn_mf32 = true;         // option "attn_mf32": prefill attention on k_attn_mf32 (else k_attn_flash)
    int pk_rows = 0, pk_batch = 0;
    std::vector<void*> pk_allocs;
    float *pk_H = nullptr, *pk_Q = nullptr, *pk_O = nullptr, *pk_S = nullptr, *pk_H1 = nullptr, *pk_F = nullptr;
    float *pk_slab = nullptr, *pk_xlast = nullptr;
    // fp16 hi / lo planes of pk_H, pk_H1, pk_F: the A operands of the pre-split large-M GEMMs
    __half *pk_Hh = nullptr, *pk_Hl = nullptr, *pk_H1h = nullptr, *pk_H1l = nullptr, *pk_Fh = nullptr, *pk_Fl = nullptr;
    bool use_presplit = true;          // option "gemm_presplit": the packed prefill's large GEMMs on pre-split A
    int *pk_rowinfo = nullptr, *pk_last = nullptr;
    int64_t* pk_prompts = nullptr;
    int* pk_tiles = nullptr;
    int pk_tile_cap = 0;
    std::vector<int> pk_host;
    int ensure_packed(int rows, int B);
    int prefill_packed(int B, const gsv_utt* utts, const gsv_sampler* sp, hipStream_t st);
    int prefill_slot(int b, const float* x, int L, const int64_t* pr, int P, const gsv_sampler* sp,
                     float* logits_out, hipStream_t st, int noise_b = -1);
    gsv::SampleArgs sampler_args(const gsv_sampler* sp, int B);
    void decode_step(int B, const gsv_sampler* sp, float* logits_out, hipStream_t st);
    hipGraphExec_t step_graph(int B, const gsv_sampler* sp, int chunk, hipStream_t st);
    int decode_loop(int B, const gsv_sampler* sp, hipStream_t st, bool allow_persist = true);
    long persist_timeouts = 0;         // persistent launches that timed out (co-running work) and re-ran as graphs
    int persist_timeout_run = 0;       // consecutive ones (2: a back-off hold on the graphs begins)
    // back-off after repeated timeouts: the next persist_hold generates (or until persist_hold_end,
    // whichever comes first) run on the per-step graphs, then the persistent path is probed again;
    // each hold that ends in another timeout doubles the next one (64 generates / 5 s up to 4096 / 60 s)
    int persist_hold = 0;
    double persist_hold_end = 0.0;     // steady-clock seconds
    int persist_backoff = 0;           // length of the next hold (0: persist_backoff_base)
    int persist_backoff_base = 64;     // option "persist_backoff" (generates; tests shorten it)
    double persist_backoff_s = 5.0;    // option "persist_backoff_ms"
    long persist_disabled = 0;         // holds begun (counter "persist_disabled")
    long persist_launches = 0;         // persistent decode launches enqueued (counter "persist_launches")
    void note_persist_timeout();
    void note_persist_ok();
    bool persist_admit();              // once per generate: false while a hold lasts
    // stop word (gsv_request_stop): host-coherent pinned int, read by the decode kernels
    int* stop_word = nullptr;
    bool stop_requested() const { return stop_word && __atomic_load_n(stop_word, __ATOMIC_ACQUIRE) != 0; }
    long stops = 0;                    // generates abandoned by a stop request (counter "stops")
    int stopped_error();
    // hand-off wait bound, 100 MHz ticks: 200 ms, >100x the longest legitimate wait (a
    // workgroup waiting out one step of a 64-sequence decode, ~1.6 ms)
    static constexpr unsigned long long PERSIST_SPIN_TICKS = 20000000ull;
    unsigned long long persist_spin_ticks = PERSIST_SPIN_TICKS;   // option "persist_spin_ticks" (test hook)
    int decode_persistent(int B, const gsv_sampler* sp, hipStream_t st);
    int decode_persistent_as(int B, const gsv_sampler* sp, hipStream_t st);
    bool persist_family(int B) const;
    // generate's results (ny, steps, y rows) -> pinned host memory, enqueued by the
    // persistent decode before its own sync (one host round trip per generate)
    char* res_pin = nullptr;
    size_t res_pin_bytes = 0;
    int res_batch = 0;                 // > 0: decode_persistent_as enqueues the copies
    bool res_ready = false;            // they were enqueued behind the final decode and synced
    int ensure_res_pin(int batch);
    void enqueue_results(int batch, hipStream_t st, char* dst);
    int trim_results(const char* res, int batch, int64_t* out_tokens, int out_stride, int32_t* out_len);
    int persist_enqueue(int B, const gsv_sampler* sp, hipStream_t st, int* perr_dst, hipEvent_t k0,
                        hipEvent_t k1, char* res_dst, int res_b);
    void probe_sample(hipEvent_t k0, hipEvent_t k1);
    // asynchronous single-utterance generate (gsv_t2s_generate_start / _finish): up to
    // two in flight on the engine stream, so the next decode is queued behind the
    // running one and the GPU never waits for the host between utterances
    struct GenSlot {
        gsv_utt u{};
        gsv_sampler sp{};
        int* perr_h = nullptr;        // pinned error word of this launch
        char* res = nullptr;          // pinned results (enqueue_results layout, batch 1)
        size_t res_bytes = 0;
        hipEvent_t d0 = nullptr, done = nullptr, k0 = nullptr, k1 = nullptr;
        bool hit = false, sync = false;
        int sync_rc = 0;
    };
    GenSlot gq[2];
    int gq_head = 0, gq_n = 0;
    int gen_start(const gsv_utt& u, const gsv_sampler& sp, hipStream_t caller);
    int gen_finish(int64_t* out_tokens, int out_stride, int32_t* out_len, hipStream_t caller);
    int gen_drain();                   // wait for every started generate (their results stay queued)
    long persist1_f16_reruns = 0;      // persistent launches re-run as per-step graphs (fp16 range)
    int persist1_f16_limit = 0;
    // GENIE_PF_DELAY / option pf_delay: s_sleep(32) x N between a B = 1 workgroup's publish and its next-layer
    // refill; 0: 4 was 0.2 % faster alone but equal in the pipelined stream (profiles/r06k_headline_ab.txt)
    int persist1_pf_delay = 0;
    int persist1_knob[4] = {0, 0, 0, 0};   // options "knob0".."knob3": single-sequence kernel tuning variants
    int vits_decode(const int64_t* text_seq, int n_text, const int64_t* sem, int n_sem,
                    const float* ref_audio, int n_audio, const float* ge, const float* ge_adv,
                    const float* eps, uint64_t noise_seed, float noise_scale, float* audio, hipStream_t st);
    int vits_decode_pass(gsv::VitsWorkspace& W, const int64_t* text_seq, int n_text, const int64_t* sem, int n_sem,
                         const float* ref_audio, int n_audio, const float* ge, const float* ge_adv,
                         const float* eps, uint64_t noise_seed, float noise_scale, float* audio, hipStream_t st,
                         int* ovf, bool timed);
    // A segmented batch's front part in one pass (vits_front with fs): the utterances back to
    // back along the frame axis (the generator's layout) and along the text axis, zero gaps.
    struct FrontSeg {
        int n = 0, Tt = 0, St = 0;             // utterances; frame / text columns incl. gaps
        const int* segT = nullptr;             // [Tt] utterance of a frame column, -1 in a gap
        const int* segS = nullptr;             // [St] ... of a text column
        const int* rowT = nullptr;             // [Tt][2] {first frame, frames} of the column's utterance
        const int* rowS = nullptr;             // [St][2] {first text column, length}
        const int* rowX = nullptr;             // [Tt][2] the text keys of a frame (MRTE)
        const int *offT = nullptr, *lenT = nullptr, *offS = nullptr;   // [n]
        const int64_t* const* sems = nullptr;  // [n] device pointers
        const int64_t* const* texts = nullptr;
        const uint64_t* seeds = nullptr;       // [n] Philox keys (0: no noise)
        const float* ge = nullptr;             // [n][gin] flow / dec.cond conditioning
        const float* gem = nullptr;            // [n][512] MRTE vector
        float* gcond = nullptr;                // [n][1536] scratch
    };
    int vits_front(gsv::VitsWorkspace& W, const int64_t* text_seq, int n_text, const int64_t* sem, int n_sem,
                   const float* ref_audio, int n_audio, const float* ge, const float* ge_adv, const float* eps,
                   uint64_t noise_seed, float noise_scale, float* dcond_out, hipStream_t st,
                   const FrontSeg* fs = nullptr);
    int seg_front(hipStream_t st);
    int seg_front_tables(hipStream_t s);   // FrontSeg of vb_items into sgb (host build, one copy)            // the packed front of vb_items (vb_packed) into sgb.z / sgb.dcond
    // segmented vocoder batch (option "seg_vocoder", default 1): every utterance's front part
    // (vits_front) on the lanes, then ONE generator pass over all of them laid out back to
    // back along time with zero gaps (gsv::ConvArgs::seg), on lane 0's stream
    struct SegBatch {
        size_t cap_t = 0;              // frames (rate T) of the buffers
        int cap_n = 0;
        float *z = nullptr, *dcond = nullptr, *audio = nullptr;
        float* g[5] = {};
        int* seg[6] = {};
        int *off = nullptr, *len = nullptr;
        int* ovf = nullptr;
        int* ovf_host = nullptr;
        int* h_pin = nullptr;          // pinned staging of the offset / length tables
        std::vector<int> h_off, h_len;
        int T = 0;                     // frames of the current batch (incl. gaps)
        int St = 0;                    // text columns of the current batch (incl. gaps)
        gsv::VitsWorkspace fw;         // the packed front's buffers (front only, no generator)
        float *ge = nullptr, *gem = nullptr, *gcond = nullptr;   // [cap_n][...] conditioning
        char* tab_dev = nullptr;       // the packed front's tables (FrontSeg), device and pinned
        char* tab_pin = nullptr;
        size_t tab_cap = 0;
        hipEvent_t tab_ev = nullptr;   // after the last table copy
        FrontSeg fs;                   // pointers into tab_dev
        const float* const* ge_ptrs = nullptr;    // [n] the items' ge / MRTE vectors (tab_dev)
        const float* const* gem_ptrs = nullptr;
        hipEvent_t done = nullptr;
        hipStream_t st = nullptr;      // the stream the generator ran on
    } sgb;
    bool seg_vocoder = true;
    bool seg_front_on = true;          // option "seg_front": the front part packed too (one pass)
    bool vb_packed = false;            // the current segmented batch runs the packed front
    static constexpr int SEG_GAP = 4;  // zero frames between utterances (>= every conv halo at rate T)
    int seg_reserve(int n, int T);
    int seg_generate(hipStream_t st, bool f16);
    void seg_copy_out(hipStream_t st);
    // concurrent vocoder lanes (gsv_vits_decode_batch)
    int vits_lanes = 4;                    // option "vits_lanes" (1..16): concurrent vocoder streams;
                                           // 4 = HIP's default hardware queues per process
    struct VitsLane {
        hipStream_t st = nullptr;
        hipEvent_t join = nullptr;
        gsv::VitsWorkspace ws;
    };
    std::vector<VitsLane> vlanes;
    hipEvent_t vfork = nullptr;
    int* vflags = nullptr;
    int* vflags_host = nullptr;
    int vflag_cap = 0;
    int vits_decode_batch(int n, const gsv_vits_item* it, float noise_scale, hipStream_t s);
    // overlapped batch (gsv_vits_decode_batch_async): issued by lane threads that may still
    // run when the call returns; vits_batch_finish joins
    std::vector<gsv_vits_item> vb_items;
    std::vector<std::thread> vb_threads;
    std::vector<int> vb_rcs;
    std::vector<std::string> vb_errs;   // each failed lane thread's error text
    int vb_k = 0;
    bool vb_seg = false;               // the running batch is a segmented one (sgb)
    float vb_scale = 0.f;
    bool vb_active = false;
    int vits_batch_launch(float noise_scale, hipStream_t s, bool join);
    int vits_batch_finish(hipStream_t s);
    bool vocoder_first = false;        // option "vocoder_first": a batched decode waits for the running vocoder batch
    void vits_batch_order(hipStream_t s);   // stream s after the running batch (issuing threads joined)
    bool vits_threads = true;          // option "vits_threads": one host thread per vocoder lane
    int lane_priority = 0;             // option "lane_priority": HIP stream priority of the lanes
    bool lanes_all_cus = false;        // option "lanes_all_cus": batch lanes unmasked under vocoder_cus
    int t2s_priority = 0;              // option "t2s_priority": of the engine stream (vocoder_cus 0)
    hipError_t make_lane_stream(hipStream_t* st);   // on the vocoder CUs under option vocoder_cus
    int remake_lane_streams();
    int vits_read_ms();
    int ref_encode(const float* ref_audio, int n_audio, float* ge, hipStream_t s);
    // overlapped vocoder (option "vocoder_cus"): CU-split streams, one call in flight
    int vocoder_cus = 0;
    // Two streams beside the engine's unmasked stream for a single VITS call (option vits_fork): the
    // front's text branch beside its SSL branch, a generator stage's resblocks 1 and 2 beside
    // resblock 0.  Made on first use; dropped (after a sync) before the engine's streams are destroyed.
    struct SideStream {   // two streams beside `main` (the generator's resblocks 1 and 2; st[0] the front's text branch)
        hipStream_t main = nullptr, st[2] = {nullptr, nullptr};
        hipEvent_t fork = nullptr, join[2] = {nullptr, nullptr};
    };
    std::vector<std::unique_ptr<SideStream>> sides;
    std::mutex side_mu;
    bool vits_fork = true;             // option "vits_fork"
    SideStream* side_of(hipStream_t s);
    void drop_sides();
    hipStream_t vstream = nullptr;     // vocoder: K CUs (the engine stream: the other n_cu - K)
    hipEvent_t vev_in = nullptr, vev_done = nullptr;
    bool vpending = false;             // launched, not yet finished
    bool vqueued = false;              // accepted, launched by the next decode (or vits_wait)
    gsv_vits_item vcall{};
    float vcall_scale = 0.f;
    int set_vocoder_cus(int K);
    int vits_async(const gsv_vits_item& u, float noise_scale, hipStream_t caller);
    int vits_wait(hipStream_t caller);
    int vits_launch_queued(hipStream_t s = nullptr);
    hipStream_t vlast = nullptr;       // stream the pending vocoder call was launched on
    // CUs of the engine (T2S) stream: under vocoder_cus K the mask bits [K + dec_cu_off, +decode_cus())
    // (options "decode_cus" / "decode_cu_offset": several engines, e.g. one per process, can
    // share the vocoder CUs [0, K) while each decodes on CUs of its own)
    int dec_cus_opt = 0, dec_cu_off = 0;
    int decode_cus() const {
        return vocoder_cus == 0 ? n_cu : dec_cus_opt > 0 ? dec_cus_opt : n_cu - vocoder_cus - dec_cu_off;
    }
    // T2S prefetch (gsv_t2s_prefetch): encode + prefill of the next utterance into
    // slot 1 on the vocoder CUs while slot 0 decodes; taken into slot 0 by the
    // generate it was made for
    struct Prefetch {
        gsv_utt u;
        gsv_sampler sp;
        int n0;
    };
    Prefetch pf_q{}, pf_p{};           // queued (launched by the next decode) / launched into slot 1
    bool pf_queued = false, pf_pending = false;
    bool pf_copied_valid = false;      // pf_copied recorded (slot 1 read by the last take)
    hipEvent_t pf_in = nullptr, pf_done = nullptr, pf_copied = nullptr;
    hipEvent_t pf_fork = nullptr;      // engine stream before the decode kernel the prefetch runs beside
    hipEvent_t pf_ev[3] = {};          // timing: encode, prefill, end (vocoder stream)
    int pf_launch_queued();
    int pf_drop(bool keep_queued = false);
    void pf_take(hipStream_t st, int force0);
    bool perr_zeroed = false;          // the next persistent launch's error word was zeroed by pf_take
    bool spin_wait = true;             // option "spin_wait"
    hipError_t host_wait(hipStream_t st);
    int prompt_encode(const float* ref_audio, int n_audio, const float* sv_emb, float* ge,
                      float* ge_adv, hipStream_t st);
};

namespace gsv {
// Orders engine work (always on the engine's own stream, which can be graph-
// captured) after the caller's stream, and the caller's stream after it.
// The caller's stream may be the HIP null stream.
struct StreamScope {
    gsv_engine* e;
    hipStream_t caller;
    StreamScope(gsv_engine* eng, void* s) : e(eng), caller((hipStream_t)s) {
        hipEventRecord(e->ev_in, caller);
        hipStreamWaitEvent(e->stream, e->ev_in, 0);
    }
    ~StreamScope() {
        hipEventRecord(e->ev_out, e->stream);
        hipStreamWaitEvent(caller, e->ev_out, 0);
    }
    hipStream_t st() const { return e->stream; }
};
}  // namespace gsv
