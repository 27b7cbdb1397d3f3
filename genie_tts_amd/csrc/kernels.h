// Host-side launchers of the engine's HIP kernels (gfx950).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>
#include <stdint.h>

namespace gsv {

// ------------------------------------------------------------ GEMM (MFMA)
// C(m,n) = epi( sum_k A(m,k) * W(n,k) + bias[n] )   -- fp32 in, fp32 accumulate
//   A(m,k) = A[m*lda + k]            (row-major, fp32)
//   W(n,k) = W[n*ldw + k]            (row-major, fp16 or fp32)
enum EpiMode {
    EPI_STORE = 0,       // C[m*ldc+n] = v
    EPI_RELU = 1,        // C = max(v, 0)
    EPI_RESID = 2,       // C = res[m*ldr+n] + v          (post-norm residual)
    EPI_QKV = 3,         // n<512 -> q[m*512+n]; n<1024 -> K cache; else V cache
    EPI_VQDIST = 4,      // C = (rowsq[m] - v) + colsq[n]   (VQ distance, encoder #30-34)
    EPI_MISH = 5,        // C = v * tanh(softplus(v))        (MelStyleEncoder spectral)
    EPI_SLAB = 6,        // split-K: C + z*slab_stride = raw partial of K slice z (no bias)
    EPI_GELU = 7,        // C = 0.5 v (1 + erf(v / sqrt 2))  (exact GELU, CN-HuBERT)
    EPI_RELU_SPLIT = 8,  // Ch / Cl = the fp16 hi / lo split of max(v, 0) (no f32 C): the A planes of a pre-split GEMM
};

struct KVScatter {
    float* k;            // [heads][tmax][32] for the sequence
    float* v;
    int tmax;
    int pos0;            // cache position of row 0
    const int* row_pos;  // optional per-row positions (batched decode), else pos0 + m
    long seq_stride;     // elements between sequences' caches (batched decode)
    const int* row_seq;  // optional per-row sequence index
    const uint8_t* row_skip; // optional: per-row "done" flags (no cache write)
};

// A GEMM weight as fp16 planes.  fp16-exact tensors (the Genie fp16 bins) have hi only.
// Any other fp32 tensor is split: hi = fp16(w), lo = fp16((w - hi) 2^11), so that lo stays
// a normal fp16 number down to |w| ~ 2^-14 and w = hi + lo 2^-11 to ~22 significant bits.
constexpr float W16_LO_SCALE = 2048.f, W16_LO_INV = 1.f / 2048.f;
struct W16 {
    __half* hi = nullptr;
    __half* lo = nullptr;   // null: the tensor is fp16-exact
    W16 at(size_t e) const { return W16{hi + e, lo ? lo + e : nullptr}; }   // element offset e
};

struct GemmArgs {
    int M, N, K;
    const float* A; long lda;
    const void* W; long ldw; int w_f16;
    const void* Wl;                  // optional lo plane of split fp32 weights (W16), same layout as W
    const float* bias;
    float* C; long ldc;
    int mode;
    const float* res; long ldr;
    const float* rowsq; const float* colsq;
    KVScatter kv;
    int ksplit; long slab_stride;    // EPI_SLAB: K split over grid.z (fp16-weight path only)
    // optional A prologue (fp16-weight path): A(m,k) = relu?(a_bias[k] + sum_z A[z * a_slab_stride + m*lda + k])
    int a_nslab; long a_slab_stride; const float* a_bias; int a_relu;
    // pre-split A (large-M fp16-weight path only, gemm_presplit_path): A's fp16 hi / lo planes
    // (lda elements per row), as the kernels' own split of the f32 values would form them
    const __half* Ah; const __half* Al;
    __half* Ch; __half* Cl;          // EPI_RELU_SPLIT outputs (ldc elements per row)
};
void gemm_nt(const GemmArgs& a, hipStream_t s);
// Args of a GEMM with fp16 weights W[N][K] (ldw = K): C = epi(A W^T + bias)
GemmArgs gemm_f16(int M, int N, int K, const float* A, long lda, const void* W, const float* bias, float* C,
                  long ldc, int mode, const float* res = nullptr, long ldr = 0);
// ... with W16 weights (lo plane, if any, in a.Wl)
GemmArgs gemm_w16(int M, int N, int K, const float* A, long lda, const W16& W, const float* bias, float* C,
                  long ldc, int mode, const float* res = nullptr, long ldr = 0);
// EPI_SLAB (split-K into slabs) is available for fp16 weights with these shapes
bool gemm_slabs_supported(int K, long lda, long ldw);
// shapes the split-weight (W16 with lo) GEMM runs
bool gemm_w16_supported(int K, long lda, long ldw);
// true when gemm_nt runs an fp16-weight GEMM of this shape on the large-M kernel, which also
// takes pre-split A planes (GemmArgs::Ah / Al); K % 128 == 0, lda % 8 == 0 assumed
bool gemm_presplit_path(int M, int N, int K, long lda);

// --------------------------------------------------------- row kernels
void layernorm_rows(const float* in, float* out, int rows, const float* g, const float* b,
                    hipStream_t s);   // D = 512, eps 1e-5
// LayerNorm of res + (bias + sum_z slab[z]) (fixed order) -- the split-K GEMM's reduce
void layernorm_rows_slabs(const float* slabs, int nsplit, long slab_stride, const float* bias,
                          const float* res, float* out, int rows, const float* g, const float* b,
                          hipStream_t s, __half* out_hi = nullptr, __half* out_lo = nullptr);
// LayerNorm over rows of D <= 1024 values with the given eps (CN-HuBERT, RoBERTa)
void layernorm_rows_d(const float* in, float* out, int rows, int D, const float* g, const float* b, float eps,
                      hipStream_t s);
// ... of res + (bias + sum_z slab[z]) (fixed order): the reduce of a split-K EPI_SLAB GEMM
void layernorm_rows_d_slabs(const float* slabs, int nslab, long slab_stride, const float* bias, const float* res,
                            float* out, int rows, int D, const float* g, const float* b, float eps, hipStream_t s);
void sumsq_rows(const float* in, long ld, int rows, int cols, float* out, hipStream_t s);
void argmin_dist_rows(const float* dist, int rows, int cols, int64_t* out, hipStream_t s);

// ------------------------------------------------------------- T2S misc
// x[l] = E_text[seq[l]] + (bias + bproj[l]) + alpha*pe[l+1]   (encoder #57-83)
void text_embed(const int64_t* ref_seq, int n_ref, const int64_t* text_seq, int n_text,
                const float* emb, const float* bproj /*[L,512] or null*/, const float* bias,
                const float* alpha, const float* pe, float* x, hipStream_t s);
// rows [0,P): out[p] = E_audio[tok[p]] + alpha*pe[p+1]; also writes y_emb raw if non-null
void audio_embed_prompts(const int64_t* tok, int P, const __half* emb, const float* alpha,
                         const float* pe, float* out, hipStream_t s);
// im2col for Conv1d(768->768, k2, s2): A[t][ci*2+j] = ssl[ci][2t+j]
void ssl_im2col(const float* ssl, int n_ssl, float* A, hipStream_t s);

// Attention over a cached prefix, one (head, row) per block.
//   q: [rows][512] (unscaled), K/V cache [heads][tmax][32] per sequence
//   len(row) = row < n_full ? n_full : (first_causal + row - n_full + 1) ... given as array
struct AttnArgs {
    const float* q; long ldq;
    const float* k; const float* v;   // cache base of sequence 0
    long seq_stride;                   // elements between sequences
    int tmax;
    const int* row_len;                // keys visible to row r: [0, row_len[r])
    const int* row_seq;                // sequence of row r (or null: 0)
    float* out; long ldo;
    int rows;
    float scale;                       // sqrt(1/sqrt(32)) applied to q and k separately
    const uint8_t* row_skip;
    const int* tiles;                  // packed prefill: [ntiles][3] {seq, row0, nrows<=16}, rows of one seq
    int ntiles;
};
constexpr int ATTN_TILE_MAXK = 448;   // keys a k_attn_tile block stages in LDS
void attn_rows(const AttnArgs& a, hipStream_t s);
// Tiled prefill attention over a.tiles (all rows' keys <= ATTN_TILE_MAXK).
void attn_rows_tiled(const AttnArgs& a, hipStream_t s);
// Packed prefill attention over a.tiles on the online-softmax kernel (any key count).
void attn_rows_flash_tiled(const AttnArgs& a, hipStream_t s);
// Batched decode attention (one block per head x sequence) whose prologue reduces
// the split-K QKV slabs of its head: q/k/v = b_in + sum_z slab[z][b][...] (fixed
// order), appends the new K/V row at position kvlen[b], attends over [0, kvlen[b]].
struct AttnDecArgs {
    const float* slabs; int nslab; long slab_stride;   // [nslab][B][1536]
    const float* b_in;
    float* k; float* v; long seq_stride; int tmax;     // caches (sequence 0 base)
    const int* kvlen; const uint8_t* done;
    float* out;                                        // [B][512]
    int B; float scale;
};
void attn_decode_slabs(const AttnDecArgs& a, hipStream_t s);
// same, with len(row) = row_len[r] + len_add (decode: kvlen + 1)
void attn_rows_plus(const AttnArgs& a, int len_add, hipStream_t s);

// ---------------------------------------------------------- decode GEMV
// Batched (B <= 8) fp16-weight GEMV with optional LayerNorm prologue:
//   xin[b] = ln ? LN(src[b]) : src[b];  if ln_out && block 0: ln_out[b] = xin[b]
//   v = W[n] . xin[b] + bias[n]; epilogue per mode (EPI_STORE/RELU/RESID/QKV)
struct GemvArgs {
    int B, N, K;
    const float* src; long lds;
    // optional split-K partial reduce in the prologue (FFN2 partials of the previous layer):
    //   src[b][k] := part_res[b][k] + (part_bias[k] + sum_j part[j][b][k])
    const float* part; int n_part; long part_stride; const float* part_bias; const float* part_res;
    const float* ln_g; const float* ln_b; float* ln_out;
    const __half* W;
    const float* bias;
    float* C; long ldc;
    int mode;
    const float* res; long ldr;
    KVScatter kv;
    unsigned long long* trace;         // phase stamps [block][8] (GENIE_KTRACE diagnostics)
    // fixed-point accumulator input (replaces part/n_part): src[b][k] :=
    //   part_res[b][k] + (part_bias[k] + acc_in[b * acc_bstride + k] * 2^-32)
    const long long* acc_in; long acc_bstride;
};
void gemv_f16(const GemvArgs& a, hipStream_t s);

// Fused decode attention + out-proj partial, one block per (head, sequence):
//   o_h = softmax((q_h s)(K_h s)^T) V_h over keys [0, kvlen[b] + 1)
//   part[h][b][n] = sum_d WoT[h*32+d][n] * o_h[d]            (n < 512)
struct AttnOutArgs {
    int B;
    const float* q;                        // [B][512]
    const float* k; const float* v; long seq_stride; int tmax;
    const int* kvlen; const uint8_t* done;
    float scale;
    const __half* WoT;                     // [512 in][512 out]
    float* part;                           // [16][B][512]
    unsigned long long* trace;
    long long* acc_out; long acc_bstride;  // if set: fixed-point adds instead of part
};
void attn_outproj(const AttnOutArgs& a, hipStream_t s);

// Fused QKV + attention + out-proj partial, one block per (head, sequence):
//   x = layer input (LN2 of the previous layer's reduced FFN partials, or h0);
//   q,k,v of head h from W_in rows; new k,v appended to the cache at kvlen[b];
//   attention over [0, kvlen] ; part[h][b] = WoT[h-slice]^T o_h.
struct QkvAttnArgs {
    int B;
    const float* src;                              // layer 0: h0 [B][512]
    const float* part; int n_part; long part_stride; const float* part_bias; const float* part_res;
    const float* ln_g; const float* ln_b; float* ln_out;   // ln_out: x for the residual
    const __half* W_in; const float* b_in;
    float* k; float* v; long seq_stride; int tmax;
    const int* kvlen; const uint8_t* done;
    float scale;
    const __half* WoT;
    float* attn_part;                              // [16][B][512]
};
void qkv_attn_outproj(const QkvAttnArgs& a, hipStream_t s);

// Fused FFN, split-K over the 2048 hidden units (one slice per block):
//   s1[b] = h[b] + (bo + sum_h attn_part[h][b]);  x = LN1(s1); block 0 writes h1 = x
//   f = relu(W1[slice] x + b1[slice]);  part[j][b][n] = sum_{r in slice} W2T[r][n] f_r
struct FfnArgs {
    int B, nslices;
    const float* h; const float* bo; const float* attn_part;   // [16][B][512]
    const float* ln_g; const float* ln_b; float* h1;
    const __half* W1; const float* b1; const __half* W2T;      // W2T [2048][512]
    float* part;                                               // [nslices][B][512]
    unsigned long long* trace;
    const long long* acc_attn; long long* acc_out; long acc_bstride;  // fixed-point hand-offs
};
void ffn_fused(const FfnArgs& a, hipStream_t s, hipEvent_t start = nullptr, hipEvent_t stop = nullptr);

// Loop-end rule of K10 + Inference.py:95-106 for sequence b after `st` executed
// steps: a per-sequence forced length, else the launch-wide one, else EOS / 500.
__host__ __device__ __forceinline__ bool seq_finished(const int* force_b, int b, int force_steps, int max_steps,
                                                      int st, bool stop) {
    const int fb = force_b ? force_b[b] : 0;
    const int fs = fb > 0 ? fb : force_steps;
    return fs > 0 ? st >= fs : (stop || st >= max_steps);
}

// Decode embedding: for active b: tok = y[b][ny[b]-1]; h[b] = E[tok] + alpha*pe[ny[b]]
void decode_embed(int B, const int64_t* y, long ldy, const int* ny, const __half* emb,
                  const float* alpha, const float* pe, float* h, const uint8_t* done,
                  hipStream_t s);

struct SampleArgs {
    int B;
    const float* logits; long ldl;     // [B][1025]
    int64_t* y; long ldy; int* ny;     // history, appended on success
    uint32_t* seen;                    // [B][33] presence bitmap (y tokens)
    uint8_t* done; uint8_t* stop_out;  // stop flags out (per b) ; done updated
    int* steps;                        // per-b executed loop steps
    int* kvlen;                        // per-b KV length, +1 per executed step
    int top_k; float temperature; float rep_penalty;
    int greedy; uint64_t seed;
    int max_steps; int force_steps;
    const int* force_b;                // optional per-sequence force_steps (>0 overrides force_steps)
    int prefill;                       // 1: first-stage sampler (no stop, no step count)
    int b0;                            // Philox sequence id of block 0 (prefill of slot b0)
    float* logits_out; long ldlo;      // optional copy of raw logits
    int ablate;                        // probe only: 1 skip top-k, 2 also skip softmax, 3 loads + tail
    long long* acc_zero; long acc_n;   // per-sequence fixed-point accumulators zeroed for the next step
    int threads;                       // 256 (default) or 512: block size of the sampler body
    const int* stop_req;               // host-mapped stop word (gsv_request_stop): set -> the sequence finishes
    int* stop_hit;                     // host-mapped, or null: set to 1 when the stop word ended a sequence, so the
                                       // host reports STOPPED even if the word is cleared before it looks
};
void sample_tokens(const SampleArgs& a, hipStream_t s);

// Decode-state init of slot b after the encoder: y[0..P) = prompts, ny = P,
// kvlen = L + P, steps = 0, done = 0, seen = bits(prompts).
void seq_state_init(int b, const int64_t* prompts, int P, int L, int64_t* y, long ldy, int* ny,
                    int* kvlen, int* steps, uint8_t* done, uint32_t* seen, hipStream_t s);


// ---------------------------------------------------------------------------
// Persistent decode (t2s_persist1.hip): the whole AR loop in one launch.
// ---------------------------------------------------------------------------
struct PLayer {
    const __half *w_in, *w_out, *w1, *w2;   // fp16, the graph's [out][in] layouts
    const float *b_in, *b_out, *b1, *b2, *n1w, *n1b, *n2w, *n2b;
};
constexpr int PERSIST_LGS = 1056;       // logits granule row stride (128-B multiple)
struct PersistArgs {
    int B;
    PLayer L[24];                                 // by value: kernarg (scalar loads)
    const __half* emb; const float* alpha; const float* pe; const __half* w_pred;
    float* kc[24]; float* vc[24];
    long sstride; int tmax; float scale;
    int64_t* y; long ldy; int* ny; int* kvlen; int* steps; uint8_t* done; uint8_t* stop_out; uint32_t* seen;
    int top_k; float temperature; float rep_penalty; int greedy; uint64_t seed; int max_steps; int force_steps;
    const int* force_b;                           // optional per-sequence force_steps (>0 overrides)
    unsigned long long* ring;                     // granule ring (persist1_ring_bytes / persist1m_ring_bytes)
    unsigned epoch;                               // launch epoch (tag high bits), 1 .. 2^20-1
    int* err;                                     // zeroed per launch; non-zero: a hand-off timed out
    const int* stop_req;                          // host-mapped stop word (gsv_request_stop), or null: once
                                                  // set, every sequence finishes at its next token (<= 2 steps)
    int smax;                                     // step cap of the launch
    int groups;                                   // layer groups (layer l -> group l % groups)
    unsigned long long* trace;                    // optional [grid][16] phase stamps (step 8, layer 12)
    unsigned long long spin_ticks;                // single-sequence kernel: hand-off wait bound (100 MHz ticks)
    int pf_delay;                                 // single-sequence kernel: s_sleep(32) ticks between a
                                                  // workgroup's publish and its next-layer prefetch
    float f16_limit;                              // single-sequence kernel: largest |activation| its fp16
                                                  // split accepts (65504; tests lower it)
    int knob[4];                                  // single-sequence kernel: tuning variants (option "knobN";
                                                  // 0 = the default path)
    const float* fold;                            // single-sequence kernel: per layer [W_in n2w_{l-1} | W_in n2b_{l-1}
                                                  // + b_in | W1 n1w | W1 n1b + b1] (1536, 1536, 2048, 2048 floats;
                                                  // layer 0: 0 | b_in), so a GEMV can run beside its LayerNorm stats;
                                                  // then [W_pred n2w_23 | W_pred n2b_23] (1025 each, the logits)
};
constexpr int PERSIST_TMAX = 4096;   // longest key range of the persistent decode (its PE table)
// Single-sequence persistent decode (t2s_persist1.hip): a.groups (3..8) layer
// groups x 32 workgroups, two hand-offs per layer.  Needs persist1_grid(groups)
// resident CUs; B must be 1.
int persist1_grid(int groups);
int persist1_max_groups();
size_t persist1_ring_bytes();
hipError_t decode_persist1(const PersistArgs& a, hipStream_t s, hipEvent_t start, hipEvent_t stop);
// The same kernel's multi-sequence form (k_decode_persist1m): 2 <= a.B <= persist1m_max_batch() (64)
// sequences, each layer's workgroups run the live sequences one after another.
int persist1m_max_batch();
size_t persist1m_ring_bytes(int B);
hipError_t decode_persist1m(const PersistArgs& a, hipStream_t s, hipEvent_t start, hipEvent_t stop);
// The batched form (k_decode_persistm, t2s_persistm.hip): a.groups sequence groups x 16
// workgroups, each group decoding up to 4 sequences (b = g, g + groups, ...) through all
// 24 layers with the batch on the MFMA M dimension.  Same ring layout as persist1m.
int persistm_groups(int B);      // the fewest groups that hold B sequences
int persistm_max_groups();
int persistm_grid(int groups);
hipError_t decode_persistm(const PersistArgs& a, hipStream_t s, hipEvent_t start, hipEvent_t stop);

}  // namespace gsv
