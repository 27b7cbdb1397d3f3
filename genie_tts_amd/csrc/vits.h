// VITS (SoVITS decoder + HiFi-GAN / MelStyleEncoder) kernels and device weights.
// Activations are fp32 channel-major [C][T] as in the reference graph
// (src/genie_tts/Data/v2/Models/vits_fp32.onnx).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>
#include <stdint.h>

#include <vector>

namespace gsv {

constexpr int MHA_MAXK_HOST = 2048;   // keys per attention row (k_mha LDS)

// ----------------------------------------------------------------- conv1d
// out(co, t_phys) = epi( bias[co] + sum_{ci,j} w[co][ci][j] * act(x(ci, t + j*dil - pad)) )
//   x(ci,t) = x[ci*x_cs + t*x_ts], zero outside [0, Tin)
//   t in [0, n_t) is the logical output index, t_phys = t*o_tstride + o_toff (+phase, see below)
//   stored only when 0 <= t_phys < o_len.
// ConvTranspose1d runs as `phases` polyphase convs (blockIdx.z = phase r):
//   w += r * w_phase_stride, t_phys = t*o_tstride + (o_toff + r).
enum ConvMode {
    CV_STORE = 0,       // out = v
    CV_RELU = 1,        // out = relu(v)
    CV_RESID = 2,       // out = res + v
    CV_VEC = 3,         // out = v + vec[co]
    CV_SUB = 4,         // out = res - v                 (flow coupling x1 - m)
    CV_TANH = 5,        // out = tanh(v)                 (conv_post)
    CV_ACC_FIRST = 6,   // acc = res + v                 (MRF: xs = rb0(x))
    CV_ACC_ADD = 7,     // acc = acc + (res + v)         (xs += rb_j(x))
    CV_ACC_MEAN = 8,    // out = (acc + (res + v)) / div (x = xs / num_kernels)
    CV_RESID_VEC = 9,   // out = (res + v) + vec[co]     (MRTE: attn + ssl_enc + ge)
    CV_SPLIT_RESID = 10,// co < split: out = res + v ; else out2 = res2 + v   (WN res/skip)
};

struct ConvArgs {
    const float* x; long x_cs, x_ts; int Cin, Tin;
    const float* w; int Cout, K, dil, pad;
    const float* bias;
    float* out; long o_cs, o_ts; int n_t, o_tstride, o_toff, o_len;
    int in_act; float in_slope;      // 1: leaky relu(in_slope) on the input
    int mode;
    const float* res; long r_cs, r_ts;
    const float* vec;
    float* acc; float div;
    int split; float* out2; const float* res2;
    int phases; long w_phase_stride;
    // split-K workspace (floats); when set, conv1d splits the Cin reduction of
    // under-filled grids over grid.z into partial slabs [split][Cout][n_t] and a
    // second kernel sums them in fixed order and applies the epilogue.
    float* part; long part_cap;
    // f16-split MFMA path (vits_convh.hip): weights fp16 [Cout][K][Cin] (the
    // fp16 values of the reference's weight_v / weight), per-output-channel
    // scale (weight norm g/||v||, 1 without it), overflow flag set when an
    // input does not fit fp16.  wh == nullptr -> f32 path.
    const __half* wh; const float* wscale; int* ovf;
    // ... a ConvTranspose's polyphase weights on that path: [phases][Cout][K][Cin] (phase
    // stride wh_phase_stride halfs); its weight norm is over the INPUT channel, applied as
    // in_scale[ci] to the (pre-activated) input instead of to the sums
    long wh_phase_stride; const float* in_scale;
    // segmented batch (several utterances back to back along time, zero gaps between
    // them): seg[tp] = the utterance of output time tp, or -1 in a gap, where the
    // output is written as 0 (so every buffer keeps zero gaps, and a conv whose halo
    // reaches into a gap reads the zero padding a single-utterance call sees);
    // CV_VEC / CV_RESID_VEC read vec + seg[tp] * vec_sstride
    const int* seg; long vec_sstride;
    // f16-split path: 0 = the cost model's tile; 1..4 = tile candidate 0..3 of launch_h (option
    // "convh_tile", tests)
    int tile_force;
    // f16-split path: > 0 = the CUs of the stream; large grids then run the persistent tile
    // loop (two blocks per CU) instead of one block per tile (option "convh_persist")
    int persist;
    // f16-split path: > 0 = the CUs of the stream; the wide MRF convs (Cin 64 / 128) then run
    // the weight-stationary persistent form, k_conv_ws (option "convh_ws")
    int ws;
};
void conv1d(const ConvArgs& a, hipStream_t s);
// seg[t] for t < n: i with off[i] * f <= t < (off[i] + len[i]) * f, else -1 (off ascending)
void seg_fill(int* seg, long n, const int* off, const int* len, int nseg, int f, hipStream_t s);
// f16-split path; returns false (nothing launched) when the shape is not covered.
bool conv1d_h(const ConvArgs& a, hipStream_t s);

// One ResBlock1 step of a narrow generator stage (C = 16 / 32) as one kernel (vits_mrf.hip):
// xt = lrelu(conv1_d(lrelu(r)) + b1) in LDS only, then conv2 (kernel k, dilation 1) with e
// as its epilogue (e.bias = conv2's bias, e.res = r, e.mode / out / acc / div / seg; e.Cout
// = C, e.n_t = T).  Weights fp16 [C][k][C] with per-output-channel scales.  e.out must not
// alias r (neighbouring blocks read r's halo).  false: shape not covered (nothing launched).
struct MrfPairArgs {
    const float* r; int T, C, K, dil;
    const __half* w1; const float* s1; const float* b1;
    const __half* w2; const float* s2;
    int* ovf;
    ConvArgs e;
};
bool mrf_pair(const MrfPairArgs& a, hipStream_t s);

// LayerNorm over channels per t: out = LN(x + y) (y may be null), eps 1e-5; seg (segmented
// batch, as ConvArgs::seg): a gap column is written as zeros
// out[i] = ((a[i] + b[i]) + c[i]) / div: the MRF mean of a stage's three resblocks in the order of the
// ACC_FIRST / ACC_ADD / ACC_MEAN chain
void mean3(const float* a, const float* b, const float* c, float* out, long n, float div, hipStream_t s);
void ln_channels(const float* x, const float* y, float* out, int C, int T, const float* g,
                 const float* b, hipStream_t s, const int* seg = nullptr);

// Multi-head attention with optional relative-position terms (window W).
//   element (i, c) of q/k/v/out at ptr[i*ts + c*cs]; head h uses channels [h*dk, (h+1)*dk)
//   score_ij = (q_i / sqrt(dk)) . k_j  [+ (q_i/sqrt(dk)) . ek[j-i+W] if |j-i|<=W]   (prescale)
//           or (q_i . k_j) / temperature                                        (postdiv)
struct MhaArgs {
    const float* q; long q_ts, q_cs;
    const float* k; long k_ts, k_cs;
    const float* v; long v_ts, v_cs;
    float* out; long o_ts, o_cs;
    int nq, nk, heads, dk;
    int postdiv; float scale;          // prescale: divisor sqrt(dk); postdiv: temperature
    const float* ek; const float* ev; int window;   // rel-pos (or null)
    const int* row_seg;   // optional (device) [nq][2] {first key, key count} per query row: packed
                          // sequences attend within their own rows; nk is then unused.  With rel-pos
                          // terms the queries are packed as the keys (self-attention): the relative
                          // offset is (key - first key) - (row - first key)
};
void mha(const MhaArgs& a, hipStream_t s);

// Small elementwise kernels
void codebook_upsample2(const int64_t* sem, int G, const float* cb, float* out, hipStream_t s);
void embed_channels(const int64_t* ids, int n, const float* emb, int C, float* out, hipStream_t s);
void wn_gate(const float* xin, float* acts, int H, int T, hipStream_t s);      // tanh(a)*sigmoid(b)
void glu_resid(const float* h, const float* x, float* out, int C, int T, long x_cs, long x_ts,
               hipStream_t s);                                                  // out = x + a*sigmoid(b)
void noise_zp(const float* m, const float* logs, const float* eps, float scale, float* z, int n,
              hipStream_t s);
void noise_zp_philox(const float* m, const float* logs, uint64_t seed, float scale, float* z, int n,
                     hipStream_t s);                                              // eps ~ Philox N(0,1)
void flip_channels(const float* in, float* out, int C, int T, hipStream_t s);
// Segmented-batch forms (utterances back to back along time, seg[t] = utterance or -1 in
// a gap, off[i] its first column): the per-utterance inputs through device pointer tables;
// gap columns are written as zeros.
void codebook_upsample2_seg(const int64_t* const* sems, const int* seg, const int* off, int T, const float* cb,
                            float* out, hipStream_t s);
void embed_channels_seg(const int64_t* const* ids, const int* seg, const int* off, int n, const float* emb, int C,
                        float* out, hipStream_t s);
// utterance i's element (c, t - off[i]) draws Philox index c * len[i] + t - off[i] under
// seeds[i] (seed 0: no noise), as noise_zp_philox / noise_zp on that utterance alone
void noise_zp_philox_seg(const float* m, const float* logs, const uint64_t* seeds, const int* seg, const int* off,
                         const int* len, float scale, float* z, int C, int T, hipStream_t s);
// out[i][0, dim) = ptrs[i][0, dim)
void gather_vecs(const float* const* ptrs, int n, int dim, float* out, hipStream_t s);
void reflect_pad(const float* x, int n, int pad, float* out, hipStream_t s);
void stft_mag(const float* reim, int frames, int bins, float* spec, hipStream_t s); // [F][2*bins] -> [F][bins]
void time_mean(const float* x, int T, int C, float* out, hipStream_t s);       // x [T][C] -> sum/T
void prelu_vec(const float* x, const float* a, float* out, int n, hipStream_t s);
void add_vec(const float* a, const float* b, float* out, int n, hipStream_t s);

// ----------------------------------------------------------------- weights
struct Conv {
    float* w = nullptr;   // [Cout][Cin][K] (or [phases][Cout][Cin][K] for ConvT)
    float* b = nullptr;
    int cout = 0, cin = 0, k = 0, phases = 1;
    __half* wh = nullptr;      // fp16 [Cout][K][Cin] when every weight value is fp16-exact
                               // (ConvT: [phases][Cout][K][Cin])
    float* wscale = nullptr;   // [Cout] weight-norm scale applied to the f16 path's sums
    float* in_scale = nullptr; // ConvT: [Cin] weight-norm scale applied to the input
};

struct AttnLayer {
    Conv qkv, o, ffn1, ffn2;
    float *ek = nullptr, *ev = nullptr;
    float *g1 = nullptr, *b1 = nullptr, *g2 = nullptr, *b2 = nullptr;
};

struct RefEnc {
    float *fc0_w = nullptr, *fc0_b = nullptr, *fc3_w = nullptr, *fc3_b = nullptr;
    Conv temporal[2];
    float *wqkv = nullptr, *bqkv = nullptr, *fcw = nullptr, *fcb = nullptr;
    float *out_w = nullptr, *out_b = nullptr;
    int out_dim = 0;
    float* dft = nullptr;   // [2*704][2048] windowed DFT basis
};

struct VitsWeights {
    bool ready = false;
    int gin = 512, upc = 512;
    int n_up = 5;
    int up_rate[5] = {}, up_k[5] = {};
    int rb_k[3] = {3, 7, 11}, rb_d[3] = {1, 3, 5};
    float* codebook = nullptr;           // [1024][768]
    Conv ssl_proj, c_pre, text_pre, c_post, mrte_qkv_q, mrte_kv, mrte_o, proj;
    float* text_emb = nullptr;           // [732][192]
    std::vector<AttnLayer> enc_ssl, enc_text, enc2;
    // flows (4 couplings, reverse order handled by the host)
    struct Flow {
        Conv pre, post, cond;
        Conv in_l[4], rs[4];
    } flows[4];
    Conv conv_pre, cond, conv_post;
    Conv ups[5];
    Conv rb[15][2][3];                   // [resblock][convs1/convs2][dilation idx]
    RefEnc ref;
};

struct VitsWorkspace {
    size_t cap_t = 0;   // capacity in frames (2G)
    size_t cap_gen = 0; // capacity of generator buffers (floats)
    int cap_spec = 0;
    float *q = nullptr, *y = nullptr, *te = nullptr, *a = nullptr, *b = nullptr, *c = nullptr;
    float *qkv = nullptr, *att = nullptr, *ffn = nullptr;
    float *tq = nullptr, *tqkv = nullptr, *tatt = nullptr, *tffn = nullptr, *ta = nullptr, *tb = nullptr;
    float *ssl_enc = nullptr, *text_enc = nullptr, *mq = nullptr, *mkv = nullptr, *mo = nullptr;
    float *stats = nullptr, *z = nullptr, *z2 = nullptr, *fh = nullptr, *fx = nullptr, *fa = nullptr;
    float *fskip = nullptr, *fm = nullptr, *gcond = nullptr, *dcond = nullptr;
    float *g0 = nullptr, *g1 = nullptr, *g2 = nullptr, *g3 = nullptr, *g4 = nullptr;
    float* gx[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};   // resblocks 1 / 2 on side streams
    float *ge = nullptr, *pad = nullptr, *reim = nullptr, *spec = nullptr, *r0 = nullptr, *r1 = nullptr;
    float *r2 = nullptr, *r3 = nullptr, *rq = nullptr, *ratt = nullptr;
    float* splitk = nullptr;   // conv split-K partial slabs
    long splitk_cap = 0;
    float* splitk2 = nullptr;  // ... of the front's text branch on the side stream (same capacity)
    float *sv = nullptr, *pe_ge = nullptr;
    int cap_text = 0;
    std::vector<void*> owned;   // the buffers above except splitk (retired when the workspace grows)
};

struct PromptEncWeights {
    bool ready = false;
    RefEnc ref;
    __half* sv_w = nullptr;   // [1024][20480] fp16
    float *sv_b = nullptr, *to512_w = nullptr, *to512_b = nullptr, *prelu = nullptr;
};

}  // namespace gsv
