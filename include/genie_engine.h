/*
 * genie_engine.h -- C ABI of the MI355X GPT-SoVITS engine (libgenie_engine.so).
 *
 * Drop-in replacement for the onnxruntime InferenceSession objects that Genie
 * holds per character in `GSVModel` (reference: src/genie_tts/ModelManager.py:48-56)
 * and calls from `GENIE.tts` / `GENIE.t2s_cpu` (src/genie_tts/Core/Inference.py:16-109).
 *
 *   reference call                                   replaced by
 *   ------------------------------------------------ ------------------------------------
 *   load_session_with_fp16_conversion (ModelManager.py:59-114)
 *                                                    gsv_engine_create + gsv_set_weight
 *                                                    + gsv_finalize_weights
 *   encoder.run            (Inference.py:76-85)      gsv_t2s_encode
 *   first_stage_decoder.run(Inference.py:88-90)      gsv_t2s_prefill
 *   stage_decoder.run      (Inference.py:102)        gsv_t2s_decode_steps (k steps)
 *   the 500-step loop + trim (Inference.py:95-109)   gsv_t2s_generate (the whole loop as ONE persistent
 *                                                    kernel launch; per-step hipGraphs only as a fallback)
 *   vocoder.run            (Inference.py:47-60)      gsv_vits_decode
 *   prompt_encoder.run     (ReferenceAudio.py:73)    gsv_prompt_encode
 *   vocoder.run's refer branch (Inference.py:50, V2)  gsv_ref_encode (once per reference)
 *   cn_hubert.run          (ReferenceAudio.py:50-52) gsv_hubert
 *   roberta_model.run      (GetPhonesAndBert.py:73)  gsv_roberta (gsv_roberta_batch: many sentences)
 *   per-sentence tts loop  (TTSPlayer.py:56-107)     gsv_t2s_prefetch, gsv_t2s_generate_start /
 *                                                    _finish, gsv_vits_decode_async / gsv_vits_wait
 *                                                    (option "vocoder_cus")
 *   stop_event.set()/.clear() (Inference.py:13-14,96-97) gsv_request_stop
 *
 * Conventions
 *   - All functions return 0 on success, a negative GSV_E* code on failure;
 *     gsv_last_error() returns a thread-local message for the last failure.
 *   - Weights are engine-owned device memory.  Every other pointer argument
 *     marked (device) is a caller-owned device buffer (e.g. a torch tensor's
 *     data_ptr()); (host) arguments are read before the call returns.
 *   - `stream` is the caller's hipStream_t passed as void* (NULL = the HIP null
 *     stream).  The engine runs on its own stream, ordered after `stream` on
 *     entry and before it on exit by events: results are stream-ordered for
 *     the caller.
 *     Calls on one engine are serialised by the caller (one engine per GPU
 *     process, as the reference serialises on its single TTS worker thread,
 *     Core/TTSPlayer.py:55).
 *   - Integer ids are int64 (the graphs' dtype); audio/features fp32.
 */
#ifndef GENIE_ENGINE_H
#define GENIE_ENGINE_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GSV_OK 0
#define GSV_E_ARG -1
#define GSV_E_HIP -2
#define GSV_E_STATE -3
#define GSV_E_WEIGHT -4
#define GSV_E_CAPACITY -5
#define GSV_E_STOPPED -6   /* the generate was abandoned by gsv_request_stop (the reference returns None) */

typedef struct gsv_engine gsv_engine;

/* dtype codes for gsv_set_weight */
#define GSV_F32 0
#define GSV_F16 1

/* Model families (ModelManager.py:287-293: prompt encoder present => V2ProPlus). */
#define GSV_V2 0
#define GSV_V2PP 1

const char* gsv_last_error(void);
const char* gsv_version(void);

/* Create an engine on HIP device `device` for model family `version`. */
int gsv_engine_create(int device, int version, gsv_engine** out);
int gsv_engine_destroy(gsv_engine* eng);

/* Stage one weight tensor (host memory, any of GSV_F32/GSV_F16) by its graph
 * initializer name (e.g. "transformer_encoder.layers.0.linear1.weight",
 * "vq_model.dec.ups.0.weight_v").  Copied before return. */
int gsv_set_weight(gsv_engine* eng, const char* name, const void* host, int dtype,
                   const int64_t* dims, int ndim);

/* Fold weight norm (w = v/||v|| * g), convert, upload; must follow the last
 * gsv_set_weight.  Missing tensors are an error (GSV_E_WEIGHT).  No weight is ever
 * rounded silently: the T2S / VITS / prompt-encoder paths take fp16 weights (the
 * Genie fp16 bins, ModelManager.py:59-114) and refuse a tensor that is not
 * fp16-exact (GSV_E_WEIGHT naming it); RoBERTa and CN-HuBERT keep fp32 values
 * (RoBERTa.onnx is loaded as fp32, ModelManager.py:139-142) as fp16 hi + lo planes
 * (counter "w16_split_tensors"). */
int gsv_finalize_weights(gsv_engine* eng);

/* Host-only check used by those loaders: 1 if all n values are exactly fp16 numbers,
 * else 0 with *first_bad = the first index that is not (-1 when all are).  Needs no
 * device. */
int gsv_f16_exact(const float* values, int64_t n, int64_t* first_bad);

/* Reserve decode capacity: up to `max_batch` sequences of up to `max_tokens`
 * positions (x + prompts + generated) each.  Allocates the KV cache. */
int gsv_reserve(gsv_engine* eng, int max_batch, int max_tokens);

/* ---------------------------------------------------------------- T2S ---- */
/* One utterance of a batch.  All pointers (device). */
typedef struct {
    const int64_t* ref_seq;   int32_t n_ref;    /* phonemes of the reference text  */
    const int64_t* text_seq;  int32_t n_text;   /* phonemes of the target text     */
    const float*   ref_bert;                    /* [n_ref, 1024]  or NULL = zeros  */
    const float*   text_bert;                   /* [n_text, 1024] or NULL = zeros  */
    const float*   ssl;       int32_t n_ssl;    /* ssl_content [768, n_ssl]        */
    int32_t force_steps;                        /* >0: this utterance ignores EOS and runs
                                                   exactly this many loop steps (overrides
                                                   gsv_sampler.force_steps; benchmarks and
                                                   ragged-batch tests); 0: the sampler's rule */
} gsv_utt;

/* Sampler (reference constants: t2s_stage_decoder_fp32.onnx#1780-1801). */
typedef struct {
    int32_t top_k;               /* 15 (1..64) */
    float   temperature;         /* 1.0 */
    float   repetition_penalty;  /* 1.35 */
    int32_t greedy;              /* 1: RandomNormalLike := 1 (argmax of penalised logits) */
    uint64_t seed;               /* Philox key for N(0,1) when !greedy */
    int32_t max_steps;           /* 500 (Inference.py:95) */
    int32_t force_steps;         /* >0: ignore EOS and run exactly this many loop steps */
} gsv_sampler;

/* Encoder (t2s_encoder_fp32.onnx) for one utterance:
 * x (device, [n_ref+n_text, 512] f32), prompts (device, [n_ssl/2] i64). */
int gsv_t2s_encode(gsv_engine* eng, const gsv_utt* u, float* x, int64_t* prompts, void* stream);

/* Full T2S of a batch: encoder, prefill (one packed pass over the batch), the decode
 * loop on the device, and the reference's token trim + EOS filter
 * (Inference.py:41-44,108-109).  The loop is one persistent kernel launch: B = 1 on
 * k_decode_persist1, B = 2..64 on its multi-sequence form k_decode_persist1m (each
 * layer's workgroups run the live sequences one after another); B > 64, an activation
 * beyond the fp16 range, or a launch whose grid could not be co-resident (a hand-off
 * timeout) re-run on replayed per-step hipGraphs.  out_tokens (host)
 * [batch][out_stride] i64, out_len (host) [batch].  Returns the trimmed semantic tokens
 * per utterance; GSV_E_STOPPED when gsv_request_stop interrupted it. */
int gsv_t2s_generate(gsv_engine* eng, int batch, const gsv_utt* utts, const gsv_sampler* s,
                     int64_t* out_tokens, int32_t out_stride, int32_t* out_len, void* stream);

/* Parity/session entry points mirroring the reference graphs one call at a time.
 * prefill: x (device [L,512]), prompts (device [P]) -> writes slot `seq` of the
 *   engine KV cache, y (device i64 [P+1]), logits (device f32 [1025], may be NULL).
 * decode_steps: runs `steps` stage-decoder steps on slot `seq`, appending to y
 *   (device i64, capacity >= P+1+steps); stop (device u8 [steps]);
 *   logits (device [steps][1025] or NULL). */
int gsv_t2s_prefill(gsv_engine* eng, int seq, const float* x, int32_t n_x, const int64_t* prompts,
                    int32_t n_prompts, const gsv_sampler* s, int64_t* y, float* logits, void* stream);
int gsv_t2s_decode_steps(gsv_engine* eng, int seq, int steps, const gsv_sampler* s, int64_t* y,
                         uint8_t* stop, float* logits, void* stream);
/* Copy the KV cache of slot `seq`, layer `layer` as [n,512] k and v (device). */
int gsv_t2s_read_kv(gsv_engine* eng, int seq, int layer, float* k, float* v, int32_t* n, void* stream);

/* --------------------------------------------------------------- VITS ---- */
/* vits_fp32.onnx.  text_seq (device i64 [n_text]), sem (device i64 [n_sem]).
 * V2: ref_audio (device f32 [n_audio] at 32 kHz), ge/ge_adv NULL; or ref_audio NULL and
 *     ge (device [512]) from gsv_ref_encode of that audio (identical output).
 * V2ProPlus: ge (device [1024]), ge_adv (device [512]), ref_audio NULL.
 * eps: (device [192, 2*n_sem]) noise for z_p, or NULL => zeros.
 * audio (device f32 [640*2*n_sem]). */
int gsv_vits_decode(gsv_engine* eng, const int64_t* text_seq, int32_t n_text,
                    const int64_t* sem, int32_t n_sem, const float* ref_audio, int32_t n_audio,
                    const float* ge, const float* ge_adv, const float* eps, float noise_scale,
                    float* audio, void* stream);

/* Several vocoder calls at once (the same graph per utterance, vits_fp32.onnx).  Option
 * "seg_vocoder" 1 (default): each utterance's text/flow part runs on the engine's lanes
 * (internal streams, own workspaces), then the HiFi-GAN generator runs ONCE over all of
 * them laid out back to back along time with zero gaps between utterances (every conv
 * treats a gap as the zero padding a single call sees), so its ~400 launches serve the
 * whole batch; each utterance matches its own gsv_vits_decode to fp32 rounding (the
 * batch's larger tiles order the reductions differently).  With option "seg_front" 1
 * (default) the text/flow part is packed the same way (one pass, attention within each
 * utterance) whenever every item carries ge (+ ge_adv) and noise_mode 0 or 2; otherwise
 * it runs per item on the lanes.  seg_vocoder 0: whole utterances on the lanes,
 * bit-identical to single calls.  Results are stream-ordered for the caller like
 * gsv_vits_decode.
 * Noise for z_p (vits(v2)#6490 RandomNormalLike x noise_scale):
 *   noise_mode 0: zeros; 1: eps (device [192, 2*n_sem]); 2: the engine's Philox
 *   N(0,1) stream keyed by noise_seed (counter = element index; Box-Muller). */
typedef struct {
    const int64_t* text_seq; int32_t n_text;   /* device */
    const int64_t* sem;      int32_t n_sem;    /* device */
    const float* ref_audio;  int32_t n_audio;  /* V2: device 32 kHz audio (or NULL with ge), else NULL */
    const float* ge;         const float* ge_adv;   /* V2ProPlus: device [1024], [512];
                                                       V2: optional ge [512] of gsv_ref_encode */
    const float* eps;                          /* noise_mode 1 */
    uint64_t noise_seed;                       /* noise_mode 2 */
    int32_t noise_mode;
    float* audio;                              /* device [1280 * n_sem] */
} gsv_vits_item;
int gsv_vits_decode_batch(gsv_engine* eng, int32_t n, const gsv_vits_item* items, float noise_scale,
                          void* stream);

/* The same batch, overlapped with the T2S of the next batch (a server batching the
 * next sentence of every pending request; each sentence a full Inference.tts,
 * Core/Inference.py:16-61).  gsv_vits_decode_batch_async forks the batch over the
 * vocoder lanes (ordered after `stream`) and returns while lane threads may still be
 * issuing; the engine stream stays free, so a gsv_t2s_generate issued next runs
 * beside it.  Items and their buffers must stay valid until gsv_vits_batch_wait,
 * which joins the lanes, re-runs fp16-range overflows on the f32 path and orders
 * `stream` (may be NULL) after the batch.  Any other vocoder call finishes it first.
 * Audio is identical to gsv_vits_decode_batch's. */
int gsv_vits_decode_batch_async(gsv_engine* eng, int32_t n, const gsv_vits_item* items, float noise_scale,
                                void* stream);
int gsv_vits_batch_wait(gsv_engine* eng, void* stream);

/* Overlapped vocoder for a stream of sentences (the reference synthesises them one
 * after the other: TTSPlayer._tts_worker_loop, Core/TTSPlayer.py:56-107, each
 * sentence a full Inference.tts, Core/Inference.py:16).  After
 * gsv_set_option(eng, "vocoder_cus", K) the engine stream runs on n_cu - K CUs and
 * the vocoder on the other K, so sentence i's vocoder overlaps sentence i+1's T2S.
 * gsv_vits_decode_async starts one vocoder call (ordered after `stream`) and returns
 * without waiting; the item's buffers must stay valid until gsv_vits_wait, which
 * finishes it (fp16-range overflow -> the f32 re-run, as gsv_vits_decode) and orders
 * `stream` (may be NULL) after it.  One call in flight: a second async call, any
 * other vocoder call or gsv_prompt_encode finishes the pending one first. */
int gsv_vits_decode_async(gsv_engine* eng, const gsv_vits_item* item, float noise_scale, void* stream);
int gsv_vits_wait(gsv_engine* eng, void* stream);

/* The T2S side of the same pipeline: encode + prefill the NEXT sentence ahead, on
 * the vocoder CUs while the current sentence decodes (the reference's per-sentence
 * encoder + first-stage decoder, Inference.py:63-72, moved off the critical path).
 * Needs option "vocoder_cus".  Call it for sentence i+1 before gsv_t2s_generate of
 * sentence i: it is queued and launched (into a spare KV slot, behind a queued
 * gsv_vits_decode_async call) right after that generate's decode kernel; the next
 * gsv_t2s_generate with batch 1 and a field-wise equal utt / sampler then decodes
 * from it (identical tokens).  A batch-1 generate of another utterance keeps a
 * queued prefetch; a batch generate or any other T2S call discards it.  The utt's
 * buffers must stay valid until the generate that uses it. */
int gsv_t2s_prefetch(gsv_engine* eng, const gsv_utt* utt, const gsv_sampler* sampler, void* stream);

/* gsv_t2s_generate for one utterance, split so the GPU never waits for the host
 * between the sentences of a stream: _start queues the utterance (taking its
 * prefetch when one matches) and returns at once; up to two may be in flight, so
 * the next decode is queued behind the running one.  _finish blocks for the oldest
 * started one and returns its trimmed tokens (host [out_stride]) as
 * gsv_t2s_generate would, ordering `stream` after it.  A launch that meets the
 * fp16-range or hand-off-timeout condition is re-run synchronously inside _finish.
 * Other T2S calls wait for the started ones first; their results stay queued. */
int gsv_t2s_generate_start(gsv_engine* eng, const gsv_utt* utt, const gsv_sampler* sampler, void* stream);
int gsv_t2s_generate_finish(gsv_engine* eng, int64_t* out_tokens, int32_t out_stride, int32_t* out_len,
                            void* stream);

/* V2: the vocoder graph's reference branch alone (vits_fp32.onnx(v2)#79-271: refer
 * spectrogram -> MelStyleEncoder; ReferenceAudio.py:40-45 feeds it the 32 kHz audio on
 * every vocoder.run) -> ge (device [512]).  It depends on the reference only: pass it as
 * the ge of gsv_vits_decode or of a gsv_vits_item, with ref_audio NULL, for every sentence spoken
 * against that reference; the audio is identical to passing ref_audio. */
int gsv_ref_encode(gsv_engine* eng, const float* ref_audio, int32_t n_audio, float* ge, void* stream);

/* prompt_encoder_fp32.onnx (V2ProPlus): ref_audio (device [n_audio]),
 * sv_emb (device [20480]) -> ge (device [1024]), ge_adv (device [512]). */
int gsv_prompt_encode(gsv_engine* eng, const float* ref_audio, int32_t n_audio,
                      const float* sv_emb, float* ge, float* ge_adv, void* stream);

/* chinese-hubert-base.onnx (CN-HuBERT, ReferenceAudio.py:48-52; session loaded at
 * ModelManager.py:172-195): input_values = raw 16 kHz audio (device [n_samples])
 * -> ssl_content (device [768][T], the graph's [1, 768, T] output), T =
 * gsv_hubert_frames(n_samples) (the conv stack's output length).  Needs an
 * engine whose weights include the HuBERT tensors (transformers HubertModel
 * names, encoder.pos_conv_embed.conv.weight already weight-normed). */
int gsv_hubert_frames(int32_t n_samples);
int gsv_hubert(gsv_engine* eng, const float* audio_16k, int32_t n_samples, float* ssl_content, void* stream);

/* speaker_encoder.onnx (V2ProPlus speaker verification, ReferenceAudio.py:71-72:
 * speaker_verification_model.run(None, {'waveform': audio_16k}); session loaded at
 * ModelManager.py:155-170): waveform = the 16 kHz reference clip (device
 * [n_samples]) -> sv_emb (device [20480], the graph's [1, 20480] output), the
 * prompt encoder's sv_emb input.  Kaldi fbank (80 mel bins, 25/10 ms frames,
 * snip edges) -> ERes2NetV2 (GPT-SoVITS sv.py, baseWidth 24 / scale 4 / expansion 4)
 * forward3.  gsv_sv_frames(n) is the fbank frame count (0: too short, GSV_E_ARG).
 * Needs an engine whose weights include the SV tensors (weights.sv_spec names). */
int gsv_sv_frames(int32_t n_samples);
int gsv_sv(gsv_engine* eng, const float* audio_16k, int32_t n_samples, float* sv_emb, void* stream);

/* RoBERTa.onnx (chinese-roberta-wwm-ext-large BERT features for Chinese text,
 * GetPhonesAndBert.py:64-74; session ModelManager.py:132-150): input_ids (device
 * i64 [n_tokens], CLS .. SEP), attention_mask (host i64 [n_tokens], all ones, or
 * NULL), repeats = word2ph (host i64 [n_chars], n_chars <= n_tokens - 2) ->
 * text_bert (device [sum(repeats)][1024]) = hidden_states[-3] of the character
 * rows 1 .. n_chars, row i repeated repeats[i - 1] times.  Needs an engine whose
 * weights include the BertModel tensors (transformers names). */
int gsv_roberta(gsv_engine* eng, const int64_t* input_ids, const int64_t* attention_mask, int32_t n_tokens,
                const int64_t* repeats, int32_t n_chars, float* text_bert, void* stream);

/* The same for n_seq sentences in one pass (the reference runs RoBERTa once per
 * Chinese sentence; packed here: every GEMM over all sentences' token rows, attention
 * within each sentence): input_ids (device i64, the sentences' CLS .. SEP ids
 * concatenated), n_tokens (host [n_seq]), repeats (host i64, the sentences' word2ph
 * concatenated), n_chars (host [n_seq]) -> text_bert (device, the sentences'
 * [sum(word2ph_s)][1024] blocks concatenated in order).  Identical to n_seq gsv_roberta
 * calls. */
int gsv_roberta_batch(gsv_engine* eng, int32_t n_seq, const int64_t* input_ids, const int32_t* n_tokens,
                      const int64_t* repeats, const int32_t* n_chars, float* text_bert, void* stream);

/* Debug hooks (tests only): copy a named VITS workspace buffer after
 * gsv_vits_decode ("ge","stats","z","y","q","te","g0","g1","spec","a");
 * run one conv1d (zero padding) on device buffers; a non-NULL splitk_ws (device,
 * splitk_cap floats) enables the split-K path for under-filled grids. */
int gsv_debug_copy(gsv_engine* eng, const char* name, float* dst, int64_t n, void* stream);
int gsv_debug_conv1d(const float* x, int cin, int tin, const float* w, int cout, int k, int dil,
                     int pad, const float* bias, float* out, int tout, int in_act, float slope,
                     float* splitk_ws, int64_t splitk_cap, void* stream);
/* The same conv on the f16-split MFMA path (vits_convh.hip, the MRF convs of
 * dec.resblocks.* in vits_fp32.onnx): wh = fp16 weights [cout][k][cin], scale =
 * per-output-channel f32 factor on the sums (weight norm g/||v||); *ovf (device
 * int) is OR-ed with 1 when an input exceeds the fp16 range.  GSV_E_ARG when the
 * shape is not covered (k in {3,7,11}, cin % 8 == 0, dil <= 5). */
int gsv_debug_conv1d_h(const float* x, int cin, int tin, const void* wh, const float* scale, int cout,
                       int k, int dil, int pad, const float* bias, float* out, int tout, int in_act,
                       float slope, int* ovf, void* stream);
/* The achievable HBM rate: `iters` grid-stride copies (16-B non-temporal
 * loads / stores, 4 per thread in flight) of `bytes`
 * (16-B aligned device buffers) on `stream`; *ms = the mean time of one copy (HIP events).
 * Read + write bytes = 2 x bytes per copy.  Measurement helper for bench.py. */
int gsv_debug_hbm_copy(const void* src, void* dst, int64_t bytes, int iters, void* stream, float* ms);
/* Phase timestamps (100 MHz) of the per-step-graph decode kernels (t2s_decode.hip:
 * the fp16-range re-run / timeout / B > 64 path, not the persistent kernels) of
 * layer 12, last step run: [kernel: QKV GEMV, attention, FFN][block 0..255][slot
 * 0..7]; needs GENIE_KTRACE=1 in the environment at gsv_finalize_weights. */
int gsv_debug_ktrace(gsv_engine* eng, uint64_t* host, int n);
/* Run the decode sampler kernel once on logits (device [B][1025]) with the
 * token-presence bitmaps seen (device u32 [B][33]) at loop step `step`
 * (Philox counter); tokens (device i64 [B]) and stop flags (device u8 [B]). */
int gsv_debug_sample(const float* logits, const uint32_t* seen, int B, const gsv_sampler* s,
                     int step, int64_t* tokens, uint8_t* stop, void* stream);

/* Probe: replay one kernel configuration `iters` times (hipGraph) between HIP
 * events on the engine stream; *us = average microseconds per launch.
 * which: 0/1 empty kernel (1/256 blocks), 2 QKV GEMV (+LN prologue), 3 QKV GEMV,
 * 4 FFN1 GEMV (+LN), 5 FFN2 GEMV, 6 out-proj GEMV, 7 decode attention,
 * 8 one full decode step (graph) for batch B.  Requires gsv_reserve(B, ...). */
int gsv_probe(gsv_engine* eng, int which, int B, int iters, float* us, void* stream);

/* Per-phase device time of the last gsv_t2s_generate / gsv_vits_decode (ms):
 * [0]=encode [1]=prefill [2]=decode [3]=vits.  Filled when timing is enabled. */
int gsv_set_timing(gsv_engine* eng, int enabled);
int gsv_get_timing(gsv_engine* eng, float* ms4);
/* Live duration of the dominant kernel, the persistent decode launch (k_decode_persist1 /
 * k_decode_persist1m: the whole decode loop of a generate): while timing is enabled each
 * launch carries start/stop events stamped from its dispatch packet
 * (hipExtLaunchKernelGGL).  On the per-step graph path the sample is one eagerly run step's
 * FFN launch instead.  Average microseconds and number of samples; a negative count is
 * -(hipError_t) of a failed hipEventElapsedTime. */
int gsv_get_kernel_timing(gsv_engine* eng, float* avg_us, int32_t* samples);

/* Stop (the reference's GENIE.stop_event, checked before every loop step:
 * Inference.py:96-97 returns None for the sentence).  on = 1 sets the engine's stop
 * word, 0 clears it (TTSPlayer.py:86 clears the event when a new job starts).  While it
 * is set, T2S generates (gsv_t2s_generate, _start/_finish) return GSV_E_STOPPED: a
 * running decode leaves within two loop steps -- the persistent kernels read the word
 * once per step at token resolution, the per-step graphs' sampler every step -- and a
 * new one returns at once.  The engine stays usable.  The only entry point that may be
 * called from another thread while a call on the engine runs: it writes one word. */
int gsv_request_stop(gsv_engine* eng, int32_t on);

/* Engine options (no reference counterpart; the reference's session options are
 * ORT's).  "persist": 1 (default) runs gsv_t2s_generate's decode loop as ONE
 * persistent launch (B <= 64), 0 as replayed per-step hipGraphs; setting it also ends
 * a timeout back-off.  "persist1m" (1): B = 2..64 on the multi-sequence kernel (0: the
 * graphs); "persistm" (1) / "persistm_min_b" (32): from that batch size on, the batched
 * kernel with the batch on the MFMA M dimension (t2s_persistm.hip; groups of <= 4
 * sequences per 16 CUs).  "persist_backoff" / "persist_backoff_ms": the first back-off hold
 * after two timed-out launches in a row (64 generates / 5 s, doubling per failed re-probe).
 * "vocoder_cus" (CU split for the sentence pipeline), "decode_cus" / "decode_cu_offset",
 * "vits_lanes", "seg_vocoder" (1, default: a vocoder batch runs its generator as ONE pass
 * over all utterances laid out back to back), "seg_front" (1, default: its text/flow part
 * too, see gsv_vits_decode_batch), "convh" (MRF convs on the split-fp16 MFMA),
 * "convt_f16" (1, default: the upsample ConvTransposes on it too), "mrf_fused" (1, default:
 * each conv pair of an MRF resblock step of the C <= 32 stages as one kernel, its
 * intermediate in LDS), "sv_f16", "packed", "attn_mf32" (1, default: the prefill's
 * attention on the f32 MFMA with k_attn_flash's exact fma chains; 0: k_attn_flash itself,
 * bit-identical results), "vits_fork" (1, default: a single VITS call on the engine's unmasked
 * stream runs the front's text branch beside its SSL branch and a generator stage's three resblocks
 * on three streams; 0: in order on one stream; bit-identical),
 * "pf_delay" (0: a B = 1 decode workgroup waits N x s_sleep(32)
 * between its publish and its next-layer refill), A/B options measured and left off:
 * "convh_persist" (the large split-fp16 convs as a persistent tile loop, bit-identical),
 * "convh_ws" (the 7- / 11-tap MRF convs with 64 / 128 input channels weight-stationary, k_conv_ws:
 * 0 off, 1 in every batched generator pass, 2 -- the default -- only in a synchronous
 * gsv_vits_decode_batch, whose vocoder has the GPU to itself;
 * bit-identical),
 * "vocoder_first" (a batched decode waits for the running vocoder batch), "lanes_all_cus"
 * (under vocoder_cus, the batch lanes on every CU), "knob0".."knob3" (decode tuning variants),
 * test hooks ("persist_spin_ticks", "persist1_f16_limit", "sv_f16_limit", "convh_tile":
 * 1..4 forces that k_conv_h tile candidate, 0 the cost model).  "ptrace": 1 allocates per-workgroup phase stamps of the persistent
 * launch (step 8, layer 12), read back with gsv_debug_ptrace ([256 workgroups][16
 * slots]: 8 stamps of the 100 MHz clock, then the same 8 of the shader clock).
 * GSV_E_ARG for an unknown name. */
int gsv_set_option(gsv_engine* eng, const char* name, int value);
/* Engine counters: "persist_timeouts" (persistent decode launches whose hand-offs
 * timed out -- e.g. other work on the device -- and re-ran as per-step graphs),
 * "persist_disabled" (back-off holds begun), "persist_hold" (generates left in the
 * current hold), "persist_launches", "persist1_f16_reruns" (fp16-range fallbacks),
 * "vits_f32_reruns", "vits_packed_fronts" (vocoder batches whose text/flow part ran
 * packed), "sv_f32_reruns", "w16_split_tensors" (fp32 weights kept as hi + lo
 * planes), "stops" (generates abandoned by gsv_request_stop), "graph_fallbacks"
 * (per-step decode loops run eagerly because their hipGraph capture failed -- e.g.
 * invalidated by another thread's device-wide synchronisation), "retired_bytes" (device
 * buffers replaced by a capacity growth and not yet freed), "reclaimed_bytes" / "reclaims"
 * (freed by the growth paths once the engine's streams drained; capacities grow in
 * quantised steps: batch to a power of two, tokens to a multiple of 256, workspaces by
 * 1.25x, so a load ramp re-allocates a few times and keeps no dead copies). */
int gsv_get_counter(gsv_engine* eng, const char* name, int64_t* value);
int gsv_debug_ptrace(gsv_engine* eng, uint64_t* host, int n);

#ifdef __cplusplus
}
#endif
#endif /* GENIE_ENGINE_H */
