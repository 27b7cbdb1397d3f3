// VITS orchestration (placeholder until the VITS kernels land).
#include "engine_internal.h"
using namespace gsv;

int gsv_engine::finalize_vits() { return 0; }
int gsv_engine::finalize_prompt_encoder() { return 0; }
int gsv_engine::vits_decode(const int64_t*, int, const int64_t*, int, const float*, int, const float*,
                            const float*, const float*, float, float*, hipStream_t) {
    return set_error(GSV_E_STATE, "VITS path not built");
}
int gsv_engine::prompt_encode(const float*, int, const float*, float*, float*, hipStream_t) {
    return set_error(GSV_E_STATE, "prompt encoder not built");
}
extern "C" int gsv_vits_decode(gsv_engine* eng, const int64_t* text_seq, int32_t n_text,
                               const int64_t* sem, int32_t n_sem, const float* ref_audio,
                               int32_t n_audio, const float* ge, const float* ge_adv,
                               const float* eps, float noise_scale, float* audio, void* stream) {
    if (!eng) return set_error(GSV_E_ARG, "null engine");
    hipSetDevice(eng->device);
    return eng->vits_decode(text_seq, n_text, sem, n_sem, ref_audio, n_audio, ge, ge_adv, eps,
                            noise_scale, audio, stream ? (hipStream_t)stream : eng->stream);
}
extern "C" int gsv_prompt_encode(gsv_engine* eng, const float* ref_audio, int32_t n_audio,
                                 const float* sv_emb, float* ge, float* ge_adv, void* stream) {
    if (!eng) return set_error(GSV_E_ARG, "null engine");
    hipSetDevice(eng->device);
    return eng->prompt_encode(ref_audio, n_audio, sv_emb, ge, ge_adv,
                              stream ? (hipStream_t)stream : eng->stream);
}
