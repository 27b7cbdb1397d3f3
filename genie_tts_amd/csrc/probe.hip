// Kernel probes: replay one kernel configuration `iters` times (captured in a
// hipGraph, as the decode loop runs) between HIP events on the engine stream
// and report the average time per launch.  Used by bench.py for the live
// roofline measurement of the dominant kernel and by tools/ microbenchmarks.
#include <hip/hip_runtime.h>

#include <chrono>
#include <string>

#include "engine_internal.h"

using namespace gsv;

__global__ void k_empty(int* p) {
    if (p && threadIdx.x == 0 && blockIdx.x == 0x7fffffff) p[0] = 1;
}

// which: 0 empty(1 block) 1 empty(256 blocks) 2 gemv QKV+LN 3 gemv QKV no-LN
//        4 gemv FFN1(+LN) 5 gemv FFN2 6 gemv out-proj 7 attention decode (kvlen as set)
//        8 full decode step (B as given) 9 attention+out-proj 10 fused FFN 11 QKV+partials+LN
//        14-17 sampler (14 full; ablations 15 no top-k, 16 no softmax, 17 loads + tail)
extern "C" int gsv_probe(gsv_engine* eng, int which, int B, int iters, float* us, void* stream) {
    if (!eng || !us || iters <= 0) return set_error(GSV_E_ARG, "bad probe args");
    hipSetDevice(eng->device);
    if (!eng->finalized) return set_error(GSV_E_STATE, "weights not finalized");
    if (eng->max_batch < B) return set_error(GSV_E_CAPACITY, "probe: reserve first");
    if (int e = eng->pf_drop()) return e;
    StreamScope sc(eng, stream);
    hipStream_t st = sc.st();
    const long sstride = (long)16 * eng->tmax * 32;
    const T2SLayerW& W = eng->layers[1];
    // sampler probes (14-17) advance their own scratch sequence state, one token per launch
    int64_t* probe_y = nullptr;
    int* probe_i = nullptr;
    uint8_t* probe_done = nullptr;
    const long probe_cap = iters + 256;   // warm-up replay (50) + ceil(iters/50)*50 launches
    if (which >= 14 && which <= 17) {
        hipMalloc(&probe_y, (size_t)B * probe_cap * 8);
        hipMalloc(&probe_i, (size_t)3 * B * 4);
        hipMalloc(&probe_done, (size_t)B);
        if (!probe_y || !probe_i || !probe_done) return set_error(GSV_E_HIP, "probe scratch");
        hipMemsetAsync(probe_i, 0, (size_t)3 * B * 4, st);
        hipMemsetAsync(probe_done, 0, (size_t)B, st);
    }
    struct Free {
        void* p[3];
        ~Free() { for (void* q : p) if (q) hipFree(q); }
    } free_guard{{probe_y, probe_i, probe_done}};
    auto launch = [&]() {
        switch (which) {
            case 0: hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, st, nullptr); break;
            case 1: hipLaunchKernelGGL(k_empty, dim3(256), dim3(256), 0, st, nullptr); break;
            case 2: case 3: {
                GemvArgs a{};
                a.B = B; a.N = 1536; a.K = 512; a.src = eng->s2; a.lds = 512;
                if (which == 2) { a.ln_g = eng->layers[0].n2w; a.ln_b = eng->layers[0].n2b; a.ln_out = eng->h; }
                a.W = W.w_in; a.bias = W.b_in; a.C = eng->q; a.ldc = 512; a.mode = EPI_QKV;
                a.kv.k = eng->kcache[1]; a.kv.v = eng->vcache[1]; a.kv.tmax = eng->tmax; a.kv.row_pos = eng->kvlen;
                a.kv.seq_stride = sstride; a.kv.row_skip = nullptr;
                gemv_f16(a, st);
            } break;
            case 4: {
                GemvArgs f1{};
                f1.B = B; f1.N = 2048; f1.K = 512; f1.src = eng->s1; f1.lds = 512;
                f1.ln_g = W.n1w; f1.ln_b = W.n1b; f1.ln_out = eng->h1;
                f1.W = W.w1; f1.bias = W.b1; f1.C = eng->f; f1.ldc = 2048; f1.mode = EPI_RELU;
                gemv_f16(f1, st);
            } break;
            case 5: {
                GemvArgs f2{};
                f2.B = B; f2.N = 512; f2.K = 2048; f2.src = eng->f; f2.lds = 2048;
                f2.W = W.w2; f2.bias = W.b2; f2.C = eng->s2; f2.ldc = 512; f2.mode = EPI_RESID;
                f2.res = eng->h1; f2.ldr = 512;
                gemv_f16(f2, st);
            } break;
            case 6: {
                GemvArgs c{};
                c.B = B; c.N = 512; c.K = 512; c.src = eng->o; c.lds = 512;
                c.W = W.w_out; c.bias = W.b_out; c.C = eng->s1; c.ldc = 512; c.mode = EPI_RESID;
                c.res = eng->h; c.ldr = 512;
                gemv_f16(c, st);
            } break;
            case 7: {
                AttnArgs at{};
                at.q = eng->q; at.ldq = 512; at.k = eng->kcache[1]; at.v = eng->vcache[1];
                at.seq_stride = sstride; at.tmax = eng->tmax; at.row_len = eng->kvlen; at.row_seq = eng->ident;
                at.out = eng->o; at.ldo = 512; at.rows = B; at.scale = eng->qk_scale; at.row_skip = nullptr;
                attn_rows_plus(at, 1, st);
            } break;
            case 9: {
                AttnOutArgs ao{};
                ao.B = B; ao.q = eng->q; ao.k = eng->kcache[1]; ao.v = eng->vcache[1];
                ao.seq_stride = sstride; ao.tmax = eng->tmax; ao.kvlen = eng->kvlen; ao.done = nullptr;
                ao.scale = eng->qk_scale; ao.WoT = W.woT; ao.part = eng->attn_part;
                attn_outproj(ao, st);
            } break;
            case 10: {
                FfnArgs fa{};
                fa.B = B; fa.nslices = eng->ffn_slices; fa.h = eng->h; fa.bo = W.b_out;
                fa.attn_part = eng->attn_part; fa.ln_g = W.n1w; fa.ln_b = W.n1b; fa.h1 = eng->h1;
                fa.W1 = W.w1; fa.b1 = W.b1; fa.W2T = W.w2T; fa.part = eng->ffn_part;
                ffn_fused(fa, st);
            } break;
            case 11: {
                GemvArgs a{};
                a.B = B; a.N = 1536; a.K = 512;
                a.part = eng->ffn_part; a.n_part = eng->ffn_slices; a.part_stride = (long)B * 512;
                a.part_bias = W.b2; a.part_res = eng->h1;
                a.ln_g = W.n2w; a.ln_b = W.n2b; a.ln_out = eng->h;
                a.W = eng->layers[2].w_in; a.bias = eng->layers[2].b_in; a.C = eng->q; a.ldc = 512;
                a.mode = EPI_QKV; a.kv.k = eng->kcache[2]; a.kv.v = eng->vcache[2]; a.kv.tmax = eng->tmax;
                a.kv.row_pos = eng->kvlen; a.kv.seq_stride = sstride; a.kv.row_skip = nullptr;
                gemv_f16(a, st);
            } break;
            case 14: case 15: case 16: case 17: {
                // scratch state (probe_y sized for every launch of this probe): never done
                gsv_sampler sp{15, 1.0f, 1.35f, 1, 0, 1 << 30, 1 << 30};
                SampleArgs sa = eng->sampler_args(&sp, B);
                sa.y = probe_y; sa.ldy = probe_cap; sa.ny = probe_i; sa.steps = probe_i + B;
                sa.kvlen = probe_i + 2 * B; sa.done = probe_done; sa.stop_out = nullptr;
                sa.ablate = which - 14;
                sample_tokens(sa, st);
            } break;
            default: break;
        }
    };
    if (which == 8 || which == 12 || which == 13) {
        // 8: 1-step graph; 12: 8-step graph (per step); 13: host cost of one 8-step graph launch
        gsv_sampler sp{15, 1.0f, 1.35f, 1, 0, 1 << 30, 1 << 30};
        const int chunk = which == 8 ? 1 : 8;
        hipGraphExec_t ex = eng->step_graph(B, &sp, chunk, st);
        if (!ex) return set_error(GSV_E_HIP, "probe graph");
        hipGraphLaunch(ex, st);
        hipStreamSynchronize(st);
        if (which == 13) {
            auto t0 = std::chrono::high_resolution_clock::now();
            for (int i = 0; i < iters; ++i) hipGraphLaunch(ex, st);
            auto t1 = std::chrono::high_resolution_clock::now();
            hipStreamSynchronize(st);
            *us = std::chrono::duration<float, std::micro>(t1 - t0).count() / iters;
            return 0;
        }
        const int reps = which == 8 ? iters : std::max(1, iters / 8);
        hipEventRecord(eng->ev[0], st);
        for (int i = 0; i < reps; ++i) hipGraphLaunch(ex, st);
        hipEventRecord(eng->ev[1], st);
        hipEventSynchronize(eng->ev[1]);
        float ms = 0.f;
        hipEventElapsedTime(&ms, eng->ev[0], eng->ev[1]);
        *us = ms * 1000.0f / (reps * chunk);
        return hipGetLastError() == hipSuccess ? 0 : set_error(GSV_E_HIP, "probe");
    } else {
        const int per = 50;
        hipGraph_t g = nullptr;
        std::shared_lock<std::shared_mutex> cl(gsv::capture_mu);
        if (hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal) != hipSuccess)
            return set_error(GSV_E_HIP, "probe capture");
        for (int i = 0; i < per; ++i) launch();
        hipStreamEndCapture(st, &g);
        hipGraphExec_t ex = nullptr;
        hipGraphInstantiate(&ex, g, nullptr, nullptr, 0);
        hipGraphDestroy(g);
        if (!ex) return set_error(GSV_E_HIP, "probe instantiate");
        hipGraphLaunch(ex, st);
        const int reps = (iters + per - 1) / per;
        hipEventRecord(eng->ev[0], st);
        for (int i = 0; i < reps; ++i) hipGraphLaunch(ex, st);
        hipEventRecord(eng->ev[1], st);
        hipEventSynchronize(eng->ev[1]);
        hipGraphExecDestroy(ex);
        float ms = 0.f;
        hipEventElapsedTime(&ms, eng->ev[0], eng->ev[1]);
        *us = ms * 1000.0f / (reps * per);
        return hipGetLastError() == hipSuccess ? 0 : set_error(GSV_E_HIP, "probe");
    }
    hipEventSynchronize(eng->ev[1]);
    float ms = 0.f;
    hipEventElapsedTime(&ms, eng->ev[0], eng->ev[1]);
    *us = ms * 1000.0f / iters;
    return hipGetLastError() == hipSuccess ? 0 : set_error(GSV_E_HIP, "probe");
}
