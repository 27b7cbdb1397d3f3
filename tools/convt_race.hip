// Standalone reproduction of the r04u/r04w nondeterminism: the HiFi-GAN generator's
// polyphase ConvTranspose stages on k_conv_h, each followed by three MRF-shaped convs,
// issued on several streams at once; every stage output of every stream is compared bit
// for bit with a run of the same chain alone on one stream.
//
// Build (in this container), as the engine (no packed-FP32 ops) and as hipcc's default:
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -Xclang -target-feature -Xclang -packed-fp32-ops \
//         tools/convt_race.hip -o tools/convt_race
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/convt_race.hip -o tools/convt_race_pk
// (profiles/r05_convt_race.txt: the second one reproduces the r04 corruption, the first does not)
// Run:   tools/convt_race <iters> <streams> <convt tile 0..3 | -1 cost model> [flags: 1 no input scale, 2 no leaky relu]
// Prints per stage the number of (stream, iteration) outputs that differ from the lone run.
#include "../genie_tts_amd/csrc/vits_convh.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <random>
#include <vector>

using namespace gsv;

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(2);                                                                   \
        }                                                                              \
    } while (0)

namespace {

struct Stage {   // one generator stage: ConvT (Cin -> Cout, rate u, kernel k) + 3 MRF convs
    int cin, cout, u, k, M;
    __half* wh;        // [u][cout][M][cin]
    float* wscale;     // ones [cout]
    float* isc;        // [cin]
    float* bias;       // [cout]
    __half* mw[3];     // MRF [cout][kt][cout]
    float* mscale[3];
    float* mbias[3];
};
const int MRF_K[3] = {3, 7, 11}, MRF_D[3] = {1, 3, 5};

template <typename T>
T* dev_upload(const std::vector<T>& h) {
    T* d = nullptr;
    CK(hipMalloc(&d, h.size() * sizeof(T)));
    CK(hipMemcpy(d, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice));
    return d;
}

std::vector<__half> rnd_h(size_t n, float sc, std::mt19937& g) {
    std::normal_distribution<float> nd(0.f, sc);
    std::vector<__half> v(n);
    for (auto& x : v) x = __float2half(nd(g));
    return v;
}
std::vector<float> rnd_f(size_t n, float mean, float sc, std::mt19937& g) {
    std::normal_distribution<float> nd(mean, sc);
    std::vector<float> v(n);
    for (auto& x : v) x = nd(g);
    return v;
}

struct Chain {   // one stream's buffers for an utterance of T frames
    int T;
    float* x0;
    float* y[5];   // ConvT outputs
    float* t[5];   // MRF scratch
    float* m[5];   // stage outputs (inputs of the next stage)
    int* ovf;
};

int g_tile = -1;
int g_flags = 0;   // bit 0: ConvT without the input-channel scale (in_scale null); bit 1: without the input leaky relu

void launch_convt(const Stage& S, const float* x, int Tc, float* out, int* ovf, hipStream_t st) {
    const int padT = (S.k - S.u) / 2;
    const int Tn = (Tc - 1) * S.u - 2 * padT + S.k;
    ConvArgs a{};
    a.x = x; a.x_cs = Tc; a.x_ts = 1; a.Cin = S.cin; a.Tin = Tc;
    a.Cout = S.cout; a.K = S.M; a.dil = 1; a.pad = S.M - 1;
    a.bias = S.bias; a.out = out; a.o_cs = Tn; a.o_ts = 1;
    a.n_t = (Tn + padT + S.u - 1) / S.u; a.o_tstride = S.u; a.o_toff = -padT; a.o_len = Tn;
    a.in_act = 1; a.in_slope = 0.1f; a.mode = CV_STORE;
    a.phases = S.u;
    a.wh = S.wh; a.wscale = S.wscale; a.ovf = ovf; a.in_scale = (g_flags & 1) ? nullptr : S.isc;
    if (g_flags & 2) a.in_act = 0;
    a.wh_phase_stride = (long)S.cout * S.M * S.cin;
    if (g_tile < 0) {   // the product's cost model (without the polyphase exclusion when built so)
        if (!conv1d_h(a, st)) { fprintf(stderr, "convt not covered\n"); exit(3); }
        return;
    }
    static const int tw[4][3] = {{2, 2, 1}, {1, 2, 2}, {1, 1, 4}, {1, 4, 1}};
    const int wm = tw[g_tile][0], wn = tw[g_tile][1], ks = tw[g_tile][2];
    const dim3 grid((a.n_t + 64 * wn - 1) / (64 * wn), (a.Cout + 32 * wm - 1) / (32 * wm), S.u);
#define LT(KT)                                                                                            \
    if (S.M == KT) {                                                                                      \
        if (g_tile == 0) hipLaunchKernelGGL((k_conv_h<KT, 32, 2, 2, 1>), grid, dim3(256), 0, st, a);      \
        else if (g_tile == 1) hipLaunchKernelGGL((k_conv_h<KT, 32, 1, 2, 2>), grid, dim3(256), 0, st, a); \
        else if (g_tile == 2) hipLaunchKernelGGL((k_conv_h<KT, 32, 1, 1, 4>), grid, dim3(256), 0, st, a); \
        else hipLaunchKernelGGL((k_conv_h<KT, 32, 1, 4, 1>), grid, dim3(256), 0, st, a);                  \
        return;                                                                                           \
    }
    LT(1) LT(2) LT(4)
#undef LT
    (void)ks;
    fprintf(stderr, "M %d\n", S.M);
    exit(3);
}

void launch_mrf(const Stage& S, int j, const float* x, float* out, const float* res, int Tc, int* ovf,
                hipStream_t st) {
    ConvArgs a{};
    a.x = x; a.x_cs = Tc; a.x_ts = 1; a.Cin = S.cout; a.Tin = Tc;
    a.Cout = S.cout; a.K = MRF_K[j]; a.dil = MRF_D[j]; a.pad = (MRF_K[j] * MRF_D[j] - MRF_D[j]) / 2;
    a.bias = S.mbias[j]; a.out = out; a.o_cs = Tc; a.o_ts = 1; a.n_t = Tc; a.o_tstride = 1; a.o_len = Tc;
    a.in_act = 1; a.in_slope = 0.1f; a.mode = CV_RESID; a.res = res; a.r_cs = Tc; a.r_ts = 1;
    a.phases = 1;
    a.wh = S.mw[j]; a.wscale = S.mscale[j]; a.ovf = ovf;
    if (!conv1d_h(a, st)) { fprintf(stderr, "mrf not covered\n"); exit(3); }
}

void run_chain(const std::vector<Stage>& st, Chain& c, hipStream_t s) {
    const float* x = c.x0;
    int Tc = c.T;
    for (int i = 0; i < 5; ++i) {
        const Stage& S = st[i];
        launch_convt(S, x, Tc, c.y[i], c.ovf, s);
        Tc *= S.u;
        // t = mrf3(y) + y ; m = mrf7(t) + t ; m = mrf11(m) + m   (in place on m, as the generator's rbuf)
        launch_mrf(S, 0, c.y[i], c.t[i], c.y[i], Tc, c.ovf, s);
        launch_mrf(S, 1, c.t[i], c.m[i], c.t[i], Tc, c.ovf, s);
        launch_mrf(S, 2, c.m[i], c.t[i], c.m[i], Tc, c.ovf, s);
        CK(hipMemcpyAsync(c.m[i], c.t[i], (size_t)S.cout * Tc * 4, hipMemcpyDeviceToDevice, s));
        x = c.m[i];
    }
}

size_t stage_elems(const std::vector<Stage>& st, int T, int i) {
    long Tc = T;
    for (int k = 0; k <= i; ++k) Tc *= st[k].u;
    return (size_t)st[i].cout * Tc;
}

}  // namespace

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 50;
    const int nstream = argc > 2 ? atoi(argv[2]) : 4;
    g_tile = argc > 3 ? atoi(argv[3]) : 2;
    g_flags = argc > 4 ? atoi(argv[4]) : 0;
    CK(hipSetDevice(0));
    std::mt19937 g(1234);
    const int cfg[5][3] = {{10, 16, 0}, {8, 16, 0}, {2, 8, 0}, {2, 2, 0}, {2, 2, 0}};
    std::vector<Stage> st(5);
    int C = 512;
    for (int i = 0; i < 5; ++i) {
        Stage& S = st[i];
        S.cin = C; S.cout = C / 2; S.u = cfg[i][0]; S.k = cfg[i][1]; S.M = (S.k + S.u - 1) / S.u;
        S.wh = dev_upload(rnd_h((size_t)S.u * S.cout * S.M * S.cin, 0.05f, g));
        S.wscale = dev_upload(std::vector<float>(S.cout, 1.f));
        S.isc = dev_upload(rnd_f(S.cin, 1.f, 0.2f, g));
        S.bias = dev_upload(rnd_f(S.cout, 0.f, 0.1f, g));
        for (int j = 0; j < 3; ++j) {
            S.mw[j] = dev_upload(rnd_h((size_t)S.cout * MRF_K[j] * S.cout, 0.3f / std::sqrt((float)S.cout * MRF_K[j]), g));
            S.mscale[j] = dev_upload(rnd_f(S.cout, 1.f, 0.1f, g));
            S.mbias[j] = dev_upload(rnd_f(S.cout, 0.f, 0.05f, g));
        }
        C /= 2;
    }
    const int Ts[8] = {52, 40, 66, 80, 94, 46, 58, 72};
    // reference chains (one per distinct T, run alone) and the per-stream chains
    std::vector<Chain> ref(nstream), ch(nstream);
    auto alloc_chain = [&](Chain& c, int T, const std::vector<float>& x0) {
        c.T = T;
        c.x0 = dev_upload(x0);
        for (int i = 0; i < 5; ++i) {
            const size_t n = stage_elems(st, T, i);
            CK(hipMalloc(&c.y[i], n * 4)); CK(hipMalloc(&c.t[i], n * 4)); CK(hipMalloc(&c.m[i], n * 4));
            CK(hipMemset(c.y[i], 0xff, n * 4)); CK(hipMemset(c.t[i], 0xff, n * 4)); CK(hipMemset(c.m[i], 0xff, n * 4));
        }
        CK(hipMalloc(&c.ovf, 64));
        CK(hipMemset(c.ovf, 0, 64));
    };
    for (int s = 0; s < nstream; ++s) {
        const int T = Ts[s % 8];
        std::vector<float> x0 = rnd_f((size_t)512 * T, 0.f, 1.f, g);
        alloc_chain(ref[s], T, x0);
        alloc_chain(ch[s], T, x0);
    }
    hipStream_t s0;
    CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
    for (int s = 0; s < nstream; ++s) {   // the lone runs, one after another, twice (determinism check)
        run_chain(st, ref[s], s0);
        CK(hipStreamSynchronize(s0));
    }
    std::vector<std::vector<std::vector<float>>> want(nstream, std::vector<std::vector<float>>(10));
    for (int s = 0; s < nstream; ++s)
        for (int i = 0; i < 5; ++i) {
            const size_t n = stage_elems(st, ref[s].T, i);
            want[s][2 * i].resize(n);
            want[s][2 * i + 1].resize(n);
            CK(hipMemcpy(want[s][2 * i].data(), ref[s].y[i], n * 4, hipMemcpyDeviceToHost));
            CK(hipMemcpy(want[s][2 * i + 1].data(), ref[s].m[i], n * 4, hipMemcpyDeviceToHost));
        }
    std::vector<hipStream_t> ss(nstream);
    for (auto& s : ss) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    long bad[10] = {};
    long first_bad[10] = {};
    std::vector<float> got;
    for (int it = 0; it < iters; ++it) {
        for (int s = 0; s < nstream; ++s) run_chain(st, ch[s], ss[s]);
        CK(hipDeviceSynchronize());
        for (int s = 0; s < nstream; ++s) {
            bool seen = false;
            for (int i = 0; i < 5; ++i)
                for (int k = 0; k < 2; ++k) {
                    const std::vector<float>& w = want[s][2 * i + k];
                    got.resize(w.size());
                    CK(hipMemcpy(got.data(), k == 0 ? ch[s].y[i] : ch[s].m[i], w.size() * 4, hipMemcpyDeviceToHost));
                    long nd = 0, f = -1;
                    for (size_t e = 0; e < w.size(); ++e)
                        if (std::memcmp(&got[e], &w[e], 4) != 0) { if (f < 0) f = (long)e; ++nd; }
                    if (nd) {
                        ++bad[2 * i + k];
                        if (!seen) {
                            ++first_bad[2 * i + k];
                            seen = true;
                            const long Tn = (long)w.size() / st[i].cout;
                            printf("iter %d stream %d T %d: stage %d %s first differs, %ld values, first (co %ld, t %ld): %g vs %g\n",
                                   it, s, ch[s].T, i, k ? "mrf" : "convT", nd, f / Tn, f % Tn, got[f], w[f]);
                            if (k == 0) {   // the differing (co, t) set: channels, and t as (block of 64 n_t columns, column, phase)
                                long cmin = 1 << 30, cmax = -1, tmin = 1L << 40, tmax = -1;
                                std::vector<int> cols(64, 0), chs(st[i].cout, 0);
                                for (size_t e = 0; e < w.size(); ++e)
                                    if (std::memcmp(&got[e], &w[e], 4) != 0) {
                                        const long co = (long)e / Tn, tp = (long)e % Tn;
                                        cmin = std::min(cmin, co); cmax = std::max(cmax, co);
                                        tmin = std::min(tmin, tp); tmax = std::max(tmax, tp);
                                        cols[(tp / st[i].u) % 64]++;
                                        chs[co]++;
                                    }
                                printf("   co %ld..%ld  tp %ld..%ld (n_t col %ld..%ld)  per-channel:", cmin, cmax, tmin, tmax,
                                       tmin / st[i].u, tmax / st[i].u);
                                for (int c2 = 0; c2 < st[i].cout; ++c2) if (chs[c2]) printf(" %d:%d", c2, chs[c2]);
                                printf("\n   cols%%64:");
                                for (int c2 = 0; c2 < 64; ++c2) if (cols[c2]) printf(" %d:%d", c2, cols[c2]);
                                printf("\n");
                            }
                        }
                    }
                }
        }
        if (it % 10 == 9) { printf("iter %d done\n", it + 1); fflush(stdout); }
    }
    printf("SUMMARY tile %d streams %d iters %d:", g_tile, nstream, iters);
    for (int i = 0; i < 5; ++i) printf(" s%d convT %ld/%ld mrf %ld/%ld;", i, bad[2 * i], first_bad[2 * i], bad[2 * i + 1], first_bad[2 * i + 1]);
    printf("\n");
    return 0;
}
