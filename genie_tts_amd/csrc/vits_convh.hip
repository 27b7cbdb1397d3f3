// HiFi-GAN MRF conv1d on the f16 MFMA (v_mfma_f32_32x32x16_f16) with split
// fp32 activations: x = hi + lo, hi = fp16(x), lo = fp16(x - hi), so
//   sum_k w_k x_k = sum_k w_k hi_k + sum_k w_k lo_k      (f32 accumulate)
// carries ~22 bits of every activation.  The weights need no split: every value
// of vits_fp16.bin is fp16 (ModelManager.py:59-114 upcasts fp16 -> fp32), and
// weight norm (vits(v2) ReduceL2 -> Div -> Mul on weight_v/weight_g) is a
// per-output-channel scale g/||v|| applied to the f32 sums in the epilogue.
// Reference ops: the resblocks' Conv nodes of vits_fp32.onnx (dec.resblocks.*),
// 130 of the 135.5 GFLOP per utterance.
//
// Implicit GEMM: M = Cout, N = time, K = (tap, Cin).  A K-chunk is CC input
// channels x KT taps.  LDS holds the chunk's input tile time-major,
// [t][ci] in fp16 hi and lo planes (a lane's B fragment = 8 consecutive
// channels at one time = one ds_read_b128), and the weight tile [co][tap][ci]
// (A fragment = one ds_read_b128); row strides are odd multiples of 16 B, so
// the reads are conflict-free.  The next chunk is loaded into registers while
// the MFMAs consume the current one.  Block = 4 waves laid out WM x WN x KS:
// each wave owns a 32 x 64 output tile (two 32x32 accumulators); KS > 1 splits
// the chunk's MFMA steps over waves and sums the partials in fixed order.
//
// Range guard: an input of magnitude > 65504 has no fp16 hi part; the kernel
// then sets *a.ovf and the host re-runs the utterance on the f32 path.
#include "common.h"
#include "vits.h"
#include "vits_epi.h"
#include <cstdlib>

namespace gsv {
namespace {

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
constexpr int DMAX = 5;   // largest dilation of the MRF convs (rb_d)

template <int KT, int CC, int WM, int WN, int KS, int WTM = 1>
struct HCfg {
    static constexpr int BM = 32 * WM * WTM, BN = 64 * WN;
    static constexpr int G8 = CC / 8;                   // 8-channel groups per tap
    static constexpr int NG = KT * G8;                  // groups per chunk
    static constexpr int NSTEP = (NG + 1) / 2;          // MFMA K-steps (2 groups each)
    static constexpr int XW = BN + (KT - 1) * DMAX;     // input rows (time) per tile
    static constexpr int XR = CC == 8 ? 24 : CC + 8;    // halves per X row (odd x 16 B)
    static constexpr int WR = KT * CC + (CC == 8 ? 16 : 8);   // halves per W row (odd x 16 B)
    static constexpr int NXI = (XW * G8 + 255) / 256;   // X items (time, group) per thread
    static constexpr int NWI = (BM * NG + 255) / 256;   // W 16-B items per thread
    static constexpr int X_BYTES = XW * XR * 2;
    static constexpr int W_BYTES = BM * WR * 2;
    static constexpr int RED_BYTES = KS > 1 ? (KS - 1) * WM * WN * WTM * 2 * 16 * 64 * 4 : 0;
    static constexpr int MAIN_BYTES = 2 * X_BYTES + W_BYTES;
    static constexpr int LDS = MAIN_BYTES > RED_BYTES ? MAIN_BYTES : RED_BYTES;
};

__device__ __forceinline__ void split8(const float (&v)[8], uint4& hi, uint4& lo) {
    _Float16 h[8], l[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        h[j] = (_Float16)v[j];
        l[j] = (_Float16)(v[j] - (float)h[j]);
    }
    hi = *reinterpret_cast<const uint4*>(h);
    lo = *reinterpret_cast<const uint4*>(l);
}

// WTM > 1 (the long-time form): each wave owns WTM x 2 accumulators, WTM 32-row output
// blocks over the same 64 time columns, so a K-step's four B fragment reads (two time
// blocks x hi / lo) feed 4 WTM MFMAs instead of 4.  Every accumulator runs the WTM = 1
// MFMA sequence (bit-identical results at the same KS).
//
// PERS (the persistent form, KS = 1): a 1-D grid of two blocks per CU walks the output tiles
// (tile = blockIdx.x, + gridDim.x, ...; time fastest, then output-channel block, then phase).
// The (tile, chunk) pairs of a block form one pipeline: the next pair's loads -- the next
// tile's first chunk after a tile's last -- are in flight during the current chunk's MFMAs
// and staged before the tile's epilogue, so no tile pays the prologue load -> stage ->
// barrier of a fresh block (the C >= 64 MRF convs have 2-8 chunks per tile, r05q: the
// per-call cost grew with a third of the tap count).  Each tile's MFMA sequence is the
// one-block kernel's: bit-identical results.
template <int KT, int CC, int WM, int WN, int KS, int WTM = 1, bool PERS = false>
__global__ __launch_bounds__(256, 2) void k_conv_h(ConvArgs a) {
    using C = HCfg<KT, CC, WM, WN, KS, WTM>;
    static_assert(WTM == 1 || KS == 1, "the multi-block wave form has no K split");
    static_assert(!PERS || KS == 1, "the persistent form has no K split (its LDS holds the next stage)");
    __shared__ __attribute__((aligned(16))) char smem[C::LDS];
    _Float16* Xh = reinterpret_cast<_Float16*>(smem);
    _Float16* Xl = reinterpret_cast<_Float16*>(smem + C::X_BYTES);
    _Float16* Ws = reinterpret_cast<_Float16*>(smem + 2 * C::X_BYTES);

    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int ks = w % KS, wn = (w / KS) % WN, wm = w / (KS * WN);
    const int dil = a.dil;
    const int xw = C::BN + (KT - 1) * dil;
    const int nch = a.Cin / CC;
    // tile coordinates: (t0, co0, ph) of tile tl
    const int ntn = (a.n_t + C::BN - 1) / C::BN, ntm = (a.Cout + C::BM - 1) / C::BM;
    const long ntiles = PERS ? (long)ntn * ntm * (a.phases > 1 ? a.phases : 1) : 1;
    auto coords = [&](long tl, int& t0, int& co0, int& ph) {
        if (!PERS) {
            t0 = blockIdx.x * C::BN; co0 = blockIdx.y * C::BM; ph = a.phases > 1 ? (int)blockIdx.z : 0;
            return;
        }
        const long r = tl / ntn;
        t0 = (int)(tl - r * ntn) * C::BN;
        co0 = (int)(r % ntm) * C::BM;
        ph = (int)(r / ntm);
    };
    const float* __restrict__ isc = a.in_scale;
    const float* __restrict__ X = a.x;

    // per-thread staging items (loop invariant): X item e -> (group c8, row u)
    int xu[C::NXI], xc[C::NXI];
#pragma unroll
    for (int i = 0; i < C::NXI; ++i) {
        const int e = tid + i * 256;
        xc[i] = e / xw;
        xu[i] = e - xc[i] * xw;
        if (xc[i] >= C::G8) xc[i] = -1;
    }
    float xr[C::NXI][8];
    uint4 wr[C::NWI];
    bool ovf = false;

    // PERS: buffer loads, one 32-bit VGPR offset per staging item (the tile part) and the
    // channel / tap offsets in SGPRs, so the current and the next tile's address sets cost a
    // few registers instead of a 64-bit pointer per load; an item outside the input (padding,
    // another output-channel block's rows) gets an offset past the buffer and reads 0
    const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(X), 0, (int)(((long)(a.Cin - 1) * a.x_cs + a.Tin) * 4), 0x00020000);
    const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<__half*>(a.wh), 0,
        (int)((a.phases > 1 ? (long)a.phases * a.wh_phase_stride : (long)a.Cout * KT * a.Cin) * 2), 0x00020000);
    constexpr unsigned OOB = 0x80000000u;
    auto load_b = [&](int t0, int co0, int ph, int ci0) {
        const int xcs4 = (int)(a.x_cs * 4);
#pragma unroll
        for (int i = 0; i < C::NXI; ++i) {
            const int tin = t0 - a.pad + xu[i];
            const bool ok = xc[i] >= 0 && tin >= 0 && tin < a.Tin;
            const unsigned vo = ok ? (unsigned)((xc[i] * 8) * xcs4 + tin * 4) : OOB;
#pragma unroll
            for (int j = 0; j < 8; ++j)
                xr[i][j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xrs, vo, (ci0 + j) * xcs4, 0));
        }
        const int wso = (int)(((long)ph * a.wh_phase_stride + ci0) * 2);
#pragma unroll
        for (int i = 0; i < C::NWI; ++i) {
            const int e = tid + i * 256;
            unsigned vo = OOB;
            if (e < C::BM * C::NG) {
                const int r = e / C::NG, g = e - r * C::NG;
                const int tap = g / C::G8, c8 = g - tap * C::G8;
                const int co = co0 + r;
                if (co < a.Cout) vo = (unsigned)((((co * KT + tap) * a.Cin) + c8 * 8) * 2);
            }
            wr[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(wrs, vo, wso, 0));
        }
    };
    auto load = [&](int t0, int co0, int ph, int ci0) {
        if constexpr (PERS) {
            load_b(t0, co0, ph, ci0);
            return;
        }
        const _Float16* __restrict__ Wg = reinterpret_cast<const _Float16*>(a.wh) + (long)ph * a.wh_phase_stride;
#pragma unroll
        for (int i = 0; i < C::NXI; ++i) {
            const int tin = t0 - a.pad + xu[i];
            const bool ok = xc[i] >= 0 && tin >= 0 && tin < a.Tin;
            const float* src = X + (long)(ci0 + xc[i] * 8) * a.x_cs + tin;
            // raw values only: the pre-activation is applied in store(), so these loads stay
            // in flight across the current chunk's MFMAs (an activation here made the
            // compiler wait vmcnt(0) for them before the MFMAs, serialising every chunk)
#pragma unroll
            for (int j = 0; j < 8; ++j) xr[i][j] = ok ? src[(long)j * a.x_cs] : 0.f;
        }
#pragma unroll
        for (int i = 0; i < C::NWI; ++i) {
            const int e = tid + i * 256;
            uint4 v = make_uint4(0, 0, 0, 0);
            if (e < C::BM * C::NG) {
                const int r = e / C::NG, g = e - r * C::NG;
                const int tap = g / C::G8, c8 = g - tap * C::G8;
                const int co = co0 + r;
                if (co < a.Cout)
                    v = *reinterpret_cast<const uint4*>(Wg + ((long)co * KT + tap) * a.Cin + ci0 + c8 * 8);
            }
            wr[i] = v;
        }
    };
    auto store = [&](int cis) {   // cis: the first input channel of the staged chunk
#pragma unroll
        for (int i = 0; i < C::NXI; ++i) {
            if (xc[i] < 0) continue;
            if (a.in_act) {
#pragma unroll
                for (int j = 0; j < 8; ++j) xr[i][j] = xr[i][j] >= 0.f ? xr[i][j] : xr[i][j] * a.in_slope;
            }
            if (isc) {   // the staged channels are cis + 8 xc + j
#pragma unroll
                for (int j = 0; j < 8; ++j) xr[i][j] *= isc[cis + xc[i] * 8 + j];
            }
            float m = 0.f;
#pragma unroll
            for (int j = 0; j < 8; ++j) m = fmaxf(m, fabsf(xr[i][j]));
            ovf |= m > 65504.f;
            uint4 hi, lo;
            split8(xr[i], hi, lo);
            *reinterpret_cast<uint4*>(Xh + xu[i] * C::XR + xc[i] * 8) = hi;
            *reinterpret_cast<uint4*>(Xl + xu[i] * C::XR + xc[i] * 8) = lo;
        }
#pragma unroll
        for (int i = 0; i < C::NWI; ++i) {
            const int e = tid + i * 256;
            if (e < C::BM * C::NG) {
                const int r = e / C::NG, g = e - r * C::NG;
                const int tap = g / C::G8, c8 = g - tap * C::G8;
                *reinterpret_cast<uint4*>(Ws + r * C::WR + tap * CC + c8 * 8) = wr[i];
            }
        }
    };

    f32x16 acc[WTM][2];
    auto zero_acc = [&]() {
#pragma unroll
        for (int m = 0; m < WTM; ++m)
#pragma unroll
            for (int f = 0; f < 2; ++f)
#pragma unroll
                for (int i = 0; i < 16; ++i) acc[m][f][i] = 0.f;
    };
    zero_acc();

    const int r32 = lane & 31, hsel = lane >> 5;
    const _Float16* wrow = Ws + (wm * 32 * WTM + r32) * C::WR;
    long tile = PERS ? (long)blockIdx.x : 0;
    if (tile >= ntiles) return;
    int t0, co0, ph;
    coords(tile, t0, co0, ph);
    load(t0, co0, ph, 0);
    store(0);
    __syncthreads();
    for (;;) {
        // the tile after this one (PERS), or none
        const long ntile = tile + (PERS ? (long)gridDim.x : 1);
        const bool more = PERS && ntile < ntiles;
        int nt0 = 0, nco0 = 0, nph = 0;
        if (more) coords(ntile, nt0, nco0, nph);
        for (int c = 0; c < nch; ++c) {
            const bool last = c + 1 == nch;
            if (!last) load(t0, co0, ph, (c + 1) * CC);
            else if (more) load(nt0, nco0, nph, 0);
            // PERS: the per-tap LDS row offsets (tap x dilation) are re-formed every chunk, not
            // hoisted out of the tile loop: hoisted, they stayed live across the epilogue and spilled
            int dl = dil;
            if constexpr (PERS) asm volatile("" : "+s"(dl));
#pragma unroll
            for (int j = ks; j < C::NSTEP; j += KS) {
                const int g = 2 * j + hsel;                 // this lane's 8-channel group
                const bool gv = g < C::NG;
                const int tap = gv ? g / C::G8 : 0, c8 = gv ? g - tap * C::G8 : 0;
                h8 A[WTM];
#pragma unroll
                for (int m = 0; m < WTM; ++m) {
                    A[m] = *reinterpret_cast<const h8*>(wrow + m * 32 * C::WR + tap * CC + c8 * 8);
                    if (!gv) A[m] = (h8){0, 0, 0, 0, 0, 0, 0, 0};
                }
#pragma unroll
                for (int f = 0; f < 2; ++f) {
                    const int row = wn * 64 + f * 32 + r32 + tap * dl;
                    const h8 Bl = *reinterpret_cast<const h8*>(Xl + row * C::XR + c8 * 8);
                    const h8 Bh = *reinterpret_cast<const h8*>(Xh + row * C::XR + c8 * 8);
#pragma unroll
                    for (int m = 0; m < WTM; ++m) {
                        acc[m][f] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A[m], Bl, acc[m][f], 0, 0, 0);
                        acc[m][f] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A[m], Bh, acc[m][f], 0, 0, 0);
                    }
                }
            }
            __syncthreads();
            if (!last) {
                store((c + 1) * CC);
                __syncthreads();
            } else if (more) {
                // the next tile's first chunk into the LDS this tile no longer reads (every wave
                // passed the barrier above); its registers are free before the epilogue
                store(0);
            }
        }
        if (KS > 1) {
            // waves ks > 0 park their partials; ks == 0 adds them in ks order
            float* red = reinterpret_cast<float*>(smem);
            const int tl = wm * WN + wn;
            if (ks > 0) {
                float* p = red + ((long)((ks - 1) * WM * WN + tl) * 2 * 16) * 64;
#pragma unroll
                for (int f = 0; f < 2; ++f)
#pragma unroll
                    for (int i = 0; i < 16; ++i) p[(f * 16 + i) * 64 + lane] = acc[0][f][i];
            }
            __syncthreads();
            if (ks > 0) break;
#pragma unroll
            for (int s = 1; s < KS; ++s) {
                const float* p = red + ((long)((s - 1) * WM * WN + tl) * 2 * 16) * 64;
#pragma unroll
                for (int f = 0; f < 2; ++f)
#pragma unroll
                    for (int i = 0; i < 16; ++i) acc[0][f][i] += p[(f * 16 + i) * 64 + lane];
            }
        }
        // epilogue of this tile: registers and global stores only (the next tile's first chunk
        // is already staged in LDS)
#pragma unroll
        for (int m = 0; m < WTM; ++m) {
            const int cobase = co0 + (wm * WTM + m) * 32 + 4 * hsel;
            float sc[16];
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int co = cobase + (r & 3) + 8 * (r >> 2);
                sc[r] = co < a.Cout ? a.wscale[co] : 0.f;
            }
#pragma unroll
            for (int f = 0; f < 2; ++f) {
                const int t = t0 + wn * 64 + f * 32 + r32;
                if (t >= a.n_t) continue;
                float v[16];
#pragma unroll
                for (int r = 0; r < 16; ++r) v[r] = acc[m][f][r] * sc[r];
                if constexpr (PERS) conv_epilogue16_lean(a, cobase, t, ph, v);
                else conv_epilogue16(a, cobase, t, ph, v);
            }
        }
        if (!more) break;
        tile = ntile;
        t0 = nt0; co0 = nco0; ph = nph;
        zero_acc();
        __syncthreads();   // the staged chunk is visible to every wave
    }
    if (ovf) atomicOr(a.ovf, 1);
}

// The (WM, WN, KS) candidate of launch_h for a conv (the cost model, or the test / env override).
struct Cand { int wm, wn, ks; };
static const Cand convh_cands[4] = {{2, 2, 1}, {1, 2, 2}, {1, 1, 4}, {1, 4, 1}};
static int convh_choice(const ConvArgs& a) {
    // (WM, WN, KS) by estimated time: block rounds at 2 blocks per CU x tile area
    // (4 waves share a block's work whatever KS), a small price per K-split way
    // (fits tools/convh_prof.sh on the generator's stage shapes).
    int best = -1;
    double best_cost = 1e30;
    for (int i = 0; i < 4; ++i) {
        const int bm = 32 * convh_cands[i].wm, bn = 64 * convh_cands[i].wn;
        const long blocks = (long)((a.n_t + bn - 1) / bn) * ((a.Cout + bm - 1) / bm) * (a.phases > 1 ? a.phases : 1);
        const long rounds = (blocks + 511) / 512;
        const double cost = (double)rounds * bm * bn * (1.0 + 0.1 * (convh_cands[i].ks - 1));
        if (cost < best_cost) { best_cost = cost; best = i; }
    }
    static const int forced = [] { const char* e = std::getenv("GENIE_CONVH_CFG"); return e ? std::atoi(e) : -1; }();
    if (forced >= 0 && forced < 4) best = forced;
    if (a.tile_force >= 1 && a.tile_force <= 4) best = a.tile_force - 1;
    return best;
}

// Weight-stationary form for the wide generator stages' 7- / 11-tap MRF convs (Cin = 64 / 128,
// Cout a multiple of 64, unit stride, one phase; option "convh_ws": by default only in a batch the
// caller waits for, not beside the next batch's T2S).  r06o (batch64's vocoder, `profiles/r06o_vocoder_stages.txt`):
// there k_conv_h takes 2-5x the larger of its HBM and MFMA times, because every 64 x 128 block
// stages its own copy of the chunk's weights (64 rows x taps x 32 channels, 12-45 KB) for 128
// output columns -- more bytes into LDS than its input tile.  Here a block holds its 64 output
// channels' whole weight slab [co][tap][ci] in LDS (25-116 KB, loaded once) and walks time tiles of
// 256 columns (8 waves, WM = 2 x WN = 4, each wave 32 x 64 as in k_conv_h's (2, 2, 1) form);
// per tile only the input chunks are staged (fp32 -> activation -> hi / lo -> LDS), the next
// tile's first chunk during the current tile's last MFMAs.  Each accumulator runs k_conv_h's
// MFMA sequence (chunk, then the chunk's (tap, 8-channel group) pairs), so the results are
// bit-identical to the (2, 2, 1) form the cost model picks for these shapes.
// Blocks b, b + 8, ... share an XCD (MI355X_MICROARCH.md): the Cout / 64 blocks of one tile
// sequence are placed there, so a tile's input is fetched from HBM once per XCD.
template <int KT, int CIN>
struct WsCfg {
    static constexpr int CC = 32, G8 = CC / 8, NG = KT * G8, NSTEP = NG / 2;
    static constexpr int BM = 64, BN = 256;
    static constexpr int XW = BN + (KT - 1) * DMAX;
    static constexpr int XR = CC + 8;                    // halves per X row (odd x 16 B)
    static constexpr int WR = KT * CIN + 8;              // halves per weight row (odd x 16 B)
    static constexpr int NXI = (XW * G8 + 511) / 512;
    static constexpr int X_BYTES = XW * XR * 2;
    static constexpr int W_BYTES = BM * WR * 2;
    static constexpr int LDS = 2 * X_BYTES + W_BYTES;
    static constexpr int NCH = CIN / CC;
    static_assert(NG % 2 == 0, "two 8-channel groups per MFMA step");
};

template <int KT, int CIN>
__global__ __launch_bounds__(512) void k_conv_ws(ConvArgs a, int nlanes, int ncob) {
    using C = WsCfg<KT, CIN>;
    __shared__ __attribute__((aligned(16))) char smem[C::LDS];
    _Float16* Xh = reinterpret_cast<_Float16*>(smem);
    _Float16* Xl = reinterpret_cast<_Float16*>(smem + C::X_BYTES);
    _Float16* Ws = reinterpret_cast<_Float16*>(smem + 2 * C::X_BYTES);

    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int wn = w & 3, wm = w >> 2;
    const int b = blockIdx.x;
    const int cob = (b >> 3) % ncob;                     // output-channel block
    const int ln = (b & 7) + 8 * ((b >> 3) / ncob);      // tile lane
    const int co0 = cob * C::BM;
    const int dil = a.dil;
    const int xw = C::BN + (KT - 1) * dil;
    const int ntn = (a.n_t + C::BN - 1) / C::BN;
    const float* __restrict__ isc = a.in_scale;
    const float* __restrict__ X = a.x;

    // the block's weight slab, once: rows co0 .. co0 + 63, [tap][ci] contiguous per row
    {
        const __half* src = a.wh + (long)co0 * KT * CIN;
        constexpr int PER_ROW = KT * CIN / 8;
        for (int e = tid; e < C::BM * PER_ROW; e += 512) {
            const int r = e / PER_ROW, q = e - r * PER_ROW;
            *reinterpret_cast<uint4*>(Ws + r * C::WR + q * 8) =
                *reinterpret_cast<const uint4*>(src + (long)r * KT * CIN + q * 8);
        }
    }

    int xu[C::NXI], xc[C::NXI];
#pragma unroll
    for (int i = 0; i < C::NXI; ++i) {
        const int e = tid + i * 512;
        xc[i] = e / xw;
        xu[i] = e - xc[i] * xw;
        if (xc[i] >= C::G8) xc[i] = -1;
    }
    float xr[C::NXI][8];
    bool ovf = false;
    auto load = [&](int t0, int ci0) {   // raw values (the activation is applied in store)
#pragma unroll
        for (int i = 0; i < C::NXI; ++i) {
            const int tin = t0 - a.pad + xu[i];
            const bool ok = xc[i] >= 0 && tin >= 0 && tin < a.Tin;
            const float* src = X + (long)(ci0 + xc[i] * 8) * a.x_cs + tin;
#pragma unroll
            for (int j = 0; j < 8; ++j) xr[i][j] = ok ? src[(long)j * a.x_cs] : 0.f;
        }
    };
    auto store = [&](int cis) {
#pragma unroll
        for (int i = 0; i < C::NXI; ++i) {
            if (xc[i] < 0) continue;
            if (a.in_act) {
#pragma unroll
                for (int j = 0; j < 8; ++j) xr[i][j] = xr[i][j] >= 0.f ? xr[i][j] : xr[i][j] * a.in_slope;
            }
            if (isc) {
#pragma unroll
                for (int j = 0; j < 8; ++j) xr[i][j] *= isc[cis + xc[i] * 8 + j];
            }
            float m = 0.f;
#pragma unroll
            for (int j = 0; j < 8; ++j) m = fmaxf(m, fabsf(xr[i][j]));
            ovf |= m > 65504.f;
            uint4 hi, lo;
            split8(xr[i], hi, lo);
            *reinterpret_cast<uint4*>(Xh + xu[i] * C::XR + xc[i] * 8) = hi;
            *reinterpret_cast<uint4*>(Xl + xu[i] * C::XR + xc[i] * 8) = lo;
        }
    };

    f32x16 acc[2];
    auto zero_acc = [&]() {
#pragma unroll
        for (int f = 0; f < 2; ++f)
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[f][i] = 0.f;
    };
    zero_acc();
    const int r32 = lane & 31, hsel = lane >> 5;
    int tile = ln;
    if (tile >= ntn) return;   // block-uniform: no barrier is skipped by part of a block
    int t0 = tile * C::BN;
    load(t0, 0);
    store(0);
    __syncthreads();   // weights and the first chunk
    for (;;) {
        const int ntile = tile + nlanes;
        const bool more = ntile < ntn;
        const int nt0 = ntile * C::BN;
        for (int c = 0; c < C::NCH; ++c) {
            const bool last = c + 1 == C::NCH;
            if (!last) load(t0, (c + 1) * C::CC);
            else if (more) load(nt0, 0);
            // the weight rows' offset for this chunk, opaque: re-formed per chunk, not hoisted
            int wro = (wm * 32 + r32) * C::WR + c * C::CC;
            asm volatile("" : "+v"(wro));
            const _Float16* wrow = Ws + wro;
#pragma unroll
            for (int j = 0; j < C::NSTEP; ++j) {
                const int g = 2 * j + hsel;
                const int tap = g / C::G8, c8 = g - tap * C::G8;
                const h8 A = *reinterpret_cast<const h8*>(wrow + tap * CIN + c8 * 8);
#pragma unroll
                for (int f = 0; f < 2; ++f) {
                    const int row = wn * 64 + f * 32 + r32 + tap * dil;
                    const h8 Bl = *reinterpret_cast<const h8*>(Xl + row * C::XR + c8 * 8);
                    const h8 Bh = *reinterpret_cast<const h8*>(Xh + row * C::XR + c8 * 8);
                    acc[f] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A, Bl, acc[f], 0, 0, 0);
                    acc[f] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A, Bh, acc[f], 0, 0, 0);
                }
            }
            __syncthreads();
            if (!last) {
                store((c + 1) * C::CC);
                __syncthreads();
            } else if (more) {
                store(0);   // the next tile's first chunk, into the X this tile no longer reads
            }
        }
        {
            const int cobase = co0 + wm * 32 + 4 * hsel;
            float sc[16];
#pragma unroll
            for (int r = 0; r < 16; ++r) sc[r] = a.wscale[cobase + (r & 3) + 8 * (r >> 2)];
#pragma unroll
            for (int f = 0; f < 2; ++f) {
                const int t = t0 + wn * 64 + f * 32 + r32;
                if (t >= a.n_t) continue;
                float v[16];
#pragma unroll
                for (int r = 0; r < 16; ++r) v[r] = acc[f][r] * sc[r];
                conv_epilogue16_lean(a, cobase, t, 0, v);
            }
        }
        if (!more) break;
        tile = ntile;
        t0 = nt0;
        zero_acc();
        __syncthreads();   // the staged chunk is visible to every wave
    }
    if (ovf) atomicOr(a.ovf, 1);
}

template <int KT, int CIN>
void launch_ws(const ConvArgs& a, hipStream_t s) {
    // one block per CU (8 waves; ~190-240 VGPRs, so a second block would not be resident)
    const int ncob = a.Cout / 64;
    int lanes = (a.ws / (8 * ncob)) * 8;   // a multiple of 8: whole XCD rounds
    if (lanes < 8) lanes = 8;
    hipLaunchKernelGGL((k_conv_ws<KT, CIN>), dim3(lanes * ncob), dim3(512), 0, s, a, lanes, ncob);
}

// The weight-stationary form covers the 7- and 11-tap MRF convs of the Cin = 64 stage and the
// 7-tap ones of Cin = 128 (the 11-tap slab of 64 x 128 channels would need 181 KB of LDS), with
// >= 2 tiles per lane.  The 3-tap convs stay on k_conv_h: there the per-tile staging and epilogue
// outweigh the MFMAs and one block per CU hides them worse than k_conv_h's two (r06p: 549 / 389 us
// against 417 / 328 at Cin 128 / 64).
template <int KT>
bool try_ws(const ConvArgs& a, hipStream_t s) {
    if constexpr (KT == 7 || KT == 11) {
        if (a.ws <= 0 || a.phases > 1 || a.o_tstride != 1 || a.o_toff != 0 || a.Cout % 64 != 0 ||
            a.Cout != a.Cin ||
            !(a.mode == CV_STORE || a.mode == CV_RESID || a.mode == CV_ACC_FIRST || a.mode == CV_ACC_ADD ||
              a.mode == CV_ACC_MEAN))
            return false;
        if ((a.n_t + 255) / 256 < 2L * a.ws) return false;   // >= 2 tiles per lane
        // only where k_conv_h would run its (2, 2, 1) form, whose MFMA sequence k_conv_ws runs: the
        // same bits either way (a K-split form sums in another order)
        if (convh_choice(a) != 0) return false;
        if (a.Cin == 64) {
            launch_ws<KT, 64>(a, s);
            return true;
        }
        if constexpr (KT <= 7) {
            if (a.Cin == 128) {
                launch_ws<KT, 128>(a, s);
                return true;
            }
        }
    }
    return false;
}

template <int KT, int CC>
bool launch_h(const ConvArgs& a, hipStream_t s) {
    const Cand* cands = convh_cands;
    const int best = convh_choice(a);
    const Cand c = cands[best];
    const dim3 grid((a.n_t + 64 * c.wn - 1) / (64 * c.wn), (a.Cout + 32 * c.wm - 1) / (32 * c.wm),
                    a.phases > 1 ? a.phases : 1);
    // the persistent form: two blocks per CU over the tiles, when there are >= 4 rounds of them
    const long nblk = (long)grid.x * grid.y * grid.z;
    const bool lean = a.mode == CV_STORE || a.mode == CV_RESID || a.mode == CV_ACC_FIRST || a.mode == CV_ACC_ADD ||
                      a.mode == CV_ACC_MEAN;
    if (a.persist > 0 && c.ks == 1 && lean && nblk >= 4L * 2 * a.persist) {
        const dim3 pg((unsigned)(2 * a.persist));
        if (c.wm == 2) hipLaunchKernelGGL((k_conv_h<KT, CC, 2, 2, 1, 1, true>), pg, dim3(256), 0, s, a);
        else hipLaunchKernelGGL((k_conv_h<KT, CC, 1, 4, 1, 1, true>), pg, dim3(256), 0, s, a);
        return true;
    }
    if (c.wm == 2) hipLaunchKernelGGL((k_conv_h<KT, CC, 2, 2, 1>), grid, dim3(256), 0, s, a);
    else if (c.ks == 2) hipLaunchKernelGGL((k_conv_h<KT, CC, 1, 2, 2>), grid, dim3(256), 0, s, a);
    else if (c.ks == 4) hipLaunchKernelGGL((k_conv_h<KT, CC, 1, 1, 4>), grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((k_conv_h<KT, CC, 1, 4, 1>), grid, dim3(256), 0, s, a);
    return true;
}

// Long-time form (the batched generator: 10^5-10^7 columns): 128 x 128 output blocks,
// each wave 64 output channels x 64 columns (WTM = 2); 16-channel K-chunks for the
// 7- and 11-tap convs keep the weight tile at 31-47 KB, two blocks per CU.  Off by default
// (GENIE_CONVH_BIG=1 turns it on): alone it makes a 64-sentence vocoder pass 3 % faster,
// but beside the next batch's prefill (the batched pipeline) its long blocks hold the CUs
// and the prefill's short GEMM launches wait -- batch64 321 -> 296 utt/s, mixed100
// 277 -> 253 (profiles/r04m_convh_big.txt).
static bool convh_big() {
    static const bool on = [] { const char* e = std::getenv("GENIE_CONVH_BIG"); return e && std::atoi(e) != 0; }();
    return on;
}
// Cout = 64 (not a multiple of 128): 64 x 256 blocks, four waves side by side in time.
template <int KT>
bool launch_big(const ConvArgs& a, hipStream_t s) {
    constexpr int CC = KT >= 7 ? 16 : 32;
    if (a.Cin % CC != 0) return false;
    const int z = a.phases > 1 ? a.phases : 1;
    if (a.Cout % 128 == 0) {
        const dim3 grid((a.n_t + 127) / 128, a.Cout / 128, z);
        hipLaunchKernelGGL((k_conv_h<KT, CC, 2, 2, 1, 2>), grid, dim3(256), 0, s, a);
    } else {
        const dim3 grid((a.n_t + 255) / 256, a.Cout / 64, z);
        hipLaunchKernelGGL((k_conv_h<KT, CC, 1, 4, 1, 2>), grid, dim3(256), 0, s, a);
    }
    return true;
}

template <int KT>
bool launch_kt(const ConvArgs& a, hipStream_t s) {
    const int z = a.phases > 1 ? a.phases : 1;
    if (try_ws<KT>(a, s)) return true;
    if (convh_big() && a.Cout % 64 == 0 &&
        (a.Cout % 128 == 0 ? (long)((a.n_t + 127) / 128) * (a.Cout / 128) * z
                           : (long)((a.n_t + 255) / 256) * (a.Cout / 64) * z) >= 1024 &&
        launch_big<KT>(a, s))
        return true;
    if (a.Cin % 32 == 0) return launch_h<KT, 32>(a, s);
    if (a.Cin % 8 == 0) return launch_h<KT, 8>(a, s);
    return false;
}

}  // namespace

bool conv1d_h(const ConvArgs& a, hipStream_t s) {
    if (!a.wh || !a.wscale || !a.ovf) return false;
    // a plain conv (one phase, unit output stride) or a ConvTranspose's polyphase form
    // (phases = output stride; dilation 1)
    const bool poly = a.phases > 1;
    if (poly ? (a.o_tstride != a.phases || a.dil != 1) : a.o_tstride != 1) return false;
    if (a.x_ts != 1 || a.dil < 1 || a.dil > DMAX) return false;
    if ((reinterpret_cast<uintptr_t>(a.wh) & 15) != 0) return false;
    switch (a.K) {
        case 1: return launch_kt<1>(a, s);
        case 2: return launch_kt<2>(a, s);
        case 4: return launch_kt<4>(a, s);
        case 3: return launch_kt<3>(a, s);
        case 7: return launch_kt<7>(a, s);
        case 11: return launch_kt<11>(a, s);
        default: return false;
    }
}

}  // namespace gsv
