// One HiFi-GAN ResBlock1 step of the narrow generator stages as ONE kernel:
//   y = e( conv2( lrelu( conv1_d( lrelu(r) ) ) ) , r )
// (vits_fp32.onnx dec.resblocks.*: convs1[i] kernel k dilation d_i, convs2[i] kernel k
// dilation 1, both C -> C with weight norm; e = the residual / MRF accumulation epilogue
// of conv2).  For the C <= 32 stages the two convs are byte-bound: run separately, conv1
// writes the intermediate xt and conv2 reads it back (5 passes over a C x T array); here
// xt lives in LDS only (2 passes: r with its halo in, y out).
//
// A block step = 224 output columns x all C channels, 8 waves.  Conv1 runs on the xt columns
// [t0 - p2, t0 + 224 + p2) (p2 = (k-1)/2, conv2's halo; 8 tiles of 32 columns), conv2 on
// the 224 output columns (7 tiles); blocks are persistent over the steps.  Both are implicit GEMMs on
// v_mfma_f32_32x32x16_f16 with split fp32 activations (x = hi + lo, two MFMAs per K step)
// and the fp16 weights held in LDS, exactly as k_conv_h (vits_convh.hip).  xt gets conv1's
// epilogue of the unfused path: weight-norm scale, bias, zero outside [0, T) and in the gap
// columns of a segmented batch, then conv2's input activation.
// Range guard: an activation beyond the fp16 range sets *ovf (the host re-runs on f32).
#include "common.h"
#include "vits.h"
#include "vits_epi.h"

#include <algorithm>

namespace gsv {
namespace {

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef _Float16 h4 __attribute__((ext_vector_type(4)));
constexpr int NT2 = 7;             // conv2 tiles of 32 output columns per block step
constexpr int BN = 32 * NT2;       // output columns per block step
constexpr int NT1 = NT2 + 1;       // conv1 tiles: BN + 2 p2 <= BN + 10 xt columns
constexpr int DMAXM = 5;           // largest dilation
constexpr int NTH = 512;           // 8 waves: one conv1 tile and one conv2 tile each

template <int K, int C>
struct MCfg {
    static constexpr int G8 = C / 8;                          // 8-channel groups
    static constexpr int XW = NT1 * 32 + (K - 1) * DMAXM;     // r rows staged (time)
    static constexpr int XR = C == 16 ? 24 : C + 8;           // halves per row (odd x 16 B)
    static constexpr int TW = NT1 * 32;                       // xt rows
    static constexpr int WR = K * C + 8;                      // halves per weight row
    static constexpr int X_BYTES = XW * XR * 2, T_BYTES = TW * XR * 2, W_BYTES = C * WR * 2;
    static constexpr int LDS = 2 * X_BYTES + 2 * T_BYTES + 2 * W_BYTES;
    static constexpr int NXI = (XW * G8 + NTH - 1) / NTH;     // r staging items per thread
    static constexpr int KS = C / 16;                         // MFMA K steps per tap
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

// conv2's epilogue for the four modes an MRF step uses (the generic conv_epilogue16 costs
// ~150 VGPRs here): rows co = cobase + (r & 3) + 8 (r >> 2) of output column t < T,
// arithmetic order as conv_epilogue16_ (bias + sum, res + y, acc + y, / div); a gap
// column of a segmented batch is written as zeros.
template <int C>
__device__ __forceinline__ void mrf_epilogue(const ConvArgs& e, int cobase, int t, const f32x16& acc,
                                             const float* s2) {
    const long T = e.o_cs;
    const int mode = e.mode;
    float* dst = (mode == CV_ACC_FIRST || mode == CV_ACC_ADD ? e.acc : e.out) + (long)cobase * T + t;
    if (e.seg && e.seg[t] < 0) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int d = (r & 3) + 8 * (r >> 2);
            if (cobase + d < C) dst[d * T] = 0.f;
        }
        return;
    }
    const float* R = e.res + (long)cobase * T + t;
    float y[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int d = (r & 3) + 8 * (r >> 2);
        y[r] = cobase + d < C ? R[d * T] + (e.bias[cobase + d] + acc[r] * s2[cobase + d]) : 0.f;
    }
    if (mode == CV_ACC_ADD || mode == CV_ACC_MEAN) {
        const float* A = e.acc + (long)cobase * T + t;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int d = (r & 3) + 8 * (r >> 2);
            if (cobase + d < C) y[r] = A[d * T] + y[r];
        }
        if (mode == CV_ACC_MEAN) {
#pragma unroll
            for (int r = 0; r < 16; ++r) y[r] = y[r] / e.div;
        }
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int d = (r & 3) + 8 * (r >> 2);
        if (cobase + d < C) dst[d * T] = y[r];
    }
}

// Persistent over column steps: the weights are staged once per block, and the next step's r
// tile is loaded into registers while the current one's MFMAs run.
template <int K, int C>
__global__ __launch_bounds__(NTH) void k_mrf_pair(MrfPairArgs a, int nsteps) {
    using M = MCfg<K, C>;
    __shared__ __attribute__((aligned(16))) char smem[M::LDS];
    _Float16* Xh = reinterpret_cast<_Float16*>(smem);
    _Float16* Xl = Xh + M::X_BYTES / 2;
    _Float16* Th = Xl + M::X_BYTES / 2;
    _Float16* Tl = Th + M::T_BYTES / 2;
    _Float16* W1 = Tl + M::T_BYTES / 2;
    _Float16* W2 = W1 + M::W_BYTES / 2;

    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int r32 = lane & 31, hsel = lane >> 5;
    const int d = a.dil, p1 = d * (K - 1) / 2, p2 = (K - 1) / 2;
    const int T = a.T;
    const float slope = 0.1f;
    bool ovf = false;
    const int xw = NT1 * 32 + (K - 1) * d;

    // per-thread staging items (loop invariant): item e -> (group c8, row u)
    int xu[M::NXI], xc[M::NXI];
#pragma unroll
    for (int i = 0; i < M::NXI; ++i) {
        const int e = tid + i * NTH;
        xc[i] = e / xw;
        xu[i] = e - xc[i] * xw;
        if (xc[i] >= M::G8) xc[i] = -1;
    }
    float xr[M::NXI][8];
    auto load = [&](int step) {   // raw r of the step's rows (activation in store)
        const int tx0 = step * BN - p2 - p1;
#pragma unroll
        for (int i = 0; i < M::NXI; ++i) {
            const int t = tx0 + xu[i];
            const bool ok = xc[i] >= 0 && t >= 0 && t < T;
            const float* src = a.r + (long)(xc[i] * 8) * T + t;
#pragma unroll
            for (int j = 0; j < 8; ++j) xr[i][j] = ok ? src[(long)j * T] : 0.f;
        }
    };
    auto store = [&]() {
#pragma unroll
        for (int i = 0; i < M::NXI; ++i) {
            if (xc[i] < 0) continue;
            float m = 0.f;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                xr[i][j] = xr[i][j] >= 0.f ? xr[i][j] : xr[i][j] * slope;
                m = fmaxf(m, fabsf(xr[i][j]));
            }
            ovf |= m > 65504.f;
            uint4 hi, lo;
            split8(xr[i], hi, lo);
            *reinterpret_cast<uint4*>(Xh + xu[i] * M::XR + xc[i] * 8) = hi;
            *reinterpret_cast<uint4*>(Xl + xu[i] * M::XR + xc[i] * 8) = lo;
        }
    };

    int step = blockIdx.x;
    if (step < nsteps) load(step);
    for (int e = tid; e < 2 * C * K * M::G8; e += NTH) {   // both weight sets, once: [co][tap][ci]
        const int which = e / (C * K * M::G8), q = e - which * (C * K * M::G8);
        const int co = q / (K * M::G8), rem = q - co * K * M::G8;
        const int tap = rem / M::G8, c8 = rem - tap * M::G8;
        const __half* src = (which ? a.w2 : a.w1) + ((long)co * K + tap) * C + c8 * 8;
        *reinterpret_cast<uint4*>((which ? W2 : W1) + co * M::WR + tap * C + c8 * 8) =
            *reinterpret_cast<const uint4*>(src);
    }
    const bool arow = r32 < C;   // C = 16: the upper 16 A rows are zero
    const int wrow0 = (arow ? r32 : 0) * M::WR;

    for (; step < nsteps; step += gridDim.x) {
        const int t0 = step * BN;
        // the weight rows' LDS offset, opaque per step: the A fragments are re-read from LDS in
        // every step instead of being hoisted into ~170 registers (which spilled at 8 waves)
        int wro = wrow0;
        asm volatile("" : "+v"(wro));
        const _Float16* w1row = W1 + wro;
        const _Float16* w2row = W2 + wro;
        store();                  // X of this step (the previous step's conv1 read X before its barrier)
        __syncthreads();          // ... and every wave is past the previous step's conv2 (T free)
        if (step + (int)gridDim.x < nsteps) load(step + gridDim.x);   // in flight across the MFMAs

        // conv1 on xt tile n = w
        {
            const int n = w;
            f32x16 acc;
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[i] = 0.f;
#pragma unroll
            for (int tap = 0; tap < K; ++tap)
#pragma unroll
                for (int ks = 0; ks < M::KS; ++ks) {
                    const int c0 = ks * 16 + hsel * 8;
                    h8 A = *reinterpret_cast<const h8*>(w1row + tap * C + c0);
                    if (!arow) A = (h8){0, 0, 0, 0, 0, 0, 0, 0};
                    const int row = n * 32 + r32 + tap * d;
                    const h8 Bl = *reinterpret_cast<const h8*>(Xl + row * M::XR + c0);
                    const h8 Bh = *reinterpret_cast<const h8*>(Xh + row * M::XR + c0);
                    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(A, Bl, acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(A, Bh, acc, 0, 0, 0);
                }
            // xt epilogue (column j at time t0 - p2 + j): scale, bias, zero outside [0, T) and in
            // gap columns, lrelu -> fp16 hi/lo planes, 4 channels per store
            const int j = n * 32 + r32;
            const int t = t0 - p2 + j;
            const bool live = t >= 0 && t < T && (!a.e.seg || a.e.seg[t] >= 0);
#pragma unroll
            for (int q = 0; q < 4; ++q) {           // acc rows 4q..4q+3: co = 8q + 4 hsel + (0..3)
                const int cb = 8 * q + 4 * hsel;
                if (cb >= C) continue;
                _Float16 hh[4], ll[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const int co = cb + k;
                    float v = live ? acc[4 * q + k] * a.s1[co] + a.b1[co] : 0.f;
                    v = v >= 0.f ? v : v * slope;
                    ovf |= fabsf(v) > 65504.f;
                    hh[k] = (_Float16)v;
                    ll[k] = (_Float16)(v - (float)hh[k]);
                }
                *reinterpret_cast<h4*>(Th + j * M::XR + cb) = *reinterpret_cast<const h4*>(hh);
                *reinterpret_cast<h4*>(Tl + j * M::XR + cb) = *reinterpret_cast<const h4*>(ll);
            }
        }
        __syncthreads();

        // conv2 on output tile n = w (< NT2)
        if (w < NT2) {
            const int n = w;
            f32x16 acc;
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[i] = 0.f;
#pragma unroll
            for (int tap = 0; tap < K; ++tap)
#pragma unroll
                for (int ks = 0; ks < M::KS; ++ks) {
                    const int c0 = ks * 16 + hsel * 8;
                    h8 A = *reinterpret_cast<const h8*>(w2row + tap * C + c0);
                    if (!arow) A = (h8){0, 0, 0, 0, 0, 0, 0, 0};
                    const int row = n * 32 + r32 + tap;
                    const h8 Bl = *reinterpret_cast<const h8*>(Tl + row * M::XR + c0);
                    const h8 Bh = *reinterpret_cast<const h8*>(Th + row * M::XR + c0);
                    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(A, Bl, acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(A, Bh, acc, 0, 0, 0);
                }
            const int t = t0 + n * 32 + r32;
            const int cobase = 4 * hsel;
            if (t < T && cobase < C) mrf_epilogue<C>(a.e, cobase, t, acc, a.s2);
        }
    }
    if (ovf) atomicOr(a.ovf, 1);
}

template <int K, int C>
void launch(const MrfPairArgs& a, hipStream_t s) {
    const int nsteps = (a.T + BN - 1) / BN;
    // one block per CU (the LDS of the C = 32 forms; C = 16 fits two): blocks loop over the steps
    const int per_cu = MCfg<K, C>::LDS <= 80 * 1024 ? 2 : 1;
    const int grid = std::min(nsteps, 256 * per_cu);
    hipLaunchKernelGGL((k_mrf_pair<K, C>), dim3(grid), dim3(NTH), 0, s, a, nsteps);
}

}  // namespace

bool mrf_pair(const MrfPairArgs& a, hipStream_t s) {
    if (!a.w1 || !a.w2 || !a.s1 || !a.s2 || !a.ovf || a.dil < 1 || a.dil > DMAXM) return false;
    if (a.e.o_tstride != 1 || a.e.o_toff != 0 || a.e.o_ts != 1 || a.e.o_cs != a.T || a.e.Cout != a.C ||
        a.e.n_t != a.T || a.e.o_len != a.T || !a.e.bias || !a.e.res || a.e.r_cs != a.T || a.e.r_ts != 1)
        return false;
    if (a.e.mode != CV_RESID && a.e.mode != CV_ACC_FIRST && a.e.mode != CV_ACC_ADD && a.e.mode != CV_ACC_MEAN)
        return false;
    const int key = a.K * 100 + a.C;
    switch (key) {
        case 332: launch<3, 32>(a, s); return true;
        case 732: launch<7, 32>(a, s); return true;
        case 1132: launch<11, 32>(a, s); return true;
        case 316: launch<3, 16>(a, s); return true;
        case 716: launch<7, 16>(a, s); return true;
        case 1116: launch<11, 16>(a, s); return true;
        default: return false;
    }
}

}  // namespace gsv
