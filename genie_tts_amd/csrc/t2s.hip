// T2S kernels for gfx950: f32-MFMA GEMM (prefill / encoder), batched fp16-weight
// GEMV with fused LayerNorm prologue (decode), prefix attention, sampler.
//
// Numerics follow the reference graphs (fp32 activations, fp16-valued weights
// upcast exactly as g/ModelManager.py:75-76): t2s_first_stage_decoder_fp32.onnx
// and t2s_stage_decoder_fp32.onnx (node indices cited per kernel).
#include "common.h"
#include "kernels.h"
#include "prefill_attn.h"
#include "sampler.h"
#include <cstdio>
#include <cstdlib>

namespace gsv {

// =====================================================================
// GEMM NT:  C(m,n) = sum_k A(m,k) W(n,k)  via v_mfma_f32_32x32x2_f32
// (exact f32 FMA chain, 157 TF/s peak).  Block tile 64x64, 4 waves of 32x32,
// K-step 32 staged through padded LDS (stride 33 -> conflict-free b32 reads).
// =====================================================================
// Shared GEMM epilogue: 32x32 accumulator tile of rows [row0, row0+32), column col.
__device__ __forceinline__ void gemm_epilogue(const GemmArgs& a, int row0, int col, int lane, const f32x16& acc) {
    if (col >= a.N) return;
    const float bv = a.bias ? a.bias[col] : 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int row = row0 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (row >= a.M) continue;
        const float v = a.bias ? bv + acc[r] : acc[r];   // Add(bias, MatMul)
        switch (a.mode) {
            case EPI_STORE: a.C[(long)row * a.ldc + col] = v; break;
            case EPI_RELU: a.C[(long)row * a.ldc + col] = fmaxf(v, 0.f); break;
            case EPI_RELU_SPLIT: {   // the consumer GEMM's split of the f32 value, done here
                float x = fmaxf(v, 0.f);
                asm volatile("" : "+v"(x));   // materialised f32: no conversion fused into its producers
                const _Float16 h = (_Float16)x;
                reinterpret_cast<_Float16*>(a.Ch)[(long)row * a.ldc + col] = h;
                reinterpret_cast<_Float16*>(a.Cl)[(long)row * a.ldc + col] = (_Float16)(x - (float)h);
            } break;
            case EPI_GELU: a.C[(long)row * a.ldc + col] = 0.5f * v * (1.f + erff(v * 0.70710678118654752f)); break;
            case EPI_RESID: a.C[(long)row * a.ldc + col] = a.res[(long)row * a.ldr + col] + v; break;
            case EPI_MISH: {
                const float sp = v > 0.f ? v + log1pf(expf(-v)) : log1pf(expf(v));
                a.C[(long)row * a.ldc + col] = v * tanhf(sp);
            } break;
            case EPI_VQDIST:   // (sum h^2) - (2h).c + (sum c^2); x2 is exact so (2h).c == 2(h.c)
                a.C[(long)row * a.ldc + col] = (a.rowsq[row] - 2.0f * acc[r]) + a.colsq[col];
                break;
            case EPI_QKV: {
                if (col < 512) {
                    a.C[(long)row * a.ldc + col] = v;
                } else {
                    if (a.kv.row_skip && a.kv.row_skip[a.kv.row_seq ? a.kv.row_seq[row] : 0]) break;
                    const int seq = a.kv.row_seq ? a.kv.row_seq[row] : 0;
                    const int pos = a.kv.row_pos ? a.kv.row_pos[row] : a.kv.pos0 + row;
                    const int c = (col - 512) & 511;
                    float* dst = (col < 1024 ? a.kv.k : a.kv.v) + (long)seq * a.kv.seq_stride;
                    dst[((long)(c >> 5) * a.kv.tmax + pos) * 32 + (c & 31)] = v;
                }
            } break;
        }
    }
}

template <bool F16W>
__global__ __launch_bounds__(256) void k_gemm_nt(GemmArgs a) {
    __shared__ float As[64][33];
    __shared__ float Ws[64][33];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int wm = w >> 1, wn = w & 1;
    const int m0 = blockIdx.y * 64, n0 = blockIdx.x * 64;
    f32x16 acc;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = 0.f;
    const int sr = tid >> 2, sc = (tid & 3) * 8;
    const int gm = m0 + sr, gn = n0 + sr;
    for (int k0 = 0; k0 < a.K; k0 += 32) {
        float av[8], wv[8];
        if (gm < a.M) {
            const float4* p = reinterpret_cast<const float4*>(a.A + (long)gm * a.lda + k0 + sc);
            float4 x0 = p[0], x1 = p[1];
            av[0] = x0.x; av[1] = x0.y; av[2] = x0.z; av[3] = x0.w;
            av[4] = x1.x; av[5] = x1.y; av[6] = x1.z; av[7] = x1.w;
        } else {
#pragma unroll
            for (int i = 0; i < 8; ++i) av[i] = 0.f;
        }
        if (gn < a.N) {
            if (F16W) {
                const __half* wp = reinterpret_cast<const __half*>(a.W) + (long)gn * a.ldw + k0 + sc;
                h8_to_f8(*reinterpret_cast<const uint4*>(wp), wv);
            } else {
                const float4* p = reinterpret_cast<const float4*>(
                    reinterpret_cast<const float*>(a.W) + (long)gn * a.ldw + k0 + sc);
                float4 x0 = p[0], x1 = p[1];
                wv[0] = x0.x; wv[1] = x0.y; wv[2] = x0.z; wv[3] = x0.w;
                wv[4] = x1.x; wv[5] = x1.y; wv[6] = x1.z; wv[7] = x1.w;
            }
        } else {
#pragma unroll
            for (int i = 0; i < 8; ++i) wv[i] = 0.f;
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            As[sr][sc + i] = av[i];
            Ws[sr][sc + i] = wv[i];
        }
        __syncthreads();
#pragma unroll
        for (int kk = 0; kk < 16; ++kk) {
            const float x = As[wm * 32 + (lane & 31)][2 * kk + (lane >> 5)];
            const float y = Ws[wn * 32 + (lane & 31)][2 * kk + (lane >> 5)];
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(x, y, acc, 0, 0, 0);
        }
        __syncthreads();
    }
    gemm_epilogue(a, m0 + wm * 32, n0 + wn * 32 + (lane & 31), lane, acc);
}

// =====================================================================
// GEMM NT with fp16 weights on the f16 MFMA (v_mfma_f32_32x32x16_f16, 16x the
// f32-MFMA rate): the weights are exactly fp16 (the reference's own values), the
// f32 activations are split a = a_hi + a_lo into two fp16 terms, so
// sum_k a*w = sum_k a_hi*w + sum_k a_lo*w with f32 accumulation -- the dropped
// residual is ~2^-22 |a|, i.e. f32-level accuracy.  64x64 block tile, 4 waves
// of 32x32, K-steps of 64 staged through LDS with the next step prefetched
// into registers while the MFMAs run.
// =====================================================================
typedef _Float16 h16x8 __attribute__((ext_vector_type(8)));
#define GX_KS 128
__device__ __forceinline__ void split8(const float4 x0, const float4 x1, h16x8& hi, h16x8& lo) {
    const float v[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const _Float16 hj = (_Float16)v[j];
        hi[j] = hj;
        lo[j] = (_Float16)(v[j] - (float)hj);
    }
}

struct GxRegs {
    float4 a[8];   // 64 rows x 128 k f32 = 2048 float4, 8 per thread
    uint4 w[4];    // 64 rows x 128 k f16 = 1024 uint4, 4 per thread
};

__global__ __launch_bounds__(256) void k_gemm_x2(GemmArgs a) {
    __shared__ float As[64][GX_KS + 4];
    __shared__ __half Ws[64][GX_KS + 8];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int wm = w >> 1, wn = w & 1;
    const int m0 = blockIdx.y * 64, n0 = blockIdx.x * 64;
    const int r = lane & 31, hh = lane >> 5;
    // K slice of this block (split-K over grid.z); slices are whole K-steps
    const int nsplit = gridDim.z, kz = blockIdx.z;
    const int steps_all = a.K / GX_KS;
    const int s_lo = kz * steps_all / nsplit, s_hi = (kz + 1) * steps_all / nsplit;
    const int nsteps = s_hi - s_lo;
    f32x16 acc;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = 0.f;
    auto load = [&](GxRegs& R, int step) {
        const int k0 = step * GX_KS;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int e = tid + 256 * i, row = e >> 5, kc = (e & 31) * 4;
            const int gm = m0 + row;
            if (a.a_nslab > 0) {
                // A = relu?(bias + sum of the producer's split-K slabs), summed in slab order
                float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
                if (gm < a.M) {
                    const float* src = a.A + (long)gm * a.lda + k0 + kc;
                    v = *reinterpret_cast<const float4*>(src);
                    for (int z = 1; z < a.a_nslab; ++z) {
                        const float4 u = *reinterpret_cast<const float4*>(src + z * a.a_slab_stride);
                        v.x += u.x; v.y += u.y; v.z += u.z; v.w += u.w;
                    }
                    const float4 bb = *reinterpret_cast<const float4*>(a.a_bias + k0 + kc);
                    v = make_float4(bb.x + v.x, bb.y + v.y, bb.z + v.z, bb.w + v.w);
                    if (a.a_relu)
                        v = make_float4(fmaxf(v.x, 0.f), fmaxf(v.y, 0.f), fmaxf(v.z, 0.f), fmaxf(v.w, 0.f));
                }
                R.a[i] = v;
            } else {
                R.a[i] = gm < a.M ? *reinterpret_cast<const float4*>(a.A + (long)gm * a.lda + k0 + kc)
                                  : make_float4(0.f, 0.f, 0.f, 0.f);
            }
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int e = tid + 256 * i, row = e >> 4, kc = (e & 15) * 8;
            const int gn = n0 + row;
            R.w[i] = gn < a.N ? *reinterpret_cast<const uint4*>(reinterpret_cast<const __half*>(a.W) +
                                                                 (long)gn * a.ldw + k0 + kc)
                              : make_uint4(0u, 0u, 0u, 0u);
        }
    };
    auto store = [&](const GxRegs& R) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int e = tid + 256 * i, row = e >> 5, kc = (e & 31) * 4;
            *reinterpret_cast<float4*>(&As[row][kc]) = R.a[i];
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int e = tid + 256 * i, row = e >> 4, kc = (e & 15) * 8;
            *reinterpret_cast<uint4*>(&Ws[row][kc]) = R.w[i];
        }
    };
    auto compute = [&]() {
#pragma unroll
        for (int ks = 0; ks < GX_KS / 16; ++ks) {
            const float* ap = &As[wm * 32 + r][ks * 16 + 8 * hh];
            const float4 x0 = *reinterpret_cast<const float4*>(ap);
            const float4 x1 = *reinterpret_cast<const float4*>(ap + 4);
            h16x8 ahi, alo;
            split8(x0, x1, ahi, alo);
            const h16x8 bw = *reinterpret_cast<const h16x8*>(&Ws[wn * 32 + r][ks * 16 + 8 * hh]);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ahi, bw, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(alo, bw, acc, 0, 0, 0);
        }
    };
    // two K-steps in flight: R0 holds even steps, R1 odd ones
    GxRegs R0, R1;
    if (nsteps > 0) load(R0, s_lo);
    if (nsteps > 1) load(R1, s_lo + 1);
    for (int s = 0; s < nsteps; s += 2) {
        store(R0);
        __syncthreads();
        if (s + 2 < nsteps) load(R0, s_lo + s + 2);
        compute();
        __syncthreads();
        if (s + 1 < nsteps) {
            store(R1);
            __syncthreads();
            if (s + 3 < nsteps) load(R1, s_lo + s + 3);
            compute();
            __syncthreads();
        }
    }
    if (a.mode == EPI_SLAB) {
        const int col = n0 + wn * 32 + r;
        if (col >= a.N) return;
        float* C = a.C + (long)kz * a.slab_stride;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int row = m0 + wm * 32 + (i & 3) + 8 * (i >> 2) + 4 * hh;
            if (row < a.M) C[(long)row * a.ldc + col] = acc[i];
        }
        return;
    }
    gemm_epilogue(a, m0 + wm * 32, n0 + wn * 32 + r, lane, acc);
}

// =====================================================================
// The same GEMM (identical MFMA sequence and split-K partition, so identical
// results) with the operand tiles brought in by LDS-DMA (global_load_lds_dwordx4:
// no VGPR staging) through a GX3_NS-deep ring of 64-k stages: GX3_NS - 1 stages
// are in flight while one is consumed, so a block pays the HBM/L2 latency once
// instead of once per K-step (k_gemm_x2 keeps two 128-k steps in registers and
// waits on each).  One DMA instruction writes 1 KB of LDS (lane i -> bytes
// [16 i, 16 i + 16)), so rows cannot be padded: the 16-byte chunks of a row are
// XOR-swizzled instead (A: chunk c of row r in slot c ^ (r & 15); W: slot
// c ^ ((n >> 1) & 7)), which keeps the MFMA fragment reads conflict-free.
// Rows past M / N read row M - 1 / N - 1 (their results are never stored).
// =====================================================================
// vmcnt(later * D): the wave's DMA instructions of the `later` newest stages may stay in flight
template <int D>
__device__ __forceinline__ void gx3_wait(int later) {
    switch (later) {
        case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
        // (a ring of NS stages asks for later <= NS - 2 only; the counts of the cases a
        // configuration cannot reach are clamped to the counter's 6 bits so they assemble)
        case 1: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(D < 63 ? D : 63) : "memory"); break;
        case 2: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * D < 63 ? 2 * D : 63) : "memory"); break;
        case 3: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * D < 63 ? 3 * D : 63) : "memory"); break;
        default: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * D < 63 ? 4 * D : 63) : "memory"); break;
    }
}
// One global -> LDS DMA of 16 B per lane (lane i -> LDS bytes [16 i, 16 i + 16) of `l`).
// Issued from inline asm: the waitcnt pass would otherwise put a vmcnt(0) (every stage
// in flight) before each fragment read, as it cannot tell the ring buffers apart; the
// waits are the explicit gx3_wait ones.
__device__ __forceinline__ void gx3_dma(const void* g, void* l) {
    const unsigned la =
        __builtin_amdgcn_readfirstlane((unsigned)(size_t)(__attribute__((address_space(3))) char*)(l));
    // M0 bound as an operand: the compiler sets and tracks it (a clobbered m0 is not
    // preserved by the compiler's own M0 users)
    asm volatile("global_load_lds_dwordx4 %1, off" ::"{m0}"(la), "v"(g) : "memory");
}

#define GX3_BK 64
// SW (split weights, a.Wl set): fp32 weights w = hi + lo 2^-11 as two fp16 planes
// (W16, kernels.h).  Each product is three MFMAs, a_hi w_hi + a_lo w_hi into acc and
// a_hi w_lo into accl, and the result is acc + accl 2^-11: a weight keeps ~22 of its
// 24 significant bits (the reference runs such models with fp32 initializers).
// WTN > 1 (the large-M form): each wave owns WTN 32 x 32 tiles side by side in N and splits
// its A fragment once for all of them, so the split's VALU and the A fragment reads are
// shared by WTN MFMA pairs; every 32 x 32 tile still runs the one-tile MFMA sequence.
// XR: blocks that share an A row tile go to one XCD (the guide's bijective remap of the
// block id; `id % 8` labels the blocks that share an XCD), so A is fetched into one L2.
// PS (pre-split A): A arrives as its fp16 hi / lo planes (a.Ah / a.Al, written by the producer
// from the same f32 values, r06), laid out in LDS like the weights; the fragment split -- ~24
// VALU instructions per MFMA pair, which kept the large-M form's VALU ~80 % busy
// (profiles/r06j_gemm_pmc.txt) -- is gone, and each product runs the same two MFMAs.
template <int BM, int BN, int NS, bool SW = false, int WTN = 1, bool XR = false, bool PS = false>
__global__ __launch_bounds__(64 * (BM / 32) * (BN / 32 / WTN)) void k_gemm_x3(GemmArgs a) {
    constexpr int WN = BN / 32 / WTN;                    // waves across N
    constexpr int WV = (BM / 32) * WN;                   // waves, WTN 32 x 32 output tiles each
    constexpr int NA = BM / 4 / WV, NW = BN / 8 / WV;    // DMA instructions per wave per stage (A, W)
    static_assert(NA * WV * 4 == BM && NW * WV * 8 == BN && WN * WTN * 32 == BN, "tile / wave split");
    constexpr int NWL = SW ? NW : 0;                     // ... of the lo plane
    __shared__ __attribute__((aligned(16))) float As[NS][BM * GX3_BK];
    __shared__ __attribute__((aligned(16))) __half Ws[NS][BN * GX3_BK];
    __shared__ __attribute__((aligned(16))) __half Wls[SW ? NS : 1][SW ? BN * GX3_BK : 8];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int wm = w / WN, wn = w % WN;
    int bx = blockIdx.x, by = blockIdx.y;
    if (XR) {
        const int nwg = gridDim.x * gridDim.y, orig = blockIdx.x + gridDim.x * blockIdx.y;
        const int q = nwg / 8, rr = nwg % 8, xcd = orig % 8;
        const int id = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + orig / 8;
        bx = id % gridDim.x;
        by = id / gridDim.x;
    }
    const int m0 = by * BM, n0 = bx * BN;
    const int r = lane & 31, hh = lane >> 5;
    // K slice of this block: k_gemm_x2's partition (whole 128-k steps), in 64-k stages
    const int nsplit = gridDim.z, kz = blockIdx.z;
    const int steps_all = a.K / GX_KS;
    const int s_lo = 2 * (kz * steps_all / nsplit), s_hi = 2 * ((kz + 1) * steps_all / nsplit);
    const int nsteps = s_hi - s_lo;
    // this lane's DMA sources: A instruction j covers rows 4 j + (lane >> 4), slot lane & 15
    // (chunk slot ^ (row & 15)); W instruction j covers rows 8 j + (lane >> 3), slot lane & 7
    // (chunk slot ^ ((row >> 1) & 7))
    const float* asrc[NA];
    // PS: plane instruction i < NA / 2 covers hi rows 8 i' + (lane >> 3) (i' = w + WV i), slot lane & 7
    // (chunk slot ^ ((row >> 1) & 7), the weights' swizzle); i >= NA / 2 the lo plane's rows
    constexpr int NAH = NA / 2;
    static_assert(!PS || NAH * WV * 8 == BM, "pre-split A: whole 8-row plane instructions");
#pragma unroll
    for (int i = 0; i < NA; ++i) {
        if (PS) {
            const int ip = i < NAH ? i : i - NAH;
            const int row = 8 * (w + WV * ip) + (lane >> 3), slot = lane & 7;
            const int gm = min(m0 + row, a.M - 1);
            const __half* pl = i < NAH ? a.Ah : a.Al;
            asrc[i] = reinterpret_cast<const float*>(pl + (long)gm * a.lda + (long)s_lo * GX3_BK +
                                                     8 * (slot ^ ((row >> 1) & 7)));
        } else {
            const int row = 4 * (w + WV * i) + (lane >> 4), slot = lane & 15;
            const int gm = min(m0 + row, a.M - 1);
            asrc[i] = a.A + (long)gm * a.lda + (long)s_lo * GX3_BK + 4 * (slot ^ (row & 15));
        }
    }
    const __half* wsrc[NW];
#pragma unroll
    for (int i = 0; i < NW; ++i) {
        const int row = 8 * (w + WV * i) + (lane >> 3), slot = lane & 7;
        const int gn = min(n0 + row, a.N - 1);
        wsrc[i] = reinterpret_cast<const __half*>(a.W) + (long)gn * a.ldw + (long)s_lo * GX3_BK +
                  8 * (slot ^ ((row >> 1) & 7));
    }
    const long wl_off = SW ? reinterpret_cast<const __half*>(a.Wl) - reinterpret_cast<const __half*>(a.W) : 0;
    auto issue = [&](int st) {
        const int k0 = st * GX3_BK, buf = st % NS;
#pragma unroll
        for (int i = 0; i < NA; ++i) {
            if (PS) {   // 1 KB = 8 plane rows of 64 halfs; the lo plane after the hi plane's BM rows
                const int ip = i < NAH ? i : i - NAH;
                __half* dst = reinterpret_cast<__half*>(As[buf]) + (i < NAH ? 0 : BM * GX3_BK) + 512 * (w + WV * ip);
                gx3_dma(reinterpret_cast<const __half*>(asrc[i]) + k0, dst);
            } else {
                gx3_dma(asrc[i] + k0, &As[buf][256 * (w + WV * i)]);
            }
        }
#pragma unroll
        for (int i = 0; i < NW; ++i) gx3_dma(wsrc[i] + k0, &Ws[buf][512 * (w + WV * i)]);
#pragma unroll
        for (int i = 0; i < NWL; ++i) gx3_dma(wsrc[i] + wl_off + k0, &Wls[buf][512 * (w + WV * i)]);
    };
    f32x16 acc[WTN], accl[WTN];
#pragma unroll
    for (int t = 0; t < WTN; ++t)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[t][i] = accl[t][i] = 0.f;
#pragma unroll
    for (int st = 0; st < NS - 1; ++st)
        if (st < nsteps) issue(st);
    const int arow = wm * 32 + r, bcol = wn * WTN * 32 + r;
    for (int st = 0; st < nsteps; ++st) {
        // stage st landed (this wave's share; later ones stay in flight), then the barrier:
        // every wave's share landed, and the buffer refilled below was consumed by all.
        // s_barrier without __syncthreads' fence, which would wait for every DMA in flight.
        gx3_wait<NA + NW + NWL>(min(NS - 2, nsteps - 1 - st));
        __builtin_amdgcn_s_barrier();
        if (st + NS - 1 < nsteps) issue(st + NS - 1);
        const float* As_ = As[st % NS];
        const __half* Ws_ = Ws[st % NS];
        const __half* Wls_ = Wls[SW ? st % NS : 0];
#pragma unroll
        for (int ks = 0; ks < GX3_BK / 16; ++ks) {
            h16x8 ahi, alo;
            if (PS) {   // this lane's 8 k of row arow: chunk 2 ks + hh of each plane
                const __half* Ah_ = reinterpret_cast<const __half*>(As_);
                const int ao = arow * GX3_BK + 8 * ((2 * ks + hh) ^ ((arow >> 1) & 7));
                ahi = *reinterpret_cast<const h16x8*>(Ah_ + ao);
                alo = *reinterpret_cast<const h16x8*>(Ah_ + BM * GX3_BK + ao);
            } else {
                const int c0 = 4 * ks + 2 * hh;   // A chunks c0, c0 + 1 (4 floats each)
                const float4 x0 = *reinterpret_cast<const float4*>(As_ + arow * GX3_BK + 4 * (c0 ^ (arow & 15)));
                const float4 x1 = *reinterpret_cast<const float4*>(As_ + arow * GX3_BK + 4 * ((c0 + 1) ^ (arow & 15)));
                split8(x0, x1, ahi, alo);
            }
            const int cb = 2 * ks + hh;       // W chunk (8 halfs)
#pragma unroll
            for (int t = 0; t < WTN; ++t) {
                const int bc = bcol + 32 * t;
                const int wo = bc * GX3_BK + 8 * (cb ^ ((bc >> 1) & 7));
                const h16x8 bw = *reinterpret_cast<const h16x8*>(Ws_ + wo);
                acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ahi, bw, acc[t], 0, 0, 0);
                acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(alo, bw, acc[t], 0, 0, 0);
                if (SW) {
                    const h16x8 bl = *reinterpret_cast<const h16x8*>(Wls_ + wo);
                    accl[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ahi, bl, accl[t], 0, 0, 0);
                }
            }
        }
    }
#pragma unroll
    for (int t = 0; t < WTN; ++t) {
        if (SW) {
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[t][i] = fmaf(accl[t][i], W16_LO_INV, acc[t][i]);
        }
        const int col = n0 + bcol + 32 * t;
        if (a.mode == EPI_SLAB) {
            if (col >= a.N) continue;
            float* C = a.C + (long)kz * a.slab_stride;
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int row = m0 + wm * 32 + (i & 3) + 8 * (i >> 2) + 4 * hh;
                if (row < a.M) C[(long)row * a.ldc + col] = acc[t][i];
            }
            continue;
        }
        gemm_epilogue(a, m0 + wm * 32, col, lane, acc[t]);
    }
}

// Tile configurations of k_gemm_x3 (GENIE_GEMM_CFG picks one for benchmarks; default: by shape)
static void launch_x3(const GemmArgs& a, int z, hipStream_t s, int cfg) {
    auto go = [&](auto kern, int bm, int bn, int threads) {
        hipLaunchKernelGGL(kern, dim3((a.N + bn - 1) / bn, (a.M + bm - 1) / bm, z), dim3(threads), 0, s, a);
    };
    if (a.Wl) {   // split weights: 4 x 32 KB stages; cfg 16: 2 stages + XCD remap (64 KB, 2 blocks per CU)
        if (cfg == 16) go(k_gemm_x3<64, 64, 2, true, 1, true>, 64, 64, 256);
        else go(k_gemm_x3<64, 64, 4, true>, 64, 64, 256);
        return;
    }
    switch (cfg) {
        // (r04: the one-block-per-CU 128 x 128 forms, four 32 x 32 tiles per wave, measured
        // slower than k_gemm_x2 at 22,848 rows and were removed; profiles/r04e_gemm_big.txt)
        case 13:   // 64 KB: 2 blocks per CU
            if (a.Ah) go(k_gemm_x3<64, 128, 2, false, 2, true, true>, 64, 128, 256);
            else go(k_gemm_x3<64, 128, 2, false, 2, true>, 64, 128, 256);
            break;
        case 14:   // 80 KB
            if (a.Ah) go(k_gemm_x3<128, 64, 2, false, 2, true, true>, 128, 64, 256);
            else go(k_gemm_x3<128, 64, 2, false, 2, true>, 128, 64, 256);
            break;
        case 15:   // 48 KB: 3 per CU
            if (a.Ah) go(k_gemm_x3<64, 64, 2, false, 1, true, true>, 64, 64, 256);
            else go(k_gemm_x3<64, 64, 2, false, 1, true>, 64, 64, 256);
            break;
        case 1: go(k_gemm_x3<64, 64, 4>, 64, 64, 256); break;
        case 2: go(k_gemm_x3<32, 64, 4>, 32, 64, 128); break;
        case 3: go(k_gemm_x3<64, 32, 4>, 64, 32, 128); break;
        case 4: go(k_gemm_x3<32, 64, 6>, 32, 64, 128); break;
        case 5: go(k_gemm_x3<64, 64, 6>, 64, 64, 256); break;
        case 6: go(k_gemm_x3<32, 32, 6>, 32, 32, 64); break;
        case 7: go(k_gemm_x3<64, 64, 3>, 64, 64, 256); break;
        case 8: go(k_gemm_x3<32, 64, 3>, 32, 64, 128); break;
        default: go(k_gemm_x3<64, 64, 4>, 64, 64, 256); break;
    }
}
static int gemm_cfg() {
    static const int c = [] {
        const char* e = std::getenv("GENIE_GEMM_CFG");
        return e ? std::atoi(e) : 0;
    }();
    return c;
}

// The large-M configuration (GENIE_GEMM_BIG = its launch_x3 configuration, 0 = k_gemm_x2):
// k_gemm_x3<64, 64, 2> with the XCD remap -- 48 KB of LDS, so three blocks (12 waves)
// share a CU and one block's MFMAs hide another's split and LDS waits.  On the packed
// prefill of 64 sentences (22,848 rows) it takes 0.67x k_gemm_x2's time, bit-identical;
// the one-block-per-CU 128 x 128 forms were slower than k_gemm_x2 (profiles/r04e_gemm_big.txt).
// Used from 1024 blocks of 64 x 64 on (4 per CU).
static int gemm_big_cfg() {
    static const int c = [] {
        const char* e = std::getenv("GENIE_GEMM_BIG");
        return e ? std::atoi(e) : 15;
    }();
    return c;
}
static bool gemm_big(const GemmArgs& a) {
    return gemm_big_cfg() != 0 && (long)((a.M + 63) / 64) * ((a.N + 63) / 64) >= 1024;
}

// Split-weight GEMMs (RoBERTa / CN-HuBERT fp32 weights): the two-stage, two-blocks-per-CU
// form with the XCD remap (cfg 16, default; bit-identical to the four-stage one, 0.75x its
// time on packed RoBERTa rows, profiles/r04k_gemm_sw.txt); GENIE_GEMM_SW=0 the four-stage form.
static int gemm_sw_cfg() {
    static const int c = [] {
        const char* e = std::getenv("GENIE_GEMM_SW");
        return e ? std::atoi(e) : 16;
    }();
    return c;
}

static int gemm_variant() {   // GENIE_GEMM_X3=0: the register-staged k_gemm_x2
    static const int v = [] {
        const char* e = std::getenv("GENIE_GEMM_X3");
        return (e && std::atoi(e) == 0) ? 2 : 3;
    }();
    return v;
}

static bool gemm_x2_enabled() {
    static const bool on = [] {
        const char* e = std::getenv("GENIE_GEMM_X2");
        return !(e && std::atoi(e) == 0);
    }();
    return on;
}

bool gemm_w16_supported(int K, long lda, long ldw) { return K % GX_KS == 0 && lda % 4 == 0 && ldw % 8 == 0; }

bool gemm_presplit_path(int M, int N, int K, long lda) {
    if (K % GX_KS != 0 || lda % 8 != 0 || !gemm_x2_enabled() || gemm_variant() != 3 || gemm_cfg() != 0) return false;
    GemmArgs t{};
    t.M = M; t.N = N;
    const int c = gemm_big_cfg();
    return gemm_big(t) && (c == 13 || c == 14 || c == 15);
}

bool gemm_slabs_supported(int K, long lda, long ldw) {
    return K % GX_KS == 0 && lda % 4 == 0 && ldw % 8 == 0 && gemm_x2_enabled();
}

void gemm_nt(const GemmArgs& a, hipStream_t s) {
    dim3 grid((a.N + 63) / 64, (a.M + 63) / 64);
    if (a.Wl) {
        // split fp32 weights run only on k_gemm_x3 (every M: its partition does not depend
        // on M, so packed and per-sentence rows stay identical); the loaders check the shapes
        if (!gemm_w16_supported(a.K, a.lda, a.ldw) || a.a_nslab != 0 || a.mode == EPI_VQDIST) {
            std::fprintf(stderr, "gemm_nt: split-weight GEMM with unsupported shape K=%d lda=%ld\n", a.K, a.lda);
            std::abort();
        }
        launch_x3(a, a.mode == EPI_SLAB ? a.ksplit : 1, s, gemm_sw_cfg());
        return;
    }
    // fp16 weights -> split-activation f16 MFMA; the VQ distance GEMM stays on the
    // exact f32 path (its argmin must see the f32 dot products).
    if (a.w_f16 && a.mode != EPI_VQDIST && a.K % GX_KS == 0 && a.lda % 4 == 0 && a.ldw % 8 == 0 &&
        gemm_x2_enabled()) {
        if (a.mode == EPI_SLAB) grid.z = a.ksplit;
        // the LDS-DMA pipeline reads A as stored: a slab-summing A prologue stays on k_gemm_x2
        // (M > 512: the register-staged kernel's 128-k steps win once the grid covers the chip)
        if (a.Ah && !gemm_presplit_path(a.M, a.N, a.K, a.lda)) {   // the caller asked gemm_presplit_path
            std::fprintf(stderr, "gemm_nt: pre-split A on a shape without the large-M path (M=%d N=%d)\n", a.M, a.N);
            std::abort();
        }
        if (a.a_nslab == 0 && a.lda % 4 == 0 && gemm_variant() == 3 && gemm_cfg() == 0 && gemm_big(a))
            launch_x3(a, grid.z, s, gemm_big_cfg());
        else if (a.a_nslab == 0 && a.lda % 4 == 0 && gemm_variant() == 3 && (a.M <= 512 || gemm_cfg() != 0))
            launch_x3(a, grid.z, s, gemm_cfg());
        else
            hipLaunchKernelGGL(k_gemm_x2, grid, dim3(256), 0, s, a);
        return;
    }
    if (a.w_f16)
        hipLaunchKernelGGL(k_gemm_nt<true>, grid, dim3(256), 0, s, a);
    else
        hipLaunchKernelGGL(k_gemm_nt<false>, grid, dim3(256), 0, s, a);
}

// =====================================================================
// Row kernels
// =====================================================================
// LayerNormalization(axis -1, eps 1e-5) over D=512 (stage#105,#114), one row per block.
__global__ __launch_bounds__(256) void k_layernorm512(const float* in, float* out, const float* g,
                                                      const float* b) {
    __shared__ float red[16];
    const long r = blockIdx.x;
    const int t = threadIdx.x;
    const float v0 = in[r * 512 + t], v1 = in[r * 512 + t + 256];
    const float mean = block_sum(v0 + v1, red) * (1.0f / 512.0f);
    const float d0 = v0 - mean, d1 = v1 - mean;
    const float var = block_sum(d0 * d0 + d1 * d1, red) * (1.0f / 512.0f);
    const float den = sqrtf(var + 1e-5f);
    out[r * 512 + t] = d0 / den * g[t] + b[t];
    out[r * 512 + t + 256] = d1 / den * g[t + 256] + b[t + 256];
}

__global__ __launch_bounds__(256) void k_layernorm512_slabs(const float* slabs, int nsplit, long sstride,
                                                            const float* bias, const float* res, float* out,
                                                            const float* g, const float* b, _Float16* oh,
                                                            _Float16* ol) {
    __shared__ float red[16];
    const long r = blockIdx.x;
    const int t = threadIdx.x;
    float p0 = 0.f, p1 = 0.f;
    for (int z = 0; z < nsplit; ++z) {
        p0 += slabs[z * sstride + r * 512 + t];
        p1 += slabs[z * sstride + r * 512 + t + 256];
    }
    const float v0 = res[r * 512 + t] + (bias[t] + p0), v1 = res[r * 512 + t + 256] + (bias[t + 256] + p1);
    const float mean = block_sum(v0 + v1, red) * (1.0f / 512.0f);
    const float d0 = v0 - mean, d1 = v1 - mean;
    const float var = block_sum(d0 * d0 + d1 * d1, red) * (1.0f / 512.0f);
    const float den = sqrtf(var + 1e-5f);
    float o0 = d0 / den * g[t] + b[t], o1 = d1 / den * g[t + 256] + b[t + 256];
    if (oh) {   // + the fp16 hi / lo planes of the stored values (a pre-split GEMM's A)
        asm volatile("" : "+v"(o0), "+v"(o1));   // materialised f32: no conversion fused into them
        const _Float16 h0 = (_Float16)o0, h1 = (_Float16)o1;
        oh[r * 512 + t] = h0;
        oh[r * 512 + t + 256] = h1;
        ol[r * 512 + t] = (_Float16)(o0 - (float)h0);
        ol[r * 512 + t + 256] = (_Float16)(o1 - (float)h1);
    }
    out[r * 512 + t] = o0;
    out[r * 512 + t + 256] = o1;
}

void layernorm_rows_slabs(const float* slabs, int nsplit, long slab_stride, const float* bias,
                          const float* res, float* out, int rows, const float* g, const float* b,
                          hipStream_t s, __half* out_hi, __half* out_lo) {
    if (rows <= 0) return;
    hipLaunchKernelGGL(k_layernorm512_slabs, dim3(rows), dim3(256), 0, s, slabs, nsplit, slab_stride, bias,
                       res, out, g, b, reinterpret_cast<_Float16*>(out_hi), reinterpret_cast<_Float16*>(out_lo));
}

void layernorm_rows(const float* in, float* out, int rows, const float* g, const float* b,
                    hipStream_t s) {
    if (rows <= 0) return;
    hipLaunchKernelGGL(k_layernorm512, dim3(rows), dim3(256), 0, s, in, out, g, b);
}

// out[r] = sum_c in[r*ld+c]^2  (encoder #25-26 / #32-33)
__global__ __launch_bounds__(256) void k_sumsq(const float* in, long ld, int cols, float* out) {
    __shared__ float red[16];
    const long r = blockIdx.x;
    float acc = 0.f;
    for (int c = threadIdx.x; c < cols; c += 256) {
        const float v = in[r * ld + c];
        acc += v * v;
    }
    acc = block_sum(acc, red);
    if (threadIdx.x == 0) out[r] = acc;
}

void sumsq_rows(const float* in, long ld, int rows, int cols, float* out, hipStream_t s) {
    if (rows <= 0) return;
    hipLaunchKernelGGL(k_sumsq, dim3(rows), dim3(256), 0, s, in, ld, cols, out);
}

// prompts[r] = argmax_c(-dist[r][c]) with first-index ties (encoder #35-36)
__global__ __launch_bounds__(256) void k_argmin_rows(const float* dist, int cols, int64_t* out) {
    __shared__ float sv[4];
    __shared__ int si[4];
    const long r = blockIdx.x;
    float best = -INFINITY;
    int bi = 0x7fffffff;
    for (int c = threadIdx.x; c < cols; c += 256) {
        const float v = -dist[r * cols + c];
        if (v > best || (v == best && c < bi)) { best = v; bi = c; }
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        const float ov = __shfl_xor(best, o, 64);
        const int oi = __shfl_xor(bi, o, 64);
        if (ov > best || (ov == best && oi < bi)) { best = ov; bi = oi; }
    }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { sv[w] = best; si[w] = bi; }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int i = 1; i < 4; ++i)
            if (sv[i] > best || (sv[i] == best && si[i] < bi)) { best = sv[i]; bi = si[i]; }
        out[r] = bi;
    }
}

void argmin_dist_rows(const float* dist, int rows, int cols, int64_t* out, hipStream_t s) {
    if (rows <= 0) return;
    hipLaunchKernelGGL(k_argmin_rows, dim3(rows), dim3(256), 0, s, dist, cols, out);
}

// =====================================================================
// Embeddings + sinusoidal PE
// =====================================================================
__global__ __launch_bounds__(256) void k_text_embed(const int64_t* ref_seq, int n_ref,
                                                    const int64_t* text_seq, const float* emb,
                                                    const float* bproj, const float* bias,
                                                    const float* alpha, const float* pe,
                                                    float* x) {
    const int l = blockIdx.x;
    const int64_t tok = l < n_ref ? ref_seq[l] : text_seq[l - n_ref];
    const float al = alpha[0];
    for (int d = threadIdx.x; d < 512; d += 256) {
        const float bp = bproj ? bias[d] + bproj[(long)l * 512 + d] : bias[d];
        const float e = emb[tok * 512 + d] + bp;
        x[(long)l * 512 + d] = e * 1.0f + al * pe[(long)(l + 1) * 512 + d];
    }
}

void text_embed(const int64_t* ref_seq, int n_ref, const int64_t* text_seq, int n_text,
                const float* emb, const float* bproj, const float* bias, const float* alpha,
                const float* pe, float* x, hipStream_t s) {
    const int L = n_ref + n_text;
    if (L <= 0) return;
    hipLaunchKernelGGL(k_text_embed, dim3(L), dim3(256), 0, s, ref_seq, n_ref, text_seq, emb,
                       bproj, bias, alpha, pe, x);
}

__global__ __launch_bounds__(256) void k_audio_embed(const int64_t* tok, const __half* emb,
                                                     const float* alpha, const float* pe,
                                                     float* out) {
    const int p = blockIdx.x;
    const int64_t t = tok[p];
    const float al = alpha[0];
    for (int d = threadIdx.x; d < 512; d += 256)
        out[(long)p * 512 + d] = __half2float(emb[t * 512 + d]) + al * pe[(long)(p + 1) * 512 + d];
}

void audio_embed_prompts(const int64_t* tok, int P, const __half* emb, const float* alpha,
                         const float* pe, float* out, hipStream_t s) {
    if (P <= 0) return;
    hipLaunchKernelGGL(k_audio_embed, dim3(P), dim3(256), 0, s, tok, emb, alpha, pe, out);
}

__global__ __launch_bounds__(256) void k_ssl_im2col(const float* ssl, int n_ssl, float* A) {
    const int t = blockIdx.x;
    for (int i = threadIdx.x; i < 1536; i += 256) {
        const int ci = i >> 1, j = i & 1;
        A[(long)t * 1536 + i] = ssl[(long)ci * n_ssl + 2 * t + j];
    }
}

void ssl_im2col(const float* ssl, int n_ssl, float* A, hipStream_t s) {
    const int P = n_ssl / 2;
    if (P <= 0) return;
    hipLaunchKernelGGL(k_ssl_im2col, dim3(P), dim3(256), 0, s, ssl, n_ssl, A);
}

__global__ __launch_bounds__(256) void k_decode_embed(const int64_t* y, long ldy, const int* ny,
                                                      const __half* emb, const float* alpha,
                                                      const float* pe, float* h,
                                                      const uint8_t* done) {
    const int b = blockIdx.x;
    if (done && done[b]) return;
    const int n = ny[b];
    const int64_t tok = y[(long)b * ldy + n - 1];
    const float al = alpha[0];
    for (int d = threadIdx.x; d < 512; d += 256)
        h[(long)b * 512 + d] = __half2float(emb[tok * 512 + d]) + al * pe[(long)n * 512 + d];
}

void decode_embed(int B, const int64_t* y, long ldy, const int* ny, const __half* emb,
                  const float* alpha, const float* pe, float* h, const uint8_t* done,
                  hipStream_t s) {
    hipLaunchKernelGGL(k_decode_embed, dim3(B), dim3(256), 0, s, y, ldy, ny, emb, alpha, pe, h,
                       done);
}

// =====================================================================
// Prefix attention: one block per (head, row); keys [0, len).
// Scores (q*s)(k*s) as stage#91-94; softmax #95; P @ V #96.
// =====================================================================
#define ATTN_MAXT 4096
__global__ __launch_bounds__(256) void k_attn_rows(AttnArgs a, int len_add) {
    __shared__ float p[ATTN_MAXT];
    __shared__ float qs[32];
    __shared__ float red[16];
    __shared__ float part[8][33];
    const int h = blockIdx.x, r = blockIdx.y, tid = threadIdx.x;
    const int seq = a.row_seq ? a.row_seq[r] : 0;
    if (a.row_skip && a.row_skip[seq]) return;
    const int len = a.row_len[r] + len_add;
    const float* K = a.k + (long)seq * a.seq_stride + (long)h * a.tmax * 32;
    const float* V = a.v + (long)seq * a.seq_stride + (long)h * a.tmax * 32;
    const float sc = a.scale;
    if (tid < 32) qs[tid] = a.q[(long)r * a.ldq + h * 32 + tid] * sc;
    __syncthreads();
    float lmax = -INFINITY;
    for (int t0 = 0; t0 < len; t0 += 512) {
        // two keys per thread in flight
        const int ta = t0 + tid, tb = t0 + 256 + tid;
        float4 ka[8], kb[8];
        const float4* kra = reinterpret_cast<const float4*>(K + (long)min(ta, len - 1) * 32);
        const float4* krb = reinterpret_cast<const float4*>(K + (long)min(tb, len - 1) * 32);
#pragma unroll
        for (int i = 0; i < 8; ++i) { ka[i] = kra[i]; kb[i] = krb[i]; }
        float sa = 0.f, sb = 0.f;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            sa += qs[4 * i] * (ka[i].x * sc); sa += qs[4 * i + 1] * (ka[i].y * sc);
            sa += qs[4 * i + 2] * (ka[i].z * sc); sa += qs[4 * i + 3] * (ka[i].w * sc);
            sb += qs[4 * i] * (kb[i].x * sc); sb += qs[4 * i + 1] * (kb[i].y * sc);
            sb += qs[4 * i + 2] * (kb[i].z * sc); sb += qs[4 * i + 3] * (kb[i].w * sc);
        }
        if (ta < len) { p[ta] = sa; lmax = fmaxf(lmax, sa); }
        if (tb < len) { p[tb] = sb; lmax = fmaxf(lmax, sb); }
    }
    const float m = block_max(lmax, red);
    float lsum = 0.f;
    for (int t = tid; t < len; t += 256) {
        const float e = expf(p[t] - m);
        p[t] = e;
        lsum += e;
    }
    const float sum = block_sum(lsum, red);
    for (int t = tid; t < len; t += 256) p[t] = p[t] / sum;
    __syncthreads();
    const int g = tid >> 5, d = tid & 31;
    float acc = 0.f;
    int t = g;
    for (; t + 56 < len; t += 64) {
        float vv[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) vv[i] = V[(long)(t + 8 * i) * 32 + d];
#pragma unroll
        for (int i = 0; i < 8; ++i) acc += p[t + 8 * i] * vv[i];
    }
    for (; t < len; t += 8) acc += p[t] * V[(long)t * 32 + d];
    part[g][d] = acc;
    __syncthreads();
    if (tid < 32) {
        float o = 0.f;
#pragma unroll
        for (int i = 0; i < 8; ++i) o += part[i][tid];
        a.out[(long)r * a.ldo + h * 32 + tid] = o;
    }
}

// Batched decode attention with the QKV split-K reduction in its prologue: block
// (head h, sequence b).  q/k/v of the head = b_in + sum_z slab[z] (z ascending,
// the same order for every block), the new K/V row goes to cache position
// kvlen[b] and is used from LDS; then (q s)(k s) over [0, kvlen[b]] (stage#91-94),
// softmax (#95), P.V (#96) as k_attn_rows.
__global__ __launch_bounds__(256) void k_attn_dec_slabs(AttnDecArgs a) {
    __shared__ float p[ATTN_MAXT];
    __shared__ float qs[32], kn[32], vn[32];
    __shared__ float red[16];
    __shared__ float part[8][33];
    const int h = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
    if (a.done[b]) return;
    const int pos = a.kvlen[b], len = pos + 1;
    float* K = a.k + (long)b * a.seq_stride + (long)h * a.tmax * 32;
    float* V = a.v + (long)b * a.seq_stride + (long)h * a.tmax * 32;
    const float sc = a.scale;
    if (tid < 96) {
        const int part_ = tid >> 5, d = tid & 31, col = part_ * 512 + h * 32 + d;
        const float* src = a.slabs + (long)b * 1536 + col;
        float v = src[0];
        for (int z = 1; z < a.nslab; ++z) v += src[z * a.slab_stride];
        v = a.b_in[col] + v;   // Add(bias, MatMul)
        if (part_ == 0) qs[d] = v * sc;
        else if (part_ == 1) { kn[d] = v; K[(long)pos * 32 + d] = v; }
        else { vn[d] = v; V[(long)pos * 32 + d] = v; }
    }
    __syncthreads();
    float lmax = -INFINITY;
    for (int t0 = 0; t0 < len; t0 += 512) {
        const int ta = t0 + tid, tb = t0 + 256 + tid;
        float4 ka[8], kb[8];
        const float4* kra = reinterpret_cast<const float4*>(ta < pos ? K + (long)ta * 32 : kn);
        const float4* krb = reinterpret_cast<const float4*>(tb < pos ? K + (long)tb * 32 : kn);
#pragma unroll
        for (int i = 0; i < 8; ++i) { ka[i] = kra[i]; kb[i] = krb[i]; }
        float sa = 0.f, sb = 0.f;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            sa += qs[4 * i] * (ka[i].x * sc); sa += qs[4 * i + 1] * (ka[i].y * sc);
            sa += qs[4 * i + 2] * (ka[i].z * sc); sa += qs[4 * i + 3] * (ka[i].w * sc);
            sb += qs[4 * i] * (kb[i].x * sc); sb += qs[4 * i + 1] * (kb[i].y * sc);
            sb += qs[4 * i + 2] * (kb[i].z * sc); sb += qs[4 * i + 3] * (kb[i].w * sc);
        }
        if (ta < len) { p[ta] = sa; lmax = fmaxf(lmax, sa); }
        if (tb < len) { p[tb] = sb; lmax = fmaxf(lmax, sb); }
    }
    const float m = block_max(lmax, red);
    float lsum = 0.f;
    for (int t = tid; t < len; t += 256) {
        const float e = expf(p[t] - m);
        p[t] = e;
        lsum += e;
    }
    const float sum = block_sum(lsum, red);
    for (int t = tid; t < len; t += 256) p[t] = p[t] / sum;
    __syncthreads();
    const int g = tid >> 5, d = tid & 31;
    float acc = 0.f;
    int t = g;
    for (; t + 56 < pos; t += 64) {
        float vv[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) vv[i] = V[(long)(t + 8 * i) * 32 + d];
#pragma unroll
        for (int i = 0; i < 8; ++i) acc += p[t + 8 * i] * vv[i];
    }
    for (; t < pos; t += 8) acc += p[t] * V[(long)t * 32 + d];
    if (t == pos) acc += p[t] * vn[d];
    part[g][d] = acc;
    __syncthreads();
    if (tid < 32) {
        float o = 0.f;
#pragma unroll
        for (int i = 0; i < 8; ++i) o += part[i][tid];
        a.out[(long)b * 512 + h * 32 + tid] = o;
    }
}

void attn_decode_slabs(const AttnDecArgs& a, hipStream_t s) {
    if (a.B <= 0) return;
    hipLaunchKernelGGL(k_attn_dec_slabs, dim3(16, a.B), dim3(256), 0, s, a);
}

// Prefill attention, one sequence: a block = one head x 16 query rows, one row
// per wave (1024 threads).  The head's keys/values [0, max row_len of the block)
// are staged in LDS once (36-float rows: conflict-free 16-B reads by 16 lanes);
// a lane owns keys t = lane + 64 i: scores, softmax numerators and P.V partials
// stay in registers, and the 32 output dims are reduce-scattered over the wave.
// Same arithmetic as k_attn_rows ((q s)(k s), exp(x - max), / sum, then P.V);
// only the summation order differs.  Replaces 16 x N0 blocks that each re-read
// the head's whole K/V from L2.
#define AT_ROWS 16
#define AT_KI 7
#define AT_MAXK (64 * AT_KI)
#define AT_KS 36
__global__ __launch_bounds__(1024) void k_attn_tile(AttnArgs a) {
    __shared__ __attribute__((aligned(16))) float Ks[AT_MAXK * AT_KS];
    __shared__ __attribute__((aligned(16))) float Vs[AT_MAXK * AT_KS];
    __shared__ int rl[AT_ROWS];
    const int h = blockIdx.x, tid = threadIdx.x;
    const int lane = tid & 63, w = tid >> 6;
    // one sequence's rows: a tile of the packed prefill, or rows [16 y, 16 y + 16) of sequence 0
    int r0, nr;
    long seq_off = 0;
    if (a.tiles) {
        const int* tl = a.tiles + 3 * blockIdx.y;
        seq_off = (long)tl[0] * a.seq_stride;
        r0 = tl[1];
        nr = tl[2];
    } else {
        r0 = blockIdx.y * AT_ROWS;
        nr = min(AT_ROWS, a.rows - r0);
    }
    if (tid < AT_ROWS) rl[tid] = tid < nr ? a.row_len[r0 + tid] : 0;
    __syncthreads();
    int kmax = 0;
#pragma unroll
    for (int i = 0; i < AT_ROWS; ++i) kmax = max(kmax, rl[i]);
    const float* K = a.k + seq_off + (long)h * a.tmax * 32;
    const float* V = a.v + seq_off + (long)h * a.tmax * 32;
    for (int e = tid; e < kmax * 8; e += 1024) {            // 16-B pieces: row e/8, piece e%8
        const int t = e >> 3, c = e & 7;
        const float4 kv = *reinterpret_cast<const float4*>(K + (long)t * 32 + 4 * c);
        const float4 vv = *reinterpret_cast<const float4*>(V + (long)t * 32 + 4 * c);
        *reinterpret_cast<float4*>(Ks + t * AT_KS + 4 * c) = kv;
        *reinterpret_cast<float4*>(Vs + t * AT_KS + 4 * c) = vv;
    }
    __syncthreads();
    if (w >= nr) return;
    const float sc = a.scale;
    const int r = r0 + w, len = rl[w];
    float q[32];
#pragma unroll
    for (int d = 0; d < 32; d += 4) {
        const float4 v = *reinterpret_cast<const float4*>(a.q + (long)r * a.ldq + h * 32 + d);
        q[d] = v.x * sc; q[d + 1] = v.y * sc; q[d + 2] = v.z * sc; q[d + 3] = v.w * sc;
    }
    float p[AT_KI];
    float lmax = -INFINITY;
#pragma unroll
    for (int i = 0; i < AT_KI; ++i) {
        const int t = lane + 64 * i;
        const float* kr = Ks + min(t, AT_MAXK - 1) * AT_KS;
        float sacc = 0.f;
#pragma unroll
        for (int d = 0; d < 32; d += 4) {
            const float4 k4 = *reinterpret_cast<const float4*>(kr + d);
            sacc += q[d] * (k4.x * sc); sacc += q[d + 1] * (k4.y * sc);
            sacc += q[d + 2] * (k4.z * sc); sacc += q[d + 3] * (k4.w * sc);
        }
        p[i] = t < len ? sacc : -INFINITY;
        lmax = fmaxf(lmax, p[i]);
    }
    const float m = wave_max(lmax);
    float lsum = 0.f;
#pragma unroll
    for (int i = 0; i < AT_KI; ++i) {
        const float e = lane + 64 * i < len ? expf(p[i] - m) : 0.f;
        p[i] = e;
        lsum += e;
    }
    const float sum = wave_sum(lsum);
    float o[32];
#pragma unroll
    for (int d = 0; d < 32; ++d) o[d] = 0.f;
#pragma unroll
    for (int i = 0; i < AT_KI; ++i) {
        const int t = lane + 64 * i;
        if (t >= len) continue;                      // rows past len: LDS not staged
        const float pn = p[i] / sum;                 // normalised numerator
        const float* vr = Vs + t * AT_KS;
#pragma unroll
        for (int d = 0; d < 32; d += 4) {
            const float4 v4 = *reinterpret_cast<const float4*>(vr + d);
            o[d] += pn * v4.x; o[d + 1] += pn * v4.y; o[d + 2] += pn * v4.z; o[d + 3] += pn * v4.w;
        }
    }
    // reduce-scatter the 32 dims over the 64 lanes: partner lane ^ (32 >> k) keeps
    // the half of the dims selected by that lane bit
#pragma unroll
    for (int k = 0; k < 5; ++k) {
        const int half = 16 >> k, bit = 32 >> k;
        const bool up = (lane & bit) != 0;
#pragma unroll
        for (int d = 0; d < half; ++d) {
            const float send = up ? o[d] : o[d + half];
            const float recv = __shfl_xor(send, bit, 64);
            o[d] = (up ? o[d + half] : o[d]) + recv;
        }
    }
    // lane now holds dim (bits 5..1 of lane, MSB first) summed over lanes with the
    // same bit 0; the pair lane ^ 1 completes the sum
    const float tot = o[0] + __shfl_xor(o[0], 1, 64);
    const int d = ((lane >> 5) & 1) * 16 + ((lane >> 4) & 1) * 8 + ((lane >> 3) & 1) * 4 + ((lane >> 2) & 1) * 2 +
                  ((lane >> 1) & 1);
    if ((lane & 1) == 0) a.out[(long)r * a.ldo + h * 32 + d] = tot;
}

// Prefill attention of one sequence, online softmax over 64-key chunks: a block
// = one head x 16 query rows (4 waves x 4 rows).  The head's K/V chunk is staged
// once per block in LDS (rows padded to 36 floats: conflict-free 16-B reads by
// 16 lanes).  Scores: lane = key (its K row in registers, scaled by s), the 4
// query rows (scaled by s) read as LDS broadcasts -> s_rj = (q s).(k s) as
// stage#91-94; per row a wave-wide running max / sum (exp(x - max) #95).  P.V:
// lane = (row, 2 dims), P rows through wave-private LDS.  The same arithmetic as
// k_attn_rows except the summation order and the running rescale.  One K/V pass
// per 16 rows instead of one per row (k_attn_rows re-reads the head's K/V from L2
// for every query row).
#define AF_ROWS 16
#define AF_KC 64
#define AF_KS 36
typedef float f32x2v __attribute__((ext_vector_type(2)));
__global__ __launch_bounds__(256) void k_attn_flash(AttnArgs a) {
    __shared__ __attribute__((aligned(16))) float Ks[AF_KC * AF_KS];
    __shared__ __attribute__((aligned(16))) float Vs[AF_KC * AF_KS];
    __shared__ __attribute__((aligned(16))) float Qs[AF_ROWS][32];
    __shared__ __attribute__((aligned(16))) float Ps[4][4][AF_KC];
    __shared__ int rl[AF_ROWS];
    const int h = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    // rows: 16 per block of one sequence, or (packed prefill) tile blockIdx.y of a.tiles:
    // {sequence, first row, rows <= 16}, every row of a tile in the same sequence
    int r0 = blockIdx.y * AF_ROWS, nr = min(AF_ROWS, a.rows - r0);
    long kvbase = (long)h * a.tmax * 32;
    if (a.tiles) {
        const int* tl = a.tiles + 3 * blockIdx.y;
        kvbase += (long)tl[0] * a.seq_stride;
        r0 = tl[1];
        nr = tl[2];
    }
    const float sc = a.scale;
    if (tid < AF_ROWS) rl[tid] = tid < nr ? a.row_len[r0 + tid] : 0;
    for (int e = tid; e < AF_ROWS * 8; e += 256) {   // q rows (scaled), 16-B pieces
        const int r = e >> 3, c = e & 7;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (r < nr) v = *reinterpret_cast<const float4*>(a.q + (long)(r0 + r) * a.ldq + h * 32 + 4 * c);
        *reinterpret_cast<float4*>(&Qs[r][4 * c]) = make_float4(v.x * sc, v.y * sc, v.z * sc, v.w * sc);
    }
    __syncthreads();
    int kmax = 0;
#pragma unroll
    for (int i = 0; i < AF_ROWS; ++i) kmax = max(kmax, rl[i]);
    const float* K = a.k + kvbase;
    const float* V = a.v + kvbase;
    int len[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) len[r] = rl[4 * w + r];
    float m[4], l[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) { m[r] = -INFINITY; l[r] = 0.f; }
    const int pr = lane >> 4, pd = 2 * (lane & 15);   // P.V: this lane's row (of the wave's 4) and dims
    f32x2v o = {0.f, 0.f};
    // K/V chunks through registers, one chunk ahead: chunk k + 1 is in flight while
    // chunk k is scored (rows past the cache: zeros)
    float4 pk[2], pv[2];
    auto fetch = [&](int k0) {
        const int nk = min(AF_KC, kmax - k0);
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int e = tid + 256 * i, t = e >> 3, c = e & 7;
            pk[i] = make_float4(0.f, 0.f, 0.f, 0.f);
            pv[i] = pk[i];
            if (t < nk) {
                pk[i] = *reinterpret_cast<const float4*>(K + (long)(k0 + t) * 32 + 4 * c);
                pv[i] = *reinterpret_cast<const float4*>(V + (long)(k0 + t) * 32 + 4 * c);
            }
        }
    };
    if (kmax > 0) fetch(0);
    for (int k0 = 0; k0 < kmax; k0 += AF_KC) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int e = tid + 256 * i, t = e >> 3, c = e & 7;
            *reinterpret_cast<float4*>(Ks + t * AF_KS + 4 * c) = pk[i];
            *reinterpret_cast<float4*>(Vs + t * AF_KS + 4 * c) = pv[i];
        }
        __syncthreads();
        if (k0 + AF_KC < kmax) fetch(k0 + AF_KC);
        // ---- scores: lane = key k0 + lane
        f32x2v kr[16];
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            const float4 k4 = *reinterpret_cast<const float4*>(Ks + lane * AF_KS + 4 * c);
            kr[2 * c] = f32x2v{k4.x * sc, k4.y * sc};
            kr[2 * c + 1] = f32x2v{k4.z * sc, k4.w * sc};
        }
        float corr[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const float* qr = Qs[4 * w + r];
            f32x2v acc = {0.f, 0.f};
#pragma unroll
            for (int c = 0; c < 8; ++c) {
                const float4 q4 = *reinterpret_cast<const float4*>(qr + 4 * c);
                acc += f32x2v{q4.x, q4.y} * kr[2 * c];
                acc += f32x2v{q4.z, q4.w} * kr[2 * c + 1];
            }
            const float s = k0 + lane < len[r] ? acc.x + acc.y : -INFINITY;
            const float mc = wave_max(s);
            const float mn = fmaxf(m[r], mc);
            corr[r] = mn == -INFINITY ? 1.f : __expf(m[r] - mn);
            const float p = s == -INFINITY ? 0.f : __expf(s - mn);
            l[r] = l[r] * corr[r] + wave_sum(p);
            m[r] = mn;
            Ps[w][r][lane] = p;
        }
        __builtin_amdgcn_wave_barrier();   // Ps of this wave written before its lanes read it
        // ---- P.V: lane = (row pr, dims pd, pd + 1)
        const float cr = pr == 0 ? corr[0] : pr == 1 ? corr[1] : pr == 2 ? corr[2] : corr[3];
        o *= cr;
        const float* prow = Ps[w][pr];
#pragma unroll 4
        for (int j = 0; j < AF_KC; j += 4) {
            const float4 p4 = *reinterpret_cast<const float4*>(prow + j);
            o += p4.x * *reinterpret_cast<const f32x2v*>(Vs + (j + 0) * AF_KS + pd);
            o += p4.y * *reinterpret_cast<const f32x2v*>(Vs + (j + 1) * AF_KS + pd);
            o += p4.z * *reinterpret_cast<const f32x2v*>(Vs + (j + 2) * AF_KS + pd);
            o += p4.w * *reinterpret_cast<const f32x2v*>(Vs + (j + 3) * AF_KS + pd);
        }
        __syncthreads();   // K/V/P consumed before the next chunk lands
    }
    const float lr = pr == 0 ? l[0] : pr == 1 ? l[1] : pr == 2 ? l[2] : l[3];
    const int row = 4 * w + pr;
    if (row < nr) {
        float* dst = a.out + (long)(r0 + row) * a.ldo + h * 32 + pd;
        dst[0] = o.x / lr;
        dst[1] = o.y / lr;
    }
}

// Prefill attention on the f16 MFMA (stage#91-96 per head): a block = one head x
// 32 NW query rows of one sequence, wave w owns rows 32 w .. 32 w + 31.  Operands are
// split hi + lo into fp16 (three MFMAs per product, f32 accumulation: the dropped term
// is ~2^-22 of each product, as in the split-activation GEMMs).  Per 64-key chunk:
//   S^T = K Q^T  (A = the chunk's K rows, B = the wave's q rows): lane l holds the
//                scores of query row l % 32 for 32 of the 64 keys, the lane l ^ 32 the
//                other 32, so the online softmax (stage#95) needs one cross-lane step;
//   O^T += V^T P^T  (B = the P values straight from the S^T accumulator registers, the
//                16 keys of a k-step taken in the accumulator's key order and V^T read
//                in that same order), so O^T's lane keeps its own query row and the
//                running rescale stays in-lane.
// K and V chunks arrive raw (f32) by LDS-DMA in a ring of AM_RING chunks, issued
// AM_RING - 1 chunks ahead of use; each is then split into the fp16 hi / lo planes of K
// (scaled by s, as q) and V^T that the MFMA fragments read.
// A block reads its head's K/V once per 32 NW rows (k_attn_flash: once per 16).  Used by
// the packed (batched) prefill: 128-row tiles of one sequence.
#define AM_KC 64
#define AM_KR 40   // K plane row stride (halfs): 32 dims + pad
#define AM_VR 72   // V^T plane row stride (halfs): 64 keys + pad
#define AM_RING 3
template <int NW>
__global__ __launch_bounds__(64 * NW) void k_attn_mfma(AttnArgs a) {
    constexpr int NT = 64 * NW, ROWS = 32 * NW, NI = AM_KC * 8 / NT;   // float4 items per thread (K and V each)
    constexpr int DPW = 16 / NW;                                       // DMA instructions per wave per chunk
    __shared__ __attribute__((aligned(16))) float Kr[AM_RING][AM_KC * 32];   // raw chunks (LDS-DMA ring)
    __shared__ __attribute__((aligned(16))) float Vr[AM_RING][AM_KC * 32];
    __shared__ __attribute__((aligned(16))) _Float16 Kh[AM_KC * AM_KR];
    __shared__ __attribute__((aligned(16))) _Float16 Kl[AM_KC * AM_KR];
    __shared__ __attribute__((aligned(16))) _Float16 Vh[32 * AM_VR];
    __shared__ __attribute__((aligned(16))) _Float16 Vl[32 * AM_VR];
    __shared__ int rl[ROWS];
    __shared__ int kmax_s;
    const int h = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int r32 = lane & 31, hs = lane >> 5;
    int r0 = blockIdx.y * ROWS, nr = min(ROWS, a.rows - r0);
    long kvbase = (long)h * a.tmax * 32;
    if (a.tiles) {   // packed prefill: tile {sequence, first row, rows <= ROWS}
        const int* tl = a.tiles + 3 * blockIdx.y;
        kvbase += (long)tl[0] * a.seq_stride;
        r0 = tl[1];
        nr = tl[2];
    }
    const float sc = a.scale;
    if (tid == 0) kmax_s = 0;
    __syncthreads();
    if (tid < ROWS) {
        rl[tid] = tid < nr ? a.row_len[r0 + tid] : 0;
        atomicMax(&kmax_s, rl[tid]);
    }
    __syncthreads();
    const int kmax = kmax_s;
    const int row = 32 * w + r32;                  // this lane's query row (of the block)
    const int len = rl[row];
    const bool wave_rows = 32 * w < nr;            // a wave past the tile's rows only stages
    // q fragments (B of S^T): row `row`, dims 16 ks + 8 hs .. + 7, scaled by s
    h16x8 qh[2], ql[2];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
        float4 x0 = make_float4(0.f, 0.f, 0.f, 0.f), x1 = x0;
        if (row < nr) {
            const float* qp = a.q + (long)(r0 + row) * a.ldq + h * 32 + 16 * ks + 8 * hs;
            x0 = *reinterpret_cast<const float4*>(qp);
            x1 = *reinterpret_cast<const float4*>(qp + 4);
        }
        x0 = make_float4(x0.x * sc, x0.y * sc, x0.z * sc, x0.w * sc);
        x1 = make_float4(x1.x * sc, x1.y * sc, x1.z * sc, x1.w * sc);
        split8(x0, x1, qh[ks], ql[ks]);
    }
    const float* K = a.k + kvbase;
    const float* V = a.v + kvbase;
    // chunk c -> ring slot c % AM_RING: DMA instruction j (8 keys x 32 dims, 1 KB) of K and of
    // V by wave j % NW; keys past kmax read row 0 (in bounds; zeroed by the split)
    auto dma = [&](int c) {
        const int slot = c % AM_RING;
#pragma unroll
        for (int i = 0; i < 8 / NW; ++i) {
            const int j = w + NW * i, key = AM_KC * c + 8 * j + (lane >> 3);
            const long src = (long)(key < kmax ? key : 0) * 32 + 4 * (lane & 7);
            gx3_dma(K + src, &Kr[slot][j * 256]);
            gx3_dma(V + src, &Vr[slot][j * 256]);
        }
    };
    // ring slot of chunk c -> the split planes (keys past kmax: 0)
    auto split_chunk = [&](int c) {
        const int slot = c % AM_RING, k0 = AM_KC * c;
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            const int e = tid + NT * i, t = e >> 3, cc = e & 7;
            const bool ok = k0 + t < kmax;
            const float4 kv4 = *reinterpret_cast<const float4*>(&Kr[slot][t * 32 + 4 * cc]);
            const float4 vv4 = *reinterpret_cast<const float4*>(&Vr[slot][t * 32 + 4 * cc]);
            const float kx[4] = {ok ? kv4.x * sc : 0.f, ok ? kv4.y * sc : 0.f, ok ? kv4.z * sc : 0.f,
                                 ok ? kv4.w * sc : 0.f};
            const float vx[4] = {ok ? vv4.x : 0.f, ok ? vv4.y : 0.f, ok ? vv4.z : 0.f, ok ? vv4.w : 0.f};
            _Float16 khi[4], klo[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                khi[j] = (_Float16)kx[j];
                klo[j] = (_Float16)(kx[j] - (float)khi[j]);
                const _Float16 vh = (_Float16)vx[j];
                Vh[(4 * cc + j) * AM_VR + t] = vh;
                Vl[(4 * cc + j) * AM_VR + t] = (_Float16)(vx[j] - (float)vh);
            }
            *reinterpret_cast<uint2*>(&Kh[t * AM_KR + 4 * cc]) = *reinterpret_cast<const uint2*>(khi);
            *reinterpret_cast<uint2*>(&Kl[t * AM_KR + 4 * cc]) = *reinterpret_cast<const uint2*>(klo);
        }
    };
    float m = -INFINITY, l = 0.f;
    f32x16 o;
#pragma unroll
    for (int i = 0; i < 16; ++i) o[i] = 0.f;
    const int nch = (kmax + AM_KC - 1) / AM_KC;
    if (nch > 0) {
        for (int c = 0; c < AM_RING && c < nch; ++c) dma(c);
        gx3_wait<DPW>(min(AM_RING, nch) - 1);      // chunk 0 (this wave's part) landed
        __syncthreads();
        split_chunk(0);
    }
    __syncthreads();
    for (int c = 0; c < nch; ++c) {
        const int k0 = c * AM_KC;
        if (wave_rows) {
            // ---- S^T: keys 32 T + {8 (i / 4) + 4 hs + i % 4} of row `row` in s[T][i]
            f32x16 s[2];
#pragma unroll
            for (int T = 0; T < 2; ++T) {
#pragma unroll
                for (int i = 0; i < 16; ++i) s[T][i] = 0.f;
#pragma unroll
                for (int ks = 0; ks < 2; ++ks) {
                    const int off = (32 * T + r32) * AM_KR + 16 * ks + 8 * hs;
                    const h16x8 ah = *reinterpret_cast<const h16x8*>(&Kh[off]);
                    const h16x8 al = *reinterpret_cast<const h16x8*>(&Kl[off]);
                    s[T] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, qh[ks], s[T], 0, 0, 0);
                    s[T] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, ql[ks], s[T], 0, 0, 0);
                    s[T] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, qh[ks], s[T], 0, 0, 0);
                }
            }
            // ---- online softmax of the row over the chunk (keys >= len: -inf)
            float mc = -INFINITY;
#pragma unroll
            for (int T = 0; T < 2; ++T)
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    const int key = k0 + 32 * T + 8 * (i >> 2) + 4 * hs + (i & 3);
                    if (key >= len) s[T][i] = -INFINITY;
                    mc = fmaxf(mc, s[T][i]);
                }
            mc = fmaxf(mc, __shfl_xor(mc, 32, 64));
            const float mn = fmaxf(m, mc);
            const float corr = mn == -INFINITY ? 1.f : __expf(m - mn);
            float ps = 0.f;
#pragma unroll
            for (int T = 0; T < 2; ++T)
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    const float p = s[T][i] == -INFINITY ? 0.f : __expf(s[T][i] - mn);
                    s[T][i] = p;
                    ps += p;
                }
            ps += __shfl_xor(ps, 32, 64);
            l = l * corr + ps;
            m = mn;
#pragma unroll
            for (int i = 0; i < 16; ++i) o[i] *= corr;
            // ---- O^T += V^T P^T, k-step (T, g): keys 32 T + 16 g + {0..3, 8..11} (+4 for hs = 1)
#pragma unroll
            for (int T = 0; T < 2; ++T)
#pragma unroll
                for (int g = 0; g < 2; ++g) {
                    h16x8 ph, pl;
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        const float p = s[T][8 * g + j];
                        ph[j] = (_Float16)p;
                        pl[j] = (_Float16)(p - (float)ph[j]);
                    }
                    const int kb = 32 * T + 16 * g + 4 * hs;
                    const _Float16* vh = &Vh[r32 * AM_VR + kb];
                    const _Float16* vl = &Vl[r32 * AM_VR + kb];
                    h16x8 ah, al;
                    const uint2 h0 = *reinterpret_cast<const uint2*>(vh), h1 = *reinterpret_cast<const uint2*>(vh + 8);
                    const uint2 l0 = *reinterpret_cast<const uint2*>(vl), l1 = *reinterpret_cast<const uint2*>(vl + 8);
                    ah = __builtin_bit_cast(h16x8, make_uint4(h0.x, h0.y, h1.x, h1.y));
                    al = __builtin_bit_cast(h16x8, make_uint4(l0.x, l0.y, l1.x, l1.y));
                    o = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, ph, o, 0, 0, 0);
                    o = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, pl, o, 0, 0, 0);
                    o = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, ph, o, 0, 0, 0);
                }
        }
        if (c + 1 < nch) {
            // chunk c + 1 landed (this wave's part; chunk c + 2 may stay in flight), then every
            // wave's part and every wave done with the split planes of chunk c
            gx3_wait<DPW>(min(c + AM_RING - 1, nch - 1) - (c + 1));
            __syncthreads();
            if (c + AM_RING < nch) dma(c + AM_RING);   // into chunk c's slot (split last round)
            split_chunk(c + 1);
            __syncthreads();
        }
    }
    // ---- O^T lane: row `row`, dims 8 (i / 4) + 4 hs + i % 4
    if (row < nr) {
        float* dst = a.out + (long)(r0 + row) * a.ldo + h * 32 + 4 * hs;
        const float rl_ = 1.f / l;
#pragma unroll
        for (int g = 0; g < 4; ++g)
            *reinterpret_cast<float4*>(dst + 8 * g) =
                make_float4(o[4 * g] * rl_, o[4 * g + 1] * rl_, o[4 * g + 2] * rl_, o[4 * g + 3] * rl_);
    }
}

// GENIE_ATTN_MFMA=1: the packed prefill's attention on the split-fp16 MFMA kernel.  Off by
// default since r05: its rounding differs from the f32 online-softmax kernels a sentence's
// own prefill runs, so a batched generate could pick a different token than the same
// sentence alone (and than the oracle) at a near-tie -- found on one input of the B = 64
// test set (profiles/r05x_batched_near_tie.txt).  With the f32 kernels a batch's tokens
// are each sentence's own.
bool attn_mfma_on() {
    static const bool on = [] { const char* e = std::getenv("GENIE_ATTN_MFMA"); return e && std::atoi(e) != 0; }();
    return on;
}

void attn_rows_mfma(const AttnArgs& a, int rows_per_block, hipStream_t s) {
    if (a.tiles ? a.ntiles <= 0 : a.rows <= 0) return;
    if (rows_per_block == 128) {
        const dim3 grid(16, a.tiles ? a.ntiles : (a.rows + 127) / 128);
        hipLaunchKernelGGL(k_attn_mfma<4>, grid, dim3(256), 0, s, a);
    } else {
        const dim3 grid(16, a.tiles ? a.ntiles : (a.rows + 63) / 64);
        hipLaunchKernelGGL(k_attn_mfma<2>, grid, dim3(128), 0, s, a);
    }
}

// Packed-prefill attention in f32 with k_attn_flash's exact per-row arithmetic, one
// query row per lane (stage#91-96 per head).  A block = one head x 64 NW rows of one
// sequence; wave w owns rows 64 w .. 64 w + 63.  k_attn_flash puts a chunk's 64 keys on
// the lanes and reduces each row's scores across the wave; here the lane owns its row, so
// per 64-key chunk it runs the same operations in-lane:
//   score(row, key): two fma chains over the even / odd dims of (q s)(k s), summed;
//   max over the chunk's 64 scores (exact, any order);
//   sum of the 64 exp(s - max) in wave_sum's xor-butterfly tree (offsets 32, 16, .. 1);
//   l = l corr + sum; o = o corr, then o += p_j v_j for j = 0 .. 63 in key order.
// So a row's output is bit-identical to k_attn_flash's (and the packed prefill's tokens
// to a sentence's own prefill) while every K/V element read from LDS is a broadcast that
// feeds 64 rows: k_attn_flash reads ~57 KB of LDS per 4 rows and 64 keys and is
// LDS-bound (281 us per layer of batch64).  K and V chunks land by LDS-DMA in a 2-slot
// ring one chunk ahead; K is then scaled by s in place.  The fused multiply-adds are
// explicit: k_attn_flash compiles to o = o corr, then fma(p, v, o), and a contraction
// left to the compiler here fused o corr into the first product's add instead.
#define AR_KC 64
template <int NW>
__global__ __launch_bounds__(64 * NW) void k_attn_rowlane(AttnArgs a) {
    constexpr int NT = 64 * NW, ROWS = 64 * NW;
    constexpr int DPW = 16 / NW;   // DMA instructions (1 KB) per wave per chunk, K and V
    static_assert(16 % NW == 0, "waves");
    __shared__ __attribute__((aligned(16))) float Ks[2][AR_KC * 32];
    __shared__ __attribute__((aligned(16))) float Vs[2][AR_KC * 32];
    __shared__ int wk[NW];
    const int h = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int* tl = a.tiles + 3 * blockIdx.y;
    const long kvbase = (long)h * a.tmax * 32 + (long)tl[0] * a.seq_stride;
    const int r0 = tl[1], nr = tl[2];
    const float sc = a.scale;
    const int rr = 64 * w + lane;   // this lane's row of the tile
    const int len = rr < nr ? a.row_len[r0 + rr] : 0;
    int wkmax = len;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) wkmax = max(wkmax, __shfl_xor(wkmax, o, 64));
    if (lane == 0) wk[w] = wkmax;
    float q[32];
    {
        const float* qp = a.q + (long)(r0 + (rr < nr ? rr : 0)) * a.ldq + h * 32;
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            const float4 v = *reinterpret_cast<const float4*>(qp + 4 * c);
            q[4 * c] = v.x * sc;
            q[4 * c + 1] = v.y * sc;
            q[4 * c + 2] = v.z * sc;
            q[4 * c + 3] = v.w * sc;
        }
    }
    __syncthreads();
    int kmax = 0;
#pragma unroll
    for (int i = 0; i < NW; ++i) kmax = max(kmax, wk[i]);
    const float* K = a.k + kvbase;
    const float* V = a.v + kvbase;
    // chunk c -> slot c & 1: DMA instruction j (8 keys x 32 dims) of K and of V by wave
    // j % NW; keys past kmax read key 0 (in bounds, never weighted)
    auto dma = [&](int c) {
#pragma unroll
        for (int i = 0; i < 8 / NW; ++i) {
            const int j = w + NW * i, key = AR_KC * c + 8 * j + (lane >> 3);
            const long src = (long)(key < kmax ? key : 0) * 32 + 4 * (lane & 7);
            gx3_dma(K + src, &Ks[c & 1][j * 256]);
            gx3_dma(V + src, &Vs[c & 1][j * 256]);
        }
    };
    float m = -INFINITY, l = 0.f;
    float o[32];
#pragma unroll
    for (int d = 0; d < 32; ++d) o[d] = 0.f;
    const int nch = (kmax + AR_KC - 1) / AR_KC;
    if (nch > 0) dma(0);
    if (nch > 1) dma(1);
    for (int c = 0; c < nch; ++c) {
        const int k0 = AR_KC * c, sl = c & 1;
        gx3_wait<DPW>(c + 1 < nch ? 1 : 0);   // this wave's part of chunk c landed
        __syncthreads();
        // K chunk scaled in place (k s, as k_attn_flash's kr)
#pragma unroll
        for (int i = 0; i < AR_KC * 8 / NT; ++i) {
            float4* p = reinterpret_cast<float4*>(&Ks[sl][4 * (tid + NT * i)]);
            const float4 v = *p;
            *p = make_float4(v.x * sc, v.y * sc, v.z * sc, v.w * sc);
        }
        __syncthreads();
        if (k0 < wkmax) {
            float s[AR_KC];
#pragma unroll
            for (int j = 0; j < AR_KC; ++j) {
                const float* kr = &Ks[sl][32 * j];
                float ax = 0.f, ay = 0.f;
#pragma unroll
                for (int cc = 0; cc < 8; ++cc) {
                    const float4 k4 = *reinterpret_cast<const float4*>(kr + 4 * cc);
                    ax = __builtin_fmaf(q[4 * cc], k4.x, ax);
                    ay = __builtin_fmaf(q[4 * cc + 1], k4.y, ay);
                    ax = __builtin_fmaf(q[4 * cc + 2], k4.z, ax);
                    ay = __builtin_fmaf(q[4 * cc + 3], k4.w, ay);
                }
                s[j] = k0 + j < len ? ax + ay : -INFINITY;
            }
            float mc = -INFINITY;
#pragma unroll
            for (int j = 0; j < AR_KC; ++j) mc = fmaxf(mc, s[j]);
            const float mn = fmaxf(m, mc);
            const float corr = mn == -INFINITY ? 1.f : __expf(m - mn);
#pragma unroll
            for (int j = 0; j < AR_KC; ++j) s[j] = s[j] == -INFINITY ? 0.f : __expf(s[j] - mn);
            // wave_sum's tree: t[k] = t[k] + t[k ^ off], off = 32 .. 1 (lane 0's operands)
            float t[32];
#pragma unroll
            for (int k = 0; k < 32; ++k) t[k] = s[k] + s[k + 32];
#pragma unroll
            for (int off = 16; off >= 1; off >>= 1)
#pragma unroll
                for (int k = 0; k < off; ++k) t[k] = t[k] + t[k + off];
            l = __builtin_fmaf(l, corr, t[0]);
            m = mn;
#pragma unroll
            for (int d = 0; d < 32; ++d) o[d] *= corr;
#pragma unroll
            for (int j = 0; j < AR_KC; ++j) {
                const float* vr = &Vs[sl][32 * j];
                const float p = s[j];
#pragma unroll
                for (int cc = 0; cc < 8; ++cc) {
                    const float4 v4 = *reinterpret_cast<const float4*>(vr + 4 * cc);
                    o[4 * cc] = __builtin_fmaf(p, v4.x, o[4 * cc]);
                    o[4 * cc + 1] = __builtin_fmaf(p, v4.y, o[4 * cc + 1]);
                    o[4 * cc + 2] = __builtin_fmaf(p, v4.z, o[4 * cc + 2]);
                    o[4 * cc + 3] = __builtin_fmaf(p, v4.w, o[4 * cc + 3]);
                }
            }
        }
        __syncthreads();                    // slot sl consumed by every wave
        if (c + 2 < nch) dma(c + 2);
    }
    if (rr < nr) {
        float* dst = a.out + (long)(r0 + rr) * a.ldo + h * 32;
#pragma unroll
        for (int c = 0; c < 8; ++c)
            *reinterpret_cast<float4*>(dst + 4 * c) =
                make_float4(o[4 * c] / l, o[4 * c + 1] / l, o[4 * c + 2] / l, o[4 * c + 3] / l);
    }
}

// Packed-prefill attention on the f32 MFMA with k_attn_flash's exact per-row arithmetic.
// v_mfma_f32_32x32x2f32 computes each element as a sequential fma chain in k order,
// fma(a1, b1, fma(a0, b0, c)) -- bit for bit on 204,800 random elements
// (tools/mfma_f32_probe.hip, profiles/r05k_mfma_f32_chain.txt) -- so the flash kernel's
// fma chains map onto it step for step.  A block = one head x 32 NW rows of one
// sequence, wave w owns rows 32 w .. 32 w + 31.  Per 64-key chunk:
//   S^T = K Q^T twice, A = the chunk's (k s) rows, B = the wave's (q s) rows: step t of
//     one accumulator takes dims (4t, 4t + 2), of the other (4t + 1, 4t + 3), i.e.
//     k_attn_flash's even and odd chains; s = even + odd.  A row r of a 32-key tile T
//     holds key 8 (r / 8) + 2 (r % 4) + (r / 4) % 2, so accumulator element i of lane
//     l holds query row l % 32 and key 32 T + 2 i + l / 32;
//   max, exp and wave_sum's butterfly tree in-lane (the offset-1 level across the
//     lane halves), l = fma(l, corr, sum);
//   O^T = O^T corr, then O^T += V^T P^T in 32 steps of keys (2s, 2s + 1): fma(v, p, o)
//     in key order; lane half h's P^T operand, key 2s + h, is its own element s % 16.
// K and V arrive raw by LDS-DMA in a 3-chunk ring, two chunks ahead; K is scaled by s
// into a padded plane (row stride 34: conflict-free 8-byte fragment reads).
#define MF_KC 64
#define MF_KR 34
#define MF_RING 3
template <int NW>
__global__ __launch_bounds__(64 * NW) void k_attn_mf32(AttnArgs a) {
    constexpr int NT = 64 * NW, ROWS = 32 * NW;
    constexpr int DPW = 16 / NW;
    __shared__ __attribute__((aligned(16))) float Kr[MF_RING][MF_KC * 32];
    __shared__ __attribute__((aligned(16))) float Vr[MF_RING][MF_KC * 32];
    __shared__ __attribute__((aligned(16))) float Kp[MF_KC * MF_KR];
    __shared__ int wk[NW];
    const int h = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int r32 = lane & 31, hs = lane >> 5;
    // a.tiles: tile blockIdx.y {sequence, first row, rows <= ROWS}; else rows
    // ROWS blockIdx.y .. of the one sequence at a.k / a.v
    long kvbase = (long)h * a.tmax * 32;
    int r0 = ROWS * blockIdx.y, nr = min(ROWS, a.rows - r0);
    if (a.tiles) {
        const int* tl = a.tiles + 3 * blockIdx.y;
        kvbase += (long)tl[0] * a.seq_stride;
        r0 = tl[1];
        nr = tl[2];
    }
    const float sc = a.scale;
    const int row = 32 * w + r32;
    const int len = row < nr ? a.row_len[r0 + row] : 0;
    int wkmax = len;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) wkmax = max(wkmax, __shfl_xor(wkmax, o, 64));
    if (lane == 0) wk[w] = wkmax;
    // B fragments of S^T: (q s)[row][4t + 2 hs] (even chain) and [4t + 2 hs + 1] (odd)
    float qe[8], qo[8];
    {
        const float* qp = a.q + (long)(r0 + (row < nr ? row : 0)) * a.ldq + h * 32 + 2 * hs;
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            const float2 v = *reinterpret_cast<const float2*>(qp + 4 * t);
            qe[t] = v.x * sc;
            qo[t] = v.y * sc;
        }
    }
    __syncthreads();
    int kmax = 0;
#pragma unroll
    for (int i = 0; i < NW; ++i) kmax = max(kmax, wk[i]);
    const float* K = a.k + kvbase;
    const float* V = a.v + kvbase;
    auto dma = [&](int c) {
        const int slot = c % MF_RING;
#pragma unroll
        for (int i = 0; i < 8 / NW; ++i) {
            const int j = w + NW * i, key = MF_KC * c + 8 * j + (lane >> 3);
            const long src = (long)(key < kmax ? key : 0) * 32 + 4 * (lane & 7);
            gx3_dma(K + src, &Kr[slot][j * 256]);
            gx3_dma(V + src, &Vr[slot][j * 256]);
        }
    };
    // raw K of chunk c -> Kp = k s (padded rows)
    auto scale_k = [&](int c) {
        const int slot = c % MF_RING;
#pragma unroll
        for (int i = 0; i < MF_KC * 8 / NT; ++i) {
            const int e = tid + NT * i, t = e >> 3, cc = e & 7;
            const float4 v = *reinterpret_cast<const float4*>(&Kr[slot][t * 32 + 4 * cc]);
            float2* d = reinterpret_cast<float2*>(&Kp[t * MF_KR + 4 * cc]);
            d[0] = make_float2(v.x * sc, v.y * sc);
            d[1] = make_float2(v.z * sc, v.w * sc);
        }
    };
    float m = -INFINITY, l = 0.f;
    f32x16 o;
#pragma unroll
    for (int i = 0; i < 16; ++i) o[i] = 0.f;
    const int nch = (kmax + MF_KC - 1) / MF_KC;
    if (nch > 0) {
        for (int c = 0; c < MF_RING && c < nch; ++c) dma(c);
        gx3_wait<DPW>(min(MF_RING, nch) - 1);
        __syncthreads();
        scale_k(0);
    }
    __syncthreads();
    for (int c = 0; c < nch; ++c) {
        const int k0 = c * MF_KC, slot = c % MF_RING;
        if (k0 < wkmax) {
            f32x16 s[2];
#pragma unroll
            for (int T = 0; T < 2; ++T) {
                f32x16 se, so;
#pragma unroll
                for (int i = 0; i < 16; ++i) { se[i] = 0.f; so[i] = 0.f; }
                // A row r32 holds key krow: accumulator element i of lane half hs is then
                // key 2 i + hs (see above)
                const int krow = 8 * (r32 >> 3) + 2 * (r32 & 3) + ((r32 >> 2) & 1);
                const float* kr = &Kp[(32 * T + krow) * MF_KR + 2 * hs];
#pragma unroll
                for (int t = 0; t < 8; ++t) {
                    const float2 kk = *reinterpret_cast<const float2*>(kr + 4 * t);
                    se = __builtin_amdgcn_mfma_f32_32x32x2f32(kk.x, qe[t], se, 0, 0, 0);
                    so = __builtin_amdgcn_mfma_f32_32x32x2f32(kk.y, qo[t], so, 0, 0, 0);
                }
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    const int key = k0 + 32 * T + 2 * i + hs;
                    s[T][i] = key < len ? se[i] + so[i] : -INFINITY;
                }
            }
            float mc = -INFINITY;
#pragma unroll
            for (int T = 0; T < 2; ++T)
#pragma unroll
                for (int i = 0; i < 16; ++i) mc = fmaxf(mc, s[T][i]);
            mc = fmaxf(mc, __shfl_xor(mc, 32, 64));
            const float mn = fmaxf(m, mc);
            const float corr = mn == -INFINITY ? 1.f : __expf(m - mn);
#pragma unroll
            for (int T = 0; T < 2; ++T)
#pragma unroll
                for (int i = 0; i < 16; ++i) s[T][i] = s[T][i] == -INFINITY ? 0.f : __expf(s[T][i] - mn);
            // wave_sum's tree over the chunk's key index k = 32 T + 2 i + hs: k + 32 (T),
            // + 16 (i + 8), + 8 (i + 4), + 4 (i + 2), + 2 (i + 1), + 1 (the other lane half)
            float u[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) u[i] = (s[0][i] + s[1][i]) + (s[0][i + 8] + s[1][i + 8]);
#pragma unroll
            for (int i = 0; i < 4; ++i) u[i] = u[i] + u[i + 4];
            float sum = (u[0] + u[2]) + (u[1] + u[3]);
            sum = sum + __shfl_xor(sum, 32, 64);
            l = __builtin_fmaf(l, corr, sum);
            m = mn;
#pragma unroll
            for (int i = 0; i < 16; ++i) o[i] *= corr;
            // O^T += V^T P^T: step st takes keys (2 st, 2 st + 1); lane half hs supplies key
            // 2 st + hs, its own element st % 16 of tile st / 16
            const float* vr = &Vr[slot][hs * 32 + r32];
#pragma unroll
            for (int st = 0; st < 32; ++st)
                o = __builtin_amdgcn_mfma_f32_32x32x2f32(vr[64 * st], s[st >> 4][st & 15], o, 0, 0, 0);
        }
        if (c + 1 < nch) {
            gx3_wait<DPW>(min(c + MF_RING - 1, nch - 1) - (c + 1));
            __syncthreads();   // chunk c + 1 landed; every wave done with Kp and slot c
            if (c + MF_RING < nch) dma(c + MF_RING);
            scale_k(c + 1);
            __syncthreads();
        }
    }
    if (row < nr) {
        float* dst = a.out + (long)(r0 + row) * a.ldo + h * 32 + 4 * hs;
#pragma unroll
        for (int g = 0; g < 4; ++g)
            *reinterpret_cast<float4*>(dst + 8 * g) =
                make_float4(o[4 * g] / l, o[4 * g + 1] / l, o[4 * g + 2] / l, o[4 * g + 3] / l);
    }
}

void attn_rows_mf32(const AttnArgs& a, hipStream_t s) {
    if (a.ntiles <= 0) return;
    hipLaunchKernelGGL(k_attn_mf32<MF32_NW>, dim3(16, a.ntiles), dim3(64 * MF32_NW), 0, s, a);
}

// One sequence's prefill (rows = its N0 positions) on k_attn_mf32, one wave per 32 rows.
// Opt-in (GENIE_PREFILL_MF32=1): bit-identical to k_attn_flash, but no faster at ~300 rows
// in the single-sentence stream (15.28 vs 15.32 ms per utterance, profiles/r05m_prefill_mf32_ab.txt)
bool prefill_mf32_on() {
    static const bool on = [] { const char* e = std::getenv("GENIE_PREFILL_MF32"); return e && std::atoi(e) != 0; }();
    return on;
}
void attn_rows_mf32_seq(const AttnArgs& a, hipStream_t s) {
    if (a.rows <= 0) return;
    hipLaunchKernelGGL(k_attn_mf32<1>, dim3(16, (a.rows + 31) / 32), dim3(64), 0, s, a);
}

void attn_rows_rowlane(const AttnArgs& a, hipStream_t s) {
    if (a.ntiles <= 0) return;
    hipLaunchKernelGGL(k_attn_rowlane<ROWLANE_NW>, dim3(16, a.ntiles), dim3(64 * ROWLANE_NW), 0, s, a);
}

// (One sequence's prefill stays on k_attn_flash: at ~300 rows the MFMA kernel's 80
// blocks of 64 rows were no faster -- prefill 2.00 vs 1.91 ms, profiles/r04q_prefill_attn.txt.)
void attn_rows(const AttnArgs& a, hipStream_t s) {
    if (a.rows <= 0) return;
    static const bool flash = [] {
        const char* e = std::getenv("GENIE_ATTN_FLASH");
        return !(e && std::atoi(e) == 0);
    }();
    if (flash && !a.row_seq && !a.row_skip) {
        hipLaunchKernelGGL(k_attn_flash, dim3(16, (a.rows + AF_ROWS - 1) / AF_ROWS), dim3(256), 0, s, a);
        return;
    }
    // prefill of one sequence (row r sees keys [0, row_len[r]) <= rows).  Off by
    // default: measured slower than k_attn_rows at N0 = 225 (prefill 2.14 vs 1.83 ms)
    static const bool tile = [] {
        const char* e = std::getenv("GENIE_ATTN_TILE");
        return e && std::atoi(e) != 0;
    }();
    if (tile && !a.row_seq && !a.row_skip && a.rows <= AT_MAXK) {
        hipLaunchKernelGGL(k_attn_tile, dim3(16, (a.rows + AT_ROWS - 1) / AT_ROWS), dim3(1024), 0, s, a);
        return;
    }
    hipLaunchKernelGGL(k_attn_rows, dim3(16, a.rows), dim3(256), 0, s, a, 0);
}

void attn_rows_tiled(const AttnArgs& a, hipStream_t s) {
    if (a.ntiles <= 0) return;
    static_assert(AT_MAXK == ATTN_TILE_MAXK, "tile key capacity");
    hipLaunchKernelGGL(k_attn_tile, dim3(16, a.ntiles), dim3(1024), 0, s, a);
}

void attn_rows_flash_tiled(const AttnArgs& a, hipStream_t s) {
    if (a.ntiles <= 0) return;
    hipLaunchKernelGGL(k_attn_flash, dim3(16, a.ntiles), dim3(256), 0, s, a);
}

void attn_rows_plus(const AttnArgs& a, int len_add, hipStream_t s) {
    if (a.rows <= 0) return;
    hipLaunchKernelGGL(k_attn_rows, dim3(16, a.rows), dim3(256), 0, s, a, len_add);
}

// =====================================================================
// Decode GEMV: fp16 weights streamed straight to VGPRs (16 B / lane), fp32
// activations from LDS, optional LayerNorm prologue (LN fused into consumer).
// Each wave owns ROWS output rows for all B sequences.
// =====================================================================
template <int K, int ROWS, int NB>
__global__ __launch_bounds__(256) void k_gemv(GemvArgs a) {
    extern __shared__ float xs[];   // [NB][K]
    __shared__ float red[64];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int B = a.B;
    // weights first: their HBM latency overlaps the activation load + LN prologue
    GSV_STAMP(a.trace, 0);
    const int nbase = (blockIdx.x * 4 + w) * ROWS;
    constexpr int KI = K / 512;
    uint4 wr[ROWS][KI];
    // weights are loaded after the prologue's activation loads (vmcnt retires in
    // order: anything issued behind the weight stream would wait for all of it)
    auto load_weights = [&]() {
#pragma unroll
        for (int r = 0; r < ROWS; ++r) {
            const int n = min(nbase + r, a.N - 1);
            const __half* wp = a.W + (long)n * K + lane * 8;
#pragma unroll
            for (int i = 0; i < KI; ++i) wr[r][i] = *reinterpret_cast<const uint4*>(wp + i * 512);
        }
    };
    // every small parameter the later phases need, loaded now (no round trip after a barrier)
    float bias_r[ROWS];
#pragma unroll
    for (int r = 0; r < ROWS; ++r) bias_r[r] = a.bias ? a.bias[min(nbase + r, a.N - 1)] : 0.f;
    float lng0 = 0.f, lng1 = 0.f, lnb0 = 0.f, lnb1 = 0.f;
    if (a.ln_g) { lng0 = a.ln_g[tid]; lng1 = a.ln_g[tid + 256]; lnb0 = a.ln_b[tid]; lnb1 = a.ln_b[tid + 256]; }
    int kvpos[NB];
#pragma unroll
    for (int b = 0; b < NB; ++b)
        kvpos[b] = (a.mode == EPI_QKV && b < B) ? (a.kv.row_pos ? a.kv.row_pos[b] : a.kv.pos0) : 0;
    if (a.ln_g) {
        float v0[NB], v1[NB];
#pragma unroll
        for (int b = 0; b < NB; ++b) {
            if (b < B) {
                if (a.acc_in) {
                    const long long* ac = a.acc_in + (long)b * a.acc_bstride;
                    v0[b] = a.part_res[(long)b * 512 + tid] + (a.part_bias[tid] + from_fx(ac[tid]));
                    v1[b] = a.part_res[(long)b * 512 + tid + 256] + (a.part_bias[tid + 256] + from_fx(ac[tid + 256]));
                } else if (a.part) {
                    // split-K partial reduce: res + (bias + sum_j part_j), fixed order
                    float p0 = a.part_bias[tid], p1 = a.part_bias[tid + 256];
                    for (int j0 = 0; j0 < a.n_part; j0 += 16) {
                        float q0[16], q1[16];
#pragma unroll
                        for (int jj = 0; jj < 16; ++jj) {
                            const float* pp = a.part + (long)(j0 + jj) * a.part_stride + (long)b * 512;
                            q0[jj] = pp[tid];
                            q1[jj] = pp[tid + 256];
                        }
#pragma unroll
                        for (int jj = 0; jj < 16; ++jj) { p0 += q0[jj]; p1 += q1[jj]; }
                    }
                    v0[b] = a.part_res[(long)b * 512 + tid] + p0;
                    v1[b] = a.part_res[(long)b * 512 + tid + 256] + p1;
                } else {
                    v0[b] = a.src[(long)b * a.lds + tid];
                    v1[b] = a.src[(long)b * a.lds + tid + 256];
                }
            }
        }
        load_weights();
        float mean[NB], den[NB];
        block_meanvar512<NB>(v0, v1, B, mean, den, red);
        GSV_STAMP(a.trace, 1);
#pragma unroll
        for (int b = 0; b < NB; ++b) {
            if (b >= B) break;
            const float o0 = (v0[b] - mean[b]) / den[b] * lng0 + lnb0;
            const float o1 = (v1[b] - mean[b]) / den[b] * lng1 + lnb1;
            xs[b * K + tid] = o0;
            xs[b * K + tid + 256] = o1;
            if (a.ln_out && blockIdx.x == 0) {
                a.ln_out[(long)b * 512 + tid] = o0;
                a.ln_out[(long)b * 512 + tid + 256] = o1;
            }
        }
    } else {
        load_weights();
        for (int b = 0; b < B; ++b)
            for (int i = tid * 4; i < K; i += 1024)
                *reinterpret_cast<float4*>(&xs[b * K + i]) =
                    *reinterpret_cast<const float4*>(a.src + (long)b * a.lds + i);
    }
    __syncthreads();
    GSV_STAMP(a.trace, 2);
    float acc[ROWS][NB];
#pragma unroll
    for (int r = 0; r < ROWS; ++r)
#pragma unroll
        for (int b = 0; b < NB; ++b) acc[r][b] = 0.f;
#pragma unroll
    for (int i = 0; i < KI; ++i) {
        float wf[ROWS][8];
#pragma unroll
        for (int r = 0; r < ROWS; ++r) h8_to_f8(wr[r][i], wf[r]);
#pragma unroll
        for (int b = 0; b < NB; ++b) {
            if (b < B) {
                const float4 x0 = *reinterpret_cast<const float4*>(&xs[b * K + i * 512 + lane * 8]);
                const float4 x1 = *reinterpret_cast<const float4*>(&xs[b * K + i * 512 + lane * 8 + 4]);
#pragma unroll
                for (int r = 0; r < ROWS; ++r) {
                    float s = acc[r][b];
                    s += wf[r][0] * x0.x; s += wf[r][1] * x0.y; s += wf[r][2] * x0.z; s += wf[r][3] * x0.w;
                    s += wf[r][4] * x1.x; s += wf[r][5] * x1.y; s += wf[r][6] * x1.z; s += wf[r][7] * x1.w;
                    acc[r][b] = s;
                }
            }
        }
    }
    GSV_STAMP(a.trace, 3);
#pragma unroll
    for (int r = 0; r < ROWS; ++r) {
        const int n = nbase + r;
#pragma unroll
        for (int b = 0; b < NB; ++b) {
            if (b >= B) continue;
            const float sum = wave_sum_dpp(acc[r][b]);
            if (lane != 0 || n >= a.N) continue;
            const float v = a.bias ? bias_r[r] + sum : sum;
            switch (a.mode) {
                case EPI_STORE: a.C[(long)b * a.ldc + n] = v; break;
                case EPI_RELU: a.C[(long)b * a.ldc + n] = fmaxf(v, 0.f); break;
                case EPI_RESID: a.C[(long)b * a.ldc + n] = a.res[(long)b * a.ldr + n] + v; break;
                case EPI_QKV:
                    if (n < 512) {
                        a.C[(long)b * a.ldc + n] = v;
                    } else {
                        if (a.kv.row_skip && a.kv.row_skip[b]) break;
                        const int pos = kvpos[b];
                        const int c = (n - 512) & 511;
                        float* dst = (n < 1024 ? a.kv.k : a.kv.v) + (long)b * a.kv.seq_stride;
                        dst[((long)(c >> 5) * a.kv.tmax + pos) * 32 + (c & 31)] = v;
                    }
                    break;
                default: break;
            }
        }
    }
    GSV_STAMP(a.trace, 4);
}

template <int K, int ROWS>
static void launch_gemv_k(const GemvArgs& a, hipStream_t s) {
    const int rows_per_block = 4 * ROWS;
    dim3 grid((a.N + rows_per_block - 1) / rows_per_block);
    int nb = a.B <= 1 ? 1 : a.B <= 2 ? 2 : a.B <= 4 ? 4 : 8;
    const size_t shm = (size_t)nb * K * sizeof(float);
    switch (nb) {
        case 1: hipLaunchKernelGGL((k_gemv<K, ROWS, 1>), grid, dim3(256), shm, s, a); break;
        case 2: hipLaunchKernelGGL((k_gemv<K, ROWS, 2>), grid, dim3(256), shm, s, a); break;
        case 4: hipLaunchKernelGGL((k_gemv<K, ROWS, 4>), grid, dim3(256), shm, s, a); break;
        default: hipLaunchKernelGGL((k_gemv<K, ROWS, 8>), grid, dim3(256), shm, s, a); break;
    }
}

void gemv_f16(const GemvArgs& a, hipStream_t s) {
    if (a.K == 512) {
        if (a.N >= 1536) launch_gemv_k<512, 2>(a, s);
        else launch_gemv_k<512, 1>(a, s);
    } else {
        launch_gemv_k<2048, 1>(a, s);
    }
}

// One NT-thread block per sequence; logits in registers.  top-k threshold = k-th
// largest penalised logit WITH multiplicity (TopK values[:, -1], stage#1786-1790).
template <int NT>
__global__ __launch_bounds__(NT) void k_sample(SampleArgs a) {
    __shared__ SampleLds<NT> sh;
    __shared__ uint32_t seen_s[33];
    const int b = blockIdx.x, tid = threadIdx.x;
    const float* lg = a.logits + (long)b * a.ldl;
    const uint32_t* seen = a.seen + (long)b * 33;
    if (a.acc_zero) {   // this step's hand-off accumulators: every reader has run
        long long* z = a.acc_zero + (long)b * a.acc_n;
        for (long i = tid * 2; i < a.acc_n; i += 2 * NT)
            *reinterpret_cast<longlong2*>(z + i) = make_longlong2(0, 0);
    }
    // sequence state for the tail, read up front (no dependent round trips at the end)
    int st_ny = 0, st_steps = 0, st_kv = 0, st_stop = 0;
    if (tid == 0) {
        st_ny = a.ny[b];
        if (!a.prefill) {
            st_steps = a.steps[b];
            st_kv = a.kvlen[b];
            if (a.stop_req) st_stop = __hip_atomic_load(a.stop_req, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
    if (tid < 33) seen_s[tid] = seen[tid];
    const bool skip = !a.prefill && a.done[b];
    if (skip) {
        if (tid == 0 && a.stop_out) a.stop_out[b] = 0;
        return;
    }
    __shared__ int step_s;
    if (tid == 0) step_s = st_steps;
    __syncthreads();
    const int step = a.prefill ? 0 : step_s + 1;
    int raw = 0;
    const int tok = sample_block<NT>([&](int i) { return lg[i]; }, seen_s, a.b0 + b, step, a.top_k, a.temperature,
                                     a.rep_penalty, a.greedy, a.seed, a.ablate,
                                     a.logits_out ? a.logits_out + (long)b * a.ldlo : nullptr, &raw, sh);
    if (tid == 0) {
        if (a.ablate == 3) { a.y[(long)b * a.ldy + st_ny] = raw; a.ny[b] = st_ny + 1; return; }
        sample_commit(a, b, tok, raw, st_ny, st_steps, st_kv, seen_s);
        if (st_stop) {   // gsv_request_stop: the sequence ends here (the host returns STOPPED)
            a.done[b] = 1;
            if (a.stop_hit) __hip_atomic_store(a.stop_hit, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

void sample_tokens(const SampleArgs& a, hipStream_t s) {
    if (a.threads == 512) hipLaunchKernelGGL(k_sample<512>, dim3(a.B), dim3(512), 0, s, a);
    else hipLaunchKernelGGL(k_sample<256>, dim3(a.B), dim3(256), 0, s, a);
}

__global__ __launch_bounds__(256) void k_seq_init(int b, const int64_t* prompts, int P, int L,
                                                  int64_t* y, long ldy, int* ny, int* kvlen,
                                                  int* steps, uint8_t* done, uint32_t* seen) {
    __shared__ uint32_t bits[33];
    if (threadIdx.x < 33) bits[threadIdx.x] = 0;
    __syncthreads();
    for (int i = threadIdx.x; i < P; i += 256) {
        const int64_t t = prompts[i];
        y[(long)b * ldy + i] = t;
        atomicOr(&bits[t >> 5], 1u << (t & 31));
    }
    __syncthreads();
    if (threadIdx.x < 33) seen[(long)b * 33 + threadIdx.x] = bits[threadIdx.x];
    if (threadIdx.x == 0) {
        ny[b] = P;
        kvlen[b] = L + P;
        steps[b] = 0;
        done[b] = 0;
    }
}

void seq_state_init(int b, const int64_t* prompts, int P, int L, int64_t* y, long ldy, int* ny,
                    int* kvlen, int* steps, uint8_t* done, uint32_t* seen, hipStream_t s) {
    hipLaunchKernelGGL(k_seq_init, dim3(1), dim3(256), 0, s, b, prompts, P, L, y, ldy, ny, kvlen,
                       steps, done, seen);
}

}  // namespace gsv
