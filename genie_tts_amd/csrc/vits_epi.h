// conv1d output epilogue (bias + ConvMode fusion), shared by the f32 MFMA conv
// (vits.hip) and the f16-split MFMA conv (vits_convh.hip).
#pragma once
#include "vits.h"

namespace gsv {

// Output epilogue shared by the direct and the split-K paths: output column t of
// phase ph -> time tp; bias; the ConvMode fusion.
__device__ __forceinline__ void conv_epilogue(const ConvArgs& a, int co, int t, int ph, float acc) {
    const int tp = t * a.o_tstride + a.o_toff + ph;
    if (tp < 0 || tp >= a.o_len) return;
    const float v = a.bias ? a.bias[co] + acc : acc;
    const long oi = (long)co * a.o_cs + (long)tp * a.o_ts;
    const float* vec = a.vec;
    if (a.seg) {   // segmented batch: gaps stay zero
        const int sg = a.seg[tp];
        if (sg < 0) {
            if (a.mode == CV_SPLIT_RESID && co >= a.split)
                a.out2[(long)(co - a.split) * a.o_cs + (long)tp * a.o_ts] = 0.f;
            else
                (a.mode == CV_ACC_FIRST || a.mode == CV_ACC_ADD ? a.acc : a.out)[oi] = 0.f;
            return;
        }
        if (vec) vec += (long)sg * a.vec_sstride;
    }
    switch (a.mode) {
        case CV_STORE: a.out[oi] = v; break;
        case CV_RELU: a.out[oi] = fmaxf(v, 0.f); break;
        case CV_RESID: a.out[oi] = a.res[(long)co * a.r_cs + (long)tp * a.r_ts] + v; break;
        case CV_VEC: a.out[oi] = v + vec[co]; break;
        case CV_SUB: a.out[oi] = a.res[(long)co * a.r_cs + (long)tp * a.r_ts] - v; break;
        case CV_TANH: a.out[oi] = tanhf(v); break;
        case CV_ACC_FIRST: a.acc[oi] = a.res[(long)co * a.r_cs + (long)tp * a.r_ts] + v; break;
        case CV_ACC_ADD: a.acc[oi] = a.acc[oi] + (a.res[(long)co * a.r_cs + (long)tp * a.r_ts] + v); break;
        case CV_ACC_MEAN:
            a.out[oi] = (a.acc[oi] + (a.res[(long)co * a.r_cs + (long)tp * a.r_ts] + v)) / a.div;
            break;
        case CV_RESID_VEC:
            a.out[oi] = (a.res[(long)co * a.r_cs + (long)tp * a.r_ts] + v) + vec[co];
            break;
        case CV_SPLIT_RESID:
            if (co < a.split) {
                a.out[oi] = a.res[(long)co * a.r_cs + (long)tp * a.r_ts] + v;
            } else {
                const long o2 = (long)(co - a.split) * a.o_cs + (long)tp * a.o_ts;
                a.out2[o2] = a.res2[o2] + v;
            }
            break;
    }
}

// The epilogue of one MFMA 32x32 accumulator column: 16 rows
// co_r = cobase + (r & 3) + 8 (r >> 2) at output column t.  The ConvMode is
// decomposed into wave-uniform flags, each a branch around a 16-row loop (a
// per-row switch unrolls into ~1000 branches and thrashes the instruction
// cache), and every load of a stage is issued before its first use; the
// arithmetic order of each mode is that of conv_epilogue.
template <bool FULL>
__device__ __forceinline__ void conv_epilogue16_(const ConvArgs& a, int cobase, int tp, int t, int ph,
                                                 const float (&val)[16]) {
    const int mode = a.mode;
    const float* vecp = a.vec;
    if (a.seg) {   // segmented batch: a gap column is written as zeros
        const int sg = a.seg[tp];
        if (sg < 0 && mode == CV_SPLIT_RESID) {   // rows past `split` belong to out2
            for (int r = 0; r < 16; ++r) {
                const int co = cobase + (r & 3) + 8 * (r >> 2);
                if (co < a.Cout) conv_epilogue(a, co, t, ph, 0.f);
            }
            return;
        }
        if (sg < 0) {
            const int nrow = FULL ? 32 : a.Cout - cobase;
            float* dst = (mode == CV_ACC_FIRST || mode == CV_ACC_ADD ? a.acc : a.out) + (long)cobase * a.o_cs +
                         (long)tp * a.o_ts;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int d = (r & 3) + 8 * (r >> 2);
                if (d < nrow) dst[(long)d * a.o_cs] = 0.f;
            }
            return;
        }
        if (vecp) vecp += (long)sg * a.vec_sstride;
    }
    if (mode == CV_SPLIT_RESID) {
        for (int r = 0; r < 16; ++r) {
            const int co = cobase + (r & 3) + 8 * (r >> 2);
            if (co < a.Cout) conv_epilogue(a, co, t, ph, val[r]);
        }
        return;
    }
    const bool f_res = mode == CV_RESID || mode == CV_SUB || mode == CV_ACC_FIRST || mode == CV_ACC_ADD ||
                       mode == CV_ACC_MEAN || mode == CV_RESID_VEC;
    const bool f_acc = mode == CV_ACC_ADD || mode == CV_ACC_MEAN;
    const bool f_vec = mode == CV_VEC || mode == CV_RESID_VEC;
    const bool to_acc = mode == CV_ACC_FIRST || mode == CV_ACC_ADD;
    const int nrow = FULL ? 32 : a.Cout - cobase;   // row r valid iff (r & 3) + 8 (r >> 2) < nrow
    float y[16];
    if (a.bias) {
        float bv[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int d = (r & 3) + 8 * (r >> 2);
            bv[r] = d < nrow ? a.bias[cobase + d] : 0.f;
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) y[r] = bv[r] + val[r];
    } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) y[r] = val[r];
    }
    if (f_res) {
        float rv[16];
        const float* R = a.res + (long)cobase * a.r_cs + (long)tp * a.r_ts;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int d = (r & 3) + 8 * (r >> 2);
            rv[r] = d < nrow ? R[(long)d * a.r_cs] : 0.f;
        }
        if (mode == CV_SUB) {
#pragma unroll
            for (int r = 0; r < 16; ++r) y[r] = rv[r] - y[r];
        } else {
#pragma unroll
            for (int r = 0; r < 16; ++r) y[r] = rv[r] + y[r];
        }
    }
    const long obase = (long)cobase * a.o_cs + (long)tp * a.o_ts;
    if (f_acc) {
        float av[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int d = (r & 3) + 8 * (r >> 2);
            av[r] = d < nrow ? a.acc[obase + (long)d * a.o_cs] : 0.f;
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) y[r] = av[r] + y[r];
    }
    if (f_vec) {
        float vv[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int d = (r & 3) + 8 * (r >> 2);
            vv[r] = d < nrow ? vecp[cobase + d] : 0.f;
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) y[r] = y[r] + vv[r];
    }
    if (mode == CV_ACC_MEAN) {
#pragma unroll
        for (int r = 0; r < 16; ++r) y[r] = y[r] / a.div;
    } else if (mode == CV_RELU) {
#pragma unroll
        for (int r = 0; r < 16; ++r) y[r] = fmaxf(y[r], 0.f);
    } else if (mode == CV_TANH) {
        for (int r = 0; r < 16; ++r) y[r] = tanhf(y[r]);
    }
    float* dst = (to_acc ? a.acc : a.out) + obase;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int d = (r & 3) + 8 * (r >> 2);
        if (d < nrow) dst[(long)d * a.o_cs] = y[r];
    }
}

// The lean form for the persistent conv (vits_convh.hip, PERS), whose epilogue sits inside
// its tile loop: modes STORE, RESID, ACC_FIRST / ADD / MEAN only (the MRF convs and the
// ConvTranspose), the same arithmetic order as conv_epilogue16_.
__device__ __forceinline__ bool conv_epilogue_lean_mode(int mode) {
    return mode == CV_STORE || mode == CV_RESID || mode == CV_ACC_FIRST || mode == CV_ACC_ADD || mode == CV_ACC_MEAN;
}
__device__ __forceinline__ void conv_epilogue16_lean(const ConvArgs& a, int cobase, int t, int ph,
                                                     const float (&val)[16]) {
    const int tp = t * a.o_tstride + a.o_toff + ph;
    if (tp < 0 || tp >= a.o_len) return;
    const int mode = a.mode;
    const int nrow = a.Cout - cobase;   // row r valid iff (r & 3) + 8 (r >> 2) < nrow
    const bool to_acc = mode == CV_ACC_FIRST || mode == CV_ACC_ADD;
    const long obase = (long)cobase * a.o_cs + (long)tp * a.o_ts;
    float* dst = (to_acc ? a.acc : a.out) + obase;
    if (a.seg && a.seg[tp] < 0) {   // a gap column of a segmented batch: zeros
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int d = (r & 3) + 8 * (r >> 2);
            if (d < nrow) dst[(long)d * a.o_cs] = 0.f;
        }
        return;
    }
    float y[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int d = (r & 3) + 8 * (r >> 2);
        y[r] = a.bias ? (d < nrow ? a.bias[cobase + d] : 0.f) + val[r] : val[r];
    }
    if (mode != CV_STORE) {
        const float* R = a.res + (long)cobase * a.r_cs + (long)tp * a.r_ts;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int d = (r & 3) + 8 * (r >> 2);
            y[r] = (d < nrow ? R[(long)d * a.r_cs] : 0.f) + y[r];
        }
    }
    if (mode == CV_ACC_ADD || mode == CV_ACC_MEAN) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int d = (r & 3) + 8 * (r >> 2);
            y[r] = (d < nrow ? a.acc[obase + (long)d * a.o_cs] : 0.f) + y[r];
        }
    }
    if (mode == CV_ACC_MEAN) {
#pragma unroll
        for (int r = 0; r < 16; ++r) y[r] = y[r] / a.div;
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int d = (r & 3) + 8 * (r >> 2);
        if (d < nrow) dst[(long)d * a.o_cs] = y[r];
    }
}

__device__ __forceinline__ void conv_epilogue16(const ConvArgs& a, int cobase, int t, int ph,
                                                const float (&val)[16]) {
    const int tp = t * a.o_tstride + a.o_toff + ph;
    if (tp < 0 || tp >= a.o_len) return;
    if (cobase + 28 < a.Cout) conv_epilogue16_<true>(a, cobase, tp, t, ph, val);   // all 16 rows (max d = 27)
    else conv_epilogue16_<false>(a, cobase, tp, t, ph, val);
}

}  // namespace gsv
