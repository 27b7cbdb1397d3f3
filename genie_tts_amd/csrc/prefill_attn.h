// Prefill attention on the split-fp16 MFMA (k_attn_mfma, t2s.hip).
#pragma once
#include "kernels.h"

namespace gsv {

// Blocks of rows_per_block (64 or 128) query rows of one head, or a.tiles of
// <= rows_per_block rows of one sequence (any key count).
void attn_rows_mfma(const AttnArgs& a, int rows_per_block, hipStream_t s);
// default off (GENIE_ATTN_MFMA=1 turns it on): the packed prefill's attention stays on the
// f32 kernels a single sentence's prefill uses, so batched and single tokens agree
bool attn_mfma_on();
// f32, k_attn_flash's per-row arithmetic with one query row per lane: a.tiles of
// <= 64 ROWLANE_NW rows of one sequence
constexpr int ROWLANE_NW = 2;
void attn_rows_rowlane(const AttnArgs& a, hipStream_t s);
// f32 MFMA, the same per-row arithmetic (v_mfma_f32_32x32x2f32 is a sequential fma
// chain): a.tiles of <= 32 MF32_NW rows of one sequence
constexpr int MF32_NW = 4;
void attn_rows_mf32(const AttnArgs& a, hipStream_t s);
// one sequence (a.tiles null, rows from 0), 32 rows per single-wave block
bool prefill_mf32_on();
void attn_rows_mf32_seq(const AttnArgs& a, hipStream_t s);

}  // namespace gsv
