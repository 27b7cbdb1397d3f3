// Prefill attention on the split-fp16 MFMA (k_attn_mfma, t2s.hip).
#pragma once
#include "kernels.h"

namespace gsv {

// Blocks of rows_per_block (64 or 128) query rows of one head, or a.tiles of
// <= rows_per_block rows of one sequence (any key count).
void attn_rows_mfma(const AttnArgs& a, int rows_per_block, hipStream_t s);
// default on; GENIE_ATTN_MFMA=0 keeps the prefill attention on the f32 kernels
bool attn_mfma_on();

}  // namespace gsv
