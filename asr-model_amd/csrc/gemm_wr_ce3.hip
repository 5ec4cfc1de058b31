// Explicit instantiation of the tied-logits wide GEMM with the fused cross-entropy statistics
// epilogue (gemm_wr.h epilogue_ce), 384-column tiles (the V = 40000 logits of every config).
#define ASRX_WR_INSTANTIATE
#include "gemm_wr.h"

ASRX_WR_DECL_CE(3)
