// Explicit instantiations of the tied-logits wide GEMM with the fused cross-entropy statistics
// epilogue (gemm_wr.h epilogue_ce), 128- and 256-column tiles.
#define ASRX_WR_INSTANTIATE
#include "gemm_wr.h"

ASRX_WR_DECL_CE(1)
ASRX_WR_DECL_CE(2)
