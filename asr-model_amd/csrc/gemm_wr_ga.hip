// Explicit instantiations of the wide GEMM with the activation-gradient epilogue (Params::G: the
// backward of a Linear + GELU / SiLU / sigmoid recomputes its pre-activation, model.py:143-147, 421-425,
// 573-574): 384-column tiles, fp32 and bf16 A.
#define ASRX_WR_INSTANTIATE
#include "gemm_wr.h"

ASRX_WR_DECL_GA(3, false)
ASRX_WR_DECL_GA(3, true)
