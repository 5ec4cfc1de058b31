// Explicit instantiations of the wide GEMM with the residual-add epilogue (out projections,
// model.py:578-580): 128- and 384-column tiles, fp32 A.
#define ASRX_WR_INSTANTIATE
#include "gemm_wr.h"

ASRX_WR_DECL_RES(1)
ASRX_WR_DECL_RES(3)
