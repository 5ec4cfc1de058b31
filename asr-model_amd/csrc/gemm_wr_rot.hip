// Explicit instantiations of the wide GEMM with the rotary epilogue (Params::rot_*: the q / k projections of
// attention with rotary applied before the store, model.py:242-245, 198-214): 128-column tiles (the text
// side's 8192-row launches) and 384-column tiles (the nj = 3 launches gemm_p2 does not take: fp32 A at
// >= 131072 rows, or gemm variant 0), bf16 and fp32 A.
#define ASRX_WR_INSTANTIATE
#include "gemm_wr.h"

ASRX_WR_DECL_ROT(1, true)
ASRX_WR_DECL_ROT(1, false)
ASRX_WR_DECL_ROT(3, true)
ASRX_WR_DECL_ROT(3, false)
