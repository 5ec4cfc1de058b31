// Explicit instantiations of the two-workgroups-per-CU wide GEMM with the rotary epilogue (the audio side's
// q / k projections, model.py:242-245, 198-214).
#define ASRX_P2_INSTANTIATE
#include "gemm_p2.h"

ASRX_P2_DECL_ROT(3, true)
ASRX_P2_DECL_ROT(3, false)
