// Explicit instantiations of the weight-stationary wide GEMM (gemm_ws.h): the residual epilogue (out projection
// + residual add, model.py:578-580) and the rotary epilogue (q / k projections, model.py:198-214).
#define ASRX_WS_INSTANTIATE
#include "gemm_ws.h"

ASRX_WS_DECL(false, true, false)
ASRX_WS_DECL(true, false, true)
ASRX_WS_DECL(false, false, true)
