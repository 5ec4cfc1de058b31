// Explicit instantiations of the weight-stationary wide GEMM (gemm_ws.h): fp32 activations, every activation
// epilogue.
#define ASRX_WS_INSTANTIATE
#include "gemm_ws.h"

ASRX_WS_DECL_ACT(false)
