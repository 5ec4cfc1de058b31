// Explicit instantiations of the weight-stationary wide GEMM (gemm_ws.h): bf16-stored activations, every
// activation epilogue.
#define ASRX_WS_INSTANTIATE
#include "gemm_ws.h"

ASRX_WS_DECL_ACT(true)
