// One explicit instantiation of the 384-column wide GEMM (gemm_wr.h) per translation unit: the
// NJ = 3 kernels take minutes each to compile, so the build runs them in parallel.
#define ASRX_WR_INSTANTIATE
#include "gemm_wr.h"

ASRX_WR_DECL(3, false, false, false)
