// Explicit instantiations of the two-workgroups-per-CU wide GEMM (gemm_p2.h), one unit per group so
// the build compiles them in parallel.
#define ASRX_P2_INSTANTIATE
#include "gemm_p2.h"

ASRX_P2_DECL(3, false, false)
