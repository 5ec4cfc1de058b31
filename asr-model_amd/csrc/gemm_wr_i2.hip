// Explicit instantiations of the wide GEMM (gemm_wr.h) for tiles of 256 columns: split over
// several translation units so the build compiles them in parallel.
#define ASRX_WR_INSTANTIATE
#include "gemm_wr.h"

ASRX_WR_SET(2)
