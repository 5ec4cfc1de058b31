// The 128-row tiles of an M-row activation whose rows r belong to a sample b = r / L at MSheath layer `layer`
// (next_i[b] == layer), listed in increasing order in mtiles[0 .. *n_out): the row-tile list the wide GEMM's row-list
// launches walk (asrx_gemm_wn_rows).  One workgroup of NT threads; every thread of it must call.  ACQ: read next_i
// with agent-scope atomic loads (values written by other workgroups of the same launch, published by a fence).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace asrx {

constexpr int RT_BM = 128;

template <int NT, bool ACQ>
__device__ __forceinline__ void build_row_tiles(const float* next_i, int layer, int64_t L, int64_t M, int* mtiles,
                                                int* n_out) {
  static_assert(NT % 64 == 0 && NT <= 1024, "whole waves");
  __shared__ int wsum[NT / 64];
  __shared__ int base;
  const int nm = (int)((M + RT_BM - 1) / RT_BM);
  if (threadIdx.x == 0) base = 0;
  __syncthreads();
  for (int t0 = 0; t0 < nm; t0 += NT) {
    const int t = t0 + threadIdx.x;
    int act = 0;
    if (t < nm) {
      const int64_t r0 = (int64_t)t * RT_BM, r1 = min<int64_t>(r0 + RT_BM, M) - 1;
      for (int64_t b = r0 / L; b <= r1 / L && !act; ++b) {
        float v;
        if constexpr (ACQ) v = __hip_atomic_load(next_i + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else v = next_i[b];
        act = v == (float)layer;
      }
    }
    // block exclusive scan of act
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int v = act;
    for (int o = 1; o < 64; o <<= 1) {
      const int u = __shfl_up(v, o);
      if (lane >= o) v += u;
    }
    if (lane == 63) wsum[w] = v;
    __syncthreads();
    int off = base;
    for (int k = 0; k < w; ++k) off += wsum[k];
    if (act) mtiles[off + v - 1] = t;
    __syncthreads();
    if (threadIdx.x == 0) {
      int tot = 0;
      for (int k = 0; k < NT / 64; ++k) tot += wsum[k];
      base += tot;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) n_out[0] = base;
}

}  // namespace asrx
