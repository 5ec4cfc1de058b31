// MaxFactor optimizer step (optimizerc.py:6-147, the optimizer model.py:783-787 builds), fused over
// every parameter of the model in eight launches instead of the reference's per-parameter loop of
// ~15 kernels and 4 host syncs (.item()) per parameter.
//
// Per parameter p with gradient g (all in fp32), step count t, group hyper-parameters:
//   beta = t^b_decay, rho = max(min_lr, min(lr, t^-1/2)), alpha = max(eps2, ||p|| / sqrt(n)) rho
//   p *= 1 - lr decay
//   matrices (dim > 1; a 3-D conv weight [A, B, C] is A matrices of B x C):
//     row_var = lerp(row_var, sum_c g^2 / (C + 1e-8), beta), col_var likewise over rows (/ (B + 1e-8))
//     var = row_var col_var^T / max(max_r row_var, eps1)
//   vectors: v = gamma v + (1 - gamma) g^2, var = v  (and v <- the normalised u afterwards, as the
//            reference's in-place ops on var_est leave it)
//   u = g rsqrt(max(var, eps1^2));  u /= max(max|u|, eps1) (when max|u| > 0)
//   denom = max(1, ||u|| / (sqrt(n) d))
//   dir = sign(u) * max_c |u|  (dim < 3 or group bias == 1)   |   sign(u) * median_c |u|  (otherwise)
//   p -= alpha / denom * dir
// Layout: every parameter is a list of rows (matrix rows, or one row for a vector); the row kernels
// walk a flat space of wave work items over all parameters (a binary search over the table's item
// offsets finds the parameter), so one launch covers the whole model.  A work item is one wave
// split into 64 / gsz lane groups of gsz = pow2 >= row length (<= 64) lanes, one row per group:
// the k3 conv weights are 2*D*D rows of 3 (a row per wave ran 3 of 64 lanes and made the step ~30x
// slower than its HBM bytes; now 16 rows share a wave).
#include "common.h"

namespace asrx {

struct MFParam {
  float* p;
  const float* g;
  float* rv;  // row_var [mats][rows]   (matrices)
  float* cv;  // col_var [mats][cols]   (matrices)
  float* v;   // v [n]                   (vectors)
  int64_t n;
  int mats, rows, cols;
  int mode;  // 0 vector (max), 1 matrix + max, 2 matrix + median
  float beta, rho, lr, decay, gamma, d, eps1, eps2;
  int64_t row0;  // offset of this parameter's rows in the flat row space (mats * rows, or 1)
  int64_t cc0;   // offset in the flat (mat, col, row-chunk) space of the column kernel
  int64_t col0;  // offset in the flat (mat, col) space
  int64_t mat0;  // offset in the flat mat space
  int64_t item0; // offset in the flat wave-work-item space of the row kernels
  int gsz;       // lanes per row (power of two <= 64); 64 / gsz rows per work item
  int pad_;
};

constexpr int MF_CHUNK = 256;  // rows per column-sum work item

__device__ __forceinline__ int find_param(const MFParam* t, int n, int64_t idx, int which) {
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    const int64_t off = which == 0 ? t[mid].row0 : which == 1 ? t[mid].cc0 : t[mid].col0;
    if (off <= idx) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

constexpr int MF_MAXP = 2048;  // parameters per call (the row-offset table is staged in LDS)

// Grid-stride loop over wave work items; the parameter of an item is found by a binary search over
// the item offsets staged in LDS (a global-memory search per row was the latency bottleneck).  The
// body gets the flat row, the parameter, whether the lane group holds a real row, the lane's index
// in its group and the group size; whole groups are valid or invalid together, so group-local
// shuffles stay well defined.
template <class F>
__device__ __forceinline__ void mf_for_rows(const MFParam* __restrict__ tab, int np, int64_t nitems, F&& body) {
  __shared__ int64_t offs[MF_MAXP];
  for (int k = threadIdx.x; k < np; k += blockDim.x) offs[k] = tab[k].item0;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  for (int64_t it = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); it < nitems; it += (int64_t)gridDim.x * 4) {
    int lo = 0, hi = np - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (offs[mid] <= it) lo = mid;
      else hi = mid - 1;
    }
    const int G = tab[lo].gsz;
    const int64_t nr = tab[lo].mode == 0 ? 1 : (int64_t)tab[lo].mats * tab[lo].rows;
    const int64_t lr_ = (it - offs[lo]) * (64 / G) + lane / G;
    body(tab[lo].row0 + lr_, lo, lr_ < nr, lane & (G - 1), G);
  }
}

// sums / maxima over the aligned group of G lanes (G a power of two)
__device__ __forceinline__ float grp_sum(float x, int G) {
  for (int o = G >> 1; o > 0; o >>= 1) x += __shfl_xor(x, o);
  return x;
}
__device__ __forceinline__ float grp_max(float x, int G) {
  for (int o = G >> 1; o > 0; o >>= 1) x = fmaxf(x, __shfl_xor(x, o));
  return x;
}

// stats per parameter: [0] sum p^2, [1] sum u^2, [2] max|u|, [3] unused
__device__ __forceinline__ float* pstats(float* stats, int i) { return stats + 4 * i; }

// ---- K1: row sums of g^2 -> row_var (matrices) or v (vectors); per-row sum of p^2 (reduced per
// parameter by K1b -- same-address atomics from thousands of rows would serialise)
__global__ __launch_bounds__(256) void mf_rows_kernel(const MFParam* __restrict__ tab, int np, int64_t nitems,
                                                      float* __restrict__ row_p2) {
  mf_for_rows(tab, np, nitems, [&](int64_t row, int i, bool ok, int sub, int G) {
    const MFParam P = tab[i];
    const int64_t lr_ = row - P.row0;
    const int64_t base = P.mode == 0 ? 0 : lr_ * P.cols;
    const int len = ok ? (P.mode == 0 ? (int)P.n : P.cols) : 0;
    float sg = 0.f, sp = 0.f;
#pragma unroll 8
    for (int c = sub; c < len; c += G) {
      const float g = P.g[base + c], w = P.p[base + c];
      sg += g * g;
      sp += w * w;
      if (P.mode == 0) P.v[c] = P.gamma * P.v[c] + (1.f - P.gamma) * g * g;
    }
    sg = grp_sum(sg, G);
    sp = grp_sum(sp, G);
    if (ok && sub == 0) {
      row_p2[row] = sp;
      if (P.mode != 0) {
        const float mean = sg / ((float)P.cols + 1e-8f);
        const float old = P.rv[lr_];
        P.rv[lr_] = old + P.beta * (mean - old);
      }
    }
  });
}

// ---- K1b / K4b: one workgroup per parameter reduces its rows' partials: stats[0] = sum p^2 and
// the per-matrix max of row_var (first pass), or stats[1] = sum u^2, stats[2] = max |u| (second)
__global__ __launch_bounds__(256) void mf_param_reduce_kernel(const MFParam* __restrict__ tab, int np, int pass,
                                                              const float* __restrict__ ra,
                                                              const float* __restrict__ rb, float* __restrict__ stats,
                                                              float* __restrict__ mrv) {
  __shared__ float red[8];
  const int i = blockIdx.x;
  const MFParam P = tab[i];
  const int64_t nr = P.mode == 0 ? 1 : (int64_t)P.mats * P.rows;
  float s = 0.f, mx = 0.f;
  for (int64_t r = threadIdx.x; r < nr; r += 256) {
    s += ra[P.row0 + r];
    if (pass == 1) mx = fmaxf(mx, rb[P.row0 + r]);
  }
  s = block_sum<256>(s, red);
  __syncthreads();
  if (pass == 1) {
    mx = wave_max(mx);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mx;
    __syncthreads();
    if (threadIdx.x == 0) {
      stats[4 * i + 1] = s;
      stats[4 * i + 2] = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    }
    return;
  }
  if (threadIdx.x == 0) stats[4 * i] = s;
  if (P.mode != 0) {  // max_r row_var per matrix (row_var >= 0)
    for (int m = threadIdx.x >> 6; m < P.mats; m += 4) {
      float v = 0.f;
      for (int r = threadIdx.x & 63; r < P.rows; r += 64) v = fmaxf(v, P.rv[(int64_t)m * P.rows + r]);
      v = wave_max(v);
      if ((threadIdx.x & 63) == 0) mrv[P.mat0 + m] = v;
    }
  }
}

// ---- K2: column sums of g^2 over chunks of MF_CHUNK rows (atomics into colacc)
__global__ __launch_bounds__(256) void mf_cols_kernel(const MFParam* __restrict__ tab, int np, int64_t ncc,
                                                      float* __restrict__ colacc) {
  const int64_t w = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (w >= ncc) return;
  const int i = find_param(tab, np, w, 1);
  const MFParam P = tab[i];
  if (P.mode == 0) return;
  const int64_t q = w - P.cc0;
  const int nch = (P.rows + MF_CHUNK - 1) / MF_CHUNK;
  const int col = (int)(q % P.cols);
  const int64_t rest = q / P.cols;
  const int ch = (int)(rest % nch), m = (int)(rest / nch);
  const int r0 = ch * MF_CHUNK, r1 = min(P.rows, r0 + MF_CHUNK);
  const float* g = P.g + (int64_t)m * P.rows * P.cols + col;
  float s = 0.f;
  for (int r = r0; r < r1; ++r) {
    const float x = g[(int64_t)r * P.cols];
    s += x * x;
  }
  atomicAdd(colacc + P.col0 + (int64_t)m * P.cols + col, s);
}

// ---- K3: col_var lerp (one thread per (param, mat, col))
__global__ __launch_bounds__(256) void mf_colfin_kernel(const MFParam* __restrict__ tab, int np, int64_t ncols,
                                                        const float* __restrict__ colacc) {
  const int64_t w = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (w >= ncols) return;
  const int i = find_param(tab, np, w, 2);
  const MFParam P = tab[i];
  if (P.mode == 0) return;
  const int64_t q = w - P.col0;
  const float mean = colacc[w] / ((float)P.rows + 1e-8f);
  const float old = P.cv[q];
  P.cv[q] = old + P.beta * (mean - old);
}

__device__ __forceinline__ float mf_u(const MFParam& P, float g, float rvi, float cvj, float mr) {
  float var;
  if (P.mode == 0) var = rvi;  // v
  else var = rvi * cvj / fmaxf(mr, P.eps1);
  return g * rsqrtf(fmaxf(var, P.eps1 * P.eps1));
}

// ---- K4: per row: u, row max |u| (or median |u|), and the parameter's sum u^2 / max |u|
__global__ __launch_bounds__(256) void mf_ustats_kernel(const MFParam* __restrict__ tab, int np, int64_t nitems,
                                                        const float* __restrict__ mrv, float* __restrict__ rowred,
                                                        float* __restrict__ row_u2, float* __restrict__ row_umax) {
  mf_for_rows(tab, np, nitems, [&](int64_t row, int i, bool ok, int sub, int G) {
    const MFParam P = tab[i];
    const int64_t lr_ = ok ? row - P.row0 : 0;
    const int len = ok ? (P.mode == 0 ? (int)P.n : P.cols) : 0;
    const int64_t base = P.mode == 0 ? 0 : lr_ * P.cols;
    const int m = P.mode == 0 ? 0 : (int)(lr_ / P.rows);
    const float rvi = P.mode == 0 ? 0.f : P.rv[lr_];
    const float mr = P.mode == 0 ? 0.f : mrv[P.mat0 + m];
    const float* cvr = P.mode == 0 ? P.v : P.cv + (int64_t)m * P.cols;
    auto u_at = [&](int c) { return mf_u(P, P.g[base + c], P.mode == 0 ? cvr[c] : rvi, cvr[c], mr); };
    float su = 0.f, mx = 0.f;
#pragma unroll 8
    for (int c = sub; c < len; c += G) {
      const float u = u_at(c);
      su += u * u;
      mx = fmaxf(mx, fabsf(u));
    }
    su = grp_sum(su, G);
    mx = grp_max(mx, G);
    float red = mx;
    if (P.mode == 2) {
      // lower median of |u| over the row (torch.median): MSB-first radix select on the float bits
      // (|u| >= 0 orders as uint), |u| recomputed per pass -- median rows are short (conv taps)
      const int k = (len - 1) / 2;
      uint32_t prefix = 0, mask = 0;
      int below = 0;
      for (int bit = 31; bit >= 0; --bit) {
        const uint32_t m2 = mask | (1u << bit);
        float cnt = 0.f;
        for (int c = sub; c < len; c += G)
          cnt += ((__builtin_bit_cast(uint32_t, fabsf(u_at(c))) & m2) == prefix) ? 1.f : 0.f;
        const int total = (int)grp_sum(cnt, G);
        if (below + total <= k) {
          below += total;
          prefix |= 1u << bit;
        }
        mask = m2;
      }
      red = __builtin_bit_cast(float, prefix);
    }
    if (ok && sub == 0) {
      rowred[row] = red;
      row_u2[row] = su;
      row_umax[row] = mx;
    }
  });
}

// ---- K5: apply
__global__ __launch_bounds__(256) void mf_apply_kernel(const MFParam* __restrict__ tab, int np, int64_t nitems,
                                                       const float* __restrict__ mrv, const float* __restrict__ rowred,
                                                       const float* __restrict__ stats) {
  mf_for_rows(tab, np, nitems, [&](int64_t row, int i, bool ok, int sub, int G) {
    if (!ok) return;  // no group-wide shuffles below
    const MFParam P = tab[i];
    const int64_t lr_ = row - P.row0;
    const int len = P.mode == 0 ? (int)P.n : P.cols;
    const int64_t base = P.mode == 0 ? 0 : lr_ * P.cols;
    const int m = P.mode == 0 ? 0 : (int)(lr_ / P.rows);
    const float rvi = P.mode == 0 ? 0.f : P.rv[lr_];
    const float mr = P.mode == 0 ? 0.f : mrv[P.mat0 + m];
    const float* st = pstats(const_cast<float*>(stats), i);
    const float n = (float)P.n;
    const float alpha = fmaxf(P.eps2, sqrtf(st[0]) / sqrtf(n)) * P.rho;
    const float inf = st[2];
    const float div = inf > 0.f ? fmaxf(inf, P.eps1) : 1.f;  // update /= max(inf, eps1) when inf > 0
    const float denom = fmaxf(1.f, sqrtf(st[1]) / div / (sqrtf(n) * P.d));
    const float scale = rowred[row] / div;
    const float step = alpha / denom;
    const float keep = 1.f - P.lr * P.decay;
    const float* cvr = P.mode == 0 ? P.v : P.cv + (int64_t)m * P.cols;
#pragma unroll 8
    for (int c = sub; c < len; c += G) {
      const float u = mf_u(P, P.g[base + c], P.mode == 0 ? cvr[c] : rvi, cvr[c], mr);
      const float sgn = u > 0.f ? 1.f : (u < 0.f ? -1.f : 0.f);
      P.p[base + c] = P.p[base + c] * keep - step * sgn * scale;
      // optimizerc.py:89-97 updates var_est in place, and for a vector var_est IS state["v"]: the
      // reference leaves the normalised update there, and the next step's EMA starts from it
      if (P.mode == 0) P.v[c] = u / div;
    }
  });
}

}  // namespace asrx

using namespace asrx;

extern "C" int asrx_maxfactor_param_bytes(void) { return (int)sizeof(MFParam); }

// table: device array of np MFParam (asrx/optim.py packs it); ws: float workspace of
// 4 np + 4 nrows + ncols + nmats floats; ncc = size of the (mat, col, row-chunk) space.
extern "C" int asrx_maxfactor_step(const void* table, int np, int64_t nrows, int64_t ncols, int64_t ncc,
                                   int64_t nmats, int64_t nitems, float* ws, hipStream_t stream) {
  ASRX_REQUIRE(np > 0, "asrx_maxfactor_step: no parameters");
  const MFParam* tab = reinterpret_cast<const MFParam*>(table);
  float* stats = ws;
  float* rowred = stats + 4 * (int64_t)np;
  float* row_a = rowred + nrows;  // sum p^2, then sum u^2 per row
  float* row_b = row_a + nrows;   // max |u| per row
  float* colacc = row_b + nrows;
  float* mrv = colacc + ncols;
  if (ncols > 0) (void)hipMemsetAsync(colacc, 0, sizeof(float) * ncols, stream);
  ASRX_REQUIRE(np <= MF_MAXP, "asrx_maxfactor_step: at most %d parameters per call", MF_MAXP);
  ASRX_REQUIRE(nitems > 0 && nitems <= nrows, "asrx_maxfactor_step: bad work-item count %ld", (long)nitems);
  const unsigned gr = (unsigned)std::min<int64_t>((nitems + 3) / 4, 4096);
  mf_rows_kernel<<<gr, 256, 0, stream>>>(tab, np, nitems, row_a);
  mf_param_reduce_kernel<<<np, 256, 0, stream>>>(tab, np, 0, row_a, nullptr, stats, mrv);
  if (ncc > 0) {
    mf_cols_kernel<<<(unsigned)((ncc + 255) / 256), 256, 0, stream>>>(tab, np, ncc, colacc);
    mf_colfin_kernel<<<(unsigned)((ncols + 255) / 256), 256, 0, stream>>>(tab, np, ncols, colacc);
  }
  mf_ustats_kernel<<<gr, 256, 0, stream>>>(tab, np, nitems, mrv, rowred, row_a, row_b);
  mf_param_reduce_kernel<<<np, 256, 0, stream>>>(tab, np, 1, row_a, row_b, stats, mrv);
  mf_apply_kernel<<<gr, 256, 0, stream>>>(tab, np, nitems, mrv, rowred, stats);
  ASRX_LAUNCHED("asrx_maxfactor_step");
}
