// Row-wise and elementwise kernels of the model's hot path (fp32 in HBM, one wave per row where a
// row reduction is needed, grid-stride elementwise otherwise).  Each kernel names the reference
// op(s) it replaces.
#include "common.h"
#include <algorithm>
#include <mutex>
#include <map>
#include <unordered_map>
#include <utility>

namespace asrx {

constexpr int RW = 4;  // waves per workgroup for row kernels

__device__ __forceinline__ int64_t row_begin() { return (int64_t)blockIdx.x * RW + (threadIdx.x >> 6); }
__device__ __forceinline__ int64_t row_step() { return (int64_t)gridDim.x * RW; }

static unsigned row_grid(int64_t rows, int64_t cap = 8192) {
  int64_t g = (rows + RW - 1) / RW;
  if (g > cap) g = cap;
  if (g < 1) g = 1;
  return (unsigned)g;
}
static unsigned ew_grid(int64_t n, int64_t cap = 16384) {
  int64_t g = (n + 255) / 256;
  if (g > cap) g = cap;
  if (g < 1) g = 1;
  return (unsigned)g;
}

// Workgroup reduction of per-wave partials `part[RW][n]` then atomicAdd into dst[n].
__device__ __forceinline__ void flush_partials(float* part, int n, float* dst) {
  __syncthreads();
  for (int j = threadIdx.x; j < n; j += 64 * RW) {
    float s = 0.f;
    for (int w = 0; w < RW; ++w) s += part[w * n + j];
    atomicAdd(dst + j, s);
  }
}

// ============================================================================ LayerNorm
// nn.LayerNorm over the last dim (MSheath layers[i].ln / mlp_ln, model.py:405, 427) and
// essentials.LayerNorm over channels (essentials.py:110-113) on channels-last activations.
// Register-resident variants for d = 64 E (E even): a lane owns E consecutive features (float2
// I/O), the row is read once, statistics by DPP wave sums, the next row is prefetched; the backward
// keeps its dw / db partials in registers.  The generic kernels below remain for other d.
// Row layout of the one-wave-per-row kernels (LayerNorm, MSheath row passes): lane l owns the E
// features 128 j + 2 l + {0, 1}, j < E / 2, so each float2 load / store instruction of the wave moves
// 512 contiguous bytes (fully coalesced).  Only reductions and per-feature maps run in this layout; every
// per-feature operand (x, w, b, gw, px, dx, the LDS partials) uses the same mapping.
template <int E>
__device__ __forceinline__ int lane_feat(int lane, int e) {
  static_assert(E % 2 == 0, "row kernels take E = D / 64 even");
  return 128 * (e >> 1) + 2 * lane + (e & 1);
}
template <int E>
__device__ __forceinline__ void ld_lane(const float* __restrict__ src, int lane, float (&v)[E]) {
  const float2* s2 = reinterpret_cast<const float2*>(src);
#pragma unroll
  for (int e = 0; e < E / 2; ++e) {
    const float2 t = s2[64 * e + lane];
    v[2 * e] = t.x;
    v[2 * e + 1] = t.y;
  }
}
template <int E>
__device__ __forceinline__ void st_lane(float* __restrict__ dst, int lane, const float (&v)[E]) {
  float2* d2 = reinterpret_cast<float2*>(dst);
#pragma unroll
  for (int e = 0; e < E / 2; ++e) d2[64 * e + lane] = make_float2(v[2 * e], v[2 * e + 1]);
}
template <int E>
__device__ __forceinline__ void st_lane(unsigned short* __restrict__ dst, int lane, const float (&v)[E]) {
  unsigned* d2 = reinterpret_cast<unsigned*>(dst);
#pragma unroll
  for (int e = 0; e < E / 2; ++e)
    d2[64 * e + lane] = (unsigned)__builtin_bit_cast(unsigned short, (__bf16)v[2 * e]) |
                        ((unsigned)__builtin_bit_cast(unsigned short, (__bf16)v[2 * e + 1]) << 16);
}

// Optional fused row outputs (MSheath, asrx/msheath.py): nrm[r] = |x_r|_2 (v_gate's normalisation of
// the same x, model.py:347) and gout[r] = sigmoid(y_r . gw + gb) (the Linear(D, 1) gate on the
// normalised row: layers[i].gate at model.py:460, mlp_gate at 503 on x itself when gate_on_x).
template <int E, typename TY = float>
__global__ __launch_bounds__(64 * RW) void ln_fwd_t_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                           const float* __restrict__ b, TY* __restrict__ y,
                                                           float* __restrict__ mean, float* __restrict__ rstd,
                                                           int64_t rows, float eps, float* __restrict__ nrm,
                                                           const float* __restrict__ gw, const float* __restrict__ gb,
                                                           float* __restrict__ gout, int gate_on_x) {
  constexpr int D = 64 * E;
  const int lane = threadIdx.x & 63;
  float wv[E], bv[E], xn[E], gwv[E];
  ld_lane<E>(w, lane, wv);
  ld_lane<E>(b, lane, bv);
  if (gw) ld_lane<E>(gw, lane, gwv);
  const float gbias = gw ? gb[0] : 0.f;
  int64_t r = row_begin();
  if (r < rows) ld_lane<E>(x + r * D, lane, xn);
  for (; r < rows; r += row_step()) {
    float xv[E];
    float s = 0.f;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      xv[e] = xn[e];
      s += xv[e];
    }
    if (r + row_step() < rows) ld_lane<E>(x + (r + row_step()) * D, lane, xn);
    const float mu = wave_sum_dpp(s) * (1.0f / D);
    float v = 0.f;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const float t = xv[e] - mu;
      v += t * t;
    }
    const float rs = rsqrtf(wave_sum_dpp(v) * (1.0f / D) + eps);
    float yv[E];
    // explicit fma: the fp32- and bf16-output instantiations must round identically (a contraction the
    // compiler chooses per instantiation would move some bf16 roundings by one ulp)
#pragma unroll
    for (int e = 0; e < E; ++e) yv[e] = __builtin_fmaf((xv[e] - mu) * rs, wv[e], bv[e]);
    st_lane<E>(y + r * D, lane, yv);
    if (nrm) {
      float q = 0.f;
#pragma unroll
      for (int e = 0; e < E; ++e) q += xv[e] * xv[e];
      q = wave_sum_dpp(q);
      if (lane == 0) nrm[r] = sqrtf(q);
    }
    if (gw) {
      float q = 0.f;
#pragma unroll
      for (int e = 0; e < E; ++e) q += (gate_on_x ? xv[e] : yv[e]) * gwv[e];
      q = wave_sum_dpp(q) + gbias;
      if (lane == 0) gout[r] = sigmoid_f(q);
    }
    if (lane == 0) {
      mean[r] = mu;
      rstd[r] = rs;
    }
  }
}

template <int E>
__global__ __launch_bounds__(64 * RW) void ln_bwd_t_kernel(const float* __restrict__ dy, const float* __restrict__ x,
                                                           const float* __restrict__ w, const float* __restrict__ mean,
                                                           const float* __restrict__ rstd, float* __restrict__ dx,
                                                           float* __restrict__ dw, float* __restrict__ db,
                                                           int64_t rows, int acc) {
  constexpr int D = 64 * E;
  __shared__ float part[RW][2 * D];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  float wv[E], aw[E], ab[E];
  ld_lane<E>(w, lane, wv);
#pragma unroll
  for (int e = 0; e < E; ++e) aw[e] = ab[e] = 0.f;
  for (int64_t r = row_begin(); r < rows; r += row_step()) {
    float xv[E], gv[E];
    ld_lane<E>(x + r * D, lane, xv);
    ld_lane<E>(dy + r * D, lane, gv);
    const float mu = mean[r], rs = rstd[r];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      xv[e] = (xv[e] - mu) * rs;  // x-hat
      const float g = gv[e] * wv[e];
      s1 += g;
      s2 += g * xv[e];
      aw[e] += gv[e] * xv[e];
      ab[e] += gv[e];
    }
    wave_sum2_dpp(s1, s2);
    s1 *= (1.0f / D);
    s2 *= (1.0f / D);
    float dv[E];
    if (acc) ld_lane<E>(dx + r * D, lane, dv);
#pragma unroll
    for (int e = 0; e < E; ++e) dv[e] = (acc ? dv[e] : 0.f) + rs * (gv[e] * wv[e] - s1 - xv[e] * s2);
    st_lane<E>(dx + r * D, lane, dv);
  }
#pragma unroll
  for (int e = 0; e < E; ++e) {
    part[wid][lane_feat<E>(lane, e)] = aw[e];
    part[wid][D + lane_feat<E>(lane, e)] = ab[e];
  }
  __syncthreads();
  for (int j = threadIdx.x; j < D; j += 64 * RW) {
    float a = 0.f, c = 0.f;
#pragma unroll
    for (int ww = 0; ww < RW; ++ww) {
      a += part[ww][j];
      c += part[ww][D + j];
    }
    atomicAdd(dw + j, a);
    atomicAdd(db + j, c);
  }
}

__global__ __launch_bounds__(64 * RW) void ln_fwd_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                         const float* __restrict__ b, float* __restrict__ y,
                                                         float* __restrict__ mean, float* __restrict__ rstd,
                                                         int64_t rows, int d, float eps) {
  const int lane = threadIdx.x & 63;
  for (int64_t r = row_begin(); r < rows; r += row_step()) {
    const float* xr = x + r * d;
    float s = 0.f;
    for (int j = lane; j < d; j += 64) s += xr[j];
    const float mu = wave_sum(s) / d;
    float v = 0.f;
    for (int j = lane; j < d; j += 64) {
      const float t = xr[j] - mu;
      v += t * t;
    }
    const float rs = rsqrtf(wave_sum(v) / d + eps);
    float* yr = y + r * d;
    for (int j = lane; j < d; j += 64) yr[j] = (xr[j] - mu) * rs * w[j] + b[j];
    if (lane == 0) {
      mean[r] = mu;
      rstd[r] = rs;
    }
  }
}

__global__ __launch_bounds__(64 * RW) void ln_bwd_kernel(const float* __restrict__ dy, const float* __restrict__ x,
                                                         const float* __restrict__ w, const float* __restrict__ mean,
                                                         const float* __restrict__ rstd, float* __restrict__ dx,
                                                         float* __restrict__ dw, float* __restrict__ db, int64_t rows,
                                                         int d, int acc) {
  extern __shared__ float part[];  // [RW][2*d]
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  float* pw = part + wid * 2 * d;
  for (int j = lane; j < 2 * d; j += 64) pw[j] = 0.f;
  for (int64_t r = row_begin(); r < rows; r += row_step()) {
    const float* xr = x + r * d;
    const float* gr = dy + r * d;
    const float mu = mean[r], rs = rstd[r];
    float s1 = 0.f, s2 = 0.f;
    for (int j = lane; j < d; j += 64) {
      const float xh = (xr[j] - mu) * rs;
      const float g = gr[j] * w[j];
      s1 += g;
      s2 += g * xh;
      pw[j] += gr[j] * xh;
      pw[d + j] += gr[j];
    }
    s1 = wave_sum(s1) / d;
    s2 = wave_sum(s2) / d;
    float* dxr = dx + r * d;
    for (int j = lane; j < d; j += 64) {
      const float xh = (xr[j] - mu) * rs;
      dxr[j] = (acc ? dxr[j] : 0.f) + rs * (gr[j] * w[j] - s1 - xh * s2);
    }
  }
  __syncthreads();
  for (int j = threadIdx.x; j < d; j += 64 * RW) {
    float a = 0.f, c = 0.f;
    for (int ww = 0; ww < RW; ++ww) {
      a += part[ww * 2 * d + j];
      c += part[ww * 2 * d + d + j];
    }
    atomicAdd(dw + j, a);
    atomicAdd(db + j, c);
  }
}

// ============================================================================ small-N linear
// y[r, n] = act(x[r] . W[n] + b[n]) for N <= 4 outputs: gate / mem_gate / mlp_gate Linear(D, 1)
// (model.py:398, 406, 420), v_gate.mlp[2] Linear(D/2, 1) and concat (model.py:341, 344),
// tgate.cs Linear(D, 3) (model.py:530), MPNet's Linear(128, 3) (model.py:381).
// x stored fp32 or bf16 (TX = unsigned short: tgate's input is a bf16-stored AbbyNormal output)
__device__ __forceinline__ float ldx(const float* p) { return *p; }
__device__ __forceinline__ float ldx(const unsigned short* p) { return __uint_as_float((unsigned)*p << 16); }

template <int NS, typename TX = float>
__global__ __launch_bounds__(64 * RW) void small_linear_fwd_kernel(const TX* __restrict__ x,
                                                                   const float* __restrict__ W,
                                                                   const float* __restrict__ b,
                                                                   float* __restrict__ y, int64_t rows, int K,
                                                                   int act) {
  const int lane = threadIdx.x & 63;
  for (int64_t r = row_begin(); r < rows; r += row_step()) {
    const TX* xr = x + r * K;
    float acc[NS];
#pragma unroll
    for (int n = 0; n < NS; ++n) acc[n] = 0.f;
    for (int k = lane; k < K; k += 64) {
      const float xv = ldx(xr + k);
#pragma unroll
      for (int n = 0; n < NS; ++n) acc[n] += xv * W[n * K + k];
    }
    if (act == ACT_SOFTMAX) {  // the row's softmax, in asrx_softmax_small's order of operations
      float v[NS], m = -INFINITY, s = 0.f;
#pragma unroll
      for (int n = 0; n < NS; ++n) {
        v[n] = wave_sum(acc[n]) + (b ? b[n] : 0.f);
        m = fmaxf(m, v[n]);
      }
#pragma unroll
      for (int n = 0; n < NS; ++n) s += expf(v[n] - m);
#pragma unroll
      for (int n = 0; n < NS; ++n)
        if (lane == n) y[r * NS + n] = expf(v[n] - m) / s;
      continue;
    }
#pragma unroll
    for (int n = 0; n < NS; ++n) {
      const float v = wave_sum(acc[n]) + (b ? b[n] : 0.f);
      if (lane == n) y[r * NS + n] = apply_act(act, v);
    }
  }
}

// dy is the gradient of the post-activation output; y the saved output (for sigmoid').
template <int NS, typename TX = float>
__global__ __launch_bounds__(64 * RW) void small_linear_bwd_kernel(
    const float* __restrict__ dy, const float* __restrict__ y, const TX* __restrict__ x,
    const float* __restrict__ W, float* __restrict__ dx, float* __restrict__ dW, float* __restrict__ db,
    int64_t rows, int K, int act, float beta, float* __restrict__ ws) {
  extern __shared__ float part[];  // [RW][NS*K + NS]
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int PN = NS * K + NS;
  float* pw = part + wid * PN;
  for (int j = lane; j < PN; j += 64) pw[j] = 0.f;
  for (int64_t r = row_begin(); r < rows; r += row_step()) {
    float dz[NS];
#pragma unroll
    for (int n = 0; n < NS; ++n) {
      float g = dy[r * NS + n];
      if (act == ACT_SIGMOID) {
        const float s = y[r * NS + n];
        g *= s * (1.f - s);
      }
      dz[n] = g;
    }
    const TX* xr = x + r * K;
    float* dxr = dx ? dx + r * K : nullptr;
    for (int k = lane; k < K; k += 64) {
      const float xv = ldx(xr + k);
      float s = 0.f;
#pragma unroll
      for (int n = 0; n < NS; ++n) {
        s += dz[n] * W[n * K + k];
        pw[n * K + k] += dz[n] * xv;
      }
      if (dxr) dxr[k] = (beta != 0.f ? beta * dxr[k] : 0.f) + s;
    }
    if (lane == 0) {
#pragma unroll
      for (int n = 0; n < NS; ++n) pw[NS * K + n] += dz[n];
    }
  }
  __syncthreads();
  // Deterministic parameter gradients: each workgroup writes its partial to ws[blockIdx.x] and
  // small_linear_colsum_kernel adds the partials in a fixed order into dW / db.  Float atomics summed them in
  // completion order, which made e.g. MSheath's mlp_gate bias gradient differ between two schedules of the
  // same step by more than the rerun spread the dead-block test measures.
  for (int j = threadIdx.x; j < PN; j += 64 * RW) {
    float s = 0.f;
    for (int ww = 0; ww < RW; ++ww) s += part[ww * PN + j];
    ws[(int64_t)blockIdx.x * PN + j] = s;
  }
}

// one wave per column j of the nb x PN partials: lane l sums rows l, l + 64, ... in order, then a fixed wave tree
__global__ __launch_bounds__(64) void small_linear_colsum_kernel(const float* __restrict__ ws, int nb, int PN, int NSK,
                                                                 float* __restrict__ dW, float* __restrict__ db) {
  const int j = blockIdx.x, lane = threadIdx.x;
  float s = 0.f;
  for (int bb = lane; bb < nb; bb += 64) s += ws[(int64_t)bb * PN + j];
  s = wave_sum(s);
  if (lane == 0) {
    if (j < NSK) dW[j] += s;
    else if (db) db[j - NSK] += s;
  }
}

// ============================================================================ row L2 norm
// torch.norm(xa, dim=-1) of rotary (model.py:201) and F.normalize in v_gate (model.py:347).
__global__ __launch_bounds__(64 * RW) void rownorm_kernel(const float* __restrict__ x, float* __restrict__ n,
                                                          int64_t rows, int d) {
  const int lane = threadIdx.x & 63;
  for (int64_t r = row_begin(); r < rows; r += row_step()) {
    float s = 0.f;
    for (int j = lane; j < d; j += 64) s += x[r * d + j] * x[r * d + j];
    s = wave_sum_dpp(s);
    if (lane == 0) n[r] = sqrtf(s);
  }
}

// dx[r] += dn[r] * x[r] / n[r]
__global__ void rownorm_bwd_kernel(const float* __restrict__ dn, const float* __restrict__ x,
                                   const float* __restrict__ n, float* __restrict__ dx, int64_t rows, int d, int acc) {
  const int64_t total = rows * d;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / d;
    const float nn = n[r];
    const float v = nn > 0.f ? dn[r] * x[i] / nn : 0.f;
    dx[i] = acc ? dx[i] + v : v;
  }
}

// ============================================================================ rotary
// rotary.forward (model.py:198-214) fused with the hd^-0.25 pre-scale (model.py:303-304):
// x (B, L, H, hd) viewed as rows of D = H*hd per position; pairs (2j, 2j+1) are complex numbers
// multiplied by polar(m[b,l], fp32(l * f[j])) and by `scale`.
// (cos, sin) of (float)l * f[j] for every position l < L and pair j < hd / 2: the angles depend only on
// (l, j), so the B samples and H heads of a rotary pass share them -- read from this table (L2-resident,
// L * hd * 4 bytes) instead of B * H sincosf calls each (the large-argument sincosf dominated the rotary
// kernels' instruction count).  Same sincosf, same arguments: bit-identical to the direct form.
__global__ void rotary_table_kernel(const float* __restrict__ f, float2* __restrict__ tab, int64_t L, int half) {
  const int64_t n = L * half;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float l = (float)(i / half);
    float sn, cs;
    sincosf(l * f[i % half], &sn, &cs);
    tab[i] = make_float2(cs, sn);
  }
}

__device__ __forceinline__ void rot_cs(const float* __restrict__ f, const float2* __restrict__ tab, int64_t lpos,
                                       int j, int half, float& cs, float& sn) {
  if (tab) {
    const float2 t = tab[lpos * half + j];
    cs = t.x;
    sn = t.y;
  } else {
    sincosf((float)lpos * f[j], &sn, &cs);
  }
}

__global__ __launch_bounds__(64 * RW) void rotary_fwd_kernel(const float* __restrict__ x, const float* __restrict__ m,
                                                             const float* __restrict__ f,
                                                             const float2* __restrict__ tab, float* __restrict__ y,
                                                             int64_t BL, int64_t L, int D, int hd, float scale) {
  const int lane = threadIdx.x & 63;
  const int half = hd / 2;
  for (int64_t r = row_begin(); r < BL; r += row_step()) {
    const int64_t lpos = r % L;
    const float mm = m[r] * scale;
    const float2* xr = reinterpret_cast<const float2*>(x + r * D);
    float2* yr = reinterpret_cast<float2*>(y + r * D);
    // the row's pairs in groups of four per lane, every load of a group issued before any use (one pair
    // per loop trip exposed a full load latency per pair)
    for (int p0 = lane; p0 < D / 2; p0 += 256) {
      float2 v[4], t[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int p = p0 + 64 * u;
        const int pc = p < D / 2 ? p : p0;
        v[u] = xr[pc];
        float sn, cs;
        rot_cs(f, tab, lpos, pc % half, half, cs, sn);
        t[u] = make_float2(cs, sn);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int p = p0 + 64 * u;
        const float cs = t[u].x, sn = t[u].y;
        if (p < D / 2) yr[p] = make_float2(mm * (v[u].x * cs - v[u].y * sn), mm * (v[u].x * sn + v[u].y * cs));
      }
    }
  }
}

// dx = scale*m*R(-ang) g ; dm[r] = sum over the row of g . (R(ang) x) * scale (i.e. g . y / m)
__global__ __launch_bounds__(64 * RW) void rotary_bwd_kernel(const float* __restrict__ g, const float* __restrict__ x,
                                                             const float* __restrict__ m, const float* __restrict__ f,
                                                             const float2* __restrict__ tab,
                                                             float* __restrict__ dx, float* __restrict__ dm,
                                                             int64_t BL, int64_t L, int D, int hd, float scale) {
  const int lane = threadIdx.x & 63;
  const int half = hd / 2;
  for (int64_t r = row_begin(); r < BL; r += row_step()) {
    const int64_t lpos = r % L;
    const float mm = m[r] * scale;
    const float2* xr = reinterpret_cast<const float2*>(x + r * D);
    const float2* gr = reinterpret_cast<const float2*>(g + r * D);
    float2* dxr = reinterpret_cast<float2*>(dx + r * D);
    float acc = 0.f;
    for (int p0 = lane; p0 < D / 2; p0 += 256) {  // groups of four pairs, loads first (rotary_fwd_kernel)
      float2 v[4], gg[4], t[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int p = p0 + 64 * u;
        const int pc = p < D / 2 ? p : p0;
        v[u] = xr[pc];
        gg[u] = gr[pc];
        float sn, cs;
        rot_cs(f, tab, lpos, pc % half, half, cs, sn);
        t[u] = make_float2(cs, sn);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int p = p0 + 64 * u;
        if (p >= D / 2) continue;
        const float cs = t[u].x, sn = t[u].y;
        dxr[p] = make_float2(mm * (gg[u].x * cs + gg[u].y * sn), mm * (-gg[u].x * sn + gg[u].y * cs));
        acc += gg[u].x * (v[u].x * cs - v[u].y * sn) + gg[u].y * (v[u].x * sn + v[u].y * cs);
      }
    }
    acc = wave_sum(acc) * scale;
    if (lane == 0) dm[r] = acc;  // written (one wave owns a row): no zero-filled dm needed
  }
}

// ============================================================================ v_gate
// model.py:346-351: key = softmax(normalize(x) . mkey_n^T / sqrt(D)); x_val = concat([key . mval,
// mlp(x)]); ion = x_val > tx (STE).  S = x . mkey_n^T (rows x M) and h = mlp[0](x) pre-activation
// (rows x D/2) come from GEMMs; nx = ||x||.
__global__ __launch_bounds__(64 * RW) void vgate_fwd_kernel(
    const float* __restrict__ S, const float* __restrict__ nx, const float* __restrict__ mval,
    const float* __restrict__ h, const float* __restrict__ w2, const float* __restrict__ b2,
    const float* __restrict__ cw, const float* __restrict__ cb, const float* __restrict__ tx,
    float* __restrict__ ion, float* __restrict__ xval, float* __restrict__ kv_out, float* __restrict__ m2_out,
    int64_t rows, int M, int Dh, float inv_sqrt_d) {
  const int lane = threadIdx.x & 63;
  for (int64_t r = row_begin(); r < rows; r += row_step()) {
    const float inx = 1.0f / fmaxf(nx[r], 1e-12f);
    // softmax over M (<= 64) logits, one per lane
    const float z = lane < M ? S[r * M + lane] * inx * inv_sqrt_d : -INFINITY;
    const float zm = wave_max(z);
    const float e = lane < M ? expf(z - zm) : 0.f;
    const float se = wave_sum(e);
    const float kv = wave_sum(lane < M ? e / se * mval[lane] : 0.f);
    float acc = 0.f;
    for (int j = lane; j < Dh; j += 64) acc += silu_f(h[r * Dh + j]) * w2[j];
    const float m2 = wave_sum(acc) + b2[0];
    const float xv = cw[0] * kv + cw[1] * m2 + cb[0];
    if (lane == 0) {
      xval[r] = xv;
      ion[r] = xv > tx[0] ? 1.f : 0.f;
      kv_out[r] = kv;
      m2_out[r] = m2;
    }
  }
}

// dion: gradient of ion (= of x_val through the STE).  Writes dS (rows x M, already divided by
// nx*sqrt(D): the gradient w.r.t. normalize(x) . mkey_n^T before the scale, i.e. dS_raw), dnx[r]
// (gradient of ||x|| through the normalisation), dh (rows x Dh) and accumulates dmval[M],
// dw2[Dh], db2, dcw[2], dcb.
__global__ __launch_bounds__(64 * RW) void vgate_bwd_kernel(
    const float* __restrict__ dion, const float* __restrict__ S, const float* __restrict__ nx,
    const float* __restrict__ mval, const float* __restrict__ h, const float* __restrict__ w2,
    const float* __restrict__ cw, const float* __restrict__ kvv, const float* __restrict__ m2v,
    float* __restrict__ dS, float* __restrict__ dnx, float* __restrict__ dh, float* __restrict__ dmval,
    float* __restrict__ dw2, float* __restrict__ db2, float* __restrict__ dcw, float* __restrict__ dcb,
    int64_t rows, int M, int Dh, float inv_sqrt_d) {
  extern __shared__ float part[];  // [RW][M + Dh + 4]
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int PN = M + Dh + 4;
  float* pw = part + wid * PN;
  for (int j = lane; j < PN; j += 64) pw[j] = 0.f;
  for (int64_t r = row_begin(); r < rows; r += row_step()) {
    const float g = dion[r];
    const float nxr = fmaxf(nx[r], 1e-12f);
    const float inx = 1.0f / nxr;
    const float z = lane < M ? S[r * M + lane] * inx * inv_sqrt_d : -INFINITY;
    const float zm = wave_max(z);
    const float e = lane < M ? expf(z - zm) : 0.f;
    const float key = e / wave_sum(e);
    const float dkv = g * cw[0];
    const float dm2 = g * cw[1];
    const float dkey = lane < M ? dkv * mval[lane] : 0.f;
    const float dot = wave_sum(key * dkey);
    const float dz = lane < M ? key * (dkey - dot) : 0.f;
    // z = S * inx * c  ->  dS = dz * inx * c ; d(inx) = sum dz * S * c
    if (lane < M) {
      dS[r * M + lane] = dz * inx * inv_sqrt_d;
      pw[lane] += dkv * key;
    }
    const float dinx = wave_sum(lane < M ? dz * S[r * M + lane] * inv_sqrt_d : 0.f);
    if (lane == 0) {
      // inx = 1/max(nx, eps): d nx = -dinx / nx^2 (zero when clamped)
      dnx[r] = nx[r] > 1e-12f ? -dinx * inx * inx : 0.f;
      pw[M + Dh + 0] += dm2;            // db2
      pw[M + Dh + 1] += g * kvv[r];     // dcw0
      pw[M + Dh + 2] += g * m2v[r];     // dcw1
      pw[M + Dh + 3] += g;              // dcb
    }
    for (int j = lane; j < Dh; j += 64) {
      const float hv = h[r * Dh + j];
      dh[r * Dh + j] = dm2 * w2[j] * silu_grad(hv);
      pw[M + j] += dm2 * silu_f(hv);
    }
  }
  __syncthreads();
  for (int j = threadIdx.x; j < PN; j += 64 * RW) {
    float s = 0.f;
    for (int ww = 0; ww < RW; ++ww) s += part[ww * PN + j];
    if (j < M) atomicAdd(dmval + j, s);
    else if (j < M + Dh) atomicAdd(dw2 + (j - M), s);
    else if (j == M + Dh) atomicAdd(db2, s);
    else if (j == M + Dh + 1) atomicAdd(dcw, s);
    else if (j == M + Dh + 2) atomicAdd(dcw + 1, s);
    else atomicAdd(dcb, s);
  }
}

// ============================================================================ MSheath layer rows
// One MSheath layer (model.py:452-461) touches each row of its input x in several per-row ops: v_gate
// (normalize(x), two projections, softmax, STE), the LayerNorm, the Linear(D, 1) gate on its output.
// The fused path (asrx/msheath.py) runs v_gate's two projections as ONE GEMM against
//   Wc = [normalize(mkey); mlp[0].weight]  ((M + Dh) x D),  bc = [0; mlp[0].bias],
// whose output SH = [x mkey_n^T | mlp[0](x)] has row stride ldsh = M + Dh, and every per-row op in
// one row pass forward (msheath_row_fwd) and one backward (msheath_row_bwd).

// Wc / bc from mkey and mlp[0]; mkn = max(|mkey_j|, 1e-12) (row_normalize's norm, for the backward);
// wb = bf16 Wc when non-null (asrx_weight_to_bf16's rounding), the wide GEMM's weight operand.
__global__ __launch_bounds__(64 * RW) void vgate_weights_kernel(const float* __restrict__ mkey,
                                                                const float* __restrict__ W1,
                                                                const float* __restrict__ b1, float* __restrict__ Wc,
                                                                float* __restrict__ bc, float* __restrict__ mkn,
                                                                unsigned short* __restrict__ wb, int M, int Dh, int D) {
  const int lane = threadIdx.x & 63;
  for (int64_t r = row_begin(); r < M + Dh; r += row_step()) {
    const bool key = r < M;
    const float* src = key ? mkey + r * D : W1 + (r - M) * D;
    float nn = 1.f;
    if (key) {
      float s = 0.f;
      for (int j = lane; j < D; j += 64) s += src[j] * src[j];
      nn = fmaxf(sqrtf(wave_sum(s)), 1e-12f);
    }
    for (int j = lane; j < D; j += 64) {
      const float v = key ? src[j] / nn : src[j];
      Wc[r * D + j] = v;
      if (wb) wb[r * D + j] = __builtin_bit_cast(unsigned short, (__bf16)v);
    }
    if (lane == 0) {
      if (key) mkn[r] = nn;
      bc[r] = key ? 0.f : b1[r - M];
    }
  }
}

struct MSRowFwd {
  const float *x, *lnw, *lnb, *gw, *gb;                   // layer input, ln, gate Linear(D, 1)
  const float *SH, *mval, *w2, *b2, *cw, *cb, *tx;         // v_gate
  float *px, *mean, *rstd, *nx, *g, *ion, *kv, *m2;
  int64_t rows, ldsh;
  int M, Dh;
  float eps, inv_sqrt_d;
  const float* next_i;  // rows of samples b with next_i[b] != layer are not at this layer (null: all are)
  int layer;
  int64_t L;
  unsigned short* pxb;  // non-null: px stored bf16 here instead (it only feeds the adapter GEMM)
  // non-null (a layer without adapter, whose update is px itself): x_new = x + g ion px (model.py:461) is formed
  // per row and its per-sample column sums over 64-row chunks go to part[b][chunk][:] -- the work of
  // axpy_row2_colsum (msheath.hip) in this pass; each wave then owns whole chunks (rows in order), and xnew (when
  // non-null) receives x_new
  float* part;
  float* xnew;
  int nchunk;
  // rows of samples not at this layer are left unwritten instead of zeroed (no-grad composite forward only:
  // nothing there reads them -- no backward, the row-list GEMMs' outputs of such rows are never consumed, the
  // column sums and the jump skip such samples)
  int nofill;
};

// Per row: px = LayerNorm(x); nx = |x|; g = sigmoid(px . gw + gb); v_gate from SH and nx (as
// vgate_fwd_kernel): ion = STE(cw0 softmax(S / (nx sqrt D)) . mval + cw1 (silu(h) . w2 + b2) + cb > tx).
template <int E>
__global__ __launch_bounds__(64 * RW) void msheath_row_fwd_kernel(MSRowFwd p) {
  constexpr int D = 64 * E;
  const int lane = threadIdx.x & 63;
  float wv[E], bv[E], gwv[E];
  ld_lane<E>(p.lnw, lane, wv);
  ld_lane<E>(p.lnb, lane, bv);
  ld_lane<E>(p.gw, lane, gwv);
  const float gbias = p.gb[0];
  const float mv_l = lane < p.M ? p.mval[lane] : 0.f;
  const float b2 = p.b2[0], cw0 = p.cw[0], cw1 = p.cw[1], cb = p.cb[0], tx = p.tx[0];
  // Which samples are at this layer: next_i is copied into LDS (dynamic, one float per sample) before
  // the loop, so the test is an LDS read, not a global load inside the loop whose wait (vmcnt counts in
  // order) would drain the prefetch queue.  32-bit sample index (rows < 2^31): a 64-bit division by the
  // runtime L cost ~3x the instructions.
  extern __shared__ float ni_s[];
  if (p.next_i) {
    const int nb = (int)((p.rows + p.L - 1) / p.L);
    for (int b = threadIdx.x; b < nb; b += 64 * RW) ni_s[b] = p.next_i[b];
    __syncthreads();
  }
  auto at_layer = [&](int64_t rr) __attribute__((always_inline)) -> bool {
    return !p.next_i || ni_s[(unsigned)rr / (unsigned)p.L] == (float)p.layer;
  };
  constexpr int HQ = (E + 1) / 2;  // h values per lane (Dh = D / 2 <= 64 HQ)
  float w2v[HQ];
#pragma unroll
  for (int i = 0; i < HQ; ++i) w2v[i] = lane + 64 * i < p.Dh ? p.w2[lane + 64 * i] : 0.f;
  float csum[E];  // chunk mode (p.part): this wave's column sums of x_new over its current chunk
  // The rows two strides ahead -- x AND the v_gate projections (S[lane], h) -- are in flight in two
  // named register sets used alternately (see abby_fwd_kernel: rotating one set into the other made the
  // compiler wait for the newest loads every row).  Loads are unconditional: past the end, or for a
  // sample not at this layer, they re-read row 0 (L2-resident) instead of skipping -- a branch around
  // them would make the compiler wait for them at the join.
  auto fetch = [&](int64_t rr, float (&xs)[E], float& ss, float (&hs)[HQ]) __attribute__((always_inline)) {
    const int64_t rc = (rr < p.rows && at_layer(rr)) ? rr : 0;
    ld_lane<E>(p.x + rc * D, lane, xs);
    const float* S = p.SH + rc * p.ldsh;
    ss = S[lane < p.M ? lane : 0];
#pragma unroll
    for (int i = 0; i < HQ; ++i) hs[i] = S[p.M + min(lane + 64 * i, p.Dh - 1)];
  };
  auto row_body = [&](int64_t r, const float (&xv)[E], float sv, const float (&hv)[HQ]) __attribute__((always_inline)) {
    if (!at_layer(r)) {  // sample not at this layer: no reads; zeros keep every later consumer finite
      if (p.nofill) return;
      float z[E];
#pragma unroll
      for (int e = 0; e < E; ++e) z[e] = 0.f;
      if (p.pxb) st_lane<E>(p.pxb + r * D, lane, z);
      else st_lane<E>(p.px + r * D, lane, z);
      if (lane == 0) {
        p.mean[r] = 0.f;
        p.rstd[r] = 0.f;
        p.nx[r] = 0.f;
        p.g[r] = 0.f;
        p.ion[r] = 0.f;
        p.kv[r] = 0.f;
        p.m2[r] = 0.f;
      }
      return;
    }
    // Eight wave reductions in four dependent levels (the values and their arithmetic are the one-at-a-time
    // order's; independent chains share a level so their DPP / permlane latencies overlap):
    // (sum x, sum x^2, SiLU(h) . w2) -> (variance, max of the key scores) -> (gate dot, sum exp) -> key mix
    float s = 0.f, q = 0.f;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      s += xv[e];
      q += xv[e] * xv[e];
    }
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < HQ; ++i)
      if (lane + 64 * i < p.Dh) acc += silu_f(hv[i]) * w2v[i];
    wave_sum3_dpp(s, q, acc);
    const float mu = s * (1.0f / D);
    const float nrm = sqrtf(q);
    const float m2 = acc + b2;
    float v = 0.f;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const float t = xv[e] - mu;
      v += t * t;
    }
    // v_gate's key scores
    const float inx = 1.0f / fmaxf(nrm, 1e-12f);
    const float z = lane < p.M ? sv * inx * p.inv_sqrt_d : -INFINITY;
    float zm = z;
    wave_sum_max_dpp(v, zm);
    const float rs = rsqrtf(v * (1.0f / D) + p.eps);
    float yv[E], gd = 0.f;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      yv[e] = __builtin_fmaf((xv[e] - mu) * rs, wv[e], bv[e]);  // explicit: as ln_fwd_t_kernel
      gd += yv[e] * gwv[e];
    }
    if (p.pxb) st_lane<E>(p.pxb + r * D, lane, yv);
    else st_lane<E>(p.px + r * D, lane, yv);
    const float ez = lane < p.M ? expf(z - zm) : 0.f;
    float se = ez;
    wave_sum2_dpp(gd, se);
    const float gate = sigmoid_f(gd + gbias);
    const float kv = wave_sum_dpp(lane < p.M ? ez / se * mv_l : 0.f);
    const float xval = cw0 * kv + cw1 * m2 + cb;
    if (p.part) {  // x_new = x + (g ion) px, as axpy_row2_colsum forms it; column sums in row order
      const float sc = gate * (xval > tx ? 1.f : 0.f);
      float xn[E];
#pragma unroll
      for (int e = 0; e < E; ++e) {
        xn[e] = __builtin_fmaf(sc, yv[e], xv[e]);
        csum[e] += xn[e];
      }
      if (p.xnew) st_lane<E>(p.xnew + r * D, lane, xn);
    }
    if (lane == 0) {
      p.mean[r] = mu;
      p.rstd[r] = rs;
      p.nx[r] = nrm;
      p.g[r] = gate;
      p.ion[r] = xval > tx ? 1.f : 0.f;
      p.kv[r] = kv;
      p.m2[r] = m2;
    }
  };
  if (p.part) {
    // one workgroup per 64-row chunk of one sample (chunks never straddle samples): wave w takes the chunk's
    // rows w, w + RW, ... in order with the next row's loads in flight, and the RW waves' column sums are added
    // in wave order through LDS (deterministic)
    // RW x D floats after the next_i copy, 16-byte aligned (the float2 lane accesses need 8)
    float* red = ni_s + (p.next_i ? (((p.rows + p.L - 1) / p.L + 3) & ~(int64_t)3) : 0);
    const int w = threadIdx.x >> 6;
    const int64_t nb = (p.rows + p.L - 1) / p.L, nc = (int64_t)nb * p.nchunk;
    for (int64_t cid = blockIdx.x; cid < nc; cid += gridDim.x) {
      const int64_t b = cid / p.nchunk, c = cid - b * p.nchunk;
      const int64_t r0 = b * p.L + c * 64, r1 = min(min(r0 + 64, (b + 1) * p.L), p.rows);
#pragma unroll
      for (int e = 0; e < E; ++e) csum[e] = 0.f;
      const bool act = r0 < r1 && at_layer(r0);  // workgroup-uniform
      if (act) {
        float xa[E], sa, ha[HQ];
        fetch(r0 + w, xa, sa, ha);
        for (int64_t r = r0 + w; r < r1; r += RW) {
          float xv[E], hv[HQ];
#pragma unroll
          for (int e = 0; e < E; ++e) xv[e] = xa[e];
#pragma unroll
          for (int i = 0; i < HQ; ++i) hv[i] = ha[i];
          const float sv = sa;
          fetch(r + RW < r1 ? r + RW : r0, xa, sa, ha);
          row_body(r, xv, sv, hv);
        }
      } else {
        float xv[E], hv[HQ];
        for (int64_t r = r0 + w; r < r1; r += RW) row_body(r, xv, 0.f, hv);  // not at this layer: zero rows
      }
      if (act) {
        st_lane<E>(red + w * D, lane, csum);
        __syncthreads();
        if (w == 0) {
          for (int k = 1; k < RW; ++k) {
            float t[E];
            ld_lane<E>(red + k * D, lane, t);
#pragma unroll
            for (int e = 0; e < E; ++e) csum[e] += t[e];
          }
        }
        __syncthreads();  // red is rewritten by the next chunk
      }
      if (w == 0) st_lane<E>(p.part + cid * D, lane, csum);  // (b, chunk) row; zeros for a sample not at the layer
    }
    return;
  }
  const int64_t st = row_step();
  int64_t r = row_begin();
  float xa[E], xb[E], sa, sb, ha[HQ], hb[HQ];
  fetch(r, xa, sa, ha);
  fetch(r + st, xb, sb, hb);
  for (; r < p.rows; r += 2 * st) {
    {
      float xv[E], hv[HQ];
#pragma unroll
      for (int e = 0; e < E; ++e) xv[e] = xa[e];
#pragma unroll
      for (int i = 0; i < HQ; ++i) hv[i] = ha[i];
      const float sv = sa;
      fetch(r + 2 * st, xa, sa, ha);
      row_body(r, xv, sv, hv);
    }
    if (r + st >= p.rows) break;
    {
      float xv[E], hv[HQ];
#pragma unroll
      for (int e = 0; e < E; ++e) xv[e] = xb[e];
#pragma unroll
      for (int i = 0; i < HQ; ++i) hv[i] = hb[i];
      const float sv = sb;
      fetch(r + 3 * st, xb, sb, hb);
      row_body(r + st, xv, sv, hv);
    }
  }
}

struct MSRowBwd {
  const float *dpx;                                        // gradient of the LayerNorm output (adapter path)
  const float *x, *lnw, *lnb, *mean, *rstd;
  const float *dg, *g, *gw;                                // gate: gradient of its output, output, weight
  const float *dion, *SH, *nx, *mval, *w2, *cw, *kv, *m2;  // v_gate
  float *dx;                                               // accumulated
  float *dlnw, *dlnb, *dgw, *dgb;
  float *dSH, *dmval, *dw2, *db2, *dcw, *dcb, *db1;
  int64_t rows, ldsh;
  int M, Dh;
  float inv_sqrt_d;
  const float* next_i;  // as MSRowFwd: rows of samples not at this layer get dSH = 0 and nothing else
  int layer;
  int64_t L;
};

// Per row, the backward of msheath_row_fwd: v_gate (dSH row with stride ldsh: dS already divided by
// nx sqrt D, dh = dm2 w2 silu'(h)), the gate (dz = dg g (1 - g) onto px), the LayerNorm with the gate
// term in its output gradient, and |x|'s gradient, all accumulated into dx; parameter gradients
// (ln w/b, gate w/b, mval, mlp[2] w/b, concat w/b, mlp[0].bias) as workgroup partials + atomics.
// Dynamic LDS: RW * (3 D + M + 2 Dh + 5) floats.
template <int E>
__global__ __launch_bounds__(64 * RW) void msheath_row_bwd_kernel(MSRowBwd p) {
  constexpr int D = 64 * E;
  extern __shared__ float part[];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int M = p.M, Dh = p.Dh;
  const int PN = M + 2 * Dh + 5;  // dmval[M] dw2[Dh] db1[Dh] db2 dcw0 dcw1 dcb dgb
  float* pw = part + RW * 3 * D + wid * PN;
  for (int j = lane; j < PN; j += 64) pw[j] = 0.f;
  float wv[E], bv[E], gwv[E], aw[E], ab[E], ag[E];
  ld_lane<E>(p.lnw, lane, wv);
  ld_lane<E>(p.lnb, lane, bv);
  ld_lane<E>(p.gw, lane, gwv);
#pragma unroll
  for (int e = 0; e < E; ++e) aw[e] = ab[e] = ag[e] = 0.f;
  const float mv_l = lane < M ? p.mval[lane] : 0.f;
  const float cw0 = p.cw[0], cw1 = p.cw[1];
  // Every input of the rows two strides ahead (x, dpx, dx, the v_gate projections and the row scalars)
  // is in flight in two named register sets used alternately (abby_fwd_kernel: rotating one set into the
  // other made the compiler wait for the newest loads every row); loads are unconditional (past the end
  // or for a sample not at this layer they re-read row 0), and the at-layer test reads an LDS copy of
  // next_i (a global load inside the loop would drain the prefetch queue at its wait).
  constexpr int HQ = (E + 1) / 2;  // h values per lane (Dh <= 64 HQ)
  struct Pre {
    float x[E], gp[E], dx[E], h[HQ];
    float s, gi, nx, g, dg, mu, rs, kv, m2;
  };
  const int ni_off = RW * (3 * D + PN);  // next_i copy (one float per sample) after the partials
  if (p.next_i) {
    const int nb = (int)((p.rows + p.L - 1) / p.L);
    for (int b = threadIdx.x; b < nb; b += 64 * RW) part[ni_off + b] = p.next_i[b];
  }
  __syncthreads();
  // 32-bit sample index (rows < 2^31): a 64-bit division by the runtime L cost ~3x the instructions.
  // (indexed off the __shared__ array itself: through a captured float* the accesses lost their
  // address space and became global loads)
  auto at_layer = [&](int64_t rr) __attribute__((always_inline)) -> bool {
    return !p.next_i || part[ni_off + (int)((unsigned)rr / (unsigned)p.L)] == (float)p.layer;
  };
  float w2v[HQ];
#pragma unroll
  for (int i = 0; i < HQ; ++i) w2v[i] = lane + 64 * i < Dh ? p.w2[lane + 64 * i] : 0.f;
  auto fetch = [&](int64_t rr, Pre& q) __attribute__((always_inline)) {
    const int64_t rc = (rr < p.rows && at_layer(rr)) ? rr : 0;
    const float* S = p.SH + rc * p.ldsh;
    q.s = S[lane < M ? lane : 0];
#pragma unroll
    for (int i = 0; i < HQ; ++i) q.h[i] = S[M + min(lane + 64 * i, Dh - 1)];
    ld_lane<E>(p.x + rc * D, lane, q.x);
    ld_lane<E>(p.dpx + rc * D, lane, q.gp);
    ld_lane<E>(p.dx + rc * D, lane, q.dx);
    q.gi = p.dion[rc];
    q.nx = p.nx[rc];
    q.g = p.g[rc];
    q.dg = p.dg[rc];
    q.mu = p.mean[rc];
    q.rs = p.rstd[rc];
    q.kv = p.kv[rc];
    q.m2 = p.m2[rc];
  };
  const int64_t st = row_step();
  int64_t r0 = row_begin();
  Pre pa, pb;
  fetch(r0, pa);
  fetch(r0 + st, pb);
  auto row_body = [&](int64_t r, Pre& q) __attribute__((always_inline)) {
    const Pre c = q;
    fetch(r + 2 * st, q);
    if (!at_layer(r)) {
      float* dz = p.dSH + r * p.ldsh;  // zero rows: the weight-gradient GEMMs sum over every row
      for (int j = lane; j < M + Dh; j += 64) dz[j] = 0.f;
      return;
    }
    // ---- v_gate backward (vgate_bwd_kernel)
    const float gi = c.gi;
    const float nxr = c.nx;
    const float inx = 1.0f / fmaxf(nxr, 1e-12f);
    float* dS = p.dSH + r * p.ldsh;
    float* dh = dS + M;
    const float sl = c.s;
    const float z = lane < M ? sl * inx * p.inv_sqrt_d : -INFINITY;
    const float zm = wave_max_dpp(z);
    const float ez = lane < M ? expf(z - zm) : 0.f;
    const float key = ez / wave_sum_dpp(ez);
    const float dkv = gi * cw0, dm2 = gi * cw1;
    const float dkey = lane < M ? dkv * mv_l : 0.f;
    const float dot = wave_sum_dpp(key * dkey);
    const float dz = lane < M ? key * (dkey - dot) : 0.f;
    if (lane < M) {
      dS[lane] = dz * inx * p.inv_sqrt_d;
      pw[lane] += dkv * key;
    }
    const float dinx = wave_sum_dpp(lane < M ? dz * sl * p.inv_sqrt_d : 0.f);
    const float dnx = nxr > 1e-12f ? -dinx * inx * inx : 0.f;
#pragma unroll
    for (int i = 0; i < HQ; ++i) {
      const int j = lane + 64 * i;
      if (j < Dh) {
        const float hv = c.h[i];
        const float t = dm2 * w2v[i] * silu_grad(hv);
        dh[j] = t;
        pw[M + j] += dm2 * silu_f(hv);
        pw[M + Dh + j] += t;
      }
    }
    // ---- gate + LayerNorm + |x| backward
    const float gg = c.g;
    const float dzg = c.dg * gg * (1.f - gg);
    if (lane == 0) {
      pw[M + 2 * Dh + 0] += dm2;
      pw[M + 2 * Dh + 1] += gi * c.kv;
      pw[M + 2 * Dh + 2] += gi * c.m2;
      pw[M + 2 * Dh + 3] += gi;
      pw[M + 2 * Dh + 4] += dzg;
    }
    float xv[E], gv[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
      xv[e] = c.x[e];
      gv[e] = c.gp[e];
    }
    const float mu = c.mu, rs = c.rs;
    const float cn = nxr > 0.f ? dnx / nxr : 0.f;
    float s1 = 0.f, s2 = 0.f, xh[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
      xh[e] = (xv[e] - mu) * rs;
      gv[e] += dzg * gwv[e];
      const float t = gv[e] * wv[e];
      s1 += t;
      s2 += t * xh[e];
      aw[e] += gv[e] * xh[e];
      ab[e] += gv[e];
      ag[e] += dzg * (xh[e] * wv[e] + bv[e]);
    }
    wave_sum2_dpp(s1, s2);
    s1 *= (1.0f / D);
    s2 *= (1.0f / D);
    float dv[E];
#pragma unroll
    for (int e = 0; e < E; ++e) dv[e] = c.dx[e] + rs * (gv[e] * wv[e] - s1 - xh[e] * s2) + cn * xv[e];
    st_lane<E>(p.dx + r * D, lane, dv);
  };
  for (int64_t r = r0; r < p.rows; r += 2 * st) {
    row_body(r, pa);
    if (r + st >= p.rows) break;
    row_body(r + st, pb);
  }
  float* pl = part + wid * 3 * D;
#pragma unroll
  for (int e = 0; e < E; ++e) {
    pl[lane_feat<E>(lane, e)] = aw[e];
    pl[D + lane_feat<E>(lane, e)] = ab[e];
    pl[2 * D + lane_feat<E>(lane, e)] = ag[e];
  }
  __syncthreads();
  for (int j = threadIdx.x; j < 3 * D; j += 64 * RW) {
    float a = 0.f;
#pragma unroll
    for (int ww = 0; ww < RW; ++ww) a += part[ww * 3 * D + j];
    atomicAdd(j < D ? p.dlnw + j : j < 2 * D ? p.dlnb + (j - D) : p.dgw + (j - 2 * D), a);
  }
  const float* pv = part + RW * 3 * D;
  for (int j = threadIdx.x; j < PN; j += 64 * RW) {
    float a = 0.f;
    for (int ww = 0; ww < RW; ++ww) a += pv[ww * PN + j];
    float* dst = j < M ? p.dmval + j
                 : j < M + Dh ? p.dw2 + (j - M)
                 : j < M + 2 * Dh ? p.db1 + (j - M - Dh)
                 : j == M + 2 * Dh ? p.db2
                 : j == M + 2 * Dh + 1 ? p.dcw
                 : j == M + 2 * Dh + 2 ? p.dcw + 1
                 : j == M + 2 * Dh + 3 ? p.dcb
                                       : p.dgb;
    atomicAdd(dst, a);
  }
}

// ============================================================================ tgate
// model.py:532-535 (num_types=3): out[d] = sum_k G[k*D + d] * softmax(c)[k], G = sigmoid(...)
template <typename TO = float>
__global__ __launch_bounds__(64 * RW) void tgate_fwd_kernel(const float* __restrict__ G, const float* __restrict__ c,
                                                            TO* __restrict__ out, int64_t rows, int D) {
  const int lane = threadIdx.x & 63;
  for (int64_t r = row_begin(); r < rows; r += row_step()) {
    const float c0 = c[r * 3], c1 = c[r * 3 + 1], c2 = c[r * 3 + 2];
    const float cm = fmaxf(c0, fmaxf(c1, c2));
    const float e0 = expf(c0 - cm), e1 = expf(c1 - cm), e2 = expf(c2 - cm);
    const float inv = 1.f / (e0 + e1 + e2);
    const float t0 = e0 * inv, t1 = e1 * inv, t2 = e2 * inv;
    const float* gr = G + r * 3 * D;
    for (int j = lane; j < D; j += 64) {
      // explicit fma chain: identical rounding in the fp32- and bf16-output instantiations
      const float v = __builtin_fmaf(gr[2 * D + j], t2, __builtin_fmaf(gr[D + j], t1, gr[j] * t0));
      if constexpr (sizeof(TO) == 4) out[r * D + j] = v;
      else out[r * D + j] = __builtin_bit_cast(unsigned short, (__bf16)v);
    }
  }
}

// dG = dout * t_k * G(1-G) (gradient of the pre-sigmoid GEMM output); dc = softmax backward.
__global__ __launch_bounds__(64 * RW) void tgate_bwd_kernel(const float* __restrict__ dout, const float* __restrict__ G,
                                                            const float* __restrict__ c, float* __restrict__ dGz,
                                                            float* __restrict__ dc, int64_t rows, int D) {
  const int lane = threadIdx.x & 63;
  for (int64_t r = row_begin(); r < rows; r += row_step()) {
    const float c0 = c[r * 3], c1 = c[r * 3 + 1], c2 = c[r * 3 + 2];
    const float cm = fmaxf(c0, fmaxf(c1, c2));
    const float e0 = expf(c0 - cm), e1 = expf(c1 - cm), e2 = expf(c2 - cm);
    const float inv = 1.f / (e0 + e1 + e2);
    const float t0 = e0 * inv, t1 = e1 * inv, t2 = e2 * inv;
    const float* gr = G + r * 3 * D;
    float* dg = dGz + r * 3 * D;
    float a0 = 0.f, a1 = 0.f, a2 = 0.f;
    for (int j = lane; j < D; j += 64) {
      const float go = dout[r * D + j];
      const float g0 = gr[j], g1 = gr[D + j], g2 = gr[2 * D + j];
      a0 += go * g0;
      a1 += go * g1;
      a2 += go * g2;
      dg[j] = go * t0 * g0 * (1.f - g0);
      dg[D + j] = go * t1 * g1 * (1.f - g1);
      dg[2 * D + j] = go * t2 * g2 * (1.f - g2);
    }
    wave_sum3_dpp(a0, a1, a2);
    const float dot = t0 * a0 + t1 * a1 + t2 * a2;
    if (lane == 0) {
      dc[r * 3] = t0 * (a0 - dot);
      dc[r * 3 + 1] = t1 * (a1 - dot);
      dc[r * 3 + 2] = t2 * (a2 - dot);
    }
  }
}

// ============================================================================ elementwise
// out = x + s[r] * y   (MSheath layer update x + g*(out*ion) with s = g*ion, model.py:461, and the
// final x + gate*output, model.py:505).  s may be null (s = 1).
__global__ void axpy_row_kernel(const float* __restrict__ x, const float* __restrict__ s, const float* __restrict__ y,
                                float* __restrict__ out, int64_t rows, int d) {
  const int64_t total = rows * d;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const float sc = s ? s[i / d] : 1.f;
    out[i] = x[i] + sc * y[i];
  }
}

// float4 form (d % 4 == 0, aligned, rows * d / 4 < 2^31): two vectors per thread and trip, loads first,
// 32-bit row index; the same x + s * y per element (bit-identical; this unit builds without contractions)
__global__ void axpy_row4_kernel(const float4* __restrict__ x, const float* __restrict__ s,
                                 const float4* __restrict__ y, float4* __restrict__ out, uint32_t n4, uint32_t d4) {
  const uint32_t st = gridDim.x * blockDim.x;
  auto one = [&](uint32_t i, float4 xv, float4 yv) __attribute__((always_inline)) {
    const float sc = s ? s[i / d4] : 1.f;
    out[i] = make_float4(xv.x + sc * yv.x, xv.y + sc * yv.y, xv.z + sc * yv.z, xv.w + sc * yv.w);
  };
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + st < n4; i += 2 * st) {
    const float4 x0 = x[i], x1 = x[i + st], y0 = y[i], y1 = y[i + st];
    one(i, x0, y0);
    one(i + st, x1, y1);
  }
  if (i < n4) one(i, x[i], y[i]);
}

// ds[r] = sum_j g[r,j] * y[r,j] ;  dy = s[r] * g  (dy may alias nothing)
// (dxc, when non-null, receives a copy of g: x's pass-through gradient as a buffer the caller owns)
__global__ __launch_bounds__(64 * RW) void axpy_row_bwd_kernel(const float* __restrict__ g, const float* __restrict__ s,
                                                               const float* __restrict__ y, float* __restrict__ dy,
                                                               float* __restrict__ ds, int64_t rows, int d,
                                                               float* __restrict__ dxc) {
  const int lane = threadIdx.x & 63;
  for (int64_t r = row_begin(); r < rows; r += row_step()) {
    const float sc = s[r];
    float acc = 0.f;
    for (int j = lane; j < d; j += 64) {
      const float gv = g[r * d + j];
      acc += gv * y[r * d + j];
      dy[r * d + j] = sc * gv;
      if (dxc) dxc[r * d + j] = gv;
    }
    acc = wave_sum_dpp(acc);
    if (lane == 0) ds[r] = acc;
  }
}

// MSheath jump / keep step (model.py:489-501) with per-sample masking (batch-1 semantics):
// out[b,l,:] = act[b] ? alpha[b]*xn + beta[b]*orig + gam[b,:] : xold
__global__ void jump_select_kernel(const float* __restrict__ xn, const float* __restrict__ orig,
                                   const float* __restrict__ xold, const float* __restrict__ act,
                                   const float* __restrict__ alpha, const float* __restrict__ beta,
                                   const float* __restrict__ gam, float* __restrict__ out, int64_t B, int64_t L,
                                   int d) {
  const int64_t total = B * L * d;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = i / (L * d);
    const int c = (int)(i % d);
    out[i] = act[b] != 0.f ? alpha[b] * xn[i] + beta[b] * orig[i] + gam[b * d + c] : xold[i];
  }
}

// Backward: per-sample reductions dalpha[b] = act*sum g*xn, dbeta[b] = act*sum g*orig,
// dgam[b,:] = act*sum_l g; elementwise dxn = act*alpha*g, dorig = act*beta*g, dxold = (1-act)*g.
// One workgroup per (sample, 256-column chunk)... implemented as: grid (ceil(d/64), B), 4 waves
// split L; column reductions through LDS.
__global__ __launch_bounds__(256) void jump_select_bwd_kernel(
    const float* __restrict__ g, const float* __restrict__ xn, const float* __restrict__ orig,
    const float* __restrict__ act, const float* __restrict__ alpha, const float* __restrict__ beta,
    float* __restrict__ dxn, float* __restrict__ dorig, float* __restrict__ dxold, float* __restrict__ dalpha,
    float* __restrict__ dbeta, float* __restrict__ dgam, int64_t L, int d) {
  __shared__ float red[3][4][64];
  const int b = blockIdx.y;
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int part = threadIdx.x >> 6;
  const float a = act[b], al = alpha[b], be = beta[b];
  float sa = 0.f, sb = 0.f, sg = 0.f;
  if (c < d) {
    for (int64_t l = part; l < L; l += 4) {
      const int64_t i = ((int64_t)b * L + l) * d + c;
      const float gv = g[i];
      if (a != 0.f) {
        sa += gv * xn[i];
        sb += gv * orig[i];
        sg += gv;
        dxn[i] = al * gv;
        dorig[i] = be * gv;
        dxold[i] = 0.f;
      } else {
        dxn[i] = 0.f;
        dorig[i] = 0.f;
        dxold[i] = gv;
      }
    }
  }
  red[0][part][threadIdx.x & 63] = sa;
  red[1][part][threadIdx.x & 63] = sb;
  red[2][part][threadIdx.x & 63] = sg;
  __syncthreads();
  if (part == 0 && c < d) {
    const int t = threadIdx.x;
    float A = 0.f, Bv = 0.f, G = 0.f;
    for (int p = 0; p < 4; ++p) {
      A += red[0][p][t];
      Bv += red[1][p][t];
      G += red[2][p][t];
    }
    dgam[(int64_t)b * d + c] = G;
    atomicAdd(dalpha + b, A);
    atomicAdd(dbeta + b, Bv);
  }
}

// Per-sample column sums: out[b, c] (+)= scale * sum_l x[b, l, c]  (x.mean(dim=1), model.py:435, 463).
// grid (ceil(d/64), B, chunks of L); each workgroup reduces a 64-column x chunk slab with float
// atomics into `out` (zeroed by the launcher unless accumulating).
__global__ __launch_bounds__(256) void seg_colsum_kernel(const float* __restrict__ x, float* __restrict__ out,
                                                         int64_t L, int d, float scale, int64_t chunk) {
  __shared__ float red[4][64];
  const int b = blockIdx.y;
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int part = threadIdx.x >> 6;
  const int64_t l0 = (int64_t)blockIdx.z * chunk, l1 = min(L, l0 + chunk);
  float s = 0.f;
  if (c < d)
    for (int64_t l = l0 + part; l < l1; l += 4) s += x[((int64_t)b * L + l) * d + c];
  red[part][threadIdx.x & 63] = s;
  __syncthreads();
  if (part == 0 && c < d) {
    const int t = threadIdx.x;
    atomicAdd(out + (int64_t)b * d + c, (red[0][t] + red[1][t] + red[2][t] + red[3][t]) * scale);
  }
}

// Deterministic form (forward values feeding hard decisions, model.py:432 MPNet pooling): chunk sums
// to part[b][chunk][:] with no atomics, then seg_reduce adds the chunks in order.
__global__ __launch_bounds__(256) void seg_partial_kernel(const float* __restrict__ x, float* __restrict__ part,
                                                          int64_t L, int d, int64_t chunk) {
  __shared__ float red[4][64];
  const int b = blockIdx.y;
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int p4 = threadIdx.x >> 6;
  const int64_t l0 = (int64_t)blockIdx.z * chunk, l1 = min(L, l0 + chunk);
  float s = 0.f;
  if (c < d)
    for (int64_t l = l0 + p4; l < l1; l += 4) s += x[((int64_t)b * L + l) * d + c];
  red[p4][threadIdx.x & 63] = s;
  __syncthreads();
  if (p4 == 0 && c < d) {
    const int t = threadIdx.x;
    part[((int64_t)b * gridDim.z + blockIdx.z) * d + c] = (red[0][t] + red[1][t]) + (red[2][t] + red[3][t]);
  }
}

__global__ void seg_reduce_kernel(const float* __restrict__ part, float* __restrict__ out, int B, int nchunk, int d,
                                  float scale) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)B * d) return;
  const int64_t b = i / d, c = i % d;
  float t = 0.f;
  for (int k = 0; k < nchunk; k += 16) {  // in chunk order, 16 loads in flight (the last group's clamped)
    float v[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) v[j] = part[(b * nchunk + min(k + j, nchunk - 1)) * d + c];
#pragma unroll
    for (int j = 0; j < 16; ++j)
      if (k + j < nchunk) t += v[j];
  }
  out[i] = t * scale;
}

// Column sums over many rows (bias gradients): out[c] += sum_r x[r, c].  grid (ceil(d/64), chunks).
__global__ __launch_bounds__(256) void colsum_kernel(const float* __restrict__ x, float* __restrict__ out,
                                                     int64_t rows, int d, int64_t chunk, int64_t ld) {
  __shared__ float red[4][64];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int part = threadIdx.x >> 6;
  const int64_t r0 = (int64_t)blockIdx.y * chunk;
  const int64_t r1 = min(rows, r0 + chunk);
  float s = 0.f, s2 = 0.f;
  if (c < d) {  // two independent chains, unrolled: keeps ~16 row loads in flight per wave
    int64_t r = r0 + part;
#pragma unroll 4
    for (; r + 4 < r1; r += 8) {
      s += x[r * ld + c];
      s2 += x[(r + 4) * ld + c];
    }
    if (r < r1) s += x[r * ld + c];
  }
  s += s2;
  red[part][threadIdx.x & 63] = s;
  __syncthreads();
  if (part == 0 && c < d) {
    const int t = threadIdx.x;
    atomicAdd(out + c, red[0][t] + red[1][t] + red[2][t] + red[3][t]);
  }
}

// out[b, l, :] = x[b, l, :] + t[l, :] (+ u[b, :]).  Sinusoid PE add (model.py:161, 580),
// position add (model.py:615) and the broadcast of per-sample vectors.
__global__ void add_rows_kernel(const float* __restrict__ x, const float* __restrict__ t, const float* __restrict__ u,
                                float* __restrict__ out, int64_t B, int64_t L, int d) {
  const int64_t total = B * L * d;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t c = i % d;
    const int64_t l = (i / d) % L;
    const int64_t b = i / (L * d);
    float v = x ? x[i] : 0.f;
    if (t) v += t[l * d + c];
    if (u) v += u[b * d + c];
    out[i] = v;
  }
}

// add_rows over float4 (d % 4 == 0, aligned): two float4 per thread and iteration, loads first; the same
// additions in the same order as add_rows_kernel (bit-identical).  32-bit indices (n / 4 < 2^31).
__global__ void add_rows4_kernel(const float4* __restrict__ x, const float4* __restrict__ t,
                                 const float4* __restrict__ u, float4* __restrict__ out, uint32_t n4, uint32_t L,
                                 uint32_t d4) {
  const uint32_t st = gridDim.x * blockDim.x;
  const float4 zero = make_float4(0.f, 0.f, 0.f, 0.f);
  auto one = [&](uint32_t i, float4 xv) __attribute__((always_inline)) {
    const uint32_t row = i / d4, c = i - row * d4;
    const uint32_t l = row % L, b = row / L;
    float4 v = xv;
    if (t) {
      const float4 tv = t[l * d4 + c];
      v.x += tv.x; v.y += tv.y; v.z += tv.z; v.w += tv.w;
    }
    if (u) {
      const float4 uv = u[b * d4 + c];
      v.x += uv.x; v.y += uv.y; v.z += uv.z; v.w += uv.w;
    }
    out[i] = v;
  };
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + st < n4; i += 2 * st) {
    const float4 x0 = x ? x[i] : zero, x1 = x ? x[i + st] : zero;
    one(i, x0);
    one(i + st, x1);
  }
  if (i < n4) one(i, x ? x[i] : zero);
}

// out = a*x + b*y (+ c*z): residual sums, e = a+b+c, blend (model.py:578-583, 624, 628)
__global__ void lincomb_kernel(const float* __restrict__ x, const float* __restrict__ y, const float* __restrict__ z,
                               float a, float b, float c, float* __restrict__ out, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    float v = a * x[i];
    if (y) v += b * y[i];
    if (z) v += c * z[i];
    out[i] = v;
  }
}

// float4 forms of lincomb / act_fwd / act_bwd (n % 4 == 0, 16-byte aligned, n / 4 < 2^32): two float4 per
// thread and iteration, every load issued before any use, 32-bit indices.  The scalar forms moved one float
// per thread per iteration behind a vmcnt(0) each (~3.9 TB/s); the per-element arithmetic is unchanged,
// so the results are bit-identical.
__global__ void lincomb4_kernel(const float4* __restrict__ x, const float4* __restrict__ y,
                                const float4* __restrict__ z, float a, float b, float c, float4* __restrict__ out,
                                uint32_t n4) {
  const uint32_t st = gridDim.x * blockDim.x;
  auto one = [&](float4 xv, float4 yv, float4 zv) __attribute__((always_inline)) {
    float4 v = make_float4(a * xv.x, a * xv.y, a * xv.z, a * xv.w);
    if (y) { v.x += b * yv.x; v.y += b * yv.y; v.z += b * yv.z; v.w += b * yv.w; }
    if (z) { v.x += c * zv.x; v.y += c * zv.y; v.z += c * zv.z; v.w += c * zv.w; }
    return v;
  };
  const float4 zero = make_float4(0.f, 0.f, 0.f, 0.f);
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + st < n4; i += 2 * st) {
    const float4 x0 = x[i], x1 = x[i + st];
    const float4 y0 = y ? y[i] : zero, y1 = y ? y[i + st] : zero;
    const float4 z0 = z ? z[i] : zero, z1 = z ? z[i + st] : zero;
    out[i] = one(x0, y0, z0);
    out[i + st] = one(x1, y1, z1);
  }
  if (i < n4) out[i] = one(x[i], y ? y[i] : zero, z ? z[i] : zero);
}
__global__ void act_fwd4_kernel(const float4* __restrict__ x, float4* __restrict__ y, uint32_t n4, int act) {
  const uint32_t st = gridDim.x * blockDim.x;
  auto one = [&](float4 v) __attribute__((always_inline)) {
    return make_float4(apply_act(act, v.x), apply_act(act, v.y), apply_act(act, v.z), apply_act(act, v.w));
  };
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + st < n4; i += 2 * st) {
    const float4 a0 = x[i], a1 = x[i + st];
    y[i] = one(a0);
    y[i + st] = one(a1);
  }
  if (i < n4) y[i] = one(x[i]);
}
__device__ __forceinline__ float act_deriv(int act, float v) {
  switch (act) {
    case ACT_GELU: return gelu_grad(v);
    case ACT_SILU: return silu_grad(v);
    case ACT_SIGMOID: {
      const float s = sigmoid_f(v);
      return s * (1.f - s);
    }
    default: return 1.f;
  }
}
__global__ void act_bwd4_kernel(const float4* __restrict__ g, const float4* __restrict__ x, float4* __restrict__ dx,
                                uint32_t n4, int act) {
  const uint32_t st = gridDim.x * blockDim.x;
  auto one = [&](float4 gv, float4 v) __attribute__((always_inline)) {
    return make_float4(gv.x * act_deriv(act, v.x), gv.y * act_deriv(act, v.y), gv.z * act_deriv(act, v.z),
                       gv.w * act_deriv(act, v.w));
  };
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + st < n4; i += 2 * st) {
    const float4 g0 = g[i], g1 = g[i + st], v0 = x[i], v1 = x[i + st];
    dx[i] = one(g0, v0);
    dx[i + st] = one(g1, v1);
  }
  if (i < n4) dx[i] = one(g[i], x[i]);
}

// activation forward / backward (GELU / SiLU / sigmoid, model.py:104, 143-147)
__global__ void act_fwd_kernel(const float* __restrict__ x, float* __restrict__ y, int64_t n, int act) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    y[i] = apply_act(act, x[i]);
}
__global__ void act_bwd_kernel(const float* __restrict__ g, const float* __restrict__ x, float* __restrict__ dx,
                               int64_t n, int act) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float v = x[i];
    float d;
    switch (act) {
      case ACT_GELU: d = gelu_grad(v); break;
      case ACT_SILU: d = silu_grad(v); break;
      case ACT_SIGMOID: {
        const float s = sigmoid_f(v);
        d = s * (1.f - s);
        break;
      }
      default: d = 1.f;
    }
    dx[i] = g[i] * d;
  }
}

// Backward of act(x W^T + b) below the GEMM, perf mode: gz = g * act'(z) stored bf16 (it only feeds the
// input- and weight-gradient GEMMs, which round it to bf16 anyway) and the bias gradient
// db += sum_rows gz (fp32, before rounding) in the same pass -- replaces act_bwd (fp32 gz) plus a
// separate colsum pass over it.  grid (ceil(N / 256), row chunks); lane -> 4 consecutive columns,
// the 4 waves of a workgroup take rows r0 + w, r0 + w + 4, ...; N % 4 == 0.
template <int ACT>
__global__ __launch_bounds__(256) void act_bwd_bias_kernel(const float* __restrict__ g, const float* __restrict__ z,
                                                           unsigned short* __restrict__ gz, float* __restrict__ db,
                                                           int64_t rows, int N, int64_t chunk) {
  __shared__ float4 red[4][64];
  const int lane = threadIdx.x & 63, part = threadIdx.x >> 6;
  const int c = 4 * (blockIdx.x * 64 + lane);
  const int64_t r0 = (int64_t)blockIdx.y * chunk, r1 = min(rows, r0 + chunk);
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  auto dact = [](float v) {
    if constexpr (ACT == ACT_GELU) return gelu_grad(v);
    else if constexpr (ACT == ACT_SILU) return silu_grad(v);
    else {
      const float sg = sigmoid_f(v);
      return sg * (1.f - sg);
    }
  };
  if (c < N) {
#pragma unroll 2
    for (int64_t r = r0 + part; r < r1; r += 4) {
      const float4 gv = *reinterpret_cast<const float4*>(g + r * N + c);
      const float4 zv = *reinterpret_cast<const float4*>(z + r * N + c);
      const float4 o = make_float4(gv.x * dact(zv.x), gv.y * dact(zv.y), gv.z * dact(zv.z), gv.w * dact(zv.w));
      acc.x += o.x; acc.y += o.y; acc.z += o.z; acc.w += o.w;
      typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
      const bf16x4 h = {(__bf16)o.x, (__bf16)o.y, (__bf16)o.z, (__bf16)o.w};
      *reinterpret_cast<bf16x4*>(gz + r * N + c) = h;
    }
  }
  red[part][lane] = acc;
  __syncthreads();
  if (part == 0 && c < N && db) {
    const float4 a = red[0][lane], b = red[1][lane], cc = red[2][lane], d = red[3][lane];
    atomicAdd(db + c + 0, a.x + b.x + cc.x + d.x);
    atomicAdd(db + c + 1, a.y + b.y + cc.y + d.y);
    atomicAdd(db + c + 2, a.z + b.z + cc.z + d.z);
    atomicAdd(db + c + 3, a.w + b.w + cc.w + d.w);
  }
}

// GLU over channels (nn.GLU(dim=1), model.py:97) on channels-last rows of 2C: out = a * sigmoid(b)
__global__ void glu_fwd_kernel(const float* __restrict__ x, float* __restrict__ y, int64_t rows, int C) {
  const int64_t total = rows * C;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / C, c = i % C;
    y[i] = x[r * 2 * C + c] * sigmoid_f(x[r * 2 * C + C + c]);
  }
}
__global__ void glu_bwd_kernel(const float* __restrict__ g, const float* __restrict__ x, float* __restrict__ dx,
                               int64_t rows, int C) {
  const int64_t total = rows * C;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / C, c = i % C;
    const float a = x[r * 2 * C + c], s = sigmoid_f(x[r * 2 * C + C + c]);
    dx[r * 2 * C + c] = g[i] * s;
    dx[r * 2 * C + C + c] = g[i] * a * s * (1.f - s);
  }
}

// nn.Dropout(0.1) in train mode (model.py:107, 147) with keyed masks on channels-last (B, T, C):
// keep iff noise_uniform(key, (sid*C + c)*8192 + t) >= p, scaled by 1/(1-p).  Same kernel for
// backward (the mask is recomputed).
__global__ void dropout_kernel(const float* __restrict__ x, float* __restrict__ y, int64_t B, int64_t T, int C,
                               int64_t sid_base, uint32_t key, float p) {
  const int64_t total = B * T * C;
  const float sc = 1.0f / (1.0f - p);
  key = noise_key(key);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t c = i % C;
    const int64_t t = (i / C) % T;
    const int64_t b = i / ((int64_t)T * C);
    const uint32_t idx = (uint32_t)(((sid_base + b) * C + c) * 8192 + t);
    y[i] = noise_uniform_k(key, idx) >= p ? x[i] * sc : 0.f;
  }
}

__device__ __forceinline__ float act_grad(int act, float v) {
  switch (act) {
    case ACT_GELU: return gelu_grad(v);
    case ACT_SILU: return silu_grad(v);
    case ACT_SIGMOID: {
      const float s = sigmoid_f(v);
      return s * (1.f - s);
    }
    default: return 1.f;
  }
}

// act + nn.Dropout fused (the encoder layer's trailing GELU -> Dropout(0.1), model.py:147; act
// NONE is plain dropout, ConvLite's model.py:107), float4 over channels with 32-bit index math:
//   fwd: y = act(z) * keep / (1 - p)        bwd: dz = g * keep / (1 - p) * act'(z)
// with the same keyed mask as dropout_kernel (identical products, so bit-identical to act then
// dropout).  Saves the intermediate act(z) round trip (one write + one read of the tensor) and the
// scalar kernel's 64-bit divisions.  Requires C % 4 == 0, 16-byte alignment and n / 4 < 2^32.
// act2 (applied after the dropout) is the NEXT encoder layer's leading GELU (model.py:143), fused in
// when the layer output has no other consumer; the backward recomputes act(z) for act2'.
// res (forward only, nullable) adds a residual after everything: ConvLite's `res + dropout(point2(.))`
// (model.py:107-118) in the same pass.
template <bool BWD>
__global__ void act_dropout4_kernel(const float4* __restrict__ g, const float4* __restrict__ z,
                                    const float4* __restrict__ res, float4* __restrict__ out, uint32_t n4,
                                    uint32_t C4, uint32_t T, uint32_t C, uint32_t sid_base, uint32_t key, float p,
                                    int act, int act2) {
  const float sc = 1.0f / (1.0f - p);
  key = noise_key(key);
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += gridDim.x * blockDim.x) {
    const uint32_t row = i / C4, c0 = (i - row * C4) * 4u;
    const uint32_t t = row % T, b = row / T;
    const uint32_t base = ((sid_base + b) * C + c0) * 8192u + t;
    const float4 v = z[i];
    float r[4] = {v.x, v.y, v.z, v.w};
    float gg[4] = {0.f, 0.f, 0.f, 0.f};
    if (BWD) {
      const float4 gv = g[i];
      gg[0] = gv.x; gg[1] = gv.y; gg[2] = gv.z; gg[3] = gv.w;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const bool keep = noise_uniform_k(key, base + (uint32_t)j * 8192u) >= p;
      if (BWD) {
        float gj = gg[j];
        if (act2 != ACT_NONE) gj = gj * act_grad(act2, keep ? apply_act(act, r[j]) * sc : 0.f);
        r[j] = (keep ? gj * sc : 0.f) * act_grad(act, r[j]);
      } else {
        const float y = keep ? apply_act(act, r[j]) * sc : 0.f;
        r[j] = act2 != ACT_NONE ? apply_act(act2, y) : y;
      }
    }
    if (!BWD && res) {
      const float4 rv = res[i];
      r[0] = rv.x + r[0]; r[1] = rv.y + r[1]; r[2] = rv.z + r[2]; r[3] = rv.w + r[3];
    }
    out[i] = make_float4(r[0], r[1], r[2], r[3]);
  }
}

// ============================================================================ depthwise conv
// groups=D Conv1d with kernel K, padding K/2 (ConvLite.depth k15, model.py:99-102; encoder k3,
// model.py:147) on channels-last (B, T, C).
__global__ void dwconv_fwd_kernel(const float* __restrict__ x, const float* __restrict__ w, const float* __restrict__ b,
                                  float* __restrict__ y, int64_t B, int64_t T, int C, int K) {
  const int64_t total = B * T * C;
  const int pad = K / 2;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t c = i % C;
    const int64_t t = (i / C) % T;
    const int64_t base = i - t * C;  // (b, 0, c)
    float s = b ? b[c] : 0.f;
    for (int k = 0; k < K; ++k) {
      const int64_t tt = t + k - pad;
      if (tt >= 0 && tt < T) s += w[c * K + k] * x[base + tt * C];
    }
    y[i] = s;
  }
}

__global__ void dwconv_bwd_data_kernel(const float* __restrict__ g, const float* __restrict__ w, float* __restrict__ dx,
                                       int64_t B, int64_t T, int C, int K) {
  const int64_t total = B * T * C;
  const int pad = K / 2;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t c = i % C;
    const int64_t t = (i / C) % T;
    const int64_t base = i - t * C;
    float s = 0.f;
    for (int k = 0; k < K; ++k) {
      const int64_t tt = t - k + pad;
      if (tt >= 0 && tt < T) s += w[c * K + k] * g[base + tt * C];
    }
    dx[i] = s;
  }
}

// dw[c, k] += sum_{b,t} g[b,t,c] x[b,t+k-pad,c] ; db[c] += sum g.  grid (ceil(C/64), B*chunks)
__global__ __launch_bounds__(256) void dwconv_bwd_w_kernel(const float* __restrict__ g, const float* __restrict__ x,
                                                           float* __restrict__ dw, float* __restrict__ db, int64_t B,
                                                           int64_t T, int C, int K, int64_t chunk) {
  __shared__ float red[4][64][17];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int part = threadIdx.x >> 6;
  const int64_t nch = (T + chunk - 1) / chunk;
  const int64_t b = blockIdx.y / nch;
  const int64_t t0 = (blockIdx.y % nch) * chunk;
  const int64_t t1 = min(T, t0 + chunk);
  const int pad = K / 2;
  float acc[16];
  float ab = 0.f;
#pragma unroll
  for (int k = 0; k < 16; ++k) acc[k] = 0.f;
  if (c < C) {
    for (int64_t t = t0 + part; t < t1; t += 4) {
      const float gv = g[(b * T + t) * C + c];
      ab += gv;
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        if (k < K) {
          const int64_t tt = t + k - pad;
          if (tt >= 0 && tt < T) acc[k] += gv * x[(b * T + tt) * C + c];
        }
      }
    }
  }
  const int tl = threadIdx.x & 63;
#pragma unroll
  for (int k = 0; k < 16; ++k) red[part][tl][k] = acc[k];
  red[part][tl][16] = ab;
  __syncthreads();
  if (part == 0 && c < C) {
    for (int k = 0; k < K; ++k) {
      const float s = red[0][tl][k] + red[1][tl][k] + red[2][tl][k] + red[3][tl][k];
      atomicAdd(dw + c * K + k, s);
    }
    if (db) atomicAdd(db + c, red[0][tl][16] + red[1][tl][16] + red[2][tl][16] + red[3][tl][16]);
  }
}

// Tiled depthwise conv for C % 4 == 0 (every call site of the model): one thread owns 4 channels
// (one float4 column) and R = 16 consecutive outputs; the R + K - 1 input rows stream through one
// register each and are scattered into the R accumulators with compile-time taps, so each input
// float4 is loaded once per tile and every x / y access is a coalesced 16-byte lane access.
// FLIP = 1 runs the transposed conv (backward data: dx[t] = sum_k w[k] g[t - k + P]).
constexpr int DW_R = 16;

template <int K, bool FLIP>
__global__ __launch_bounds__(256) void dwconv_tile_kernel(const float4* __restrict__ x, const float* __restrict__ w,
                                                          const float* __restrict__ b, float4* __restrict__ y,
                                                          int B, int T, int C4, int ntile) {
  constexpr int P = K / 2, W = DW_R + K - 1;
  const int64_t gid = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (gid >= (int64_t)B * ntile * C4) return;
  const int c4 = (int)(gid % C4);
  const int64_t rest = gid / C4;
  const int t0 = (int)(rest % ntile) * DW_R;
  const int64_t bb = rest / ntile;
  const float4* xs = x + bb * T * C4 + c4;
  float4 wk[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int kk = FLIP ? K - 1 - k : k;
    const float* wc = w + (int64_t)(4 * c4) * K + kk;
    wk[k] = make_float4(wc[0], wc[K], wc[2 * K], wc[3 * K]);
  }
  float4 bias = make_float4(0.f, 0.f, 0.f, 0.f);
  if (b) bias = *reinterpret_cast<const float4*>(b + 4 * c4);
  float4 acc[DW_R];
#pragma unroll
  for (int r = 0; r < DW_R; ++r) acc[r] = bias;
#pragma unroll
  for (int j = 0; j < W; ++j) {
    const int row = t0 - P + j;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (row >= 0 && row < T) v = xs[(int64_t)row * C4];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int r = j - k;
      if (r >= 0 && r < DW_R) {
        acc[r].x += wk[k].x * v.x;
        acc[r].y += wk[k].y * v.y;
        acc[r].z += wk[k].z * v.z;
        acc[r].w += wk[k].w * v.w;
      }
    }
  }
  float4* ys = y + bb * T * C4 + c4;
#pragma unroll
  for (int r = 0; r < DW_R; ++r)
    if (t0 + r < T) ys[(int64_t)(t0 + r) * C4] = acc[r];
}

// Weight/bias gradient: dw[c, k] += sum_{b,t} g[b,t,c] x[b,t+k-P,c], db[c] += sum g.  A workgroup
// owns 32 float4 columns (128 channels) x 8 row groups (two per wave: lanes 0-31 / 32-63) of
// DW_S tiles of R rows each; partials are combined lane l + l^32 by a shuffle, then across the 4
// waves in LDS, and the workgroup's 128 x (K + 1) sums -- a contiguous slice of the (C, K) weight
// -- leave as coalesced atomics.
constexpr int DW_S = 4;

template <int K>
__global__ __launch_bounds__(256) void dwconv_wgrad_kernel(const float4* __restrict__ g, const float4* __restrict__ x,
                                                           float* __restrict__ dw, float* __restrict__ db, int T,
                                                           int C4, int nchunk) {
  constexpr int P = K / 2, W = DW_R + K - 1;
  __shared__ float4 red[4][32][K + 1];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int cl = lane & 31, grp = wid * 2 + (lane >> 5);
  const int cchunks = (C4 + 31) / 32;
  const int cc = blockIdx.x % cchunks;
  const int chunk = (blockIdx.x / cchunks) % nchunk;
  const int64_t bb = blockIdx.x / ((int64_t)cchunks * nchunk);
  const int c4 = cc * 32 + cl;
  float4 acc[K + 1];
#pragma unroll
  for (int k = 0; k <= K; ++k) acc[k] = make_float4(0.f, 0.f, 0.f, 0.f);
  if (c4 < C4) {
    const float4* gs = g + bb * T * C4 + c4;
    const float4* xs = x + bb * T * C4 + c4;
    for (int s = 0; s < DW_S; ++s) {
      const int t0 = ((chunk * 8 + grp) * DW_S + s) * DW_R;
      if (t0 >= T) break;
      float4 gv[DW_R];
#pragma unroll
      for (int r = 0; r < DW_R; ++r) {
        gv[r] = (t0 + r < T) ? gs[(int64_t)(t0 + r) * C4] : make_float4(0.f, 0.f, 0.f, 0.f);
        acc[K].x += gv[r].x; acc[K].y += gv[r].y; acc[K].z += gv[r].z; acc[K].w += gv[r].w;
      }
#pragma unroll
      for (int j = 0; j < W; ++j) {
        const int row = t0 - P + j;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (row >= 0 && row < T) v = xs[(int64_t)row * C4];
#pragma unroll
        for (int k = 0; k < K; ++k) {
          const int r = j - k;
          if (r >= 0 && r < DW_R) {
            acc[k].x += gv[r].x * v.x;
            acc[k].y += gv[r].y * v.y;
            acc[k].z += gv[r].z * v.z;
            acc[k].w += gv[r].w * v.w;
          }
        }
      }
    }
  }
#pragma unroll
  for (int k = 0; k <= K; ++k) {
    acc[k].x += __shfl_xor(acc[k].x, 32);
    acc[k].y += __shfl_xor(acc[k].y, 32);
    acc[k].z += __shfl_xor(acc[k].z, 32);
    acc[k].w += __shfl_xor(acc[k].w, 32);
    if (lane < 32) red[wid][cl][k] = acc[k];
  }
  __syncthreads();
  // the workgroup's slice: channels [128 cc, 128 cc + 128) x taps, contiguous in dw
  const int c_base = cc * 128;
  const int nch = min(128, 4 * C4 - c_base);
  const float* rf = reinterpret_cast<const float*>(&red[0][0][0]);
  constexpr int WS = 32 * (K + 1) * 4;  // floats per wave slice
  for (int i = threadIdx.x; i < nch * K; i += 256) {
    const int c = i / K, k = i % K;  // channel within slice, tap
    const int off = ((c >> 2) * (K + 1) + k) * 4 + (c & 3);
    atomicAdd(dw + (int64_t)(c_base + c) * K + k, rf[off] + rf[WS + off] + rf[2 * WS + off] + rf[3 * WS + off]);
  }
  if (db)
    for (int c = threadIdx.x; c < nch; c += 256) {
      const int off = ((c >> 2) * (K + 1) + K) * 4 + (c & 3);
      atomicAdd(db + c_base + c, rf[off] + rf[WS + off] + rf[2 * WS + off] + rf[3 * WS + off]);
    }
}

template <int K>
static void dwconv_tiled(const float* x, const float* w, const float* b, float* y, const float* g, float* dx,
                         float* dw, float* db, int64_t B, int64_t T, int64_t C, hipStream_t stream) {
  const int C4 = (int)(C / 4);
  const int ntile = (int)((T + DW_R - 1) / DW_R);
  const int64_t threads = B * ntile * C4;
  const unsigned grid = (unsigned)((threads + 255) / 256);
  if (y) dwconv_tile_kernel<K, false><<<grid, 256, 0, stream>>>((const float4*)x, w, b, (float4*)y, (int)B, (int)T, C4,
                                                                 ntile);
  if (dx) dwconv_tile_kernel<K, true><<<grid, 256, 0, stream>>>((const float4*)g, w, nullptr, (float4*)dx, (int)B,
                                                                 (int)T, C4, ntile);
  if (dw) {
    const int nchunk = (int)((T + 8 * DW_S * DW_R - 1) / (8 * DW_S * DW_R));
    const int64_t blocks = B * nchunk * ((C4 + 31) / 32);
    dwconv_wgrad_kernel<K><<<(unsigned)blocks, 256, 0, stream>>>((const float4*)g, (const float4*)x, dw, db, (int)T,
                                                                   C4, nchunk);
  }
}

static bool dwconv_dispatch(const float* x, const float* w, const float* b, float* y, const float* g, float* dx,
                            float* dw, float* db, int64_t B, int64_t T, int64_t C, int64_t K, hipStream_t stream) {
  if (C % 4 != 0 || ((uintptr_t)(x ? x : g) & 15) || (y && ((uintptr_t)y & 15)) || (dx && ((uintptr_t)dx & 15)) ||
      (b && ((uintptr_t)b & 15)) || B * T * C >= (1LL << 31))
    return false;
  switch (K) {
    case 3: dwconv_tiled<3>(x, w, b, y, g, dx, dw, db, B, T, C, stream); return true;
    case 5: dwconv_tiled<5>(x, w, b, y, g, dx, dw, db, B, T, C, stream); return true;
    case 7: dwconv_tiled<7>(x, w, b, y, g, dx, dw, db, B, T, C, stream); return true;
    case 15: dwconv_tiled<15>(x, w, b, y, g, dx, dw, db, B, T, C, stream); return true;
    default: return false;
  }
}

// ============================================================================ BatchNorm (per sample)
// nn.BatchNorm1d in train mode at batch 1 (ConvLite.bn, model.py:103, 114): statistics over T for
// each (sample, channel).  Stats kernel: grid (ceil(C/64), B).
__global__ __launch_bounds__(256) void bn_stats_kernel(const float* __restrict__ x, float* __restrict__ mean,
                                                       float* __restrict__ rstd, int64_t T, int C, float eps) {
  __shared__ float red[4][64];
  __shared__ float mu_s[64];
  const int b = blockIdx.y;
  const int tl = threadIdx.x & 63;
  const int c = blockIdx.x * 64 + tl;
  const int part = threadIdx.x >> 6;
  float s = 0.f;
  if (c < C)
    for (int64_t t = part; t < T; t += 4) s += x[((int64_t)b * T + t) * C + c];
  red[part][tl] = s;
  __syncthreads();
  if (part == 0) mu_s[tl] = (red[0][tl] + red[1][tl] + red[2][tl] + red[3][tl]) / T;
  __syncthreads();
  const float mu = mu_s[tl];
  float v = 0.f;
  if (c < C)
    for (int64_t t = part; t < T; t += 4) {
      const float d = x[((int64_t)b * T + t) * C + c] - mu;
      v += d * d;
    }
  __syncthreads();
  red[part][tl] = v;
  __syncthreads();
  if (part == 0 && c < C) {
    const float var = (red[0][tl] + red[1][tl] + red[2][tl] + red[3][tl]) / T;
    mean[(int64_t)b * C + c] = mu;
    rstd[(int64_t)b * C + c] = rsqrtf(var + eps);
  }
}

// float4 variant (C % 4 == 0): a 1024-thread workgroup per (sample, 128 channels); 32 row groups
// of 32 lanes stride over T, each lane keeping a Welford (mean, M2) for its 4 channels, combined
// across row groups with Chan's formula -- one HBM pass, numerically as stable as two passes.
__device__ __forceinline__ void chan_combine(float& na, float& ma, float& m2a, float nb, float mb, float m2b) {
  const float n = na + nb;
  if (n == 0.f) return;
  const float d = mb - ma;
  const float f = nb / n;
  ma += d * f;
  m2a += m2b + d * d * na * f;
  na = n;
}

__global__ __launch_bounds__(1024) void bn_stats4_kernel(const float4* __restrict__ x, float* __restrict__ mean,
                                                         float* __restrict__ rstd, int T, int C4, float eps) {
  __shared__ float4 sm[32][32], sq[32][32];
  const int lane = threadIdx.x & 31, grp = threadIdx.x >> 5;
  const int cchunks = (C4 + 31) / 32;
  const int cc = blockIdx.x % cchunks;
  const int64_t b = blockIdx.x / cchunks;
  const int c4 = cc * 32 + lane;
  float4 mu = make_float4(0.f, 0.f, 0.f, 0.f), m2 = mu;
  float n = 0.f;
  if (c4 < C4) {
    const float4* xs = x + b * T * C4 + c4;
    for (int t = grp; t < T; t += 32) {
      const float4 v = xs[(int64_t)t * C4];
      n += 1.f;
      const float r = 1.f / n;
      float d;
      d = v.x - mu.x; mu.x += d * r; m2.x += d * (v.x - mu.x);
      d = v.y - mu.y; mu.y += d * r; m2.y += d * (v.y - mu.y);
      d = v.z - mu.z; mu.z += d * r; m2.z += d * (v.z - mu.z);
      d = v.w - mu.w; mu.w += d * r; m2.w += d * (v.w - mu.w);
    }
  }
  sm[grp][lane] = mu;
  sq[grp][lane] = m2;
  __syncthreads();
  if (grp == 0 && c4 < C4) {
    // row group g saw rows g, g + 32, ...: count_g = ceil((T - g) / 32)
    float na = (float)((T + 31) / 32);
    float4 ma = sm[0][lane], qa = sq[0][lane];
    for (int g2 = 1; g2 < 32; ++g2) {
      const float nb = (float)((T - g2 + 31) / 32 > 0 ? (T - g2 + 31) / 32 : 0);
      const float4 mb = sm[g2][lane], qb = sq[g2][lane];
      float nx = na, ny = na, nz = na, nw = na;
      chan_combine(nx, ma.x, qa.x, nb, mb.x, qb.x);
      chan_combine(ny, ma.y, qa.y, nb, mb.y, qb.y);
      chan_combine(nz, ma.z, qa.z, nb, mb.z, qb.z);
      chan_combine(nw, ma.w, qa.w, nb, mb.w, qb.w);
      na = nx;
    }
    float* mo = mean + b * 4 * C4 + 4 * c4;
    float* ro = rstd + b * 4 * C4 + 4 * c4;
    mo[0] = ma.x; mo[1] = ma.y; mo[2] = ma.z; mo[3] = ma.w;
    ro[0] = rsqrtf(qa.x / T + eps); ro[1] = rsqrtf(qa.y / T + eps);
    ro[2] = rsqrtf(qa.z / T + eps); ro[3] = rsqrtf(qa.w / T + eps);
  }
}

// float4 variant of the backward sums (same workgroup shape as bn_stats4_kernel).
__global__ __launch_bounds__(1024) void bn_bwd_stats4_kernel(const float4* __restrict__ g, const float4* __restrict__ x,
                                                             const float* __restrict__ mean,
                                                             const float* __restrict__ rstd,
                                                             const float* __restrict__ w, float* __restrict__ sg,
                                                             float* __restrict__ sgx, float* __restrict__ dw,
                                                             float* __restrict__ db, int T, int C4) {
  __shared__ float4 sa[32][32], sx[32][32];
  const int lane = threadIdx.x & 31, grp = threadIdx.x >> 5;
  const int cchunks = (C4 + 31) / 32;
  const int cc = blockIdx.x % cchunks;
  const int64_t b = blockIdx.x / cchunks;
  const int c4 = cc * 32 + lane;
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f), ax = a;
  if (c4 < C4) {
    const float4 mu = *reinterpret_cast<const float4*>(mean + b * 4 * C4 + 4 * c4);
    const float4 rs = *reinterpret_cast<const float4*>(rstd + b * 4 * C4 + 4 * c4);
    const float4* gs = g + b * T * C4 + c4;
    const float4* xs = x + b * T * C4 + c4;
    for (int t = grp; t < T; t += 32) {
      const float4 gv = gs[(int64_t)t * C4], xv = xs[(int64_t)t * C4];
      a.x += gv.x; a.y += gv.y; a.z += gv.z; a.w += gv.w;
      ax.x += gv.x * (xv.x - mu.x) * rs.x;
      ax.y += gv.y * (xv.y - mu.y) * rs.y;
      ax.z += gv.z * (xv.z - mu.z) * rs.z;
      ax.w += gv.w * (xv.w - mu.w) * rs.w;
    }
  }
  sa[grp][lane] = a;
  sx[grp][lane] = ax;
  __syncthreads();
  if (grp < 8 && c4 < C4) {  // 8 x 32 lanes: one (channel, sum) each
    const int q = grp & 3, which = grp >> 2;
    float s = 0.f;
    for (int g2 = 0; g2 < 32; ++g2) {
      const float4 v = which ? sx[g2][lane] : sa[g2][lane];
      s += q == 0 ? v.x : q == 1 ? v.y : q == 2 ? v.z : v.w;
    }
    const int c = 4 * c4 + q;
    if (which) {
      sgx[b * 4 * C4 + c] = s * w[c];
      atomicAdd(dw + c, s);
    } else {
      sg[b * 4 * C4 + c] = s * w[c];
      atomicAdd(db + c, s);
    }
  }
}

// y = (x - mean[b,c]) * rstd[b,c] * w[c] + bb[c]   (mean/rstd per sample, or shared when B_stats == 1)
__global__ void bn_apply_kernel(const float* __restrict__ x, const float* __restrict__ mean,
                                const float* __restrict__ rstd, const float* __restrict__ w, const float* __restrict__ bb,
                                float* __restrict__ y, int64_t B, int64_t T, int C, int per_sample) {
  const int64_t total = B * T * C;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t c = i % C;
    const int64_t b = i / (T * C);
    const int64_t s = per_sample ? b * C + c : c;
    y[i] = (x[i] - mean[s]) * rstd[s] * w[c] + bb[c];
  }
}

// per-(b,c) sums for backward: sg[b,c] = sum_t g*w, sgx[b,c] = sum_t g*w*xhat ; dw += sum g*xhat,
// db += sum g.  grid (ceil(C/64), B)
__global__ __launch_bounds__(256) void bn_bwd_stats_kernel(const float* __restrict__ g, const float* __restrict__ x,
                                                           const float* __restrict__ mean, const float* __restrict__ rstd,
                                                           const float* __restrict__ w, float* __restrict__ sg,
                                                           float* __restrict__ sgx, float* __restrict__ dw,
                                                           float* __restrict__ db, int64_t T, int C) {
  __shared__ float red[2][4][64];
  const int b = blockIdx.y;
  const int tl = threadIdx.x & 63;
  const int c = blockIdx.x * 64 + tl;
  const int part = threadIdx.x >> 6;
  float a = 0.f, ax = 0.f;
  if (c < C) {
    const float mu = mean[(int64_t)b * C + c], rs = rstd[(int64_t)b * C + c];
    for (int64_t t = part; t < T; t += 4) {
      const int64_t i = ((int64_t)b * T + t) * C + c;
      const float gv = g[i];
      a += gv;
      ax += gv * (x[i] - mu) * rs;
    }
  }
  red[0][part][tl] = a;
  red[1][part][tl] = ax;
  __syncthreads();
  if (part == 0 && c < C) {
    const float A = red[0][0][tl] + red[0][1][tl] + red[0][2][tl] + red[0][3][tl];
    const float AX = red[1][0][tl] + red[1][1][tl] + red[1][2][tl] + red[1][3][tl];
    sg[(int64_t)b * C + c] = A * w[c];
    sgx[(int64_t)b * C + c] = AX * w[c];
    atomicAdd(dw + c, AX);
    atomicAdd(db + c, A);
  }
}

__global__ void bn_bwd_apply_kernel(const float* __restrict__ g, const float* __restrict__ x,
                                    const float* __restrict__ mean, const float* __restrict__ rstd,
                                    const float* __restrict__ w, const float* __restrict__ sg,
                                    const float* __restrict__ sgx, float* __restrict__ dx, int64_t B, int64_t T, int C) {
  const int64_t total = B * T * C;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t c = i % C;
    const int64_t b = i / (T * C);
    const int64_t s = b * C + c;
    const float rs = rstd[s];
    const float xh = (x[i] - mean[s]) * rs;
    dx[i] = rs * (g[i] * w[c] - sg[s] / T - xh * sgx[s] / T);
  }
}

// ============================================================================ Conv1d(1, D, 3) stem
// AudioEncoder.conv2 (model.py:132-135) for single-channel streams: y[b,t,o] = bias[o] +
// sum_k W[o,k] x[b, t+k-1].  Output channels-last.
__global__ void stem1_fwd_kernel(const float* __restrict__ x, const float* __restrict__ W, const float* __restrict__ bias,
                                 float* __restrict__ y, int64_t B, int64_t T, int D) {
  const int64_t total = B * T * D;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t o = i % D;
    const int64_t t = (i / D) % T;
    const int64_t b = i / (T * D);
    const float* xr = x + b * T;
    float s = bias[o];
    if (t > 0) s += W[o * 3 + 0] * xr[t - 1];
    s += W[o * 3 + 1] * xr[t];
    if (t + 1 < T) s += W[o * 3 + 2] * xr[t + 1];
    y[i] = s;
  }
}
// dW[o,k] += sum_{b,t} g[b,t,o] x[b,t+k-1]; db[o] += sum g.  grid (ceil(D/64), B*chunks)
__global__ __launch_bounds__(256) void stem1_bwd_w_kernel(const float* __restrict__ g, const float* __restrict__ x,
                                                          float* __restrict__ dW, float* __restrict__ db, int64_t B,
                                                          int64_t T, int D, int64_t chunk) {
  __shared__ float red[4][64][4];
  const int tl = threadIdx.x & 63;
  const int o = blockIdx.x * 64 + tl;
  const int part = threadIdx.x >> 6;
  const int64_t nch = (T + chunk - 1) / chunk;
  const int64_t b = blockIdx.y / nch;
  const int64_t t0 = (blockIdx.y % nch) * chunk, t1 = min(T, t0 + chunk);
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, ab = 0.f;
  if (o < D) {
    const float* xr = x + b * T;
    for (int64_t t = t0 + part; t < t1; t += 4) {
      const float gv = g[(b * T + t) * D + o];
      ab += gv;
      if (t > 0) a0 += gv * xr[t - 1];
      a1 += gv * xr[t];
      if (t + 1 < T) a2 += gv * xr[t + 1];
    }
  }
  red[part][tl][0] = a0;
  red[part][tl][1] = a1;
  red[part][tl][2] = a2;
  red[part][tl][3] = ab;
  __syncthreads();
  if (part == 0 && o < D) {
    for (int k = 0; k < 4; ++k) {
      const float s = red[0][tl][k] + red[1][tl][k] + red[2][tl][k] + red[3][tl][k];
      if (k < 3) atomicAdd(dW + o * 3 + k, s);
      else atomicAdd(db + o, s);
    }
  }
}

// ============================================================================ embedding
// processor.token (model.py:592, 606): y[r] = E[ids[r]]; backward scatter-adds rows.
__global__ void embed_fwd_kernel(const int64_t* __restrict__ ids, const float* __restrict__ E, float* __restrict__ y,
                                 int64_t rows, int d) {
  const int64_t total = rows * d;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / d, c = i % d;
    y[i] = E[ids[r] * d + c];
  }
}
__global__ void embed_bwd_kernel(const int64_t* __restrict__ ids, const float* __restrict__ g, float* __restrict__ dE,
                                 int64_t rows, int d) {
  const int64_t total = rows * d;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / d, c = i % d;
    atomicAdd(dE + ids[r] * d + c, g[i]);
  }
}

// ============================================================================ cross entropy
// F.cross_entropy(logits, labels, ignore_index=0) (model.py:670) over fp32 logits rows of V:
// loss[r] = logsumexp(z_r) - z_r[label] (0 for ignored rows), lse[r] saved.
__global__ __launch_bounds__(256) void ce_fwd_kernel(const float* __restrict__ z, const int64_t* __restrict__ labels,
                                                     float* __restrict__ loss, float* __restrict__ lse, int64_t V) {
  __shared__ float red[4];
  const int64_t r = blockIdx.x;
  const float* zr = z + r * V;
  float m = -INFINITY;
  for (int64_t j = threadIdx.x; j < V; j += 256) m = fmaxf(m, zr[j]);
  m = wave_max_dpp(m);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  __syncthreads();
  float s = 0.f;
  for (int64_t j = threadIdx.x; j < V; j += 256) s += expf(zr[j] - m);
  s = block_sum<256>(s, red);
  if (threadIdx.x == 0) {
    const float l = m + logf(s);
    lse[r] = l;
    const int64_t y = labels[r];
    loss[r] = (y == 0) ? 0.f : l - zr[y];
  }
}
// dz = scale * (softmax - onehot) for non-ignored rows, 0 otherwise (in place allowed)
__global__ __launch_bounds__(256) void ce_bwd_kernel(const float* __restrict__ z, const int64_t* __restrict__ labels,
                                                     const float* __restrict__ lse, const float* __restrict__ scale,
                                                     float* __restrict__ dz, int64_t V) {
  const int64_t r = blockIdx.x;
  const int64_t y = labels[r];
  const float sc = (y == 0) ? 0.f : scale[0];
  const float l = lse[r];
  for (int64_t j = threadIdx.x; j < V; j += 256) {
    const float p = expf(z[r * V + j] - l);
    dz[r * V + j] = sc * (p - (j == y ? 1.f : 0.f));
  }
}

// F.normalize(x, p=2, dim=-1) rows (v_gate's memory keys, model.py:347): y = x / max(|x|, 1e-12),
// n = max(|x|, 1e-12); backward dx (+)= (dy - y (y.dy)) / n (the clamp is never active at random
// init, |mkey| ~ sqrt(D); a clamped row gets dy / n).
__global__ __launch_bounds__(64 * RW) void row_normalize_kernel(const float* __restrict__ x, float* __restrict__ y,
                                                                float* __restrict__ n, int64_t rows, int d) {
  const int lane = threadIdx.x & 63;
  for (int64_t r = row_begin(); r < rows; r += row_step()) {
    float s = 0.f;
    for (int j = lane; j < d; j += 64) s += x[r * d + j] * x[r * d + j];
    const float nn = fmaxf(sqrtf(wave_sum_dpp(s)), 1e-12f);
    for (int j = lane; j < d; j += 64) y[r * d + j] = x[r * d + j] / nn;
    if (lane == 0) n[r] = nn;
  }
}
__global__ __launch_bounds__(64 * RW) void row_normalize_bwd_kernel(const float* __restrict__ dy,
                                                                    const float* __restrict__ y,
                                                                    const float* __restrict__ n, float* __restrict__ dx,
                                                                    int64_t rows, int d, int acc) {
  const int lane = threadIdx.x & 63;
  constexpr int C = 16;  // d <= 64 C: every operand of the row (y, dy, the accumulated dx) loaded at once
  for (int64_t r = row_begin(); r < rows; r += row_step()) {
    const float nn = n[r];
    if (d <= 64 * C) {  // same arithmetic and order as the general loop below, one load round trip per row
      float yv[C], gv[C], ov[C];
#pragma unroll
      for (int i = 0; i < C; ++i) {
        const int j = lane + 64 * i;
        const bool ok = j < d;
        yv[i] = ok ? y[r * d + j] : 0.f;
        gv[i] = ok ? dy[r * d + j] : 0.f;
        ov[i] = ok && acc ? dx[r * d + j] : 0.f;
      }
      float s = 0.f;
#pragma unroll
      for (int i = 0; i < C; ++i)
        if (lane + 64 * i < d) s += yv[i] * gv[i];
      s = wave_sum_dpp(s);
      const bool clamped = nn <= 1e-12f;
#pragma unroll
      for (int i = 0; i < C; ++i) {
        const int j = lane + 64 * i;
        if (j < d) dx[r * d + j] = ov[i] + (gv[i] - (clamped ? 0.f : yv[i] * s)) / nn;
      }
      continue;
    }
    float s = 0.f;
    for (int j = lane; j < d; j += 64) s += y[r * d + j] * dy[r * d + j];
    s = wave_sum_dpp(s);
    const bool clamped = nn <= 1e-12f;
    for (int j = lane; j < d; j += 64) {
      const float v = (dy[r * d + j] - (clamped ? 0.f : y[r * d + j] * s)) / nn;
      dx[r * d + j] = (acc ? dx[r * d + j] : 0.f) + v;
    }
  }
}

// softmax over short rows (N <= 8): MPNet's policy, model.py:385
__global__ void softmax_small_kernel(const float* __restrict__ x, float* __restrict__ y, int64_t rows, int N) {
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < rows; r += (int64_t)gridDim.x * blockDim.x) {
    float m = -INFINITY;
    for (int k = 0; k < N; ++k) m = fmaxf(m, x[r * N + k]);
    float s = 0.f;
    for (int k = 0; k < N; ++k) s += expf(x[r * N + k] - m);
    for (int k = 0; k < N; ++k) y[r * N + k] = expf(x[r * N + k] - m) / s;
  }
}
__global__ void softmax_small_bwd_kernel(const float* __restrict__ g, const float* __restrict__ y, float* __restrict__ dx,
                                         int64_t rows, int N) {
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < rows; r += (int64_t)gridDim.x * blockDim.x) {
    float s = 0.f;
    for (int k = 0; k < N; ++k) s += g[r * N + k] * y[r * N + k];
    for (int k = 0; k < N; ++k) dx[r * N + k] = y[r * N + k] * (g[r * N + k] - s);
  }
}

}  // namespace asrx

using namespace asrx;

#define LAUNCH_ROWS(kernel, rows, shm, ...) \
  kernel<<<row_grid(rows), 64 * RW, shm, stream>>>(__VA_ARGS__)
#define LAUNCH_EW(kernel, n, ...) kernel<<<ew_grid(n), 256, 0, stream>>>(__VA_ARGS__)

extern "C" {

int asrx_layernorm_fwd(const float* x, const float* w, const float* b, float* y, float* mean, float* rstd,
                       int64_t rows, int64_t d, float eps, hipStream_t stream) {
  if (rows == 0) return 0;
  const bool al = ((((uintptr_t)x | (uintptr_t)w | (uintptr_t)b | (uintptr_t)y) & 7) == 0);
  switch (al ? d : 0) {
#define LNF(E) LAUNCH_ROWS(ln_fwd_t_kernel<E>, rows, 0, x, w, b, y, mean, rstd, rows, eps, nullptr, nullptr, nullptr, \
                           nullptr, 0)
    case 128: LNF(2); break;
    case 256: LNF(4); break;
    case 384: LNF(6); break;
    case 512: LNF(8); break;
    case 768: LNF(12); break;
    case 1024: LNF(16); break;
#undef LNF
    default: LAUNCH_ROWS(ln_fwd_kernel, rows, 0, x, w, b, y, mean, rstd, rows, (int)d, eps);
  }
  ASRX_LAUNCHED("asrx_layernorm_fwd");
}

// LayerNorm forward with the fused row outputs of ln_fwd_t_kernel (nrm and/or the sigmoid gate; each
// may be null).  d must be one of 128, 256, 384, 512, 768, 1024.
// y stored fp32 (y_bf16 = 0) or bf16 (1: MSheath's mlp_ln output only feeds mlp[0], model.py:503-506)
int asrx_layernorm_fwd3(const float* x, const float* w, const float* b, void* y, int y_bf16, float* mean, float* rstd,
                        float* nrm, const float* gw, const float* gb, float* gout, int gate_on_x, int64_t rows,
                        int64_t d, float eps, hipStream_t stream) {
  if (rows == 0) return 0;
  const bool al = ((((uintptr_t)x | (uintptr_t)w | (uintptr_t)b | (uintptr_t)y | (uintptr_t)gw) & 7) == 0);
  ASRX_REQUIRE(al, "asrx_layernorm_fwd2: 8-byte aligned rows required");
  switch (d) {
#define LNF(E)                                                                                                    \
  if (y_bf16)                                                                                                     \
    LAUNCH_ROWS((ln_fwd_t_kernel<E, unsigned short>), rows, 0, x, w, b, (unsigned short*)y, mean, rstd, rows, eps, \
                nrm, gw, gb, gout, gate_on_x);                                                                    \
  else                                                                                                            \
    LAUNCH_ROWS((ln_fwd_t_kernel<E, float>), rows, 0, x, w, b, (float*)y, mean, rstd, rows, eps, nrm, gw, gb, gout, \
                gate_on_x)
    case 128: LNF(2); break;
    case 256: LNF(4); break;
    case 384: LNF(6); break;
    case 512: LNF(8); break;
    case 768: LNF(12); break;
    case 1024: LNF(16); break;
#undef LNF
    default: ASRX_REQUIRE(false, "asrx_layernorm_fwd2: d=%ld unsupported", (long)d);
  }
  ASRX_LAUNCHED("asrx_layernorm_fwd2");
}

int asrx_layernorm_fwd2(const float* x, const float* w, const float* b, float* y, float* mean, float* rstd,
                        float* nrm, const float* gw, const float* gb, float* gout, int gate_on_x, int64_t rows,
                        int64_t d, float eps, hipStream_t stream) {
  return asrx_layernorm_fwd3(x, w, b, y, 0, mean, rstd, nrm, gw, gb, gout, gate_on_x, rows, d, eps, stream);
}

int asrx_layernorm_bwd_acc(const float* dy, const float* x, const float* w, const float* mean, const float* rstd,
                           float* dx, float* dw, float* db, int64_t rows, int64_t d, int acc, hipStream_t stream) {
  ASRX_REQUIRE(d <= 2048, "layernorm_bwd: d too large");
  if (rows == 0) return 0;
  const bool al = ((((uintptr_t)dy | (uintptr_t)x | (uintptr_t)w | (uintptr_t)dx) & 7) == 0);
  const unsigned g = row_grid(rows, 1024);
  switch (al ? d : 0) {
    case 128: ln_bwd_t_kernel<2><<<g, 64 * RW, 0, stream>>>(dy, x, w, mean, rstd, dx, dw, db, rows, acc); break;
    case 256: ln_bwd_t_kernel<4><<<g, 64 * RW, 0, stream>>>(dy, x, w, mean, rstd, dx, dw, db, rows, acc); break;
    case 384: ln_bwd_t_kernel<6><<<g, 64 * RW, 0, stream>>>(dy, x, w, mean, rstd, dx, dw, db, rows, acc); break;
    case 512: ln_bwd_t_kernel<8><<<g, 64 * RW, 0, stream>>>(dy, x, w, mean, rstd, dx, dw, db, rows, acc); break;
    case 768: ln_bwd_t_kernel<12><<<g, 64 * RW, 0, stream>>>(dy, x, w, mean, rstd, dx, dw, db, rows, acc); break;
    case 1024: ln_bwd_t_kernel<16><<<g, 64 * RW, 0, stream>>>(dy, x, w, mean, rstd, dx, dw, db, rows, acc); break;
    default: {
      const size_t shm = (size_t)RW * 2 * d * sizeof(float);
      ln_bwd_kernel<<<g, 64 * RW, shm, stream>>>(dy, x, w, mean, rstd, dx, dw, db, rows, (int)d, acc);
    }
  }
  ASRX_LAUNCHED("asrx_layernorm_bwd");
}

// dx = LN backward (overwritten); dw / db accumulated.
int asrx_layernorm_bwd(const float* dy, const float* x, const float* w, const float* mean, const float* rstd,
                       float* dx, float* dw, float* db, int64_t rows, int64_t d, hipStream_t stream) {
  return asrx_layernorm_bwd_acc(dy, x, w, mean, rstd, dx, dw, db, rows, d, 0, stream);
}

}  // extern "C"
template <typename TX>
static int small_linear_fwd_t(const TX* x, const float* W, const float* b, float* y, int64_t rows, int64_t K,
                              int64_t N, int act, hipStream_t stream) {
  switch (N) {
    case 1: LAUNCH_ROWS((small_linear_fwd_kernel<1, TX>), rows, 0, x, W, b, y, rows, (int)K, act); break;
    case 2: LAUNCH_ROWS((small_linear_fwd_kernel<2, TX>), rows, 0, x, W, b, y, rows, (int)K, act); break;
    case 3: LAUNCH_ROWS((small_linear_fwd_kernel<3, TX>), rows, 0, x, W, b, y, rows, (int)K, act); break;
    case 4: LAUNCH_ROWS((small_linear_fwd_kernel<4, TX>), rows, 0, x, W, b, y, rows, (int)K, act); break;
    default: ASRX_REQUIRE(false, "small_linear: N=%ld not in 1..4", (long)N);
  }
  return 0;
}

extern "C" {
// x stored fp32 (x_bf16 = 0) or bf16 (1)
int asrx_small_linear_fwd2(const void* x, int x_bf16, const float* W, const float* b, float* y, int64_t rows,
                           int64_t K, int64_t N, int act, hipStream_t stream) {
  if (rows == 0) return 0;
  const int rc = x_bf16 ? small_linear_fwd_t((const unsigned short*)x, W, b, y, rows, K, N, act, stream)
                        : small_linear_fwd_t((const float*)x, W, b, y, rows, K, N, act, stream);
  if (rc) return rc;
  ASRX_LAUNCHED("asrx_small_linear_fwd");
}

int asrx_small_linear_fwd(const float* x, const float* W, const float* b, float* y, int64_t rows, int64_t K,
                          int64_t N, int act, hipStream_t stream) {
  return asrx_small_linear_fwd2(x, 0, W, b, y, rows, K, N, act, stream);
}

}  // extern "C"
// per-stream partial buffer of small_linear_bwd_kernel, allocated once at its largest size (grid <= 1024
// workgroups x (N K + N) <= 64 KB / RW floats: 16 MB) so it never grows: a stream's launches reuse it in stream
// order, and nothing is freed or synchronised while a graph capture may be running.  A stream's first use may
// come inside a capture (bench.py --graph captures on its own stream), so the allocation runs in relaxed
// capture mode, as PyTorch's allocator does; the buffer outlives the graph that records its address.
constexpr size_t SL_WS_BYTES = (size_t)1024 * (64 * 1024 / RW);
// Keyed by (device, stream): the null stream's handle is the same on every device, and a destroyed stream's
// handle can come back on another device, so the handle alone could hand one device's buffer to another.
static int sl_workspace(hipStream_t stream, float** ws) {
  static std::map<std::pair<int, hipStream_t>, float*> pool;
  static std::mutex mu;
  int dev = 0;
  const hipError_t de = hipGetDevice(&dev);
  if (de != hipSuccess) {
    asrx::set_error("small_linear_bwd workspace: hipGetDevice: %s", hipGetErrorString(de));
    return (int)de;
  }
  std::lock_guard<std::mutex> lk(mu);
  float*& buf = pool[std::make_pair(dev, stream)];
  if (!buf) {
    hipStreamCaptureMode mode = hipStreamCaptureModeRelaxed;
    (void)hipThreadExchangeStreamCaptureMode(&mode);
    const hipError_t e = hipMalloc(&buf, SL_WS_BYTES);
    (void)hipThreadExchangeStreamCaptureMode(&mode);
    if (e != hipSuccess) {
      buf = nullptr;
      asrx::set_error("small_linear_bwd workspace: %s", hipGetErrorString(e));
      return (int)e;
    }
  }
  *ws = buf;
  return 0;
}

template <typename TX>
static int small_linear_bwd_t(const float* dy, const float* y, const TX* x, const float* W, float* dx, float* dW,
                              float* db, int64_t rows, int64_t K, int64_t N, int act, float beta, hipStream_t stream) {
  const size_t shm = (size_t)RW * (N * K + N) * sizeof(float);
  ASRX_REQUIRE(shm <= 64 * 1024, "small_linear_bwd: K too large");
  const unsigned g = row_grid(rows, 1024);
  ASRX_REQUIRE((size_t)g * (N * K + N) * sizeof(float) <= SL_WS_BYTES, "small_linear_bwd: partials exceed the workspace");
  float* ws = nullptr;
  const int rc = sl_workspace(stream, &ws);
  if (rc) return rc;
  switch (N) {
    case 1: small_linear_bwd_kernel<1, TX><<<g, 64 * RW, shm, stream>>>(dy, y, x, W, dx, dW, db, rows, (int)K, act, beta, ws); break;
    case 2: small_linear_bwd_kernel<2, TX><<<g, 64 * RW, shm, stream>>>(dy, y, x, W, dx, dW, db, rows, (int)K, act, beta, ws); break;
    case 3: small_linear_bwd_kernel<3, TX><<<g, 64 * RW, shm, stream>>>(dy, y, x, W, dx, dW, db, rows, (int)K, act, beta, ws); break;
    case 4: small_linear_bwd_kernel<4, TX><<<g, 64 * RW, shm, stream>>>(dy, y, x, W, dx, dW, db, rows, (int)K, act, beta, ws); break;
    default: ASRX_REQUIRE(false, "small_linear: N=%ld not in 1..4", (long)N);
  }
  small_linear_colsum_kernel<<<(unsigned)(N * K + N), 64, 0, stream>>>(ws, (int)g, (int)(N * K + N), (int)(N * K), dW, db);
  return 0;
}

extern "C" {
int asrx_small_linear_bwd2(const float* dy, const float* y, const void* x, int x_bf16, const float* W, float* dx,
                           float* dW, float* db, int64_t rows, int64_t K, int64_t N, int act, float beta,
                           hipStream_t stream) {
  if (rows == 0) return 0;
  const int rc = x_bf16 ? small_linear_bwd_t(dy, y, (const unsigned short*)x, W, dx, dW, db, rows, K, N, act, beta, stream)
                        : small_linear_bwd_t(dy, y, (const float*)x, W, dx, dW, db, rows, K, N, act, beta, stream);
  if (rc) return rc;
  ASRX_LAUNCHED("asrx_small_linear_bwd");
}

int asrx_small_linear_bwd(const float* dy, const float* y, const float* x, const float* W, float* dx, float* dW,
                          float* db, int64_t rows, int64_t K, int64_t N, int act, float beta, hipStream_t stream) {
  return asrx_small_linear_bwd2(dy, y, x, 0, W, dx, dW, db, rows, K, N, act, beta, stream);
}

int asrx_row_normalize(const float* x, float* y, float* n, int64_t rows, int64_t d, hipStream_t stream) {
  if (rows == 0) return 0;
  LAUNCH_ROWS(row_normalize_kernel, rows, 0, x, y, n, rows, (int)d);
  ASRX_LAUNCHED("asrx_row_normalize");
}

int asrx_row_normalize_bwd(const float* dy, const float* y, const float* n, float* dx, int64_t rows, int64_t d,
                           int acc, hipStream_t stream) {
  if (rows == 0) return 0;
  LAUNCH_ROWS(row_normalize_bwd_kernel, rows, 0, dy, y, n, dx, rows, (int)d, acc);
  ASRX_LAUNCHED("asrx_row_normalize_bwd");
}

int asrx_softmax_small(const float* x, float* y, int64_t rows, int64_t N, hipStream_t stream) {
  ASRX_REQUIRE(N >= 1 && N <= 8, "softmax_small: N in 1..8");
  if (rows == 0) return 0;
  softmax_small_kernel<<<ew_grid(rows, 1024), 256, 0, stream>>>(x, y, rows, (int)N);
  ASRX_LAUNCHED("asrx_softmax_small");
}

int asrx_softmax_small_bwd(const float* g, const float* y, float* dx, int64_t rows, int64_t N, hipStream_t stream) {
  ASRX_REQUIRE(N >= 1 && N <= 8, "softmax_small: N in 1..8");
  if (rows == 0) return 0;
  softmax_small_bwd_kernel<<<ew_grid(rows, 1024), 256, 0, stream>>>(g, y, dx, rows, (int)N);
  ASRX_LAUNCHED("asrx_softmax_small_bwd");
}

// zero `bytes` bytes of device memory (stream-ordered memset; no ATen fill kernel)
int asrx_zero(void* p, int64_t bytes, hipStream_t stream) {
  if (bytes == 0) return 0;
  hipError_t e = hipMemsetAsync(p, 0, (size_t)bytes, stream);
  if (e != hipSuccess) {
    set_error("asrx_zero: %s", hipGetErrorString(e));
    return (int)e;
  }
  return 0;
}

int asrx_rownorm(const float* x, float* n, int64_t rows, int64_t d, hipStream_t stream) {
  if (rows == 0) return 0;
  LAUNCH_ROWS(rownorm_kernel, rows, 0, x, n, rows, (int)d);
  ASRX_LAUNCHED("asrx_rownorm");
}

int asrx_rownorm_bwd(const float* dn, const float* x, const float* n, float* dx, int64_t rows, int64_t d,
                     hipStream_t stream) {
  if (rows == 0) return 0;
  LAUNCH_EW(rownorm_bwd_kernel, rows * d, dn, x, n, dx, rows, (int)d, 1);
  ASRX_LAUNCHED("asrx_rownorm_bwd");
}

// acc == 0: dx = the |x| gradient (written, not accumulated)
int asrx_rownorm_bwd2(const float* dn, const float* x, const float* n, float* dx, int64_t rows, int64_t d, int acc,
                      hipStream_t stream) {
  if (rows == 0) return 0;
  LAUNCH_EW(rownorm_bwd_kernel, rows * d, dn, x, n, dx, rows, (int)d, acc);
  ASRX_LAUNCHED("asrx_rownorm_bwd2");
}

int asrx_rotary_fwd2(const float* x, const float* m, const float* f, const float* tab, float* y, int64_t BL, int64_t L,
                     int64_t D, int64_t hd, float scale, hipStream_t stream);
int asrx_rotary_bwd2(const float* g, const float* x, const float* m, const float* f, const float* tab, float* dx,
                     float* dm, int64_t BL, int64_t L, int64_t D, int64_t hd, float scale, hipStream_t stream);
int asrx_rotary_fwd(const float* x, const float* m, const float* f, float* y, int64_t BL, int64_t L, int64_t D,
                    int64_t hd, float scale, hipStream_t stream) {
  return asrx_rotary_fwd2(x, m, f, nullptr, y, BL, L, D, hd, scale, stream);
}

int asrx_rotary_bwd(const float* g, const float* x, const float* m, const float* f, float* dx, float* dm, int64_t BL,
                    int64_t L, int64_t D, int64_t hd, float scale, hipStream_t stream) {
  return asrx_rotary_bwd2(g, x, m, f, nullptr, dx, dm, BL, L, D, hd, scale, stream);
}

int asrx_rotary_table(const float* f, float* tab, int64_t L, int64_t hd, hipStream_t stream) {
  ASRX_REQUIRE(hd % 2 == 0 && L > 0, "asrx_rotary_table: bad head dim / length");
  const int64_t n = L * (hd / 2);
  rotary_table_kernel<<<ew_grid(n), 256, 0, stream>>>(f, reinterpret_cast<float2*>(tab), L, (int)(hd / 2));
  ASRX_LAUNCHED("asrx_rotary_table");
}

int asrx_rotary_fwd2(const float* x, const float* m, const float* f, const float* tab, float* y, int64_t BL, int64_t L,
                     int64_t D, int64_t hd, float scale, hipStream_t stream) {
  ASRX_REQUIRE(hd % 2 == 0 && D % hd == 0, "rotary: bad head dim");
  if (BL == 0) return 0;
  LAUNCH_ROWS(rotary_fwd_kernel, BL, 0, x, m, f, reinterpret_cast<const float2*>(tab), y, BL, L, (int)D, (int)hd,
              scale);
  ASRX_LAUNCHED("asrx_rotary_fwd");
}

int asrx_rotary_bwd2(const float* g, const float* x, const float* m, const float* f, const float* tab, float* dx,
                     float* dm, int64_t BL, int64_t L, int64_t D, int64_t hd, float scale, hipStream_t stream) {
  if (BL == 0) return 0;
  LAUNCH_ROWS(rotary_bwd_kernel, BL, 0, g, x, m, f, reinterpret_cast<const float2*>(tab), dx, dm, BL, L, (int)D,
              (int)hd, scale);
  ASRX_LAUNCHED("asrx_rotary_bwd");
}

int asrx_vgate_fwd(const float* S, const float* nx, const float* mval, const float* h, const float* w2,
                   const float* b2, const float* cw, const float* cb, const float* tx, float* ion, float* xval,
                   float* kv, float* m2, int64_t rows, int64_t M, int64_t Dh, float inv_sqrt_d, hipStream_t stream) {
  ASRX_REQUIRE(M <= 64, "vgate: memory size must be <= 64");
  if (rows == 0) return 0;
  LAUNCH_ROWS(vgate_fwd_kernel, rows, 0, S, nx, mval, h, w2, b2, cw, cb, tx, ion, xval, kv, m2, rows, (int)M,
              (int)Dh, inv_sqrt_d);
  ASRX_LAUNCHED("asrx_vgate_fwd");
}

int asrx_vgate_bwd(const float* dion, const float* S, const float* nx, const float* mval, const float* h,
                   const float* w2, const float* cw, const float* kv, const float* m2, float* dS, float* dnx,
                   float* dh, float* dmval, float* dw2, float* db2, float* dcw, float* dcb, int64_t rows, int64_t M,
                   int64_t Dh, float inv_sqrt_d, hipStream_t stream) {
  if (rows == 0) return 0;
  const size_t shm = (size_t)RW * (M + Dh + 4) * sizeof(float);
  vgate_bwd_kernel<<<row_grid(rows, 1024), 64 * RW, shm, stream>>>(dion, S, nx, mval, h, w2, cw, kv, m2, dS, dnx, dh,
                                                                    dmval, dw2, db2, dcw, dcb, rows, (int)M, (int)Dh,
                                                                    inv_sqrt_d);
  ASRX_LAUNCHED("asrx_vgate_bwd");
}

int asrx_vgate_weights(const float* mkey, const float* W1, const float* b1, float* Wc, float* bc, float* mkn,
                       unsigned short* wb, int64_t M, int64_t Dh, int64_t D, hipStream_t stream) {
  if (M + Dh == 0) return 0;
  LAUNCH_ROWS(vgate_weights_kernel, M + Dh, 0, mkey, W1, b1, Wc, bc, mkn, wb, (int)M, (int)Dh, (int)D);
  ASRX_LAUNCHED("asrx_vgate_weights");
}

#define MS_DISPATCH(KER, GRID, SHM, P)                                             \
  switch (d) {                                                                     \
    case 128: KER<2><<<GRID, 64 * RW, SHM, stream>>>(P); break;                    \
    case 256: KER<4><<<GRID, 64 * RW, SHM, stream>>>(P); break;                    \
    case 384: KER<6><<<GRID, 64 * RW, SHM, stream>>>(P); break;                    \
    case 512: KER<8><<<GRID, 64 * RW, SHM, stream>>>(P); break;                    \
    case 768: KER<12><<<GRID, 64 * RW, SHM, stream>>>(P); break;                   \
    case 1024: KER<16><<<GRID, 64 * RW, SHM, stream>>>(P); break;                  \
    default: ASRX_REQUIRE(false, #KER ": d=%ld unsupported", (long)d);             \
  }

static bool ms_aligned(std::initializer_list<const void*> ps) {
  for (const void* q : ps)
    if ((uintptr_t)q & 7) return false;
  return true;
}

}  // extern "C"
namespace asrx {
static bool g_row_nofill = false;
// asrx_msheath_fwd (msheath_plan.cpp, the no-grad composite) sets this around its layer loop
void set_msheath_row_nofill(bool on) { g_row_nofill = on; }
}  // namespace asrx
extern "C" {

// Fused MSheath layer row pass (msheath_row_fwd_kernel); SH = [S | h] with row stride ldsh >= M + Dh.
int asrx_msheath_row_fwd2(const float* x, const float* lnw, const float* lnb, const float* gw, const float* gb,
                          const float* SH, int64_t ldsh, const float* mval, const float* w2, const float* b2,
                          const float* cw, const float* cb, const float* tx, void* px, int px_bf16, float* mean,
                          float* rstd, float* nx, float* g, float* ion, float* kv, float* m2, int64_t rows, int64_t d,
                          int64_t M, int64_t Dh, float eps, float inv_sqrt_d, const float* next_i, int64_t layer,
                          int64_t L, hipStream_t stream) {
  ASRX_REQUIRE(M <= 64 && ldsh >= M + Dh, "asrx_msheath_row_fwd: M <= 64 and ldsh >= M + Dh required");
  ASRX_REQUIRE(Dh <= 64 * ((d / 64 + 1) / 2), "asrx_msheath_row_fwd: v_gate hidden size Dh <= d / 2 required");
  ASRX_REQUIRE(ms_aligned({x, lnw, lnb, gw, (const float*)px}), "asrx_msheath_row_fwd: 8-byte aligned rows required");
  ASRX_REQUIRE(!next_i || L > 0, "asrx_msheath_row_fwd: L > 0 required with next_i");
  if (rows == 0) return 0;
  MSRowFwd p{x, lnw, lnb, gw, gb, SH, mval, w2, b2, cw, cb, tx, px_bf16 ? nullptr : (float*)px, mean, rstd, nx, g,
             ion, kv, m2, rows, ldsh, (int)M, (int)Dh, eps, inv_sqrt_d, next_i, (int)layer, L > 0 ? L : 1,
             px_bf16 ? (unsigned short*)px : nullptr, nullptr, nullptr, 0, asrx::g_row_nofill ? 1 : 0};
  const size_t shm = next_i ? (size_t)((rows + p.L - 1) / p.L) * sizeof(float) : 0;  // next_i copy
  ASRX_REQUIRE(shm <= 48 * 1024, "msheath_row_fwd: %ld samples exceed the next_i LDS copy", (long)(shm / 4));
  MS_DISPATCH(msheath_row_fwd_kernel, row_grid(rows), shm, p);
  ASRX_LAUNCHED("asrx_msheath_row_fwd");
}

// asrx_msheath_row_fwd2 for a layer without adapter (px fp32, the update itself) that also does
// asrx_axpy_row2_colsum's work: x_new = x + g ion px into xnew (when non-null) and the per-sample 64-row chunk
// column sums into part (B x asrx_mem_chunks(L) x d) -- one launch and one pass over x and px fewer per layer.
int asrx_msheath_row_fwd3(const float* x, const float* lnw, const float* lnb, const float* gw, const float* gb,
                          const float* SH, int64_t ldsh, const float* mval, const float* w2, const float* b2,
                          const float* cw, const float* cb, const float* tx, float* px, float* mean, float* rstd,
                          float* nx, float* g, float* ion, float* kv, float* m2, float* xnew, float* part, int64_t rows,
                          int64_t d, int64_t M, int64_t Dh, float eps, float inv_sqrt_d, const float* next_i,
                          int64_t layer, int64_t L, hipStream_t stream) {
  ASRX_REQUIRE(M <= 64 && ldsh >= M + Dh, "asrx_msheath_row_fwd3: M <= 64 and ldsh >= M + Dh required");
  ASRX_REQUIRE(Dh <= 64 * ((d / 64 + 1) / 2), "asrx_msheath_row_fwd3: v_gate hidden size Dh <= d / 2 required");
  ASRX_REQUIRE(ms_aligned({x, lnw, lnb, gw, (const float*)px, (const float*)xnew, (const float*)part}),
               "asrx_msheath_row_fwd3: 8-byte aligned rows required");
  ASRX_REQUIRE(part && L > 0 && rows % L == 0, "asrx_msheath_row_fwd3: part and rows = B L required");
  if (rows == 0) return 0;
  MSRowFwd p{x, lnw, lnb, gw, gb, SH, mval, w2, b2, cw, cb, tx, px, mean, rstd, nx, g, ion, kv, m2, rows, ldsh,
             (int)M, (int)Dh, eps, inv_sqrt_d, next_i, (int)layer, L, nullptr, part, xnew, (int)((L + 63) / 64),
             asrx::g_row_nofill ? 1 : 0};
  // next_i copy, then the RW waves' column sums of a chunk
  const size_t shm = (next_i ? (size_t)((rows / L + 3) & ~(int64_t)3) : 0) * sizeof(float) + (size_t)RW * d * sizeof(float);
  ASRX_REQUIRE(shm <= 48 * 1024, "msheath_row_fwd3: %ld samples exceed the next_i LDS copy", (long)(rows / L));
  const int64_t chunks = (rows / L) * p.nchunk;
  MS_DISPATCH(msheath_row_fwd_kernel, (unsigned)std::min<int64_t>(chunks, 65535), shm, p);
  ASRX_LAUNCHED("asrx_msheath_row_fwd3");
}

int asrx_msheath_row_fwd(const float* x, const float* lnw, const float* lnb, const float* gw, const float* gb,
                         const float* SH, int64_t ldsh, const float* mval, const float* w2, const float* b2,
                         const float* cw, const float* cb, const float* tx, float* px, float* mean, float* rstd,
                         float* nx, float* g, float* ion, float* kv, float* m2, int64_t rows, int64_t d, int64_t M,
                         int64_t Dh, float eps, float inv_sqrt_d, const float* next_i, int64_t layer, int64_t L,
                         hipStream_t stream) {
  return asrx_msheath_row_fwd2(x, lnw, lnb, gw, gb, SH, ldsh, mval, w2, b2, cw, cb, tx, px, 0, mean, rstd, nx, g, ion,
                               kv, m2, rows, d, M, Dh, eps, inv_sqrt_d, next_i, layer, L, stream);
}

// Its backward (msheath_row_bwd_kernel).  dx is accumulated; every parameter gradient is accumulated
// (atomics); dSH (stride ldsh) is written.
int asrx_msheath_row_bwd(const float* dpx, const float* x, const float* lnw, const float* lnb, const float* mean,
                         const float* rstd, const float* dg, const float* g, const float* gw, const float* dion,
                         const float* SH, int64_t ldsh, const float* nx, const float* mval, const float* w2,
                         const float* cw, const float* kv, const float* m2, float* dx, float* dlnw, float* dlnb,
                         float* dgw, float* dgb, float* dSH, float* dmval, float* dw2, float* db2, float* dcw,
                         float* dcb, float* db1, int64_t rows, int64_t d, int64_t M, int64_t Dh, float inv_sqrt_d,
                         const float* next_i, int64_t layer, int64_t L, hipStream_t stream) {
  ASRX_REQUIRE(M <= 64 && ldsh >= M + Dh, "asrx_msheath_row_bwd: M <= 64 and ldsh >= M + Dh required");
  ASRX_REQUIRE(Dh <= 64 * ((d / 64 + 1) / 2), "asrx_msheath_row_bwd: v_gate hidden size Dh <= d / 2 required");
  ASRX_REQUIRE(ms_aligned({dpx, x, lnw, lnb, gw, dx}), "asrx_msheath_row_bwd: 8-byte aligned rows required");
  ASRX_REQUIRE(!next_i || L > 0, "asrx_msheath_row_bwd: L > 0 required with next_i");
  if (rows == 0) return 0;
  MSRowBwd p{dpx, x, lnw, lnb, mean, rstd, dg, g, gw, dion, SH, nx, mval, w2, cw, kv, m2, dx, dlnw, dlnb, dgw, dgb,
             dSH, dmval, dw2, db2, dcw, dcb, db1, rows, ldsh, (int)M, (int)Dh, inv_sqrt_d, next_i, (int)layer,
             L > 0 ? L : 1};
  const size_t nb = next_i ? (size_t)((rows + p.L - 1) / p.L) : 0;  // + the next_i copy
  const size_t shm = ((size_t)RW * (3 * d + M + 2 * Dh + 5) + nb) * sizeof(float);
  ASRX_REQUIRE(shm <= 160 * 1024, "msheath_row_bwd: %ld samples exceed the LDS budget", (long)nb);
  MS_DISPATCH(msheath_row_bwd_kernel, row_grid(rows, 1024), shm, p);
  ASRX_LAUNCHED("asrx_msheath_row_bwd");
}
#undef MS_DISPATCH

int asrx_tgate_fwd2(const float* G, const float* c, void* out, int out_bf16, int64_t rows, int64_t D,
                    hipStream_t stream) {
  if (rows == 0) return 0;
  if (out_bf16)
    LAUNCH_ROWS(tgate_fwd_kernel<unsigned short>, rows, 0, G, c, (unsigned short*)out, rows, (int)D);
  else
    LAUNCH_ROWS(tgate_fwd_kernel<float>, rows, 0, G, c, (float*)out, rows, (int)D);
  ASRX_LAUNCHED("asrx_tgate_fwd");
}

int asrx_tgate_fwd(const float* G, const float* c, float* out, int64_t rows, int64_t D, hipStream_t stream) {
  return asrx_tgate_fwd2(G, c, out, 0, rows, D, stream);
}

int asrx_tgate_bwd(const float* dout, const float* G, const float* c, float* dGz, float* dc, int64_t rows, int64_t D,
                   hipStream_t stream) {
  if (rows == 0) return 0;
  LAUNCH_ROWS(tgate_bwd_kernel, rows, 0, dout, G, c, dGz, dc, rows, (int)D);
  ASRX_LAUNCHED("asrx_tgate_bwd");
}

int asrx_axpy_row(const float* x, const float* s, const float* y, float* out, int64_t rows, int64_t d,
                  hipStream_t stream) {
  if (rows == 0) return 0;
  if (d % 4 == 0 && rows * d / 4 < (1LL << 31) &&
      ((((uintptr_t)x | (uintptr_t)y | (uintptr_t)out) & 15) == 0)) {
    const int64_t n4 = rows * d / 4;
    axpy_row4_kernel<<<ew_grid((n4 + 1) / 2, 8192), 256, 0, stream>>>((const float4*)x, s, (const float4*)y,
                                                                      (float4*)out, (uint32_t)n4, (uint32_t)(d / 4));
  } else {
    LAUNCH_EW(axpy_row_kernel, rows * d, x, s, y, out, rows, (int)d);
  }
  ASRX_LAUNCHED("asrx_axpy_row");
}

int asrx_axpy_row_bwd(const float* g, const float* s, const float* y, float* dy, float* ds, int64_t rows, int64_t d,
                      hipStream_t stream) {
  if (rows == 0) return 0;
  LAUNCH_ROWS(axpy_row_bwd_kernel, rows, 0, g, s, y, dy, ds, rows, (int)d, (float*)nullptr);
  ASRX_LAUNCHED("asrx_axpy_row_bwd");
}

int asrx_axpy_row_bwd2(const float* g, const float* s, const float* y, float* dy, float* ds, float* dxc, int64_t rows,
                       int64_t d, hipStream_t stream) {
  if (rows == 0) return 0;
  LAUNCH_ROWS(axpy_row_bwd_kernel, rows, 0, g, s, y, dy, ds, rows, (int)d, dxc);
  ASRX_LAUNCHED("asrx_axpy_row_bwd2");
}

int asrx_jump_select(const float* xn, const float* orig, const float* xold, const float* act, const float* alpha,
                     const float* beta, const float* gam, float* out, int64_t B, int64_t L, int64_t d,
                     hipStream_t stream) {
  if (B * L == 0) return 0;
  LAUNCH_EW(jump_select_kernel, B * L * d, xn, orig, xold, act, alpha, beta, gam, out, B, L, (int)d);
  ASRX_LAUNCHED("asrx_jump_select");
}

int asrx_jump_select_bwd(const float* g, const float* xn, const float* orig, const float* act, const float* alpha,
                         const float* beta, float* dxn, float* dorig, float* dxold, float* dalpha, float* dbeta,
                         float* dgam, int64_t B, int64_t L, int64_t d, hipStream_t stream) {
  if (B * L == 0) return 0;
  dim3 grid((unsigned)((d + 63) / 64), (unsigned)B);
  jump_select_bwd_kernel<<<grid, 256, 0, stream>>>(g, xn, orig, act, alpha, beta, dxn, dorig, dxold, dalpha, dbeta,
                                                   dgam, L, (int)d);
  ASRX_LAUNCHED("asrx_jump_select_bwd");
}

int asrx_seg_colsum(const float* x, float* out, int64_t B, int64_t L, int64_t d, float scale, int accumulate,
                    hipStream_t stream) {
  if (B == 0) return 0;
  if (!accumulate) (void)hipMemsetAsync(out, 0, (size_t)B * d * sizeof(float), stream);
  const int64_t chunk = 64;
  dim3 grid((unsigned)((d + 63) / 64), (unsigned)B, (unsigned)((L + chunk - 1) / chunk));
  seg_colsum_kernel<<<grid, 256, 0, stream>>>(x, out, L, (int)d, scale, chunk);
  ASRX_LAUNCHED("asrx_seg_colsum");
}

// out (B, d) = scale * sum_l x[b, l, :], deterministic; part: B * ceil(L / 64) * d floats of workspace.
int asrx_seg_colsum_det(const float* x, float* part, float* out, int64_t B, int64_t L, int64_t d, float scale,
                        hipStream_t stream) {
  if (B == 0) return 0;
  const int64_t chunk = 64, nchunk = (L + chunk - 1) / chunk;
  dim3 grid((unsigned)((d + 63) / 64), (unsigned)B, (unsigned)nchunk);
  seg_partial_kernel<<<grid, 256, 0, stream>>>(x, part, L, (int)d, chunk);
  seg_reduce_kernel<<<(unsigned)((B * d + 255) / 256), 256, 0, stream>>>(part, out, (int)B, (int)nchunk, (int)d, scale);
  ASRX_LAUNCHED("asrx_seg_colsum_det");
}

int asrx_colsum(const float* x, float* out, int64_t rows, int64_t d, hipStream_t stream) {
  if (rows == 0) return 0;
  int64_t chunks = std::min<int64_t>(std::max<int64_t>(rows / 512, 1), 1024);
  const int64_t chunk = (rows + chunks - 1) / chunks;
  chunks = (rows + chunk - 1) / chunk;
  dim3 grid((unsigned)((d + 63) / 64), (unsigned)chunks);
  colsum_kernel<<<grid, 256, 0, stream>>>(x, out, rows, (int)d, chunk, d);
  ASRX_LAUNCHED("asrx_colsum");
}

// out[c] += sum_r x[r * ld + c]: the bias gradient of a column block of a wider GEMM output
int asrx_colsum_ld(const float* x, int64_t ld, float* out, int64_t rows, int64_t d, hipStream_t stream) {
  if (rows == 0) return 0;
  int64_t chunks = std::min<int64_t>(std::max<int64_t>(rows / 512, 1), 1024);
  const int64_t chunk = (rows + chunks - 1) / chunks;
  chunks = (rows + chunk - 1) / chunk;
  dim3 grid((unsigned)((d + 63) / 64), (unsigned)chunks);
  colsum_kernel<<<grid, 256, 0, stream>>>(x, out, rows, (int)d, chunk, ld);
  ASRX_LAUNCHED("asrx_colsum_ld");
}

int asrx_add_rows(const float* x, const float* t, const float* u, float* out, int64_t B, int64_t L, int64_t d,
                  hipStream_t stream) {
  if (B * L * d == 0) return 0;
  const int64_t n = B * L * d;
  if (d % 4 == 0 && n / 4 < (1LL << 31) &&
      ((((uintptr_t)x | (uintptr_t)t | (uintptr_t)u | (uintptr_t)out) & 15) == 0)) {
    const int64_t n4 = n / 4;
    add_rows4_kernel<<<ew_grid((n4 + 1) / 2, 8192), 256, 0, stream>>>((const float4*)x, (const float4*)t,
                                                                      (const float4*)u, (float4*)out, (uint32_t)n4,
                                                                      (uint32_t)L, (uint32_t)(d / 4));
  } else {
    LAUNCH_EW(add_rows_kernel, B * L * d, x, t, u, out, B, L, (int)d);
  }
  ASRX_LAUNCHED("asrx_add_rows");
}

int asrx_lincomb(const float* x, const float* y, const float* z, float a, float b, float c, float* out, int64_t n,
                 hipStream_t stream) {
  if (n == 0) return 0;
  if (n % 4 == 0 && n / 4 < (1LL << 31) && ((((uintptr_t)x | (uintptr_t)y | (uintptr_t)z | (uintptr_t)out) & 15) == 0)) {
    const int64_t n4 = n / 4;
    lincomb4_kernel<<<ew_grid((n4 + 1) / 2, 8192), 256, 0, stream>>>((const float4*)x, (const float4*)y,
                                                                     (const float4*)z, a, b, c, (float4*)out,
                                                                     (uint32_t)n4);
  } else {
    LAUNCH_EW(lincomb_kernel, n, x, y, z, a, b, c, out, n);
  }
  ASRX_LAUNCHED("asrx_lincomb");
}

int asrx_act_fwd(const float* x, float* y, int64_t n, int act, hipStream_t stream) {
  if (n == 0) return 0;
  if (n % 4 == 0 && n / 4 < (1LL << 31) && ((((uintptr_t)x | (uintptr_t)y) & 15) == 0)) {
    const int64_t n4 = n / 4;
    act_fwd4_kernel<<<ew_grid((n4 + 1) / 2, 8192), 256, 0, stream>>>((const float4*)x, (float4*)y, (uint32_t)n4, act);
  } else {
    LAUNCH_EW(act_fwd_kernel, n, x, y, n, act);
  }
  ASRX_LAUNCHED("asrx_act_fwd");
}

int asrx_act_bwd(const float* g, const float* x, float* dx, int64_t n, int act, hipStream_t stream) {
  if (n == 0) return 0;
  if (n % 4 == 0 && n / 4 < (1LL << 31) && ((((uintptr_t)g | (uintptr_t)x | (uintptr_t)dx) & 15) == 0)) {
    const int64_t n4 = n / 4;
    act_bwd4_kernel<<<ew_grid((n4 + 1) / 2, 8192), 256, 0, stream>>>((const float4*)g, (const float4*)x, (float4*)dx,
                                                                     (uint32_t)n4, act);
  } else {
    LAUNCH_EW(act_bwd_kernel, n, g, x, dx, n, act);
  }
  ASRX_LAUNCHED("asrx_act_bwd");
}

int asrx_act_bwd_bias(const float* g, const float* z, unsigned short* gz, float* db, int64_t rows, int64_t N, int act,
                      hipStream_t stream) {
  ASRX_REQUIRE(N % 4 == 0 && (((uintptr_t)g | (uintptr_t)z) & 15) == 0 && ((uintptr_t)gz & 7) == 0,
               "asrx_act_bwd_bias: N %% 4 == 0 and aligned rows required");
  ASRX_REQUIRE(act == ACT_GELU || act == ACT_SILU || act == ACT_SIGMOID, "asrx_act_bwd_bias: gelu/silu/sigmoid only");
  if (rows == 0) return 0;
  const int gx = (int)((N / 4 + 63) / 64);
  int64_t chunks = std::max<int64_t>(1, std::min<int64_t>((rows + 63) / 64, 2048 / gx));
  const int64_t chunk = (rows + chunks - 1) / chunks;
  chunks = (rows + chunk - 1) / chunk;
  const dim3 grid((unsigned)gx, (unsigned)chunks);
  if (act == ACT_GELU) act_bwd_bias_kernel<ACT_GELU><<<grid, 256, 0, stream>>>(g, z, gz, db, rows, (int)N, chunk);
  else if (act == ACT_SILU) act_bwd_bias_kernel<ACT_SILU><<<grid, 256, 0, stream>>>(g, z, gz, db, rows, (int)N, chunk);
  else act_bwd_bias_kernel<ACT_SIGMOID><<<grid, 256, 0, stream>>>(g, z, gz, db, rows, (int)N, chunk);
  ASRX_LAUNCHED("asrx_act_bwd_bias");
}

int asrx_glu_fwd(const float* x, float* y, int64_t rows, int64_t C, hipStream_t stream) {
  if (rows == 0) return 0;
  LAUNCH_EW(glu_fwd_kernel, rows * C, x, y, rows, (int)C);
  ASRX_LAUNCHED("asrx_glu_fwd");
}

int asrx_glu_bwd(const float* g, const float* x, float* dx, int64_t rows, int64_t C, hipStream_t stream) {
  if (rows == 0) return 0;
  LAUNCH_EW(glu_bwd_kernel, rows * C, g, x, dx, rows, (int)C);
  ASRX_LAUNCHED("asrx_glu_bwd");
}

static bool act_dropout_vec_ok(const void* a, const void* b, const void* c, int64_t n, int64_t C) {
  return C % 4 == 0 && ((((uintptr_t)a | (uintptr_t)b | (uintptr_t)c) & 15) == 0) && n / 4 < (1LL << 32);
}

int asrx_dropout(const float* x, float* y, int64_t B, int64_t T, int64_t C, int64_t sid_base, uint32_t key, float p,
                 hipStream_t stream) {
  const int64_t n = B * T * C;
  if (n == 0) return 0;
  if (act_dropout_vec_ok(x, y, nullptr, n, C))
    LAUNCH_EW(act_dropout4_kernel<false>, n / 4, nullptr, reinterpret_cast<const float4*>(x), nullptr,
              reinterpret_cast<float4*>(y), (uint32_t)(n / 4), (uint32_t)(C / 4), (uint32_t)T, (uint32_t)C,
              (uint32_t)sid_base, key, p, (int)ACT_NONE, (int)ACT_NONE);
  else
    LAUNCH_EW(dropout_kernel, n, x, y, B, T, (int)C, sid_base, key, p);
  ASRX_LAUNCHED("asrx_dropout");
}

int asrx_act_dropout_fwd(const float* z, const float* res, float* y, int64_t B, int64_t T, int64_t C,
                         int64_t sid_base, uint32_t key, float p, int act, int act2, hipStream_t stream) {
  const int64_t n = B * T * C;
  if (n == 0) return 0;
  ASRX_REQUIRE(act_dropout_vec_ok(z, y, res, n, C), "act_dropout: needs C %% 4 == 0 and 16-byte aligned tensors");
  LAUNCH_EW(act_dropout4_kernel<false>, n / 4, nullptr, reinterpret_cast<const float4*>(z),
            reinterpret_cast<const float4*>(res), reinterpret_cast<float4*>(y), (uint32_t)(n / 4), (uint32_t)(C / 4), (uint32_t)T, (uint32_t)C,
            (uint32_t)sid_base, key, p, act, act2);
  ASRX_LAUNCHED("asrx_act_dropout_fwd");
}

int asrx_act_dropout_bwd(const float* g, const float* z, float* dz, int64_t B, int64_t T, int64_t C,
                         int64_t sid_base, uint32_t key, float p, int act, int act2, hipStream_t stream) {
  const int64_t n = B * T * C;
  if (n == 0) return 0;
  ASRX_REQUIRE(act_dropout_vec_ok(g, z, dz, n, C), "act_dropout: needs C %% 4 == 0 and 16-byte aligned tensors");
  LAUNCH_EW(act_dropout4_kernel<true>, n / 4, reinterpret_cast<const float4*>(g), reinterpret_cast<const float4*>(z),
            nullptr, reinterpret_cast<float4*>(dz), (uint32_t)(n / 4), (uint32_t)(C / 4), (uint32_t)T, (uint32_t)C,
            (uint32_t)sid_base, key, p, act, act2);
  ASRX_LAUNCHED("asrx_act_dropout_bwd");
}

int asrx_dwconv_fwd(const float* x, const float* w, const float* b, float* y, int64_t B, int64_t T, int64_t C,
                    int64_t K, hipStream_t stream) {
  ASRX_REQUIRE(K % 2 == 1 && K <= 16, "dwconv: K must be odd and <= 15");
  if (B * T == 0) return 0;
  if (!dwconv_dispatch(x, w, b, y, nullptr, nullptr, nullptr, nullptr, B, T, C, K, stream))
    LAUNCH_EW(dwconv_fwd_kernel, B * T * C, x, w, b, y, B, T, (int)C, (int)K);
  ASRX_LAUNCHED("asrx_dwconv_fwd");
}

int asrx_dwconv_bwd(const float* g, const float* x, const float* w, float* dx, float* dw, float* db, int64_t B,
                    int64_t T, int64_t C, int64_t K, hipStream_t stream) {
  if (B * T == 0) return 0;
  if (dwconv_dispatch(x, w, nullptr, nullptr, g, dx, dw, db, B, T, C, K, stream)) ASRX_LAUNCHED("asrx_dwconv_bwd");
  if (dx) LAUNCH_EW(dwconv_bwd_data_kernel, B * T * C, g, w, dx, B, T, (int)C, (int)K);
  const int64_t chunk = 256;
  const int64_t nch = (T + chunk - 1) / chunk;
  dim3 grid((unsigned)((C + 63) / 64), (unsigned)(B * nch));
  dwconv_bwd_w_kernel<<<grid, 256, 0, stream>>>(g, x, dw, db, B, T, (int)C, (int)K, chunk);
  ASRX_LAUNCHED("asrx_dwconv_bwd");
}

int asrx_bn_fwd(const float* x, const float* w, const float* b, float* y, float* mean, float* rstd, int64_t B,
                int64_t T, int64_t C, float eps, int use_batch_stats, hipStream_t stream) {
  if (B * T == 0) return 0;
  if (use_batch_stats) {
    if (C % 4 == 0 && ((uintptr_t)x & 15) == 0) {
      const int C4 = (int)(C / 4);
      bn_stats4_kernel<<<(unsigned)(B * ((C4 + 31) / 32)), 1024, 0, stream>>>((const float4*)x, mean, rstd, (int)T,
                                                                             C4, eps);
    } else {
      dim3 grid((unsigned)((C + 63) / 64), (unsigned)B);
      bn_stats_kernel<<<grid, 256, 0, stream>>>(x, mean, rstd, T, (int)C, eps);
    }
  }
  LAUNCH_EW(bn_apply_kernel, B * T * C, x, mean, rstd, w, b, y, B, T, (int)C, use_batch_stats);
  ASRX_LAUNCHED("asrx_bn_fwd");
}

int asrx_bn_bwd(const float* g, const float* x, const float* mean, const float* rstd, const float* w, float* sg_ws,
                float* sgx_ws, float* dx, float* dw, float* db, int64_t B, int64_t T, int64_t C, hipStream_t stream) {
  if (B * T == 0) return 0;
  if (C % 4 == 0 && ((uintptr_t)x & 15) == 0 && ((uintptr_t)g & 15) == 0 && ((uintptr_t)mean & 15) == 0 &&
      ((uintptr_t)rstd & 15) == 0) {
    const int C4 = (int)(C / 4);
    bn_bwd_stats4_kernel<<<(unsigned)(B * ((C4 + 31) / 32)), 1024, 0, stream>>>(
        (const float4*)g, (const float4*)x, mean, rstd, w, sg_ws, sgx_ws, dw, db, (int)T, C4);
  } else {
    dim3 grid((unsigned)((C + 63) / 64), (unsigned)B);
    bn_bwd_stats_kernel<<<grid, 256, 0, stream>>>(g, x, mean, rstd, w, sg_ws, sgx_ws, dw, db, T, (int)C);
  }
  LAUNCH_EW(bn_bwd_apply_kernel, B * T * C, g, x, mean, rstd, w, sg_ws, sgx_ws, dx, B, T, (int)C);
  ASRX_LAUNCHED("asrx_bn_bwd");
}

int asrx_stem1_fwd(const float* x, const float* W, const float* bias, float* y, int64_t B, int64_t T, int64_t D,
                   hipStream_t stream) {
  if (B * T == 0) return 0;
  LAUNCH_EW(stem1_fwd_kernel, B * T * D, x, W, bias, y, B, T, (int)D);
  ASRX_LAUNCHED("asrx_stem1_fwd");
}

int asrx_stem1_bwd(const float* g, const float* x, float* dW, float* db, int64_t B, int64_t T, int64_t D,
                   hipStream_t stream) {
  if (B * T == 0) return 0;
  const int64_t chunk = 256, nch = (T + chunk - 1) / chunk;
  dim3 grid((unsigned)((D + 63) / 64), (unsigned)(B * nch));
  stem1_bwd_w_kernel<<<grid, 256, 0, stream>>>(g, x, dW, db, B, T, (int)D, chunk);
  ASRX_LAUNCHED("asrx_stem1_bwd");
}

int asrx_embed_fwd(const int64_t* ids, const float* E, float* y, int64_t rows, int64_t d, hipStream_t stream) {
  if (rows == 0) return 0;
  LAUNCH_EW(embed_fwd_kernel, rows * d, ids, E, y, rows, (int)d);
  ASRX_LAUNCHED("asrx_embed_fwd");
}

int asrx_embed_bwd(const int64_t* ids, const float* g, float* dE, int64_t rows, int64_t d, hipStream_t stream) {
  if (rows == 0) return 0;
  LAUNCH_EW(embed_bwd_kernel, rows * d, ids, g, dE, rows, (int)d);
  ASRX_LAUNCHED("asrx_embed_bwd");
}

int asrx_ce_fwd(const float* z, const int64_t* labels, float* loss, float* lse, int64_t rows, int64_t V,
                hipStream_t stream) {
  if (rows == 0) return 0;
  ASRX_REQUIRE(rows < (1LL << 31), "ce: too many rows");
  ce_fwd_kernel<<<(unsigned)rows, 256, 0, stream>>>(z, labels, loss, lse, V);
  ASRX_LAUNCHED("asrx_ce_fwd");
}

int asrx_ce_bwd(const float* z, const int64_t* labels, const float* lse, const float* scale, float* dz, int64_t rows,
                int64_t V, hipStream_t stream) {
  if (rows == 0) return 0;
  ce_bwd_kernel<<<(unsigned)rows, 256, 0, stream>>>(z, labels, lse, scale, dz, V);
  ASRX_LAUNCHED("asrx_ce_bwd");
}

}  // extern "C"

// MSheath policy gumbel noise (model.py:476): out[b, i, k] = gumbel(key, ((sid_base + b)*64 + i)*3 + k)
namespace asrx {
__global__ void policy_noise_kernel(float* out, int64_t B, int64_t layers, int64_t sid_base, uint32_t key) {
  const int64_t n = B * layers * 3;
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (int64_t)gridDim.x * blockDim.x) {
    const int64_t k = j % 3, i = (j / 3) % layers, b = j / (3 * layers);
    out[j] = noise_gumbel(key, (uint32_t)(((sid_base + b) * 64 + i) * 3 + k));
  }
}
}  // namespace asrx
extern "C" int asrx_policy_noise(float* out, int64_t B, int64_t layers, int64_t sid_base, uint32_t key,
                                 hipStream_t stream) {
  ASRX_REQUIRE(layers <= 64, "policy noise: at most 64 layers");
  if (B * layers == 0) return 0;
  asrx::policy_noise_kernel<<<(unsigned)((B * layers * 3 + 255) / 256), 256, 0, stream>>>(out, B, layers, sid_base, key);
  ASRX_LAUNCHED("asrx_policy_noise");
}

ASRX_NOISE_EPOCH_SETTER(asrx_set_noise_epoch_rowops)
