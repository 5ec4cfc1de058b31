// AbbyNormal (essentials.py:140-191, n_type="AbbyNormal", confidence=None), fused per row:
//
//   logits = Linear(d,3)(SiLU(h_pre)),  h_pre = Linear(d,d)(x)      (the d x d GEMM runs before)
//   cv     = std(x, unbiased) / (mean|x| + 1e-6)
//   dec    = gumbel_softmax(logits + cv, tau=1, hard=True)          (straight-through)
//   avg/max = avg_pool1d / max_pool1d of x^2 along the feature axis, window w = odd(max(3,
//            int(0.05 d))), zero padding w/2 (count_include_pad) / -inf padding
//   div    = dec0*avg + dec1*(max > 2 avg ? max : avg) + dec2*avg
//   out    = x / (1 + 1e-4 div)^0.75
//
// One wave per row (d % 64 == 0, d <= 1024); x^2 is staged in LDS for the windowed pools.
// Noise: gumbel g_k = -log(-log(u)) with u = noise_uniform(key, ((sid*H + h)*4096 + l)*3 + k); the
// row r (kernel order: sample-major, then position, then head) maps to sid = sid_base + r/(L*H),
// l = (r % (L*H)) / H, h = r % H.
//
// Backward (same kernel family) returns dx (direct + pooling + cv paths), dh_pre (rows x d) and
// accumulates dW2 (3 x d) / db2 (3) with one atomic per element per workgroup; the host adds
// dh_pre @ W1 into dx and computes dW1 / db1 with the GEMM.
#include "common.h"

namespace asrx {

constexpr int ABBY_WAVES = 4;
constexpr int ABBY_MAXE = 16;  // d <= 1024

struct AbbyGeom {
  int64_t rows, d;
  int64_t L, H;
  int64_t sid_base;
  uint32_t key;
  int use_noise;
};

__device__ __forceinline__ int abby_window(int d) {
  int w = (int)(d * 0.05f);
  if (w < 3) w = 3;
  if ((w & 1) == 0) w += 1;
  return w;
}

__device__ __forceinline__ uint32_t abby_noise_idx(const AbbyGeom& g, int64_t r, int k) {
  const int64_t per = g.L * g.H;
  const int64_t sid = g.sid_base + r / per;
  const int64_t q = r % per;
  const int64_t l = q / g.H, h = q % g.H;
  return (uint32_t)(((sid * g.H + h) * 4096 + l) * 3 + k);
}

// Row statistics shared by fwd and bwd.
template <int E>
__device__ __forceinline__ void abby_row_stats(const float (&xv)[ABBY_MAXE], int d, float& mu, float& sd,
                                               float& mabs) {
  float s = 0.f, sa = 0.f;
#pragma unroll
  for (int e = 0; e < E; ++e) {
    s += xv[e];
    sa += fabsf(xv[e]);
  }
  s = wave_sum(s);
  sa = wave_sum(sa);
  mu = s / d;
  mabs = sa / d;
  float v = 0.f;
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const float t = xv[e] - mu;
    v += t * t;
  }
  v = wave_sum(v);
  sd = sqrtf(v / (d - 1));
}

// avg / max pool of sq (LDS row) at element j.  Returns avg, max and the argmax index (first max).
__device__ __forceinline__ void abby_pool(const float* sq, int d, int w, int j, float& avg, float& mx,
                                          int& amax) {
  const int pad = w >> 1;
  float s = 0.f, m = -INFINITY;
  int am = j;
  const int lo = j - pad, hi = j + pad;
  for (int i = lo; i <= hi; ++i) {
    if (i < 0 || i >= d) continue;
    const float v = sq[i];
    s += v;
    if (v > m) {
      m = v;
      am = i;
    }
  }
  avg = s / (float)w;
  mx = m;
  amax = am;
}

template <int E>
__global__ __launch_bounds__(64 * ABBY_WAVES) void abby_fwd_kernel(const float* __restrict__ x,
                                                                  const float* __restrict__ hpre,
                                                                  const float* __restrict__ W2,
                                                                  const float* __restrict__ b2,
                                                                  float* __restrict__ out, float* __restrict__ ys,
                                                                  int* __restrict__ idx_out, AbbyGeom g,
                                                                  const float* __restrict__ logits) {
  __shared__ float sq_all[ABBY_WAVES][64 * ABBY_MAXE];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  float* sq = sq_all[wid];
  const int d = (int)g.d;
  const int w = abby_window(d);
  for (int64_t r = (int64_t)blockIdx.x * ABBY_WAVES + wid; r < g.rows; r += (int64_t)gridDim.x * ABBY_WAVES) {
    const float* xr = x + r * d;
    float xv[ABBY_MAXE];
    float l0 = 0.f, l1 = 0.f, l2 = 0.f;
    if (logits) {  // router logits from the GEMM epilogue (asrx_gemm_wn_router)
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const int j = e * 64 + lane;
        xv[e] = xr[j];
        sq[j] = xv[e] * xv[e];
      }
      l0 = logits[r * 3 + 0];
      l1 = logits[r * 3 + 1];
      l2 = logits[r * 3 + 2];
    } else {
      const float* hr = hpre + r * d;
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const int j = e * 64 + lane;
        xv[e] = xr[j];
        const float hs = silu_f(hr[j]);
        l0 += hs * W2[j];
        l1 += hs * W2[d + j];
        l2 += hs * W2[2 * d + j];
        sq[j] = xv[e] * xv[e];
      }
      l0 = wave_sum(l0);
      l1 = wave_sum(l1);
      l2 = wave_sum(l2);
    }
    float mu, sd, mabs;
    abby_row_stats<E>(xv, d, mu, sd, mabs);
    const float cv = sd / (mabs + 1e-6f);
    float z0 = l0 + b2[0] + cv, z1 = l1 + b2[1] + cv, z2 = l2 + b2[2] + cv;
    if (g.use_noise) {
      z0 += noise_gumbel(g.key, abby_noise_idx(g, r, 0));
      z1 += noise_gumbel(g.key, abby_noise_idx(g, r, 1));
      z2 += noise_gumbel(g.key, abby_noise_idx(g, r, 2));
    }
    const float zm = fmaxf(z0, fmaxf(z1, z2));
    const float e0 = expf(z0 - zm), e1 = expf(z1 - zm), e2 = expf(z2 - zm);
    const float inv = 1.0f / (e0 + e1 + e2);
    const float y0 = e0 * inv, y1 = e1 * inv, y2 = e2 * inv;
    int sel = 0;
    float ym = y0;
    if (y1 > ym) {
      sel = 1;
      ym = y1;
    }
    if (y2 > ym) sel = 2;
    if (lane == 0) {
      ys[r * 3 + 0] = y0;
      ys[r * 3 + 1] = y1;
      ys[r * 3 + 2] = y2;
      idx_out[r] = sel;
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    float* o = out + r * d;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int j = e * 64 + lane;
      float avg, mx;
      int am;
      abby_pool(sq, d, w, j, avg, mx, am);
      const float div = (sel == 1 && mx > 2.0f * avg) ? mx : avg;
      const float denom = powf(div * 1e-4f + 1.0f, 0.75f);
      o[j] = xv[e] / denom;
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  }
}

template <int E>
__global__ __launch_bounds__(64 * ABBY_WAVES) void abby_bwd_kernel(
    const float* __restrict__ dout, const float* __restrict__ x, const float* __restrict__ hpre,
    const float* __restrict__ W2, const float* __restrict__ ys, const int* __restrict__ idx_in,
    float* __restrict__ dx, float* __restrict__ dhpre, float* __restrict__ dW2, float* __restrict__ db2,
    AbbyGeom g) {
  __shared__ float sq_all[ABBY_WAVES][64 * ABBY_MAXE];
  __shared__ float cA_all[ABBY_WAVES][64 * ABBY_MAXE];  // q_j * coefA_j / w
  __shared__ float cM_all[ABBY_WAVES][64 * ABBY_MAXE];  // q_j * coefM_j
  __shared__ int am_all[ABBY_WAVES][64 * ABBY_MAXE];
  __shared__ float red[ABBY_WAVES][4];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  float* sq = sq_all[wid];
  float* cA = cA_all[wid];
  float* cM = cM_all[wid];
  int* amx = am_all[wid];
  const int d = (int)g.d;
  const int w = abby_window(d);
  float accW[3][ABBY_MAXE];
  float accb[3] = {0.f, 0.f, 0.f};
#pragma unroll
  for (int k = 0; k < 3; ++k)
#pragma unroll
    for (int e = 0; e < ABBY_MAXE; ++e) accW[k][e] = 0.f;

  for (int64_t r = (int64_t)blockIdx.x * ABBY_WAVES + wid; r < g.rows; r += (int64_t)gridDim.x * ABBY_WAVES) {
    const float* xr = x + r * d;
    const float* gr = dout + r * d;
    float xv[ABBY_MAXE], gv[ABBY_MAXE], qv[ABBY_MAXE], avgv[ABBY_MAXE], m2v[ABBY_MAXE];
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int j = e * 64 + lane;
      xv[e] = xr[j];
      gv[e] = gr[j];
      sq[j] = xv[e] * xv[e];
    }
    const int sel = idx_in[r];
    const float y0 = ys[r * 3 + 0], y1 = ys[r * 3 + 1], y2 = ys[r * 3 + 2];
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    float dd0 = 0.f, dd1 = 0.f;  // dd2 == dd0 (mode3 == mode1 == avg)
    float dxv[ABBY_MAXE];
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int j = e * 64 + lane;
      float avg, mx;
      int am;
      abby_pool(sq, d, w, j, avg, mx, am);
      const bool cnd = mx > 2.0f * avg;
      const float mode2 = cnd ? mx : avg;
      const float div = (sel == 1) ? mode2 : avg;
      const float base = div * 1e-4f + 1.0f;
      const float denom = powf(base, 0.75f);
      dxv[e] = gv[e] / denom;
      const float q = -gv[e] * xv[e] * (1e-4f * 0.75f) / (denom * base);
      qv[e] = q;
      avgv[e] = avg;
      m2v[e] = mode2;
      dd0 += q * avg;
      dd1 += q * mode2;
      float coefA, coefM;
      if (sel == 1) {
        coefA = cnd ? 0.f : 1.f;
        coefM = cnd ? 1.f : 0.f;
      } else {
        coefA = 1.f;
        coefM = 0.f;
      }
      cA[j] = q * coefA / (float)w;
      cM[j] = q * coefM;
      amx[j] = am;
    }
    dd0 = wave_sum(dd0);
    dd1 = wave_sum(dd1);
    const float dd2 = dd0;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    // pool backward (gather form): dsq_i = sum_{j in win(i)} cA_j + sum_{j in win(i), amax_j == i} cM_j
    const int pad = w >> 1;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int i = e * 64 + lane;
      float s = 0.f;
      for (int j = i - pad; j <= i + pad; ++j) {
        if (j < 0 || j >= d) continue;
        s += cA[j];
        if (amx[j] == i) s += cM[j];
      }
      dxv[e] += 2.0f * xv[e] * s;
    }
    // straight-through softmax backward
    const float dot = y0 * dd0 + y1 * dd1 + y2 * dd2;
    const float dz0 = y0 * (dd0 - dot), dz1 = y1 * (dd1 - dot), dz2 = y2 * (dd2 - dot);
    const float dcv = dz0 + dz1 + dz2;
    // cv = sd / (mabs + 1e-6)
    float mu, sd, mabs;
    abby_row_stats<E>(xv, d, mu, sd, mabs);
    const float den = mabs + 1e-6f;
    const float dsd = dcv / den;
    const float dmabs = -dcv * sd / (den * den);
    const float csd = sd > 0.f ? dsd / ((d - 1) * sd) : 0.f;
    const float cma = dmabs / d;
    const float* hr = hpre + r * d;
    float* dxo = dx + r * d;
    float* dho = dhpre + r * d;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int j = e * 64 + lane;
      const float sgn = xv[e] > 0.f ? 1.f : (xv[e] < 0.f ? -1.f : 0.f);
      dxo[j] = dxv[e] + csd * (xv[e] - mu) + cma * sgn;
      const float h = hr[j];
      const float wsum = dz0 * W2[j] + dz1 * W2[d + j] + dz2 * W2[2 * d + j];
      dho[j] = silu_grad(h) * wsum;
      const float hs = silu_f(h);
      accW[0][e] += dz0 * hs;
      accW[1][e] += dz1 * hs;
      accW[2][e] += dz2 * hs;
    }
    accb[0] += dz0;
    accb[1] += dz1;
    accb[2] += dz2;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  }
  // workgroup reduction of dW2 / db2, then one atomic per element
  __syncthreads();
  float* buf = sq_all[0];  // reuse: 3 * d floats <= 3072 < 4 * 1024
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int j = e * 64 + lane;
    if (wid == 0) {
      buf[j] = accW[0][e];
      buf[d + j] = accW[1][e];
      buf[2 * d + j] = accW[2][e];
    }
  }
  __syncthreads();
  for (int ww = 1; ww < ABBY_WAVES; ++ww) {
    if (wid == ww) {
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const int j = e * 64 + lane;
        buf[j] += accW[0][e];
        buf[d + j] += accW[1][e];
        buf[2 * d + j] += accW[2][e];
      }
    }
    __syncthreads();
  }
  for (int j = threadIdx.x; j < 3 * d; j += 64 * ABBY_WAVES) atomicAdd(dW2 + j, buf[j]);
  if (lane == 0) {
    red[wid][0] = accb[0];
    red[wid][1] = accb[1];
    red[wid][2] = accb[2];
  }
  __syncthreads();
  if (threadIdx.x < 3) {
    float s = 0.f;
    for (int ww = 0; ww < ABBY_WAVES; ++ww) s += red[ww][threadIdx.x];
    atomicAdd(db2 + threadIdx.x, s);
  }
}

}  // namespace asrx

using namespace asrx;

#define ABBY_DISPATCH(KERNEL, ...)                                                 \
  switch (E) {                                                                     \
    case 1: KERNEL<1><<<grid, 64 * ABBY_WAVES, 0, stream>>>(__VA_ARGS__); break;   \
    case 2: KERNEL<2><<<grid, 64 * ABBY_WAVES, 0, stream>>>(__VA_ARGS__); break;   \
    case 4: KERNEL<4><<<grid, 64 * ABBY_WAVES, 0, stream>>>(__VA_ARGS__); break;   \
    case 6: KERNEL<6><<<grid, 64 * ABBY_WAVES, 0, stream>>>(__VA_ARGS__); break;   \
    case 8: KERNEL<8><<<grid, 64 * ABBY_WAVES, 0, stream>>>(__VA_ARGS__); break;   \
    case 12: KERNEL<12><<<grid, 64 * ABBY_WAVES, 0, stream>>>(__VA_ARGS__); break; \
    case 16: KERNEL<16><<<grid, 64 * ABBY_WAVES, 0, stream>>>(__VA_ARGS__); break; \
    default: set_error("AbbyNormal: unsupported d=%ld", (long)d); return 2;        \
  }

static AbbyGeom make_geom(int64_t rows, int64_t d, int64_t L, int64_t H, int64_t sid_base, uint32_t key,
                          int use_noise) {
  AbbyGeom g;
  g.rows = rows;
  g.d = d;
  g.L = L > 0 ? L : 1;
  g.H = H > 0 ? H : 1;
  g.sid_base = sid_base;
  g.key = key;
  g.use_noise = use_noise;
  return g;
}

// x, hpre: (rows, d); W2 (3, d), b2 (3); out (rows, d); ys (rows, 3); idx (rows) int32.
extern "C" int asrx_abby_fwd(const float* x, const float* hpre, const float* W2, const float* b2, float* out,
                             float* ys, int* idx, int64_t rows, int64_t d, int64_t L, int64_t H,
                             int64_t sid_base, uint32_t key, int use_noise, hipStream_t stream) {
  ASRX_REQUIRE(d % 64 == 0 && d >= 64 && d <= 1024, "AbbyNormal: d=%ld must be a multiple of 64 in [64,1024]",
               (long)d);
  if (rows == 0) return 0;
  const int E = (int)(d / 64);
  AbbyGeom g = make_geom(rows, d, L, H, sid_base, key, use_noise);
  const unsigned grid = (unsigned)std::min<int64_t>((rows + ABBY_WAVES - 1) / ABBY_WAVES, 4096);
  ABBY_DISPATCH(abby_fwd_kernel, x, hpre, W2, b2, out, ys, idx, g, nullptr);
  ASRX_LAUNCHED("asrx_abby_fwd");
}

// Same, with the router logits (rows x 3, without b2) precomputed by asrx_gemm_wn_router.
extern "C" int asrx_abby_fwd_logits(const float* x, const float* logits, const float* b2, float* out, float* ys,
                                    int* idx, int64_t rows, int64_t d, int64_t L, int64_t H, int64_t sid_base,
                                    uint32_t key, int use_noise, hipStream_t stream) {
  ASRX_REQUIRE(d % 64 == 0 && d >= 64 && d <= 1024, "AbbyNormal: d=%ld must be a multiple of 64 in [64,1024]",
               (long)d);
  if (rows == 0) return 0;
  const int E = (int)(d / 64);
  AbbyGeom g = make_geom(rows, d, L, H, sid_base, key, use_noise);
  const unsigned grid = (unsigned)std::min<int64_t>((rows + ABBY_WAVES - 1) / ABBY_WAVES, 4096);
  ABBY_DISPATCH(abby_fwd_kernel, x, nullptr, nullptr, b2, out, ys, idx, g, logits);
  ASRX_LAUNCHED("asrx_abby_fwd_logits");
}

// dW2 / db2 are accumulated (caller zeroes them).  dx, dhpre are overwritten.
extern "C" int asrx_abby_bwd(const float* dout, const float* x, const float* hpre, const float* W2,
                             const float* ys, const int* idx, float* dx, float* dhpre, float* dW2, float* db2,
                             int64_t rows, int64_t d, hipStream_t stream) {
  ASRX_REQUIRE(d % 64 == 0 && d >= 64 && d <= 1024, "AbbyNormal: d=%ld must be a multiple of 64 in [64,1024]",
               (long)d);
  if (rows == 0) return 0;
  const int E = (int)(d / 64);
  AbbyGeom g = make_geom(rows, d, 1, 1, 0, 0, 0);
  const unsigned grid = (unsigned)std::min<int64_t>((rows + ABBY_WAVES - 1) / ABBY_WAVES, 1024);
  ABBY_DISPATCH(abby_bwd_kernel, dout, x, hpre, W2, ys, idx, dx, dhpre, dW2, db2, g);
  ASRX_LAUNCHED("asrx_abby_bwd");
}
