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
// One wave per row (d % 64 == 0, d <= 1024); each lane owns d/64 consecutive features and reads
// its window halo of x^2 from a padded per-wave LDS row (see AbbyShape).
// Noise: gumbel g_k = -log(-log(u)) with u = noise_uniform(key, ((sid*H + h)*8192 + l)*3 + k); the
// row r (kernel order: sample-major, then position, then head) maps to sid = sid_base + r/(L*H),
// l = (r % (L*H)) / H, h = r % H.
//
// Backward (same kernel family) returns dx (direct + pooling + cv paths), dh_pre (rows x d) and
// accumulates dW2 (3 x d) / db2 (3) with one atomic per element per workgroup; the host adds
// dh_pre @ W1 into dx and computes dW1 / db1 with the GEMM.
#include "common.h"

namespace asrx {

constexpr int ABBY_WAVES = 4;

struct AbbyGeom {
  int64_t rows, d;
  int64_t L, H;
  int64_t sid_base;
  uint32_t key;
  int use_noise;
  int acc;  // backward: dx += (one buffer collects every consumer's gradient of x)
  // decision recorder (parity tests only, null otherwise): the forward writes mode 2's per-feature
  // choice (max > 2 avg, essentials.py:176-177) of every row that picked mode 2, cond[r * d + f]
  unsigned char* cond;
  // residual input (d >= 128 forward, fp32 out): out = res + x / denom -- the block's closing residual
  // add (model.py:583 x + mlp(x) with mlp's last AbbyNormal) without a separate add pass
  const float* res;
  // row L2 norm output (optional, d >= 128 forward): ||x[r]|| for rotary's |src| (model.py:201), the
  // rows' sum of squares taken from the values already in registers instead of a second pass over x
  float* nrm;
};

// Per-row layout (MI355X design): lane l owns the E = d/64 CONSECUTIVE features [l E, l E + E), read
// and written as float2; a wave reads the 2 PAD neighbours its windows need (the halo) from a
// per-wave LDS row of x^2 padded with PAD entries of -1 on both sides (-inf for the max pool, 0
// for the zero-padded avg pool after fmax(.,0)).  Window sums are running sums and window maxima
// a register scan, so the pools cost O(E + W) per lane instead of W LDS reads per feature.
template <int E>
struct AbbyShape {
  static constexpr int D = 64 * E;
  static constexpr int W0 = (int)(D * 0.05f);
  static constexpr int W = ((W0 < 3 ? 3 : W0) % 2 == 0) ? (W0 < 3 ? 3 : W0) + 1 : (W0 < 3 ? 3 : W0);
  static constexpr int PAD = W / 2;
  static constexpr int HL = E + 2 * PAD;      // halo length per lane
  static constexpr int ROW = D + 2 * PAD + 2;  // padded LDS row (even, so lane bases stay 8-byte aligned)
};

__device__ __forceinline__ uint32_t abby_noise_idx(const AbbyGeom& g, int64_t r, int k) {
  // 32-bit index arithmetic (rows < 2^32; the index is taken mod 2^32 either way): the 64-bit
  // divisions cost ~3x the instructions
  const uint32_t per = (uint32_t)(g.L * g.H), H = (uint32_t)g.H, rr = (uint32_t)r;
  const uint32_t sid = (uint32_t)g.sid_base + rr / per;
  const uint32_t q = rr % per;
  const uint32_t l = q / H, h = q % H;
  return ((sid * H + h) * 8192u + l) * 3u + (uint32_t)k;
}

// the row's three gumbel draws, one per lane (lanes 0-2; the others repeat draw 0) and broadcast: a
// third of the hash / log work of every lane computing all three
__device__ __forceinline__ void abby_gumbel3(const AbbyGeom& g, int64_t r, int lane, float& z0, float& z1,
                                             float& z2) {
  const float gk = noise_gumbel_k(g.key, abby_noise_idx(g, r, lane < 3 ? lane : 0));  // key: noise_key'd
  const int gi = __builtin_bit_cast(int, gk);
  z0 += __builtin_bit_cast(float, __builtin_amdgcn_readlane(gi, 0));
  z1 += __builtin_bit_cast(float, __builtin_amdgcn_readlane(gi, 1));
  z2 += __builtin_bit_cast(float, __builtin_amdgcn_readlane(gi, 2));
}

template <int E>
__device__ __forceinline__ void ld_row(const float* __restrict__ src, int lane, float (&v)[E]) {
  if constexpr (E % 2 == 0) {
    const float2* s2 = reinterpret_cast<const float2*>(src + lane * E);
#pragma unroll
    for (int e = 0; e < E / 2; ++e) {
      const float2 t = s2[e];
      v[2 * e] = t.x;
      v[2 * e + 1] = t.y;
    }
  } else {
#pragma unroll
    for (int e = 0; e < E; ++e) v[e] = src[lane * E + e];
  }
}

// bf16 storage (the output of an AbbyNormal whose only consumers are GEMM / attention operands)
__device__ __forceinline__ unsigned pack_bf16x2(float a, float b) {
  return (unsigned)__builtin_bit_cast(unsigned short, (__bf16)a) |
         ((unsigned)__builtin_bit_cast(unsigned short, (__bf16)b) << 16);
}
template <int E>
__device__ __forceinline__ void st_row(unsigned short* __restrict__ dst, int lane, const float (&v)[E]) {
  static_assert(E % 2 == 0, "bf16 rows store feature pairs");
  unsigned* d2 = reinterpret_cast<unsigned*>(dst + lane * E);
#pragma unroll
  for (int e = 0; e < E / 2; ++e) d2[e] = pack_bf16x2(v[2 * e], v[2 * e + 1]);
}

template <int E>
__device__ __forceinline__ void st_row(float* __restrict__ dst, int lane, const float (&v)[E]) {
  if constexpr (E % 2 == 0) {
    float2* d2 = reinterpret_cast<float2*>(dst + lane * E);
#pragma unroll
    for (int e = 0; e < E / 2; ++e) d2[e] = make_float2(v[2 * e], v[2 * e + 1]);
  } else {
#pragma unroll
    for (int e = 0; e < E; ++e) dst[lane * E + e] = v[e];
  }
}

// Coalesced layout for global memory: lane l holds features 128 j + 2 l + {0, 1} (j < E / 2), so every
// float2 access of the wave covers 512 contiguous bytes.  The window pools need E consecutive features
// per lane, so the forward keeps the pool arithmetic in the consecutive layout and exchanges through
// the per-wave LDS rows (x^2 in, denominators out).
template <int E>
__device__ __forceinline__ int cfeat(int lane, int e) {
  return 128 * (e >> 1) + 2 * lane + (e & 1);
}
template <int E>
__device__ __forceinline__ void ld_rowc(const float* __restrict__ src, int lane, float (&v)[E]) {
  const float2* s2 = reinterpret_cast<const float2*>(src);
#pragma unroll
  for (int j = 0; j < E / 2; ++j) {
    const float2 t = s2[64 * j + lane];
    v[2 * j] = t.x;
    v[2 * j + 1] = t.y;
  }
}
template <int E>
__device__ __forceinline__ void st_rowc(float* __restrict__ dst, int lane, const float (&v)[E]) {
  float2* d2 = reinterpret_cast<float2*>(dst);
#pragma unroll
  for (int j = 0; j < E / 2; ++j) d2[64 * j + lane] = make_float2(v[2 * j], v[2 * j + 1]);
}
template <int E>
__device__ __forceinline__ void st_rowc(unsigned short* __restrict__ dst, int lane, const float (&v)[E]) {
  unsigned* d2 = reinterpret_cast<unsigned*>(dst);
#pragma unroll
  for (int j = 0; j < E / 2; ++j) d2[64 * j + lane] = pack_bf16x2(v[2 * j], v[2 * j + 1]);
}

// row statistics (cv = std(x, unbiased) / (mean|x| + 1e-6)) from the lane-contiguous values
template <int E>
__device__ __forceinline__ void abby_row_stats(const float (&xv)[E], float& mu, float& sd, float& mabs) {
  constexpr int D = 64 * E;
  float s = 0.f, sa = 0.f;
#pragma unroll
  for (int e = 0; e < E; ++e) {
    s += xv[e];
    sa += fabsf(xv[e]);
  }
  wave_sum2_dpp(s, sa);
  mu = s * (1.0f / D);
  mabs = sa * (1.0f / D);
  float v = 0.f;
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const float t = xv[e] - mu;
    v += t * t;
  }
  v = wave_sum_dpp(v);
  sd = sqrtf(v * (1.0f / (D - 1)));
}

// stage x^2 of this lane's features in the wave's padded LDS row and read back the halo
template <int E>
__device__ __forceinline__ void abby_halo(float* row, int lane, const float (&xv)[E], float (&h)[AbbyShape<E>::HL]) {
  typedef AbbyShape<E> S;
#pragma unroll
  for (int e = 0; e < E; ++e) row[S::PAD + lane * E + e] = xv[e] * xv[e];
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
#pragma unroll
  for (int i = 0; i < S::HL; ++i) h[i] = row[lane * E + i];
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
}

// window sums (zero padding) of the halo for the lane's E outputs.  ZPAD: the halo's pads already hold 0 (the
// forward's rows; the backward's hold -1 for its argmax), so the fmax(., 0) that maps a -1 pad to the zero
// padding is skipped -- x^2 >= 0, so the sums are identical
template <int E, bool ZPAD = false>
__device__ __forceinline__ void abby_wsum(const float (&h)[AbbyShape<E>::HL], float (&avg)[E]) {
  typedef AbbyShape<E> S;
  auto z = [](float v) __attribute__((always_inline)) { return ZPAD ? v : fmaxf(v, 0.f); };
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < S::W; ++i) s += z(h[i]);
  avg[0] = s * (1.0f / S::W);
#pragma unroll
  for (int e = 1; e < E; ++e) {
    s += z(h[e + S::W - 1]) - z(h[e - 1]);
    avg[e] = s * (1.0f / S::W);
  }
}

// window max and first argmax (as an offset into the halo) for the lane's E outputs
template <int E, bool ARG>
__device__ __forceinline__ void abby_wmax(const float (&h)[AbbyShape<E>::HL], float (&mx)[E], int (&am)[E]) {
  typedef AbbyShape<E> S;
  if constexpr (S::W >= E && E > 1) {
    // the E windows h[e, e + W) share the core h[E - 1, W): its max once, then a suffix scan of the
    // left parts h[e, E - 1) and a prefix scan of the right parts h[W, W + e) -- ~3 ops per output
    // instead of W - 1.  max is exact and the first-argmax order is kept (left parts win ties against
    // the core, the core against the right parts), so the results are identical to the plain scan.
    float cm = h[E - 1];
    int ca = E - 1;
#pragma unroll
    for (int i = E; i < S::W; ++i) {
      if (ARG) ca = h[i] > cm ? i : ca;
      cm = fmaxf(cm, h[i]);
    }
    float lm[E];
    int la[E];
    lm[E - 1] = cm;
    la[E - 1] = ca;
#pragma unroll
    for (int e = E - 2; e >= 0; --e) {
      if (ARG) la[e] = h[e] >= lm[e + 1] ? e : la[e + 1];
      lm[e] = fmaxf(lm[e + 1], h[e]);
    }
    mx[0] = lm[0];
    if (ARG) am[0] = la[0];
    float rm = h[S::W];
    int ra = S::W;
#pragma unroll
    for (int e = 1; e < E; ++e) {
      if (e > 1) {
        if (ARG) ra = h[S::W + e - 1] > rm ? S::W + e - 1 : ra;
        rm = fmaxf(rm, h[S::W + e - 1]);
      }
      if (ARG) am[e] = rm > lm[e] ? ra : la[e];
      mx[e] = fmaxf(lm[e], rm);
    }
    return;
  }
#pragma unroll
  for (int e = 0; e < E; ++e) {
    float m = h[e];
    int a = e;
#pragma unroll
    for (int i = 1; i < S::W; ++i) {
      const float v = h[e + i];
      if (ARG) {
        a = v > m ? e + i : a;
      }
      m = fmaxf(m, v);
    }
    mx[e] = m;
    if (ARG) am[e] = a;
  }
}

// 1 / (1 + 1e-4 div)^0.75 = exp2(-0.75 log2(base)), base >= 1: the output is x times this (no IEEE
// division -- ~10 instructions each -- per feature); lb = log2(base) for the backward's base^-1.75
__device__ __forceinline__ float abby_idenom(float div, float& lb) {
  lb = __builtin_amdgcn_logf(div * 1e-4f + 1.0f);
  return __builtin_amdgcn_exp2f(-0.75f * lb);
}

template <int E, typename TO = float>
__global__ __launch_bounds__(64 * ABBY_WAVES) void abby_fwd_kernel(const float* __restrict__ x,
                                                                  const float* __restrict__ hpre,
                                                                  const float* __restrict__ W2,
                                                                  const float* __restrict__ b2,
                                                                  TO* __restrict__ out, float* __restrict__ ys,
                                                                  int* __restrict__ idx_out, AbbyGeom g,
                                                                  const float* __restrict__ logits,
                                                                  const float* __restrict__ tw,
                                                                  const float* __restrict__ tb,
                                                                  float* __restrict__ tc) {
  typedef AbbyShape<E> S;
  // tw / tb / tc (optional): the consumer tgate's cs = Linear(d, 3) (model.py:530) applied to the fp32
  // output row here, so the output itself can be stored bf16 for the consumer's GEMM
  float twv[3][E];
  if (tw) {
#pragma unroll
    for (int k = 0; k < 3; ++k) ld_rowc<E>(tw + k * S::D, threadIdx.x & 63, twv[k]);
  }
  // x^2 row: feature f at P0 + f (P0 = PAD rounded up to even, so the coalesced float2 writes stay
  // 8-byte aligned), pads of 0 on both sides (the avg pool's zero padding; for the max pool a 0 pad equals
  // the reference's -inf one: every window holds a real x^2 >= 0 and the forward takes no argmax); den row:
  // the denominators by feature.  The halo is read as float2 from the even index at or below its start
  // (HS = the offset of the halo in that read), so the row stride is even too.
  constexpr int P0 = (S::PAD + 1) & ~1;
  constexpr int HS = (P0 - S::PAD) & 1;
  constexpr int HR = (S::HL + HS + 1) / 2;  // float2 reads per lane
  constexpr int ROWC = (P0 + S::D + S::PAD + 1 + 1) & ~1;
  static_assert(P0 - S::PAD - HS >= 0 && P0 - S::PAD - HS + 63 * E + 2 * HR <= ROWC, "halo read inside the row");
  __shared__ __attribute__((aligned(16))) float rows_all[ABBY_WAVES][ROWC];
  __shared__ __attribute__((aligned(16))) float den_all[ABBY_WAVES][S::D];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  float* row = rows_all[wid];
  float* drow = den_all[wid];
  for (int i = lane; i < S::PAD; i += 64) {
    row[P0 - S::PAD + i] = 0.f;
    row[P0 + S::D + i] = 0.f;
  }
  const int64_t stride = (int64_t)gridDim.x * ABBY_WAVES;
  int64_t r = (int64_t)blockIdx.x * ABBY_WAVES + wid;
  g.key = noise_key(g.key);
  // The next TWO rows' x (coalesced layout) and router logits are in flight while a row is processed,
  // in two NAMED register sets used alternately (the loop is unrolled by two): rotating one set into
  // the other (x1 = x2 at the top of each row) made the compiler wait for the newest prefetch at every
  // row, i.e. one row of prefetch in effect.  Loads past the end re-read the last row (unconditional,
  // so the wait counts stay uniform).
  float xa[E], xb[E], la[3] = {0.f, 0.f, 0.f}, lb[3] = {0.f, 0.f, 0.f};
  auto fetch = [&](int64_t rr, float (&xs)[E], float (&ls)[3]) __attribute__((always_inline)) {
    const int64_t rc = rr < g.rows ? rr : g.rows - 1;
    ld_rowc<E>(x + rc * S::D, lane, xs);
    if (logits) {
      ls[0] = logits[rc * 3 + 0];
      ls[1] = logits[rc * 3 + 1];
      ls[2] = logits[rc * 3 + 2];
    }
  };
  if (r < g.rows) {
    fetch(r, xa, la);
    fetch(r + stride, xb, lb);
  }
  // one row: xv / l0..l2 its x and router logits
  auto row_body = [&](int64_t r, const float (&xv)[E], float l0, float l1, float l2) __attribute__((always_inline)) {
    if (!logits) {
      float hv[E];
      ld_rowc<E>(hpre + r * S::D, lane, hv);
      l0 = l1 = l2 = 0.f;
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const int j = cfeat<E>(lane, e);
        const float hs = silu_f(hv[e]);
        l0 += hs * W2[j];
        l1 += hs * W2[S::D + j];
        l2 += hs * W2[2 * S::D + j];
      }
      wave_sum3_dpp(l0, l1, l2);
    }
    float mu, sd, mabs;
    abby_row_stats<E>(xv, mu, sd, mabs);
    if (g.nrm) {
      float ss = 0.f;
#pragma unroll
      for (int e = 0; e < E; ++e) ss += xv[e] * xv[e];
      ss = wave_sum_dpp(ss);
      if (lane == 0) g.nrm[r] = sqrtf(ss);
    }
    const float cv = sd / (mabs + 1e-6f);
    float z0 = l0 + b2[0] + cv, z1 = l1 + b2[1] + cv, z2 = l2 + b2[2] + cv;
    if (g.use_noise) abby_gumbel3(g, r, lane, z0, z1, z2);
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
    // x^2 in (coalesced layout) -> halo of the lane's E consecutive features -> pools -> denominators
#pragma unroll
    for (int j = 0; j < E / 2; ++j)
      *reinterpret_cast<float2*>(row + P0 + 128 * j + 2 * lane) =
          make_float2(xv[2 * j] * xv[2 * j], xv[2 * j + 1] * xv[2 * j + 1]);
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    float hh[2 * HR];
#pragma unroll
    for (int i = 0; i < HR; ++i) {
      const float2 t = *reinterpret_cast<const float2*>(row + P0 - S::PAD - HS + lane * E + 2 * i);
      hh[2 * i] = t.x;
      hh[2 * i + 1] = t.y;
    }
    float h[S::HL];
#pragma unroll
    for (int i = 0; i < S::HL; ++i) h[i] = hh[i + HS];
    float avg[E];
    abby_wsum<E, true>(h, avg);
    if (sel == 1) {  // wave-uniform: mode 2 (max pool where max > 2 avg)
      float mx[E];
      int am[E];
      abby_wmax<E, false>(h, mx, am);
      if (g.cond) {
#pragma unroll
        for (int e = 0; e < E; ++e) g.cond[r * S::D + lane * E + e] = mx[e] > 2.0f * avg[e] ? 1 : 0;
      }
#pragma unroll
      for (int e = 0; e < E; ++e) avg[e] = mx[e] > 2.0f * avg[e] ? mx[e] : avg[e];
    }
#pragma unroll
    for (int e = 0; e < E; ++e) {
      float lb;
      drow[lane * E + e] = abby_idenom(avg[e], lb);  // inverse denominators
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    float ov[E];
#pragma unroll
    for (int j = 0; j < E / 2; ++j) {
      const float2 dn = *reinterpret_cast<const float2*>(drow + 128 * j + 2 * lane);
      ov[2 * j] = xv[2 * j] * dn.x;
      ov[2 * j + 1] = xv[2 * j + 1] * dn.y;
    }
    if (g.res) {
      float rv[E];
      ld_rowc<E>(g.res + r * S::D, lane, rv);
#pragma unroll
      for (int e = 0; e < E; ++e) ov[e] += rv[e];
    }
    st_rowc<E>(out + r * S::D, lane, ov);
    if (tw) {
      float c0 = 0.f, c1 = 0.f, c2 = 0.f;
#pragma unroll
      for (int e = 0; e < E; ++e) {
        c0 += ov[e] * twv[0][e];
        c1 += ov[e] * twv[1][e];
        c2 += ov[e] * twv[2][e];
      }
      wave_sum3_dpp(c0, c1, c2);
      if (lane == 0) {
        tc[r * 3 + 0] = c0 + tb[0];
        tc[r * 3 + 1] = c1 + tb[1];
        tc[r * 3 + 2] = c2 + tb[2];
      }
    }
    __builtin_amdgcn_wave_barrier();  // the next row overwrites both LDS rows
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  };
  for (; r < g.rows; r += 2 * stride) {
    {
      float xv[E];
      const float l0 = la[0], l1 = la[1], l2 = la[2];
#pragma unroll
      for (int e = 0; e < E; ++e) xv[e] = xa[e];
      fetch(r + 2 * stride, xa, la);
      row_body(r, xv, l0, l1, l2);
    }
    const int64_t r2 = r + stride;
    if (r2 >= g.rows) break;
    {
      float xv[E];
      const float l0 = lb[0], l1 = lb[1], l2 = lb[2];
#pragma unroll
      for (int e = 0; e < E; ++e) xv[e] = xb[e];
      fetch(r2 + 2 * stride, xb, lb);
      row_body(r2, xv, l0, l1, l2);
    }
  }
}

template <int E>
__global__ __launch_bounds__(64 * ABBY_WAVES) void abby_bwd_kernel(
    const float* __restrict__ dout, const float* __restrict__ x, const float* __restrict__ hpre,
    const float* __restrict__ W2, const float* __restrict__ ys, const int* __restrict__ idx_in,
    float* __restrict__ dx, float* __restrict__ dhpre, float* __restrict__ dW2, float* __restrict__ db2,
    AbbyGeom g) {
  typedef AbbyShape<E> S;
  __shared__ __attribute__((aligned(16))) float rows_all[ABBY_WAVES][S::ROW];   // x^2, then q coefA / w
  __shared__ __attribute__((aligned(16))) float cm_all[ABBY_WAVES][S::ROW];     // q coefM (sel == 1)
  __shared__ __attribute__((aligned(16))) int am_all[ABBY_WAVES][S::ROW];       // argmax (halo offset + base)
  // layout exchange rows: global memory is read and written in the coalesced layout (cfeat), the pool
  // arithmetic runs on E consecutive features per lane
  __shared__ __attribute__((aligned(16))) float xr_all[ABBY_WAVES][S::D];  // x, then dx (pool part)
  __shared__ __attribute__((aligned(16))) float gr_all[ABBY_WAVES][S::D];  // dout
  __shared__ float red[ABBY_WAVES][3];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  float* row = rows_all[wid];
  float* cmr = cm_all[wid];
  int* amr = am_all[wid];
  float* xr = xr_all[wid];
  float* gr = gr_all[wid];
  float accW[3][E];
  float accb[3] = {0.f, 0.f, 0.f};
#pragma unroll
  for (int k = 0; k < 3; ++k)
#pragma unroll
    for (int e = 0; e < E; ++e) accW[k][e] = 0.f;

  const int64_t stride = (int64_t)gridDim.x * ABBY_WAVES;
  int64_t r = (int64_t)blockIdx.x * ABBY_WAVES + wid;
  // x and dout of the next TWO rows (coalesced layout) are in flight while this row is processed
  // (one row ahead left the kernel latency-bound); past the end the last row is re-read
  // (the row's mode and softmax outputs travel with it: read at the top of the row they stalled every
  // row for a full memory latency before the pools could start)
  // d >= 768: one row ahead (two register sets of x and dout would not fit: 512 VGPRs and scratch
  // spills at d = 1024)
  constexpr int AHEAD = E >= 12 ? 1 : 2;
  float xn1[E], gn1[E], xn2[E], gn2[E], yn1[3], yn2[3];
  int sn1, sn2;
  auto fetch = [&](int64_t rr, float (&xb)[E], float (&gb)[E], float (&yb)[3], int& sb) __attribute__((always_inline)) {
    const int64_t rc = rr < g.rows ? rr : g.rows - 1;
    ld_rowc<E>(x + rc * S::D, lane, xb);
    ld_rowc<E>(dout + rc * S::D, lane, gb);
    yb[0] = ys[rc * 3 + 0];
    yb[1] = ys[rc * 3 + 1];
    yb[2] = ys[rc * 3 + 2];
    sb = idx_in[rc];
  };
  if (r < g.rows) {
    fetch(r, xn1, gn1, yn1, sn1);
    if constexpr (AHEAD == 2) fetch(r + stride, xn2, gn2, yn2, sn2);
  }
  // one row from register set 1 or 2 (alternating, see abby_fwd_kernel), refilled with the row two
  // strides ahead once its values are in LDS / locals
  auto row_body = [&](int64_t r, float (&xs)[E], float (&gs)[E], float (&ysv)[3], int& ss) __attribute__((always_inline)) {
    float xc[E], xv[E], gv[E];  // xc: coalesced layout; xv, gv: the lane's E consecutive features
    // this row's later operands, issued now so their latency overlaps the pool work
    float hv[E], old[E];
    ld_rowc<E>(hpre + r * S::D, lane, hv);
    if (g.acc) ld_rowc<E>(dx + r * S::D, lane, old);
#pragma unroll
    for (int j = 0; j < E / 2; ++j) {
      xc[2 * j] = xs[2 * j];
      xc[2 * j + 1] = xs[2 * j + 1];
      *reinterpret_cast<float2*>(xr + 128 * j + 2 * lane) = make_float2(xs[2 * j], xs[2 * j + 1]);
      *reinterpret_cast<float2*>(gr + 128 * j + 2 * lane) = make_float2(gs[2 * j], gs[2 * j + 1]);
    }
    const int sel = __builtin_amdgcn_readfirstlane(ss);
    const float y0 = ysv[0], y1 = ysv[1], y2 = ysv[2];
    fetch(r + AHEAD * stride, xs, gs, ysv, ss);
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
#pragma unroll
    for (int e = 0; e < E; ++e) {
      xv[e] = xr[lane * E + e];
      gv[e] = gr[lane * E + e];
    }
    // the pad entries of `row` hold -1 for the x^2 halo; the coefficient pass below re-pads with 0
    for (int i = lane; i < S::PAD; i += 64) {
      row[i] = -1.f;
      row[S::PAD + S::D + i] = -1.f;
    }
    float h[S::HL];
    abby_halo<E>(row, lane, xv, h);
    // mode 2 enters dd1 (the straight-through gradient of the mode choice) on every row; its
    // argmax is needed only where mode 2 was chosen (sel == 1, wave-uniform)
    float avg[E], m2[E], mx[E];
    int am[E];
    abby_wsum<E>(h, avg);
    if (sel == 1) {
      abby_wmax<E, true>(h, mx, am);
    } else {
      abby_wmax<E, false>(h, mx, am);
    }
#pragma unroll
    for (int e = 0; e < E; ++e) m2[e] = mx[e] > 2.0f * avg[e] ? mx[e] : avg[e];
    float dxv[E], qa[E], qm[E];
    float dd0 = 0.f, dd1 = 0.f;  // dd2 == dd0 (mode3 == mode1 == avg)
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const float div = sel == 1 ? m2[e] : avg[e];
      float lb;
      const float idn = abby_idenom(div, lb);
      dxv[e] = gv[e] * idn;
      // d out / d div = -0.75e-4 x base^-1.75
      const float q = -gv[e] * xv[e] * (1e-4f * 0.75f) * __builtin_amdgcn_exp2f(-1.75f * lb);
      dd0 += q * avg[e];
      dd1 += q * m2[e];
      const bool maxsel = sel == 1 && m2[e] != avg[e];
      qa[e] = maxsel ? 0.f : q * (1.0f / S::W);
      qm[e] = maxsel ? q : 0.f;
    }
    wave_sum2_dpp(dd0, dd1);
    const float dd2 = dd0;
    // pool backward in gather form: dsq_i = sum_{j in win(i)} qa_j + sum_{j in win(i), am_j == i} qm_j
    for (int i = lane; i < S::PAD; i += 64) {
      row[i] = 0.f;
      row[S::PAD + S::D + i] = 0.f;
      if (sel == 1) {
        cmr[i] = 0.f;
        cmr[S::PAD + S::D + i] = 0.f;
        amr[i] = -1;
        amr[S::PAD + S::D + i] = -1;
      }
    }
#pragma unroll
    for (int e = 0; e < E; ++e) row[S::PAD + lane * E + e] = qa[e];
    if (sel == 1) {
#pragma unroll
      for (int e = 0; e < E; ++e) {
        cmr[S::PAD + lane * E + e] = qm[e];
        amr[S::PAD + lane * E + e] = lane * E + am[e] - S::PAD;  // feature index of the argmax
      }
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    {
      float ha[S::HL];
#pragma unroll
      for (int i = 0; i < S::HL; ++i) ha[i] = row[lane * E + i];
      float s = 0.f;
#pragma unroll
      for (int i = 0; i < S::W; ++i) s += ha[i];
      dxv[0] += 2.0f * xv[0] * s;
#pragma unroll
      for (int e = 1; e < E; ++e) {
        s += ha[e + S::W - 1] - ha[e - 1];
        dxv[e] += 2.0f * xv[e] * s;
      }
    }
    if (sel == 1) {
      float hc[S::HL];
      int hm[S::HL];
#pragma unroll
      for (int i = 0; i < S::HL; ++i) {  // halo position i holds feature lane E - PAD + i
        hc[i] = cmr[lane * E + i];
        hm[i] = amr[lane * E + i];
      }
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const int fi = lane * E + e;
        float s = 0.f;
#pragma unroll
        for (int i = 0; i < S::W; ++i) s += hm[e + i] == fi ? hc[e + i] : 0.f;
        dxv[e] += 2.0f * xv[e] * s;
      }
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    // straight-through softmax backward
    const float dot = y0 * dd0 + y1 * dd1 + y2 * dd2;
    const float dz0 = y0 * (dd0 - dot), dz1 = y1 * (dd1 - dot), dz2 = y2 * (dd2 - dot);
    const float dcv = dz0 + dz1 + dz2;
    // cv = sd / (mabs + 1e-6)
    float mu, sd, mabs;
    abby_row_stats<E>(xc, mu, sd, mabs);
    const float den = mabs + 1e-6f;
    const float dsd = dcv / den;
    const float dmabs = -dcv * sd / (den * den);
    const float csd = sd > 0.f ? dsd / ((S::D - 1) * sd) : 0.f;
    const float cma = dmabs / S::D;
    // the pool part of dx back to the coalesced layout; everything below is elementwise in it
#pragma unroll
    for (int e = 0; e < E; ++e) xr[lane * E + e] = dxv[e];
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    float dxc[E], dh[E], w2v[3][E];
#pragma unroll
    for (int j = 0; j < E / 2; ++j) {
      const float2 t = *reinterpret_cast<const float2*>(xr + 128 * j + 2 * lane);
      dxc[2 * j] = t.x;
      dxc[2 * j + 1] = t.y;
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) ld_rowc<E>(W2 + k * S::D, lane, w2v[k]);  // L1-resident
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const float sgn = xc[e] > 0.f ? 1.f : (xc[e] < 0.f ? -1.f : 0.f);
      dxc[e] += csd * (xc[e] - mu) + cma * sgn;
      const float wsum = dz0 * w2v[0][e] + dz1 * w2v[1][e] + dz2 * w2v[2][e];
      dh[e] = silu_grad(hv[e]) * wsum;
      const float hs = silu_f(hv[e]);
      accW[0][e] += dz0 * hs;
      accW[1][e] += dz1 * hs;
      accW[2][e] += dz2 * hs;
    }
    if (g.acc) {
#pragma unroll
      for (int e = 0; e < E; ++e) dxc[e] += old[e];
    }
    st_rowc<E>(dx + r * S::D, lane, dxc);
    st_rowc<E>(dhpre + r * S::D, lane, dh);
    __builtin_amdgcn_wave_barrier();  // the next row overwrites the exchange rows
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    accb[0] += dz0;
    accb[1] += dz1;
    accb[2] += dz2;
  };
  if constexpr (AHEAD == 1) {
    for (; r < g.rows; r += stride) row_body(r, xn1, gn1, yn1, sn1);
  } else {
    for (; r < g.rows; r += 2 * stride) {
      row_body(r, xn1, gn1, yn1, sn1);
      if (r + stride >= g.rows) break;
      row_body(r + stride, xn2, gn2, yn2, sn2);
    }
  }
  // workgroup reduction of dW2 / db2 through LDS, then one atomic per element
  __syncthreads();
  float* buf = &rows_all[0][0];  // 3 D floats fit in the 4 x ROW x-rows plus the cm rows
  float* buf2 = &cm_all[0][0];
  static_assert(3 * S::D <= 2 * ABBY_WAVES * S::ROW, "dW2 staging must fit");
  auto slot = [&](int k, int j) -> float* {
    const int i = k * S::D + j;
    return i < ABBY_WAVES * S::ROW ? buf + i : buf2 + (i - ABBY_WAVES * S::ROW);
  };
  for (int ww = 0; ww < ABBY_WAVES; ++ww) {
    if (wid == ww) {
#pragma unroll
      for (int k = 0; k < 3; ++k)
#pragma unroll
        for (int e = 0; e < E; ++e) {  // accW is in the coalesced layout
          float* sl = slot(k, cfeat<E>(lane, e));
          *sl = (ww == 0 ? 0.f : *sl) + accW[k][e];
        }
    }
    __syncthreads();
  }
  for (int j = threadIdx.x; j < 3 * S::D; j += 64 * ABBY_WAVES) atomicAdd(dW2 + j, *slot(j / S::D, j % S::D));
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

// ---------------------------------------------------------------------------------------------
// d = 64 (the per-head AbbyNormal on q and k, model.py:302-306): a 64-feature row is one DPP row of
// 16 lanes holding 4 consecutive features each (float4 in, float4 out), 4 rows per wave.  Every
// reduction is 4 in-row DPP steps and the w = 3 window halo is one row_shr / row_shl (the source
// lane outside the 16-lane row leaves the pad value), so the kernel never touches LDS.
__device__ __forceinline__ float row16_sum(float v) {
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x141, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x140, 0xF, 0xF, false));
  return v;
}
// value of lane - 1 (row_shr:1) / lane + 1 (row_shl:1) in the same 16-lane row, `pad` at the row ends
__device__ __forceinline__ float from_prev(float v, float pad) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, pad), __builtin_bit_cast(int, v),
                                                               0x111, 0xF, 0xF, false));
}
__device__ __forceinline__ float from_next(float v, float pad) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, pad), __builtin_bit_cast(int, v),
                                                               0x101, 0xF, 0xF, false));
}
__device__ __forceinline__ int from_prev_i(int v, int pad) { return __builtin_amdgcn_update_dpp(pad, v, 0x111, 0xF, 0xF, false); }
__device__ __forceinline__ int from_next_i(int v, int pad) { return __builtin_amdgcn_update_dpp(pad, v, 0x101, 0xF, 0xF, false); }

struct Row64 {
  float v[4];
};
__device__ __forceinline__ Row64 ld64(const float* p) {
  const float4 t = *reinterpret_cast<const float4*>(p);
  return Row64{{t.x, t.y, t.z, t.w}};
}
__device__ __forceinline__ void st64(float* p, const float (&v)[4]) {
  *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
}
__device__ __forceinline__ void st64(unsigned short* p, const float (&v)[4]) {
  *reinterpret_cast<uint2*>(p) = make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
}

// x^2 halo of the lane's 4 features: h[0] = feature 4l - 1, h[1..4] own, h[5] = feature 4l + 4
__device__ __forceinline__ void halo64(const float (&sq)[4], float (&h)[6]) {
  h[0] = from_prev(sq[3], -1.f);
  h[1] = sq[0]; h[2] = sq[1]; h[3] = sq[2]; h[4] = sq[3];
  h[5] = from_next(sq[0], -1.f);
}

__device__ __forceinline__ void stats64(const float (&xv)[4], float& mu, float& sd, float& mabs) {
  float s = xv[0] + xv[1] + xv[2] + xv[3];
  float sa = fabsf(xv[0]) + fabsf(xv[1]) + fabsf(xv[2]) + fabsf(xv[3]);
  s = row16_sum(s);
  sa = row16_sum(sa);
  mu = s * (1.0f / 64.f);
  mabs = sa * (1.0f / 64.f);
  float v = 0.f;
#pragma unroll
  for (int e = 0; e < 4; ++e) v += (xv[e] - mu) * (xv[e] - mu);
  sd = sqrtf(row16_sum(v) * (1.0f / 63.f));
}

template <typename TO = float>
__global__ __launch_bounds__(64 * ABBY_WAVES) void abby_fwd64_kernel(const float* __restrict__ x,
                                                                    const float* __restrict__ hpre,
                                                                    const float* __restrict__ W2,
                                                                    const float* __restrict__ b2,
                                                                    TO* __restrict__ out, float* __restrict__ ys,
                                                                    int* __restrict__ idx_out, AbbyGeom g,
                                                                    const float* __restrict__ logits) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, l16 = lane & 15;
  const int64_t stride = (int64_t)gridDim.x * ABBY_WAVES * 4;
  g.key = noise_key(g.key);
  for (int64_t r = ((int64_t)blockIdx.x * ABBY_WAVES + wid) * 4 + (lane >> 4); r < g.rows; r += stride) {
    // (rows is a multiple of nothing in particular: a 16-lane row past the end simply idles; the
    // DPP reductions never cross rows, so the live rows are unaffected)
    const Row64 xr = ld64(x + r * 64 + 4 * l16);
    const float(&xv)[4] = xr.v;
    float l0, l1, l2;
    if (logits) {
      l0 = logits[r * 3 + 0];
      l1 = logits[r * 3 + 1];
      l2 = logits[r * 3 + 2];
    } else {
      const Row64 hr = ld64(hpre + r * 64 + 4 * l16);
      l0 = l1 = l2 = 0.f;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int j = 4 * l16 + e;
        const float hs = silu_f(hr.v[e]);
        l0 += hs * W2[j];
        l1 += hs * W2[64 + j];
        l2 += hs * W2[128 + j];
      }
      l0 = row16_sum(l0);
      l1 = row16_sum(l1);
      l2 = row16_sum(l2);
    }
    float mu, sd, mabs;
    stats64(xv, mu, sd, mabs);
    const float cv = sd / (mabs + 1e-6f);
    float z0 = l0 + b2[0] + cv, z1 = l1 + b2[1] + cv, z2 = l2 + b2[2] + cv;
    if (g.use_noise) {  // lanes 0-2 of the 16-lane row draw one gumbel each, then broadcast in the row
      const float gk = noise_gumbel_k(g.key, abby_noise_idx(g, r, l16 < 3 ? l16 : 0));
      const int base = lane & 48;
      z0 += __shfl(gk, base + 0);
      z1 += __shfl(gk, base + 1);
      z2 += __shfl(gk, base + 2);
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
    if (l16 == 0) {
      ys[r * 3 + 0] = y0;
      ys[r * 3 + 1] = y1;
      ys[r * 3 + 2] = y2;
      idx_out[r] = sel;
    }
    float sq[4] = {xv[0] * xv[0], xv[1] * xv[1], xv[2] * xv[2], xv[3] * xv[3]};
    float h[6];
    halo64(sq, h);
    float ov[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float avg = (fmaxf(h[e], 0.f) + h[e + 1] + fmaxf(h[e + 2], 0.f)) * (1.0f / 3.0f);
      const float mx = fmaxf(h[e], fmaxf(h[e + 1], h[e + 2]));
      const float div = (sel == 1 && mx > 2.0f * avg) ? mx : avg;
      if (g.cond && sel == 1) g.cond[r * 64 + 4 * l16 + e] = mx > 2.0f * avg ? 1 : 0;
      float base;
      ov[e] = xv[e] * abby_idenom(div, base);
    }
    st64(out + r * 64 + 4 * l16, ov);
  }
}

__global__ __launch_bounds__(64 * ABBY_WAVES) void abby_bwd64_kernel(
    const float* __restrict__ dout, const float* __restrict__ x, const float* __restrict__ hpre,
    const float* __restrict__ W2, const float* __restrict__ ys, const int* __restrict__ idx_in,
    float* __restrict__ dx, float* __restrict__ dhpre, float* __restrict__ dW2, float* __restrict__ db2,
    AbbyGeom g) {
  __shared__ float wred[ABBY_WAVES * 4][3 * 64 + 3];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, l16 = lane & 15;
  float accW[3][4] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
  float accb[3] = {0.f, 0.f, 0.f};
  float w2v[3][4];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const Row64 t = ld64(W2 + k * 64 + 4 * l16);
#pragma unroll
    for (int e = 0; e < 4; ++e) w2v[k][e] = t.v[e];
  }
  const int64_t stride = (int64_t)gridDim.x * ABBY_WAVES * 4;
  for (int64_t r = ((int64_t)blockIdx.x * ABBY_WAVES + wid) * 4 + (lane >> 4); r < g.rows; r += stride) {
    const Row64 xr = ld64(x + r * 64 + 4 * l16);
    const Row64 gr = ld64(dout + r * 64 + 4 * l16);
    const Row64 hr = ld64(hpre + r * 64 + 4 * l16);
    const float(&xv)[4] = xr.v;
    const float(&gv)[4] = gr.v;
    const int sel = idx_in[r];
    const float y0 = ys[r * 3 + 0], y1 = ys[r * 3 + 1], y2 = ys[r * 3 + 2];
    float sq[4] = {xv[0] * xv[0], xv[1] * xv[1], xv[2] * xv[2], xv[3] * xv[3]};
    float h[6];
    halo64(sq, h);
    float dxv[4], qa[4], qm[4];
    int am[4];
    float dd0 = 0.f, dd1 = 0.f;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float avg = (fmaxf(h[e], 0.f) + h[e + 1] + fmaxf(h[e + 2], 0.f)) * (1.0f / 3.0f);
      // max and first argmax over features 4l+e-1 .. 4l+e+1
      float mx = h[e];
      int a = 4 * l16 + e - 1;
      if (h[e + 1] > mx) { mx = h[e + 1]; a = 4 * l16 + e; }
      if (h[e + 2] > mx) { mx = h[e + 2]; a = 4 * l16 + e + 1; }
      am[e] = a;
      const bool cnd = mx > 2.0f * avg;
      const float m2 = cnd ? mx : avg;
      const float div = sel == 1 ? m2 : avg;
      float base;
      const float idn = abby_idenom(div, base);  // base: log2 of the denominator's base here
      dxv[e] = gv[e] * idn;
      const float q = -gv[e] * xv[e] * (1e-4f * 0.75f) * __builtin_amdgcn_exp2f(-1.75f * base);
      dd0 += q * avg;
      dd1 += q * m2;
      const bool maxsel = sel == 1 && cnd;
      qa[e] = maxsel ? 0.f : q * (1.0f / 3.0f);
      qm[e] = maxsel ? q : 0.f;
    }
    dd0 = row16_sum(dd0);
    dd1 = row16_sum(dd1);
    const float dd2 = dd0;
    // pool backward: dsq_i = qa_{i-1} + qa_i + qa_{i+1} + sum_{j in i-1..i+1, am_j == i} qm_j
    {
      const float qa_p = from_prev(qa[3], 0.f), qa_n = from_next(qa[0], 0.f);
      const float qm_p = from_prev(qm[3], 0.f), qm_n = from_next(qm[0], 0.f);
      const int am_p = from_prev_i(am[3], -2), am_n = from_next_i(am[0], -2);
      const float qa6[6] = {qa_p, qa[0], qa[1], qa[2], qa[3], qa_n};
      const float qm6[6] = {qm_p, qm[0], qm[1], qm[2], qm[3], qm_n};
      const int am6[6] = {am_p, am[0], am[1], am[2], am[3], am_n};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int fi = 4 * l16 + e;
        float s = qa6[e] + qa6[e + 1] + qa6[e + 2];
#pragma unroll
        for (int i = 0; i < 3; ++i) s += am6[e + i] == fi ? qm6[e + i] : 0.f;
        dxv[e] += 2.0f * xv[e] * s;
      }
    }
    const float dot = y0 * dd0 + y1 * dd1 + y2 * dd2;
    const float dz0 = y0 * (dd0 - dot), dz1 = y1 * (dd1 - dot), dz2 = y2 * (dd2 - dot);
    const float dcv = dz0 + dz1 + dz2;
    float mu, sd, mabs;
    stats64(xv, mu, sd, mabs);
    const float den = mabs + 1e-6f;
    const float dsd = dcv / den;
    const float dmabs = -dcv * sd / (den * den);
    const float csd = sd > 0.f ? dsd / (63.f * sd) : 0.f;
    const float cma = dmabs * (1.0f / 64.f);
    float dh[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float sgn = xv[e] > 0.f ? 1.f : (xv[e] < 0.f ? -1.f : 0.f);
      dxv[e] += csd * (xv[e] - mu) + cma * sgn;
      const float hv = hr.v[e];
      dh[e] = silu_grad(hv) * (dz0 * w2v[0][e] + dz1 * w2v[1][e] + dz2 * w2v[2][e]);
      const float hs = silu_f(hv);
      accW[0][e] += dz0 * hs;
      accW[1][e] += dz1 * hs;
      accW[2][e] += dz2 * hs;
    }
    if (g.acc) {
      const float4 o = *reinterpret_cast<const float4*>(dx + r * 64 + 4 * l16);
      dxv[0] += o.x;
      dxv[1] += o.y;
      dxv[2] += o.z;
      dxv[3] += o.w;
    }
    st64(dx + r * 64 + 4 * l16, dxv);
    st64(dhpre + r * 64 + 4 * l16, dh);
    accb[0] += dz0;
    accb[1] += dz1;
    accb[2] += dz2;
  }
  // reduce the 16 row-groups of the workgroup (4 per wave), then one atomic per element
  const int grp = wid * 4 + (lane >> 4);
#pragma unroll
  for (int k = 0; k < 3; ++k)
#pragma unroll
    for (int e = 0; e < 4; ++e) wred[grp][k * 64 + 4 * l16 + e] = accW[k][e];
  if (l16 == 0) {
    wred[grp][192] = accb[0];
    wred[grp][193] = accb[1];
    wred[grp][194] = accb[2];
  }
  __syncthreads();
  for (int j = threadIdx.x; j < 195; j += 64 * ABBY_WAVES) {
    float sacc = 0.f;
    for (int q = 0; q < ABBY_WAVES * 4; ++q) sacc += wred[q][j];
    atomicAdd(j < 192 ? dW2 + j : db2 + (j - 192), sacc);
  }
}

}  // namespace asrx

using namespace asrx;

#define ABBY_DISPATCH_T(KERNEL, TO, ...)                                                      \
  switch (E) {                                                                               \
    case 2: KERNEL<2, TO><<<grid, 64 * ABBY_WAVES, 0, stream>>>(__VA_ARGS__); break;         \
    case 4: KERNEL<4, TO><<<grid, 64 * ABBY_WAVES, 0, stream>>>(__VA_ARGS__); break;         \
    case 6: KERNEL<6, TO><<<grid, 64 * ABBY_WAVES, 0, stream>>>(__VA_ARGS__); break;         \
    case 8: KERNEL<8, TO><<<grid, 64 * ABBY_WAVES, 0, stream>>>(__VA_ARGS__); break;         \
    case 12: KERNEL<12, TO><<<grid, 64 * ABBY_WAVES, 0, stream>>>(__VA_ARGS__); break;       \
    case 16: KERNEL<16, TO><<<grid, 64 * ABBY_WAVES, 0, stream>>>(__VA_ARGS__); break;       \
    default: set_error("AbbyNormal: unsupported d=%ld", (long)d); return 2;                  \
  }

#define ABBY_DISPATCH(KERNEL, ...)                                                 \
  switch (E) {                                                                     \
    case 2: KERNEL<2><<<grid, 64 * ABBY_WAVES, 0, stream>>>(__VA_ARGS__); break;   \
    case 4: KERNEL<4><<<grid, 64 * ABBY_WAVES, 0, stream>>>(__VA_ARGS__); break;   \
    case 6: KERNEL<6><<<grid, 64 * ABBY_WAVES, 0, stream>>>(__VA_ARGS__); break;   \
    case 8: KERNEL<8><<<grid, 64 * ABBY_WAVES, 0, stream>>>(__VA_ARGS__); break;   \
    case 12: KERNEL<12><<<grid, 64 * ABBY_WAVES, 0, stream>>>(__VA_ARGS__); break; \
    case 16: KERNEL<16><<<grid, 64 * ABBY_WAVES, 0, stream>>>(__VA_ARGS__); break; \
    default: set_error("AbbyNormal: unsupported d=%ld", (long)d); return 2;        \
  }

// host-side decision recorder target (asrx_abby_record_cond; parity tests, eager only)
static unsigned char* g_cond_record = nullptr;

static AbbyGeom make_geom(int64_t rows, int64_t d, int64_t L, int64_t H, int64_t sid_base, uint32_t key,
                          int use_noise) {
  AbbyGeom g;
  g.cond = nullptr;
  g.res = nullptr;
  g.nrm = nullptr;
  g.rows = rows;
  g.d = d;
  g.L = L > 0 ? L : 1;
  g.H = H > 0 ? H : 1;
  g.sid_base = sid_base;
  g.key = key;
  g.use_noise = use_noise;
  g.acc = 0;
  return g;
}

// x, hpre: (rows, d); W2 (3, d), b2 (3); out (rows, d) fp32 (out_bf16 = 0) or bf16 (1); ys (rows, 3);
// idx (rows) int32.
extern "C" int asrx_abby_fwd2(const float* x, const float* hpre, const float* W2, const float* b2, void* out,
                              int out_bf16, float* ys, int* idx, int64_t rows, int64_t d, int64_t L, int64_t H,
                              int64_t sid_base, uint32_t key, int use_noise, const float* tw, const float* tb,
                              float* tc, hipStream_t stream) {
  ASRX_REQUIRE(!tw || d >= 128, "AbbyNormal: the fused tgate cs needs d >= 128");
  ASRX_REQUIRE(d % 64 == 0 && d >= 64 && d <= 1024, "AbbyNormal: d=%ld must be a multiple of 64 in [64,1024]",
               (long)d);
  if (rows == 0) return 0;
  const int E = (int)(d / 64);
  AbbyGeom g = make_geom(rows, d, L, H, sid_base, key, use_noise);
  g.cond = g_cond_record;
  const unsigned grid = (unsigned)std::min<int64_t>((rows + ABBY_WAVES - 1) / ABBY_WAVES, 4096);
  if (d == 64) {
    const unsigned g64 = (unsigned)std::min<int64_t>((rows + 4 * ABBY_WAVES - 1) / (4 * ABBY_WAVES), 4096);
    if (out_bf16)
      abby_fwd64_kernel<unsigned short><<<g64, 64 * ABBY_WAVES, 0, stream>>>(x, hpre, W2, b2, (unsigned short*)out, ys,
                                                                           idx, g, nullptr);
    else
      abby_fwd64_kernel<float><<<g64, 64 * ABBY_WAVES, 0, stream>>>(x, hpre, W2, b2, (float*)out, ys, idx, g, nullptr);
    ASRX_LAUNCHED("asrx_abby_fwd");
  }
  if (out_bf16) {
    ABBY_DISPATCH_T(abby_fwd_kernel, unsigned short, x, hpre, W2, b2, (unsigned short*)out, ys, idx, g, nullptr, tw,
                    tb, tc);
  } else {
    ABBY_DISPATCH_T(abby_fwd_kernel, float, x, hpre, W2, b2, (float*)out, ys, idx, g, nullptr, tw, tb, tc);
  }
  ASRX_LAUNCHED("asrx_abby_fwd");
}

extern "C" int asrx_abby_fwd(const float* x, const float* hpre, const float* W2, const float* b2, float* out,
                             float* ys, int* idx, int64_t rows, int64_t d, int64_t L, int64_t H,
                             int64_t sid_base, uint32_t key, int use_noise, hipStream_t stream) {
  return asrx_abby_fwd2(x, hpre, W2, b2, out, 0, ys, idx, rows, d, L, H, sid_base, key, use_noise, nullptr, nullptr,
                        nullptr, stream);
}

// Same, with the router logits (rows x 3, without b2) precomputed by asrx_gemm_wn_router; out is stored
// fp32 (out_bf16 = 0) or bf16 (1).
extern "C" int asrx_abby_fwd_logits2(const float* x, const float* logits, const float* b2, void* out, int out_bf16,
                                     float* ys, int* idx, int64_t rows, int64_t d, int64_t L, int64_t H,
                                     int64_t sid_base, uint32_t key, int use_noise, const float* tw,
                                     const float* tb, float* tc, hipStream_t stream) {
  ASRX_REQUIRE(!tw || d >= 128, "AbbyNormal: the fused tgate cs needs d >= 128");
  ASRX_REQUIRE(d % 64 == 0 && d >= 64 && d <= 1024, "AbbyNormal: d=%ld must be a multiple of 64 in [64,1024]",
               (long)d);
  if (rows == 0) return 0;
  const int E = (int)(d / 64);
  AbbyGeom g = make_geom(rows, d, L, H, sid_base, key, use_noise);
  g.cond = g_cond_record;
  const unsigned grid = (unsigned)std::min<int64_t>((rows + ABBY_WAVES - 1) / ABBY_WAVES, 4096);
  if (d == 64) {
    const unsigned g64 = (unsigned)std::min<int64_t>((rows + 4 * ABBY_WAVES - 1) / (4 * ABBY_WAVES), 4096);
    if (out_bf16)
      abby_fwd64_kernel<unsigned short><<<g64, 64 * ABBY_WAVES, 0, stream>>>(x, nullptr, nullptr, b2,
                                                                           (unsigned short*)out, ys, idx, g, logits);
    else
      abby_fwd64_kernel<float><<<g64, 64 * ABBY_WAVES, 0, stream>>>(x, nullptr, nullptr, b2, (float*)out, ys, idx, g,
                                                                  logits);
    ASRX_LAUNCHED("asrx_abby_fwd_logits");
  }
  if (out_bf16) {
    ABBY_DISPATCH_T(abby_fwd_kernel, unsigned short, x, nullptr, nullptr, b2, (unsigned short*)out, ys, idx, g, logits,
                    tw, tb, tc);
  } else {
    ABBY_DISPATCH_T(abby_fwd_kernel, float, x, nullptr, nullptr, b2, (float*)out, ys, idx, g, logits, tw, tb, tc);
  }
  ASRX_LAUNCHED("asrx_abby_fwd_logits");
}

// asrx_abby_fwd2 (logits NULL) / asrx_abby_fwd_logits2 (logits given, hpre / W2 unused) that also writes
// the input rows' L2 norms to nrm (rows,) when nrm is non-NULL (d >= 128).
extern "C" int asrx_abby_fwd3(const float* x, const float* hpre, const float* W2, const float* logits,
                              const float* b2, void* out, int out_bf16, float* ys, int* idx, int64_t rows, int64_t d,
                              int64_t L, int64_t H, int64_t sid_base, uint32_t key, int use_noise, const float* tw,
                              const float* tb, float* tc, float* nrm, hipStream_t stream) {
  if (!nrm) {
    if (logits)
      return asrx_abby_fwd_logits2(x, logits, b2, out, out_bf16, ys, idx, rows, d, L, H, sid_base, key, use_noise, tw,
                                   tb, tc, stream);
    return asrx_abby_fwd2(x, hpre, W2, b2, out, out_bf16, ys, idx, rows, d, L, H, sid_base, key, use_noise, tw, tb,
                          tc, stream);
  }
  ASRX_REQUIRE(!tw || d >= 128, "AbbyNormal: the fused tgate cs needs d >= 128");
  ASRX_REQUIRE(d % 64 == 0 && d >= 128 && d <= 1024,
               "asrx_abby_fwd3: d=%ld must be a multiple of 64 in [128,1024] with a norm output", (long)d);
  ASRX_REQUIRE(logits || (hpre && W2), "asrx_abby_fwd3: logits or hpre/W2");
  if (rows == 0) return 0;
  const int E = (int)(d / 64);
  AbbyGeom g = make_geom(rows, d, L, H, sid_base, key, use_noise);
  g.cond = g_cond_record;
  g.nrm = nrm;
  const float* hp = logits ? nullptr : hpre;
  const float* w2 = logits ? nullptr : W2;
  const unsigned grid = (unsigned)std::min<int64_t>((rows + ABBY_WAVES - 1) / ABBY_WAVES, 4096);
  if (out_bf16) {
    ABBY_DISPATCH_T(abby_fwd_kernel, unsigned short, x, hp, w2, b2, (unsigned short*)out, ys, idx, g, logits, tw, tb,
                    tc);
  } else {
    ABBY_DISPATCH_T(abby_fwd_kernel, float, x, hp, w2, b2, (float*)out, ys, idx, g, logits, tw, tb, tc);
  }
  ASRX_LAUNCHED("asrx_abby_fwd3");
}

// asrx_abby_fwd_logits2 / asrx_abby_fwd2 (hpre given, logits NULL) with a residual input: out = res +
// AbbyNormal(x) (fp32 out, d >= 128).
extern "C" int asrx_abby_fwd_res(const float* x, const float* hpre, const float* W2, const float* logits,
                                 const float* b2, const float* res, float* out, float* ys, int* idx, int64_t rows,
                                 int64_t d, int64_t L, int64_t H, int64_t sid_base, uint32_t key, int use_noise,
                                 hipStream_t stream) {
  ASRX_REQUIRE(d % 64 == 0 && d >= 128 && d <= 1024, "asrx_abby_fwd_res: d=%ld must be a multiple of 64 in [128,1024]",
               (long)d);
  ASRX_REQUIRE(res && res != out && (logits || (hpre && W2)), "asrx_abby_fwd_res: res (!= out) and logits or hpre/W2");
  if (rows == 0) return 0;
  const int E = (int)(d / 64);
  AbbyGeom g = make_geom(rows, d, L, H, sid_base, key, use_noise);
  g.cond = g_cond_record;
  g.res = res;
  const unsigned grid = (unsigned)std::min<int64_t>((rows + ABBY_WAVES - 1) / ABBY_WAVES, 4096);
  ABBY_DISPATCH_T(abby_fwd_kernel, float, x, logits ? nullptr : hpre, logits ? nullptr : W2, b2, out, ys, idx, g,
                  logits, nullptr, nullptr, nullptr);
  ASRX_LAUNCHED("asrx_abby_fwd_res");
}

extern "C" int asrx_abby_fwd_logits(const float* x, const float* logits, const float* b2, float* out, float* ys,
                                    int* idx, int64_t rows, int64_t d, int64_t L, int64_t H, int64_t sid_base,
                                    uint32_t key, int use_noise, hipStream_t stream) {
  return asrx_abby_fwd_logits2(x, logits, b2, out, 0, ys, idx, rows, d, L, H, sid_base, key, use_noise, nullptr,
                               nullptr, nullptr, stream);
}

// dW2 / db2 are accumulated (caller zeroes them).  dx (acc == 0) and dhpre are overwritten; acc != 0
// adds x's gradient into dx.
extern "C" int asrx_abby_bwd2(const float* dout, const float* x, const float* hpre, const float* W2,
                              const float* ys, const int* idx, float* dx, float* dhpre, float* dW2, float* db2,
                              int64_t rows, int64_t d, int acc, hipStream_t stream) {
  ASRX_REQUIRE(d % 64 == 0 && d >= 64 && d <= 1024, "AbbyNormal: d=%ld must be a multiple of 64 in [64,1024]",
               (long)d);
  if (rows == 0) return 0;
  const int E = (int)(d / 64);
  AbbyGeom g = make_geom(rows, d, 1, 1, 0, 0, 0);
  g.acc = acc;
  const unsigned grid = (unsigned)std::min<int64_t>((rows + ABBY_WAVES - 1) / ABBY_WAVES, 1024);
  if (d == 64) {
    const unsigned g64 = (unsigned)std::min<int64_t>((rows + 4 * ABBY_WAVES - 1) / (4 * ABBY_WAVES), 1024);
    abby_bwd64_kernel<<<g64, 64 * ABBY_WAVES, 0, stream>>>(dout, x, hpre, W2, ys, idx, dx, dhpre, dW2, db2, g);
    ASRX_LAUNCHED("asrx_abby_bwd2");
  }
  ABBY_DISPATCH(abby_bwd_kernel, dout, x, hpre, W2, ys, idx, dx, dhpre, dW2, db2, g);
  ASRX_LAUNCHED("asrx_abby_bwd2");
}

extern "C" int asrx_abby_bwd(const float* dout, const float* x, const float* hpre, const float* W2,
                             const float* ys, const int* idx, float* dx, float* dhpre, float* dW2, float* db2,
                             int64_t rows, int64_t d, hipStream_t stream) {
  return asrx_abby_bwd2(dout, x, hpre, W2, ys, idx, dx, dhpre, dW2, db2, rows, d, 0, stream);
}

// Decision recorder for the parity tests: while buf != NULL, every AbbyNormal forward writes mode 2's
// per-feature max-vs-avg choice of its rows that picked mode 2 into buf (rows x d bytes, caller-zeroed,
// large enough for the next call); NULL turns it off.  Not for graph capture.
extern "C" int asrx_abby_record_cond(unsigned char* buf) {
  g_cond_record = buf;
  return 0;
}

ASRX_NOISE_EPOCH_SETTER(asrx_set_noise_epoch_abby)
