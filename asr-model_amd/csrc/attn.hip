// Flash attention for F.scaled_dot_product_attention(q, k, v, is_causal) as called at model.py:307
// (after rotary and the per-head AbbyNormal): head dim HD = 64 or 128, default scale 1/sqrt(HD),
// non-causal (audio self / cross / text cross) or causal with top-left alignment (the masked text
// self call), Lq != Lk, ragged tails.  Layout: q/k/v/o are (B, L, H, HD) with arbitrary batch/seq/
// head strides (the natural output of the q / kv projections, no transposes); lse is (B, H, Lq).
//
// This file holds the entry points and the exact-fp32 PARITY-mode kernels (v_mfma_f32_16x16x4f32,
// no rounding of any operand); the perf modes live in attn_mf.hip (bf16) and attn_f8.hip (fp8 QK^T).
//
// Parity kernels use the accurate expf (not __expf): the model's scores reach ~1e3-1e4 (rotary scales q/k by
// the source row norm), where the fast exp's argument rounding is visible in the whole-model parity.
// Parity kernels: workgroup = 4 waves x 16 rows = 64 rows of one (b, h).  Every wave keeps the
// A-operand fragments of its own 16 rows in registers for the whole sweep (HD/4 floats per lane per
// operand: Q in the forward and dQ kernels, K and V in the dK/dV kernel); the swept operand is
// staged 64 rows at a time in LDS, row-major with a 4-float pad, and read transposed where a
// product contracts over its rows (V in P V, dO / Q in dV / dK, K in dQ), so no transposed copy
// is staged.  P and dS go through a per-wave [16][64] LDS tile into the second product.
// Forward: S = Q K^T, online softmax with running (m, l) per row, O += P V; saves lse = m + log l.
// Backward (FA2 recompute, no atomics): dK/dV kernel (workgroup per 64 keys sweeping query tiles)
// and dQ kernel (workgroup per 64 queries sweeping key tiles), delta = rowsum(dO * O) precomputed.
#include "common.h"
#include <cstdlib>

namespace asrx {

constexpr int ATILE = 64;       // rows per tile (queries or keys)
constexpr int PST = ATILE + 4;  // row stride of the per-wave P / dS tiles

struct AttnStrides {
  int64_t b, l, h;
};

template <int HD>
struct F32T {
  static constexpr int S = HD + 4;  // LDS row stride of a staged [64][HD] tile
  static constexpr int NK = HD / 4; // k-steps of a d-contraction (16x16x4)
  static constexpr int NB = HD / 16; // 16-wide output blocks over d
};

// Stage a 64 x HD fp32 tile (rows r0.., ragged to `rows`, zero past it) into LDS row-major.
template <int HD>
__device__ __forceinline__ void stage_f32(float* dst, const float* src, AttnStrides st, int64_t r0, int64_t rows) {
  constexpr int S = F32T<HD>::S, C4 = HD / 4;
#pragma unroll
  for (int i = 0; i < ATILE * C4 / 256; ++i) {
    const int qd = threadIdx.x + 256 * i;
    const int r = qd / C4, d4 = (qd % C4) * 4;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (r0 + r < rows) v = *reinterpret_cast<const float4*>(src + (r0 + r) * st.l + d4);
    *reinterpret_cast<float4*>(dst + r * S + d4) = v;
  }
}

// A fragments of one row for a d-contraction: f[ks] = X[row][4 ks + lk] (zero past `rows`)
template <int HD>
__device__ __forceinline__ void load_frag(float (&f)[HD / 4], const float* base, int64_t stride_l, int64_t row,
                                          int64_t rows, int lk) {
#pragma unroll
  for (int ks = 0; ks < HD / 4; ++ks) f[ks] = row < rows ? base[row * stride_l + 4 * ks + lk] : 0.f;
}

// acc (16 register rows x 16 LDS rows b0..) += F . X[b0 + lc]^T over the HD dims
template <int HD>
__device__ __forceinline__ void dot_d(f32x4& acc, const float (&f)[HD / 4], const float* X, int b0, int lr, int lk) {
  constexpr int S = F32T<HD>::S;
#pragma unroll
  for (int ks = 0; ks < HD / 4; ++ks) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(f[ks], X[(b0 + lr) * S + 4 * ks + lk], acc, 0, 0, 0);
}

// acc[nb] (16 rows of the per-wave tile T x 16 d) += T[16][64] . X[64][d] (contraction over X's rows)
template <int HD>
__device__ __forceinline__ void dot_rows_t(f32x4 (&acc)[HD / 16], const float* T, const float* X, int lr, int lk) {
  constexpr int S = F32T<HD>::S;
#pragma unroll
  for (int kk = 0; kk < ATILE / 4; ++kk) {
    const float a = T[lr * PST + 4 * kk + lk];
#pragma unroll
    for (int nb = 0; nb < HD / 16; ++nb)
      acc[nb] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, X[(4 * kk + lk) * S + 16 * nb + lr], acc[nb], 0, 0, 0);
  }
}

// ------------------------------------------------------------------------------------ forward
template <int HD>
__global__ __launch_bounds__(256) void attn_fwd_f32_kernel(const float* __restrict__ q, const float* __restrict__ k,
                                                           const float* __restrict__ v, float* __restrict__ o,
                                                           float* __restrict__ lse, AttnStrides sq, AttnStrides sk,
                                                           AttnStrides sv, AttnStrides so, int64_t H, int64_t Lq,
                                                           int64_t Lk, int causal, float scale) {
  constexpr int S = F32T<HD>::S;
  __shared__ __attribute__((aligned(16))) float Ks[ATILE * S];
  __shared__ __attribute__((aligned(16))) float Vs[ATILE * S];
  __shared__ __attribute__((aligned(16))) float Ps[4][16 * PST];

  const int b = blockIdx.z, h = blockIdx.y;
  const int64_t q0 = (int64_t)blockIdx.x * ATILE;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int lc = lane & 15, lk = lane >> 4, lr4 = lk * 4;
  const float* kb = k + b * sk.b + h * sk.h;
  const float* vb = v + b * sv.b + h * sv.h;
  const int64_t qw = q0 + wid * 16;  // first query row of this wave

  float qa[HD / 4];
  load_frag<HD>(qa, q + b * sq.b + h * sq.h, sq.l, qw + lc, Lq, lk);

  f32x4 acc[HD / 16];
#pragma unroll
  for (int n = 0; n < HD / 16; ++n) acc[n] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m[4], l[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    m[r] = -1e30f;
    l[r] = 0.f;
  }
  int64_t kend = Lk;
  if (causal) kend = min(Lk, q0 + ATILE);
  for (int64_t k0 = 0; k0 < kend; k0 += ATILE) {
    __syncthreads();
    stage_f32<HD>(Ks, kb, sk, k0, Lk);
    stage_f32<HD>(Vs, vb, sv, k0, Lk);
    __syncthreads();
    f32x4 s[4];
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      s[n] = f32x4{0.f, 0.f, 0.f, 0.f};
      dot_d<HD>(s[n], qa, Ks, n * 16, lc, lk);
    }
    float tmax[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) tmax[r] = -1e30f;
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      const int64_t key = k0 + n * 16 + lc;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t qi = qw + lr4 + r;
        float val = s[n][r] * scale;
        if (key >= Lk || (causal && key > qi)) val = -INFINITY;
        s[n][r] = val;
        tmax[r] = fmaxf(tmax[r], val);
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
#pragma unroll
      for (int off = 1; off < 16; off <<= 1) tmax[r] = fmaxf(tmax[r], __shfl_xor(tmax[r], off, 64));
    }
    float alpha[4], rs[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float mn = fmaxf(m[r], tmax[r]);
      alpha[r] = expf(m[r] - mn);
      m[r] = mn;
      rs[r] = 0.f;
    }
    float* P = Ps[wid];
#pragma unroll
    for (int n = 0; n < 4; ++n) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = expf(s[n][r] - m[r]);
        rs[r] += p;
        P[(lr4 + r) * PST + n * 16 + lc] = p;
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
#pragma unroll
      for (int off = 1; off < 16; off <<= 1) rs[r] += __shfl_xor(rs[r], off, 64);
      l[r] = l[r] * alpha[r] + rs[r];
    }
#pragma unroll
    for (int n = 0; n < HD / 16; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[n][r] *= alpha[r];
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    dot_rows_t<HD>(acc, P, Vs, lc, lk);
    __builtin_amdgcn_wave_barrier();  // the next tile's P writes wait for these reads
  }
  float* ob = o + b * so.b + h * so.h;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int64_t qi = qw + lr4 + r;
    if (qi >= Lq) continue;
    const float inv = 1.0f / l[r];
#pragma unroll
    for (int n = 0; n < HD / 16; ++n) ob[qi * so.l + n * 16 + lc] = acc[n][r] * inv;
    if (lc == 0) lse[((int64_t)b * H + h) * Lq + qi] = m[r] + logf(l[r]);
  }
}

__device__ __forceinline__ float ld_f(const float* p) { return *p; }
__device__ __forceinline__ float ld_f(const unsigned short* p) {
  return __uint_as_float((unsigned)*p << 16);
}

// delta[b,h,i] = sum_d dO[b,i,h,d] * O[b,i,h,d]   (one wave per row, HD/64 elements per lane);
// o / dO stored fp32 or bf16 (unsigned short).  RD (bf16 mode): dO rounded to bf16 first, as the backward's
// dP = dO V^T MFMA sees it -- dS = P (dP - delta) relies on sum_j P_ij dP_ij == delta_i, and an fp32
// delta against a bf16 dP leaves a systematic row error that dominates dQ / dK where the values barely
// vary over the keys
template <int HD, typename TO = float, typename TD = float, bool RD = false>
__global__ __launch_bounds__(256) void attn_delta_kernel(const TO* __restrict__ o, const TD* __restrict__ dO,
                                                         float* __restrict__ delta, AttnStrides so, AttnStrides sd,
                                                         int64_t B, int64_t H, int64_t Lq) {
  const int lane = threadIdx.x & 63;
  const int64_t rows = B * H * Lq;
  for (int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); r < rows; r += (int64_t)gridDim.x * 4) {
    const int64_t i = r % Lq, bh = r / Lq, hh = bh % H, bb = bh / H;
    float s = 0.f;
#pragma unroll
    for (int e = 0; e < HD / 64; ++e) {
      float g = ld_f(dO + bb * sd.b + i * sd.l + hh * sd.h + 64 * e + lane);
      if constexpr (RD) g = (float)(__bf16)g;
      s += ld_f(o + bb * so.b + i * so.l + hh * so.h + 64 * e + lane) * g;
    }
    s = wave_sum(s);
    if (lane == 0) delta[r] = s;
  }
}

// ------------------------------------------------------------------------------------ dK / dV
template <int HD>
__global__ __launch_bounds__(256) void attn_bwd_dkdv_f32_kernel(
    const float* __restrict__ q, const float* __restrict__ k, const float* __restrict__ v,
    const float* __restrict__ dO, const float* __restrict__ lse, const float* __restrict__ delta,
    float* __restrict__ dk, float* __restrict__ dv, AttnStrides sq, AttnStrides sk, AttnStrides sv, AttnStrides sd,
    AttnStrides sdk, AttnStrides sdv, int64_t H, int64_t Lq, int64_t Lk, int causal, float scale) {
  constexpr int S = F32T<HD>::S;
  __shared__ __attribute__((aligned(16))) float Qs[ATILE * S];
  __shared__ __attribute__((aligned(16))) float dOs[ATILE * S];
  __shared__ __attribute__((aligned(16))) float Pst[4][16 * PST];
  __shared__ __attribute__((aligned(16))) float dSt[4][16 * PST];
  __shared__ float lse_s[ATILE], del_s[ATILE];

  const int b = blockIdx.z, h = blockIdx.y;
  const int64_t k0 = (int64_t)blockIdx.x * ATILE;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int lc = lane & 15, lk = lane >> 4, lr4 = lk * 4;
  const float* qb = q + b * sq.b + h * sq.h;
  const float* gb = dO + b * sd.b + h * sd.h;
  const float* lb = lse + ((int64_t)b * H + h) * Lq;
  const float* db_ = delta + ((int64_t)b * H + h) * Lq;
  const int64_t kw = k0 + wid * 16;

  float ka[HD / 4], va[HD / 4];
  load_frag<HD>(ka, k + b * sk.b + h * sk.h, sk.l, kw + lc, Lk, lk);
  load_frag<HD>(va, v + b * sv.b + h * sv.h, sv.l, kw + lc, Lk, lk);

  f32x4 adk[HD / 16], adv[HD / 16];
#pragma unroll
  for (int n = 0; n < HD / 16; ++n) {
    adk[n] = f32x4{0.f, 0.f, 0.f, 0.f};
    adv[n] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const int64_t qstart = causal ? (k0 / ATILE) * ATILE : 0;
  for (int64_t q0 = qstart; q0 < Lq; q0 += ATILE) {
    __syncthreads();
    stage_f32<HD>(Qs, qb, sq, q0, Lq);
    stage_f32<HD>(dOs, gb, sd, q0, Lq);
    if (threadIdx.x < ATILE) {
      const int64_t qi = q0 + threadIdx.x;
      lse_s[threadIdx.x] = qi < Lq ? lb[qi] : 0.f;
      del_s[threadIdx.x] = qi < Lq ? db_[qi] : 0.f;
    }
    __syncthreads();
    float* P = Pst[wid];
    float* D = dSt[wid];
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      f32x4 st = f32x4{0.f, 0.f, 0.f, 0.f};
      f32x4 dp = f32x4{0.f, 0.f, 0.f, 0.f};
      dot_d<HD>(st, ka, Qs, n * 16, lc, lk);   // S^T: rows = keys, cols = queries
      dot_d<HD>(dp, va, dOs, n * 16, lc, lk);  // dP^T
      const int qcol = n * 16 + lc;
      const int64_t qi = q0 + qcol;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t key = kw + lr4 + r;
        float p = expf(st[r] * scale - lse_s[qcol]);
        if (qi >= Lq || key >= Lk || (causal && key > qi)) p = 0.f;
        P[(lr4 + r) * PST + qcol] = p;
        D[(lr4 + r) * PST + qcol] = p * (dp[r] - del_s[qcol]);
      }
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    dot_rows_t<HD>(adv, P, dOs, lc, lk);  // dV += P^T-rows . dO
    dot_rows_t<HD>(adk, D, Qs, lc, lk);   // dK += dS^T-rows . Q
  }
  float* dkb = dk + b * sdk.b + h * sdk.h;
  float* dvb = dv + b * sdv.b + h * sdv.h;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int64_t key = kw + lr4 + r;
    if (key >= Lk) continue;
#pragma unroll
    for (int n = 0; n < HD / 16; ++n) {
      dkb[key * sdk.l + n * 16 + lc] = adk[n][r] * scale;
      dvb[key * sdv.l + n * 16 + lc] = adv[n][r];
    }
  }
}

// ------------------------------------------------------------------------------------ dQ
template <int HD>
__global__ __launch_bounds__(256) void attn_bwd_dq_f32_kernel(
    const float* __restrict__ q, const float* __restrict__ k, const float* __restrict__ v,
    const float* __restrict__ dO, const float* __restrict__ lse, const float* __restrict__ delta,
    float* __restrict__ dq, AttnStrides sq, AttnStrides sk, AttnStrides sv, AttnStrides sd, AttnStrides sdq,
    int64_t H, int64_t Lq, int64_t Lk, int causal, float scale) {
  constexpr int S = F32T<HD>::S;
  __shared__ __attribute__((aligned(16))) float Ks[ATILE * S];
  __shared__ __attribute__((aligned(16))) float Vs[ATILE * S];
  __shared__ __attribute__((aligned(16))) float dSs[4][16 * PST];

  const int b = blockIdx.z, h = blockIdx.y;
  const int64_t q0 = (int64_t)blockIdx.x * ATILE;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int lc = lane & 15, lk = lane >> 4, lr4 = lk * 4;
  const float* kb = k + b * sk.b + h * sk.h;
  const float* vb = v + b * sv.b + h * sv.h;
  const float* lb = lse + ((int64_t)b * H + h) * Lq;
  const float* db_ = delta + ((int64_t)b * H + h) * Lq;
  const int64_t qw = q0 + wid * 16;

  float qa[HD / 4], ga[HD / 4];
  load_frag<HD>(qa, q + b * sq.b + h * sq.h, sq.l, qw + lc, Lq, lk);
  load_frag<HD>(ga, dO + b * sd.b + h * sd.h, sd.l, qw + lc, Lq, lk);
  float lsev[4], delv[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int64_t qi = qw + lr4 + r;
    lsev[r] = qi < Lq ? lb[qi] : 0.f;
    delv[r] = qi < Lq ? db_[qi] : 0.f;
  }
  f32x4 adq[HD / 16];
#pragma unroll
  for (int n = 0; n < HD / 16; ++n) adq[n] = f32x4{0.f, 0.f, 0.f, 0.f};
  int64_t kend = Lk;
  if (causal) kend = min(Lk, q0 + ATILE);
  for (int64_t k0 = 0; k0 < kend; k0 += ATILE) {
    __syncthreads();
    stage_f32<HD>(Ks, kb, sk, k0, Lk);
    stage_f32<HD>(Vs, vb, sv, k0, Lk);
    __syncthreads();
    float* D = dSs[wid];
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      f32x4 s = f32x4{0.f, 0.f, 0.f, 0.f};
      f32x4 dp = f32x4{0.f, 0.f, 0.f, 0.f};
      dot_d<HD>(s, qa, Ks, n * 16, lc, lk);
      dot_d<HD>(dp, ga, Vs, n * 16, lc, lk);
      const int64_t key = k0 + n * 16 + lc;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t qi = qw + lr4 + r;
        float p = expf(s[r] * scale - lsev[r]);
        if (qi >= Lq || key >= Lk || (causal && key > qi)) p = 0.f;
        D[(lr4 + r) * PST + n * 16 + lc] = p * (dp[r] - delv[r]);
      }
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    dot_rows_t<HD>(adq, D, Ks, lc, lk);
    __builtin_amdgcn_wave_barrier();
  }
  float* dqb = dq + b * sdq.b + h * sdq.h;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int64_t qi = qw + lr4 + r;
    if (qi >= Lq) continue;
#pragma unroll
    for (int n = 0; n < HD / 16; ++n) dqb[qi * sdq.l + n * 16 + lc] = adq[n][r] * scale;
  }
}

}  // namespace asrx

using namespace asrx;

static bool attn_ok(const int64_t* st) { return st[0] % 4 == 0 && st[1] % 4 == 0 && st[2] % 4 == 0; }

// Strides are passed as int64[3] = {batch, seq, head} in elements; the head-dim stride must be 1.
namespace asrx {
int attn_fwd_mf(int io, const void* q, const int64_t* sq, const void* k, const int64_t* sk, const void* v,
                const int64_t* sv, void* o, const int64_t* so, float* lse, int64_t B, int64_t H, int64_t Lq,
                int64_t Lk, int64_t hd, int causal, float scale, hipStream_t stream);
int attn_bwd_mf(int io, const void* q, const int64_t* sq, const void* k, const int64_t* sk, const void* v,
                const int64_t* sv, const void* dO, const int64_t* sd, const float* lse, const float* delta,
                float* dq, const int64_t* sdq, float* dk, const int64_t* sdk, float* dv, const int64_t* sdv,
                int64_t B, int64_t H, int64_t Lq, int64_t Lk, int64_t hd, int causal, float scale,
                hipStream_t stream);
int attn_fwd_f8(const float* q, const int64_t* sq, const float* k, const int64_t* sk, const float* v,
                const int64_t* sv, float* o, const int64_t* so, float* lse, int64_t B, int64_t H, int64_t Lq,
                int64_t Lk, int64_t hd, int causal, float scale, hipStream_t stream);
constexpr int PREC_FP8ATT = 2;  // forward only: e4m3 QK^T (attn_f8.hip)
}

template <int HD>
static void attn_fwd_f32(const float* q, AttnStrides Sq, const float* k, AttnStrides Sk, const float* v,
                         AttnStrides Sv, float* o, AttnStrides So, float* lse, int64_t B, int64_t H, int64_t Lq,
                         int64_t Lk, int causal, float scale, hipStream_t stream) {
  dim3 g((unsigned)((Lq + ATILE - 1) / ATILE), (unsigned)H, (unsigned)B);
  attn_fwd_f32_kernel<HD><<<g, 256, 0, stream>>>(q, k, v, o, lse, Sq, Sk, Sv, So, H, Lq, Lk, causal, scale);
}

template <int HD>
static void attn_bwd_f32(const float* q, AttnStrides Sq, const float* k, AttnStrides Sk, const float* v,
                         AttnStrides Sv, const float* dO, AttnStrides Sd, const float* lse, const float* delta,
                         float* dq, AttnStrides Sdq, float* dk, AttnStrides Sdk, float* dv, AttnStrides Sdv,
                         int64_t B, int64_t H, int64_t Lq, int64_t Lk, int causal, float scale, hipStream_t stream) {
  dim3 gk((unsigned)((Lk + ATILE - 1) / ATILE), (unsigned)H, (unsigned)B);
  dim3 gq((unsigned)((Lq + ATILE - 1) / ATILE), (unsigned)H, (unsigned)B);
  attn_bwd_dkdv_f32_kernel<HD><<<gk, 256, 0, stream>>>(q, k, v, dO, lse, delta, dk, dv, Sq, Sk, Sv, Sd, Sdk, Sdv, H, Lq,
                                                       Lk, causal, scale);
  attn_bwd_dq_f32_kernel<HD><<<gq, 256, 0, stream>>>(q, k, v, dO, lse, delta, dq, Sq, Sk, Sv, Sd, Sdq, H, Lq, Lk,
                                                     causal, scale);
}

extern "C" int asrx_attn_fwd2(int prec, int io, const void* q_, const int64_t* sq, const void* k_, const int64_t* sk,
                              const void* v_, const int64_t* sv, void* o_, const int64_t* so, float* lse, int64_t B,
                              int64_t H, int64_t Lq, int64_t Lk, int64_t hd, int causal, float scale,
                              hipStream_t stream) {
  const float *q = (const float*)q_, *k = (const float*)k_, *v = (const float*)v_;
  float* o = (float*)o_;
  ASRX_REQUIRE(io == 0 || prec == PREC_BF16, "attention: bf16 storage (io %d) is a bf16-mode layout", io);
  ASRX_REQUIRE(hd == 64 || hd == 128, "attention: head dim %ld unsupported (64 or 128)", (long)hd);
  ASRX_REQUIRE(attn_ok(sq) && attn_ok(sk) && attn_ok(sv) && attn_ok(so), "attention: strides must be multiples of 4");
  ASRX_REQUIRE(H < 65536 && B < 65536, "attention: grid too large");
  if (B * H * Lq == 0) return 0;
  ASRX_REQUIRE(Lk > 0, "attention: empty key sequence");
  AttnStrides Sq{sq[0], sq[1], sq[2]}, Sk{sk[0], sk[1], sk[2]}, Sv{sv[0], sv[1], sv[2]}, So{so[0], so[1], so[2]};
  const bool al16 = (((uintptr_t)q | (uintptr_t)k | (uintptr_t)v | (uintptr_t)o) & 15) == 0;
  ASRX_REQUIRE(prec == PREC_F32 || prec == PREC_BF16 || prec == PREC_FP8ATT, "attention: bad precision %d", prec);
  ASRX_REQUIRE(prec == PREC_F32 || al16, "attention: bf16/fp8 modes need 16-byte aligned q/k/v/o");
  if (prec == PREC_FP8ATT)
    attn_fwd_f8(q, sq, k, sk, v, sv, o, so, lse, B, H, Lq, Lk, hd, causal, scale, stream);
  else if (prec == PREC_BF16)
    attn_fwd_mf(io, q, sq, k, sk, v, sv, o, so, lse, B, H, Lq, Lk, hd, causal, scale, stream);
  else if (hd == 64)
    attn_fwd_f32<64>(q, Sq, k, Sk, v, Sv, o, So, lse, B, H, Lq, Lk, causal, scale, stream);
  else
    attn_fwd_f32<128>(q, Sq, k, Sk, v, Sv, o, So, lse, B, H, Lq, Lk, causal, scale, stream);
  ASRX_LAUNCHED("asrx_attn_fwd");
}

extern "C" int asrx_attn_fwd(int prec, const float* q, const int64_t* sq, const float* k, const int64_t* sk,
                             const float* v, const int64_t* sv, float* o, const int64_t* so, float* lse, int64_t B,
                             int64_t H, int64_t Lq, int64_t Lk, int64_t hd, int causal, float scale,
                             hipStream_t stream) {
  return asrx_attn_fwd2(prec, 0, q, sq, k, sk, v, sv, o, so, lse, B, H, Lq, Lk, hd, causal, scale, stream);
}

// delta_ws: workspace of B*H*Lq floats.
extern "C" int asrx_attn_bwd2(int prec, int io, const void* q_, const int64_t* sq, const void* k_, const int64_t* sk,
                              const void* v_, const int64_t* sv, const void* o_, const int64_t* so, const void* dO_,
                              const int64_t* sd, const float* lse, float* delta_ws, float* dq, const int64_t* sdq,
                              float* dk, const int64_t* sdk, float* dv, const int64_t* sdv, int64_t B, int64_t H,
                              int64_t Lq, int64_t Lk, int64_t hd, int causal, float scale, hipStream_t stream) {
  const float *q = (const float*)q_, *k = (const float*)k_, *v = (const float*)v_, *o = (const float*)o_;
  const float* dO = (const float*)dO_;
  ASRX_REQUIRE(io == 0 || prec == PREC_BF16, "attention backward: bf16 storage (io %d) is a bf16-mode layout", io);
  ASRX_REQUIRE(prec == PREC_F32 || prec == PREC_BF16, "attention backward: precision %d (fp8 is forward only)", prec);
  ASRX_REQUIRE(hd == 64 || hd == 128, "attention: head dim %ld unsupported (64 or 128)", (long)hd);
  ASRX_REQUIRE(attn_ok(sq) && attn_ok(sk) && attn_ok(sv) && attn_ok(sd) && attn_ok(sdq) && attn_ok(sdk) &&
                   attn_ok(sdv),
               "attention: strides must be multiples of 4");
  if (B * H * Lq == 0) return 0;
  ASRX_REQUIRE(Lk > 0, "attention: empty key sequence");
  AttnStrides Sq{sq[0], sq[1], sq[2]}, Sk{sk[0], sk[1], sk[2]}, Sv{sv[0], sv[1], sv[2]}, So{so[0], so[1], so[2]};
  AttnStrides Sd{sd[0], sd[1], sd[2]}, Sdq{sdq[0], sdq[1], sdq[2]}, Sdk{sdk[0], sdk[1], sdk[2]},
      Sdv{sdv[0], sdv[1], sdv[2]};
  const int64_t rows = B * H * Lq;
  const unsigned gd = (unsigned)std::min<int64_t>((rows + 3) / 4, 8192);
#define ASRX_DL(HDV, TO, TD, RD) \
  attn_delta_kernel<HDV, TO, TD, RD><<<gd, 256, 0, stream>>>((const TO*)o_, (const TD*)dO_, delta_ws, So, Sd, B, H, Lq)
  const int dsel = ((io >> 1) & 1) | ((io >> 1) & 2);  // bit 0: o bf16, bit 1: dO bf16
  const bool rd = prec == PREC_BF16;                  // fp32 dO rounded as the bf16 dP MFMA sees it
  if (hd == 64) {
    switch (dsel) {
      case 0: if (rd) ASRX_DL(64, float, float, true); else ASRX_DL(64, float, float, false); break;
      case 1: if (rd) ASRX_DL(64, unsigned short, float, true); else ASRX_DL(64, unsigned short, float, false); break;
      case 2: ASRX_DL(64, float, unsigned short, false); break;
      default: ASRX_DL(64, unsigned short, unsigned short, false); break;
    }
  } else {
    switch (dsel) {
      case 0: if (rd) ASRX_DL(128, float, float, true); else ASRX_DL(128, float, float, false); break;
      case 1: if (rd) ASRX_DL(128, unsigned short, float, true); else ASRX_DL(128, unsigned short, float, false); break;
      case 2: ASRX_DL(128, float, unsigned short, false); break;
      default: ASRX_DL(128, unsigned short, unsigned short, false); break;
    }
  }
#undef ASRX_DL
  const bool al16 = (((uintptr_t)q | (uintptr_t)k | (uintptr_t)v | (uintptr_t)dO | (uintptr_t)dq | (uintptr_t)dk |
                       (uintptr_t)dv) & 15) == 0;
  ASRX_REQUIRE(prec == PREC_F32 || al16, "attention backward: bf16 mode needs 16-byte aligned tensors");
  if (prec == PREC_BF16)
    attn_bwd_mf(io, q, sq, k, sk, v, sv, dO, sd, lse, delta_ws, dq, sdq, dk, sdk, dv, sdv, B, H, Lq, Lk, hd, causal,
                scale, stream);
  else if (hd == 64)
    attn_bwd_f32<64>(q, Sq, k, Sk, v, Sv, dO, Sd, lse, delta_ws, dq, Sdq, dk, Sdk, dv, Sdv, B, H, Lq, Lk, causal, scale,
                     stream);
  else
    attn_bwd_f32<128>(q, Sq, k, Sk, v, Sv, dO, Sd, lse, delta_ws, dq, Sdq, dk, Sdk, dv, Sdv, B, H, Lq, Lk, causal,
                      scale, stream);
  ASRX_LAUNCHED("asrx_attn_bwd");
}

extern "C" int asrx_attn_bwd(int prec, const float* q, const int64_t* sq, const float* k, const int64_t* sk,
                             const float* v, const int64_t* sv, const float* o, const int64_t* so, const float* dO,
                             const int64_t* sd, const float* lse, float* delta_ws, float* dq, const int64_t* sdq,
                             float* dk, const int64_t* sdk, float* dv, const int64_t* sdv, int64_t B, int64_t H,
                             int64_t Lq, int64_t Lk, int64_t hd, int causal, float scale, hipStream_t stream) {
  return asrx_attn_bwd2(prec, 0, q, sq, k, sk, v, sv, o, so, dO, sd, lse, delta_ws, dq, sdq, dk, sdk, dv, sdv, B, H, Lq,
                        Lk, hd, causal, scale, stream);
}
