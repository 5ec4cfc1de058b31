// Flash attention for F.scaled_dot_product_attention(q, k, v, is_causal) as called at model.py:307
// (after rotary and the per-head AbbyNormal): head dim 64, default scale 1/sqrt(64), non-causal
// (audio self / cross / text cross) or causal with top-left alignment (the masked text self call),
// Lq != Lk, ragged tails.  Layout: q/k/v/o are (B, L, H, 64) with arbitrary batch/seq/head
// strides (the natural output of the q / kv projections, no transposes); lse is (B, H, Lq).
//
// Forward: one workgroup = 64 query rows of one (b, h), 4 waves x 16 rows.  K/V tiles of 64 keys
// are staged in LDS (K row-major, V transposed), S = Q K^T on MFMA, online softmax with running
// (m, l) per row, P goes through a per-wave LDS tile into the P V MFMA.  Saves lse = m + log l.
// Backward (FA2 recompute, no atomics): dK/dV kernel (workgroup per 64-key tile sweeping query
// tiles) and dQ kernel (workgroup per 64-query tile sweeping key tiles), with
// delta = rowsum(dO * O) precomputed.
//
// PREC_BF16 rounds MFMA operands (Q, K, V, P, dO, dS) to bf16 with fp32 accumulation;
// PREC_F32 uses exact fp32 MFMA (parity mode).
#include "common.h"
#include <cstdlib>

namespace asrx {

constexpr int AHD = 64;   // head dim
constexpr int ATILE = 64; // rows per tile (queries or keys)

template <int PREC>
struct AT;
template <>
struct AT<PREC_BF16> {
  typedef unsigned short T;
  static constexpr int S = AHD + 8;  // LDS row stride (elements) for 64-wide rows
};
template <>
struct AT<PREC_F32> {
  typedef float T;
  static constexpr int S = AHD + 4;
};

__device__ __forceinline__ unsigned short bf(float f) {
  __bf16 h = (__bf16)f;
  return __builtin_bit_cast(unsigned short, h);
}

template <int PREC>
__device__ __forceinline__ typename AT<PREC>::T cvt(float f) {
  if constexpr (PREC == PREC_BF16) return bf(f);
  else return f;
}

// acc (16x16) += A[a0 .. a0+16)[0..64) * B[b0 .. b0+16)[0..64)^T, both row-major in LDS with
// row stride AT<PREC>::S (the contraction runs over the 64 contiguous columns).
template <int PREC>
__device__ __forceinline__ void mma16x64(f32x4& acc, const typename AT<PREC>::T* A, int a0,
                                         const typename AT<PREC>::T* B, int b0) {
  constexpr int S = AT<PREC>::S;
  const int lane = threadIdx.x & 63, lr = lane & 15, lk = lane >> 4;
  if constexpr (PREC == PREC_BF16) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const bf16x8 a = *reinterpret_cast<const bf16x8*>(A + (a0 + lr) * S + ks * 32 + 8 * lk);
      const bf16x8 b = *reinterpret_cast<const bf16x8*>(B + (b0 + lr) * S + ks * 32 + 8 * lk);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc, 0, 0, 0);
    }
  } else {
#pragma unroll
    for (int ks = 0; ks < 16; ++ks) {
      const float a = A[(a0 + lr) * S + ks * 4 + lk];
      const float b = B[(b0 + lr) * S + ks * 4 + lk];
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc, 0, 0, 0);
    }
  }
}

struct AttnStrides {
  int64_t b, l, h;
};

// Stage a 64 x 64 fp32 tile (rows r0.., ragged to `rows`) into LDS as T; row-major (dst[r][d]) or
// transposed (dst[d][r]).  256 threads, 4 float4 each.
template <int PREC, bool TRANS>
__device__ __forceinline__ void stage_tile(typename AT<PREC>::T* dst, const float* src, AttnStrides st, int64_t r0,
                                           int64_t rows) {
  constexpr int S = AT<PREC>::S;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int q = threadIdx.x + 256 * i;
    const int r = q >> 4, d4 = (q & 15) * 4;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (r0 + r < rows) v = *reinterpret_cast<const float4*>(src + (r0 + r) * st.l + d4);
    if (TRANS) {
      dst[(d4 + 0) * S + r] = cvt<PREC>(v.x);
      dst[(d4 + 1) * S + r] = cvt<PREC>(v.y);
      dst[(d4 + 2) * S + r] = cvt<PREC>(v.z);
      dst[(d4 + 3) * S + r] = cvt<PREC>(v.w);
    } else {
      typename AT<PREC>::T* p = dst + r * S + d4;
      p[0] = cvt<PREC>(v.x);
      p[1] = cvt<PREC>(v.y);
      p[2] = cvt<PREC>(v.z);
      p[3] = cvt<PREC>(v.w);
    }
  }
}

// ------------------------------------------------------------------------------------ forward
template <int PREC>
__global__ __launch_bounds__(256) void attn_fwd_kernel(const float* __restrict__ q, const float* __restrict__ k,
                                                       const float* __restrict__ v, float* __restrict__ o,
                                                       float* __restrict__ lse, AttnStrides sq, AttnStrides sk,
                                                       AttnStrides sv, AttnStrides so, int64_t H, int64_t Lq,
                                                       int64_t Lk, int causal, float scale) {
  typedef typename AT<PREC>::T T;
  constexpr int S = AT<PREC>::S;
  __shared__ __attribute__((aligned(16))) T Qs[ATILE * S];
  __shared__ __attribute__((aligned(16))) T Ks[ATILE * S];
  __shared__ __attribute__((aligned(16))) T Vt[AHD * S];
  __shared__ __attribute__((aligned(16))) T Ps[4][16 * S];

  const int b = blockIdx.z, h = blockIdx.y;
  const int64_t q0 = (int64_t)blockIdx.x * ATILE;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int lc = lane & 15, lr4 = (lane >> 4) * 4;
  const float* qb = q + b * sq.b + h * sq.h;
  const float* kb = k + b * sk.b + h * sk.h;
  const float* vb = v + b * sv.b + h * sv.h;

  stage_tile<PREC, false>(Qs, qb, sq, q0, Lq);

  f32x4 acc[4];
#pragma unroll
  for (int n = 0; n < 4; ++n) acc[n] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m[4], l[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    m[r] = -1e30f;
    l[r] = 0.f;
  }
  const int64_t qw = q0 + wid * 16;  // first query row of this wave
  int64_t kend = Lk;
  if (causal) kend = min(Lk, q0 + ATILE);
  for (int64_t k0 = 0; k0 < kend; k0 += ATILE) {
    __syncthreads();
    stage_tile<PREC, false>(Ks, kb, sk, k0, Lk);
    stage_tile<PREC, true>(Vt, vb, sv, k0, Lk);
    __syncthreads();
    f32x4 s[4];
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      s[n] = f32x4{0.f, 0.f, 0.f, 0.f};
      mma16x64<PREC>(s[n], Qs, wid * 16, Ks, n * 16);
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
      alpha[r] = __expf(m[r] - mn);
      m[r] = mn;
      rs[r] = 0.f;
    }
    T* P = Ps[wid];
#pragma unroll
    for (int n = 0; n < 4; ++n) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = __expf(s[n][r] - m[r]);
        rs[r] += p;
        P[(lr4 + r) * S + n * 16 + lc] = cvt<PREC>(p);
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
#pragma unroll
      for (int off = 1; off < 16; off <<= 1) rs[r] += __shfl_xor(rs[r], off, 64);
      l[r] = l[r] * alpha[r] + rs[r];
    }
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[n][r] *= alpha[r];
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
#pragma unroll
    for (int n = 0; n < 4; ++n) mma16x64<PREC>(acc[n], P, 0, Vt, n * 16);
  }
  float* ob = o + b * so.b + h * so.h;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int64_t qi = qw + lr4 + r;
    if (qi >= Lq) continue;
    const float inv = 1.0f / l[r];
#pragma unroll
    for (int n = 0; n < 4; ++n) ob[qi * so.l + n * 16 + lc] = acc[n][r] * inv;
    if (lc == 0) lse[((int64_t)b * H + h) * Lq + qi] = m[r] + logf(l[r]);
  }
}

// delta[b,h,i] = sum_d dO[b,i,h,d] * O[b,i,h,d]
__global__ __launch_bounds__(256) void attn_delta_kernel(const float* __restrict__ o, const float* __restrict__ dO,
                                                         float* __restrict__ delta, AttnStrides so, AttnStrides sd,
                                                         int64_t B, int64_t H, int64_t Lq) {
  const int lane = threadIdx.x & 63;
  const int64_t rows = B * H * Lq;
  for (int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); r < rows; r += (int64_t)gridDim.x * 4) {
    const int64_t i = r % Lq, bh = r / Lq, hh = bh % H, bb = bh / H;
    const float a = o[bb * so.b + i * so.l + hh * so.h + lane];
    const float g = dO[bb * sd.b + i * sd.l + hh * sd.h + lane];
    const float s = wave_sum(a * g);
    if (lane == 0) delta[r] = s;
  }
}

// ------------------------------------------------------------------------------------ dK / dV
template <int PREC>
__global__ __launch_bounds__(256) void attn_bwd_dkdv_kernel(
    const float* __restrict__ q, const float* __restrict__ k, const float* __restrict__ v,
    const float* __restrict__ dO, const float* __restrict__ lse, const float* __restrict__ delta,
    float* __restrict__ dk, float* __restrict__ dv, AttnStrides sq, AttnStrides sk, AttnStrides sv, AttnStrides sd,
    AttnStrides sdk, AttnStrides sdv, int64_t H, int64_t Lq, int64_t Lk, int causal, float scale) {
  typedef typename AT<PREC>::T T;
  constexpr int S = AT<PREC>::S;
  __shared__ __attribute__((aligned(16))) T Ks[ATILE * S];
  __shared__ __attribute__((aligned(16))) T Vs[ATILE * S];
  __shared__ __attribute__((aligned(16))) T Qs[ATILE * S];
  __shared__ __attribute__((aligned(16))) T Qt[AHD * S];
  __shared__ __attribute__((aligned(16))) T dOs[ATILE * S];
  __shared__ __attribute__((aligned(16))) T dOt[AHD * S];
  __shared__ __attribute__((aligned(16))) T Pst[4][16 * S];
  __shared__ __attribute__((aligned(16))) T dSt[4][16 * S];
  __shared__ float lse_s[ATILE], del_s[ATILE];

  const int b = blockIdx.z, h = blockIdx.y;
  const int64_t k0 = (int64_t)blockIdx.x * ATILE;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int lc = lane & 15, lr4 = (lane >> 4) * 4;
  const float* qb = q + b * sq.b + h * sq.h;
  const float* kb = k + b * sk.b + h * sk.h;
  const float* vb = v + b * sv.b + h * sv.h;
  const float* gb = dO + b * sd.b + h * sd.h;
  const float* lb = lse + ((int64_t)b * H + h) * Lq;
  const float* db_ = delta + ((int64_t)b * H + h) * Lq;

  stage_tile<PREC, false>(Ks, kb, sk, k0, Lk);
  stage_tile<PREC, false>(Vs, vb, sv, k0, Lk);

  f32x4 adk[4], adv[4];
#pragma unroll
  for (int n = 0; n < 4; ++n) {
    adk[n] = f32x4{0.f, 0.f, 0.f, 0.f};
    adv[n] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const int64_t kw = k0 + wid * 16;
  const int64_t qstart = causal ? (k0 / ATILE) * ATILE : 0;
  for (int64_t q0 = qstart; q0 < Lq; q0 += ATILE) {
    __syncthreads();
    stage_tile<PREC, false>(Qs, qb, sq, q0, Lq);
    stage_tile<PREC, true>(Qt, qb, sq, q0, Lq);
    stage_tile<PREC, false>(dOs, gb, sd, q0, Lq);
    stage_tile<PREC, true>(dOt, gb, sd, q0, Lq);
    if (threadIdx.x < ATILE) {
      const int64_t qi = q0 + threadIdx.x;
      lse_s[threadIdx.x] = qi < Lq ? lb[qi] : 0.f;
      del_s[threadIdx.x] = qi < Lq ? db_[qi] : 0.f;
    }
    __syncthreads();
    T* P = Pst[wid];
    T* D = dSt[wid];
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      f32x4 st = f32x4{0.f, 0.f, 0.f, 0.f};
      f32x4 dp = f32x4{0.f, 0.f, 0.f, 0.f};
      mma16x64<PREC>(st, Ks, wid * 16, Qs, n * 16);   // S^T: rows = keys, cols = queries
      mma16x64<PREC>(dp, Vs, wid * 16, dOs, n * 16);  // dP^T
      const int qcol = n * 16 + lc;
      const int64_t qi = q0 + qcol;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t key = kw + lr4 + r;
        float p = __expf(st[r] * scale - lse_s[qcol]);
        if (qi >= Lq || key >= Lk || (causal && key > qi)) p = 0.f;
        const float ds = p * (dp[r] - del_s[qcol]);
        P[(lr4 + r) * S + qcol] = cvt<PREC>(p);
        D[(lr4 + r) * S + qcol] = cvt<PREC>(ds);
      }
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      mma16x64<PREC>(adv[n], P, 0, dOt, n * 16);
      mma16x64<PREC>(adk[n], D, 0, Qt, n * 16);
    }
  }
  float* dkb = dk + b * sdk.b + h * sdk.h;
  float* dvb = dv + b * sdv.b + h * sdv.h;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int64_t key = kw + lr4 + r;
    if (key >= Lk) continue;
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      dkb[key * sdk.l + n * 16 + lc] = adk[n][r] * scale;
      dvb[key * sdv.l + n * 16 + lc] = adv[n][r];
    }
  }
}

// ------------------------------------------------------------------------------------ dQ
template <int PREC>
__global__ __launch_bounds__(256) void attn_bwd_dq_kernel(
    const float* __restrict__ q, const float* __restrict__ k, const float* __restrict__ v,
    const float* __restrict__ dO, const float* __restrict__ lse, const float* __restrict__ delta,
    float* __restrict__ dq, AttnStrides sq, AttnStrides sk, AttnStrides sv, AttnStrides sd, AttnStrides sdq,
    int64_t H, int64_t Lq, int64_t Lk, int causal, float scale) {
  typedef typename AT<PREC>::T T;
  constexpr int S = AT<PREC>::S;
  __shared__ __attribute__((aligned(16))) T Qs[ATILE * S];
  __shared__ __attribute__((aligned(16))) T dOs[ATILE * S];
  __shared__ __attribute__((aligned(16))) T Ks[ATILE * S];
  __shared__ __attribute__((aligned(16))) T Kt[AHD * S];
  __shared__ __attribute__((aligned(16))) T Vs[ATILE * S];
  __shared__ __attribute__((aligned(16))) T dSs[4][16 * S];

  const int b = blockIdx.z, h = blockIdx.y;
  const int64_t q0 = (int64_t)blockIdx.x * ATILE;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int lc = lane & 15, lr4 = (lane >> 4) * 4;
  const float* qb = q + b * sq.b + h * sq.h;
  const float* kb = k + b * sk.b + h * sk.h;
  const float* vb = v + b * sv.b + h * sv.h;
  const float* gb = dO + b * sd.b + h * sd.h;
  const float* lb = lse + ((int64_t)b * H + h) * Lq;
  const float* db_ = delta + ((int64_t)b * H + h) * Lq;

  stage_tile<PREC, false>(Qs, qb, sq, q0, Lq);
  stage_tile<PREC, false>(dOs, gb, sd, q0, Lq);
  const int64_t qw = q0 + wid * 16;
  float lsev[4], delv[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int64_t qi = qw + lr4 + r;
    lsev[r] = qi < Lq ? lb[qi] : 0.f;
    delv[r] = qi < Lq ? db_[qi] : 0.f;
  }
  f32x4 adq[4];
#pragma unroll
  for (int n = 0; n < 4; ++n) adq[n] = f32x4{0.f, 0.f, 0.f, 0.f};
  int64_t kend = Lk;
  if (causal) kend = min(Lk, q0 + ATILE);
  for (int64_t k0 = 0; k0 < kend; k0 += ATILE) {
    __syncthreads();
    stage_tile<PREC, false>(Ks, kb, sk, k0, Lk);
    stage_tile<PREC, true>(Kt, kb, sk, k0, Lk);
    stage_tile<PREC, false>(Vs, vb, sv, k0, Lk);
    __syncthreads();
    T* D = dSs[wid];
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      f32x4 s = f32x4{0.f, 0.f, 0.f, 0.f};
      f32x4 dp = f32x4{0.f, 0.f, 0.f, 0.f};
      mma16x64<PREC>(s, Qs, wid * 16, Ks, n * 16);
      mma16x64<PREC>(dp, dOs, wid * 16, Vs, n * 16);
      const int64_t key = k0 + n * 16 + lc;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t qi = qw + lr4 + r;
        float p = __expf(s[r] * scale - lsev[r]);
        if (qi >= Lq || key >= Lk || (causal && key > qi)) p = 0.f;
        D[(lr4 + r) * S + n * 16 + lc] = cvt<PREC>(p * (dp[r] - delv[r]));
      }
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
#pragma unroll
    for (int n = 0; n < 4; ++n) mma16x64<PREC>(adq[n], D, 0, Kt, n * 16);
  }
  float* dqb = dq + b * sdq.b + h * sdq.h;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int64_t qi = qw + lr4 + r;
    if (qi >= Lq) continue;
#pragma unroll
    for (int n = 0; n < 4; ++n) dqb[qi * sdq.l + n * 16 + lc] = adq[n][r] * scale;
  }
}

}  // namespace asrx

using namespace asrx;

static bool attn_ok(const int64_t* st) { return st[0] % 4 == 0 && st[1] % 4 == 0 && st[2] % 4 == 0; }

// Strides are passed as int64[3] = {batch, seq, head} in elements; the head-dim stride must be 1.
namespace asrx {
int attn_fwd_mf(const float* q, const int64_t* sq, const float* k, const int64_t* sk, const float* v,
                const int64_t* sv, float* o, const int64_t* so, float* lse, int64_t B, int64_t H, int64_t Lq,
                int64_t Lk, int causal, float scale, hipStream_t stream);
int attn_bwd_mf(const float* q, const int64_t* sq, const float* k, const int64_t* sk, const float* v,
                const int64_t* sv, const float* dO, const int64_t* sd, const float* lse, const float* delta,
                float* dq, const int64_t* sdq, float* dk, const int64_t* sdk, float* dv, const int64_t* sdv,
                int64_t B, int64_t H, int64_t Lq, int64_t Lk, int causal, float scale, hipStream_t stream);
int attn_fwd_f8(const float* q, const int64_t* sq, const float* k, const int64_t* sk, const float* v,
                const int64_t* sv, float* o, const int64_t* so, float* lse, int64_t B, int64_t H, int64_t Lq,
                int64_t Lk, int causal, float scale, hipStream_t stream);
constexpr int PREC_FP8ATT = 2;  // forward only: e4m3 QK^T (attn_f8.hip)
}

extern "C" int asrx_attn_fwd(int prec, const float* q, const int64_t* sq, const float* k, const int64_t* sk,
                             const float* v, const int64_t* sv, float* o, const int64_t* so, float* lse, int64_t B,
                             int64_t H, int64_t Lq, int64_t Lk, int64_t hd, int causal, float scale,
                             hipStream_t stream) {
  ASRX_REQUIRE(hd == AHD, "attention: head dim %ld unsupported (64 only)", (long)hd);
  ASRX_REQUIRE(attn_ok(sq) && attn_ok(sk) && attn_ok(sv) && attn_ok(so), "attention: strides must be multiples of 4");
  ASRX_REQUIRE(H < 65536 && B < 65536, "attention: grid too large");
  if (B * H * Lq == 0) return 0;
  ASRX_REQUIRE(Lk > 0, "attention: empty key sequence");
  dim3 g((unsigned)((Lq + ATILE - 1) / ATILE), (unsigned)H, (unsigned)B);
  AttnStrides Sq{sq[0], sq[1], sq[2]}, Sk{sk[0], sk[1], sk[2]}, Sv{sv[0], sv[1], sv[2]}, So{so[0], so[1], so[2]};
  const bool al16 = (((uintptr_t)q | (uintptr_t)k | (uintptr_t)v | (uintptr_t)o) & 15) == 0;
  ASRX_REQUIRE(prec == PREC_F32 || prec == PREC_BF16 || prec == PREC_FP8ATT, "attention: bad precision %d", prec);
  if (prec == PREC_FP8ATT) {
    ASRX_REQUIRE(al16, "attention: fp8 mode needs 16-byte aligned q/k/v/o");
    attn_fwd_f8(q, sq, k, sk, v, sv, o, so, lse, B, H, Lq, Lk, causal, scale, stream);
  } else if (prec == PREC_BF16 && al16 && getenv("ASRX_ATTN_OLD") == nullptr)
    attn_fwd_mf(q, sq, k, sk, v, sv, o, so, lse, B, H, Lq, Lk, causal, scale, stream);
  else if (prec == PREC_BF16)
    attn_fwd_kernel<PREC_BF16><<<g, 256, 0, stream>>>(q, k, v, o, lse, Sq, Sk, Sv, So, H, Lq, Lk, causal, scale);
  else
    attn_fwd_kernel<PREC_F32><<<g, 256, 0, stream>>>(q, k, v, o, lse, Sq, Sk, Sv, So, H, Lq, Lk, causal, scale);
  ASRX_LAUNCHED("asrx_attn_fwd");
}

// delta_ws: workspace of B*H*Lq floats.
extern "C" int asrx_attn_bwd(int prec, const float* q, const int64_t* sq, const float* k, const int64_t* sk,
                             const float* v, const int64_t* sv, const float* o, const int64_t* so, const float* dO,
                             const int64_t* sd, const float* lse, float* delta_ws, float* dq, const int64_t* sdq,
                             float* dk, const int64_t* sdk, float* dv, const int64_t* sdv, int64_t B, int64_t H,
                             int64_t Lq, int64_t Lk, int64_t hd, int causal, float scale, hipStream_t stream) {
  ASRX_REQUIRE(prec == PREC_F32 || prec == PREC_BF16, "attention backward: precision %d (fp8 is forward only)", prec);
  ASRX_REQUIRE(hd == AHD, "attention: head dim %ld unsupported (64 only)", (long)hd);
  ASRX_REQUIRE(attn_ok(sq) && attn_ok(sk) && attn_ok(sv) && attn_ok(sd) && attn_ok(sdq) && attn_ok(sdk) &&
                   attn_ok(sdv),
               "attention: strides must be multiples of 4");
  if (B * H * Lq == 0) return 0;
  AttnStrides Sq{sq[0], sq[1], sq[2]}, Sk{sk[0], sk[1], sk[2]}, Sv{sv[0], sv[1], sv[2]}, So{so[0], so[1], so[2]};
  AttnStrides Sd{sd[0], sd[1], sd[2]}, Sdq{sdq[0], sdq[1], sdq[2]}, Sdk{sdk[0], sdk[1], sdk[2]},
      Sdv{sdv[0], sdv[1], sdv[2]};
  const int64_t rows = B * H * Lq;
  attn_delta_kernel<<<(unsigned)std::min<int64_t>((rows + 3) / 4, 8192), 256, 0, stream>>>(o, dO, delta_ws, So, Sd, B,
                                                                                          H, Lq);
  dim3 gk((unsigned)((Lk + ATILE - 1) / ATILE), (unsigned)H, (unsigned)B);
  dim3 gq((unsigned)((Lq + ATILE - 1) / ATILE), (unsigned)H, (unsigned)B);
  const bool al16 = (((uintptr_t)q | (uintptr_t)k | (uintptr_t)v | (uintptr_t)dO | (uintptr_t)dq | (uintptr_t)dk |
                       (uintptr_t)dv) & 15) == 0;
  if (prec == PREC_BF16 && al16 && getenv("ASRX_ATTN_OLD") == nullptr) {
    attn_bwd_mf(q, sq, k, sk, v, sv, dO, sd, lse, delta_ws, dq, sdq, dk, sdk, dv, sdv, B, H, Lq, Lk, causal, scale,
                stream);
  } else if (prec == PREC_BF16) {
    attn_bwd_dkdv_kernel<PREC_BF16><<<gk, 256, 0, stream>>>(q, k, v, dO, lse, delta_ws, dk, dv, Sq, Sk, Sv, Sd, Sdk,
                                                            Sdv, H, Lq, Lk, causal, scale);
    attn_bwd_dq_kernel<PREC_BF16><<<gq, 256, 0, stream>>>(q, k, v, dO, lse, delta_ws, dq, Sq, Sk, Sv, Sd, Sdq, H, Lq,
                                                          Lk, causal, scale);
  } else {
    attn_bwd_dkdv_kernel<PREC_F32><<<gk, 256, 0, stream>>>(q, k, v, dO, lse, delta_ws, dk, dv, Sq, Sk, Sv, Sd, Sdk,
                                                           Sdv, H, Lq, Lk, causal, scale);
    attn_bwd_dq_kernel<PREC_F32><<<gq, 256, 0, stream>>>(q, k, v, dO, lse, delta_ws, dq, Sq, Sk, Sv, Sd, Sdq, H, Lq,
                                                         Lk, causal, scale);
  }
  ASRX_LAUNCHED("asrx_attn_bwd");
}
