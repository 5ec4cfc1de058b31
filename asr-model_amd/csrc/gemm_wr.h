#pragma once
// Wide-N GEMM for activation x weight products (perf mode): every nn.Linear / 1x1 / k3 conv forward
// and input-gradient on the hot path (model.py:96-147, 242-245, 341, 398-425, 529-574;
// essentials.py:149-153), i.e. Y = act(alpha * A W^T + beta * Y + bias) with
//   A  activations (M x K, row-major, or the implicit k3 im2col of a channels-last sequence), fp32 or
//      bf16 in HBM (ABF: an activation whose only consumers are GEMM operands is stored bf16 by its
//      producer, halving its bytes -- the products are bit-identical, A is rounded to bf16 either way),
//   W  the weight pre-converted to bf16, stored N x K (K contiguous) -- asrx_weight_to_bf16,
//   Y  fp32, or bf16 (Cb) when Y itself only feeds GEMMs.
//
// At the model's shapes (M = 8k..192k rows, N, K = 64..1536) the kernel is bound by bytes moved
// (A from HBM, W from L2, C back to HBM), not by MFMA.  Design (gemm_wr_kernel):
//  * 128 x BN tiles, BN = 128 * NJ up to 384, so an activation row panel is read once per 384
//    output columns; 512 threads = 8 waves (2 x 4), each 64 x 32*NJ of the output.
//  * Persistent workgroups (grid = resident capacity) walk their tiles in an XCD-grouped order;
//    operands travel global -> VGPR -> LDS with plain 16-byte loads issued 3 k-steps ahead (the
//    register pipeline runs across tile boundaries), fp32 A is converted to bf16 once on the way
//    in, the LDS images are double-buffered with one barrier per k-step.  (An LDS-DMA ring variant
//    was measured slower -- 219 vs 195 us at M = 192064, N = K = 384 -- and removed.)
//  * Images are XOR-swizzled so the ds_read_b128 fragment reads are bank-conflict-free under
//    gfx950's 64-bank, 16-lane-group rule.
//  * MFMA 16x16x32 bf16 with the W fragment as the row operand: each lane ends up owning 4
//    consecutive output columns of one row; the epilogue is staged through LDS so every store
//    instruction writes whole row segments.
#include "common.h"

namespace asrx {

namespace wn {

constexpr int BM = 128, BK = 32, NTHR = 512;
constexpr int A_BYTES = BM * BK * 4;  // 16 KB fp32

static __device__ __attribute__((aligned(16))) float zero_page[4];

struct Params {
  const float* A;
  int lda;
  const unsigned short* W;  // bf16 N x K
  int ldw;
  float* C;
  int ldc;
  const float* bias;
  float* Z;
  int M, N, K;
  int convF, convC;
  float alpha, beta;
  int act;
  const float* W2;  // router: Linear(d, 3) weight (3 x N) applied to SiLU(C) in the epilogue
  float* R;         // router: logits without bias (M x 3); C may be null (h_pre not kept)
  // optional row-tile list (gemm_wr_kernel): only the BM-row tiles mtiles[0 .. *n_mtiles) are
  // computed (MSheath layers skip the rows of samples that are not at the layer); other rows of C
  // are left untouched
  const int* mtiles;
  const int* n_mtiles;
  // bf16 output (gemm_wr_kernel): when non-null, act(v) is written here as bf16 instead of to C
  // (an activation whose only consumers are GEMM operands -- they round it to bf16 anyway); beta = 0
  unsigned short* Cb;
  // fused cross-entropy statistics (gemm_wr_kernel<..., CE>): the tied-logits GEMM (model.py:629) writes
  // the logits bf16 (Cb) and, per row and BN-column tile, the (max, sum exp(z - max)) of the tile's
  // bf16-rounded logits into ce_part[row * ce_ld + tile] (float2), so the cross entropy never re-reads
  // the logits for its log-sum-exp (asrx_ce_part_fwd merges the partials)
  float2* ce_part;
  int ce_ld;
  // residual input (gemm_wr epilogues, act none, fp32 C): C = R + alpha A W^T + bias -- the residual add
  // around an out projection (model.py:578-580 x = x + attn(...)) without a separate add pass
  const float* Rres;
  int ldr;
  // activation-gradient epilogue (gemm_wr_kernel<..., GA>): the GEMM recomputes the pre-activation
  // z = alpha A W^T + bias of a Linear + act whose forward did not keep it, and stores
  // gz = bf16(G * act'(z)) to Cb (G: the output gradient, fp32, row stride ldg) with the bias gradient's
  // column sums of gz added into dB (nullable) -- the backward never reads a stored z
  const float* G;
  int ldg;
  float* dB;
  // rotary epilogue (ROT instantiations, act none, fp32 C): the q / k projection's rotary (model.py:198-214)
  // applied to the product before it is stored -- C = rot(alpha A W^T + bias), the pairs (2j, 2j+1) of each
  // head times polar(rot_scale * rot_m[row], angle(row % rot_L, j)) from the (cos, sin) table rot_tab
  // ((positions, rot_half) float2, asrx_rotary_table); Z, when non-null, receives the unrotated product
  // (the rotary backward's input)
  const float* rot_m;
  const float2* rot_tab;
  int rot_L, rot_half;
  float rot_scale;
};

__device__ __forceinline__ void st_bf16x4(unsigned short* dst, float a, float b, float c, float d) {
  typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
  const bf16x4 h = {(__bf16)a, (__bf16)b, (__bf16)c, (__bf16)d};
  __builtin_nontemporal_store(__builtin_bit_cast(unsigned long long, h), reinterpret_cast<unsigned long long*>(dst));
}

template <int NJ>
struct Cfg {
  static constexpr int BN = 128 * NJ;
  static constexpr int B_BYTES = BN * BK * 2;  // bf16
  static constexpr int STAGE = A_BYTES + B_BYTES;
  static constexpr int PIECES = 2 + NJ;  // 1 KB DMAs per wave per k-step: A 2, W NJ
  static constexpr int BNR = (BN + NTHR - 1) / NTHR * NTHR;  // bias slice in whole DMA rounds
  static constexpr int BIAS_OPS = BNR / NTHR;
};

// conflict-free swizzles (chunk XOR by row) for the A image (rows of 8 x 16 B) and the W image
// (rows of 4 x 16 B) under ds_read_b128 lane groups {0-3,12-15,20-27}, {4-11,16-19,28-31}, ...
__device__ __forceinline__ int swa(int row) { return ((row >> 1) & 1) | (((row >> 3) & 1) << 2); }
__device__ __forceinline__ int swb(int n) { return ((n >> 3) & 1) << 1; }

__device__ __forceinline__ bool vec_ok(const Params& p) {
  return ((p.N | p.ldc) & 3) == 0 && ((uintptr_t)p.C & 15) == 0 && ((uintptr_t)p.Z & 15) == 0 &&
         ((uintptr_t)p.Cb & 7) == 0;
}

template <int ACT>
__device__ __forceinline__ float act_t(float x) {
  if constexpr (ACT == ACT_GELU) return gelu_f(x);
  else if constexpr (ACT == ACT_SILU) return silu_f(x);
  else if constexpr (ACT == ACT_SIGMOID) return sigmoid_f(x);
  else if constexpr (ACT == ACT_RELU) return x > 0.f ? x : 0.f;
  else return x;
}

// Tile epilogue: v = alpha * acc + bias (+ beta * C); Z <- v (pre-activation); C <- act(v).
// Full float4 rows go out as non-temporal stores (streaming writes that would otherwise sit dirty
// in L2 ahead of the next tile's loads: -8 % at M = 192064, N = K = 384).
template <int NJ, int ACT>
__device__ __forceinline__ void epilogue(const Params& p, f32x4 (&acc)[4][2 * NJ], const float* bsl, int m0, int n0,
                                         int wm, int wn, int lr, int lk) {
  constexpr int NT = 2 * NJ;
  const bool vec = vec_ok(p);
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    const int nl = wn * (32 * NJ) + nt * 16 + 4 * lk;
    const int col = n0 + nl;
    if (col >= p.N) continue;
    float4 bv = make_float4(0.f, 0.f, 0.f, 0.f);
    if (p.bias) bv = *reinterpret_cast<const float4*>(bsl + nl);
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      const int row = m0 + wm * 64 + mt * 16 + lr;
      if (row >= p.M) continue;
      float v[4] = {p.alpha * acc[mt][nt][0] + bv.x, p.alpha * acc[mt][nt][1] + bv.y,
                    p.alpha * acc[mt][nt][2] + bv.z, p.alpha * acc[mt][nt][3] + bv.w};
      float* dst = p.C + (int64_t)row * p.ldc + col;
      float* zdst = p.Z ? p.Z + (int64_t)row * p.ldc + col : nullptr;
      if (p.Cb) {  // bf16 output (beta = 0)
        unsigned short* hd = p.Cb + (int64_t)row * p.ldc + col;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          if (col + r >= p.N) break;
          if (zdst) zdst[r] = v[r];
          hd[r] = __builtin_bit_cast(unsigned short, (__bf16)act_t<ACT>(v[r]));
        }
        continue;
      }
      if (vec) {
        if (p.beta != 0.f) {
          const float4 o = *reinterpret_cast<const float4*>(dst);
          v[0] += p.beta * o.x; v[1] += p.beta * o.y; v[2] += p.beta * o.z; v[3] += p.beta * o.w;
        }

        if (zdst) __builtin_nontemporal_store(f32x4{v[0], v[1], v[2], v[3]}, reinterpret_cast<f32x4*>(zdst));
        __builtin_nontemporal_store(f32x4{act_t<ACT>(v[0]), act_t<ACT>(v[1]), act_t<ACT>(v[2]), act_t<ACT>(v[3])},
                                    reinterpret_cast<f32x4*>(dst));
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          if (col + r >= p.N) break;
          float x = v[r];
          if (p.beta != 0.f) x += p.beta * dst[r];
          if (zdst) zdst[r] = x;
          dst[r] = act_t<ACT>(x);
        }
      }
    }
  }
}

// The same epilogue staged through a per-wave LDS slab, one 16-row slice (mt) at a time: the MFMA
// layout gives each lane 4 columns of one row, so a direct store instruction writes 16 rows x 64 B;
// re-read from LDS, every store instruction writes whole contiguous row segments (32*NJ floats per
// row: 384 B at NJ = 3).  Requires vec_ok(p) (float4-aligned C/Z, N % 4 == 0).
#ifndef WR_ABL_EPI
#define WR_ABL_EPI 0  // timing ablations (wrong results): 1 no epilogue, 2 epilogue without its global stores
#endif
constexpr int EP_PAD = 4;
template <int NJ>
struct EpLds {
  static constexpr int W = 32 * NJ;           // columns of a wave's sub-tile
  static constexpr int LD = W + EP_PAD;       // slab row stride (floats)
  static constexpr int FLOATS = 16 * LD;      // one 16-row slice
};
// rot_apply: rotary's complex product on one float4 of columns (col % 4 == 0, so two whole pairs), with the
// arithmetic of rowops.hip rotary_fwd_kernel (no contractions: bit-identical to the separate pass)
__device__ __forceinline__ float4 rot_apply(const Params& p, float4 x, int row, int col) {
#pragma clang fp contract(off)
  const int hd = 2 * p.rot_half;
  const int j = (col % hd) >> 1;
  const float4 t = *reinterpret_cast<const float4*>(p.rot_tab + (int64_t)(row % p.rot_L) * p.rot_half + j);
  const float mm = p.rot_m[row] * p.rot_scale;
  return make_float4(mm * (x.x * t.x - x.y * t.y), mm * (x.x * t.y + x.y * t.x), mm * (x.z * t.z - x.w * t.w),
                     mm * (x.z * t.w + x.w * t.z));
}

template <int NJ, int ACT, bool RES = false, bool ROT = false>
__device__ __forceinline__ void epilogue_lds(const Params& p, f32x4 (&acc)[4][2 * NJ], const float* bsl, int m0,
                                             int n0, int wm, int wn, int lr, int lk, float* ep) {
  constexpr int NT = 2 * NJ, W = EpLds<NJ>::W, LD = EpLds<NJ>::LD, W4 = W / 4;
  constexpr int PER = 16 * W4 / 64;  // float4 per lane per slice
  static_assert((16 * W4) % 64 == 0, "slice must split evenly over the wave");
  const int lane = threadIdx.x & 63;
  const int cbase = n0 + wn * W;
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) {
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const int nl = nt * 16 + 4 * lk;
      float4 bv = make_float4(0.f, 0.f, 0.f, 0.f);
      if (p.bias) bv = *reinterpret_cast<const float4*>(bsl + wn * W + nl);
      *reinterpret_cast<float4*>(ep + lr * LD + nl) =
          make_float4(p.alpha * acc[mt][nt][0] + bv.x, p.alpha * acc[mt][nt][1] + bv.y,
                      p.alpha * acc[mt][nt][2] + bv.z, p.alpha * acc[mt][nt][3] + bv.w);
    }
    __builtin_amdgcn_wave_barrier();
    const int rbase = m0 + wm * 64 + mt * 16;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int f = j * 64 + lane, r = f / W4, c = 4 * (f % W4);
      float4 x = *reinterpret_cast<const float4*>(ep + r * LD + c);
      const int row = rbase + r, col = cbase + c;
      if (row >= p.M || col >= p.N) continue;
#if WR_ABL_EPI == 2  // timing ablation (wrong results): the epilogue without its global stores
      if (x.x + x.y + x.z + x.w != 1.2345e-37f) continue;
#endif
      if (p.Cb) {  // bf16 output (beta = 0)
        if (p.Z)
          __builtin_nontemporal_store(f32x4{x.x, x.y, x.z, x.w},
                                      reinterpret_cast<f32x4*>(p.Z + (int64_t)row * p.ldc + col));
        st_bf16x4(p.Cb + (int64_t)row * p.ldc + col, act_t<ACT>(x.x), act_t<ACT>(x.y), act_t<ACT>(x.z),
                  act_t<ACT>(x.w));
        continue;
      }
      float* dst = p.C + (int64_t)row * p.ldc + col;
      if (p.beta != 0.f) {
        const float4 o = *reinterpret_cast<const float4*>(dst);
        x.x += p.beta * o.x; x.y += p.beta * o.y; x.z += p.beta * o.z; x.w += p.beta * o.w;
      }
      if constexpr (RES) {  // the residual add of an out projection (RES instantiations only)
        const float4 o = *reinterpret_cast<const float4*>(p.Rres + (int64_t)row * p.ldr + col);
        x.x += o.x; x.y += o.y; x.z += o.z; x.w += o.w;
      }
      if (p.Z)
        __builtin_nontemporal_store(f32x4{x.x, x.y, x.z, x.w},
                                    reinterpret_cast<f32x4*>(p.Z + (int64_t)row * p.ldc + col));
      if constexpr (ROT) x = rot_apply(p, x, row, col);  // act none (ROT instantiations)
      __builtin_nontemporal_store(f32x4{act_t<ACT>(x.x), act_t<ACT>(x.y), act_t<ACT>(x.z), act_t<ACT>(x.w)},
                                  reinterpret_cast<f32x4*>(dst));
    }
    __builtin_amdgcn_wave_barrier();  // the next slice overwrites the slab
  }
}

// Activation-gradient epilogue (Params::G): slab = z (as epilogue_lds stages it, so z is bit-identical to
// the pre-activation the forward would have stored), then per coalesced float4: o = G * act'(z) (the
// arithmetic of rowops.hip act_bwd_bias_kernel, up to the compiler's contractions), bf16 o to Cb and fp32
// o back into the slab (0 outside M x N); each lane then sums columns lane, lane + 64 of the slice and
// keeps the partials over the tile's 4 slices; one atomicAdd per column and wave into dB at the end.
template <int ACT>
__device__ __forceinline__ float dact_t(float v) {
  if constexpr (ACT == ACT_GELU) return gelu_grad(v);
  else if constexpr (ACT == ACT_SILU) return silu_grad(v);
  else {
    const float sg = sigmoid_f(v);
    return sg * (1.f - sg);
  }
}
template <int NJ, int ACT>
__device__ __forceinline__ void epilogue_gact(const Params& p, f32x4 (&acc)[4][2 * NJ], const float* bsl, int m0,
                                              int n0, int wm, int wn, int lr, int lk, float* ep) {
  constexpr int NT = 2 * NJ, W = EpLds<NJ>::W, LD = EpLds<NJ>::LD, W4 = W / 4;
  constexpr int PER = 16 * W4 / 64;
  constexpr int CS = (W + 63) / 64;  // column-sum slots per lane
  const int lane = threadIdx.x & 63;
  const int cbase = n0 + wn * W;
  float csum[CS];
#pragma unroll
  for (int i = 0; i < CS; ++i) csum[i] = 0.f;
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) {
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const int nl = nt * 16 + 4 * lk;
      float4 bv = make_float4(0.f, 0.f, 0.f, 0.f);
      if (p.bias) bv = *reinterpret_cast<const float4*>(bsl + wn * W + nl);
      *reinterpret_cast<float4*>(ep + lr * LD + nl) =
          make_float4(p.alpha * acc[mt][nt][0] + bv.x, p.alpha * acc[mt][nt][1] + bv.y,
                      p.alpha * acc[mt][nt][2] + bv.z, p.alpha * acc[mt][nt][3] + bv.w);
    }
    __builtin_amdgcn_wave_barrier();
    const int rbase = m0 + wm * 64 + mt * 16;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int f = j * 64 + lane, r = f / W4, c = 4 * (f % W4);
      float* sl = ep + r * LD + c;
      const float4 z = *reinterpret_cast<const float4*>(sl);
      const int row = rbase + r, col = cbase + c;
      float4 o = make_float4(0.f, 0.f, 0.f, 0.f);
      if (row < p.M && col < p.N) {
        const float4 g = *reinterpret_cast<const float4*>(p.G + (int64_t)row * p.ldg + col);
        o = make_float4(g.x * dact_t<ACT>(z.x), g.y * dact_t<ACT>(z.y), g.z * dact_t<ACT>(z.z),
                        g.w * dact_t<ACT>(z.w));
        st_bf16x4(p.Cb + (int64_t)row * p.ldc + col, o.x, o.y, o.z, o.w);
      }
      *reinterpret_cast<float4*>(sl) = o;
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int i = 0; i < CS; ++i) {
      const int cc = lane + 64 * i;
      if (cc < W) {
#pragma unroll
        for (int r = 0; r < 16; ++r) csum[i] += ep[r * LD + cc];
      }
    }
    __builtin_amdgcn_wave_barrier();  // the next slice overwrites the slab
  }
  if (p.dB) {
#pragma unroll
    for (int i = 0; i < CS; ++i) {
      const int cc = lane + 64 * i;
      if (cc < W && cbase + cc < p.N) atomicAdd(p.dB + cbase + cc, csum[i]);
    }
  }
}

// Tied-logits epilogue with cross-entropy statistics: the epilogue_lds store (alpha * acc, no bias /
// activation) -- bf16 to Cb, or fp32 to C when Cb is null (the logits the drop-in boundary returns,
// model.py:629 .float()) -- and from the same LDS slab each row's (max, sum exp) over the wave's 32*NJ
// columns of the STORED values (what the backward will read back): lane -> row lane/4, quarter
// lane%4 of the columns, merged over the 4 lanes by shuffles and over the 4 column waves through LDS
// (red: BM x 4 float2); threads < BM then write the tile's partial of their row.
template <int NJ>
__device__ __forceinline__ void epilogue_ce(const Params& p, f32x4 (&acc)[4][2 * NJ], int m0, int n0, int wm, int wn,
                                            int lr, int lk, float* ep, float2* red) {
  constexpr int NT = 2 * NJ, W = EpLds<NJ>::W, LD = EpLds<NJ>::LD, W4 = W / 4, Q = W / 4;
  constexpr int PER = 16 * W4 / 64;
  const int lane = threadIdx.x & 63;
  const int cbase = n0 + wn * W;
  const bool rb = p.Cb != nullptr;  // bf16 logits (statistics of the rounded values) or fp32 logits in C
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) {
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const int nl = nt * 16 + 4 * lk;
      *reinterpret_cast<float4*>(ep + lr * LD + nl) =
          make_float4(p.alpha * acc[mt][nt][0], p.alpha * acc[mt][nt][1], p.alpha * acc[mt][nt][2],
                      p.alpha * acc[mt][nt][3]);
    }
    __builtin_amdgcn_wave_barrier();
    const int rbase = m0 + wm * 64 + mt * 16;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int f = j * 64 + lane, r = f / W4, c = 4 * (f % W4);
      const float4 x = *reinterpret_cast<const float4*>(ep + r * LD + c);
      const int row = rbase + r, col = cbase + c;
      if (row >= p.M || col >= p.N) continue;
      if (rb)
        st_bf16x4(p.Cb + (int64_t)row * p.ldc + col, x.x, x.y, x.z, x.w);
      else
        __builtin_nontemporal_store(f32x4{x.x, x.y, x.z, x.w},
                                    reinterpret_cast<f32x4*>(p.C + (int64_t)row * p.ldc + col));
    }
    {
      const int rr = lane >> 2, q = lane & 3;
      const float* src = ep + rr * LD + q * Q;
      const int c0 = cbase + q * Q;
      float m = -INFINITY;
#pragma unroll
      for (int i = 0; i < Q; ++i)
        if (c0 + i < p.N) m = fmaxf(m, rb ? (float)(__bf16)src[i] : src[i]);
      float sm = 0.f;
      if (m != -INFINITY) {
#pragma unroll
        for (int i = 0; i < Q; ++i)
          if (c0 + i < p.N) sm += __expf((rb ? (float)(__bf16)src[i] : src[i]) - m);
      }
#pragma unroll
      for (int o = 1; o <= 2; o <<= 1) {
        const float mo = __shfl_xor(m, o), so = __shfl_xor(sm, o);
        const float mn = fmaxf(m, mo);
        sm = (m == -INFINITY ? 0.f : sm * __expf(m - mn)) + (mo == -INFINITY ? 0.f : so * __expf(mo - mn));
        m = mn;
      }
      if (q == 0) red[(wm * 64 + mt * 16 + rr) * 4 + wn] = make_float2(m, sm);
    }
    __builtin_amdgcn_wave_barrier();  // the next slice overwrites the slab
  }
  // every column wave's row partials in LDS, then one merge per row -- s_barrier without
  // __syncthreads()'s vmcnt(0) fence (the next tile's operand loads stay in flight)
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  if (threadIdx.x < BM) {
    const int row = m0 + threadIdx.x;
    if (row < p.M) {
      float m = -INFINITY, sm = 0.f;
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        const float2 v = red[threadIdx.x * 4 + w];
        const float mn = fmaxf(m, v.x);
        sm = (m == -INFINITY ? 0.f : sm * __expf(m - mn)) + (v.x == -INFINITY ? 0.f : v.y * __expf(v.x - mn));
        m = mn;
      }
      p.ce_part[(int64_t)row * p.ce_ld + n0 / Cfg<NJ>::BN] = make_float2(m, sm);
    }
  }
}

// AbbyNormal router epilogue (essentials.py:155-161): h = alpha*acc + bias is h_pre; the tile holds
// whole rows (N <= BN), so logits[row][k] = sum_n SiLU(h[row][n]) W2[k][n] reduce in-tile: over
// each lane's 4 columns and NT sub-tiles, across the 4 lanes of a row (shuffles) and across the 4
// column waves (LDS).  h_pre is stored only when C != null (it is needed by the backward).
template <int NJ>
__device__ __forceinline__ void epilogue_router(const Params& p, f32x4 (&acc)[4][2 * NJ], const float* bsl,
                                                const float* w2s, float* red, int m0, int wm, int wn, int lr,
                                                int lk) {
  constexpr int NT = 2 * NJ, BNL = 128 * NJ;
  const bool vec = vec_ok(p);
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) {
    const int row = m0 + wm * 64 + mt * 16 + lr;
    float s0 = 0.f, s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const int nl = wn * (32 * NJ) + nt * 16 + 4 * lk;
      if (nl >= p.N) continue;
      float4 bv = make_float4(0.f, 0.f, 0.f, 0.f);
      if (p.bias) bv = *reinterpret_cast<const float4*>(bsl + nl);
      const float v[4] = {p.alpha * acc[mt][nt][0] + bv.x, p.alpha * acc[mt][nt][1] + bv.y,
                          p.alpha * acc[mt][nt][2] + bv.z, p.alpha * acc[mt][nt][3] + bv.w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (nl + q < p.N) {
          const float h = silu_f(v[q]);
          s0 += h * w2s[nl + q];
          s1 += h * w2s[BNL + nl + q];
          s2 += h * w2s[2 * BNL + nl + q];
        }
      }
      if (p.C && row < p.M) {
        float* dst = p.C + (int64_t)row * p.ldc + nl;
        if (vec) {
          *reinterpret_cast<float4*>(dst) = make_float4(v[0], v[1], v[2], v[3]);
        } else {
#pragma unroll
          for (int q = 0; q < 4; ++q)
            if (nl + q < p.N) dst[q] = v[q];
        }
      }
    }
    s0 += __shfl_xor(s0, 16); s1 += __shfl_xor(s1, 16); s2 += __shfl_xor(s2, 16);
    s0 += __shfl_xor(s0, 32); s1 += __shfl_xor(s1, 32); s2 += __shfl_xor(s2, 32);
    if (lk == 0) {
      float* rr = red + ((wm * 64 + mt * 16 + lr) * 4 + wn) * 3;
      rr[0] = s0; rr[1] = s1; rr[2] = s2;
    }
  }
  // LDS writes visible, then barrier -- not __syncthreads(), whose fence would emit vmcnt(0) and
  // drain the next tile's LDS-DMA prefetch
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  for (int i = threadIdx.x; i < BM * 3; i += NTHR) {
    const int rl = i / 3, k = i % 3;
    const int row = m0 + rl;
    if (row < p.M) {
      const float* rr = red + rl * 12 + k;
      p.R[(int64_t)row * 3 + k] = rr[0] + rr[3] + rr[6] + rr[9];
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Register-staged variant (gemm_wr_kernel): the same tiles, waves, MFMA and epilogues, but both
// operands travel global -> VGPR -> LDS with plain dwordx4 loads issued DEPTH k-steps ahead (the
// compiler counts their vmcnt), A is converted to bf16 once on the way into LDS (the four waves
// that share an A fragment no longer convert it four times, and the A image halves to 8 KB), and
// the LDS images are double-buffered with one barrier per k-step.  An LDS-DMA piece costs ~100+
// issue cycles per KB on gfx950 (MI355X_MICROARCH.md constants table); a dwordx4 load + ds_write
// moves the same KB for a fraction of that, which is what bounded gemm_wn_kernel's pipeline.
#ifndef WR_EPI_LDS
#define WR_EPI_LDS 1  // LDS-staged epilogue (whole row segments per store instruction)
#endif
#ifndef WR_DEPTH
#define WR_DEPTH 3  // register stages in flight (k-steps of prefetch)
#endif
// DEP (template): register stages, 0 = WR_DEPTH

// ABF: A is stored bf16 (M x K, lda in elements): one 16-byte chunk of 8 k per thread and k-step
// (row t/4, k chunk t%4), already in the image's element type -- half the bytes, no conversion
// stage registers are native vectors: a HIP_vector_type (uint4 / float4) copy lowers to a memcpy
// that keeps the whole stage in scratch (measured: 80-144 B/lane of scratch plus an LDS-promoted
// stage in the bf16-A instantiations)
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
template <int NJ, bool ABF>
struct WrStage {
  float4 a[2];     // 2 x 4 fp32 of the A tile (row q/8, k chunk q%8), q = tid + 512 i
  u32x4 b[NJ];     // NJ x 8 bf16 of the W tile (row q/4, k chunk q%4), q = tid + 512 i
};
template <int NJ>
struct WrStage<NJ, true> {
  u32x4 ah;        // 8 bf16 of the A tile (row tid/4, k chunk tid%4)
  u32x4 b[NJ];
};

template <int NJ, bool CONV, bool ABF>
__device__ __forceinline__ void wr_load(const Params& p, WrStage<NJ, ABF>& st, int m0, int n0, int k0) {
  const int t = threadIdx.x;
  if constexpr (ABF) {
    const int row = t >> 2, c = t & 3;
    const int r = m0 + row, k = k0 + 8 * c;
    bool ok = r < p.M && k < p.K;
    int64_t o = (int64_t)r * p.lda + k;
    if (CONV) {  // convC % 8 == 0: a chunk never straddles two taps
      const int pos = r % p.convF + k / p.convC - 1;
      ok = ok && pos >= 0 && pos < p.convF;
      o -= p.convC;
    }
    const unsigned short* Ah = reinterpret_cast<const unsigned short*>(p.A);
    st.ah = *reinterpret_cast<const u32x4*>(ok ? (const void*)(Ah + o) : (const void*)zero_page);
  } else
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int q = t + NTHR * i;
    const int row = q >> 3, c = q & 7;
    const int r = m0 + row, k = k0 + 4 * c;
    bool ok = r < p.M && k < p.K;
    int64_t o = (int64_t)r * p.lda + k;
    if (CONV) {
      const int pos = r % p.convF + k / p.convC - 1;
      ok = ok && pos >= 0 && pos < p.convF;
      o -= p.convC;
    }
    // unconditional load from a clamped address (a branch around the load would make the
    // compiler drain vmcnt at the join, serialising the prefetch)
    st.a[i] = *reinterpret_cast<const float4*>(ok ? (const void*)(p.A + o) : (const void*)zero_page);
  }
#pragma unroll
  for (int i = 0; i < NJ; ++i) {
    const int q = t + NTHR * i;
    const int n = n0 + (q >> 2), k = k0 + 8 * (q & 3);
    st.b[i] = *reinterpret_cast<const u32x4*>((n < p.N && k < p.K) ? (const void*)(p.W + (int64_t)n * p.ldw + k)
                                                                  : (const void*)zero_page);
  }
}

// Fast operand addressing (non-conv launches whose operands span < 4 GiB and whose K is a multiple of the
// k-step): each thread's row byte offsets are computed once per tile -- rows past M / N clamped to the last
// row (they only feed accumulator rows / columns the epilogues never store) -- and a k-step's load is
// base (SGPR) + offset + k bytes, one address add per load.  The general path selects between the row
// address and the zero page per load and k-step (~15 instructions per load, exec-masked); the k-step is
// issue-bound, and one extra load per k-step measured 5-12 % slower.
#ifndef WR_FAST
#define WR_FAST 1  // 0: every load takes the general (zero-page select) path -- A/B builds only
#endif
template <int NJ, bool ABF>
struct WrOff {
  uint32_t a[ABF ? 1 : 2];
  uint32_t w[NJ];
};
template <int NJ, bool ABF>
__device__ __forceinline__ void wr_offsets(const Params& p, WrOff<NJ, ABF>& o, int m0, int n0) {
  const int t = threadIdx.x;
  if constexpr (ABF) {
    const int row = min(m0 + (t >> 2), p.M - 1);
    o.a[0] = (uint32_t)(((int64_t)row * p.lda + 8 * (t & 3)) * 2);
  } else {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int q = t + NTHR * i;
      const int row = min(m0 + (q >> 3), p.M - 1);
      o.a[i] = (uint32_t)(((int64_t)row * p.lda + 4 * (q & 7)) * 4);
    }
  }
#pragma unroll
  for (int i = 0; i < NJ; ++i) {
    const int q = t + NTHR * i;
    const int n = min(n0 + (q >> 2), p.N - 1);
    o.w[i] = (uint32_t)(((int64_t)n * p.ldw + 8 * (q & 3)) * 2);
  }
}
template <int NJ, bool ABF>
__device__ __forceinline__ void wr_load_fast(const Params& p, WrStage<NJ, ABF>& st, const WrOff<NJ, ABF>& o,
                                             uint32_t ka, uint32_t kw) {
  const char* A = reinterpret_cast<const char*>(p.A);
  const char* W = reinterpret_cast<const char*>(p.W);
  if constexpr (ABF) {
    st.ah = *reinterpret_cast<const u32x4*>(A + (o.a[0] + ka));
  } else {
#pragma unroll
    for (int i = 0; i < 2; ++i) st.a[i] = *reinterpret_cast<const float4*>(A + (o.a[i] + ka));
  }
#pragma unroll
  for (int i = 0; i < NJ; ++i) st.b[i] = *reinterpret_cast<const u32x4*>(W + (o.w[i] + kw));
}

// (Raw buffer loads against a per-tile resource -- 32-bit offsets, out-of-range chunks read 0 -- were
// measured against these zero-page-clamped global loads: 13.1 -> 14.9 us at M = 8192, N = K = 384 and
// no change on the 192k-row launches, profiles/r03_gemm_micro_v2.txt.)
// A image: [128 rows][4 chunks of 8 bf16] (64 B rows), W image: [BN rows][4 chunks], both with the
// chunk XOR swizzle swb(row) (conflict-free ds_read_b128 fragment reads).
template <int NJ, bool ABF>
__device__ __forceinline__ void wr_store(const WrStage<NJ, ABF>& st, char* At, char* Bt) {
  const int t = threadIdx.x;
  if constexpr (ABF) {
    const int row = t >> 2, c = t & 3;
    *reinterpret_cast<u32x4*>(At + row * 64 + 16 * (c ^ swb(row))) = st.ah;
  } else
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int q = t + NTHR * i;
    const int row = q >> 3, c = q & 7;
    const float4 v = st.a[i];
    typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
    bf16x4 h;
    h[0] = (__bf16)v.x; h[1] = (__bf16)v.y; h[2] = (__bf16)v.z; h[3] = (__bf16)v.w;
    *reinterpret_cast<bf16x4*>(At + row * 64 + 16 * ((c >> 1) ^ swb(row)) + 8 * (c & 1)) = h;
  }
#pragma unroll
  for (int i = 0; i < NJ; ++i) {
    const int q = t + NTHR * i;
    const int n = q >> 2, c = q & 3;
    *reinterpret_cast<u32x4*>(Bt + n * 64 + 16 * (c ^ swb(n))) = st.b[i];
  }
}

// 64-deep k-steps for the one-tile-column (nj = 1, no conv) launches: their k-step is 8 MFMAs per wave at
// BK = 32, too little work to cover a step's fixed instruction overhead (loads, LDS, barrier, cursors);
// at 64 each step carries 16 and a K-long reduction takes half the steps.  Images: rows of 128 B (8
// chunks of 8 bf16) with the chunk XOR swizzle sw64(row) = (row >> 1) & 7, conflict-free for the 16-lane
// ds_read_b128 groups (16 consecutive rows of one chunk column cover all 16 16-B bank slots of 256 B).
template <bool ABF>
struct WrStage64 {
  float4 a[4];  // fp32 A: row q/16, k chunk of 4 q%16, q = tid + 512 i
  u32x4 b[2];   // W: row q/8, k chunk of 8 q%8
};
template <>
struct WrStage64<true> {
  u32x4 a[2];  // bf16 A: row q/8, k chunk of 8 q%8
  u32x4 b[2];
};
template <bool C, typename T, typename F>
struct pick_t { typedef T type; };
template <typename T, typename F>
struct pick_t<false, T, F> { typedef F type; };

__device__ __forceinline__ int sw64(int row) { return (row >> 1) & 7; }

template <bool ABF>
__device__ __forceinline__ void wr_load64(const Params& p, WrStage64<ABF>& st, int m0, int n0, int k0) {
  const int t = threadIdx.x;
  if constexpr (ABF) {
    const unsigned short* Ah = reinterpret_cast<const unsigned short*>(p.A);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int q = t + NTHR * i;
      const int r = m0 + (q >> 3), k = k0 + 8 * (q & 7);
      st.a[i] = *reinterpret_cast<const u32x4*>((r < p.M && k < p.K) ? (const void*)(Ah + (int64_t)r * p.lda + k)
                                                                     : (const void*)zero_page);
    }
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int q = t + NTHR * i;
      const int r = m0 + (q >> 4), k = k0 + 4 * (q & 15);
      st.a[i] = *reinterpret_cast<const float4*>((r < p.M && k < p.K) ? (const void*)(p.A + (int64_t)r * p.lda + k)
                                                                      : (const void*)zero_page);
    }
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int q = t + NTHR * i;
    const int n = n0 + (q >> 3), k = k0 + 8 * (q & 7);
    st.b[i] = *reinterpret_cast<const u32x4*>((n < p.N && k < p.K) ? (const void*)(p.W + (int64_t)n * p.ldw + k)
                                                                  : (const void*)zero_page);
  }
}

template <bool ABF>
__device__ __forceinline__ void wr_store64(const WrStage64<ABF>& st, char* At, char* Bt) {
  const int t = threadIdx.x;
  if constexpr (ABF) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int q = t + NTHR * i;
      const int row = q >> 3, c = q & 7;
      *reinterpret_cast<u32x4*>(At + row * 128 + 16 * (c ^ sw64(row))) = st.a[i];
    }
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int q = t + NTHR * i;
      const int row = q >> 4, c = q & 15;
      const float4 v = st.a[i];
      typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
      bf16x4 h;
      h[0] = (__bf16)v.x; h[1] = (__bf16)v.y; h[2] = (__bf16)v.z; h[3] = (__bf16)v.w;
      *reinterpret_cast<bf16x4*>(At + row * 128 + 16 * ((c >> 1) ^ sw64(row)) + 8 * (c & 1)) = h;
    }
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int q = t + NTHR * i;
    const int n = q >> 3, c = q & 7;
    *reinterpret_cast<u32x4*>(Bt + n * 128 + 16 * (c ^ sw64(n))) = st.b[i];
  }
}

template <bool ABF>
struct WrOff64 {
  uint32_t a[ABF ? 2 : 4];
  uint32_t w[2];
};
template <bool ABF>
__device__ __forceinline__ void wr_offsets64(const Params& p, WrOff64<ABF>& o, int m0, int n0) {
  const int t = threadIdx.x;
#pragma unroll
  for (int i = 0; i < (ABF ? 2 : 4); ++i) {
    const int q = t + NTHR * i;
    if constexpr (ABF) {
      const int row = min(m0 + (q >> 3), p.M - 1);
      o.a[i] = (uint32_t)(((int64_t)row * p.lda + 8 * (q & 7)) * 2);
    } else {
      const int row = min(m0 + (q >> 4), p.M - 1);
      o.a[i] = (uint32_t)(((int64_t)row * p.lda + 4 * (q & 15)) * 4);
    }
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int q = t + NTHR * i;
    const int n = min(n0 + (q >> 3), p.N - 1);
    o.w[i] = (uint32_t)(((int64_t)n * p.ldw + 8 * (q & 7)) * 2);
  }
}
template <bool ABF>
__device__ __forceinline__ void wr_load64_fast(const Params& p, WrStage64<ABF>& st, const WrOff64<ABF>& o, uint32_t ka,
                                               uint32_t kw) {
  const char* A = reinterpret_cast<const char*>(p.A);
  const char* W = reinterpret_cast<const char*>(p.W);
#pragma unroll
  for (int i = 0; i < (ABF ? 2 : 4); ++i) {
    if constexpr (ABF) st.a[i] = *reinterpret_cast<const u32x4*>(A + (o.a[i] + ka));
    else st.a[i] = *reinterpret_cast<const float4*>(A + (o.a[i] + ka));
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) st.b[i] = *reinterpret_cast<const u32x4*>(W + (o.w[i] + kw));
}

template <int NJ, bool CONV, bool RT, int DEP = 0, bool ABF = false, bool CE = false, bool RES = false,
          bool GA = false, bool ROT = false>
__global__ __launch_bounds__(NTHR, 1) void gemm_wr_kernel(Params p, int ntiles) {  // ntiles: all tiles
  typedef Cfg<NJ> CF;
  constexpr int BN = CF::BN, NT = 2 * NJ, BNR = CF::BNR;
  constexpr bool K64 = NJ == 1 && !CONV;  // 64-deep k-steps (WrStage64)
  constexpr int BKW = K64 ? 64 : BK;
  typedef typename pick_t<K64, WrStage64<ABF>, WrStage<NJ, ABF>>::type Stg;
  constexpr int AB = BM * BKW * 2, BB = BN * BKW * 2;  // bf16 images
  __shared__ __attribute__((aligned(16))) char a_img[2][AB];
  __shared__ __attribute__((aligned(16))) char b_img[2][BB];
  __shared__ __attribute__((aligned(16))) float bias_s[2][BNR];
  __shared__ float w2s[RT ? 3 * BN : 1];
  __shared__ __attribute__((aligned(16))) float red[RT ? BM * 12 : (CE ? BM * 8 : 1)];
  __shared__ __attribute__((aligned(16))) float ep_s[RT ? 1 : 8 * EpLds<NJ>::FLOATS];
  if constexpr (RT) {
    for (int i = threadIdx.x; i < 3 * BN; i += NTHR) {
      const int k = i / BN, n = i % BN;
      w2s[i] = n < p.N ? p.W2[k * p.N + n] : 0.f;
    }
  }

  const int nN = (p.N + BN - 1) / BN;
  const int nk = (p.K + BKW - 1) / BKW;
  const int G = gridDim.x, bid = blockIdx.x;
  const int r = (G % 8 == 0) ? (bid & 7) * (G >> 3) + (bid >> 3) : bid;  // XCD-grouped tile ranks
  const int* mlist = p.mtiles;
  if (mlist) ntiles = *p.n_mtiles * nN;  // device-side count (the list is built on the device)
  const int my = r < ntiles ? (ntiles - r + G - 1) / G : 0;
  const int S = my * nk;
  float* ep = ep_s + (threadIdx.x >> 6) * EpLds<NJ>::FLOATS;
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wm = wid >> 2, wn = wid & 3;
  const int lr = lane & 15, lk = lane >> 4;
  const bool vec = vec_ok(p);

  // Step -> (tile, k) coordinates are tracked incrementally by three cursors (the load cursor runs
  // DEPTH steps ahead of the epilogue cursor, the store cursor one ahead): a tile's (m0, n0) is
  // computed once when a cursor enters it.  Deriving them per k-step (s / nk, t / nN, t % nN with
  // runtime divisors) cost ~250 scalar instructions per k-step and wave against 8-24 MFMAs -- the
  // kernel was bound by instruction issue, not by MFMA or HBM (cursors: M = 8192, N = K = 384 14.9 ->
  // 11.2 us, M = 192064 bf16-A 138 -> 105 us at nj 1; profiles/r03_gemm_micro_v3.txt).
  struct Cur {
    int j, kk, m0, n0;  // tile ordinal of this workgroup, k-step within the tile, tile origin
  };
  auto enter = [&](Cur& c) __attribute__((always_inline)) {
    const int t = c.j * G + r;
    // past this workgroup's tiles (prefetch only) the raw index is kept: in range or beyond M
    if constexpr (CE) {
      // tied logits: row tiles fastest, so the 32 ranks of one XCD keep revisiting the same half of
      // the (small) activation rows out of their L2 while the vocabulary's weight tiles stream past
      const int nM = (p.M + BM - 1) / BM;
      c.m0 = (t < ntiles ? t % nM : nM + t) * BM;
      c.n0 = (t < ntiles ? t / nM : 0) * BN;
    } else {
      // the tile list is read through the constant address space: a uniform index then becomes a
      // scalar load (lgkmcnt) -- a vector load of it made the compiler drain every prefetch in flight
      // (vmcnt(0)) behind the branch around the load
      const int tm = t / nN;
      c.m0 = ((mlist && t < ntiles) ? ((const __attribute__((address_space(4))) int*)mlist)[tm] : tm) * BM;
      c.n0 = (t - tm * nN) * BN;
    }
  };
  auto advance = [&](Cur& c) __attribute__((always_inline)) {
    if (++c.kk == nk) {
      c.kk = 0;
      ++c.j;
      enter(c);
    }
  };
  Cur cl{0, 0, 0, 0}, cs{0, 0, 0, 0}, ce{0, 0, 0, 0};  // load, store, epilogue cursors
  enter(cl);
  cs = cl;
  ce = cl;
  // fast operand addressing (wr_offsets) when the launch allows it; offsets of the load cursor's tile
  constexpr int AES = ABF ? 2 : 4;
  // nj = 1 (64-deep k-steps) only: measured 4-7 % faster there, but 10-14 % slower on the fp32-A nj = 3
  // kernel (its five offsets at 253 VGPRs; profiles/r04_gemm_micro_fastaddr_ab.txt)
  const bool fast = WR_FAST && K64 && p.K % BKW == 0 && (uint64_t)p.M * p.lda * AES < (1ull << 32) &&
                    (uint64_t)p.N * p.ldw * 2 < (1ull << 32);
  typedef typename pick_t<K64, WrOff64<ABF>, WrOff<NJ, ABF>>::type Off;
  Off off;
  auto load = [&](Stg& st, bool issue) __attribute__((always_inline)) {
    if (issue) {
      if (fast) {
        if (cl.kk == 0) {
          if constexpr (K64) wr_offsets64<ABF>(p, off, cl.m0, cl.n0);
          else wr_offsets<NJ, ABF>(p, off, cl.m0, cl.n0);
        }
        const uint32_t k0 = (uint32_t)(cl.kk * BKW);
        if constexpr (K64) wr_load64_fast<ABF>(p, st, off, k0 * AES, k0 * 2);
        else wr_load_fast<NJ, ABF>(p, st, off, k0 * AES, k0 * 2);
      } else {
        if constexpr (K64) wr_load64<ABF>(p, st, cl.m0, cl.n0, cl.kk * BKW);
        else wr_load<NJ, CONV, ABF>(p, st, cl.m0, cl.n0, cl.kk * BK);
      }
    }
    advance(cl);
  };
  auto store = [&](int s, const Stg& st) __attribute__((always_inline)) {
    if constexpr (K64) wr_store64<ABF>(st, a_img[s & 1], b_img[s & 1]);
    else wr_store<NJ, ABF>(st, a_img[s & 1], b_img[s & 1]);
    if (cs.kk == 0) {  // first k-step of a tile: its bias slice (read by the tile's epilogue)
      float* dst = bias_s[cs.j & 1];
      for (int c = threadIdx.x; c < BN; c += NTHR) dst[c] = (p.bias && cs.n0 + c < p.N) ? p.bias[cs.n0 + c] : 0.f;
    }
    advance(cs);
  };

  f32x4 acc[4][NT];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // stage register sets are named variables (an array, even constant-indexed after unrolling,
  // ends up in scratch)
  constexpr int DEPTH = DEP ? DEP : WR_DEPTH;
  static_assert(DEPTH >= 3 && DEPTH <= 5, "stage sets are written out for depths 3..5");
  Stg st0, st1, st2, st3, st4;  // st3 / st4 unused (eliminated) below depth 4 / 5
  load(st0, S > 0);
  load(st1, S > 1);
  load(st2, S > 2);
  if constexpr (DEPTH >= 4) load(st3, S > 3);
  if constexpr (DEPTH >= 5) load(st4, S > 4);
  if (S > 0) store(0, st0);
  __syncthreads();

  // one k-step: `cur` held step s (already in LDS) and is refilled with step s + 3; `nxt` holds
  // step s + 1, which goes into the other LDS image after this step's MFMAs
  auto kstep = [&](int s, Stg& cur, const Stg& nxt) __attribute__((always_inline)) {
    // unconditional: past the last step the A rows fall beyond M and read the zero page, so the
    // number of loads in flight is the same on every path and the compiler's vmcnt waits stay
    // counted (a conditional load here would force vmcnt(0) at every later wait)
    load(cur, true);
    const char* At = a_img[s & 1];
    const char* Bt = b_img[s & 1];
    if constexpr (K64) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {  // two 32-deep halves of the 64-deep step
        bf16x8 a[4], b[NT];
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) {
          const int rr = wm * 64 + mt * 16 + lr;
          a[mt] = *reinterpret_cast<const bf16x8*>(At + rr * 128 + 16 * ((4 * h + lk) ^ sw64(rr)));
        }
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          const int n = wn * 32 + nt * 16 + lr;
          b[nt] = *reinterpret_cast<const bf16x8*>(Bt + n * 128 + 16 * ((4 * h + lk) ^ sw64(n)));
        }
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
#pragma unroll
          for (int nt = 0; nt < NT; ++nt)
            acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[nt], a[mt], acc[mt][nt], 0, 0, 0);
      }
    } else {
      bf16x8 a[4], b[NT];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        const int rr = wm * 64 + mt * 16 + lr;
        a[mt] = *reinterpret_cast<const bf16x8*>(At + rr * 64 + 16 * (lk ^ swb(rr)));
      }
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        const int n = wn * (32 * NJ) + nt * 16 + lr;
        b[nt] = *reinterpret_cast<const bf16x8*>(Bt + n * 64 + 16 * (lk ^ swb(n)));
      }
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[nt], a[mt], acc[mt][nt], 0, 0, 0);
    }
    if (s + 1 < S) store(s + 1, nxt);
    if (ce.kk == nk - 1) {
      const int m0 = ce.m0, n0 = ce.n0;
      const float* bsl = bias_s[ce.j & 1];
#if WR_ABL_EPI == 1  // timing ablation (wrong results): no epilogue, the accumulators only feed a never-taken store
      {
        float t = 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int q = 0; q < NT; ++q) t += acc[i][q][0] + acc[i][q][1] + acc[i][q][2] + acc[i][q][3];
        if (t == 1.2345e-37f) p.C[m0] = t;
      }
      if constexpr (true) {
      } else
#endif
      if constexpr (RT) {
        epilogue_router<NJ>(p, acc, bsl, w2s, red, m0, wm, wn, lr, lk);
      } else if constexpr (CE) {
        epilogue_ce<NJ>(p, acc, m0, n0, wm, wn, lr, lk, ep, reinterpret_cast<float2*>(red));
      } else if constexpr (RES) {  // act none, vec_ok (checked by the launcher)
        epilogue_lds<NJ, ACT_NONE, true>(p, acc, bsl, m0, n0, wm, wn, lr, lk, ep);
      } else if constexpr (ROT) {  // act none, fp32 C, vec_ok (checked by the launcher)
        epilogue_lds<NJ, ACT_NONE, false, true>(p, acc, bsl, m0, n0, wm, wn, lr, lk, ep);
      } else if constexpr (GA) {  // gelu / silu / sigmoid (checked by the launcher)
        switch (p.act) {
          case ACT_GELU: epilogue_gact<NJ, ACT_GELU>(p, acc, bsl, m0, n0, wm, wn, lr, lk, ep); break;
          case ACT_SILU: epilogue_gact<NJ, ACT_SILU>(p, acc, bsl, m0, n0, wm, wn, lr, lk, ep); break;
          default: epilogue_gact<NJ, ACT_SIGMOID>(p, acc, bsl, m0, n0, wm, wn, lr, lk, ep); break;
        }
      } else if (WR_EPI_LDS && vec) switch (p.act) {
        case ACT_GELU: epilogue_lds<NJ, ACT_GELU>(p, acc, bsl, m0, n0, wm, wn, lr, lk, ep); break;
        case ACT_SILU: epilogue_lds<NJ, ACT_SILU>(p, acc, bsl, m0, n0, wm, wn, lr, lk, ep); break;
        case ACT_SIGMOID: epilogue_lds<NJ, ACT_SIGMOID>(p, acc, bsl, m0, n0, wm, wn, lr, lk, ep); break;
        case ACT_RELU: epilogue_lds<NJ, ACT_RELU>(p, acc, bsl, m0, n0, wm, wn, lr, lk, ep); break;
        default: epilogue_lds<NJ, ACT_NONE>(p, acc, bsl, m0, n0, wm, wn, lr, lk, ep); break;
      } else switch (p.act) {
        case ACT_GELU: epilogue<NJ, ACT_GELU>(p, acc, bsl, m0, n0, wm, wn, lr, lk); break;
        case ACT_SILU: epilogue<NJ, ACT_SILU>(p, acc, bsl, m0, n0, wm, wn, lr, lk); break;
        case ACT_SIGMOID: epilogue<NJ, ACT_SIGMOID>(p, acc, bsl, m0, n0, wm, wn, lr, lk); break;
        case ACT_RELU: epilogue<NJ, ACT_RELU>(p, acc, bsl, m0, n0, wm, wn, lr, lk); break;
        default: epilogue<NJ, ACT_NONE>(p, acc, bsl, m0, n0, wm, wn, lr, lk); break;
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int q = 0; q < NT; ++q) acc[i][q] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    advance(ce);
    __syncthreads();
  };

  for (int s = 0; s < S; s += DEPTH) {
    if constexpr (DEPTH == 3) {
      kstep(s, st0, st1);
      if (s + 1 < S) kstep(s + 1, st1, st2);
      if (s + 2 < S) kstep(s + 2, st2, st0);
    } else if constexpr (DEPTH == 4) {
      kstep(s, st0, st1);
      if (s + 1 < S) kstep(s + 1, st1, st2);
      if (s + 2 < S) kstep(s + 2, st2, st3);
      if (s + 3 < S) kstep(s + 3, st3, st0);
    } else {
      kstep(s, st0, st1);
      if (s + 1 < S) kstep(s + 1, st1, st2);
      if (s + 2 < S) kstep(s + 2, st2, st3);
      if (s + 3 < S) kstep(s + 3, st3, st4);
      if (s + 4 < S) kstep(s + 4, st4, st0);
    }
  }
}

// Register pipeline depth per instantiation (0 = WR_DEPTH = 3).  A bf16-stored A halves a k-step's A slab,
// but a deeper pipeline for it measured no faster on the 192k-row launches (166 us at 3 and at 4 k-steps)
// and slower on the 8192-row ones (28 -> 35 us; depth 5 spills): the bf16-A kernel is not bound by the A
// bytes in flight (profiles/r03_kernel_stats_*.csv)
template <bool ABF>
constexpr int wr_dep() { return 0; }

template <int NJ, bool CONV, bool RT = false, bool ABF = false, bool CE = false, bool RES = false, bool GA = false,
          bool ROT = false>
void launch_wr(const Params& p, hipStream_t s) {
  static int resident = 0;
  const void* fn = (const void*)gemm_wr_kernel<NJ, CONV, RT, wr_dep<ABF>(), ABF, CE, RES, GA, ROT>;
  if (!resident) {
    int per_cu = 0, dev = 0, cus = 0;
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, NTHR, 0);
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    resident = std::max(1, per_cu) * std::max(1, cus);
  }
  const int tiles = ((p.M + BM - 1) / BM) * ((p.N + Cfg<NJ>::BN - 1) / Cfg<NJ>::BN);
  const int grid = std::min(tiles, resident);
  // a 5-deep pipeline (DEP = 5) for the one-wave 8192-row text-side launches measured 32.4 us vs
  // 30.1 us at depth 3 (profiles/r02_bench_v8_kernel_stats.csv): their time is not load latency
  gemm_wr_kernel<NJ, CONV, RT, wr_dep<ABF>(), ABF, CE, RES, GA, ROT><<<grid, NTHR, 0, s>>>(p, tiles);
}

}  // namespace wn
}  // namespace asrx

// Every instantiation lives in one of gemm_wr_i{1,2,3}.hip (compiled in parallel); other units only
// declare them.
#ifndef ASRX_WR_INSTANTIATE
#define ASRX_WR_DECL(NJ, CONV, RT, ABF) extern template void asrx::wn::launch_wr<NJ, CONV, RT, ABF>(const asrx::wn::Params&, hipStream_t);
#define ASRX_WR_DECL_CE(NJ) extern template void asrx::wn::launch_wr<NJ, false, false, true, true>(const asrx::wn::Params&, hipStream_t);
#define ASRX_WR_DECL_RES(NJ) extern template void asrx::wn::launch_wr<NJ, false, false, false, false, true>(const asrx::wn::Params&, hipStream_t);
#define ASRX_WR_DECL_GA(NJ, ABF) extern template void asrx::wn::launch_wr<NJ, false, false, ABF, false, false, true>(const asrx::wn::Params&, hipStream_t);
#define ASRX_WR_DECL_ROT(NJ, ABF) extern template void asrx::wn::launch_wr<NJ, false, false, ABF, false, false, false, true>(const asrx::wn::Params&, hipStream_t);
#else
#define ASRX_WR_DECL(NJ, CONV, RT, ABF) template void asrx::wn::launch_wr<NJ, CONV, RT, ABF>(const asrx::wn::Params&, hipStream_t);
#define ASRX_WR_DECL_CE(NJ) template void asrx::wn::launch_wr<NJ, false, false, true, true>(const asrx::wn::Params&, hipStream_t);
#define ASRX_WR_DECL_RES(NJ) template void asrx::wn::launch_wr<NJ, false, false, false, false, true>(const asrx::wn::Params&, hipStream_t);
#define ASRX_WR_DECL_GA(NJ, ABF) template void asrx::wn::launch_wr<NJ, false, false, ABF, false, false, true>(const asrx::wn::Params&, hipStream_t);
#define ASRX_WR_DECL_ROT(NJ, ABF) template void asrx::wn::launch_wr<NJ, false, false, ABF, false, false, false, true>(const asrx::wn::Params&, hipStream_t);
#endif
#define ASRX_WR_SET(NJ) ASRX_WR_DECL(NJ, false, false, false) ASRX_WR_DECL(NJ, true, false, false) \
  ASRX_WR_DECL(NJ, false, false, true) ASRX_WR_DECL(NJ, true, false, true) ASRX_WR_DECL(NJ, false, true, false)
#ifndef ASRX_WR_INSTANTIATE
ASRX_WR_SET(1)
ASRX_WR_SET(2)
ASRX_WR_SET(3)
ASRX_WR_DECL_CE(1)
ASRX_WR_DECL_CE(2)
ASRX_WR_DECL_CE(3)
ASRX_WR_DECL_RES(1)
ASRX_WR_DECL_RES(3)
ASRX_WR_DECL_GA(3, false)
ASRX_WR_DECL_GA(3, true)
ASRX_WR_DECL_ROT(1, true)
ASRX_WR_DECL_ROT(1, false)
ASRX_WR_DECL_ROT(3, true)
ASRX_WR_DECL_ROT(3, false)
#endif
