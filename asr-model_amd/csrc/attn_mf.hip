// Flash attention for the perf (bf16 MFMA) mode: F.scaled_dot_product_attention at model.py:307,
// head dim HD = 64 (tiny/small/medium configs) or 128 (the reference's own Dimensions(dims=512,
// head=4), model.py:746), non-causal or causal (top-left), Lq != Lk, ragged tails; q/k/v/o fp32
// (B, L, H, HD) with arbitrary strides, lse (B, H, Lq) natural log (consumed by the backward).
//
// Forward: workgroup = 8 waves = 256 query rows of one (b, h); wave = 32 rows.  Per 64-key tile:
//   S^T = K Q^T     v_mfma_f32_32x32x16_bf16 (K rows from LDS, Q^T fragments held in registers)
//                   -> each lane owns ONE query row (lane & 31) and 32 of the tile's 64 keys, so the
//                   row max is 31 in-lane fmax + one xor-32 exchange, and l is a per-lane partial sum
//   P^T = exp2(S^T * scale * log2e - m)   in registers, packed to bf16: the packed registers ARE the
//                   B operand of the next product (no LDS round trip, no lane permutes)
//   O^T += V^T P^T  32x32x16 MFMA, V^T fragments by ds_read_b64_tr_b16 (hardware transpose read
//                   of the row-major V tile), so O^T keeps the query on the lane too: the online-
//                   softmax rescale and the final 1/l are lane-local
// K/V tiles are register-staged (issue the next tile's global loads before the MFMAs, convert to
// bf16 and write LDS after them), double-buffered, one barrier per tile.  LDS images are XOR-
// swizzled at 16-byte granularity: K for the ds_read_b128 row reads, V for the transposed reads
// (both bank-conflict-free under the gfx950 lane-group rules).
//
// HD = 128 keeps every tile as NH = HD/64 separate 64-wide "halves" with exactly the HD = 64 image
// layout and swizzle, so one tile read pattern serves both head dims: the d-contractions run over
// both halves, and O^T / dK^T / dV^T / dQ^T hold HD/32 accumulator blocks (block dd -> half dd/2).
#include "common.h"

namespace asrx {

struct AttnStridesMF {
  int64_t b, l, h;
};

typedef short v4i16 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4i16 lds_v4i16;

namespace amf {

constexpr int QB = 256;  // query rows per forward workgroup
constexpr int KT = 64;   // keys per tile
constexpr int NTHR = 512;
constexpr int HALF = KT * 64;  // elements of one 64-wide half tile
constexpr float LOG2E = 1.4426950408889634f;
constexpr float LN2 = 0.6931471805599453f;

__device__ __forceinline__ int kswz(int key) { return (key >> 1) & 7; }
__device__ __forceinline__ int vswz(int key) { return ((key >> 1) & 1) << 2; }

// two floats -> one packed bf16 pair (RNE) in ONE v_cvt_pk_bf16_f32 (converting them separately and
// combining took a conversion, a shift and an or per pair)
__device__ __forceinline__ unsigned pack2(float a, float b) {
  typedef __attribute__((ext_vector_type(2))) float f2;
  typedef __attribute__((ext_vector_type(2))) __bf16 b2;
  return __builtin_bit_cast(unsigned, __builtin_convertvector((f2){a, b}, b2));
}

__device__ __forceinline__ bf16x8 pack8(const float (&v)[8]) {
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  u32x4 u = {pack2(v[0], v[1]), pack2(v[2], v[3]), pack2(v[4], v[5]), pack2(v[6], v[7])};
  return __builtin_bit_cast(bf16x8, u);
}

// Storage types of the attention operands: float (fp32) or bf16 (`bf16s`, the raw 16-bit pattern).
// q / k / v in bf16 are what the producers (per-head AbbyNormal, the k/v projection) write when
// attention is their only consumer: the kernels round fp32 inputs to bf16 anyway, so the products are
// bit-identical and a bf16 input halves the bytes and drops the per-tile conversions.
typedef unsigned short bf16s;

// 8 consecutive elements of one row, as staged through registers
template <typename T>
struct Row8 {
  float4 a, b;
};
template <>
struct Row8<bf16s> {
  uint4 u;
};

// one 16-byte chunk (8 consecutive d of half `hf`) of one key row of a K or V tile -> registers.
// Rows past Lk load the last row (always in bounds) and are zeroed, so there is no branch.
template <typename T>
__device__ __forceinline__ void stage_load(const T* base, AttnStridesMF st, int64_t key, int64_t Lk, int hf, int c,
                                           Row8<T>& x) {
  const int64_t kc = key < Lk ? key : Lk - 1;
  const T* p = base + kc * st.l + 64 * hf + 8 * c;
  if constexpr (sizeof(T) == 4) {
    x.a = *reinterpret_cast<const float4*>(p);
    x.b = *reinterpret_cast<const float4*>(p + 4);
    if (key >= Lk) {
      x.a = make_float4(0.f, 0.f, 0.f, 0.f);
      x.b = x.a;
    }
  } else {
    x.u = *reinterpret_cast<const uint4*>(p);
    if (key >= Lk) x.u = make_uint4(0u, 0u, 0u, 0u);
  }
}
// registers -> the bf16 LDS image (fp32 rounded here)
template <typename T>
__device__ __forceinline__ void stage_store(unsigned short* tile, int key, int pc, const Row8<T>& x) {
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  if constexpr (sizeof(T) == 4) {
    u32x4 u = {pack2(x.a.x, x.a.y), pack2(x.a.z, x.a.w), pack2(x.b.x, x.b.y), pack2(x.b.z, x.b.w)};
    *reinterpret_cast<u32x4*>(tile + key * 64 + 8 * pc) = u;
  } else {
    *reinterpret_cast<uint4*>(tile + key * 64 + 8 * pc) = x.u;
  }
}

// A operand of X^T (d rows 32 dd.. of one 64-wide half, k = 16 rows of X in the MFMA-output order
// of block kb2, half s2) from a transpose-swizzled [row][64] bf16 half tile (the V^T read)
__device__ __forceinline__ bf16x8 tr_frag(const unsigned short* X, int lane, int kb2, int s2, int dd) {
  const int g = lane >> 4, gi = lane & 15;
  const int trow = gi >> 2, tcol = 4 * (gi & 3);
  const int kbase = 32 * kb2 + 16 * s2 + 4 * (g >> 1);
  const int col = 32 * dd + 16 * (g & 1) + tcol;
  const int r1 = kbase + trow, r2 = kbase + 8 + trow;
  const v4i16 t1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(X + r1 * 64 + 8 * ((col >> 3) ^ vswz(r1)) + (col & 7)));
  const v4i16 t2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(X + r2 * 64 + 8 * ((col >> 3) ^ vswz(r2)) + (col & 7)));
  typedef short v8i16 __attribute__((ext_vector_type(8)));
  const v8i16 a8 = {t1[0], t1[1], t1[2], t1[3], t2[0], t2[1], t2[2], t2[3]};
  return __builtin_bit_cast(bf16x8, a8);
}

// register fragments (B operand of a d-contraction): row `row` of X, f[s] = d 64 (s/4) + 16 (s%4)
// + 8 hi .. +7, as bf16; rows past `rows` are zero
template <int HD, typename T>
__device__ __forceinline__ void row_frags(const T* base, int64_t stride_l, int64_t row, int64_t rows, int hi,
                                          bf16x8 (&f)[HD / 16]) {
#pragma unroll
  for (int s = 0; s < HD / 16; ++s) {
    const T* p = base + row * stride_l + 64 * (s >> 2) + 16 * (s & 3) + 8 * hi;
    if constexpr (sizeof(T) == 4) {
      float t[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      if (row < rows) {
        const float4 x = *reinterpret_cast<const float4*>(p), y = *reinterpret_cast<const float4*>(p + 4);
        t[0] = x.x; t[1] = x.y; t[2] = x.z; t[3] = x.w; t[4] = y.x; t[5] = y.y; t[6] = y.z; t[7] = y.w;
      }
      f[s] = pack8(t);
    } else {
      const uint4 u = row < rows ? *reinterpret_cast<const uint4*>(p) : make_uint4(0u, 0u, 0u, 0u);
      f[s] = __builtin_bit_cast(bf16x8, u);
    }
  }
}

// acc (32 rows of X from LDS x 32 register rows) += X[row 32 kb + j] . F over all HD dims
template <int HD>
__device__ __forceinline__ void dot_rows(f32x16& acc, const unsigned short* X, int row, int hi,
                                         const bf16x8 (&f)[HD / 16]) {
#pragma unroll
  for (int hf = 0; hf < HD / 64; ++hf)
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const bf16x8 a = *reinterpret_cast<const bf16x8*>(X + hf * HALF + row * 64 + 8 * ((2 * s + hi) ^ kswz(row)));
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, f[4 * hf + s], acc, 0, 0, 0);
    }
}

// store a (32 rows on the lane) x HD accumulator set scaled by `sc` to row `r` of Y
template <int HD, typename T = float>
__device__ __forceinline__ void store_rowT(T* yr, const f32x16 (&acc)[HD / 32], float sc, int hi) {
#pragma unroll
  for (int dd = 0; dd < HD / 32; ++dd)
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      const int c = 64 * (dd >> 1) + 32 * (dd & 1) + 8 * g4 + 4 * hi;
      if constexpr (sizeof(T) == 4) {
        *reinterpret_cast<float4*>(yr + c) = make_float4(acc[dd][4 * g4] * sc, acc[dd][4 * g4 + 1] * sc,
                                                         acc[dd][4 * g4 + 2] * sc, acc[dd][4 * g4 + 3] * sc);
      } else {
        *reinterpret_cast<uint2*>(yr + c) = make_uint2(pack2(acc[dd][4 * g4] * sc, acc[dd][4 * g4 + 1] * sc),
                                                       pack2(acc[dd][4 * g4 + 2] * sc, acc[dd][4 * g4 + 3] * sc));
      }
    }
}

// logical workgroup of hardware workgroup `bid` of G: consecutive logical ids on one XCD (hardware
// ids are dealt to the 8 XCDs round-robin), so the query blocks of one (b, h) share that XCD's L2
// copy of their K / V rows
__device__ __forceinline__ int64_t xcd_logical(int64_t bid, int64_t G) {
  const int64_t per = G / 8, rem = G % 8, x = bid % 8, q = bid / 8;
  return (x < rem ? x * (per + 1) : rem * (per + 1) + (x - rem) * per) + q;
}

// WPE: waves per SIMD the register budget is sized for (1: one 8-wave workgroup per CU; 4: two).
// XCD: 1-D grid remapped with xcd_logical.  PRIO: MFMA issue at raised wave priority (s_setprio),
// so a SIMD's other wave fills the matrix-core gaps with its softmax VALU work.
// TI: storage type of q / k / v, TO: of o (float or bf16s).
template <int HD, int WPE = 1, bool XCD = false, bool PRIO = false, typename TI = float, typename TO = float>
__global__ __launch_bounds__(NTHR, WPE) void attn_fwd_mf_kernel(const TI* __restrict__ q, const TI* __restrict__ k,
                                                              const TI* __restrict__ v, TO* __restrict__ o,
                                                              float* __restrict__ lse, AttnStridesMF sq,
                                                              AttnStridesMF sk, AttnStridesMF sv, AttnStridesMF so,
                                                              int64_t H, int64_t Lq, int64_t Lk, int causal,
                                                              float scale) {
  constexpr int NH = HD / 64;
  __shared__ __attribute__((aligned(16))) unsigned short Ks[2][NH * HALF];
  __shared__ __attribute__((aligned(16))) unsigned short Vs[2][NH * HALF];

  int b, h;
  int64_t q0;
  if (XCD) {
    const int64_t nqb = (Lq + QB - 1) / QB;
    const int64_t G = (int64_t)gridDim.x, L = xcd_logical(blockIdx.x, G);
    q0 = (L % nqb) * QB;
    h = (int)((L / nqb) % H);
    b = (int)(L / (nqb * H));
  } else {
    b = blockIdx.z;
    h = blockIdx.y;
    q0 = (int64_t)blockIdx.x * QB;
  }
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int j = lane & 31, hi = lane >> 5;
  const int64_t qi = q0 + wid * 32 + j;  // this lane's query row
  const TI* kb = k + b * sk.b + h * sk.h;
  const TI* vb = v + b * sv.b + h * sv.h;
  const float c = scale * LOG2E;

  // Q^T fragments (B operand): lane (q = j, hi) holds Q[q][64 hf + 16 s + 8 hi .. +7]
  bf16x8 qf[HD / 16];
  row_frags<HD>(q + b * sq.b + h * sq.h, sq.l, qi, Lq, hi, qf);

  int64_t kend = Lk;
  if (causal) kend = min(Lk, q0 + QB);
  const int ntiles = (int)((kend + KT - 1) / KT);
  const int skey = tid >> 3, sc = tid & 7;  // staging: one 16-B chunk of each half of one key row

  Row8<TI> ka[NH], va[NH];
#pragma unroll
  for (int hf = 0; hf < NH; ++hf) {
    stage_load(kb, sk, skey, Lk, hf, sc, ka[hf]);
    stage_load(vb, sv, skey, Lk, hf, sc, va[hf]);
    stage_store(Ks[0] + hf * HALF, skey, sc ^ kswz(skey), ka[hf]);
    stage_store(Vs[0] + hf * HALF, skey, sc ^ vswz(skey), va[hf]);
  }
  __syncthreads();

  f32x16 oacc[HD / 32];
#pragma unroll
  for (int d = 0; d < HD / 32; ++d)
#pragma unroll
    for (int r = 0; r < 16; ++r) oacc[d][r] = 0.f;
  float m = -INFINITY;  // running max of raw scores (log2 domain after * c)
  float l = 0.f;        // partial (this half's keys) running denominator

  for (int t = 0; t < ntiles; ++t) {
    const int buf = t & 1;
    const int64_t k0 = (int64_t)t * KT;
    if (t + 1 < ntiles) {  // next tile's loads fly under this tile's MFMAs
#pragma unroll
      for (int hf = 0; hf < NH; ++hf) {
        stage_load(kb, sk, k0 + KT + skey, Lk, hf, sc, ka[hf]);
        stage_load(vb, sv, k0 + KT + skey, Lk, hf, sc, va[hf]);
      }
    }
    const unsigned short* Kt = Ks[buf];
    const unsigned short* Vt = Vs[buf];

    // ---- S^T = K Q^T : two 32-key blocks
    f32x16 sacc[2];
    if (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kb2 = 0; kb2 < 2; ++kb2) {
#pragma unroll
      for (int r = 0; r < 16; ++r) sacc[kb2][r] = 0.f;
      dot_rows<HD>(sacc[kb2], Kt, 32 * kb2 + j, hi, qf);
    }
    if (PRIO) __builtin_amdgcn_s_setprio(0);

    // ---- mask + online softmax (lane = query j, keys crow(r, hi) of each block)
    // wave-uniform (readfirstlane: the compiler cannot prove wid uniform, and a per-lane mask flag turned the
    // block below into a 32-deep exec-masked branch chain run on EVERY tile, ~100 scalar instructions)
    const bool need_mask =
        __builtin_amdgcn_readfirstlane((int)((k0 + KT > Lk) || (causal && k0 + KT - 1 > q0 + wid * 32))) != 0;
    if (need_mask) {  // keys of this tile at or past lim are masked: key >= Lk, or key > qi when causal
      const int lim = (int)min(min(Lk - k0, (int64_t)KT), causal ? qi - k0 + 1 : (int64_t)KT);
#pragma unroll
      for (int kb2 = 0; kb2 < 2; ++kb2)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = 32 * kb2 + (r & 3) + 8 * (r >> 2) + 4 * hi;
          sacc[kb2][r] = key >= lim ? -INFINITY : sacc[kb2][r];
        }
    }
    float tmax = -INFINITY;
#pragma unroll
    for (int kb2 = 0; kb2 < 2; ++kb2)
#pragma unroll
      for (int r = 0; r < 16; ++r) tmax = fmaxf(tmax, sacc[kb2][r]);
    {  // xor-32 partner by v_permlane32_swap (VALU) instead of a ds_bpermute round trip
      float ta = tmax, tb = tmax;
      xrow32(ta, tb);
      tmax = fmaxf(ta, tb);
    }
    // lazy rescale: the running max moves only when a score passes it by more than 2^8 in the exp2
    // domain (p <= 256 otherwise, exact in the fp32 sums and fine in bf16), so most tiles skip the
    // O / l rescale; m = -inf (nothing seen yet) moves on the first finite score
    const bool up = tmax * c > m * c + 8.f;
    if (__any(up)) {  // wave-uniform
      const float alpha = up ? __builtin_amdgcn_exp2f(m * c - tmax * c) : 1.f;  // m = -inf -> 0
      if (up) m = tmax;
      l *= alpha;
#pragma unroll
      for (int d = 0; d < HD / 32; ++d)
#pragma unroll
        for (int r = 0; r < 16; ++r) oacc[d][r] *= alpha;
    }
    const float mc = m == -INFINITY ? 0.f : m * c;
    // exp arguments and the row-sum partials two at a time on the packed FP32 ALU (v_pk_fma_f32 /
    // v_pk_add_f32: half the issue of the scalar forms); four independent partial sums instead of one
    // dependent chain of 32 adds
    typedef __attribute__((ext_vector_type(2))) float f2;
    const f2 c2 = {c, c}, m2 = {-mc, -mc};
    bf16x8 pb[2][2];
    f2 ls[2] = {{0.f, 0.f}, {0.f, 0.f}};
#pragma unroll
    for (int kb2 = 0; kb2 < 2; ++kb2)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        float pv[8];
#pragma unroll
        for (int e = 0; e < 8; e += 2) {
          const f2 x = {sacc[kb2][8 * s2 + e], sacc[kb2][8 * s2 + e + 1]};
          const f2 a = __builtin_elementwise_fma(x, c2, m2);
          pv[e] = __builtin_amdgcn_exp2f(a.x);
          pv[e + 1] = __builtin_amdgcn_exp2f(a.y);
          ls[(e >> 1) & 1] += (f2){pv[e], pv[e + 1]};
        }
        pb[kb2][s2] = pack8(pv);
      }
    const f2 lt2 = ls[0] + ls[1];
    l += lt2.x + lt2.y;

    // ---- O^T += V^T P^T
    if (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kb2 = 0; kb2 < 2; ++kb2)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int d = 0; d < HD / 32; ++d)
          oacc[d] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tr_frag(Vt + (d >> 1) * HALF, lane, kb2, s2, d & 1),
                                                            pb[kb2][s2], oacc[d], 0, 0, 0);
    if (PRIO) __builtin_amdgcn_s_setprio(0);

    if (t + 1 < ntiles) {  // every wave finished reading buf^1 (tile t-1) before the last barrier
#pragma unroll
      for (int hf = 0; hf < NH; ++hf) {
        stage_store(Ks[buf ^ 1] + hf * HALF, skey, sc ^ kswz(skey), ka[hf]);
        stage_store(Vs[buf ^ 1] + hf * HALF, skey, sc ^ vswz(skey), va[hf]);
      }
    }
    __syncthreads();
  }

  // ---- finalize: l over both halves, O = O^T / l, lse in natural log
  const float lt = l + __shfl_xor(l, 32);
  if (qi < Lq) {
    store_rowT<HD, TO>(o + b * so.b + h * so.h + qi * so.l, oacc, 1.0f / lt, hi);
    if (hi == 0) lse[((int64_t)b * H + h) * Lq + qi] = (m * c + __builtin_amdgcn_logf(lt)) * LN2;
  }
}

// Software-pipelined forward (HD = 64; asrx_set_attn_variant, 1 = this kernel, the default): the same
// per-element arithmetic in the same order as attn_fwd_mf_kernel (bit-identical outputs), re-timed so the
// score MFMAs of tile t + 1 share one basic block with the softmax VALU of tile t and the compiler can
// put the exp / convert / sum work in the MFMA gaps (one wave alone had nothing to issue under its
// score MFMAs, and the softmax had no MFMA to hide under).  K runs one tile ahead of V: iteration t
// reads K(t + 1) and V(t), and writes K(t + 2) into K(t)'s buffer and V(t + 1) into V(t - 1)'s, so one
// barrier per tile still separates every write from the reads of its buffer.  The boundary mask of a
// tile is applied when its scores are made (end of the previous iteration), outside the interleaved
// block; loads past the last tile are clamped (stage_load) and their scores never used.  Two named
// score sets (loop unrolled by two) instead of a runtime index, which would go to scratch.
template <bool XCD, typename TI, typename TO>
__global__ __launch_bounds__(NTHR, 1) void attn_fwd_sp_kernel(const TI* __restrict__ q, const TI* __restrict__ k,
                                                            const TI* __restrict__ v, TO* __restrict__ o,
                                                            float* __restrict__ lse, AttnStridesMF sq,
                                                            AttnStridesMF sk, AttnStridesMF sv, AttnStridesMF so,
                                                            int64_t H, int64_t Lq, int64_t Lk, int causal,
                                                            float scale) {
  constexpr int HD = 64;
  __shared__ __attribute__((aligned(16))) unsigned short Ks[2][HALF];
  __shared__ __attribute__((aligned(16))) unsigned short Vs[2][HALF];

  int b, h;
  int64_t q0;
  if (XCD) {
    const int64_t nqb = (Lq + QB - 1) / QB;
    const int64_t G = (int64_t)gridDim.x, L = xcd_logical(blockIdx.x, G);
    q0 = (L % nqb) * QB;
    h = (int)((L / nqb) % H);
    b = (int)(L / (nqb * H));
  } else {
    b = blockIdx.z;
    h = blockIdx.y;
    q0 = (int64_t)blockIdx.x * QB;
  }
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int j = lane & 31, hi = lane >> 5;
  const int64_t qi = q0 + wid * 32 + j;
  const TI* kb = k + b * sk.b + h * sk.h;
  const TI* vb = v + b * sv.b + h * sv.h;
  const float c = scale * LOG2E;

  bf16x8 qf[HD / 16];
  row_frags<HD>(q + b * sq.b + h * sq.h, sq.l, qi, Lq, hi, qf);

  int64_t kend = Lk;
  if (causal) kend = min(Lk, q0 + QB);
  const int ntiles = (int)((kend + KT - 1) / KT);
  const int skey = tid >> 3, sc = tid & 7;

  Row8<TI> ka, va;
  stage_load(kb, sk, skey, Lk, 0, sc, ka);
  stage_load(vb, sv, skey, Lk, 0, sc, va);
  stage_store(Ks[0], skey, sc ^ kswz(skey), ka);
  stage_store(Vs[0], skey, sc ^ vswz(skey), va);
  stage_load(kb, sk, KT + skey, Lk, 0, sc, ka);
  stage_store(Ks[1], skey, sc ^ kswz(skey), ka);
  __syncthreads();

  // scores of tile tt (K image Kt) into s, boundary keys masked (wave-uniform test, as attn_fwd_mf_kernel)
  auto scores = [&](f32x16 (&s)[2], const unsigned short* Kt, int tt) {
#pragma unroll
    for (int kb2 = 0; kb2 < 2; ++kb2) {
#pragma unroll
      for (int r = 0; r < 16; ++r) s[kb2][r] = 0.f;
      dot_rows<HD>(s[kb2], Kt, 32 * kb2 + j, hi, qf);
    }
  };
  auto mask = [&](f32x16 (&s)[2], int tt) {
    const int64_t k0 = (int64_t)tt * KT;
    const bool need_mask =
        __builtin_amdgcn_readfirstlane((int)((k0 + KT > Lk) || (causal && k0 + KT - 1 > q0 + wid * 32))) != 0;
    if (need_mask) {
      const int lim = (int)min(min(Lk - k0, (int64_t)KT), causal ? qi - k0 + 1 : (int64_t)KT);
#pragma unroll
      for (int kb2 = 0; kb2 < 2; ++kb2)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = 32 * kb2 + (r & 3) + 8 * (r >> 2) + 4 * hi;
          s[kb2][r] = key >= lim ? -INFINITY : s[kb2][r];
        }
    }
  };

  f32x16 sA[2], sB[2];
  scores(sA, Ks[0], 0);
  mask(sA, 0);

  f32x16 oacc[HD / 32];
#pragma unroll
  for (int d = 0; d < HD / 32; ++d)
#pragma unroll
    for (int r = 0; r < 16; ++r) oacc[d][r] = 0.f;
  float m = -INFINITY;
  float l = 0.f;

  auto step = [&](int t, f32x16 (&cur)[2], f32x16 (&nxt)[2]) {
    const int buf = t & 1;
    const int64_t k0 = (int64_t)t * KT;
    stage_load(vb, sv, k0 + KT + skey, Lk, 0, sc, va);      // V(t + 1)
    stage_load(kb, sk, k0 + 2 * KT + skey, Lk, 0, sc, ka);  // K(t + 2)

    float tmax = -INFINITY;
#pragma unroll
    for (int kb2 = 0; kb2 < 2; ++kb2)
#pragma unroll
      for (int r = 0; r < 16; ++r) tmax = fmaxf(tmax, cur[kb2][r]);
    {
      float ta = tmax, tb = tmax;
      xrow32(ta, tb);
      tmax = fmaxf(ta, tb);
    }
    const bool up = tmax * c > m * c + 8.f;
    if (__any(up)) {
      const float alpha = up ? __builtin_amdgcn_exp2f(m * c - tmax * c) : 1.f;
      if (up) m = tmax;
      l *= alpha;
#pragma unroll
      for (int d = 0; d < HD / 32; ++d)
#pragma unroll
        for (int r = 0; r < 16; ++r) oacc[d][r] *= alpha;
    }
    const float mc = m == -INFINITY ? 0.f : m * c;

    scores(nxt, Ks[buf ^ 1], t + 1);  // tile t + 1 (unused past the last tile)

    // exp arguments and row-sum partials as single (not packed) FP32 ops: the same roundings as the packed
    // forms, and the packed forms cost more than two singles beside MFMAs (MI355X_MICROARCH.md)
    bf16x8 pb[2][2];
    float l0x = 0.f, l0y = 0.f, l1x = 0.f, l1y = 0.f;
#pragma unroll
    for (int kb2 = 0; kb2 < 2; ++kb2)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        float pv[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) pv[e] = __builtin_amdgcn_exp2f(__builtin_fmaf(cur[kb2][8 * s2 + e], c, -mc));
        l0x += pv[0]; l0y += pv[1]; l1x += pv[2]; l1y += pv[3];
        l0x += pv[4]; l0y += pv[5]; l1x += pv[6]; l1y += pv[7];
        pb[kb2][s2] = pack8(pv);
      }
    const float ltx = l0x + l1x, lty = l0y + l1y;
    l += ltx + lty;

#pragma unroll
    for (int kb2 = 0; kb2 < 2; ++kb2)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int d = 0; d < HD / 32; ++d)
          oacc[d] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tr_frag(Vs[buf], lane, kb2, s2, d & 1), pb[kb2][s2],
                                                            oacc[d], 0, 0, 0);

    mask(nxt, t + 1);
    stage_store(Ks[buf], skey, sc ^ kswz(skey), ka);
    stage_store(Vs[buf ^ 1], skey, sc ^ vswz(skey), va);
    __syncthreads();
  };

  int t = 0;
  for (; t + 2 <= ntiles; t += 2) {
    step(t, sA, sB);
    step(t + 1, sB, sA);
  }
  if (t < ntiles) step(t, sA, sB);

  const float lt = l + __shfl_xor(l, 32);
  if (qi < Lq) {
    store_rowT<HD, TO>(o + b * so.b + h * so.h + qi * so.l, oacc, 1.0f / lt, hi);
    if (hi == 0) lse[((int64_t)b * H + h) * Lq + qi] = (m * c + __builtin_amdgcn_logf(lt)) * LN2;
  }
}

// ============================================================================================
// Backward (perf mode), the same operand tricks as the forward:
//   Delta_i = rowsum(dO_i * O_i) (attn_delta_kernel), P = exp(S * scale - lse), dS = P (dP - Delta)
//   dkdv kernel (key-major, lane = key): S = Q K^T and dP = dO V^T with K^T / V^T fragments held in
//     registers for the wave's 32 keys, Q / dO rows read from LDS; P and dS are MFMA outputs with
//     the query on the row, so they pack straight into the B operand of dV^T += dO^T P and
//     dK^T += Q^T dS (dO^T / Q^T by transposed LDS reads) and both accumulators keep the key on
//     the lane.  Q and dO tiles are staged twice: row-read and transpose-read swizzles.
//   dq kernel (query-major, lane = query, the forward's layout): S^T = K Q^T, dP^T = V dO^T with
//     Q^T / dO^T fragments in registers, dS^T packed into the B operand of dQ^T += K^T dS^T.
// No atomics; every accumulator is written once.  HD = 128 runs 4 waves per workgroup (one wave
// per SIMD: its K/V fragments and four accumulator blocks need more than the 256 registers a
// wave gets at two waves per SIMD); HD = 64 runs 8.

template <int HD>
struct BwdCfg {
  static constexpr int NW = HD == 64 ? 8 : 4;
  static constexpr int NT = 64 * NW;
  static constexpr int RI = KT * 8 / NT;  // staging row iterations (a thread stages chunk tid&7 of rows tid/8 + i NT/8)
};

constexpr int BQT = 64;  // queries per tile of the dkdv loop

// TI: storage type of q / k / v, TD: of dO (float or bf16s).
template <int HD, typename TI = float, typename TD = float>
__global__ __launch_bounds__(BwdCfg<HD>::NT, 1) void attn_bwd_dkdv_mf_kernel(
    const TI* __restrict__ q, const TI* __restrict__ k, const TI* __restrict__ v,
    const TD* __restrict__ dO, const float* __restrict__ lse, const float* __restrict__ delta,
    float* __restrict__ dk, float* __restrict__ dv, AttnStridesMF sq, AttnStridesMF sk, AttnStridesMF sv,
    AttnStridesMF sd, AttnStridesMF sdk, AttnStridesMF sdv, int64_t H, int64_t Lq, int64_t Lk, int causal,
    float scale) {
  typedef BwdCfg<HD> C;
  constexpr int NH = HD / 64;
  __shared__ __attribute__((aligned(16))) unsigned short Qr[2][NH * HALF], Qt[2][NH * HALF];
  __shared__ __attribute__((aligned(16))) unsigned short Dr[2][NH * HALF], Dt[2][NH * HALF];
  __shared__ __attribute__((aligned(16))) float2 LD[2][BQT];  // (lse * log2e or +inf past Lq, Delta)

  // 1-D grid, key blocks of one (b, h) contiguous on one XCD (xcd_logical)
  const int64_t nkb = (Lk + 32 * C::NW - 1) / (32 * C::NW), L = xcd_logical(blockIdx.x, gridDim.x);
  const int b = (int)(L / (nkb * H)), h = (int)((L / nkb) % H);
  const int64_t k0 = (L % nkb) * (32 * C::NW);
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int j = lane & 31, hi = lane >> 5;
  const int64_t key = k0 + wid * 32 + j;  // this lane's key
  const TI* qb = q + b * sq.b + h * sq.h;
  const TD* gb = dO + b * sd.b + h * sd.h;
  const float* lb = lse + ((int64_t)b * H + h) * Lq;
  const float* db = delta + ((int64_t)b * H + h) * Lq;
  const float c = scale * LOG2E;

  bf16x8 kf[HD / 16], vf[HD / 16];
  row_frags<HD>(k + b * sk.b + h * sk.h, sk.l, key, Lk, hi, kf);
  row_frags<HD>(v + b * sv.b + h * sv.h, sv.l, key, Lk, hi, vf);

  const int64_t qt0 = causal ? k0 / BQT : 0;  // causal: tiles entirely before the block's keys are masked
  const int ntiles = (int)((Lq + BQT - 1) / BQT - qt0);
  const int srow = tid >> 3, sc = tid & 7;
  Row8<TI> qa[C::RI][NH];
  Row8<TD> ga[C::RI][NH];
  float2 ld = make_float2(0.f, 0.f);
  auto stage_ld = [&](int t) {
    const int64_t q0 = (qt0 + t) * BQT;
#pragma unroll
    for (int i = 0; i < C::RI; ++i)
#pragma unroll
      for (int hf = 0; hf < NH; ++hf) {
        stage_load(qb, sq, q0 + srow + i * (C::NT / 8), Lq, hf, sc, qa[i][hf]);
        stage_load(gb, sd, q0 + srow + i * (C::NT / 8), Lq, hf, sc, ga[i][hf]);
      }
    if (tid < BQT) {
      const int64_t qi = q0 + tid;
      ld = qi < Lq ? make_float2(lb[qi] * LOG2E, db[qi]) : make_float2(INFINITY, 0.f);
    }
  };
  auto stage_st = [&](int buf) {
#pragma unroll
    for (int i = 0; i < C::RI; ++i)
#pragma unroll
      for (int hf = 0; hf < NH; ++hf) {
        const int row = srow + i * (C::NT / 8);
        stage_store(Qr[buf] + hf * HALF, row, sc ^ kswz(row), qa[i][hf]);
        stage_store(Qt[buf] + hf * HALF, row, sc ^ vswz(row), qa[i][hf]);
        stage_store(Dr[buf] + hf * HALF, row, sc ^ kswz(row), ga[i][hf]);
        stage_store(Dt[buf] + hf * HALF, row, sc ^ vswz(row), ga[i][hf]);
      }
    if (tid < BQT) LD[buf][tid] = ld;
  };

  f32x16 dvacc[HD / 32], dkacc[HD / 32];
#pragma unroll
  for (int d = 0; d < HD / 32; ++d)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      dvacc[d][r] = 0.f;
      dkacc[d][r] = 0.f;
    }
  if (ntiles > 0) {
    stage_ld(0);
    stage_st(0);
  }
  __syncthreads();

  for (int t = 0; t < ntiles; ++t) {
    const int buf = t & 1;
    const int64_t q0 = (qt0 + t) * BQT;
    if (t + 1 < ntiles) stage_ld(t + 1);
    const bool need_mask = __builtin_amdgcn_readfirstlane((int)(causal && q0 < k0 + wid * 32 + 32)) != 0;
    const int kq = (int)(key - q0);  // this lane's key relative to the tile's first query
    // one 32-query half at a time (keeps S / dP / P / dS of a single half live)
#pragma unroll
    for (int qb2 = 0; qb2 < 2; ++qb2) {
      // ---- S = Q K^T, dP = dO V^T (rows = queries, lane = key)
      f32x16 sacc, pacc;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        sacc[r] = 0.f;
        pacc[r] = 0.f;
      }
      dot_rows<HD>(sacc, Qr[buf], 32 * qb2 + j, hi, kf);
      dot_rows<HD>(pacc, Dr[buf], 32 * qb2 + j, hi, vf);
      // ---- P, dS (query row of register r: 32 qb2 + (r & 3) + 8 (r >> 2) + 4 hi)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        float pv[8], dsv[8];
#pragma unroll
        for (int e4 = 0; e4 < 2; ++e4) {
          const int ql = 32 * qb2 + 8 * (2 * s2 + e4) + 4 * hi;  // 4 consecutive queries
          const float4 lo = *reinterpret_cast<const float4*>(&LD[buf][ql]);
          const float4 hi4 = *reinterpret_cast<const float4*>(&LD[buf][ql + 2]);
          const float l2v[4] = {lo.x, lo.z, hi4.x, hi4.z}, dlv[4] = {lo.y, lo.w, hi4.y, hi4.w};
          // two elements at a time on the packed FP32 ALU (exp stays scalar)
#pragma unroll
          for (int e = 0; e < 4; e += 2) {
            typedef __attribute__((ext_vector_type(2))) float f2;
            const int r = 8 * s2 + 4 * e4 + e;
            const f2 a = __builtin_elementwise_fma((f2){sacc[r], sacc[r + 1]}, (f2){c, c}, (f2){-l2v[e], -l2v[e + 1]});
            f2 p = {__builtin_amdgcn_exp2f(a.x), __builtin_amdgcn_exp2f(a.y)};
            if (need_mask) {
              p.x = kq > ql + e ? 0.f : p.x;
              p.y = kq > ql + e + 1 ? 0.f : p.y;
            }
            const f2 ds = p * ((f2){pacc[r], pacc[r + 1]} - (f2){dlv[e], dlv[e + 1]});
            pv[4 * e4 + e] = p.x;
            pv[4 * e4 + e + 1] = p.y;
            dsv[4 * e4 + e] = ds.x;
            dsv[4 * e4 + e + 1] = ds.y;
          }
        }
        const bf16x8 pb = pack8(pv), sb = pack8(dsv);
        // ---- dV^T += dO^T P, dK^T += Q^T dS  (lane = key)
#pragma unroll
        for (int d = 0; d < HD / 32; ++d) {
          dvacc[d] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tr_frag(Dt[buf] + (d >> 1) * HALF, lane, qb2, s2, d & 1),
                                                             pb, dvacc[d], 0, 0, 0);
          dkacc[d] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tr_frag(Qt[buf] + (d >> 1) * HALF, lane, qb2, s2, d & 1),
                                                             sb, dkacc[d], 0, 0, 0);
        }
      }
    }
    if (t + 1 < ntiles) stage_st(buf ^ 1);
    __syncthreads();
  }

  if (key < Lk) {
    store_rowT<HD>(dk + b * sdk.b + h * sdk.h + key * sdk.l, dkacc, scale, hi);
    store_rowT<HD>(dv + b * sdv.b + h * sdv.h + key * sdv.l, dvacc, 1.f, hi);
  }
}

template <int HD, typename TI = float, typename TD = float>
__global__ __launch_bounds__(BwdCfg<HD>::NT, 1) void attn_bwd_dq_mf_kernel(
    const TI* __restrict__ q, const TI* __restrict__ k, const TI* __restrict__ v,
    const TD* __restrict__ dO, const float* __restrict__ lse, const float* __restrict__ delta,
    float* __restrict__ dq, AttnStridesMF sq, AttnStridesMF sk, AttnStridesMF sv, AttnStridesMF sd,
    AttnStridesMF sdq, int64_t H, int64_t Lq, int64_t Lk, int causal, float scale) {
  typedef BwdCfg<HD> C;
  constexpr int NH = HD / 64;
  __shared__ __attribute__((aligned(16))) unsigned short Kr[2][NH * HALF], Kt2[2][NH * HALF], Vr[2][NH * HALF];

  // 1-D grid, query blocks of one (b, h) contiguous on one XCD (xcd_logical)
  const int64_t nqb = (Lq + 32 * C::NW - 1) / (32 * C::NW), L = xcd_logical(blockIdx.x, gridDim.x);
  const int b = (int)(L / (nqb * H)), h = (int)((L / nqb) % H);
  const int64_t q0 = (L % nqb) * (32 * C::NW);
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int j = lane & 31, hi = lane >> 5;
  const int64_t qi = q0 + wid * 32 + j;  // this lane's query row
  const TI* kbp = k + b * sk.b + h * sk.h;
  const TI* vbp = v + b * sv.b + h * sv.h;
  const float c = scale * LOG2E;

  bf16x8 qf[HD / 16], gf[HD / 16];
  row_frags<HD>(q + b * sq.b + h * sq.h, sq.l, qi, Lq, hi, qf);
  row_frags<HD>(dO + b * sd.b + h * sd.h, sd.l, qi, Lq, hi, gf);
  const float l2 = qi < Lq ? lse[((int64_t)b * H + h) * Lq + qi] * LOG2E : 0.f;
  const float dl = qi < Lq ? delta[((int64_t)b * H + h) * Lq + qi] : 0.f;

  int64_t kend = Lk;
  if (causal) kend = min(Lk, q0 + 32 * C::NW);
  const int ntiles = (int)((kend + KT - 1) / KT);
  const int skey = tid >> 3, sc = tid & 7;

  Row8<TI> ka[C::RI][NH], va[C::RI][NH];
  auto stage_ld = [&](int64_t k0) {
#pragma unroll
    for (int i = 0; i < C::RI; ++i)
#pragma unroll
      for (int hf = 0; hf < NH; ++hf) {
        stage_load(kbp, sk, k0 + skey + i * (C::NT / 8), Lk, hf, sc, ka[i][hf]);
        stage_load(vbp, sv, k0 + skey + i * (C::NT / 8), Lk, hf, sc, va[i][hf]);
      }
  };
  auto stage_st = [&](int buf) {
#pragma unroll
    for (int i = 0; i < C::RI; ++i)
#pragma unroll
      for (int hf = 0; hf < NH; ++hf) {
        const int row = skey + i * (C::NT / 8);
        stage_store(Kr[buf] + hf * HALF, row, sc ^ kswz(row), ka[i][hf]);
        stage_store(Kt2[buf] + hf * HALF, row, sc ^ vswz(row), ka[i][hf]);
        stage_store(Vr[buf] + hf * HALF, row, sc ^ kswz(row), va[i][hf]);
      }
  };
  stage_ld(0);
  stage_st(0);
  __syncthreads();

  f32x16 dqacc[HD / 32];
#pragma unroll
  for (int d = 0; d < HD / 32; ++d)
#pragma unroll
    for (int r = 0; r < 16; ++r) dqacc[d][r] = 0.f;

  for (int t = 0; t < ntiles; ++t) {
    const int buf = t & 1;
    const int64_t k0 = (int64_t)t * KT;
    if (t + 1 < ntiles) stage_ld(k0 + KT);
    f32x16 sacc[2], pacc[2];
#pragma unroll
    for (int kb2 = 0; kb2 < 2; ++kb2) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        sacc[kb2][r] = 0.f;
        pacc[kb2][r] = 0.f;
      }
      dot_rows<HD>(sacc[kb2], Kr[buf], 32 * kb2 + j, hi, qf);
      dot_rows<HD>(pacc[kb2], Vr[buf], 32 * kb2 + j, hi, gf);
    }
    const bool need_mask =
        __builtin_amdgcn_readfirstlane((int)((k0 + KT > Lk) || (causal && k0 + KT - 1 > q0 + wid * 32))) != 0;
    const int lim = need_mask ? (int)min(min(Lk - k0, (int64_t)KT), causal ? qi - k0 + 1 : (int64_t)KT) : KT;
    bf16x8 sb[2][2];
#pragma unroll
    for (int kb2 = 0; kb2 < 2; ++kb2)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        float dsv[8];
#pragma unroll
        for (int e = 0; e < 8; e += 2) {  // two elements at a time on the packed FP32 ALU
          typedef __attribute__((ext_vector_type(2))) float f2;
          const int r = 8 * s2 + e;
          const f2 a = __builtin_elementwise_fma((f2){sacc[kb2][r], sacc[kb2][r + 1]}, (f2){c, c}, (f2){-l2, -l2});
          f2 p = {__builtin_amdgcn_exp2f(a.x), __builtin_amdgcn_exp2f(a.y)};
          if (need_mask) {
            p.x = (32 * kb2 + (r & 3) + 8 * (r >> 2) + 4 * hi) >= lim ? 0.f : p.x;
            p.y = (32 * kb2 + ((r + 1) & 3) + 8 * ((r + 1) >> 2) + 4 * hi) >= lim ? 0.f : p.y;
          }
          const f2 ds = p * ((f2){pacc[kb2][r], pacc[kb2][r + 1]} - (f2){dl, dl});
          dsv[e] = ds.x;
          dsv[e + 1] = ds.y;
        }
        sb[kb2][s2] = pack8(dsv);
      }
#pragma unroll
    for (int kb2 = 0; kb2 < 2; ++kb2)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int d = 0; d < HD / 32; ++d)
          dqacc[d] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tr_frag(Kt2[buf] + (d >> 1) * HALF, lane, kb2, s2, d & 1),
                                                             sb[kb2][s2], dqacc[d], 0, 0, 0);
    if (t + 1 < ntiles) stage_st(buf ^ 1);
    __syncthreads();
  }

  if (qi < Lq) store_rowT<HD>(dq + b * sdq.b + h * sdq.h + qi * sdq.l, dqacc, scale, hi);
}

}  // namespace amf

// forward kernel for HD = 64 (asrx_set_attn_variant): 1 attn_fwd_sp_kernel (default), 0 attn_fwd_mf_kernel
static int g_attn_fwd_variant = 1;

template <int HD, typename TI, typename TO>
static void attn_fwd_mf_t(const void* q, AttnStridesMF Sq, const void* k, AttnStridesMF Sk, const void* v,
                          AttnStridesMF Sv, void* o, AttnStridesMF So, float* lse, int64_t B, int64_t H, int64_t Lq,
                          int64_t Lk, int causal, float scale, hipStream_t stream) {
  const TI *qq = (const TI*)q, *kk = (const TI*)k, *vv = (const TI*)v;
  TO* oo = (TO*)o;
  dim3 g((unsigned)((Lq + amf::QB - 1) / amf::QB), (unsigned)H, (unsigned)B);
  // query blocks of one (b, h) on one XCD when there are several (3.6 % at 3001 x 3001, H = 6,
  // B = 64; profiles/r02_attn_fwd_variants.txt, which also records the rejected 4-waves-per-SIMD
  // and s_setprio variants)
  if (HD == 64 && g_attn_fwd_variant == 1) {
    if (g.x > 1)
      amf::attn_fwd_sp_kernel<true, TI, TO><<<dim3((unsigned)((int64_t)g.x * g.y * g.z)), amf::NTHR, 0, stream>>>(
          qq, kk, vv, oo, lse, Sq, Sk, Sv, So, H, Lq, Lk, causal, scale);
    else
      amf::attn_fwd_sp_kernel<false, TI, TO><<<g, amf::NTHR, 0, stream>>>(qq, kk, vv, oo, lse, Sq, Sk, Sv, So, H, Lq,
                                                                          Lk, causal, scale);
  } else if (HD == 64 && g.x > 1)
    amf::attn_fwd_mf_kernel<HD, 1, true, false, TI, TO><<<dim3((unsigned)((int64_t)g.x * g.y * g.z)), amf::NTHR, 0,
                                                          stream>>>(qq, kk, vv, oo, lse, Sq, Sk, Sv, So, H, Lq, Lk,
                                                                    causal, scale);
  else
    amf::attn_fwd_mf_kernel<HD, 1, false, false, TI, TO><<<g, amf::NTHR, 0, stream>>>(qq, kk, vv, oo, lse, Sq, Sk, Sv,
                                                                                     So, H, Lq, Lk, causal, scale);
}

// bf16 flash-attention forward (see header); called by asrx_attn_fwd for prec == PREC_BF16.  io: bit 0
// q / k / v stored bf16, bit 1 o stored bf16.
int attn_fwd_mf(int io, const void* q, const int64_t* sq, const void* k, const int64_t* sk, const void* v,
                const int64_t* sv, void* o, const int64_t* so, float* lse, int64_t B, int64_t H, int64_t Lq,
                int64_t Lk, int64_t hd, int causal, float scale, hipStream_t stream) {
  AttnStridesMF Sq{sq[0], sq[1], sq[2]}, Sk{sk[0], sk[1], sk[2]}, Sv{sv[0], sv[1], sv[2]}, So{so[0], so[1], so[2]};
#define ASRX_AF(HDV, TI, TO) attn_fwd_mf_t<HDV, TI, TO>(q, Sq, k, Sk, v, Sv, o, So, lse, B, H, Lq, Lk, causal, scale, stream)
  if (hd == 64) {
    switch (io & 3) {
      case 0: ASRX_AF(64, float, float); break;
      case 1: ASRX_AF(64, amf::bf16s, float); break;
      case 2: ASRX_AF(64, float, amf::bf16s); break;
      default: ASRX_AF(64, amf::bf16s, amf::bf16s); break;
    }
  } else {
    switch (io & 3) {
      case 0: ASRX_AF(128, float, float); break;
      case 1: ASRX_AF(128, amf::bf16s, float); break;
      case 2: ASRX_AF(128, float, amf::bf16s); break;
      default: ASRX_AF(128, amf::bf16s, amf::bf16s); break;
    }
  }
#undef ASRX_AF
  return 0;
}

template <int HD, typename TI, typename TD>
static void attn_bwd_mf_t(const void* q, AttnStridesMF Sq, const void* k, AttnStridesMF Sk, const void* v,
                          AttnStridesMF Sv, const void* dO, AttnStridesMF Sd, const float* lse, const float* delta,
                          float* dq, AttnStridesMF Sdq, float* dk, AttnStridesMF Sdk, float* dv, AttnStridesMF Sdv,
                          int64_t B, int64_t H, int64_t Lq, int64_t Lk, int causal, float scale, hipStream_t stream) {
  typedef amf::BwdCfg<HD> C;
  const TI *qq = (const TI*)q, *kk = (const TI*)k, *vv = (const TI*)v;
  const TD* gg = (const TD*)dO;
  const int64_t rows_per_wg = 32 * C::NW;
  dim3 gk((unsigned)(((Lk + rows_per_wg - 1) / rows_per_wg) * H * B));
  amf::attn_bwd_dkdv_mf_kernel<HD, TI, TD><<<gk, C::NT, 0, stream>>>(qq, kk, vv, gg, lse, delta, dk, dv, Sq, Sk, Sv, Sd,
                                                                     Sdk, Sdv, H, Lq, Lk, causal, scale);
  dim3 gq((unsigned)(((Lq + rows_per_wg - 1) / rows_per_wg) * H * B));
  amf::attn_bwd_dq_mf_kernel<HD, TI, TD><<<gq, C::NT, 0, stream>>>(qq, kk, vv, gg, lse, delta, dq, Sq, Sk, Sv, Sd, Sdq,
                                                                   H, Lq, Lk, causal, scale);
}

// bf16 flash-attention backward (dkdv + dq kernels above); delta = rowsum(dO * O) already computed.
// io: bit 0 q / k / v stored bf16, bit 2 dO stored bf16.
int attn_bwd_mf(int io, const void* q, const int64_t* sq, const void* k, const int64_t* sk, const void* v,
                const int64_t* sv, const void* dO, const int64_t* sd, const float* lse, const float* delta,
                float* dq, const int64_t* sdq, float* dk, const int64_t* sdk, float* dv, const int64_t* sdv,
                int64_t B, int64_t H, int64_t Lq, int64_t Lk, int64_t hd, int causal, float scale,
                hipStream_t stream) {
  AttnStridesMF Sq{sq[0], sq[1], sq[2]}, Sk{sk[0], sk[1], sk[2]}, Sv{sv[0], sv[1], sv[2]}, Sd{sd[0], sd[1], sd[2]};
  AttnStridesMF Sdq{sdq[0], sdq[1], sdq[2]}, Sdk{sdk[0], sdk[1], sdk[2]}, Sdv{sdv[0], sdv[1], sdv[2]};
#define ASRX_AB(HDV, TI, TD)                                                                                       \
  attn_bwd_mf_t<HDV, TI, TD>(q, Sq, k, Sk, v, Sv, dO, Sd, lse, delta, dq, Sdq, dk, Sdk, dv, Sdv, B, H, Lq, Lk, causal, \
                             scale, stream)
  const int sel = (io & 1) | ((io >> 1) & 2);
  if (hd == 64) {
    switch (sel) {
      case 0: ASRX_AB(64, float, float); break;
      case 1: ASRX_AB(64, amf::bf16s, float); break;
      case 2: ASRX_AB(64, float, amf::bf16s); break;
      default: ASRX_AB(64, amf::bf16s, amf::bf16s); break;
    }
  } else {
    switch (sel) {
      case 0: ASRX_AB(128, float, float); break;
      case 1: ASRX_AB(128, amf::bf16s, float); break;
      case 2: ASRX_AB(128, float, amf::bf16s); break;
      default: ASRX_AB(128, amf::bf16s, amf::bf16s); break;
    }
  }
#undef ASRX_AB
  return 0;
}

}  // namespace asrx

// A / B switch of the HD = 64 forward kernel (host state): 1 the software-pipelined kernel (default), 0 the
// round-4 kernel.  Bit-identical outputs.  Returns the previous value.
extern "C" int asrx_set_attn_variant(int v) {
  const int old = asrx::g_attn_fwd_variant;
  asrx::g_attn_fwd_variant = v;
  return old;
}
