// Weight-gradient GEMM, perf (bf16) mode: dW (M x N) += dY^T X summed over R rows, with dY (R x M)
// and X (R x N) the row-major fp32 activations of a Linear's backward (the feature index is the
// contiguous one on both sides).  Replaces gemm_kernel's split-K LDS-DMA path for these GEMMs
// (asrx/gemm.py linear_wgrad / wgrad_cols): 288 launches and ~27 ms of the tiny step.
//
// Design (MI355X): the row (reduction) index is the MFMA k.  Operand slabs of 32 rows x 128
// features travel global -> VGPR -> LDS as float4 loads issued two k-steps ahead (register staging,
// as gemm_wr_kernel), are rounded to bf16 on the way and stored row-major ([32 k][128 features],
// 256-B rows with an XOR chunk swizzle), and the MFMA fragments -- 8 consecutive k of one feature --
// come back through ds_read_b64_tr_b16 (the hardware transpose read), so neither operand is ever
// transposed in registers.  128 x 128 output tiles, 4 waves (2 x 2) of 64 x 64 on
// v_mfma_f32_16x16x32_bf16, LDS double-buffered with one barrier per k-step.  The rows are split
// over work items (split-K) dealt out XCD-contiguously; each item adds its partial tile into dW
// with float atomics (dW holds the gradient accumulated so far: beta = 1 by construction).
#include "common.h"

namespace asrx {
namespace wg {

constexpr int TM = 128, TN = 128, TK = 32, NT = 256;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef short v4i16 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4i16 lds_v4i16;

__device__ __attribute__((aligned(16))) float zero16[4];

struct Params {
  const float* A;  // dY  (R x M, lda)
  const float* B;  // X   (R x N, ldb)
  float* C;        // dW  (M x N, ldc), accumulated
  int64_t lda, ldb, ldc;
  int M, N;
  int64_t R, kchunk;
  int splitk;
  // optional bias gradient (asrx_wgrad_bias): db[m] += sum over rows of dY[:, m], summed from the dY
  // stages this kernel loads anyway (column tile 0 only), instead of a separate column-sum pass
  float* db;
};

// byte offset of 16-B chunk ch (8 features) of k-row `row` in a [32][128] bf16 image
__device__ __forceinline__ int off(int row, int ch) { return 256 * row + 16 * (ch ^ (((row & 3) << 2) | ((row >> 2) & 3))); }

// BBF: X stored bf16 (an activation whose only consumers are GEMM operands): 16-byte loads of 8
// features, rows (t >> 4) + 16 i, already in the image's element type.  ABF: dY stored bf16 the same
// way (the tied-logits gradient, written bf16 by the fused cross entropy).  The bf16 halves are
// native vectors (a HIP_vector_type copy can keep a stage in scratch).
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
template <bool ABF, bool BBF>
struct Stage {
  float4 a[4], b[4];  // rows (t >> 5) + 8 i, features 4 (t & 31) .. +3
};
template <>
struct Stage<false, true> {
  float4 a[4];
  u32x4 bh[2];  // rows (t >> 4) + 16 i, features 8 (t & 15) .. +7
};
template <>
struct Stage<true, true> {
  u32x4 ah[2], bh[2];
};
template <>
struct Stage<true, false> {
  u32x4 ah[2];
  float4 b[4];
};

template <bool ABF, bool BBF>
__device__ __forceinline__ void load(const Params& p, Stage<ABF, BBF>& st, int64_t r0, int64_t rend, int m0, int n0) {
  const int t = threadIdx.x;
  const int c = 4 * (t & 31);
  const int cb = 8 * (t & 15);
  if constexpr (BBF) {
    const unsigned short* Bh = reinterpret_cast<const unsigned short*>(p.B);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int64_t r = r0 + (t >> 4) + 16 * i;
      st.bh[i] = *reinterpret_cast<const u32x4*>((r < rend && n0 + cb < p.N) ? (const void*)(Bh + r * p.ldb + n0 + cb)
                                                                            : (const void*)zero16);
    }
  }
  if constexpr (ABF) {
    const unsigned short* Ah = reinterpret_cast<const unsigned short*>(p.A);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int64_t r = r0 + (t >> 4) + 16 * i;
      st.ah[i] = *reinterpret_cast<const u32x4*>((r < rend && m0 + cb < p.M) ? (const void*)(Ah + r * p.lda + m0 + cb)
                                                                            : (const void*)zero16);
    }
    if constexpr (!BBF) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int64_t r = r0 + (t >> 5) + 8 * i;
        st.b[i] = *reinterpret_cast<const float4*>((r < rend && n0 + c < p.N) ? (const void*)(p.B + r * p.ldb + n0 + c)
                                                                              : (const void*)zero16);
      }
    }
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t r = r0 + (t >> 5) + 8 * i;
      const bool okr = r < rend;
      // unconditional loads from clamped addresses (a branch would make the compiler drain vmcnt)
      st.a[i] = *reinterpret_cast<const float4*>((okr && m0 + c < p.M) ? (const void*)(p.A + r * p.lda + m0 + c)
                                                                       : (const void*)zero16);
      if constexpr (!BBF)
        st.b[i] = *reinterpret_cast<const float4*>((okr && n0 + c < p.N) ? (const void*)(p.B + r * p.ldb + n0 + c)
                                                                         : (const void*)zero16);
    }
  }
}

template <bool ABF, bool BBF>
__device__ __forceinline__ void store(const Stage<ABF, BBF>& st, char* Ai, char* Bi) {
  const int t = threadIdx.x;
  const int c = 4 * (t & 31);
  const int ch = c >> 3, hb = (c >> 2) & 1;
  typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
  if constexpr (ABF) {
#pragma unroll
    for (int i = 0; i < 2; ++i) *reinterpret_cast<u32x4*>(Ai + off((t >> 4) + 16 * i, t & 15)) = st.ah[i];
    if constexpr (!BBF) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = (t >> 5) + 8 * i;
        bf16x4 hb4;
        hb4[0] = (__bf16)st.b[i].x; hb4[1] = (__bf16)st.b[i].y; hb4[2] = (__bf16)st.b[i].z; hb4[3] = (__bf16)st.b[i].w;
        *reinterpret_cast<bf16x4*>(Bi + off(row, ch) + 8 * hb) = hb4;
      }
    }
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = (t >> 5) + 8 * i;
      bf16x4 ha;
      ha[0] = (__bf16)st.a[i].x; ha[1] = (__bf16)st.a[i].y; ha[2] = (__bf16)st.a[i].z; ha[3] = (__bf16)st.a[i].w;
      *reinterpret_cast<bf16x4*>(Ai + off(row, ch) + 8 * hb) = ha;
      if constexpr (!BBF) {
        bf16x4 hb4;
        hb4[0] = (__bf16)st.b[i].x; hb4[1] = (__bf16)st.b[i].y; hb4[2] = (__bf16)st.b[i].z; hb4[3] = (__bf16)st.b[i].w;
        *reinterpret_cast<bf16x4*>(Bi + off(row, ch) + 8 * hb) = hb4;
      }
    }
  }
  if constexpr (BBF) {
#pragma unroll
    for (int i = 0; i < 2; ++i) *reinterpret_cast<u32x4*>(Bi + off((t >> 4) + 16 * i, t & 15)) = st.bh[i];
  }
}

// MFMA 16x16x32 operand of features c0 .. c0+15: lane l gets feature c0 + (l & 15), k = 8 (l >> 4) .. +7
__device__ __forceinline__ bf16x8 frag(const char* img, int c0, int lane) {
  const int g = lane >> 4, gi = lane & 15, q = gi >> 2, p = gi & 3;
  const int col = c0 + 4 * p;
  const int ch = col >> 3, hb = (col >> 2) & 1;
  const v4i16 t1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(img + off(8 * g + q, ch) + 8 * hb));
  const v4i16 t2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(img + off(8 * g + 4 + q, ch) + 8 * hb));
  typedef short v8i16 __attribute__((ext_vector_type(8)));
  const v8i16 a8 = {t1[0], t1[1], t1[2], t1[3], t2[0], t2[1], t2[2], t2[3]};
  return __builtin_bit_cast(bf16x8, a8);
}

// work item -> XCD-contiguous runs (blocks b and b+8 share an XCD): the output tiles of one row
// slice run on one XCD together and share its L2
__device__ __forceinline__ int xcd_item(int bid, int nblk) {
  const int xcd = bid & 7, q = nblk >> 3, r = nblk & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

// per-thread column partials of a dY stage: fp32 dY -- features 4 (t & 31) .. +3 of rows (t >> 5) + 8 i;
// bf16 dY -- features 8 (t & 15) .. +7 of rows (t >> 4) + 16 i (zero-page rows past the end add 0)
template <bool ABF, bool BBF>
__device__ __forceinline__ void colacc(const Stage<ABF, BBF>& st, float (&cs)[8]) {
  if constexpr (ABF) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        const unsigned u = st.ah[i][w];
        cs[2 * w] += __builtin_bit_cast(float, u << 16);
        cs[2 * w + 1] += __builtin_bit_cast(float, u & 0xffff0000u);
      }
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      cs[0] += st.a[i].x;
      cs[1] += st.a[i].y;
      cs[2] += st.a[i].z;
      cs[3] += st.a[i].w;
    }
  }
}

template <bool ABF, bool BBF>
__global__ __launch_bounds__(NT, 2) void wgrad_wr_kernel(Params p) {
  __shared__ __attribute__((aligned(16))) char Ai[2][TK * TM * 2];
  __shared__ __attribute__((aligned(16))) char Bi[2][TK * TN * 2];
  const int nN = (p.N + TN - 1) / TN, nM = (p.M + TM - 1) / TM;
  const int ntile = nM * nN;
  const int item = xcd_item(blockIdx.x, gridDim.x);
  const int split = item / ntile, tile = item % ntile;
  const int m0 = (tile / nN) * TM, n0 = (tile % nN) * TN;
  const int64_t rb = (int64_t)split * p.kchunk, re = min<int64_t>(p.R, rb + p.kchunk);
  const int nk = rb < re ? (int)((re - rb + TK - 1) / TK) : 0;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm = wid >> 1, wn = wid & 1;

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  Stage<ABF, BBF> s0, s1;
  const bool dbon = p.db && n0 == 0;  // uniform
  float cs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  load(p, s0, rb, re, m0, n0);
  load(p, s1, rb + TK, re, m0, n0);
  if (dbon && nk > 0) colacc(s0, cs);
  store(s0, Ai[0], Bi[0]);
  __syncthreads();

  auto kstep = [&](int s, Stage<ABF, BBF>& cur, const Stage<ABF, BBF>& nxt) __attribute__((always_inline)) {
    load(p, cur, rb + (int64_t)(s + 2) * TK, re, m0, n0);  // past the end: zero page, counts stay uniform
    const char* At = Ai[s & 1];
    const char* Bt = Bi[s & 1];
    bf16x8 a[4], b[4];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) a[mt] = frag(At, wm * 64 + mt * 16, lane);
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) b[nt] = frag(Bt, wn * 64 + nt * 16, lane);
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
        acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[mt], b[nt], acc[mt][nt], 0, 0, 0);
    if (s + 1 < nk) {
      if (dbon) colacc(nxt, cs);
      store(nxt, Ai[(s + 1) & 1], Bi[(s + 1) & 1]);
    }
    __syncthreads();
  };
  for (int s = 0; s < nk; s += 2) {
    kstep(s, s0, s1);
    if (s + 1 < nk) kstep(s + 1, s1, s0);
  }

  // D map of the 16x16 MFMA: n = lane & 15, m = 4 (lane >> 4) + r
  const int ln = lane & 15, lm = 4 * (lane >> 4);
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const int n = n0 + wn * 64 + nt * 16 + ln;
      if (n >= p.N) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * 64 + mt * 16 + lm + r;
        if (m < p.M && nk > 0) atomicAdd(p.C + (int64_t)m * p.ldc + n, acc[mt][nt][r]);
      }
    }
  if (dbon && nk > 0) {
    // lanes sharing a feature group: fp32 dY -- t and t ^ 32 within a wave, then the 4 waves;
    // bf16 dY -- t, t ^ 16, t ^ 32, t ^ 48, then the 4 waves (through the retired A images)
    constexpr int F = ABF ? 8 : 4;
#pragma unroll
    for (int f = 0; f < F; ++f) {
      cs[f] += __shfl_xor(cs[f], 32);
      if (ABF) cs[f] += __shfl_xor(cs[f], 16);
    }
    __syncthreads();  // every wave is past its last LDS read of the images
    float* red = reinterpret_cast<float*>(Ai[0]);  // [4 waves][128 features]
    const int t = threadIdx.x, lane = t & 63;
    const bool wr = ABF ? lane < 16 : lane < 32;
    if (wr) {
      const int f0 = ABF ? 8 * (lane & 15) : 4 * (lane & 31);
#pragma unroll
      for (int f = 0; f < F; ++f) red[(t >> 6) * TM + f0 + f] = cs[f];
    }
    __syncthreads();
    if (t < TM && m0 + t < p.M)
      atomicAdd(p.db + m0 + t, red[t] + red[TM + t] + red[2 * TM + t] + red[3 * TM + t]);
  }
}

// ---------------------------------------------------------------------------------------------
// Wide form (wgrad_w3_kernel): 128 dY features x 384 X features per work item, 8 waves (2 x 4) of 64 x 96.
// A k-step stages 32 rows of dY (128 features) and of X (384 features): per output element 1.3 B of operand
// reads per k-step instead of the 128 x 128 tile's 2.0 (each dY slab is read by N / 384 items instead of
// N / 128), which is what bounds the D x D weight gradients at 192k rows (the slabs come from L2, not
// HBM).  Same MFMA, fragment reads and k order as wgrad_wr_kernel; the X image rows are 768 B (48 chunks,
// the low four chunk bits XOR-swizzled as off()).  fp32 dY only; launched for bf16 X (the fp32-X form needs
// 24 more stage registers per set than the 256 two waves per SIMD leave and spilled).
constexpr int TN3 = 384, NT3 = 512;
__device__ __forceinline__ int off3(int row, int ch) {
  return 768 * row + 16 * ((ch & ~15) | ((ch ^ (((row & 3) << 2) | ((row >> 2) & 3))) & 15));
}
__device__ __forceinline__ bf16x8 frag3(const char* img, int c0, int lane) {
  const int g = lane >> 4, gi = lane & 15, q = gi >> 2, p = gi & 3;
  const int col = c0 + 4 * p;
  const int ch = col >> 3, hb = (col >> 2) & 1;
  const v4i16 t1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(img + off3(8 * g + q, ch) + 8 * hb));
  const v4i16 t2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(img + off3(8 * g + 4 + q, ch) + 8 * hb));
  typedef short v8i16 __attribute__((ext_vector_type(8)));
  const v8i16 a8 = {t1[0], t1[1], t1[2], t1[3], t2[0], t2[1], t2[2], t2[3]};
  return __builtin_bit_cast(bf16x8, a8);
}
// stage registers: dY fp32 32 x 128 (2 float4 per thread: rows (t >> 5) + 16 i, features 4 (t & 31));
// X fp32 32 x 384 (6 float4: item q = t + 512 i -> row q / 96, features 4 (q % 96)) or bf16 (3 x 8 features:
// item q = t + 512 i -> row q / 48, features 8 (q % 48))
template <bool BBF>
struct Stage3 {
  float4 a[2];
  float4 b[6];
};
template <>
struct Stage3<true> {
  float4 a[2];
  u32x4 bh[3];
};
template <bool BBF>
__device__ __forceinline__ void load3(const Params& p, Stage3<BBF>& st, int64_t r0, int64_t rend, int m0, int n0) {
  const int t = threadIdx.x;
  const int c = 4 * (t & 31);
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int64_t r = r0 + (t >> 5) + 16 * i;
    st.a[i] = *reinterpret_cast<const float4*>((r < rend && m0 + c < p.M) ? (const void*)(p.A + r * p.lda + m0 + c)
                                                                          : (const void*)zero16);
  }
  if constexpr (BBF) {
    const unsigned short* Bh = reinterpret_cast<const unsigned short*>(p.B);
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int q = t + NT3 * i;
      const int64_t r = r0 + q / 48;
      const int f = 8 * (q % 48);
      st.bh[i] = *reinterpret_cast<const u32x4*>((r < rend && n0 + f < p.N) ? (const void*)(Bh + r * p.ldb + n0 + f)
                                                                            : (const void*)zero16);
    }
  } else {
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      const int q = t + NT3 * i;
      const int64_t r = r0 + q / 96;
      const int f = 4 * (q % 96);
      st.b[i] = *reinterpret_cast<const float4*>((r < rend && n0 + f < p.N) ? (const void*)(p.B + r * p.ldb + n0 + f)
                                                                            : (const void*)zero16);
    }
  }
}
template <bool BBF>
__device__ __forceinline__ void store3(const Stage3<BBF>& st, char* Ai, char* Bi) {
  const int t = threadIdx.x;
  typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
  {
    const int c = 4 * (t & 31), ch = c >> 3, hb = (c >> 2) & 1;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int row = (t >> 5) + 16 * i;
      bf16x4 ha;
      ha[0] = (__bf16)st.a[i].x; ha[1] = (__bf16)st.a[i].y; ha[2] = (__bf16)st.a[i].z; ha[3] = (__bf16)st.a[i].w;
      *reinterpret_cast<bf16x4*>(Ai + off(row, ch) + 8 * hb) = ha;
    }
  }
  if constexpr (BBF) {
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int q = t + NT3 * i;
      *reinterpret_cast<u32x4*>(Bi + off3(q / 48, q % 48)) = st.bh[i];
    }
  } else {
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      const int q = t + NT3 * i;
      const int row = q / 96, c = 4 * (q % 96), ch = c >> 3, hb = (c >> 2) & 1;
      bf16x4 hb4;
      hb4[0] = (__bf16)st.b[i].x; hb4[1] = (__bf16)st.b[i].y; hb4[2] = (__bf16)st.b[i].z; hb4[3] = (__bf16)st.b[i].w;
      *reinterpret_cast<bf16x4*>(Bi + off3(row, ch) + 8 * hb) = hb4;
    }
  }
}

template <bool BBF>
__global__ __launch_bounds__(NT3, 1) void wgrad_w3_kernel(Params p) {
  __shared__ __attribute__((aligned(16))) char Ai[2][TK * TM * 2];
  __shared__ __attribute__((aligned(16))) char Bi[2][TK * TN3 * 2];
  const int nN = (p.N + TN3 - 1) / TN3, nM = (p.M + TM - 1) / TM;
  const int ntile = nM * nN;
  const int item = xcd_item(blockIdx.x, gridDim.x);
  const int split = item / ntile, tile = item % ntile;
  const int m0 = (tile / nN) * TM, n0 = (tile % nN) * TN3;
  const int64_t rb = (int64_t)split * p.kchunk, re = min<int64_t>(p.R, rb + p.kchunk);
  const int nk = rb < re ? (int)((re - rb + TK - 1) / TK) : 0;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm = wid >> 2, wn = wid & 3;

  f32x4 acc[4][6];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 6; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  Stage3<BBF> s0, s1;
  const bool dbon = p.db && n0 == 0;  // uniform
  float cs[4] = {0.f, 0.f, 0.f, 0.f};
  auto colacc3 = [&](const Stage3<BBF>& st) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      cs[0] += st.a[i].x;
      cs[1] += st.a[i].y;
      cs[2] += st.a[i].z;
      cs[3] += st.a[i].w;
    }
  };
  load3(p, s0, rb, re, m0, n0);
  load3(p, s1, rb + TK, re, m0, n0);
  if (dbon && nk > 0) colacc3(s0);
  store3(s0, Ai[0], Bi[0]);
  __syncthreads();

  auto kstep = [&](int s, Stage3<BBF>& cur, const Stage3<BBF>& nxt) __attribute__((always_inline)) {
    load3(p, cur, rb + (int64_t)(s + 2) * TK, re, m0, n0);  // past the end: zero page, counts stay uniform
    const char* At = Ai[s & 1];
    const char* Bt = Bi[s & 1];
    bf16x8 b[6];  // the dY fragment is read per 16-feature block (fewer live registers)
#pragma unroll
    for (int nt = 0; nt < 6; ++nt) b[nt] = frag3(Bt, wn * 96 + nt * 16, lane);
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      const bf16x8 a = frag(At, wm * 64 + mt * 16, lane);
#pragma unroll
      for (int nt = 0; nt < 6; ++nt)
        acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b[nt], acc[mt][nt], 0, 0, 0);
    }
    if (s + 1 < nk) {
      if (dbon) colacc3(nxt);
      store3(nxt, Ai[(s + 1) & 1], Bi[(s + 1) & 1]);
    }
    __syncthreads();
  };
  for (int s = 0; s < nk; s += 2) {
    kstep(s, s0, s1);
    if (s + 1 < nk) kstep(s + 1, s1, s0);
  }

  const int ln = lane & 15, lm = 4 * (lane >> 4);
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int nt = 0; nt < 6; ++nt) {
      const int n = n0 + wn * 96 + nt * 16 + ln;
      if (n >= p.N) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * 64 + mt * 16 + lm + r;
        if (m < p.M && nk > 0) atomicAdd(p.C + (int64_t)m * p.ldc + n, acc[mt][nt][r]);
      }
    }
  if (dbon && nk > 0) {
    // lanes t and t ^ 32 hold the same features (rows (t >> 5) + 16 i), then the 8 waves through the A images
#pragma unroll
    for (int f = 0; f < 4; ++f) cs[f] += __shfl_xor(cs[f], 32);
    __syncthreads();  // every wave is past its last LDS read of the images
    float* red = reinterpret_cast<float*>(Ai[0]);  // [8 waves][128 features] = 4 KB of the 8 KB image
    const int t = threadIdx.x;
    if (lane < 32) {
#pragma unroll
      for (int f = 0; f < 4; ++f) red[(t >> 6) * TM + 4 * lane + f] = cs[f];
    }
    __syncthreads();
    if (t < TM && m0 + t < p.M) {
      float v = red[t];
#pragma unroll
      for (int w = 1; w < NT3 / 64; ++w) v += red[w * TM + t];
      atomicAdd(p.db + m0 + t, v);
    }
  }
}

}  // namespace wg
}  // namespace asrx

using namespace asrx;

// dW (M x N, ldc) += dY^T X over R rows; dY (R x M, lda), X (R x N, ldb) fp32 row-major; the rows
// split over `splitk` work items (bf16 operands, fp32 accumulate).  M, N, lda, ldb multiples of 4,
// 16-byte aligned operands.
// weight-gradient kernel for fp32 dY, bf16 X, N % 384 == 0 (asrx_set_wgrad_variant): 1 wgrad_w3_kernel
// (default), 0 wgrad_wr_kernel
static int g_wgrad_variant = 1;
extern "C" int asrx_set_wgrad_variant(int v) {
  const int old = g_wgrad_variant;
  g_wgrad_variant = v;
  return old;
}

static int wgrad_launch(const void* A, int a_bf16, int64_t lda, const void* B, int b_bf16, int64_t ldb, float* C,
                        int64_t ldc, int64_t M, int64_t N, int64_t R, int64_t splitk, hipStream_t stream,
                        float* db = nullptr) {
  ASRX_REQUIRE(M > 0 && N > 0 && R >= 0, "asrx_wgrad_bf16: empty problem");
  ASRX_REQUIRE(M % 4 == 0 && N % 4 == 0 && lda % 4 == 0 && ldb % 4 == 0, "asrx_wgrad_bf16: M, N, lda, ldb %% 4 required");
  ASRX_REQUIRE(!b_bf16 || (N % 8 == 0 && ldb % 8 == 0), "asrx_wgrad_bf16: a bf16 X needs N, ldb %% 8");
  ASRX_REQUIRE(!a_bf16 || (M % 8 == 0 && lda % 8 == 0), "asrx_wgrad_bf16: a bf16 dY needs M, lda %% 8");
  ASRX_REQUIRE((((uintptr_t)A | (uintptr_t)B) & 15) == 0, "asrx_wgrad_bf16: operands must be 16-byte aligned");
  if (R == 0) return 0;
  if (splitk < 1) splitk = 1;
  int64_t kchunk = (R + splitk - 1) / splitk;
  kchunk = (kchunk + wg::TK - 1) / wg::TK * wg::TK;
  splitk = (R + kchunk - 1) / kchunk;
  // wide items where they measured faster (profiles/r05_wgrad_w3_ab.txt: 384 x 1536 and 1536 x 384 outputs 10-17 %;
  // the 3-item 384 x 384 outputs equal at 192k rows and slower at 96k, so they keep the 128 x 128 items)
  if (!a_bf16 && b_bf16 && g_wgrad_variant == 1 && N % wg::TN3 == 0 && R >= 4096 &&
      ((M + wg::TM - 1) / wg::TM) * (N / wg::TN3) >= 8) {
    // wide items: one resident 8-wave workgroup per CU, each K slice >= 512 rows
    static int cus = 0;
    if (!cus) {
      int dev = 0;
      (void)hipGetDevice(&dev);
      (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
      cus = cus > 0 ? cus : 1;
    }
    const int64_t tiles = ((M + wg::TM - 1) / wg::TM) * (N / wg::TN3);
    int64_t sk = cus / tiles;
    if (sk > R / 512) sk = R / 512;
    if (sk < 1) sk = 1;
    int64_t kc = (R + sk - 1) / sk;
    kc = (kc + wg::TK - 1) / wg::TK * wg::TK;
    sk = (R + kc - 1) / kc;
    wg::Params p3{(const float*)A, (const float*)B, C, lda, ldb, ldc, (int)M, (int)N, R, kc, (int)sk, db};
    wg::wgrad_w3_kernel<true><<<(unsigned)(tiles * sk), wg::NT3, 0, stream>>>(p3);
    ASRX_LAUNCHED("asrx_wgrad_bf16");
  }
  wg::Params p{(const float*)A, (const float*)B, C, lda, ldb, ldc, (int)M, (int)N, R, kchunk, (int)splitk, db};
  const int64_t items = ((M + wg::TM - 1) / wg::TM) * ((N + wg::TN - 1) / wg::TN) * splitk;
  ASRX_REQUIRE(items < (1LL << 31), "asrx_wgrad_bf16: too many work items");
  if (a_bf16 && b_bf16)
    wg::wgrad_wr_kernel<true, true><<<(unsigned)items, wg::NT, 0, stream>>>(p);
  else if (a_bf16)
    wg::wgrad_wr_kernel<true, false><<<(unsigned)items, wg::NT, 0, stream>>>(p);
  else if (b_bf16)
    wg::wgrad_wr_kernel<false, true><<<(unsigned)items, wg::NT, 0, stream>>>(p);
  else
    wg::wgrad_wr_kernel<false, false><<<(unsigned)items, wg::NT, 0, stream>>>(p);
  ASRX_LAUNCHED("asrx_wgrad_bf16");
}

extern "C" int asrx_wgrad_bf16(const float* A, int64_t lda, const float* B, int64_t ldb, float* C, int64_t ldc,
                               int64_t M, int64_t N, int64_t R, int64_t splitk, hipStream_t stream) {
  return wgrad_launch(A, 0, lda, B, 0, ldb, C, ldc, M, N, R, splitk, stream);
}

// asrx_wgrad_bf16 with X (B) stored fp32 (b_bf16 = 0) or bf16 (1; N, ldb multiples of 8).
extern "C" int asrx_wgrad_bf16_ex(const float* A, int64_t lda, const void* B, int b_bf16, int64_t ldb, float* C,
                                  int64_t ldc, int64_t M, int64_t N, int64_t R, int64_t splitk, hipStream_t stream) {
  return wgrad_launch(A, 0, lda, B, b_bf16, ldb, C, ldc, M, N, R, splitk, stream);
}

// asrx_wgrad_bf16 with dY (A) stored bf16 (M, lda multiples of 8) and X (B) stored fp32 (b_bf16 = 0) or
// bf16 (1; N, ldb multiples of 8): the tied token embedding's gradient from the bf16 logits gradient
// (model.py:629) and the weight gradients under an activation (asrx_act_bwd_bias's bf16 gz).
extern "C" int asrx_wgrad_bf16_ab(const void* A, int64_t lda, const void* B, int b_bf16, int64_t ldb, float* C,
                                  int64_t ldc, int64_t M, int64_t N, int64_t R, int64_t splitk, hipStream_t stream) {
  return wgrad_launch(A, 1, lda, B, b_bf16, ldb, C, ldc, M, N, R, splitk, stream);
}

// dW += dY^T X and db += column sums of dY in one pass (the bias gradient of y = x W^T + b summed from
// the dY stages the weight-gradient kernel loads anyway; replaces a separate asrx_colsum over dY):
// dY fp32 (a_bf16 = 0) or bf16 (1), X fp32 or bf16, as asrx_wgrad_bf16_ex / _ab.
extern "C" int asrx_wgrad_bias(const void* A, int a_bf16, int64_t lda, const void* B, int b_bf16, int64_t ldb,
                               float* C, int64_t ldc, float* db, int64_t M, int64_t N, int64_t R, int64_t splitk,
                               hipStream_t stream) {
  ASRX_REQUIRE(db, "asrx_wgrad_bias: db required");
  return wgrad_launch(A, a_bf16, lda, B, b_bf16, ldb, C, ldc, M, N, R, splitk, stream, db);
}
