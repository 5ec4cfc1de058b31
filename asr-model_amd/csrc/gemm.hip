// MFMA GEMM for every projection on the hot path (nn.Linear, 1x1 and k3 Conv1d; fwd, dgrad,
// wgrad).  Replaces F.linear / conv1d as called from model.py:96-147 (ConvLite, AudioEncoder),
// 242-245 (attention q/kv/out), 341 (v_gate.mlp), 398-425 (MSheath), 529-574 (tgate, mlp) and
// essentials.py:149-153 (AbbyNormal.mode_router).
//
//   C[b] = act(alpha * A[b] @ B[b] + beta * C[b] + bias)        (fp32 in HBM, fp32 accumulate)
//
// A is MxK, B is KxN.  Each operand is either K-contiguous (A: row-major MxK, B: "NT", stored NxK)
// or MN-contiguous (A stored KxM, B stored KxN).  A K-contiguous A or an MN-contiguous B may be an
// implicit im2col of a channels-last sequence (k3 conv, padding 1): element (s, k*C + c) of the
// im2col is X[s + k - 1, c] inside a length-F segment, zero outside.
//
// PREC_BF16: operands are rounded to bf16 while staging into LDS and multiplied with
//            v_mfma_f32_16x16x32_bf16 (fp32 accumulate)          — the perf mode;
// PREC_F32:  exact fp32 v_mfma_f32_16x16x4_f32                    — the parity mode.
//
// Tiling: 128x128 block tile, 256 threads = 4 waves (2x2), 64x64 per wave = 4x4 MFMA 16x16 tiles.
// Register-staged double buffering: the next K-tile's global loads are issued before the MFMAs
// of the current one and written to the other LDS buffer after them.
#include "common.h"

namespace asrx {

struct GemmOperand {
  const float* p;
  int64_t ld;       // leading dimension (elements)
  int64_t bstride;  // batch stride (elements)
  int conv;         // implicit k3 im2col
};

struct GemmParams {
  GemmOperand a, b;
  float* c;
  int64_t ldc, sC;
  const float* bias;
  float* z;  // optional pre-activation output (same layout as C)
  int64_t M, N, K;
  int64_t convF, convC;
  float alpha, beta;
  int act;
  int splitk;
  int64_t kchunk;
};

constexpr int BM = 128, BN = 128, NTHR = 256;

template <int PREC>
struct GemmCfg;
template <>
struct GemmCfg<PREC_BF16> {
  static constexpr int BK = 64;
  static constexpr int LDS_STRIDE = BK + 8;  // bf16 elements per LDS row (144 B)
  typedef unsigned short T;
};
template <>
struct GemmCfg<PREC_F32> {
  static constexpr int BK = 32;
  static constexpr int LDS_STRIDE = BK + 2;  // floats per LDS row (conflict-free b32 reads)
  typedef float T;
};

__device__ __forceinline__ unsigned short f2bf(float f) {
  __bf16 h = (__bf16)f;
  return __builtin_bit_cast(unsigned short, h);
}

// Tile loader for one operand (ROWS x BK tile, ROWS = BM or BN).
//   KC: element (r, k) at p[r*ld + k]     (float4 along k)
//   !KC: element (r, k) at p[k*ld + r]    (float4 along r)
template <int PREC, bool KC, int ROWS>
struct TileLoader {
  static constexpr int BK = GemmCfg<PREC>::BK;
  static constexpr int NV = ROWS * BK / 4 / NTHR;  // float4 per thread
  float4 v[NV];

  __device__ __forceinline__ void load(const GemmOperand& op, int64_t r0, int64_t k0, int64_t R,
                                       int64_t K, int64_t convF, int64_t convC) {
    const int t = threadIdx.x;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int q = t + NTHR * i;
      int64_t r, k;
      if (KC) {
        r = r0 + q / (BK / 4);
        k = k0 + 4 * (q % (BK / 4));
      } else {
        k = k0 + q / (ROWS / 4);
        r = r0 + 4 * (q % (ROWS / 4));
      }
      bool ok = (r < R) && (k < K);
      int64_t off = KC ? (r * op.ld + k) : (k * op.ld + r);
      if (op.conv) {
        // spatial index s: the row for KC (A of a conv fwd), the k index for !KC (B of a wgrad);
        // channel index c: the other one.
        const int64_t s = KC ? r : k;
        const int64_t c = KC ? k : r;
        const int64_t pos = (s % convF) + c / convC - 1;
        ok = ok && pos >= 0 && pos < convF;
        off -= convC;
      }
      if (ok) {
        v[i] = *reinterpret_cast<const float4*>(op.p + off);
      } else {
        v[i] = make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
  }

  __device__ __forceinline__ void store(typename GemmCfg<PREC>::T* lds) const {
    constexpr int S = GemmCfg<PREC>::LDS_STRIDE;
    const int t = threadIdx.x;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int q = t + NTHR * i;
      if (KC) {
        const int r = q / (BK / 4), k = 4 * (q % (BK / 4));
        if constexpr (PREC == PREC_BF16) {
          ushort4 h = make_ushort4(f2bf(v[i].x), f2bf(v[i].y), f2bf(v[i].z), f2bf(v[i].w));
          *reinterpret_cast<ushort4*>(lds + r * S + k) = h;
        } else {
          float* d = lds + r * S + k;
          *reinterpret_cast<float2*>(d) = make_float2(v[i].x, v[i].y);
          *reinterpret_cast<float2*>(d + 2) = make_float2(v[i].z, v[i].w);
        }
      } else {
        const int k = q / (ROWS / 4), r = 4 * (q % (ROWS / 4));
        if constexpr (PREC == PREC_BF16) {
          lds[(r + 0) * S + k] = f2bf(v[i].x);
          lds[(r + 1) * S + k] = f2bf(v[i].y);
          lds[(r + 2) * S + k] = f2bf(v[i].z);
          lds[(r + 3) * S + k] = f2bf(v[i].w);
        } else {
          lds[(r + 0) * S + k] = v[i].x;
          lds[(r + 1) * S + k] = v[i].y;
          lds[(r + 2) * S + k] = v[i].z;
          lds[(r + 3) * S + k] = v[i].w;
        }
      }
    }
  }
};

// acc[mt][nt] += As[wave rows][BK] * Bs[wave cols][BK]^T for one K-tile.
template <int PREC>
__device__ __forceinline__ void mma_tile(f32x4 (&acc)[4][4], const typename GemmCfg<PREC>::T* As,
                                         const typename GemmCfg<PREC>::T* Bs, int wm, int wn) {
  constexpr int S = GemmCfg<PREC>::LDS_STRIDE;
  constexpr int BK = GemmCfg<PREC>::BK;
  const int lane = threadIdx.x & 63;
  const int lr = lane & 15, lk = lane >> 4;
  if constexpr (PREC == PREC_BF16) {
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) {
      bf16x8 a[4], b[4];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
        a[mt] = *reinterpret_cast<const bf16x8*>(As + (wm * 64 + mt * 16 + lr) * S + ks * 32 + 8 * lk);
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
        b[nt] = *reinterpret_cast<const bf16x8*>(Bs + (wn * 64 + nt * 16 + lr) * S + ks * 32 + 8 * lk);
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int nt = 0; nt < 4; ++nt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[mt], b[nt], acc[mt][nt], 0, 0, 0);
    }
  } else {
#pragma unroll
    for (int ks = 0; ks < BK / 4; ++ks) {
      float a[4], b[4];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) a[mt] = As[(wm * 64 + mt * 16 + lr) * S + ks * 4 + lk];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) b[nt] = Bs[(wn * 64 + nt * 16 + lr) * S + ks * 4 + lk];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int nt = 0; nt < 4; ++nt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[mt], b[nt], acc[mt][nt], 0, 0, 0);
    }
  }
}

template <int PREC, bool A_KC, bool B_KC>
__global__ __launch_bounds__(NTHR) void gemm_kernel(GemmParams p) {
  typedef typename GemmCfg<PREC>::T T;
  constexpr int BK = GemmCfg<PREC>::BK;
  constexpr int S = GemmCfg<PREC>::LDS_STRIDE;
  __shared__ __attribute__((aligned(16))) T lds[2][(BM + BN) * S];

  const int64_t n0 = (int64_t)blockIdx.x * BN;
  const int64_t m0 = (int64_t)blockIdx.y * BM;
  const int z = blockIdx.z;
  const int batch = z / p.splitk, split = z % p.splitk;
  const int64_t kbeg = (int64_t)split * p.kchunk;
  const int64_t kend = min(p.K, kbeg + p.kchunk);

  GemmOperand a = p.a, b = p.b;
  a.p += batch * a.bstride;
  b.p += batch * b.bstride;
  float* C = p.c + batch * p.sC;
  float* Z = p.z ? p.z + batch * p.sC : nullptr;

  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wm = wid >> 1, wn = wid & 1;

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  TileLoader<PREC, A_KC, BM> la;
  TileLoader<PREC, B_KC, BN> lb;
  const int64_t nk = (kend - kbeg + BK - 1) / BK;
  if (nk > 0) {
    la.load(a, m0, kbeg, p.M, kend, p.convF, p.convC);
    lb.load(b, n0, kbeg, p.N, kend, p.convF, p.convC);
    la.store(lds[0]);
    lb.store(lds[0] + BM * S);
    __syncthreads();
  }
  int cur = 0;
  for (int64_t kt = 0; kt < nk; ++kt) {
    const bool more = kt + 1 < nk;
    if (more) {
      la.load(a, m0, kbeg + (kt + 1) * BK, p.M, kend, p.convF, p.convC);
      lb.load(b, n0, kbeg + (kt + 1) * BK, p.N, kend, p.convF, p.convC);
    }
    mma_tile<PREC>(acc, lds[cur], lds[cur] + BM * S, wm, wn);
    if (more) {
      la.store(lds[cur ^ 1]);
      lb.store(lds[cur ^ 1] + BM * S);
    }
    __syncthreads();
    cur ^= 1;
  }

  // epilogue: C/D map of 16x16 MFMA: col = lane & 15, row = (lane >> 4) * 4 + r
  const int lc = lane & 15, lr4 = (lane >> 4) * 4;
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) {
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const int64_t col = n0 + wn * 64 + nt * 16 + lc;
      if (col >= p.N) continue;
      const float bv = (p.bias && split == 0) ? p.bias[col] : 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t row = m0 + wm * 64 + mt * 16 + lr4 + r;
        if (row >= p.M) continue;
        float* dst = C + row * p.ldc + col;
        float v = p.alpha * acc[mt][nt][r] + bv;
        if (p.splitk > 1) {
          atomicAdd(dst, v);
        } else {
          if (p.beta != 0.f) v += p.beta * *dst;
          if (Z) Z[row * p.ldc + col] = v;
          *dst = apply_act(p.act, v);
        }
      }
    }
  }
}

template <int PREC>
static void launch_prec(const GemmParams& p, bool akc, bool bkc, dim3 g, hipStream_t s) {
  if (akc && bkc) gemm_kernel<PREC, true, true><<<g, NTHR, 0, s>>>(p);
  else if (akc && !bkc) gemm_kernel<PREC, true, false><<<g, NTHR, 0, s>>>(p);
  else if (!akc && bkc) gemm_kernel<PREC, false, true><<<g, NTHR, 0, s>>>(p);
  else gemm_kernel<PREC, false, false><<<g, NTHR, 0, s>>>(p);
}

}  // namespace asrx

using namespace asrx;

static bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

extern "C" int asrx_gemm(int prec, const float* A, int64_t lda, int64_t sA, int a_kc, int conv_a,
                         const float* B, int64_t ldb, int64_t sB, int b_kc, int conv_b, float* C,
                         int64_t ldc, int64_t sC, const float* bias, float* Z, int64_t M, int64_t N,
                         int64_t K, int64_t batch, float alpha, float beta, int act, int64_t conv_F,
                         int64_t conv_C, int splitk, hipStream_t stream) {
  ASRX_REQUIRE(prec == PREC_F32 || prec == PREC_BF16, "asrx_gemm: bad precision %d", prec);
  ASRX_REQUIRE(M > 0 && N > 0 && K > 0 && batch > 0, "asrx_gemm: empty problem M=%ld N=%ld K=%ld",
               (long)M, (long)N, (long)K);
  ASRX_REQUIRE(aligned16(A) && aligned16(B), "asrx_gemm: A/B must be 16-byte aligned");
  ASRX_REQUIRE(lda % 4 == 0 && ldb % 4 == 0, "asrx_gemm: lda/ldb must be multiples of 4");
  ASRX_REQUIRE(a_kc ? (K % 4 == 0) : (M % 4 == 0), "asrx_gemm: A vector dim must be a multiple of 4");
  ASRX_REQUIRE(b_kc ? (K % 4 == 0) : (N % 4 == 0), "asrx_gemm: B vector dim must be a multiple of 4");
  ASRX_REQUIRE(!conv_a || a_kc, "asrx_gemm: implicit im2col on A needs K-contiguous A");
  ASRX_REQUIRE(!conv_b || !b_kc, "asrx_gemm: implicit im2col on B needs N-contiguous B");
  ASRX_REQUIRE(!(conv_a || conv_b) || (conv_F > 0 && conv_C > 0 && conv_C % 4 == 0),
               "asrx_gemm: conv needs F>0 and C%%4==0");
  ASRX_REQUIRE(sA % 4 == 0 && sB % 4 == 0, "asrx_gemm: batch strides must be multiples of 4");
  if (splitk < 1) splitk = 1;
  ASRX_REQUIRE(splitk == 1 || (beta == 1.f && act == ACT_NONE && Z == nullptr),
               "asrx_gemm: split-K accumulates into C (beta=1, no activation)");
  GemmParams p;
  p.a = GemmOperand{A, lda, sA, conv_a};
  p.b = GemmOperand{B, ldb, sB, conv_b};
  p.c = C;
  p.ldc = ldc;
  p.sC = sC;
  p.bias = bias;
  p.z = Z;
  p.M = M;
  p.N = N;
  p.K = K;
  p.convF = conv_F > 0 ? conv_F : 1;
  p.convC = conv_C > 0 ? conv_C : 1;
  p.alpha = alpha;
  p.beta = beta;
  p.act = act;
  const int BK = prec == PREC_BF16 ? GemmCfg<PREC_BF16>::BK : GemmCfg<PREC_F32>::BK;
  int64_t kchunk = (K + splitk - 1) / splitk;
  kchunk = (kchunk + BK - 1) / BK * BK;
  splitk = (int)((K + kchunk - 1) / kchunk);
  p.splitk = splitk;
  p.kchunk = kchunk;
  ASRX_REQUIRE(batch * splitk < 65536, "asrx_gemm: batch*splitk too large");
  dim3 g((unsigned)((N + BN - 1) / BN), (unsigned)((M + BM - 1) / BM), (unsigned)(batch * splitk));
  ASRX_REQUIRE(g.y < 65536u, "asrx_gemm: M too large for grid.y");
  if (prec == PREC_BF16) launch_prec<PREC_BF16>(p, a_kc, b_kc, g, stream);
  else launch_prec<PREC_F32>(p, a_kc, b_kc, g, stream);
  ASRX_LAUNCHED("asrx_gemm");
}
