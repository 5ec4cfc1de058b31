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
// PREC_F32:  exact fp32 v_mfma_f32_16x16x4_f32                    — the parity mode;
// PREC_X3:   split bf16 ("bf16x3"): each fp32 fragment value x is split into hi = bf16(x) and
//            lo = bf16(x - hi) when it is read from LDS, and the product is lo*hi + hi*lo + hi*hi on
//            v_mfma_f32_16x16x32_bf16 (the lo*lo term, ~2^-16 of an operand's ulp, is dropped): ~16-bit
//            operand precision at 3/16 of the fp32 MFMA's cycles -- the reference-faithful training mode
//            (tools/bf16_sensitivity.py x3: whole-gradient cosine 0.993 with float64 where one bf16
//            rounding gives 0.35, profiles/r05_split_bf16_sensitivity.txt).
//
// Tiling: 128x128 block tile, 256 threads = 4 waves (2x2), 64x64 per wave = 4x4 MFMA 16x16 tiles,
// BK = 32.  fp32 tiles stream HBM -> LDS by LDS-DMA (global_load_lds_dwordx4, 8 x 1 KB per wave per
// stage) into a 3-stage ring; a counted s_waitcnt vmcnt + raw s_barrier per K-step keeps the next
// stage's DMA in flight under the current stage's MFMAs.  Fragments are read from the swizzled fp32
// images and rounded to bf16 in registers.  Tail / conv-padding lanes read a zero page.
#include "common.h"
#include <cstdlib>

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

constexpr int BM = 128, BN = 128, NTHR = 256, BK = 32;
constexpr int TILE_BYTES = 128 * BK * 4;                 // one fp32 operand tile per stage (16 KB)
constexpr int STAGE_BYTES = 2 * TILE_BYTES;              // A + B
constexpr int GLDS_PER_WAVE = 2 * TILE_BYTES / 1024 / 4; // 1-KB LDS-DMA pieces per wave per stage (8)

__device__ __attribute__((aligned(16))) float g_zero_page[4];  // source of zero-filled tile lanes

typedef __attribute__((address_space(3))) void lds_void;
typedef const __attribute__((address_space(1))) void gbl_void;

// ---------------------------------------------------------------------------------------------
// LDS images (fp32, unpadded, written lane-linearly by global_load_lds_dwordx4; the swizzles are
// applied to the per-lane SOURCE address and undone on the read, see cdna_hip_programming.md
// rule 21):
//   K-contiguous operand: [128 rows][32 k]   row = 128 B = 8 chunks of 16 B; chunk c of row r is
//     stored at position c ^ ((r >> 1) & 7)  -> the 16 lanes of a fragment read hit 16 slots.
//   MN-contiguous operand: [32 k][128 rows]  k-row = 512 B = 32 chunks; chunk c of k-row kr is
//     stored at c ^ (((kr >> 3) & 1) << 2)   -> the two 16-lane halves of a b32 read differ.
// ---------------------------------------------------------------------------------------------
// Per-lane LDS-DMA issue state for one operand: everything that does not change along K is
// computed once.  Element offsets are 32-bit (the host checks every operand spans < 2^31 elements).
template <bool KC, bool CONV>
struct Stager {
  const float* base;
  int ld;
  uint32_t off[4];  // KC: row * ld + 4c ; !KC: row0 + 4c   (k contribution added per stage)
  int kk[4];        // KC: 4c (k within the tile) ; !KC: k-row within the tile
  int cpos[4];      // CONV: KC: row % F ; !KC: column / C (tap)
  bool rok[4];

  __device__ __forceinline__ void init(const GemmOperand& op, int r0, int R, int convF, int convC) {
    base = op.p;
    ld = (int)op.ld;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int q = wid * 4 + i;  // 1-KB piece index within the 16-KB tile
      if (KC) {
        const int row = 8 * q + (lane >> 3);
        const int c = (lane & 7) ^ ((row >> 1) & 7);
        const int r = r0 + row;
        rok[i] = r < R;
        off[i] = (uint32_t)r * (uint32_t)ld + 4 * c;
        kk[i] = 4 * c;
        cpos[i] = CONV ? r % convF : 0;
      } else {
        const int kr = 2 * q + (lane >> 5);
        const int c = (lane & 31) ^ (((kr >> 3) & 1) << 2);
        const int r = r0 + 4 * c;
        rok[i] = r < R;
        off[i] = (uint32_t)r;
        kk[i] = kr;
        cpos[i] = CONV ? r / convC : 0;
      }
    }
  }

  __device__ __forceinline__ void issue(char* lds_tile, int k0, int K, int convF, int convC) const {
    const int wid = threadIdx.x >> 6;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int k = k0 + kk[i];
      bool ok = rok[i] && k < K;
      uint32_t o = KC ? off[i] + (uint32_t)k0 : off[i] + (uint32_t)k * (uint32_t)ld;
      if (CONV) {
        const int pos = KC ? cpos[i] + (k0 + kk[i]) / convC - 1 : (k % convF) + cpos[i] - 1;
        ok = ok && pos >= 0 && pos < convF;
        o -= (uint32_t)convC;
      }
      const float* src = ok ? base + o : g_zero_page;
      glds16(src, lds_addr(lds_tile + (wid * 4 + i) * 1024));
    }
  }
};

// 8 consecutive k (k = kb .. kb+7) of tile row r, as fp32.
template <bool KC>
__device__ __forceinline__ void read8(const char* tile, int r, int kb, float (&o)[8]) {
  if (KC) {
    const int sw = (r >> 1) & 7;
    const char* row = tile + r * 128;
    const float4 x = *reinterpret_cast<const float4*>(row + 16 * ((kb >> 2) ^ sw));
    const float4 y = *reinterpret_cast<const float4*>(row + 16 * (((kb >> 2) + 1) ^ sw));
    o[0] = x.x; o[1] = x.y; o[2] = x.z; o[3] = x.w;
    o[4] = y.x; o[5] = y.y; o[6] = y.z; o[7] = y.w;
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = kb + j;
      const int c = (r >> 2) ^ (((k >> 3) & 1) << 2);
      o[j] = *reinterpret_cast<const float*>(tile + k * 512 + 16 * c + 4 * (r & 3));
    }
  }
}

template <bool KC>
__device__ __forceinline__ float read1(const char* tile, int r, int k) {
  if (KC) {
    return *reinterpret_cast<const float*>(tile + r * 128 + 16 * ((k >> 2) ^ ((r >> 1) & 7)) + 4 * (k & 3));
  } else {
    const int c = (r >> 2) ^ (((k >> 3) & 1) << 2);
    return *reinterpret_cast<const float*>(tile + k * 512 + 16 * c + 4 * (r & 3));
  }
}

__device__ __forceinline__ bf16x8 to_bf16x8(const float (&f)[8]) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (__bf16)f[j];
  return r;
}

// x = hi + lo to ~16 bits: hi = bf16(x) (RNE), lo = bf16(x - hi) (x - hi is exact in fp32)
__device__ __forceinline__ void split_bf16x8(const float (&f)[8], bf16x8& hi, bf16x8& lo) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const __bf16 h = (__bf16)f[j];
    hi[j] = h;
    lo[j] = (__bf16)(f[j] - (float)h);
  }
}

// acc[mt][nt] += A(wave rows, 32 k) * B(wave cols, 32 k)^T from one stage.
template <int PREC, bool A_KC, bool B_KC>
__device__ __forceinline__ void mma_stage(f32x4 (&acc)[4][4], const char* At, const char* Bt, int wm, int wn) {
  const int lane = threadIdx.x & 63;
  const int lr = lane & 15, lk = lane >> 4;
  if constexpr (PREC == PREC_BF16) {
    bf16x8 a[4], b[4];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      float f[8];
      read8<A_KC>(At, wm * 64 + mt * 16 + lr, 8 * lk, f);
      a[mt] = to_bf16x8(f);
    }
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      float f[8];
      read8<B_KC>(Bt, wn * 64 + nt * 16 + lr, 8 * lk, f);
      b[nt] = to_bf16x8(f);
    }
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
        acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[mt], b[nt], acc[mt][nt], 0, 0, 0);
  } else if constexpr (PREC == PREC_X3) {
    bf16x8 ah[4], al[4], bh[4], bl[4];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      float f[8];
      read8<A_KC>(At, wm * 64 + mt * 16 + lr, 8 * lk, f);
      split_bf16x8(f, ah[mt], al[mt]);
    }
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      float f[8];
      read8<B_KC>(Bt, wn * 64 + nt * 16 + lr, 8 * lk, f);
      split_bf16x8(f, bh[nt], bl[nt]);
    }
    // small terms first: they are added to the accumulator before the leading product
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[mt], bh[nt], acc[mt][nt], 0, 0, 0);
        acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[mt], bl[nt], acc[mt][nt], 0, 0, 0);
        acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[mt], bh[nt], acc[mt][nt], 0, 0, 0);
      }
  } else {
#pragma unroll
    for (int ks = 0; ks < BK / 4; ++ks) {
      float a[4], b[4];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) a[mt] = read1<A_KC>(At, wm * 64 + mt * 16 + lr, ks * 4 + lk);
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) b[nt] = read1<B_KC>(Bt, wn * 64 + nt * 16 + lr, ks * 4 + lk);
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int nt = 0; nt < 4; ++nt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[mt], b[nt], acc[mt][nt], 0, 0, 0);
    }
  }
}

// Workgroup -> work item (batch/split z, output tile).  Blocks b and b+8 share an XCD (round-robin
// dispatch), so the remap hands each XCD a contiguous run of work items; items are ordered
// z-major, tiles N-fastest, so the tiles that re-read one A row panel -- and, for a split-K weight
// gradient with only a few output tiles, every tile of one K slice -- run on the same XCD at about
// the same time and hit its L2.  (Speed only: with the slices spread over XCDs the 3x3-tile
// weight gradients fetched 2.8x their algorithmic bytes from HBM.)
__device__ __forceinline__ int xcd_item(int bid, int nblk) {
  const int xcd = bid & 7, q = nblk >> 3, r = nblk & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if constexpr (N == 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
}

template <int PREC, bool A_KC, bool B_KC, bool CA, bool CB, int NSTAGE>
__global__ __launch_bounds__(NTHR, 1) void gemm_kernel(GemmParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];  // NSTAGE x [A tile | B tile]

  const int nN = (int)((p.N + BN - 1) / BN);
  const int ntile = nN * (int)((p.M + BM - 1) / BM);
  const int item = xcd_item(blockIdx.x, gridDim.x);
  const int z = item / ntile, tile = item % ntile;
  const int tn = tile % nN, tm = tile / nN;
  const int n0 = tn * BN;
  const int m0 = tm * BM;
  const int batch = z / p.splitk, split = z % p.splitk;
  const int64_t kbeg = (int64_t)split * p.kchunk;
  const int64_t kend = min(p.K, kbeg + p.kchunk);

  GemmOperand a = p.a, b = p.b;
  a.p += batch * a.bstride;
  b.p += batch * b.bstride;
  float* C = p.c + batch * p.sC;
  float* Z = p.z ? p.z + batch * p.sC : nullptr;
  const int M = (int)p.M, N = (int)p.N;
  const int convF = (int)p.convF, convC = (int)p.convC;

  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wm = wid >> 1, wn = wid & 1;

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = (int)((kend - kbeg + BK - 1) / BK);
  const int kb0 = (int)kbeg, kE = (int)kend;
  Stager<A_KC, CA> sa;
  Stager<B_KC, CB> sb;
  sa.init(a, m0, M, convF, convC);
  sb.init(b, n0, N, convF, convC);
  // prologue: stages 0 .. NSTAGE-2
#pragma unroll
  for (int s = 0; s < NSTAGE - 1; ++s) {
    if (s < nk) {
      char* st = smem + s * STAGE_BYTES;
      sa.issue(st, kb0 + s * BK, kE, convF, convC);
      sb.issue(st + TILE_BYTES, kb0 + s * BK, kE, convF, convC);
    }
  }
  for (int kt = 0; kt < nk; ++kt) {
    // stage kt must have landed: leave the younger stages (issued after it) in flight
    const int younger = min(kt + NSTAGE - 1, nk) - kt - 1;
    if (younger >= 1) wait_vm<GLDS_PER_WAVE>();
    else wait_vm<0>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const int nxt = kt + NSTAGE - 1;
    if (nxt < nk) {  // refill the slot every wave finished reading before this barrier
      char* st = smem + (nxt % NSTAGE) * STAGE_BYTES;
      sa.issue(st, kb0 + nxt * BK, kE, convF, convC);
      sb.issue(st + TILE_BYTES, kb0 + nxt * BK, kE, convF, convC);
    }
    const char* st = smem + (kt % NSTAGE) * STAGE_BYTES;
    mma_stage<PREC, A_KC, B_KC>(acc, st, st + TILE_BYTES, wm, wn);
  }
  wait_vm<0>();

  // epilogue: C/D map of 16x16 MFMA: col = lane & 15, row = (lane >> 4) * 4 + r
  const int lc = lane & 15, lr4 = (lane >> 4) * 4;
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) {
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const int col = n0 + wn * 64 + nt * 16 + lc;
      if (col >= N) continue;
      const float bv = (p.bias && split == 0) ? p.bias[col] : 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm * 64 + mt * 16 + lr4 + r;
        if (row >= M) continue;
        float* dst = C + (int64_t)row * p.ldc + col;
        float v = p.alpha * acc[mt][nt][r] + bv;
        if (p.splitk > 1) {
          atomicAdd(dst, v);
        } else {
          if (p.beta != 0.f) v += p.beta * *dst;
          if (Z) Z[(int64_t)row * p.ldc + col] = v;
          *dst = apply_act(p.act, v);
        }
      }
    }
  }
}

static int g_stages = 0;  // 2 or 3 (ASRX_GEMM_STAGES, default 2)

template <int PREC, bool AK, bool BKC, bool CA, bool CB, int NS>
static void launch_ns(const GemmParams& p, dim3 g, hipStream_t s) {
  static bool attr_set = false;  // benign race: idempotent attribute
  const int shm = NS * STAGE_BYTES;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)gemm_kernel<PREC, AK, BKC, CA, CB, NS>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, shm);
    attr_set = true;
  }
  gemm_kernel<PREC, AK, BKC, CA, CB, NS><<<g, NTHR, shm, s>>>(p);
}

template <int PREC, bool AK, bool BKC, bool CA, bool CB>
static void launch_one(const GemmParams& p, dim3 g, hipStream_t s) {
  if (g_stages == 0) {
    const char* e = getenv("ASRX_GEMM_STAGES");
    g_stages = (e && atoi(e) == 3) ? 3 : 2;
  }
  if (g_stages == 3) launch_ns<PREC, AK, BKC, CA, CB, 3>(p, g, s);
  else launch_ns<PREC, AK, BKC, CA, CB, 2>(p, g, s);
}

template <int PREC>
static void launch_prec(const GemmParams& p, bool akc, bool bkc, bool ca, bool cb, dim3 g, hipStream_t s) {
  if (ca) launch_one<PREC, true, true, true, false>(p, g, s);        // k3 conv fwd / dgrad
  else if (cb) launch_one<PREC, false, false, false, true>(p, g, s); // k3 conv wgrad
  else if (akc && bkc) launch_one<PREC, true, true, false, false>(p, g, s);
  else if (akc && !bkc) launch_one<PREC, true, false, false, false>(p, g, s);
  else if (!akc && bkc) launch_one<PREC, false, true, false, false>(p, g, s);
  else launch_one<PREC, false, false, false, false>(p, g, s);
}

}  // namespace asrx

using namespace asrx;

static bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

extern "C" int asrx_gemm(int prec, const float* A, int64_t lda, int64_t sA, int a_kc, int conv_a,
                         const float* B, int64_t ldb, int64_t sB, int b_kc, int conv_b, float* C,
                         int64_t ldc, int64_t sC, const float* bias, float* Z, int64_t M, int64_t N,
                         int64_t K, int64_t batch, float alpha, float beta, int act, int64_t conv_F,
                         int64_t conv_C, int splitk, hipStream_t stream) {
  ASRX_REQUIRE(prec == PREC_F32 || prec == PREC_BF16 || prec == PREC_X3, "asrx_gemm: bad precision %d", prec);
  ASRX_REQUIRE(M > 0 && N > 0 && K > 0 && batch > 0, "asrx_gemm: empty problem M=%ld N=%ld K=%ld",
               (long)M, (long)N, (long)K);
  ASRX_REQUIRE(aligned16(A) && aligned16(B), "asrx_gemm: A/B must be 16-byte aligned");
  ASRX_REQUIRE(!conv_a || (conv_F < (1LL << 30)), "asrx_gemm: conv segment too long");
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
  int64_t kchunk = (K + splitk - 1) / splitk;
  kchunk = (kchunk + BK - 1) / BK * BK;
  splitk = (int)((K + kchunk - 1) / kchunk);
  p.splitk = splitk;
  p.kchunk = kchunk;
  ASRX_REQUIRE(batch * splitk < 65536, "asrx_gemm: batch*splitk too large");
  ASRX_REQUIRE(M < (1LL << 31) && N < (1LL << 31), "asrx_gemm: M/N must fit int32");
  const int64_t tiles = ((N + BN - 1) / BN) * ((M + BM - 1) / BM);
  ASRX_REQUIRE(tiles * batch * splitk < (1LL << 31), "asrx_gemm: too many tiles");
  dim3 g((unsigned)(tiles * batch * splitk), 1u);
  ASRX_REQUIRE(!conv_a || b_kc, "asrx_gemm: conv fwd needs a K-contiguous B");
  ASRX_REQUIRE(!conv_b || !a_kc, "asrx_gemm: conv wgrad needs an M-contiguous A");
  ASRX_REQUIRE(!(conv_a && conv_b), "asrx_gemm: one implicit im2col operand at most");
  // 32-bit element offsets inside each operand
  const int64_t spanA = a_kc ? M * lda : K * lda, spanB = b_kc ? N * ldb : K * ldb;
  ASRX_REQUIRE(spanA < (1LL << 31) && spanB < (1LL << 31) && K < (1LL << 31),
               "asrx_gemm: operand spans >= 2^31 elements");
  if (prec == PREC_BF16) launch_prec<PREC_BF16>(p, a_kc, b_kc, conv_a, conv_b, g, stream);
  else if (prec == PREC_X3) launch_prec<PREC_X3>(p, a_kc, b_kc, conv_a, conv_b, g, stream);
  else launch_prec<PREC_F32>(p, a_kc, b_kc, conv_a, conv_b, g, stream);
  ASRX_LAUNCHED("asrx_gemm");
}
