// Wide-N GEMM for activation x weight products (perf mode): every nn.Linear / 1x1 / k3 conv forward
// and input-gradient on the hot path (model.py:96-147, 242-245, 341, 398-425, 529-574;
// essentials.py:149-153), i.e. Y = act(alpha * A W^T + beta * Y + bias) with
//   A  fp32 activations (M x K, row-major, or the implicit k3 im2col of a channels-last sequence),
//   W  the weight pre-converted to bf16, stored N x K (K contiguous) -- asrx_weight_to_bf16.
//
// Why a second GEMM: at the model's shapes (M = 8k..192k rows, N, K = 64..1536) the kernel is bound
// by bytes moved HBM/L2 -> LDS, not by MFMA.  A 128 x BN tile with BN = 128 * NJ up to 384 reads
// each activation row panel once (instead of once per 128-column tile) and the bf16 weight panel
// costs half the fp32 bytes.  512 threads = 8 waves (2 x 4), each wave 64 x 32*NJ of the output
// (4 x 2*NJ MFMA 16x16x32 bf16 tiles).  A (fp32, 16 KB) and W (bf16, 8*NJ KB) tiles of 32 k stream
// HBM -> LDS by LDS-DMA into a 3-stage ring with counted vmcnt; A fragments are rounded to bf16 in
// registers.  Images are XOR-swizzled through the per-lane source address (rule 21).
#include "common.h"

namespace asrx {

namespace wn {

constexpr int BM = 128, BK = 32, NTHR = 512, NSTAGE = 3;
constexpr int A_BYTES = BM * BK * 4;  // 16 KB fp32

__device__ __attribute__((aligned(16))) float zero_page[4];

typedef __attribute__((address_space(3))) void lds_void;
typedef const __attribute__((address_space(1))) void gbl_void;

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
};

template <int NJ>
struct Cfg {
  static constexpr int BN = 128 * NJ;
  static constexpr int B_BYTES = BN * BK * 2;  // bf16
  static constexpr int STAGE = A_BYTES + B_BYTES;
  static constexpr int A_PIECES = A_BYTES / 1024 / 8;  // per wave: 2
  static constexpr int B_PIECES = B_BYTES / 1024 / 8;  // per wave: NJ
  static constexpr int PIECES = A_PIECES + B_PIECES;
};

template <int NJ, bool CONV>
struct Loader {
  uint32_t aoff[2];
  int akk[2], apos[2];
  bool aok[2];
  uint32_t boff[NJ];
  bool bok[NJ];

  __device__ __forceinline__ void init(const Params& p, int m0, int n0) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
    for (int i = 0; i < 2; ++i) {  // A: [128 rows][8 chunks of 4 fp32]; piece q = 8 rows
      const int q = wid * 2 + i;
      const int row = 8 * q + (lane >> 3);
      const int c = (lane & 7) ^ ((row >> 1) & 7);
      const int r = m0 + row;
      aok[i] = r < p.M;
      aoff[i] = (uint32_t)r * (uint32_t)p.lda + 4 * c;
      akk[i] = 4 * c;
      apos[i] = CONV ? r % p.convF : 0;
    }
#pragma unroll
    for (int i = 0; i < NJ; ++i) {  // W: [BN rows][4 chunks of 8 bf16]; piece q = 16 rows
      const int q = wid * NJ + i;
      const int row = 16 * q + (lane >> 2);
      const int c = (lane & 3) ^ ((row >> 2) & 3);
      const int n = n0 + row;
      bok[i] = n < p.N;
      boff[i] = (uint32_t)n * (uint32_t)p.ldw + 8 * c;
    }
  }

  __device__ __forceinline__ void issue(const Params& p, char* st, int k0) const {
    const int wid = threadIdx.x >> 6;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int k = k0 + akk[i];
      bool ok = aok[i] && k < p.K;
      uint32_t o = aoff[i] + (uint32_t)k0;
      if (CONV) {
        const int pos = apos[i] + k / p.convC - 1;
        ok = ok && pos >= 0 && pos < p.convF;
        o -= (uint32_t)p.convC;
      }
      const float* src = ok ? p.A + o : zero_page;
      __builtin_amdgcn_global_load_lds((gbl_void*)src, (lds_void*)(st + (wid * 2 + i) * 1024), 16, 0, 0);
    }
    char* bt = st + A_BYTES;
#pragma unroll
    for (int i = 0; i < NJ; ++i) {
      const int lane = threadIdx.x & 63;
      const int kc = k0 + 8 * ((lane & 3) ^ (((16 * (wid * NJ + i) + (lane >> 2)) >> 2) & 3));
      const bool ok = bok[i] && kc < p.K;
      const void* src = ok ? (const void*)(p.W + boff[i] + k0) : (const void*)zero_page;
      __builtin_amdgcn_global_load_lds((gbl_void*)src, (lds_void*)(bt + (wid * NJ + i) * 1024), 16, 0, 0);
    }
  }
};

template <int N>
__device__ __forceinline__ void wait_vm() {
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (N == 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
  else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if constexpr (N == 5) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
}

__device__ __forceinline__ void tile_of(int bid, int nblk, int nN, int& tm, int& tn) {
  const int xcd = bid & 7, q = nblk >> 3, r = nblk & 7;
  const int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  tn = wg % nN;
  tm = wg / nN;
}

template <int NJ, bool CONV>
__global__ __launch_bounds__(NTHR, 1) void gemm_wn_kernel(Params p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  typedef Cfg<NJ> CF;
  constexpr int BN = CF::BN;
  constexpr int NT = 2 * NJ;  // 16-wide n tiles per wave

  const int nN = (p.N + BN - 1) / BN;
  int tm, tn;
  tile_of(blockIdx.x, gridDim.x, nN, tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wm = wid >> 2, wn = wid & 3;
  const int lr = lane & 15, lk = lane >> 4;

  f32x4 acc[4][NT];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  Loader<NJ, CONV> ld;
  ld.init(p, m0, n0);
  const int nk = (p.K + BK - 1) / BK;
#pragma unroll
  for (int s = 0; s < NSTAGE - 1; ++s)
    if (s < nk) ld.issue(p, smem + s * CF::STAGE, s * BK);

  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) wait_vm<CF::PIECES>();
    else wait_vm<0>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const int nxt = kt + NSTAGE - 1;
    if (nxt < nk) ld.issue(p, smem + (nxt % NSTAGE) * CF::STAGE, nxt * BK);
    const char* At = smem + (kt % NSTAGE) * CF::STAGE;
    const char* Bt = At + A_BYTES;
    bf16x8 a[4], b[NT];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      const int r = wm * 64 + mt * 16 + lr;
      const int sw = (r >> 1) & 7;
      const char* row = At + r * 128;
      const float4 x = *reinterpret_cast<const float4*>(row + 16 * ((2 * lk) ^ sw));
      const float4 y = *reinterpret_cast<const float4*>(row + 16 * ((2 * lk + 1) ^ sw));
      bf16x8 v;
      v[0] = (__bf16)x.x; v[1] = (__bf16)x.y; v[2] = (__bf16)x.z; v[3] = (__bf16)x.w;
      v[4] = (__bf16)y.x; v[5] = (__bf16)y.y; v[6] = (__bf16)y.z; v[7] = (__bf16)y.w;
      a[mt] = v;
    }
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const int n = wn * (32 * NJ) + nt * 16 + lr;
      b[nt] = *reinterpret_cast<const bf16x8*>(Bt + n * 64 + 16 * (lk ^ ((n >> 2) & 3)));
    }
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt)
        acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[mt], b[nt], acc[mt][nt], 0, 0, 0);
  }

  const int lc = lane & 15, lr4 = (lane >> 4) * 4;
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    const int col = n0 + wn * (32 * NJ) + nt * 16 + lc;
    if (col >= p.N) continue;
    const float bv = p.bias ? p.bias[col] : 0.f;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm * 64 + mt * 16 + lr4 + r;
        if (row >= p.M) continue;
        float* dst = p.C + (int64_t)row * p.ldc + col;
        float v = p.alpha * acc[mt][nt][r] + bv;
        if (p.beta != 0.f) v += p.beta * *dst;
        if (p.Z) p.Z[(int64_t)row * p.ldc + col] = v;
        *dst = apply_act(p.act, v);
      }
    }
  }
}

// fp32 (rows x cols, row stride ld) -> bf16 N x K contiguous.  trans == 0: N = rows, K = cols;
// trans == 1: N = cols, K = rows (the weight is used transposed, e.g. dgrad's dY W).
__global__ void weight_to_bf16_kernel(const float* __restrict__ src, unsigned short* __restrict__ dst, int rows,
                                      int cols, int64_t ld, int trans) {
  const int64_t total = (int64_t)rows * cols;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    int64_t r, c, o;
    if (!trans) {
      r = i / cols;
      c = i % cols;
      o = r * cols + c;
    } else {
      c = i / rows;  // output row n = source column
      r = i % rows;
      o = c * rows + r;
    }
    __bf16 h = (__bf16)src[r * ld + c];
    dst[o] = __builtin_bit_cast(unsigned short, h);
  }
}

template <int NJ, bool CONV>
static void launch(const Params& p, hipStream_t s) {
  typedef Cfg<NJ> CF;
  static bool attr = false;
  const int shm = NSTAGE * CF::STAGE;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)gemm_wn_kernel<NJ, CONV>, hipFuncAttributeMaxDynamicSharedMemorySize, shm);
    attr = true;
  }
  const int tiles = ((p.M + BM - 1) / BM) * ((p.N + CF::BN - 1) / CF::BN);
  gemm_wn_kernel<NJ, CONV><<<tiles, NTHR, shm, s>>>(p);
}

}  // namespace wn
}  // namespace asrx

using namespace asrx;

extern "C" int asrx_weight_to_bf16(const float* src, unsigned short* dst, int64_t rows, int64_t cols, int64_t ld,
                                   int trans, hipStream_t stream) {
  if (rows * cols == 0) return 0;
  const int64_t n = rows * cols;
  wn::weight_to_bf16_kernel<<<(unsigned)std::min<int64_t>((n + 255) / 256, 16384), 256, 0, stream>>>(
      src, dst, (int)rows, (int)cols, ld, trans);
  ASRX_LAUNCHED("asrx_weight_to_bf16");
}

// Y (M x N, ldc) = act(alpha * A W^T + beta * Y + bias); A fp32 (M x K, lda) or its k3 im2col
// (conv: lda = channels, K = 3 * channels, segment length convF); W bf16 (N x K, ldw).  nj selects
// the tile width 128 * nj (1..3).
extern "C" int asrx_gemm_wn(const float* A, int64_t lda, int conv, int64_t convF, int64_t convC,
                            const unsigned short* W, int64_t ldw, float* C, int64_t ldc, const float* bias, float* Z,
                            int64_t M, int64_t N, int64_t K, float alpha, float beta, int act, int nj,
                            hipStream_t stream) {
  ASRX_REQUIRE(M > 0 && N > 0 && K > 0, "asrx_gemm_wn: empty problem");
  ASRX_REQUIRE(((uintptr_t)A & 15) == 0 && ((uintptr_t)W & 15) == 0, "asrx_gemm_wn: A/W must be 16-byte aligned");
  ASRX_REQUIRE(K % 8 == 0 && lda % 4 == 0 && ldw % 8 == 0, "asrx_gemm_wn: K%%8, lda%%4, ldw%%8 required");
  ASRX_REQUIRE(M * lda < (1LL << 31) && N * ldw < (1LL << 31), "asrx_gemm_wn: operand spans >= 2^31 elements");
  ASRX_REQUIRE(!conv || (convF > 0 && convC % 4 == 0), "asrx_gemm_wn: conv needs F > 0 and C %% 4 == 0");
  wn::Params p{A, (int)lda, W, (int)ldw, C, (int)ldc, bias, Z, (int)M, (int)N, (int)K,
               (int)(convF > 0 ? convF : 1), (int)(convC > 0 ? convC : 1), alpha, beta, act};
  if (nj == 3) conv ? wn::launch<3, true>(p, stream) : wn::launch<3, false>(p, stream);
  else if (nj == 2) conv ? wn::launch<2, true>(p, stream) : wn::launch<2, false>(p, stream);
  else conv ? wn::launch<1, true>(p, stream) : wn::launch<1, false>(p, stream);
  ASRX_LAUNCHED("asrx_gemm_wn");
}
