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
#include "../../asr-model_amd/csrc/common.h"
#define EXP_REQUIRE(c, m) if (!(c)) return -1

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
  int dbg;
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

__device__ __forceinline__ int swa(int row, bool sw2) { return sw2 ? (((row >> 1) & 1) | (((row >> 3) & 1) << 2)) : ((row >> 1) & 7); }
__device__ __forceinline__ int swb(int n, bool sw2) { return sw2 ? (((n >> 3) & 1) << 1) : ((n >> 2) & 3); }

typedef __attribute__((address_space(3))) char lds_char;
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(uintptr_t)(const lds_char*)p);
}
// LDS-DMA issued from inline asm: invisible to the compiler's waitcnt model, so it neither drains
// the ring before every ds_read nor counts these ops -- completion is tracked by hand (vmcnt).
__device__ __forceinline__ void glds16(const void* gsrc, uint32_t lds_dst) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(gsrc), "s"(lds_dst) : "memory");
}
__device__ __forceinline__ void glds4(const void* gsrc, uint32_t lds_dst) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(gsrc), "s"(lds_dst) : "memory");
}

template <int NJ, bool CONV, bool SW2 = false, bool ASM = false>
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
      const int c = (lane & 7) ^ swa(row, SW2);
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
      const int c = (lane & 3) ^ swb(row, SW2);
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
      if constexpr (ASM) glds16(src, lds_addr(st + (wid * 2 + i) * 1024));
      else __builtin_amdgcn_global_load_lds((gbl_void*)src, (lds_void*)(st + (wid * 2 + i) * 1024), 16, 0, 0);
    }
    char* bt = st + A_BYTES;
    if (p.dbg & 4) return;
#pragma unroll
    for (int i = 0; i < NJ; ++i) {
      const int lane = threadIdx.x & 63;
      const int kc = k0 + 8 * ((lane & 3) ^ swb(16 * (wid * NJ + i) + (lane >> 2), SW2));
      const bool ok = bok[i] && kc < p.K;
      const void* src = ok ? (const void*)(p.W + boff[i] + k0) : (const void*)zero_page;
      if constexpr (ASM) glds16(src, lds_addr(bt + (wid * NJ + i) * 1024));
      else __builtin_amdgcn_global_load_lds((gbl_void*)src, (lds_void*)(bt + (wid * NJ + i) * 1024), 16, 0, 0);
    }
  }
};

template <int N>
__device__ __forceinline__ void wait_vm() {
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (N == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
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
    if (kt + 1 < nk) { if (p.dbg & 4) wait_vm<2>(); else wait_vm<CF::PIECES>(); }
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
    if (!(p.dbg & 2)) {
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt)
        acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[mt], b[nt], acc[mt][nt], 0, 0, 0);
    } else {
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) acc[mt][nt][0] += (float)a[mt][0] * (float)b[nt][0];
    }
  }

  if (p.dbg & 1) {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j) s += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
    if (s == 12345.678f) p.C[threadIdx.x] = s;
    return;
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


// ---------------------------------------------------------------- persistent variant
// Persistent workgroups (one per CU) walk their tiles with the LDS-DMA ring running across tile
// boundaries: the next tile's first k-steps are in flight while the current tile's epilogue
// stores drain.  MFMA operands are swapped (W fragment as the 16-row operand) so each lane owns
// 4 consecutive output columns of one row: float4 epilogue stores (4x fewer store instructions).
__device__ __forceinline__ void wait_le(int n) {
  // s_waitcnt vmcnt(k) for the largest listed k <= n (waiting for more than needed is safe)
  if (n >= 48) asm volatile("s_waitcnt vmcnt(48)" ::: "memory");
  else if (n >= 40) asm volatile("s_waitcnt vmcnt(40)" ::: "memory");
  else if (n >= 32) asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
  else if (n >= 28) asm volatile("s_waitcnt vmcnt(28)" ::: "memory");
  else if (n >= 24) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
  else if (n >= 20) asm volatile("s_waitcnt vmcnt(20)" ::: "memory");
  else if (n >= 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  else if (n >= 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  else if (n >= 10) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
  else if (n >= 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if (n >= 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else if (n >= 5) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
  else if (n >= 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if (n >= 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
  else if (n >= 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else if (n >= 1) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <int NJ, bool CONV, int NS, int DBG, bool SWZ>
__global__ __launch_bounds__(NTHR, 1) void gemm_wnp_kernel(Params p, int ntiles) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  typedef Cfg<NJ> CF;
  constexpr int BN = CF::BN;
  constexpr int NT = 2 * NJ;
  constexpr int P = CF::PIECES;
  constexpr int BNR = (BN + NTHR - 1) / NTHR * NTHR;  // bias slice rounded to whole DMA rounds
  float* bias_s = reinterpret_cast<float*>(smem + NS * CF::STAGE);  // [2][BNR]

  const int nN = (p.N + BN - 1) / BN;
  const int nk = (p.K + BK - 1) / BK;
  const int G = gridDim.x;
  const int bid = blockIdx.x;
  const int r = (G % 8 == 0) ? (bid & 7) * (G >> 3) + (bid >> 3) : bid;
  const int my = r < ntiles ? (ntiles - r + G - 1) / G : 0;
  const int S = my * nk;
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wm = wid >> 2, wn = wid & 3;
  const int lr = lane & 15, lk = lane >> 4;
  const bool has_bias = p.bias != nullptr;
  const int E = (DBG & 1) ? 0 : 4 * NT * (p.Z ? 2 : 1);  // vector-memory ops per lane in one epilogue

  auto coords = [&](int j, int& m0, int& n0) {
    const int t = j * G + r;
    m0 = (t / nN) * BM;
    n0 = (t % nN) * BN;
  };

  Loader<NJ, CONV, SWZ, true> ld;
  int ld_tile = -1;
  auto issue = [&](int s) {
    const int j = s / nk, kt = s - j * nk;
    if (j != ld_tile) {
      int m0, n0;
      coords(j, m0, n0);
      ld.init(p, m0, n0);
      ld_tile = j;
    }
    char* st = smem + (s % NS) * CF::STAGE;
    if constexpr (DBG & 4) return;
    ld.issue(p, st, kt * BK);
    if (kt == 0 && has_bias) {  // this tile's bias slice, one dword per thread by LDS-DMA
      int m0, n0;
      coords(j, m0, n0);
      float* dst = bias_s + (j & 1) * BNR;
#pragma unroll
      for (int c0 = 0; c0 < BNR; c0 += NTHR) {  // every lane of every wave issues: uniform vmcnt
        const int c = c0 + threadIdx.x;
        const float* src = (c < BN && n0 + c < p.N) ? p.bias + n0 + c : zero_page;
        glds4(src, lds_addr(dst + c0 + wid * 64));
      }
    }
  };
  // vector-memory ops one issue() puts in flight per lane
  auto pieces = [&](int s) {
    if constexpr (DBG & 4) return 0;
    const int kt = s % nk;
    return P + ((kt == 0 && has_bias) ? BNR / NTHR : 0);
  };

  f32x4 acc[4][NT];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (s < S) issue(s);

  for (int s = 0; s < S; ++s) {
    // ops younger than step s's loads: later issued steps + epilogues after step s was issued
    int younger = 0;
    for (int q = s + 1; q <= min(s + NS - 2, S - 1); ++q) younger += pieces(q);
    for (int it = max(s - NS + 1, 0); it < s; ++it)
      if (it % nk == nk - 1) younger += E;
    wait_le(younger);
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (s + NS - 1 < S) issue(s + NS - 1);
    const char* At = smem + (s % NS) * CF::STAGE;
    const char* Bt = At + A_BYTES;
    bf16x8 a[4], b[NT];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      const int rr = wm * 64 + mt * 16 + lr;
      const int sw = swa(rr, SWZ);
      const char* row = At + rr * 128;
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
      b[nt] = *reinterpret_cast<const bf16x8*>(Bt + n * 64 + 16 * (lk ^ swb(n, SWZ)));
    }
    if constexpr (!(DBG & 2)) {
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt)
        acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[nt], a[mt], acc[mt][nt], 0, 0, 0);
    } else {
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) acc[mt][nt][0] += (float)a[mt][0] * (float)b[nt][0];
    }

    if (s % nk == nk - 1 && (DBG & 1)) {
      float sx = 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j2 = 0; j2 < NT; ++j2) { sx += acc[i][j2][0] + acc[i][j2][3]; acc[i][j2] = f32x4{0.f, 0.f, 0.f, 0.f}; }
      if (sx == 12345.678f) p.C[threadIdx.x] = sx;
    } else if (s % nk == nk - 1) {
      const int j = s / nk;
      int m0, n0;
      coords(j, m0, n0);
      const float* bsl = bias_s + (j & 1) * BNR;
      auto finish = [&](int mt, int nt) -> float4 {
        const int nl = wn * (32 * NJ) + nt * 16 + 4 * lk;
        float4 bv = make_float4(0.f, 0.f, 0.f, 0.f);
        if (has_bias) bv = *reinterpret_cast<const float4*>(bsl + nl);
        float4 v = make_float4(p.alpha * acc[mt][nt][0] + bv.x, p.alpha * acc[mt][nt][1] + bv.y,
                               p.alpha * acc[mt][nt][2] + bv.z, p.alpha * acc[mt][nt][3] + bv.w);
        const int row = m0 + wm * 64 + mt * 16 + lr, col = n0 + nl;
        if (p.beta != 0.f && row < p.M && col < p.N) {
          const float4 o = *reinterpret_cast<const float4*>(p.C + (int64_t)row * p.ldc + col);
          v.x += p.beta * o.x; v.y += p.beta * o.y; v.z += p.beta * o.z; v.w += p.beta * o.w;
        }
        if (p.Z && row < p.M && col < p.N) *reinterpret_cast<float4*>(p.Z + (int64_t)row * p.ldc + col) = v;
        v.x = apply_act(p.act, v.x); v.y = apply_act(p.act, v.y);
        v.z = apply_act(p.act, v.z); v.w = apply_act(p.act, v.w);
        acc[mt][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
        return v;
      };
      auto put = [&](int row, int col, float4 v) {
        if (row < p.M && col < p.N) {
          if constexpr (DBG & 16) {
            f32x4* dst = reinterpret_cast<f32x4*>(p.C + (int64_t)row * p.ldc + col);
            __builtin_nontemporal_store(f32x4{v.x, v.y, v.z, v.w}, dst);
          } else {
            *reinterpret_cast<float4*>(p.C + (int64_t)row * p.ldc + col) = v;
          }
        }
      };
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        const int rb = m0 + wm * 64 + mt * 16;
        if constexpr (DBG & 8) {
#pragma unroll
          for (int nt = 0; nt < NT; nt += 2) {
            const float4 a = finish(mt, nt), bq = finish(mt, nt + 1);
            float4 y;
            y.x = __shfl_xor(bq.x, 8); y.y = __shfl_xor(bq.y, 8); y.z = __shfl_xor(bq.z, 8); y.w = __shfl_xor(bq.w, 8);
            const int c0 = n0 + wn * (32 * NJ) + nt * 16 + 4 * lk, c1 = c0 + 16;
            if (lr < 8) { put(rb + lr, c0, a); put(rb + lr + 8, c1, y); }
            else { put(rb + lr - 8, c1, y); put(rb + lr, c0, a); }
          }
        } else {
#pragma unroll
          for (int nt = 0; nt < NT; ++nt) {
            const float4 a = finish(mt, nt);
            put(rb + lr, n0 + wn * (32 * NJ) + nt * 16 + 4 * lk, a);
          }
        }
      }
    }
  }
}

template <int NJ, bool CONV, int NS, int DBG, bool SWZ>
static void launch_p(const Params& p, int grid_cap, hipStream_t s) {
  typedef Cfg<NJ> CF;
  static bool attr = false;
  const int shm = NS * CF::STAGE + 2 * ((CF::BN + NTHR - 1) / NTHR * NTHR) * 4;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)gemm_wnp_kernel<NJ, CONV, NS, DBG, SWZ>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              shm);
    attr = true;
  }
  const int tiles = ((p.M + BM - 1) / BM) * ((p.N + CF::BN - 1) / CF::BN);
  const int grid = std::min(tiles, grid_cap);
  gemm_wnp_kernel<NJ, CONV, NS, DBG, SWZ><<<grid, NTHR, shm, s>>>(p, tiles);
}
}  // namespace wn
}  // namespace asrx

using namespace asrx;

extern "C" int exp_gemm_wn(int dbg, const float* A, int64_t lda, int conv, int64_t convF, int64_t convC,
                            const unsigned short* W, int64_t ldw, float* C, int64_t ldc, const float* bias, float* Z,
                            int64_t M, int64_t N, int64_t K, float alpha, float beta, int act, int nj,
                            hipStream_t stream) {
  EXP_REQUIRE(M > 0 && N > 0 && K > 0, "asrx_gemm_wn: empty problem");
  EXP_REQUIRE(((uintptr_t)A & 15) == 0 && ((uintptr_t)W & 15) == 0, "asrx_gemm_wn: A/W must be 16-byte aligned");
  EXP_REQUIRE(K % 8 == 0 && lda % 4 == 0 && ldw % 8 == 0, "asrx_gemm_wn: K%%8, lda%%4, ldw%%8 required");
  EXP_REQUIRE(M * lda < (1LL << 31) && N * ldw < (1LL << 31), "asrx_gemm_wn: operand spans >= 2^31 elements");
  EXP_REQUIRE(!conv || (convF > 0 && convC % 4 == 0), "asrx_gemm_wn: conv needs F > 0 and C %% 4 == 0");
  wn::Params p{A, (int)lda, W, (int)ldw, C, (int)ldc, bias, Z, (int)M, (int)N, (int)K,
               (int)(convF > 0 ? convF : 1), (int)(convC > 0 ? convC : 1), alpha, beta, act, dbg};
  if (nj == 3) conv ? wn::launch<3, true>(p, stream) : wn::launch<3, false>(p, stream);
  else if (nj == 2) conv ? wn::launch<2, true>(p, stream) : wn::launch<2, false>(p, stream);
  else conv ? wn::launch<1, true>(p, stream) : wn::launch<1, false>(p, stream);
  return (int)hipGetLastError();
}

template <int NJ, int NS>
static void disp(const wn::Params& p, int dbg, int swz, int cap, hipStream_t stream) {
  if (swz) {
    if (dbg == 0) wn::launch_p<NJ, false, NS, 0, true>(p, cap, stream);
    else if (dbg == 1) wn::launch_p<NJ, false, NS, 1, true>(p, cap, stream);
    else if (dbg == 6) wn::launch_p<NJ, false, NS, 6, true>(p, cap, stream);
    else if (dbg == 8) wn::launch_p<NJ, false, NS, 8, true>(p, cap, stream);
    else if (dbg == 16) wn::launch_p<NJ, false, NS, 16, true>(p, cap, stream);
    else if (dbg == 24) wn::launch_p<NJ, false, NS, 24, true>(p, cap, stream);
    else if (dbg == 14) wn::launch_p<NJ, false, NS, 14, true>(p, cap, stream);
    else if (dbg == 30) wn::launch_p<NJ, false, NS, 30, true>(p, cap, stream);
    else wn::launch_p<NJ, false, NS, 3, true>(p, cap, stream);
  } else {
    if (dbg == 0) wn::launch_p<NJ, false, NS, 0, false>(p, cap, stream);
    else if (dbg == 1) wn::launch_p<NJ, false, NS, 1, false>(p, cap, stream);
    else wn::launch_p<NJ, false, NS, 3, false>(p, cap, stream);
  }
}

extern "C" int exp_gemm_wnp(int cfg, const float* A, int64_t lda, int conv, int64_t convF, int64_t convC,
                            const unsigned short* W, int64_t ldw, float* C, int64_t ldc, const float* bias, float* Z,
                            int64_t M, int64_t N, int64_t K, float alpha, float beta, int act, int nj,
                            hipStream_t stream) {
  // cfg = swz * 1000000 + dbg * 100000 + ns * 1000 + grid_cap
  wn::Params p{A, (int)lda, W, (int)ldw, C, (int)ldc, bias, Z, (int)M, (int)N, (int)K,
               (int)(convF > 0 ? convF : 1), (int)(convC > 0 ? convC : 1), alpha, beta, act, 0};
  const int ns = (cfg / 1000) % 100, cap = cfg % 1000, dbg = (cfg / 100000) % 100, swz = cfg / 10000000;
  if (nj == 3) {
    if (ns == 2) disp<3, 2>(p, dbg, swz, cap, stream); else disp<3, 3>(p, dbg, swz, cap, stream);
  } else {
    disp<1, 3>(p, dbg, swz, cap, stream);
  }
  return (int)hipGetLastError();
}
