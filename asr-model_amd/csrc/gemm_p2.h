#pragma once
// Wide GEMM, two workgroups per CU (gemm_p2_kernel): the plain and residual products of gemm_wr.h
// (Y = act(alpha A W^T + beta Y + bias) [+ R]; model.py:242-245, 421-425, 573-580) at the shapes that
// dominate the step (M = 8k..192k rows, N = 256..1536, K = 384..1536).
//
// Why a second kernel: gemm_wr_kernel runs ONE 512-thread workgroup per CU whose eight waves step
// through a tile's k-loop and then its epilogue together.  While the epilogue drains the fp32 C tile
// (196 KB at 128 x 384; stores count in vmcnt, so the next tile's first loads wait behind them) the
// matrix pipes idle, and while the k-loop runs the CU pulls only its A panel from HBM -- the two halves
// of the kernel alternate instead of overlapping (profiles/r04_gemm_epilogue_ablation.txt: the epilogue
// is a third of a K = 384 launch).  Here each CU holds TWO independent 256-thread workgroups (2 x 2
// waves of 64 x 32*NJ each, tile 128 x 64*NJ): their barriers and vmcnt counters are separate, so one
// workgroup's epilogue stores drain while the other's k-loop keeps the matrix pipes and the LDS busy.
// Per wave the k-step is gemm_wr_kernel's: the same operand images (bf16, XOR-swizzled, double
// buffered), the same 16x16x32 bf16 MFMA fragments and the same LDS-staged epilogue, so the results
// are bit-identical to gemm_wr_kernel's (tests/test_gpu_bf16_storage.py compares the two).
// The A panel of a 128-row tile is read by the N / (64 NJ) workgroups of its column tiles; their tile
// ranks are adjacent and XCD-grouped, so they run together on one XCD and share the panel in its L2.
#include "gemm_wr.h"

namespace asrx {
namespace wn {

namespace p2 {
constexpr int NT2 = 256;  // threads per workgroup: 2 (rows) x 2 (columns) waves
constexpr int WNC = 2;    // column waves

template <int NJ, bool ABF>
struct Geo {
  static constexpr int BN = WNC * 32 * NJ;                    // tile columns
  static constexpr int ACH = BM * BK * (ABF ? 2 : 4) / 16 / NT2;  // 16-B A chunks per thread and k-step
  static constexpr int WCH = BN * BK * 2 / 16 / NT2;          // 16-B W chunks per thread and k-step
  static_assert(BM * BK * (ABF ? 2 : 4) % (16 * NT2) == 0 && BN * BK * 2 % (16 * NT2) == 0, "chunking");
};

template <int NJ, bool ABF>
struct Stage {
  u32x4 a[Geo<NJ, ABF>::ACH];  // ABF: 8 bf16 (row q/4, k chunk q%4); fp32: 4 floats (row q/8, chunk q%8)
  u32x4 b[Geo<NJ, ABF>::WCH];  // 8 bf16 of W (row q/4, k chunk q%4)
};

// global -> registers: unconditional loads from clamped addresses (rows past M / N and k past K read the
// zero page), so the count of loads in flight is the same on every path and the vmcnt waits stay counted
template <int NJ, bool ABF>
__device__ __forceinline__ void load(const Params& p, Stage<NJ, ABF>& st, int m0, int n0, int k0) {
  const int t = threadIdx.x;
#pragma unroll
  for (int i = 0; i < Geo<NJ, ABF>::ACH; ++i) {
    const int q = t + NT2 * i;
    const int row = ABF ? (q >> 2) : (q >> 3), c = ABF ? (q & 3) : (q & 7);
    const int r = m0 + row, k = k0 + (ABF ? 8 : 4) * c;
    const bool ok = r < p.M && k < p.K;
    const char* src = ABF ? (const char*)(reinterpret_cast<const unsigned short*>(p.A) + (int64_t)r * p.lda + k)
                          : (const char*)(p.A + (int64_t)r * p.lda + k);
    st.a[i] = *reinterpret_cast<const u32x4*>(ok ? (const void*)src : (const void*)zero_page);
  }
#pragma unroll
  for (int i = 0; i < Geo<NJ, ABF>::WCH; ++i) {
    const int q = t + NT2 * i;
    const int n = n0 + (q >> 2), k = k0 + 8 * (q & 3);
    st.b[i] = *reinterpret_cast<const u32x4*>((n < p.N && k < p.K) ? (const void*)(p.W + (int64_t)n * p.ldw + k)
                                                                  : (const void*)zero_page);
  }
}

// Fast addressing (launches whose operands span < 4 GiB and whose K is a multiple of the k-step): each
// thread's row byte offsets are computed once per tile (rows past M / N clamped to the last row: they only
// feed accumulator rows / columns the epilogue never stores), and a k-step's load is a uniform base
// (operand + k bytes, SGPR) plus that offset -- one address add per load instead of the general path's
// ~15 instructions of row / zero-page selection, which made the k-step issue-bound.
template <int NJ, bool ABF>
struct Off {
  uint32_t a[Geo<NJ, ABF>::ACH];
  uint32_t w[Geo<NJ, ABF>::WCH];
};
template <int NJ, bool ABF>
__device__ __forceinline__ void offsets(const Params& p, Off<NJ, ABF>& o, int m0, int n0) {
  const int t = threadIdx.x;
#pragma unroll
  for (int i = 0; i < Geo<NJ, ABF>::ACH; ++i) {
    const int q = t + NT2 * i;
    const int row = min(m0 + (ABF ? (q >> 2) : (q >> 3)), p.M - 1), c = ABF ? (q & 3) : (q & 7);
    o.a[i] = ABF ? (uint32_t)(((int64_t)row * p.lda + 8 * c) * 2) : (uint32_t)(((int64_t)row * p.lda + 4 * c) * 4);
  }
#pragma unroll
  for (int i = 0; i < Geo<NJ, ABF>::WCH; ++i) {
    const int q = t + NT2 * i;
    const int n = min(n0 + (q >> 2), p.N - 1);
    o.w[i] = (uint32_t)(((int64_t)n * p.ldw + 8 * (q & 3)) * 2);
  }
}
template <int NJ, bool ABF>
__device__ __forceinline__ void load_fast(const Params& p, Stage<NJ, ABF>& st, const Off<NJ, ABF>& o, int k0) {
  const char* A = reinterpret_cast<const char*>(p.A) + (size_t)k0 * (ABF ? 2 : 4);
  const char* W = reinterpret_cast<const char*>(p.W) + (size_t)k0 * 2;
#pragma unroll
  for (int i = 0; i < Geo<NJ, ABF>::ACH; ++i) st.a[i] = *reinterpret_cast<const u32x4*>(A + o.a[i]);
#pragma unroll
  for (int i = 0; i < Geo<NJ, ABF>::WCH; ++i) st.b[i] = *reinterpret_cast<const u32x4*>(W + o.w[i]);
}

// registers -> LDS images ([rows][4 chunks of 8 bf16], chunk XOR swb(row), as gemm_wr.h wr_store)
template <int NJ, bool ABF>
__device__ __forceinline__ void store(const Stage<NJ, ABF>& st, char* At, char* Bt) {
  const int t = threadIdx.x;
#pragma unroll
  for (int i = 0; i < Geo<NJ, ABF>::ACH; ++i) {
    const int q = t + NT2 * i;
    if constexpr (ABF) {
      const int row = q >> 2, c = q & 3;
      *reinterpret_cast<u32x4*>(At + row * 64 + 16 * (c ^ swb(row))) = st.a[i];
    } else {
      const int row = q >> 3, c = q & 7;
      const float4 v = __builtin_bit_cast(float4, st.a[i]);
      typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
      bf16x4 h;
      h[0] = (__bf16)v.x; h[1] = (__bf16)v.y; h[2] = (__bf16)v.z; h[3] = (__bf16)v.w;
      *reinterpret_cast<bf16x4*>(At + row * 64 + 16 * ((c >> 1) ^ swb(row)) + 8 * (c & 1)) = h;
    }
  }
#pragma unroll
  for (int i = 0; i < Geo<NJ, ABF>::WCH; ++i) {
    const int q = t + NT2 * i;
    const int n = q >> 2, c = q & 3;
    *reinterpret_cast<u32x4*>(Bt + n * 64 + 16 * (c ^ swb(n))) = st.b[i];
  }
}
}  // namespace p2

#ifndef P2_ABL
#define P2_ABL 0  // timing ablations (wrong results): 1 no global loads, 2 no LDS image writes, 4 no MFMA, 8 no epilogue
#endif
#ifndef P2_FAST
#define P2_FAST 1  // 0: every load takes the general (zero-page select) path -- A/B builds only
#endif
#ifndef P2_DEPTH
#define P2_DEPTH 3  // register stages in flight (k-steps of prefetch)
#endif

template <int NJ, bool ABF, int ACT, bool RES, bool ROT = false>
__global__ __launch_bounds__(p2::NT2, 2) void gemm_p2_kernel(Params p, int ntiles) {
  using namespace p2;
  typedef Geo<NJ, ABF> GE;
  constexpr int BN = GE::BN, NT = 2 * NJ;
  constexpr int AB = BM * BK * 2, BB = BN * BK * 2;  // bf16 images
  __shared__ __attribute__((aligned(16))) char a_img[2][AB];
  __shared__ __attribute__((aligned(16))) char b_img[2][BB];
  __shared__ __attribute__((aligned(16))) float bias_s[2][BN];
  __shared__ __attribute__((aligned(16))) float ep_s[4 * EpLds<NJ>::FLOATS];

  const int nN = (p.N + BN - 1) / BN;
  const int nk = (p.K + BK - 1) / BK;
  const int G = gridDim.x, bid = blockIdx.x;
  const int r = (G % 8 == 0) ? (bid & 7) * (G >> 3) + (bid >> 3) : bid;  // XCD-grouped tile ranks
  const int* mlist = p.mtiles;
  if (mlist) ntiles = *p.n_mtiles * nN;  // device-side count (the list is built on the device)
  const int my = r < ntiles ? (ntiles - r + G - 1) / G : 0;
  const int S = my * nk;
  float* ep = ep_s + (threadIdx.x >> 6) * EpLds<NJ>::FLOATS;
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wm = wid >> 1, wn = wid & 1;
  const int lr = lane & 15, lk = lane >> 4;

  // step -> (tile, k) by incremental cursors (gemm_wr_kernel): load cursor DEPTH steps ahead of the
  // epilogue cursor, store cursor one ahead
  struct Cur {
    int j, kk, m0, n0;
  };
  auto enter = [&](Cur& c) __attribute__((always_inline)) {
    const int t = c.j * G + r;
    const int tm = t / nN;
    c.m0 = ((mlist && t < ntiles) ? ((const __attribute__((address_space(4))) int*)mlist)[tm] : tm) * BM;
    c.n0 = (t - tm * nN) * BN;
  };
  auto advance = [&](Cur& c) __attribute__((always_inline)) {
    if (++c.kk == nk) {
      c.kk = 0;
      ++c.j;
      enter(c);
    }
  };
  Cur cl{0, 0, 0, 0}, cs{0, 0, 0, 0}, ce{0, 0, 0, 0};
  enter(cl);
  cs = cl;
  ce = cl;
  typedef Stage<NJ, ABF> Stg;
  // past this workgroup's last tile the load cursor's rows lie beyond M: the fast path clamps them to row
  // M - 1 (in bounds; the data feeds no stored output), the general path reads the zero page
  // (not for fp32 A at NJ = 3: its seven offsets push the kernel into scratch)
  const bool fast = P2_FAST && (ABF || NJ < 3) && p.K % BK == 0 && (uint64_t)p.M * p.lda * (ABF ? 2 : 4) < (1ull << 32) &&
                    (uint64_t)p.N * p.ldw * 2 < (1ull << 32);
  Off<NJ, ABF> off;
  auto ld = [&](Stg& st) __attribute__((always_inline)) {
    if (fast) {
      if (cl.kk == 0) offsets<NJ, ABF>(p, off, cl.m0, cl.n0);
      load_fast<NJ, ABF>(p, st, off, cl.kk * BK);
    } else {
      load<NJ, ABF>(p, st, cl.m0, cl.n0, cl.kk * BK);
    }
    advance(cl);
  };
  auto st_lds = [&](int s, const Stg& st) __attribute__((always_inline)) {
    store<NJ, ABF>(st, a_img[s & 1], b_img[s & 1]);
    if (cs.kk == 0) {  // first k-step of a tile: its bias slice (read by the tile's epilogue)
      float* dst = bias_s[cs.j & 1];
      for (int c = threadIdx.x; c < BN; c += NT2) dst[c] = (p.bias && cs.n0 + c < p.N) ? p.bias[cs.n0 + c] : 0.f;
    }
    advance(cs);
  };

  f32x4 acc[4][NT];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  static_assert(P2_DEPTH == 3, "stage sets are written out for depth 3");
  Stg st0, st1, st2;
  if (S > 0) ld(st0);
  if (S > 1) ld(st1);
  if (S > 2) ld(st2);
  if (S > 0) st_lds(0, st0);
  __syncthreads();

  auto kstep = [&](int s, Stg& cur, const Stg& nxt) __attribute__((always_inline)) {
#if !(P2_ABL & 1)
    ld(cur);  // step s + 3 (unconditional: past the last step the rows read the zero page)
#else
    advance(cl);
#endif
    const char* At = a_img[s & 1];
    const char* Bt = b_img[s & 1];
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
#if !(P2_ABL & 4)
        acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[nt], a[mt], acc[mt][nt], 0, 0, 0);
#else
        acc[mt][nt][0] += (float)a[mt][0] * (float)b[nt][0];
#endif
#if !(P2_ABL & 2)
    if (s + 1 < S) st_lds(s + 1, nxt);
#else
    advance(cs);
#endif
    if (ce.kk == nk - 1) {
#if !(P2_ABL & 8)
      epilogue_lds<NJ, ACT, RES, ROT>(p, acc, bias_s[ce.j & 1], ce.m0, ce.n0, wm, wn, lr, lk, ep);
#else
      {  // the accumulators feed a never-taken store
        float t = 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int q = 0; q < NT; ++q) t += acc[i][q][0] + acc[i][q][1] + acc[i][q][2] + acc[i][q][3];
        if (t == 1.2345e-37f) p.C[ce.m0] = t;
      }
#endif
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int q = 0; q < NT; ++q) acc[i][q] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    advance(ce);
    __syncthreads();
  };

  for (int s = 0; s < S; s += 3) {
    kstep(s, st0, st1);
    if (s + 1 < S) kstep(s + 1, st1, st2);
    if (s + 2 < S) kstep(s + 2, st2, st0);
  }
}

// launch: resident workgroups (2 per CU) walk the tiles persistently
template <int NJ, bool ABF, int ACT, bool RES, bool ROT = false>
void launch_p2(const Params& p, hipStream_t s) {
  static int resident = 0;
  const void* fn = (const void*)gemm_p2_kernel<NJ, ABF, ACT, RES, ROT>;
  if (!resident) {
    int per_cu = 0, dev = 0, cus = 0;
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, p2::NT2, 0);
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    resident = std::max(1, per_cu) * std::max(1, cus);
  }
  const int tiles = ((p.M + BM - 1) / BM) * ((p.N + p2::Geo<NJ, ABF>::BN - 1) / p2::Geo<NJ, ABF>::BN);
  const int grid = std::min(tiles, resident);
  gemm_p2_kernel<NJ, ABF, ACT, RES, ROT><<<grid, p2::NT2, 0, s>>>(p, tiles);
}

// dispatch over the activation (runtime act -> template)
template <int NJ, bool ABF, bool RES>
void launch_p2_act(const Params& p, hipStream_t s) {
  if constexpr (RES) {
    launch_p2<NJ, ABF, ACT_NONE, true>(p, s);
  } else {
    switch (p.act) {
      case ACT_GELU: launch_p2<NJ, ABF, ACT_GELU, false>(p, s); break;
      case ACT_SILU: launch_p2<NJ, ABF, ACT_SILU, false>(p, s); break;
      case ACT_SIGMOID: launch_p2<NJ, ABF, ACT_SIGMOID, false>(p, s); break;
      case ACT_RELU: launch_p2<NJ, ABF, ACT_RELU, false>(p, s); break;
      default: launch_p2<NJ, ABF, ACT_NONE, false>(p, s); break;
    }
  }
}

}  // namespace wn
}  // namespace asrx

#ifndef ASRX_P2_INSTANTIATE
#define ASRX_P2_DECL(NJ, ABF, RES) extern template void asrx::wn::launch_p2_act<NJ, ABF, RES>(const asrx::wn::Params&, hipStream_t);
#else
#define ASRX_P2_DECL(NJ, ABF, RES) template void asrx::wn::launch_p2_act<NJ, ABF, RES>(const asrx::wn::Params&, hipStream_t);
#endif
#ifndef ASRX_P2_INSTANTIATE
#define ASRX_P2_DECL_ROT(NJ, ABF) extern template void asrx::wn::launch_p2<NJ, ABF, asrx::ACT_NONE, false, true>(const asrx::wn::Params&, hipStream_t);
#else
#define ASRX_P2_DECL_ROT(NJ, ABF) template void asrx::wn::launch_p2<NJ, ABF, asrx::ACT_NONE, false, true>(const asrx::wn::Params&, hipStream_t);
#endif
#ifndef ASRX_P2_INSTANTIATE
ASRX_P2_DECL_ROT(3, true)
ASRX_P2_DECL_ROT(3, false)
ASRX_P2_DECL(3, false, false)
ASRX_P2_DECL(3, true, false)
ASRX_P2_DECL(2, false, false)
ASRX_P2_DECL(2, true, false)
ASRX_P2_DECL(3, false, true)
#endif
