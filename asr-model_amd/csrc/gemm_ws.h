#pragma once
// Weight-stationary wide GEMM (gemm_ws_kernel) for the K <= 384 activation x weight products that dominate
// the step (every projection of model.py:242-245, 421-425, 573-580 on D = 384 inputs, and their input
// gradients): Y = act(alpha A W^T + beta Y + bias) [+ R] [rotary], the epilogues of gemm_wr.h.
//
// Why a third kernel.  Ablations of gemm_p2_kernel at 192064 x 384 x 384 (profiles/r05_p2_ablation.txt) put
// the LDS IMAGE WRITES at a third of its time (103.5 -> 68.2 us without them; -165 us of 380 at K = 1536): a
// ds_write_b128 moves 16 B per lane at ~77 B/clk/CU (MI355X_MICROARCH.md LDS table), and every k-step of
// every 128 x 192 tile re-stages the weight tile (12 KB) beside the activation tile (8 KB).  Here the
// weight is staged ONCE per workgroup: each workgroup owns one 128-column slice of W for the whole launch
// (128 x K bf16 <= 96 KB of LDS, XOR-swizzled for conflict-free fragment reads) and walks row tiles down
// that slice, so a k-step writes only the 8 KB activation tile (fp32 activations are converted to bf16 on
// the way in) -- 60 % fewer LDS write bytes per output than gemm_p2.  The activation panel of a row tile
// is read by the ceil(N / 128) workgroups of its column slices; their logical ranks are adjacent and
// XCD-grouped, they run in lockstep over the same row tiles, so the panel comes from HBM about once and from
// the XCD's L2 for the other slices.  Activation tiles travel global -> VGPR -> LDS with plain 16-B loads
// DEPTH k-steps ahead (the register pipeline runs across tile boundaries, so the next tile's first loads are
// in flight before a tile's epilogue stores).
//
// Per wave the k-step is gemm_wr_kernel's (16x16x32 bf16 MFMA, the W fragment as the row operand, the same
// k order), and the epilogue is its epilogue_lds with a 32-column wave tile (NJ = 1), so the results are
// bit-identical to gemm_wr_kernel / gemm_p2_kernel (tests/test_gpu_gemm_ws.py).
#include "gemm_wr.h"

namespace asrx {
namespace wn {
namespace ws {

constexpr int BN = 128;     // columns of a slice (= of a tile)
constexpr int KMAX = 384;   // the resident slice holds K <= KMAX
constexpr int ROWB = KMAX * 2;  // W image row stride (bytes): 48 chunks of 8 bf16
constexpr int WTHR = 512;   // 8 waves: 2 (rows) x 4 (columns) of 64 x 32
// k-step geometry per activation storage type (measured, profiles/r05_ws_micro.txt): bf16 activations take
// 32-deep k-steps with THREE activation images -- during step t the MFMAs run on fragments read during step
// t - 1, the fragments of step t + 1 are read while they run, step t + 2 is staged -- and 6 steps in flight
// (4-6 % over gemm_p2 at N >= 768); fp32 activations (16 KB per 32-deep step) take 64-deep steps with two
// images and 4 in flight (the pipelined form was 6-8 % slower for them: twice the stage bytes per step)
template <bool ABF>
struct WsCfg {
  static constexpr int KS = ABF ? 32 : 64;     // k-step depth
  static constexpr int CH = KS / 8;            // 16-B chunks of 8 bf16 per activation-image row
  static constexpr bool PIPE = ABF;            // three images, fragment prefetch
  static constexpr int NBUF = PIPE ? 3 : 2;
  static constexpr int DEPTH = ABF ? 6 : 4;    // activation k-steps in flight
};
// activation-image chunk swizzle: conflict-free ds_read_b128 fragment reads (gemm_wr.h swb / sw64)
template <int KS>
__device__ __forceinline__ int aswz(int row) {
  if constexpr (KS == 64) return sw64(row);
  else return swb(row);
}

// W image chunk position: the low 4 bits of the chunk index XORed with the row's low 4 bits -- rows are 768 B
// (a multiple of 256 B), so without it the 16 rows a ds_read_b128 lane group reads would share one bank set
__device__ __forceinline__ int wchunk(int n, int c) { return (c & ~15) | ((c ^ n) & 15); }

// 16-B activation loads per thread and k-step: bf16 KS/32, fp32 KS/16 (q = t + 512 i: bf16 row q / CH, chunk
// q % CH of 8 elements; fp32 row q / (2 CH), chunk q % (2 CH) of 4 elements)
template <bool ABF>
struct Stage {
  static constexpr int NA = ABF ? WsCfg<ABF>::KS / 32 : WsCfg<ABF>::KS / 16;
  u32x4 a[NA];
};

template <bool ABF>
__device__ __forceinline__ void stage_store(const Stage<ABF>& st, char* At) {
  constexpr int KS = WsCfg<ABF>::KS, CH = WsCfg<ABF>::CH;
  const int t = threadIdx.x;
#pragma unroll
  for (int i = 0; i < Stage<ABF>::NA; ++i) {
    const int q = t + WTHR * i;
    if constexpr (ABF) {
      const int row = q / CH, c = q % CH;
      *reinterpret_cast<u32x4*>(At + row * (2 * KS) + 16 * (c ^ aswz<KS>(row))) = st.a[i];
    } else {
      const int row = q / (2 * CH), c = q % (2 * CH);
      const float4 v = __builtin_bit_cast(float4, st.a[i]);
      typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
      bf16x4 h;
      h[0] = (__bf16)v.x; h[1] = (__bf16)v.y; h[2] = (__bf16)v.z; h[3] = (__bf16)v.w;
      *reinterpret_cast<bf16x4*>(At + row * (2 * KS) + 16 * ((c >> 1) ^ aswz<KS>(row)) + 8 * (c & 1)) = h;
    }
  }
}

}  // namespace ws

// grid = nS * lanes workgroups: slice s = rank % nS, row tiles rank / nS + i * lanes
template <bool ABF, int ACT, bool RES, bool ROT>
__global__ __launch_bounds__(ws::WTHR, 1) void gemm_ws_kernel(Params p, int nS, int lanes) {
  using namespace ws;
  constexpr int KS = WsCfg<ABF>::KS, CH = WsCfg<ABF>::CH, NBUF = WsCfg<ABF>::NBUF, DEPTH = WsCfg<ABF>::DEPTH;
  constexpr bool PIPE = WsCfg<ABF>::PIPE;
  __shared__ __attribute__((aligned(16))) char w_img[BN * ROWB];      // 96 KB resident weight slice
  __shared__ __attribute__((aligned(16))) char a_img[NBUF][BM * KS * 2];  // 2-3 x 8 / 16 KB activation tiles
  __shared__ __attribute__((aligned(16))) float bias_s[BN];
  __shared__ __attribute__((aligned(16))) float ep_s[8 * EpLds<1>::FLOATS];

  const int G = gridDim.x;
  // XCD-grouped logical rank (hardware ids are dealt to the 8 XCDs round-robin), so the nS consecutive ranks
  // that share a row tile sit on one XCD
  int r;
  {
    const int per = G / 8, rem = G % 8, x = blockIdx.x % 8, q = blockIdx.x / 8;
    r = (x < rem ? x * (per + 1) : rem * (per + 1) + (x - rem) * per) + q;
  }
  const int s = r % nS, lane0 = r / nS;
  const int n0 = s * BN;
  const int nM = (p.M + BM - 1) / BM;
  const int my = lane0 < nM ? (nM - lane0 + lanes - 1) / lanes : 0;
  const int nk = p.K / KS;  // K % KS == 0 (launcher)
  const int S = my * nk;
  const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63;
  const int wm = wid >> 2, wn = wid & 3;
  const int lr = lane & 15, lk = lane >> 4;
  float* ep = ep_s + wid * EpLds<1>::FLOATS;

  // ---- the weight slice (rows n0 .. n0 + 127 of W, K columns; rows past N and chunks past K are zero)
  {
    const int nch = p.K / 8;
    for (int i = tid; i < BN * nch; i += WTHR) {
      const int n = i / nch, c = i - n * nch;
      u32x4 v = {0u, 0u, 0u, 0u};
      if (n0 + n < p.N) v = *reinterpret_cast<const u32x4*>(p.W + (int64_t)(n0 + n) * p.ldw + 8 * c);
      *reinterpret_cast<u32x4*>(w_img + n * ROWB + 16 * wchunk(n, c)) = v;
    }
    for (int c = tid; c < BN; c += WTHR) bias_s[c] = (p.bias && n0 + c < p.N) ? p.bias[n0 + c] : 0.f;
  }

  // ---- load cursor: (tile ordinal j, k-step kk) DEPTH steps ahead of the compute cursor; its row base is
  // computed once per tile (rows past M clamped to M - 1: they feed only accumulator rows the epilogue drops)
  constexpr int AES = ABF ? 2 : 4;
  int lj = 0, lkk = 0;
  constexpr int NA = Stage<ABF>::NA, CE = ABF ? CH : 2 * CH, EL = ABF ? 8 : 4;  // chunks per row, elements per chunk
  // named, not an array (an array of them is placed in scratch)
  const char *ab0 = nullptr, *ab1 = nullptr, *ab2 = nullptr, *ab3 = nullptr;
  auto enter = [&]() __attribute__((always_inline)) {
    const int m0 = (lane0 + lj * lanes) * BM;
    const char* A = reinterpret_cast<const char*>(p.A);
    auto at = [&](int i) __attribute__((always_inline)) {
      const int q = tid + WTHR * i;
      return A + ((int64_t)min(m0 + q / CE, p.M - 1) * p.lda + EL * (q % CE)) * AES;
    };
    ab0 = at(0);
    if constexpr (NA > 1) ab1 = at(1);
    if constexpr (NA > 2) {
      ab2 = at(2);
      ab3 = at(3);
    }
  };
  enter();
  auto load = [&](Stage<ABF>& st) __attribute__((always_inline)) {
    const size_t ko = (size_t)lkk * KS * AES;
    st.a[0] = *reinterpret_cast<const u32x4*>(ab0 + ko);
    if constexpr (NA > 1) st.a[1] = *reinterpret_cast<const u32x4*>(ab1 + ko);
    if constexpr (NA > 2) {
      st.a[2] = *reinterpret_cast<const u32x4*>(ab2 + ko);
      st.a[3] = *reinterpret_cast<const u32x4*>(ab3 + ko);
    }
    if (++lkk == nk) {  // past this workgroup's last tile the clamped rows keep the loads in bounds
      lkk = 0;
      ++lj;
      enter();
    }
  };

  f32x4 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if constexpr (PIPE) {
    // Three activation images: during step t the MFMAs run on fragments read during step t - 1, the fragments of
    // step t + 1 are read from image (t + 1) % 3 (written during step t - 1, visible since the last barrier) and
    // step t + 2 is written into image (t + 2) % 3 (last read during step t - 2): the LDS read latency hides
    // under the MFMAs instead of opening every step.  Stage registers hold steps t + 2 .. t + 7 (6 in flight).
    static_assert(DEPTH == 6, "the pipelined loop is written out for 6 stage sets");
    struct Frag {
      bf16x8 a[4], b[2];
    };
    Stage<ABF> st0, st1, st2, st3, st4, st5;
    load(st0);
    load(st1);
    load(st2);
    load(st3);
    load(st4);
    load(st5);
    if (S > 0) ws::stage_store<ABF>(st0, a_img[0]);
    if (S > 1) ws::stage_store<ABF>(st1, a_img[1]);
    load(st0);  // step 6
    load(st1);  // step 7
    __syncthreads();
    auto rdfrag = [&](Frag& F, const char* At, int kk) __attribute__((always_inline)) {
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        const int rr = wm * 64 + mt * 16 + lr;
        F.a[mt] = *reinterpret_cast<const bf16x8*>(At + rr * 64 + 16 * (lk ^ swb(rr)));
      }
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        const int n = wn * 32 + nt * 16 + lr;
        F.b[nt] = *reinterpret_cast<const bf16x8*>(w_img + n * ROWB + 16 * wchunk(n, 4 * kk + lk));
      }
    };
    Frag F0, F1;
    if (S > 0) rdfrag(F0, a_img[0], 0);
    int ej = 0, ekk = 0;  // compute cursor
    // WB / RB: the images step t + 2 is written to and step t + 1 is read from (t % 3 is fixed per unrolled slot)
    auto kstep3 = [&](int t, Stage<ABF>& cur, const Frag& Fc, Frag& Fn, char* Wimg, const char* Rimg)
        __attribute__((always_inline)) {
      if (t + 2 < S) ws::stage_store<ABF>(cur, Wimg);
      load(cur);  // step t + 8 (unconditional, clamped rows)
      if (t + 1 < S) rdfrag(Fn, Rimg, ekk + 1 == nk ? 0 : ekk + 1);
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(Fc.b[nt], Fc.a[mt], acc[mt][nt], 0, 0, 0);
      if (++ekk == nk) {
        const int m0 = (lane0 + ej * lanes) * BM;
        epilogue_lds<1, ACT, RES, ROT>(p, acc, bias_s, m0, n0, wm, wn, lr, lk, ep);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        ekk = 0;
        ++ej;
      }
      __syncthreads();
    };
    for (int t = 0; t < S; t += 6) {
      kstep3(t, st2, F0, F1, a_img[2], a_img[1]);
      if (t + 1 < S) kstep3(t + 1, st3, F1, F0, a_img[0], a_img[2]);
      if (t + 2 < S) kstep3(t + 2, st4, F0, F1, a_img[1], a_img[0]);
      if (t + 3 < S) kstep3(t + 3, st5, F1, F0, a_img[2], a_img[1]);
      if (t + 4 < S) kstep3(t + 4, st0, F0, F1, a_img[0], a_img[2]);
      if (t + 5 < S) kstep3(t + 5, st1, F1, F0, a_img[1], a_img[0]);
    }
    return;
  }
  Stage<ABF> st0, st1, st2, st3, st4, st5, st6, st7;  // the unused ones are eliminated
  load(st0);
  load(st1);
  load(st2);
  load(st3);
  if constexpr (DEPTH >= 6) {
    load(st4);
    load(st5);
  }
  if constexpr (DEPTH >= 8) {
    load(st6);
    load(st7);
  }
  if (S > 0) ws::stage_store<ABF>(st0, a_img[0]);
  __syncthreads();

  int ej = 0, ekk = 0;  // compute cursor
  // one k-step: `cur` held step t (in LDS image t & 1) and is refilled with step t + DEPTH; `nxt` holds step
  // t + 1, written into the other image after this step's MFMAs
  auto kstep = [&](int t, Stage<ABF>& cur, const Stage<ABF>& nxt) __attribute__((always_inline)) {
    load(cur);  // unconditional (clamped rows): a constant count of loads in flight keeps the vmcnt waits counted
    const char* At = a_img[t & 1];
#pragma unroll
    for (int h = 0; h < KS / 32; ++h) {  // 32-deep halves of the k-step
      bf16x8 a[4], b[2];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        const int rr = wm * 64 + mt * 16 + lr;
        a[mt] = *reinterpret_cast<const bf16x8*>(At + rr * (2 * KS) + 16 * ((4 * h + lk) ^ aswz<KS>(rr)));
      }
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        const int n = wn * 32 + nt * 16 + lr;
        b[nt] = *reinterpret_cast<const bf16x8*>(w_img + n * ROWB + 16 * wchunk(n, CH * ekk + 4 * h + lk));
      }
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[nt], a[mt], acc[mt][nt], 0, 0, 0);
    }
    if (t + 1 < S) ws::stage_store<ABF>(nxt, a_img[(t + 1) & 1]);
    if (++ekk == nk) {
      const int m0 = (lane0 + ej * lanes) * BM;
      epilogue_lds<1, ACT, RES, ROT>(p, acc, bias_s, m0, n0, wm, wn, lr, lk, ep);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      ekk = 0;
      ++ej;
    }
    __syncthreads();
  };

  for (int t = 0; t < S; t += DEPTH) {
    kstep(t, st0, st1);
    if (t + 1 < S) kstep(t + 1, st1, st2);
    if (t + 2 < S) kstep(t + 2, st2, st3);
    if constexpr (DEPTH == 4) {
      if (t + 3 < S) kstep(t + 3, st3, st0);
    } else if constexpr (DEPTH == 6) {
      if (t + 3 < S) kstep(t + 3, st3, st4);
      if (t + 4 < S) kstep(t + 4, st4, st5);
      if (t + 5 < S) kstep(t + 5, st5, st0);
    } else {
      if (t + 3 < S) kstep(t + 3, st3, st4);
      if (t + 4 < S) kstep(t + 4, st4, st5);
      if (t + 5 < S) kstep(t + 5, st5, st6);
      if (t + 6 < S) kstep(t + 6, st6, st7);
      if (t + 7 < S) kstep(t + 7, st7, st0);
    }
  }
}

// The launches it takes: plain products (no k3 conv, no row-tile list), K % k-step == 0, K <= 384, float4-aligned
// C / Z / Cb rows (the LDS-staged epilogue), enough rows that every workgroup has several tiles (the slice
// load is amortised over them), and the shapes where it measured faster than gemm_p2 / gemm_wr on one box
// (profiles/r05_ws_micro.txt: bf16 A at N >= 768 4-6 %, fp32 A at N <= 768 3-10 %; equal or slower elsewhere).
inline bool ws_ok(const Params& p, bool a_bf16, bool any_shape = false) {
  const bool vec = ((p.N | p.ldc) & 3) == 0 && ((uintptr_t)p.C & 15) == 0 && ((uintptr_t)p.Z & 15) == 0 &&
                   ((uintptr_t)p.Cb & 7) == 0;
  return vec && !p.mtiles && p.K % (a_bf16 ? ws::WsCfg<true>::KS : ws::WsCfg<false>::KS) == 0 &&
         p.K <= ws::KMAX && p.M >= 32768 && ((p.N + ws::BN - 1) / ws::BN) <= 64 &&
         (any_shape || (a_bf16 ? p.N >= 768 : p.N <= 768));
}

template <bool ABF, int ACT, bool RES, bool ROT>
void launch_ws(const Params& p, hipStream_t s) {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    cus = std::max(1, cus);
  }
  const int nS = (p.N + ws::BN - 1) / ws::BN;
  const int nM = (p.M + BM - 1) / BM;
  const int lanes = std::max(1, std::min(cus / nS, nM));  // row lanes per slice: one resident workgroup per CU
  gemm_ws_kernel<ABF, ACT, RES, ROT><<<nS * lanes, ws::WTHR, 0, s>>>(p, nS, lanes);
}

template <bool ABF>
void launch_ws_act(const Params& p, hipStream_t s) {
  switch (p.act) {
    case ACT_GELU: launch_ws<ABF, ACT_GELU, false, false>(p, s); break;
    case ACT_SILU: launch_ws<ABF, ACT_SILU, false, false>(p, s); break;
    case ACT_SIGMOID: launch_ws<ABF, ACT_SIGMOID, false, false>(p, s); break;
    case ACT_RELU: launch_ws<ABF, ACT_RELU, false, false>(p, s); break;
    default: launch_ws<ABF, ACT_NONE, false, false>(p, s); break;
  }
}

}  // namespace wn
}  // namespace asrx

#ifndef ASRX_WS_INSTANTIATE
#define ASRX_WS_DECL_ACT(ABF) extern template void asrx::wn::launch_ws_act<ABF>(const asrx::wn::Params&, hipStream_t);
#define ASRX_WS_DECL(ABF, RES, ROT) \
  extern template void asrx::wn::launch_ws<ABF, asrx::ACT_NONE, RES, ROT>(const asrx::wn::Params&, hipStream_t);
ASRX_WS_DECL_ACT(true)
ASRX_WS_DECL_ACT(false)
ASRX_WS_DECL(false, true, false)
ASRX_WS_DECL(true, false, true)
ASRX_WS_DECL(false, false, true)
#else
#define ASRX_WS_DECL_ACT(ABF) template void asrx::wn::launch_ws_act<ABF>(const asrx::wn::Params&, hipStream_t);
#define ASRX_WS_DECL(ABF, RES, ROT) \
  template void asrx::wn::launch_ws<ABF, asrx::ACT_NONE, RES, ROT>(const asrx::wn::Params&, hipStream_t);
#endif
