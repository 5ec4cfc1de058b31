// Entry points of the wide GEMM (kernel and design: gemm_wr.h), the bulk weight conversion to
// bf16 and the MSheath row-tile lists.
#include "gemm_wr.h"
#include "gemm_p2.h"
#include "gemm_ws.h"
#include <string>

// Which wide-GEMM kernel runs the plain / residual products that gemm_p2_kernel covers (asrx_set_gemm_variant):
// 1 gemm_p2_kernel (two workgroups per CU) for tile widths 3 and 2, 2 also for width 1 (the 128-column
// tiles: gemm_p2's NJ = 2 tile is 128 x 128), 0 gemm_wr_kernel -- A/B measurements and the tests that compare them;
// + 4: the weight-stationary gemm_ws_kernel first for the launches it takes (ws_ok: K <= 384, >= 32768 rows, the
// shapes where it measured faster).
// + 16: the AbbyNormal router at d = 64 on gemm_wr_kernel instead of router64_kernel (A/B, tests).
// Default 5.
static int g_wide_variant = 5;
static bool ws_on() { return (g_wide_variant & 4) != 0; }
static bool ws_any() { return (g_wide_variant & 8) != 0; }  // + 8: every shape gemm_ws can run (tests)
extern "C" int asrx_set_gemm_variant(int v) {
  const int old = g_wide_variant;
  g_wide_variant = v;
  return old;
}
// gemm_p2_kernel takes: no k3 conv, float4-aligned C / Z (LDS-staged epilogue), tile widths 3 and 2
// (measured, profiles/r05_p2_micro.txt: bf16-stored A 5-10 % faster at every shape; fp32 A faster up to 96000
// rows but 9-18 % slower at 192064 rows, where its four A loads per thread and k-step cost more than the
// overlap gains -- so fp32 A at >= 131072 rows stays on gemm_wr_kernel)
static bool p2_ok(const asrx::wn::Params& p, int conv, int nj, int a_bf16) {
  if (!a_bf16 && p.M >= 131072) return false;
  const bool vec = ((p.N | p.ldc) & 3) == 0 && ((uintptr_t)p.C & 15) == 0 && ((uintptr_t)p.Z & 15) == 0 &&
                   ((uintptr_t)p.Cb & 7) == 0;
  return (g_wide_variant & 3) >= 1 && !conv && (nj == 3 || nj == 2 || (nj == 1 && (g_wide_variant & 3) == 2)) &&
         vec && p.K >= 64;
}

namespace asrx {
namespace wn {

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

// Every GEMM weight of a step converted in ONE launch (asrx/gemm.py bulk plan): entry e converts
// src (rows x cols, row stride ld) to bf16 dst (N x K contiguous; trans as weight_to_bf16).  A
// workgroup walks one entry's elements; grid (ceil(max elements / 4096), entries).
struct WConv {
  const float* src;
  unsigned short* dst;
  int64_t ld;
  int rows, cols, trans, pad;
};

namespace asrx {
__global__ __launch_bounds__(256) void weights_to_bf16_kernel(const WConv* __restrict__ tab) {
  const WConv e = tab[blockIdx.y];
  const int64_t total = (int64_t)e.rows * e.cols;
  const int64_t i0 = (int64_t)blockIdx.x * 4096;
  if (i0 >= total) return;
  const int64_t i1 = min<int64_t>(total, i0 + 4096);
  for (int64_t i = i0 + threadIdx.x; i < i1; i += 256) {
    int64_t r, c, o;
    if (!e.trans) {
      r = i / e.cols;
      c = i % e.cols;
      o = r * e.cols + c;
    } else {
      c = i / e.rows;
      r = i % e.rows;
      o = c * e.rows + r;
    }
    e.dst[o] = __builtin_bit_cast(unsigned short, (__bf16)e.src[r * e.ld + c]);
  }
}
}  // namespace asrx

extern "C" int64_t asrx_wconv_entry_bytes(void) { return (int64_t)sizeof(WConv); }

// tab: n device-resident WConv entries (asrx_wconv_entry_bytes() each); max_elems: the largest
// rows * cols among them.
extern "C" int asrx_weights_to_bf16(const void* tab, int64_t n, int64_t max_elems, hipStream_t stream) {
  if (n == 0) return 0;
  ASRX_REQUIRE(n < 65536, "asrx_weights_to_bf16: too many entries");
  dim3 grid((unsigned)((max_elems + 4095) / 4096), (unsigned)n);
  weights_to_bf16_kernel<<<grid, 256, 0, stream>>>((const WConv*)tab);
  ASRX_LAUNCHED("asrx_weights_to_bf16");
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
               (int)(convF > 0 ? convF : 1), (int)(convC > 0 ? convC : 1), alpha, beta, act, nullptr, nullptr};
  if (nj == 3) conv ? wn::launch_wr<3, true>(p, stream) : wn::launch_wr<3, false>(p, stream);
  else if (nj == 2) conv ? wn::launch_wr<2, true>(p, stream) : wn::launch_wr<2, false>(p, stream);
  else conv ? wn::launch_wr<1, true>(p, stream) : wn::launch_wr<1, false>(p, stream);
  ASRX_LAUNCHED("asrx_gemm_wn");
}

// asrx_gemm_wn with storage types: A fp32 (a_bf16 = 0) or bf16 (1); C fp32 (c_bf16 = 0) or bf16 (1,
// beta = 0; Z, when given, stays fp32); optionally restricted to the device tile list mtiles (as
// asrx_gemm_wn_rows, non-conv only).
extern "C" int asrx_gemm_wn_ex(const void* A, int a_bf16, int64_t lda, int conv, int64_t convF, int64_t convC,
                               const unsigned short* W, int64_t ldw, void* C, int c_bf16, int64_t ldc,
                               const float* bias, float* Z, int64_t M, int64_t N, int64_t K, float alpha, float beta,
                               int act, int nj, const int* mtiles, const int* n_mtiles, hipStream_t stream) {
  ASRX_REQUIRE(M > 0 && N > 0 && K > 0, "asrx_gemm_wn_ex: empty problem");
  ASRX_REQUIRE(((uintptr_t)A & 15) == 0 && ((uintptr_t)W & 15) == 0, "asrx_gemm_wn_ex: A/W must be 16-byte aligned");
  ASRX_REQUIRE(K % 8 == 0 && lda % (a_bf16 ? 8 : 4) == 0 && ldw % 8 == 0,
               "asrx_gemm_wn_ex: K%%8, lda%%4 (fp32) / lda%%8 (bf16), ldw%%8 required");
  ASRX_REQUIRE(M * lda < (1LL << 31) && N * ldw < (1LL << 31), "asrx_gemm_wn_ex: operand spans >= 2^31 elements");
  ASRX_REQUIRE(!conv || (convF > 0 && convC % (a_bf16 ? 8 : 4) == 0), "asrx_gemm_wn_ex: conv needs F > 0 and C %% 4 (8 for bf16)");
  ASRX_REQUIRE(!c_bf16 || beta == 0.f, "asrx_gemm_wn_ex: a bf16 output takes beta = 0");
  ASRX_REQUIRE(!(conv && mtiles), "asrx_gemm_wn_ex: tile lists are for plain GEMMs");
  wn::Params p{(const float*)A, (int)lda, W, (int)ldw, c_bf16 ? nullptr : (float*)C, (int)ldc, bias, Z, (int)M,
               (int)N, (int)K, (int)(convF > 0 ? convF : 1), (int)(convC > 0 ? convC : 1), alpha, beta, act,
               nullptr, nullptr, mtiles, n_mtiles, c_bf16 ? (unsigned short*)C : nullptr};
#define ASRX_WN_EX(NJV)                                                                              \
  if (a_bf16) conv ? wn::launch_wr<NJV, true, false, true>(p, stream) : wn::launch_wr<NJV, false, false, true>(p, stream); \
  else conv ? wn::launch_wr<NJV, true>(p, stream) : wn::launch_wr<NJV, false>(p, stream);
  if (ws_on() && !conv && wn::ws_ok(p, a_bf16, ws_any())) {
    a_bf16 ? wn::launch_ws_act<true>(p, stream) : wn::launch_ws_act<false>(p, stream);
  } else if (p2_ok(p, conv, nj, a_bf16)) {
    if (nj == 3) a_bf16 ? wn::launch_p2_act<3, true, false>(p, stream) : wn::launch_p2_act<3, false, false>(p, stream);
    else a_bf16 ? wn::launch_p2_act<2, true, false>(p, stream) : wn::launch_p2_act<2, false, false>(p, stream);  // nj 2 / 1
  } else if (nj == 3) { ASRX_WN_EX(3) }
  else if (nj == 2) { ASRX_WN_EX(2) }
  else { ASRX_WN_EX(1) }
#undef ASRX_WN_EX
  ASRX_LAUNCHED("asrx_gemm_wn_ex");
}

// Tied logits with the cross entropy's statistics fused (model.py:629 logits = x @ token.weight^T,
// model.py:670 F.cross_entropy): Zb (M x N, ldc) = bf16(A W^T) for a bf16-stored A, and per row and
// 128*nj-column tile the (max, sum exp(z - max)) of the tile's bf16 logits in part[row * nparts + tile]
// (float2, nparts = ceil(N / (128 nj))) -- asrx_ce_part_fwd turns them into the loss without re-reading
// the logits.
extern "C" int asrx_gemm_wn_ce(const void* A, int64_t lda, const unsigned short* W, int64_t ldw, unsigned short* Zb,
                               int64_t ldc, float* part, int64_t M, int64_t N, int64_t K, int nj, hipStream_t stream) {
  ASRX_REQUIRE(M > 0 && N > 0 && K > 0, "asrx_gemm_wn_ce: empty problem");
  ASRX_REQUIRE(((uintptr_t)A & 15) == 0 && ((uintptr_t)W & 15) == 0 && ((uintptr_t)Zb & 7) == 0 &&
                   ((uintptr_t)part & 7) == 0,
               "asrx_gemm_wn_ce: A/W 16-byte, Zb/part 8-byte aligned");
  ASRX_REQUIRE(K % 8 == 0 && lda % 8 == 0 && ldw % 8 == 0 && N % 4 == 0 && ldc % 4 == 0,
               "asrx_gemm_wn_ce: K, lda, ldw %% 8 and N, ldc %% 4 required");
  ASRX_REQUIRE(M * lda < (1LL << 31) && N * ldw < (1LL << 31), "asrx_gemm_wn_ce: operand spans >= 2^31 elements");
  ASRX_REQUIRE(nj >= 1 && nj <= 3, "asrx_gemm_wn_ce: nj in 1..3");
  wn::Params p{(const float*)A, (int)lda, W, (int)ldw, nullptr, (int)ldc, nullptr, nullptr, (int)M, (int)N, (int)K,
               1, 1, 1.f, 0.f, ACT_NONE, nullptr, nullptr, nullptr, nullptr, Zb, (float2*)part,
               (int)((N + 128 * nj - 1) / (128 * nj))};
  if (nj == 3) wn::launch_wr<3, false, false, true, true>(p, stream);
  else if (nj == 2) wn::launch_wr<2, false, false, true, true>(p, stream);
  else wn::launch_wr<1, false, false, true, true>(p, stream);
  ASRX_LAUNCHED("asrx_gemm_wn_ce");
}

// As asrx_gemm_wn_ce with the logits stored fp32 (Zf) and the statistics taken of the fp32 values.
extern "C" int asrx_gemm_wn_ce_f32(const void* A, int64_t lda, const unsigned short* W, int64_t ldw, float* Zf,
                               int64_t ldc, float* part, int64_t M, int64_t N, int64_t K, int nj, hipStream_t stream) {
  ASRX_REQUIRE(M > 0 && N > 0 && K > 0, "asrx_gemm_wn_ce_f32: empty problem");
  ASRX_REQUIRE(((uintptr_t)A & 15) == 0 && ((uintptr_t)W & 15) == 0 && ((uintptr_t)Zf & 15) == 0 &&
                   ((uintptr_t)part & 7) == 0,
               "asrx_gemm_wn_ce_f32: A/W 16-byte, Zf 16-byte, part 8-byte aligned");
  ASRX_REQUIRE(K % 8 == 0 && lda % 8 == 0 && ldw % 8 == 0 && N % 4 == 0 && ldc % 4 == 0,
               "asrx_gemm_wn_ce_f32: K, lda, ldw %% 8 and N, ldc %% 4 required");
  ASRX_REQUIRE(M * lda < (1LL << 31) && N * ldw < (1LL << 31), "asrx_gemm_wn_ce_f32: operand spans >= 2^31 elements");
  ASRX_REQUIRE(nj >= 1 && nj <= 3, "asrx_gemm_wn_ce_f32: nj in 1..3");
  wn::Params p{(const float*)A, (int)lda, W, (int)ldw, Zf, (int)ldc, nullptr, nullptr, (int)M, (int)N, (int)K,
               1, 1, 1.f, 0.f, ACT_NONE, nullptr, nullptr, nullptr, nullptr, nullptr, (float2*)part,
               (int)((N + 128 * nj - 1) / (128 * nj))};
  if (nj == 3) wn::launch_wr<3, false, false, true, true>(p, stream);
  else if (nj == 2) wn::launch_wr<2, false, false, true, true>(p, stream);
  else wn::launch_wr<1, false, false, true, true>(p, stream);
  ASRX_LAUNCHED("asrx_gemm_wn_ce_f32");
}

// Out projection with its residual add (model.py:578-580 x = x + attn(...).out): C = R + A W^T + bias, A, C
// and R fp32 (R may not alias C), 16-byte aligned rows; nj 1 or 3 (the residual epilogue is compiled into
// dedicated instantiations only, so the other GEMMs keep their register budget).
extern "C" int asrx_gemm_wn_res(const float* A, int64_t lda, const unsigned short* W, int64_t ldw, float* C, int64_t ldc,
                                const float* bias, const float* R, int64_t ldr, int64_t M, int64_t N, int64_t K, int nj,
                                hipStream_t stream) {
  ASRX_REQUIRE(M > 0 && N > 0 && K > 0, "asrx_gemm_wn_res: empty problem");
  ASRX_REQUIRE(((uintptr_t)A & 15) == 0 && ((uintptr_t)W & 15) == 0 && ((uintptr_t)C & 15) == 0 &&
                   ((uintptr_t)R & 15) == 0,
               "asrx_gemm_wn_res: A/W/C/R must be 16-byte aligned");
  ASRX_REQUIRE(K % 8 == 0 && lda % 4 == 0 && ldw % 8 == 0 && N % 4 == 0 && ldc % 4 == 0 && ldr % 4 == 0,
               "asrx_gemm_wn_res: K, ldw %% 8; lda, N, ldc, ldr %% 4");
  ASRX_REQUIRE(M * lda < (1LL << 31) && N * ldw < (1LL << 31), "asrx_gemm_wn_res: operand spans >= 2^31 elements");
  ASRX_REQUIRE(R && R != C, "asrx_gemm_wn_res: a residual input distinct from C is required");
  ASRX_REQUIRE(nj == 1 || nj == 3, "asrx_gemm_wn_res: nj 1 or 3");
  wn::Params p{A, (int)lda, W, (int)ldw, C, (int)ldc, bias, nullptr, (int)M, (int)N, (int)K, 1, 1, 1.f, 0.f,
               ACT_NONE, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 0, R, (int)ldr};
  if (ws_on() && wn::ws_ok(p, false, ws_any())) wn::launch_ws<false, ACT_NONE, true, false>(p, stream);
  else if (nj == 3 && p2_ok(p, 0, nj, 0)) wn::launch_p2_act<3, false, true>(p, stream);
  else if (nj == 3) wn::launch_wr<3, false, false, false, false, true>(p, stream);
  else wn::launch_wr<1, false, false, false, false, true>(p, stream);
  ASRX_LAUNCHED("asrx_gemm_wn_res");
}

// q / k projection with rotary fused (model.py:242-245 then 198-214, with the hd^-0.25 scale of model.py:303-304):
// C = rot(A W^T + bias), i.e. each head's pairs (2j, 2j+1) of the product times polar(scale * m[row], angle(row %
// L, j)) from the (cos, sin) table tab (positions >= L, hd / 2) float2 -- asrx_rotary_fwd2's arithmetic, so C is
// bit-identical to the GEMM followed by that pass; Z (nullable) receives the unrotated product (what the rotary
// backward reads).  A fp32 (a_bf16 = 0) or bf16 (1); C, Z fp32, 16-byte aligned rows; nj 1 or 3.
extern "C" int asrx_gemm_wn_rot(const void* A, int a_bf16, int64_t lda, const unsigned short* W, int64_t ldw,
                                float* C, float* Z, int64_t ldc, const float* bias, const float* m, const float* tab,
                                int64_t L, int64_t hd, float scale, int64_t M, int64_t N, int64_t K, int nj,
                                hipStream_t stream) {
  ASRX_REQUIRE(M > 0 && N > 0 && K > 0 && L > 0, "asrx_gemm_wn_rot: empty problem");
  ASRX_REQUIRE(((uintptr_t)A & 15) == 0 && ((uintptr_t)W & 15) == 0 && ((uintptr_t)C & 15) == 0 &&
                   ((uintptr_t)Z & 15) == 0 && ((uintptr_t)tab & 15) == 0,
               "asrx_gemm_wn_rot: A/W/C/Z/tab must be 16-byte aligned");
  ASRX_REQUIRE(K % 8 == 0 && lda % (a_bf16 ? 8 : 4) == 0 && ldw % 8 == 0 && N % 4 == 0 && ldc % 4 == 0,
               "asrx_gemm_wn_rot: K, ldw %% 8; lda %% 4 (8 bf16); N, ldc %% 4");
  ASRX_REQUIRE(hd >= 4 && hd % 4 == 0 && N % hd == 0, "asrx_gemm_wn_rot: head dim %% 4, N %% hd");
  ASRX_REQUIRE(M * lda < (1LL << 31) && N * ldw < (1LL << 31), "asrx_gemm_wn_rot: operand spans >= 2^31 elements");
  ASRX_REQUIRE(m && tab, "asrx_gemm_wn_rot: row norms and angle table required");
  ASRX_REQUIRE(nj == 1 || nj == 3, "asrx_gemm_wn_rot: nj 1 or 3");
  wn::Params p{(const float*)A, (int)lda, W, (int)ldw, C, (int)ldc, bias, Z, (int)M, (int)N, (int)K, 1, 1, 1.f, 0.f,
               ACT_NONE};
  p.rot_m = m;
  p.rot_tab = reinterpret_cast<const float2*>(tab);
  p.rot_L = (int)L;
  p.rot_half = (int)(hd / 2);
  p.rot_scale = scale;
  // the same kernel choice as asrx_gemm_wn_ex: gemm_ws where it takes the shape, gemm_p2 where p2_ok (so fp32 A at
  // >= 131072 rows and gemm variant 0 stay on gemm_wr), gemm_wr otherwise -- every form bit-identical
  if (ws_on() && wn::ws_ok(p, a_bf16, ws_any())) a_bf16 ? wn::launch_ws<true, ACT_NONE, false, true>(p, stream)
                                      : wn::launch_ws<false, ACT_NONE, false, true>(p, stream);
  else if (nj == 3 && p2_ok(p, 0, nj, a_bf16)) a_bf16 ? wn::launch_p2<3, true, ACT_NONE, false, true>(p, stream)
                                                   : wn::launch_p2<3, false, ACT_NONE, false, true>(p, stream);
  else if (nj == 3) a_bf16 ? wn::launch_wr<3, false, false, true, false, false, false, true>(p, stream)
                           : wn::launch_wr<3, false, false, false, false, false, false, true>(p, stream);
  else a_bf16 ? wn::launch_wr<1, false, false, true, false, false, false, true>(p, stream)
              : wn::launch_wr<1, false, false, false, false, false, false, true>(p, stream);
  ASRX_LAUNCHED("asrx_gemm_wn_rot");
}

// Backward of y = act(A W^T + bias) (act gelu / silu / sigmoid) without a stored pre-activation: the GEMM
// recomputes z = A W^T + bias with the forward's tile width (nj 3 only: the instantiation the forward's
// shapes use) and writes gz = bf16(G * act'(z)) (M x N, ldc) from the output gradient G (fp32, ldg), adding
// the column sums of gz into db when non-null.  A fp32 (a_bf16 = 0) or bf16 (1).
extern "C" int asrx_gemm_wn_gact(const void* A, int a_bf16, int64_t lda, const unsigned short* W, int64_t ldw,
                                 const float* bias, const float* G, int64_t ldg, unsigned short* gz, int64_t ldc,
                                 float* db, int64_t M, int64_t N, int64_t K, int act, int nj, hipStream_t stream) {
  ASRX_REQUIRE(M > 0 && N > 0 && K > 0, "asrx_gemm_wn_gact: empty problem");
  ASRX_REQUIRE(nj == 3, "asrx_gemm_wn_gact: nj 3 only");
  ASRX_REQUIRE(act == ACT_GELU || act == ACT_SILU || act == ACT_SIGMOID, "asrx_gemm_wn_gact: gelu/silu/sigmoid only");
  ASRX_REQUIRE(((uintptr_t)A & 15) == 0 && ((uintptr_t)W & 15) == 0 && ((uintptr_t)G & 15) == 0 &&
                   ((uintptr_t)gz & 7) == 0,
               "asrx_gemm_wn_gact: A/W/G 16-byte, gz 8-byte aligned");
  ASRX_REQUIRE(K % 8 == 0 && lda % (a_bf16 ? 8 : 4) == 0 && ldw % 8 == 0 && N % 4 == 0 && ldc % 4 == 0 &&
                   ldg % 4 == 0,
               "asrx_gemm_wn_gact: K, ldw %% 8; lda %% 4 (8 bf16); N, ldc, ldg %% 4");
  ASRX_REQUIRE(M * lda < (1LL << 31) && N * ldw < (1LL << 31), "asrx_gemm_wn_gact: operand spans >= 2^31 elements");
  wn::Params p{(const float*)A, (int)lda, W, (int)ldw, nullptr, (int)ldc, bias, nullptr, (int)M, (int)N, (int)K, 1,
               1, 1.f, 0.f, act, nullptr, nullptr, nullptr, nullptr, gz, nullptr, 0, nullptr, 0, G, (int)ldg, db};
  if (a_bf16) wn::launch_wr<3, false, false, true, false, false, true>(p, stream);
  else wn::launch_wr<3, false, false, false, false, false, true>(p, stream);
  ASRX_LAUNCHED("asrx_gemm_wn_gact");
}

// asrx_gemm_wn restricted to the BM-row tiles listed in mtiles (n_mtiles entries, both on the device,
// from asrx_row_tiles); rows of other tiles are not written.
extern "C" int asrx_gemm_wn_rows(const float* A, int64_t lda, const unsigned short* W, int64_t ldw, float* C,
                                 int64_t ldc, const float* bias, float* Z, int64_t M, int64_t N, int64_t K,
                                 float alpha, float beta, int act, int nj, const int* mtiles, const int* n_mtiles,
                                 hipStream_t stream) {
  ASRX_REQUIRE(M > 0 && N > 0 && K > 0, "asrx_gemm_wn_rows: empty problem");
  ASRX_REQUIRE(((uintptr_t)A & 15) == 0 && ((uintptr_t)W & 15) == 0, "asrx_gemm_wn_rows: A/W must be 16-byte aligned");
  ASRX_REQUIRE(K % 8 == 0 && lda % 4 == 0 && ldw % 8 == 0, "asrx_gemm_wn_rows: K%%8, lda%%4, ldw%%8 required");
  ASRX_REQUIRE(M * lda < (1LL << 31) && N * ldw < (1LL << 31), "asrx_gemm_wn_rows: operand spans >= 2^31 elements");
  ASRX_REQUIRE(mtiles && n_mtiles, "asrx_gemm_wn_rows: tile list required");
  wn::Params p{A, (int)lda, W, (int)ldw, C, (int)ldc, bias, Z, (int)M, (int)N, (int)K, 1, 1, alpha, beta, act,
               nullptr, nullptr, mtiles, n_mtiles};
  if (nj == 3) wn::launch_wr<3, false>(p, stream);
  else if (nj == 2) wn::launch_wr<2, false>(p, stream);
  else wn::launch_wr<1, false>(p, stream);
  ASRX_LAUNCHED("asrx_gemm_wn_rows");
}

// The BM-row tiles of an M-row activation whose rows r belong to a sample b = r / L that is at MSheath
// layer `layer` (next_i[b] == layer): mtiles[0 .. *n_mtiles) in increasing order.  One workgroup.
namespace asrx {
__global__ __launch_bounds__(1024) void row_tiles_kernel(const float* __restrict__ next_i, int layer, int64_t L,
                                                         int64_t M, int* __restrict__ mtiles, int* __restrict__ n_out) {
  __shared__ int wsum[16];
  __shared__ int base;
  const int nm = (int)((M + wn::BM - 1) / wn::BM);
  if (threadIdx.x == 0) base = 0;
  __syncthreads();
  for (int t0 = 0; t0 < nm; t0 += 1024) {
    const int t = t0 + threadIdx.x;
    int act = 0;
    if (t < nm) {
      const int64_t r0 = (int64_t)t * wn::BM, r1 = min<int64_t>(r0 + wn::BM, M) - 1;
      for (int64_t b = r0 / L; b <= r1 / L && !act; ++b) act = next_i[b] == (float)layer;
    }
    // block exclusive scan of act
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int v = act;
    for (int o = 1; o < 64; o <<= 1) {
      const int u = __shfl_up(v, o);
      if (lane >= o) v += u;
    }
    if (lane == 63) wsum[w] = v;
    __syncthreads();
    int off = base;
    for (int k = 0; k < w; ++k) off += wsum[k];
    if (act) mtiles[off + v - 1] = t;
    __syncthreads();
    if (threadIdx.x == 0) {
      int tot = 0;
      for (int k = 0; k < 16; ++k) tot += wsum[k];
      base += tot;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) n_out[0] = base;
}
}  // namespace asrx

extern "C" int64_t asrx_row_tiles_max(int64_t M) { return (M + wn::BM - 1) / wn::BM; }

extern "C" int asrx_row_tiles(const float* next_i, int64_t layer, int64_t L, int64_t M, int* mtiles, int* n_mtiles,
                              hipStream_t stream) {
  ASRX_REQUIRE(L > 0 && M > 0, "asrx_row_tiles: empty");
  row_tiles_kernel<<<1, 1024, 0, stream>>>(next_i, (int)layer, L, M, mtiles, n_mtiles);
  ASRX_LAUNCHED("asrx_row_tiles");
}

// AbbyNormal router (essentials.py:155-161) in one pass: h_pre = A W1^T + b1 (kept in hpre when
// non-null, for the backward) and logits = SiLU(h_pre) W2^T (M x 3, without b2), for d <= 384.
namespace asrx {
namespace wn {

// AbbyNormal router at d = 64 (the per-head norms of model.py:303-304's q / k; essentials.py:155-161):
// logits = SiLU(x W1^T + b1) W2^T over 1.15 M rows of 64 features at the tiny config.  gemm_wr_kernel ran it on
// a 128-column tile with half the columns empty and two k-steps per 128-row tile (prologue and epilogue bound,
// 1.8 TB/s).  Here a wave streams 16-row groups straight from global memory into MFMA fragments: W1 (64 x 64 bf16)
// sits in 32 registers as the row operand for the whole launch, each group is 8 v_mfma_f32_16x16x32_bf16, and the
// epilogue reduces in registers.  The fragment layout, k order, epilogue expressions and the logit sum order
// (each 32-column group over its lane's columns, xor-16 / xor-32 partners, then the groups in order, plus the
// two empty groups' +0.0) are gemm_wr_kernel's (epilogue_router), so h_pre and the logits are bit-identical.
// The next group's x is in flight while a group is computed (two named register sets, loop unrolled by two).
struct R64X {
  float4 v[4];  // lane (row l & 15): k 8 (l >> 4) .. + 7 of k-halves 0 and 1
};
__global__ __launch_bounds__(256) void router64_kernel(Params p) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int lr = lane & 15, lk = lane >> 4;
  bf16x8 wf[4][2];
#pragma unroll
  for (int nb = 0; nb < 4; ++nb)
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
      wf[nb][kb] = *reinterpret_cast<const bf16x8*>(p.W + (int64_t)(16 * nb + lr) * p.ldw + 32 * kb + 8 * lk);
  float bv[4][4], w2v[3][4][4];
#pragma unroll
  for (int nb = 0; nb < 4; ++nb)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int n = 16 * nb + 4 * lk + q;
      bv[nb][q] = p.bias ? p.bias[n] : 0.f;
#pragma unroll
      for (int k = 0; k < 3; ++k) w2v[k][nb][q] = p.W2[k * 64 + n];
    }
  const int64_t ngroups = ((int64_t)p.M + 15) / 16;
  const int64_t step = (int64_t)gridDim.x * 4;
  const float* A = reinterpret_cast<const float*>(p.A);
  auto fetch = [&](int64_t g, R64X& x) __attribute__((always_inline)) {
    const int64_t row = min(g * 16 + lr, (int64_t)p.M - 1);  // past the end: a valid row, results dropped
    const float* src = A + row * p.lda + 8 * lk;
    x.v[0] = *reinterpret_cast<const float4*>(src);
    x.v[1] = *reinterpret_cast<const float4*>(src + 4);
    x.v[2] = *reinterpret_cast<const float4*>(src + 32);
    x.v[3] = *reinterpret_cast<const float4*>(src + 36);
  };
  auto group = [&](int64_t g, const R64X& x) __attribute__((always_inline)) {
    bf16x8 xf[2];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      const float4 a = x.v[2 * kb], b = x.v[2 * kb + 1];
      xf[kb] = bf16x8{(__bf16)a.x, (__bf16)a.y, (__bf16)a.z, (__bf16)a.w,
                      (__bf16)b.x, (__bf16)b.y, (__bf16)b.z, (__bf16)b.w};
    }
    f32x4 acc[4];
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) acc[nb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) acc[nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[nb][kb], xf[kb], acc[nb], 0, 0, 0);
    const int64_t row = g * 16 + lr;
    float s[2][3];
#pragma unroll
    for (int grp = 0; grp < 2; ++grp) {
      float s0 = 0.f, s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        const int nb = 2 * grp + nt;
        const float v[4] = {p.alpha * acc[nb][0] + bv[nb][0], p.alpha * acc[nb][1] + bv[nb][1],
                            p.alpha * acc[nb][2] + bv[nb][2], p.alpha * acc[nb][3] + bv[nb][3]};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float h = silu_f(v[q]);
          s0 += h * w2v[0][nb][q];
          s1 += h * w2v[1][nb][q];
          s2 += h * w2v[2][nb][q];
        }
        if (p.C && row < p.M)
          *reinterpret_cast<float4*>(p.C + row * p.ldc + 16 * nb + 4 * lk) = make_float4(v[0], v[1], v[2], v[3]);
      }
      s0 += __shfl_xor(s0, 16); s1 += __shfl_xor(s1, 16); s2 += __shfl_xor(s2, 16);
      s0 += __shfl_xor(s0, 32); s1 += __shfl_xor(s1, 32); s2 += __shfl_xor(s2, 32);
      s[grp][0] = s0; s[grp][1] = s1; s[grp][2] = s2;
    }
    if (lk == 0 && row < p.M) {
#pragma unroll
      for (int k = 0; k < 3; ++k) p.R[row * 3 + k] = s[0][k] + s[1][k] + 0.f + 0.f;
    }
  };
  int64_t g = (int64_t)blockIdx.x * 4 + wid;
  if (g >= ngroups) return;
  R64X xa, xb;
  fetch(g, xa);
  fetch(g + step, xb);
  for (;; g += 2 * step) {
    {
      const R64X x = xa;
      fetch(g + 2 * step, xa);
      group(g, x);
    }
    if (g + step >= ngroups) break;
    {
      const R64X x = xb;
      fetch(g + 3 * step, xb);
      group(g + step, x);
    }
    if (g + 2 * step >= ngroups) break;
  }
}

}  // namespace wn
}  // namespace asrx

extern "C" int asrx_gemm_wn_router(const float* A, int64_t lda, const unsigned short* W1, int64_t ldw,
                                   const float* b1, const float* W2, float* hpre, int64_t ldc, float* logits,
                                   int64_t M, int64_t N, int64_t K, hipStream_t stream) {
  ASRX_REQUIRE(M > 0 && N > 0 && K > 0, "asrx_gemm_wn_router: empty problem");
  ASRX_REQUIRE(N <= 384, "asrx_gemm_wn_router: N must be <= 384 (one tile column)");
  ASRX_REQUIRE(((uintptr_t)A & 15) == 0 && ((uintptr_t)W1 & 15) == 0, "asrx_gemm_wn_router: A/W must be 16-byte aligned");
  ASRX_REQUIRE(K % 8 == 0 && lda % 4 == 0 && ldw % 8 == 0, "asrx_gemm_wn_router: K%%8, lda%%4, ldw%%8 required");
  ASRX_REQUIRE(M * lda < (1LL << 31), "asrx_gemm_wn_router: operand spans >= 2^31 elements");
  wn::Params p{A, (int)lda, W1, (int)ldw, hpre, (int)ldc, b1, nullptr, (int)M, (int)N, (int)K, 1, 1, 1.f, 0.f,
               ACT_NONE, W2, logits};
  const bool r64 = N == 64 && K == 64 && W2 && (g_wide_variant & 16) == 0 && ldw % 8 == 0 &&
                   (!hpre || (ldc % 4 == 0 && ((uintptr_t)hpre & 15) == 0));
  if (r64) {
    static int cus = 0;
    if (!cus) {
      int dev = 0;
      (void)hipGetDevice(&dev);
      (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
      cus = std::max(1, cus);
    }
    const int64_t groups = (M + 15) / 16;
    const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>((groups + 3) / 4, (int64_t)cus * 8));
    wn::router64_kernel<<<grid, 256, 0, stream>>>(p);
  } else if (N <= 128) wn::launch_wr<1, false, true>(p, stream);
  else if (N <= 256) wn::launch_wr<2, false, true>(p, stream);
  else wn::launch_wr<3, false, true>(p, stream);
  ASRX_LAUNCHED("asrx_gemm_wn_router");
}
