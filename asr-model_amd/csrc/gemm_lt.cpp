// Plain activation x weight products on the vendor GEMM library (hipBLASLt): Y = alpha A W^T (+ bias) (+ beta Y) for
// a bf16-stored activation A (M x K) and a bf16 weight copy W (N x K), Y fp32 or bf16 -- no other epilogue.  Where
// the library's tuned kernels beat the hand-written wide GEMM (csrc/gemm_wr.h, gemm_p2.h, gemm_ws.h) is measured,
// not assumed: at K >= 768 with >= 16384 rows it runs 25-40 % faster (profiles/r06_blaslt_vs_wide.txt: e.g. 48016 x
// 768 x 2304 147 vs 196 us, 192064 x 384 x 1536 235 vs 332 us), at K = 384 the wide GEMM stays ahead (114 vs 127 us
// at 192064 x 384 x 384), and every fused epilogue (activations, saved pre-activation, residual, rotary, router,
// tied logits + CE statistics, row-tile lists, k3 convs, fp32 activations converted on the fly) stays on the
// hand-written kernels.  asrx/gemm.py decides per launch (LIBRARY_GEMM).
//
// Row-major Y (M x N) is column-major Y^T (N x M) = W A^T: the library's A operand is the weight (column-major K x N,
// transposed), its B operand the activation (column-major K x M), so the bias broadcasts over D's columns as the
// library's bias epilogue does.  One handle per device; per (device, stream) a 64 MB workspace allocated on first use
// (relaxed capture mode, as the small-linear partials); per problem shape the descriptors and the heuristic's first
// algorithm are cached.
#include "common.h"

#include <hipblaslt/hipblaslt.h>

#include <map>
#include <mutex>
#include <tuple>

namespace {

constexpr size_t LT_WS_BYTES = (size_t)64 << 20;

struct LtPlan {
  hipblasLtMatmulDesc_t op = nullptr;
  hipblasLtMatrixLayout_t la = nullptr, lb = nullptr, lc = nullptr;
  hipblasLtMatmulAlgo_t algo;
  size_t ws = 0;
};

std::mutex g_mu;
std::map<int, hipblasLtHandle_t> g_handles;
std::map<std::pair<int, hipStream_t>, void*> g_ws;
// (device, M, N, K, lda, ldw, ldc, c_bf16, bias, beta != 0)
typedef std::tuple<int, int64_t, int64_t, int64_t, int64_t, int64_t, int64_t, int, int, int> LtKey;
std::map<LtKey, LtPlan> g_plans;

#define LT_CHECK(expr)                                                                \
  do {                                                                                \
    const hipblasStatus_t s_ = (expr);                                                \
    if (s_ != HIPBLAS_STATUS_SUCCESS) {                                               \
      asrx::set_error("asrx_gemm_lt: %s failed (hipblas status %d)", #expr, (int)s_); \
      return -1;                                                                      \
    }                                                                                 \
  } while (0)

int get_handle(int dev, hipblasLtHandle_t* h) {
  auto it = g_handles.find(dev);
  if (it != g_handles.end()) {
    *h = it->second;
    return 0;
  }
  LT_CHECK(hipblasLtCreate(h));
  g_handles[dev] = *h;
  return 0;
}

int get_ws(int dev, hipStream_t st, void** ws) {
  void*& buf = g_ws[std::make_pair(dev, st)];
  if (!buf) {
    hipStreamCaptureMode mode = hipStreamCaptureModeRelaxed;
    (void)hipThreadExchangeStreamCaptureMode(&mode);
    const hipError_t e = hipMalloc(&buf, LT_WS_BYTES);
    (void)hipThreadExchangeStreamCaptureMode(&mode);
    if (e != hipSuccess) {
      buf = nullptr;
      asrx::set_error("asrx_gemm_lt workspace: %s", hipGetErrorString(e));
      return (int)e;
    }
  }
  *ws = buf;
  return 0;
}

int make_plan(hipblasLtHandle_t h, const LtKey& k, LtPlan* P) {
  const int64_t M = std::get<1>(k), N = std::get<2>(k), K = std::get<3>(k);
  const int64_t lda = std::get<4>(k), ldw = std::get<5>(k), ldc = std::get<6>(k);
  const int c_bf16 = std::get<7>(k), has_bias = std::get<8>(k);
  const hipDataType dt = c_bf16 ? HIP_R_16BF : HIP_R_32F;
  LT_CHECK(hipblasLtMatmulDescCreate(&P->op, HIPBLAS_COMPUTE_32F, HIP_R_32F));
  const int32_t opT = HIPBLAS_OP_T, opN = HIPBLAS_OP_N;
  LT_CHECK(hipblasLtMatmulDescSetAttribute(P->op, HIPBLASLT_MATMUL_DESC_TRANSA, &opT, sizeof(opT)));
  LT_CHECK(hipblasLtMatmulDescSetAttribute(P->op, HIPBLASLT_MATMUL_DESC_TRANSB, &opN, sizeof(opN)));
  if (has_bias) {
    const uint32_t epi = HIPBLASLT_EPILOGUE_BIAS;
    const int32_t bt = HIP_R_32F;
    LT_CHECK(hipblasLtMatmulDescSetAttribute(P->op, HIPBLASLT_MATMUL_DESC_EPILOGUE, &epi, sizeof(epi)));
    LT_CHECK(hipblasLtMatmulDescSetAttribute(P->op, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt)));
  }
  // column-major: library A = W^T stored K x N (ld ldw), library B = A^T stored K x M (ld lda), D = Y^T N x M (ld ldc)
  LT_CHECK(hipblasLtMatrixLayoutCreate(&P->la, HIP_R_16BF, K, N, ldw));
  LT_CHECK(hipblasLtMatrixLayoutCreate(&P->lb, HIP_R_16BF, K, M, lda));
  LT_CHECK(hipblasLtMatrixLayoutCreate(&P->lc, dt, N, M, ldc));
  hipblasLtMatmulPreference_t pref;
  LT_CHECK(hipblasLtMatmulPreferenceCreate(&pref));
  const uint64_t wsmax = LT_WS_BYTES;
  LT_CHECK(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsmax, sizeof(wsmax)));
  hipblasLtMatmulHeuristicResult_t res[1];
  int n = 0;
  const hipblasStatus_t hs = hipblasLtMatmulAlgoGetHeuristic(h, P->op, P->la, P->lb, P->lc, P->lc, pref, 1, res, &n);
  (void)hipblasLtMatmulPreferenceDestroy(pref);
  if (hs != HIPBLAS_STATUS_SUCCESS || n < 1) {
    asrx::set_error("asrx_gemm_lt: no algorithm for M=%ld N=%ld K=%ld (status %d)", (long)M, (long)N, (long)K, (int)hs);
    return -1;
  }
  P->algo = res[0].algo;
  P->ws = res[0].workspaceSize;
  return 0;
}

}  // namespace

extern "C" {

// Y (M x N, row stride ldc; fp32, or bf16 with c_bf16) = alpha A W^T + bias + beta Y.  A bf16 (M x K, lda), W bf16
// (N x K, ldw), bias fp32 (N) or NULL.  16-byte aligned operands.  Returns 0 or an error code (asrx_last_error).
int asrx_gemm_lt(const void* A, int64_t lda, const unsigned short* W, int64_t ldw, void* C, int c_bf16, int64_t ldc,
                 const float* bias, int64_t M, int64_t N, int64_t K, float alpha, float beta, hipStream_t stream) {
  ASRX_REQUIRE(M > 0 && N > 0 && K > 0, "asrx_gemm_lt: empty problem");
  ASRX_REQUIRE(((uintptr_t)A & 15) == 0 && ((uintptr_t)W & 15) == 0 && ((uintptr_t)C & 15) == 0,
               "asrx_gemm_lt: 16-byte aligned operands required");
  ASRX_REQUIRE(lda >= K && ldw >= K && ldc >= N, "asrx_gemm_lt: leading dimensions");
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) {
    asrx::set_error("asrx_gemm_lt: hipGetDevice failed");
    return -1;
  }
  std::lock_guard<std::mutex> lk(g_mu);
  hipblasLtHandle_t h;
  int rc = get_handle(dev, &h);
  if (rc) return rc;
  void* ws = nullptr;
  rc = get_ws(dev, stream, &ws);
  if (rc) return rc;
  const LtKey key{dev, M, N, K, lda, ldw, ldc, c_bf16 ? 1 : 0, bias ? 1 : 0, beta != 0.f ? 1 : 0};
  auto it = g_plans.find(key);
  if (it == g_plans.end()) {
    LtPlan P;
    rc = make_plan(h, key, &P);
    if (rc) return rc;
    it = g_plans.emplace(key, P).first;
  }
  LtPlan& P = it->second;
  if (bias) LT_CHECK(hipblasLtMatmulDescSetAttribute(P.op, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bias, sizeof(bias)));
  LT_CHECK(hipblasLtMatmul(h, P.op, &alpha, W, P.la, A, P.lb, &beta, C, P.lc, C, P.lc, &P.algo, ws, P.ws, stream));
  return 0;
}

}  // extern "C"
