// MSheath.forward (model.py:429-507) without a backward, issued from C++: one C-ABI call enqueues every
// per-layer launch of a call (policy, then per layer the v_gate projection GEMM, the fused row pass, the adapter
// GEMM, x_new's column sums, the control step and the jump update, then the gated MLP tail) -- the launch
// sequence of asrx/msheath.py forward(save=False), entry point for entry point, so the results are
// bit-identical.  A call that runs eagerly from Python costs ~7 Python-side launches of ~30 us of host time
// per layer; the dead blocks (model.py:617-626) and decoding run ~5700 such layers per medium-config step
// (profiles/r06_medium_b8_kernel_stats.csv).  (The steps turned out GPU-bound: the host time saved here is now spent
// waiting on full GPU queues, profiles/r06_host_vs_gpu.txt.)
//
// The per-module constants (parameter addresses, the bf16 weight copies, v_gate's combined projection) arrive as
// an asrx_msheath_plan the caller builds once per step and stream; the per-call buffers are carved from one
// caller-allocated workspace (asrx_msheath_fwd_ws_bytes).  bf16 perf mode only (the wide GEMM with bf16
// weights); the caller keeps the Python path for the other modes.
#include "common.h"

#include <cstdlib>

#include <cmath>

extern "C" {
int asrx_seg_colsum_det(const float* x, float* part, float* out, int64_t B, int64_t L, int64_t d, float scale,
                        hipStream_t stream);
int asrx_gemm_wn_ex(const void* A, int a_bf16, int64_t lda, int conv, int64_t convF, int64_t convC,
                    const unsigned short* W, int64_t ldw, void* C, int c_bf16, int64_t ldc, const float* bias, float* Z,
                    int64_t M, int64_t N, int64_t K, float alpha, float beta, int act, int nj, const int* mtiles,
                    const int* n_mtiles, hipStream_t stream);
int asrx_small_linear_fwd(const float* x, const float* W, const float* b, float* y, int64_t rows, int64_t K,
                          int64_t N, int act, hipStream_t stream);
int64_t asrx_row_tiles_max(int64_t M);
int asrx_row_tiles(const float* next_i, int64_t layer, int64_t L, int64_t M, int* mtiles, int* n_mtiles,
                   hipStream_t stream);
int asrx_msheath_row_fwd2(const float* x, const float* lnw, const float* lnb, const float* gw, const float* gb,
                          const float* SH, int64_t ldsh, const float* mval, const float* w2, const float* b2,
                          const float* cw, const float* cb, const float* tx, void* px, int px_bf16, float* mean,
                          float* rstd, float* nx, float* g, float* ion, float* kv, float* m2, int64_t rows, int64_t d,
                          int64_t M, int64_t Dh, float eps, float inv_sqrt_d, const float* next_i, int64_t layer,
                          int64_t L, hipStream_t stream);
int64_t asrx_mem_chunks(int64_t L);
int64_t asrx_msheath_rec_bytes(void);
int asrx_msheath_row_fwd3(const float* x, const float* lnw, const float* lnb, const float* gw, const float* gb,
                          const float* SH, int64_t ldsh, const float* mval, const float* w2, const float* b2,
                          const float* cw, const float* cb, const float* tx, float* px, float* mean, float* rstd,
                          float* nx, float* g, float* ion, float* kv, float* m2, float* xnew, float* part, int64_t rows,
                          int64_t d, int64_t M, int64_t Dh, float eps, float inv_sqrt_d, const float* next_i,
                          int64_t layer, int64_t L, hipStream_t stream);
int asrx_axpy_row2_colsum(const float* x, const float* s1, const float* s2, const float* y, float* out, float* part,
                          int64_t B, int64_t L, int64_t d, const float* next_i, int64_t layer, hipStream_t stream);
int asrx_msheath_ctrl_fwd3(const float* policy, const float* gpol, int64_t ld_gpol, const float* ion,
                           const float* mg_w, const float* mg_b, float* mem_v_out, const float* mem_w,
                           int64_t ld_mem_w, const float* mem_part, float* mem, const float* jump_s,
                           const float* next_i, int64_t layer_i, int64_t layers, int64_t B, int64_t L, int64_t D,
                           float* alpha, float* beta, float* gam, float* mem_w_out, float* active, float* next_out,
                           void* rec, hipStream_t stream);
int asrx_jump_axpy_inplace(const float* xin, float* xout, const float* s1, const float* s2, const float* y,
                           const float* orig, const float* act, const float* alpha, const float* beta, const float* gam,
                           int64_t B, int64_t L, int64_t d, hipStream_t stream);
int asrx_layernorm_fwd3(const float* x, const float* w, const float* b, void* y, int y_bf16, float* mean, float* rstd,
                        float* nrm, const float* gw, const float* gb, float* gout, int gate_on_x, int64_t rows,
                        int64_t d, float eps, hipStream_t stream);
int asrx_axpy_row(const float* x, const float* s, const float* y, float* out, int64_t rows, int64_t d,
                  hipStream_t stream);
}

// One MSheath layer (model.py:396-402 ModuleDict + v_gate, model.py:336-358).
struct asrx_msheath_layer {
  const float *ln_w, *ln_b;          // layers[i]["ln"]
  const float *gate_w, *gate_b;      // layers[i]["gate"][0]  Linear(D, 1)
  const float *mval;                 // v_gate.mval (M, 1)
  const float *vw2, *vb2;            // v_gate.mlp[2]  Linear(Dh, 1)
  const float *cw, *cb;              // v_gate.concat  Linear(2, 1)
  const float *tx;                   // v_gate.tx (threshold)
  const float *bc;                   // [0 (M) | v_gate.mlp[0].bias]  (asrx_vgate_weights)
  const unsigned short *wcb;         // bf16 [normalize(mkey); v_gate.mlp[0].weight]  (M + Dh, D)
  const unsigned short *ad_wb;       // bf16 adapter weight (D, D), null on odd layers
  const float *ad_b;                 // adapter bias
  int64_t M, Dh;                     // v_gate memory slots, MLP hidden
  float ln_eps;
  int32_t px_bf16;                   // px stored bf16 (it feeds only the adapter GEMM)
};

struct asrx_msheath_plan {
  const unsigned short *p0_wb;       // MPNet net[0] Linear(D, 128): bf16 weight, bias
  const float *p0_b;
  const float *p2_w, *p2_b;          // MPNet net[2] Linear(128, 3)
  int64_t p_hidden;                  // 128
  const float *mem_w;                // (1, 1, D) parameter
  const float *mg_w, *mg_b;          // mem_gate[0] Linear(D, 1)
  const float *jump_s;               // (3,)
  const float *mln_w, *mln_b;        // mlp_ln
  float mln_eps;
  int32_t hln_bf16;                  // mlp_ln's output stored bf16 (it feeds only mlp[0])
  const float *mgate_w, *mgate_b;    // mlp_gate[0] Linear(D, 1)
  const unsigned short *m0_wb;       // mlp[0] Linear(D, H1): bf16 weight, bias
  const float *m0_b;
  const unsigned short *m2_wb;       // mlp[2] Linear(H1, D)
  const float *m2_b;
  int64_t H1;
  int32_t a1_bf16;                   // SiLU(mlp[0]) stored bf16 (it feeds only mlp[2])
  int32_t n_layers;
  const asrx_msheath_layer* layers;
};

namespace asrx {
void set_msheath_row_nofill(bool on);  // rowops.hip
}

namespace {

// The composite's row passes leave the rows of samples not at a layer unwritten (nothing in a no-grad forward reads
// them; the Python path, whose saved tensors a backward reads, keeps zeroing them).  ASRX_ROW_NOFILL=0: zero them
// here too (A/B).  Reset on every exit from asrx_msheath_fwd.
struct RowNoFill {
  RowNoFill() {
    const char* e = std::getenv("ASRX_ROW_NOFILL");
    asrx::set_msheath_row_nofill(!(e && e[0] == '0'));
  }
  ~RowNoFill() { asrx::set_msheath_row_nofill(false); }
};

// asrx/gemm.py _nj (NJ_MIN_TILES): the widest 128 * nj tile with enough tiles -- 200 for either width at >= 16384
// rows, 180 (nj 3) / 144 (nj 2) below
int wide_nj(int64_t M, int64_t N, bool a_bf16) {
  const int64_t tm = (M + 127) / 128;
  const bool large = M >= 16384;
  for (int nj = 3; nj >= 2; --nj) {
    if (nj == 3 && !a_bf16 && N % 384) continue;  // an fp32 activation skips a partly empty 384-wide tile
    const int64_t th = large ? 200 : (nj == 3 ? 180 : 144);
    if (128 * nj <= ((N + 127) / 128) * 128 && tm * ((N + 128 * nj - 1) / (128 * nj)) >= th) return nj;
  }
  return 1;
}

constexpr int64_t ALIGN = 256;

struct Carver {
  char* base;
  int64_t off = 0;
  void* take(int64_t bytes) {
    void* p = base ? base + off : nullptr;
    off += (bytes + ALIGN - 1) / ALIGN * ALIGN;
    return p;
  }
};

struct Bufs {
  float *part, *pooled, *hp, *policy, *wsr, *wsb, *wsd;
  unsigned char* wsc;
  int *tl, *cnt;
  float *SH, *out, *xrun, *gate, *mean2, *rstd2, *hh;
  void *px, *hln, *a1;
};

Bufs carve(const asrx_msheath_plan& P, int64_t B, int64_t L, int64_t D, char* base, int64_t* total) {
  const int64_t rows = B * L, nl = P.n_layers, nchunk = asrx_mem_chunks(L);
  int64_t nmax = 0;
  for (int i = 0; i < nl; ++i) nmax = std::max(nmax, P.layers[i].M + P.layers[i].Dh);
  Carver c{base};
  Bufs b;
  b.part = (float*)c.take(4 * (nl + 1) * B * nchunk * D);
  b.pooled = (float*)c.take(4 * B * D);
  b.hp = (float*)c.take(4 * B * P.p_hidden);
  b.policy = (float*)c.take(4 * B * 3);
  b.wsr = (float*)c.take(4 * nl * 7 * rows);
  b.wsb = (float*)c.take(4 * nl * 5 * B);
  b.wsd = (float*)c.take(4 * nl * 3 * B * D);
  b.wsc = (unsigned char*)c.take(nl * B * asrx_msheath_rec_bytes());
  b.tl = (int*)c.take(4 * asrx_row_tiles_max(rows));
  b.cnt = (int*)c.take(4);
  b.SH = (float*)c.take(4 * rows * nmax);
  b.px = c.take(4 * rows * D);
  b.out = (float*)c.take(4 * rows * D);
  b.xrun = (float*)c.take(4 * rows * D);
  b.gate = (float*)c.take(4 * rows);
  b.hln = c.take(4 * rows * D);
  b.mean2 = (float*)c.take(4 * rows);
  b.rstd2 = (float*)c.take(4 * rows);
  b.a1 = c.take(4 * rows * P.H1);
  b.hh = (float*)c.take(4 * rows * D);
  *total = c.off;
  return b;
}

}  // namespace

#define MS_CALL(expr)          \
  do {                         \
    const int rc_ = (expr);    \
    if (rc_) return rc_;       \
  } while (0)

extern "C" {

int64_t asrx_msheath_fwd_ws_bytes(const asrx_msheath_plan* plan, int64_t B, int64_t L, int64_t D) {
  int64_t total = 0;
  carve(*plan, B, L, D, nullptr, &total);
  return total;
}

int64_t asrx_msheath_plan_bytes(void) { return (int64_t)sizeof(asrx_msheath_plan); }
int64_t asrx_msheath_layer_bytes(void) { return (int64_t)sizeof(asrx_msheath_layer); }

// y (B, L, D) = MSheath(x0) with policy noise gpol (B, layers, 3; row stride ld_gpol floats) -- asrx/msheath.py
// forward(save=False).  x0 and y contiguous fp32, distinct; ws: asrx_msheath_fwd_ws_bytes bytes of device memory.
int asrx_msheath_fwd(const asrx_msheath_plan* plan, const float* x0, const float* gpol, int64_t ld_gpol, float* y,
                     void* ws, int64_t ws_bytes, int64_t B, int64_t L, int64_t D, hipStream_t st) {
  ASRX_REQUIRE(plan && plan->layers && plan->n_layers > 0, "asrx_msheath_fwd: empty plan");
  ASRX_REQUIRE(B > 0 && L > 0 && D % 8 == 0 && plan->H1 % 8 == 0, "asrx_msheath_fwd: B, L > 0, D and H1 %% 8 required");
  ASRX_REQUIRE(x0 != y, "asrx_msheath_fwd: y must not alias x0");
  const asrx_msheath_plan& P = *plan;
  int64_t need = 0;
  Bufs b = carve(P, B, L, D, (char*)ws, &need);
  ASRX_REQUIRE(ws && ws_bytes >= need, "asrx_msheath_fwd: workspace %ld < %ld bytes", (long)ws_bytes, (long)need);
  const int64_t rows = B * L, nl = P.n_layers, nchunk = asrx_mem_chunks(L);
  const int64_t rec_bytes = asrx_msheath_rec_bytes();
  const RowNoFill nofill;
  const float inv_sqrt_d = (float)(1.0 / std::sqrt((double)D));
  // policy = softmax(MPNet(mean_l x0))   model.py:432-435, 375-385
  float* part_last = b.part + nl * B * nchunk * D;
  MS_CALL(asrx_seg_colsum_det(x0, part_last, b.pooled, B, L, D, (float)(1.0 / (double)L), st));
  MS_CALL(asrx_gemm_wn_ex(b.pooled, 0, D, 0, 0, 0, P.p0_wb, D, b.hp, 0, P.p_hidden, P.p0_b, nullptr, B, P.p_hidden, D,
                          1.f, 0.f, asrx::ACT_SILU, wide_nj(B, P.p_hidden, false), nullptr, nullptr, st));
  MS_CALL(asrx_small_linear_fwd(b.hp, P.p2_w, P.p2_b, b.policy, B, P.p_hidden, 3, asrx::ACT_SOFTMAX, st));
  const float* mem_w = P.mem_w;
  int64_t ld_mw = 0;
  const float* next_i = nullptr;
  const float* x = x0;
  for (int64_t i = 0; i < nl; ++i) {
    const asrx_msheath_layer& Ly = P.layers[i];
    const int64_t N = Ly.M + Ly.Dh;
    // rows of samples not at this layer are skipped: by whole 128-row tiles in the GEMMs, by row in the row kernels
    const int* tl = nullptr;
    const int* cnt = nullptr;
    if (next_i) {
      MS_CALL(asrx_row_tiles(next_i, i, L, rows, b.tl, b.cnt, st));
      tl = b.tl;
      cnt = b.cnt;
    }
    // SH = [x normalize(mkey)^T | mlp[0](x)]     model.py:346-349
    MS_CALL(asrx_gemm_wn_ex(x, 0, D, 0, 0, 0, Ly.wcb, D, b.SH, 0, N, Ly.bc, nullptr, rows, N, D, 1.f, 0.f,
                            asrx::ACT_NONE, wide_nj(rows, N, false), tl, cnt, st));
    float* wr = b.wsr + 7 * rows * i;  // mean, rstd, nx, g, ion, kv, m2
    float *mean = wr, *rstd = wr + rows, *nx = wr + 2 * rows, *gv = wr + 3 * rows, *ion = wr + 4 * rows,
          *kv = wr + 5 * rows, *m2 = wr + 6 * rows;
    const int pxb = Ly.ad_wb ? Ly.px_bf16 : 0;
    const float* out = (const float*)b.px;
    float* part_i = b.part + i * B * nchunk * D;
    if (Ly.ad_wb) {
      MS_CALL(asrx_msheath_row_fwd2(x, Ly.ln_w, Ly.ln_b, Ly.gate_w, Ly.gate_b, b.SH, N, Ly.mval, Ly.vw2, Ly.vb2,
                                    Ly.cw, Ly.cb, Ly.tx, b.px, pxb, mean, rstd, nx, gv, ion, kv, m2, rows, D, Ly.M, Ly.Dh,
                                    Ly.ln_eps, inv_sqrt_d, next_i, i, L, st));
      MS_CALL(asrx_gemm_wn_ex(b.px, pxb, D, 0, 0, 0, Ly.ad_wb, D, b.out, 0, D, Ly.ad_b, nullptr, rows, D, D, 1.f, 0.f,
                              asrx::ACT_NONE, wide_nj(rows, D, pxb != 0), tl, cnt, st));
      out = b.out;
      MS_CALL(asrx_axpy_row2_colsum(x, gv, ion, out, nullptr, part_i, B, L, D, next_i, i, st));
    } else {  // out = px: the row pass takes the column sums of x_new itself (asrx.msheath.ROW_COLSUM)
      MS_CALL(asrx_msheath_row_fwd3(x, Ly.ln_w, Ly.ln_b, Ly.gate_w, Ly.gate_b, b.SH, N, Ly.mval, Ly.vw2, Ly.vb2,
                                    Ly.cw, Ly.cb, Ly.tx, (float*)b.px, mean, rstd, nx, gv, ion, kv, m2, nullptr, part_i,
                                    rows, D, Ly.M, Ly.Dh, Ly.ln_eps, inv_sqrt_d, next_i, i, L, st));
    }
    float* wb5 = b.wsb + 5 * B * i;  // alpha, beta, active, next_out, mem_v
    float *alpha = wb5, *beta = wb5 + B, *active = wb5 + 2 * B, *next_out = wb5 + 3 * B, *mem_v = wb5 + 4 * B;
    float* wd3 = b.wsd + 3 * B * D * i;  // gam, mwo, mem
    float *gam = wd3, *mwo = wd3 + B * D, *mem = wd3 + 2 * B * D;
    MS_CALL(asrx_msheath_ctrl_fwd3(b.policy, gpol + 3 * i, ld_gpol, ion, P.mg_w, P.mg_b, mem_v, mem_w, ld_mw, part_i,
                                   mem, P.jump_s, next_i, i, nl, B, L, D, alpha, beta, gam, mwo, active, next_out,
                                   b.wsc + rec_bytes * B * i, st));
    // one pass, in place from layer 1 on (samples not at the layer keep their rows untouched)
    MS_CALL(asrx_jump_axpy_inplace(x, b.xrun, gv, ion, out, x0, active, alpha, beta, gam, B, L, D, st));
    mem_w = mwo;
    ld_mw = D;
    next_i = next_out;
    x = b.xrun;
  }
  // x + sigmoid(mlp_gate(x)) * mlp(mlp_ln(x))   (503-506): the gate from the LayerNorm's row pass
  MS_CALL(asrx_layernorm_fwd3(x, P.mln_w, P.mln_b, b.hln, P.hln_bf16, b.mean2, b.rstd2, nullptr, P.mgate_w,
                              P.mgate_b, b.gate, 1, rows, D, P.mln_eps, st));
  MS_CALL(asrx_gemm_wn_ex(b.hln, P.hln_bf16, D, 0, 0, 0, P.m0_wb, D, b.a1, P.a1_bf16, P.H1, P.m0_b, nullptr, rows,
                          P.H1, D, 1.f, 0.f, asrx::ACT_SILU, wide_nj(rows, P.H1, P.hln_bf16 != 0), nullptr, nullptr, st));
  MS_CALL(asrx_gemm_wn_ex(b.a1, P.a1_bf16, P.H1, 0, 0, 0, P.m2_wb, P.H1, b.hh, 0, D, P.m2_b, nullptr, rows, D, P.H1,
                          1.f, 0.f, asrx::ACT_NONE, wide_nj(rows, D, P.a1_bf16 != 0), nullptr, nullptr, st));
  MS_CALL(asrx_axpy_row(x, b.gate, b.hh, y, rows, D, st));
  return 0;
}

}  // extern "C"
