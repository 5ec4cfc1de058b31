/* asrx — C-ABI of the MI355X-native ASR hot path (libasrx.so, built from asr-model_amd/csrc).
 *
 * Conventions
 *   - every compute entry point takes raw DEVICE pointers (float32 unless noted), int64 sizes and
 *     strides in elements, and a hipStream_t (passed as void*); it enqueues on that stream and
 *     returns 0, or a nonzero code with a message readable through asrx_last_error();
 *   - nothing allocates: the caller owns outputs and workspaces; nothing synchronises;
 *   - entry points are reentrant (only immutable global state).
 * Each entry names the reference operation it replaces (sine2pi/ASR-model, file:line).
 */
#ifndef ASRX_H
#define ASRX_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* asrx_stream_t; /* hipStream_t */

/* ---- plumbing ------------------------------------------------------------------------------ */
const char* asrx_last_error(void);
int asrx_abi_version(void);
/* Keyed noise hash shared by device kernels and oracle/noise.py (gumbel_softmax noise at
 * essentials.py:170 / model.py:476, dropout masks at model.py:107,147). Host function. */
uint32_t asrx_noise_hash(uint32_t key, uint32_t idx);
/* Noise epoch (stream-ordered): when nonzero it is mixed into every site key, so a captured HIP graph
 * of a training step draws fresh dropout masks / gumbel noise per replay (the reference draws fresh
 * noise every step, essentials.py:751-824); 0 (default) = the keys of oracle/keys.py. */
int asrx_set_noise_epoch(uint32_t epoch, asrx_stream_t stream);
/* Wide-GEMM kernel selection for the activation x weight products (host state, not stream-ordered), a bit set:
 * low two bits 0 = gemm_wr_kernel (one workgroup per CU) only, 1 = gemm_p2_kernel (two per CU) for 384- and
 * 256-column tiles, 2 = also for 128-column tiles; + 4 the weight-stationary gemm_ws_kernel first where it measured
 * faster, + 8 gemm_ws on every shape it can run (tests), + 16 the d = 64 AbbyNormal router on gemm_wr_kernel instead
 * of router64_kernel.  Default 5 (gemm_p2 + gemm_ws).  Same results bit for bit in every setting; an A/B switch for
 * measurements and tests.  Returns the previous value. */
int asrx_set_gemm_variant(int variant);
/* Attention forward kernel selection at head dim 64 (host state): 1 (default) the software-pipelined kernel
 * (scores of the next key tile computed beside this tile's softmax), 0 the round-4 kernel.  Same results bit
 * for bit; an A/B switch for measurements and tests.  Returns the previous value. */
int asrx_set_attn_variant(int variant);
/* Weight-gradient kernel selection for fp32 dY with bf16 X and N % 384 == 0 (host state): 1 (default) the
 * 128 x 384 work items of wgrad_w3_kernel, 0 the 128 x 128 items of wgrad_wr_kernel.  Same products, summed
 * over K slices by float atomics in either case (fp32 reassociation only).  Returns the previous value. */
int asrx_set_wgrad_variant(int variant);

/* ---- log-mel front end: replaces torchaudio MelSpectrogram + log10 + clip-max floor,
 *      essentials.py:469-491, and the waveform adaptive_avg_pool1d, essentials.py:493-510 -------- */
int asrx_mel_frames(int64_t n_samples); /* 1 + N/160 (host) */
/* wav (B,N) at row stride ld_wav; consts = window|tw512|tw1024 (see asrx/mel.py); fbw/fbs the
 * lane-packed HTK filterbank of asrx/mel.py lane_filterbank (fbs int32[256] = band_a | band_b |
 * even start bins a | b, fbw float[8][64][4] = weights/4); out (B,F,128) when layout==0 or
 * (B,128,F) when layout==1, clip stride ld_out; ws a device workspace of asrx_logmel_ws_bytes(B, N)
 * bytes (per-tile max | min of the log values, overwritten); pool (B,T_pool) or NULL (needs
 * N == 160*T_pool).  Two launches: the tile transform (writes (x+4)/4 and the tile stats) and the
 * clip-max floor, which rewrites only the tiles holding a value below max - 8. */
int64_t asrx_logmel_ws_bytes(int64_t B, int64_t N); /* host */
int asrx_logmel(const float* wav, int64_t B, int64_t N, int64_t ld_wav, const float* consts,
                const float* fbw, const int* fbs, float* out, int layout, int64_t ld_out,
                void* ws, float* pool, int64_t T_pool, asrx_stream_t stream);
/* waveform feature for any clip length: adaptive_avg_pool1d(audio, T) (essentials.py:493-510), bin i the
 * mean of samples [floor(i N / T), ceil((i + 1) N / T)); wav (B, N) at row stride ld_wav, out (B, T). */
int asrx_wave_pool(const float* wav, int64_t B, int64_t N, int64_t ld_wav, int64_t T, float* out,
                   asrx_stream_t stream);

/* ---- audio IO: load_wave's soundfile.read + peak normalisation,
 *      essentials.py:301-319, for the prepare_datasets path (998-1026). -------------------------
 * FLAC (RFC 9639) decoding, host functions on an in-memory file: asrx_flac_info returns STREAMINFO
 * (samples per channel, channels, rate, bits, MD5 of the audio); asrx_flac_decode writes planar int32
 * (channels x cap), checking every frame's CRC-8 / CRC-16. */
int asrx_flac_info(const uint8_t* buf, int64_t n, int64_t* frames, int* channels, int* rate, int* bits,
                   uint8_t* md5);
int asrx_flac_decode(const uint8_t* buf, int64_t n, int32_t* out, int64_t cap);
/* Device: pcm (B,C,ld) int32 (is_float = 0) or fp32 (1) -> out (B,C,ld_out) fp32 = pcm * scale[b],
 * then (normalize != 0) divided by max|x| (mono) or by each channel's max(x) (multi-channel, the
 * reference's quirk); zero past lengths[b] (int64, device). */
int asrx_pcm_normalize(const void* pcm, int is_float, int64_t B, int64_t C, int64_t ld, const int64_t* lengths,
                       const float* scale, float* out, int64_t ld_out, int normalize, asrx_stream_t stream);

/* ---- GEMM: replaces F.linear / 1x1 and k3 conv1d (fwd, dgrad, wgrad) at model.py:96-147,
 *      242-245, 341, 398-425, 529-574, essentials.py:149-153 ------------------------------------
 * C[b] = act(alpha*A[b]@B[b] + beta*C[b] + bias); A MxK (a_kc: row-major MxK, else KxM), B KxN
 * (b_kc: stored NxK, else KxN). conv_a/conv_b: implicit k3 pad-1 im2col of a channels-last
 * sequence with segment length conv_F and conv_C channels. prec 0 = fp32 MFMA, 1 = bf16 MFMA.
 * act: 0 none, 1 gelu(erf), 2 silu, 3 sigmoid, 4 relu. Z (optional) receives the pre-activation.
 * splitk > 1 accumulates partial sums into C with atomics (beta must be 1, act none). */
int asrx_gemm(int prec, const float* A, int64_t lda, int64_t sA, int a_kc, int conv_a,
              const float* B, int64_t ldb, int64_t sB, int b_kc, int conv_b, float* C, int64_t ldc,
              int64_t sC, const float* bias, float* Z, int64_t M, int64_t N, int64_t K,
              int64_t batch, float alpha, float beta, int act, int64_t conv_F, int64_t conv_C,
              int splitk, asrx_stream_t stream);


/* ---- wide-N GEMM for activation x weight products in perf mode (same call sites as asrx_gemm):
 * C (M x N) = act(alpha * A W^T + beta * C + bias); A fp32 (M x K, lda) or its implicit k3 im2col
 * (conv: lda = channels, convF segment length, convC channels); W bf16 N x K (ldw) prepared by
 * asrx_weight_to_bf16; nj in 1..3 selects the 128*nj-wide output tile. ------------------------- */
int asrx_weight_to_bf16(const float* src, unsigned short* dst, int64_t rows, int64_t cols, int64_t ld, int trans,
                        asrx_stream_t stream);
/* every weight of a step in one launch: tab = n device-resident entries {const float* src; uint16*
 * dst; int64 ld; int32 rows, cols, trans, pad} (asrx_wconv_entry_bytes() each), max_elems = the
 * largest rows*cols */
int64_t asrx_wconv_entry_bytes(void);
int asrx_weights_to_bf16(const void* tab, int64_t n, int64_t max_elems, asrx_stream_t stream);
/* AbbyNormal router in one GEMM pass (essentials.py:155-161): hpre = A W1^T + b1 (stored when
 * hpre != NULL) and logits = SiLU(hpre) W2^T (M x 3, without b2); W1 bf16 (N x K), N <= 384. */
int asrx_gemm_wn_router(const float* A, int64_t lda, const unsigned short* W1, int64_t ldw, const float* b1,
                        const float* W2, float* hpre, int64_t ldc, float* logits, int64_t M, int64_t N, int64_t K,
                        asrx_stream_t stream);
int asrx_gemm_wn(const float* A, int64_t lda, int conv, int64_t convF, int64_t convC, const unsigned short* W,
                 int64_t ldw, float* C, int64_t ldc, const float* bias, float* Z, int64_t M, int64_t N, int64_t K,
                 float alpha, float beta, int act, int nj, asrx_stream_t stream);
/* asrx_gemm_wn on the BM(=128)-row tiles listed on the device (mtiles[0 .. *n_mtiles)); other rows of
 * C are not written.  asrx_row_tiles lists the tiles holding rows of samples at MSheath layer
 * `layer` (next_i[b] == layer, L rows per sample), at most asrx_row_tiles_max(M) entries. */
/* weight gradient in perf mode: dW (M x N, ldc) += dY^T X over R rows (dY: R x M, lda; X: R x N, ldb;
 * fp32 row-major, rounded to bf16 for the MFMA, fp32 accumulate, split over `splitk` row slices
 * with float atomics).  M, N, lda, ldb multiples of 4; 16-byte aligned operands. */
int asrx_wgrad_bf16(const float* A, int64_t lda, const float* B, int64_t ldb, float* C, int64_t ldc, int64_t M,
                    int64_t N, int64_t R, int64_t splitk, asrx_stream_t stream);
int asrx_gemm_wn_rows(const float* A, int64_t lda, const unsigned short* W, int64_t ldw, float* C, int64_t ldc,
                      const float* bias, float* Z, int64_t M, int64_t N, int64_t K, float alpha, float beta, int act,
                      int nj, const int* mtiles, const int* n_mtiles, asrx_stream_t stream);
/* bf16 activation storage (perf mode; an activation whose only consumers are GEMM operands is stored
 * bf16 by its producer -- the GEMMs round it to bf16 anyway, so the products are unchanged).
 * asrx_gemm_wn_ex: asrx_gemm_wn with A stored fp32 (a_bf16 = 0) or bf16 (1: lda % 8, conv C % 8) and C
 * stored fp32 (c_bf16 = 0) or bf16 (1: beta = 0; Z stays fp32), optionally on a device tile list
 * (mtiles / n_mtiles as asrx_gemm_wn_rows, non-conv; NULL = every tile).  Replaces F.linear / 1x1 / k3
 * conv1d at the call sites listed for asrx_gemm (model.py:96-147, 242-245, 341, 398-425, 529-574).
 * asrx_wgrad_bf16_ex: asrx_wgrad_bf16 with X (B) stored fp32 (b_bf16 = 0) or bf16 (1: N, ldb % 8). */
int asrx_gemm_wn_ex(const void* A, int a_bf16, int64_t lda, int conv, int64_t convF, int64_t convC,
                    const unsigned short* W, int64_t ldw, void* C, int c_bf16, int64_t ldc, const float* bias,
                    float* Z, int64_t M, int64_t N, int64_t K, float alpha, float beta, int act, int nj,
                    const int* mtiles, const int* n_mtiles, asrx_stream_t stream);
int asrx_wgrad_bf16_ex(const float* A, int64_t lda, const void* B, int b_bf16, int64_t ldb, float* C, int64_t ldc,
                       int64_t M, int64_t N, int64_t R, int64_t splitk, asrx_stream_t stream);
int64_t asrx_row_tiles_max(int64_t M);
int asrx_row_tiles(const float* next_i, int64_t layer, int64_t L, int64_t M, int* mtiles, int* n_mtiles,
                   asrx_stream_t stream);

/* ---- AbbyNormal: essentials.py:140-191 (router SiLU-MLP, cv, gumbel hard decision, avg/max pool of
 *      x^2 along the feature axis, x / (1 + 1e-4 div)^0.75).  hpre = x @ W1^T + b1 from asrx_gemm.
 *      Rows are (sample, position, head)-major; noise index ((sid*H+h)*8192+l)*3+k, sid = sid_base + b.
 *      ys (rows,3) / idx (rows) int32 are saved for backward. ----------------------------------- */
/* decision recorder (parity tests, eager only): while buf != NULL every AbbyNormal forward writes mode
 * 2's per-feature choice max > 2 avg (essentials.py:176-177) of its mode-2 rows into buf (rows x d
 * bytes, caller-zeroed) */
int asrx_abby_record_cond(unsigned char* buf);
int asrx_abby_fwd(const float* x, const float* hpre, const float* W2, const float* b2, float* out, float* ys,
                  int* idx, int64_t rows, int64_t d, int64_t L, int64_t H, int64_t sid_base, uint32_t key,
                  int use_noise, asrx_stream_t stream);
/* AbbyNormal with a residual input: out = res + AbbyNormal(x) (fp32, d >= 128), router logits given (rows x 3,
 * no b2) or computed from hpre / W2 (logits NULL) -- the closing residual add of residual.forward
 * (model.py:583) fused into the mlp's last norm. */
int asrx_abby_fwd_res(const float* x, const float* hpre, const float* W2, const float* logits, const float* b2,
                      const float* res, float* out, float* ys, int* idx, int64_t rows, int64_t d, int64_t L, int64_t H,
                      int64_t sid_base, uint32_t key, int use_noise, asrx_stream_t stream);
/* dx, dhpre overwritten; dW2 (3,d) / db2 (3) accumulated. */
/* AbbyNormal forward from precomputed router logits (rows x 3, no b2) -- asrx_gemm_wn_router. */
int asrx_abby_fwd_logits(const float* x, const float* logits, const float* b2, float* out, float* ys, int* idx,
                         int64_t rows, int64_t d, int64_t L, int64_t H, int64_t sid_base, uint32_t key,
                         int use_noise, asrx_stream_t stream);
/* asrx_abby_fwd / asrx_abby_fwd_logits with out stored fp32 (out_bf16 = 0) or bf16 (1: the AbbyNormal
 * output feeds only a projection GEMM or attention -- attention.q[0] / kv[0] and the per-head norm,
 * model.py:244-245, 248; the final norm before the tied logits, model.py:629; mlp's first norm, 573).
 * tw (3 x d) / tb (3) / tc (rows x 3), optional (d >= 128): the consuming tgate's cs = Linear(d, 3)
 * (model.py:530) evaluated on the fp32 output rows, so that output can be stored bf16. */
int asrx_abby_fwd2(const float* x, const float* hpre, const float* W2, const float* b2, void* out, int out_bf16,
                   float* ys, int* idx, int64_t rows, int64_t d, int64_t L, int64_t H, int64_t sid_base, uint32_t key,
                   int use_noise, const float* tw, const float* tb, float* tc, asrx_stream_t stream);
int asrx_abby_fwd_logits2(const float* x, const float* logits, const float* b2, void* out, int out_bf16, float* ys,
                          int* idx, int64_t rows, int64_t d, int64_t L, int64_t H, int64_t sid_base, uint32_t key,
                          int use_noise, const float* tw, const float* tb, float* tc, asrx_stream_t stream);
/* asrx_abby_fwd2 (logits NULL) / asrx_abby_fwd_logits2 (logits given) that also writes ||x[r]||_2 to nrm
   (rows,) when nrm is non-NULL (d >= 128): the |src| of rotary (model.py:201) without a second pass. */
int asrx_abby_fwd3(const float* x, const float* hpre, const float* W2, const float* logits, const float* b2,
                   void* out, int out_bf16, float* ys, int* idx, int64_t rows, int64_t d, int64_t L, int64_t H,
                   int64_t sid_base, uint32_t key, int use_noise, const float* tw, const float* tb, float* tc,
                   float* nrm, asrx_stream_t stream);
int asrx_abby_bwd(const float* dout, const float* x, const float* hpre, const float* W2, const float* ys,
                  const int* idx, float* dx, float* dhpre, float* dW2, float* db2, int64_t rows, int64_t d,
                  asrx_stream_t stream);
/* as asrx_abby_bwd; acc != 0 adds x's gradient into dx instead of writing it */
int asrx_abby_bwd2(const float* dout, const float* x, const float* hpre, const float* W2, const float* ys,
                   const int* idx, float* dx, float* dhpre, float* dW2, float* db2, int64_t rows, int64_t d, int acc,
                   asrx_stream_t stream);

/* ---- attention: F.scaled_dot_product_attention(q,k,v,is_causal) at model.py:307, head dim hd = 64
 *      (tiny/small/medium) or 128 (the reference's Dimensions(dims=512, head=4), model.py:746).
 *      q/k/v/o are (B,L,H,hd) with strides sX = int64[3] {batch, seq, head}; lse (B,H,Lq).
 *      asrx_attn_fwd also takes prec 2 = fp8 attention: QK^T on e4m3 with
 *      per-row scales (MX-rate MFMA), softmax and PV in bf16; the backward takes 0 or 1 only. ---- */
int asrx_attn_fwd(int prec, const float* q, const int64_t* sq, const float* k, const int64_t* sk, const float* v,
                  const int64_t* sv, float* o, const int64_t* so, float* lse, int64_t B, int64_t H, int64_t Lq,
                  int64_t Lk, int64_t hd, int causal, float scale, asrx_stream_t stream);
/* asrx_attn_fwd / _bwd with storage types (prec 1 only when io != 0): io bit 0 = q / k / v stored bf16
 * (what the per-head AbbyNormal and the v projection write when attention is their only consumer),
 * bit 1 = o stored bf16 (it only feeds the out projection, model.py:316-317), bit 2 = dO stored bf16. */
int asrx_attn_fwd2(int prec, int io, const void* q, const int64_t* sq, const void* k, const int64_t* sk,
                   const void* v, const int64_t* sv, void* o, const int64_t* so, float* lse, int64_t B, int64_t H,
                   int64_t Lq, int64_t Lk, int64_t hd, int causal, float scale, asrx_stream_t stream);
int asrx_attn_bwd2(int prec, int io, const void* q, const int64_t* sq, const void* k, const int64_t* sk,
                   const void* v, const int64_t* sv, const void* o, const int64_t* so, const void* dO,
                   const int64_t* sd, const float* lse, float* delta_ws, float* dq, const int64_t* sdq, float* dk,
                   const int64_t* sdk, float* dv, const int64_t* sdv, int64_t B, int64_t H, int64_t Lq, int64_t Lk,
                   int64_t hd, int causal, float scale, asrx_stream_t stream);
/* delta_ws: B*H*Lq floats of workspace. */
int asrx_attn_bwd(int prec, const float* q, const int64_t* sq, const float* k, const int64_t* sk, const float* v,
                  const int64_t* sv, const float* o, const int64_t* so, const float* dO, const int64_t* sd,
                  const float* lse, float* delta_ws, float* dq, const int64_t* sdq, float* dk, const int64_t* sdk,
                  float* dv, const int64_t* sdv, int64_t B, int64_t H, int64_t Lq, int64_t Lk, int64_t hd,
                  int causal, float scale, asrx_stream_t stream);

/* ---- LayerNorm over the last dim: nn.LayerNorm in MSheath (model.py:405, 427) and the channel
 *      LayerNorm of the encoder (essentials.py:110-113) on channels-last rows. ------------------ */
int asrx_layernorm_fwd(const float* x, const float* w, const float* b, float* y, float* mean, float* rstd,
                       int64_t rows, int64_t d, float eps, asrx_stream_t stream);
int asrx_layernorm_bwd(const float* dy, const float* x, const float* w, const float* mean, const float* rstd,
                       float* dx, float* dw, float* db, int64_t rows, int64_t d, asrx_stream_t stream);
/* acc != 0: dx += the LayerNorm input gradient (one buffer collects every consumer's contribution). */
int asrx_layernorm_bwd_acc(const float* dy, const float* x, const float* w, const float* mean, const float* rstd,
                           float* dx, float* dw, float* db, int64_t rows, int64_t d, int acc, asrx_stream_t stream);

/* LayerNorm forward with fused row outputs (each may be NULL): nrm = |x| (v_gate's norm of the same
 * x, model.py:347) and gout = sigmoid(v . gw + gb) with v = y, or v = x when gate_on_x (the Linear(D,1)
 * gates at model.py:460, 503).  d in {128, 256, 384, 512, 768, 1024}. */
int asrx_layernorm_fwd2(const float* x, const float* w, const float* b, float* y, float* mean, float* rstd,
                        float* nrm, const float* gw, const float* gb, float* gout, int gate_on_x, int64_t rows,
                        int64_t d, float eps, asrx_stream_t stream);
/* asrx_layernorm_fwd2 with y stored fp32 (y_bf16 = 0) or bf16 (1: MSheath's mlp_ln output only feeds
 * mlp[0], model.py:503-506) */
int asrx_layernorm_fwd3(const float* x, const float* w, const float* b, void* y, int y_bf16, float* mean, float* rstd,
                        float* nrm, const float* gw, const float* gb, float* gout, int gate_on_x, int64_t rows,
                        int64_t d, float eps, asrx_stream_t stream);

/* ---- small-N linear (N <= 4): gate / mem_gate / mlp_gate Linear(D,1) (model.py:398, 406, 420),
 *      v_gate.mlp[2] (341), tgate.cs Linear(D,3) (530), MPNet's Linear(128,3) (381).
 *      act: 0 none, 3 sigmoid; forward only: 16 = softmax over the N outputs of the row (MPNet + the
 *      softmax of model.py:435 in one launch).  Backward: dx = beta*dx + dz W; dW/db accumulated from
 *      per-workgroup partials in a fixed order (deterministic; a 16 MB partial buffer per stream, allocated on
 *      the stream's first call, capture-safe, kept for the process lifetime). ------ */
int asrx_small_linear_fwd(const float* x, const float* W, const float* b, float* y, int64_t rows, int64_t K,
                          int64_t N, int act, asrx_stream_t stream);
int asrx_small_linear_bwd(const float* dy, const float* y, const float* x, const float* W, float* dx, float* dW,
                          float* db, int64_t rows, int64_t K, int64_t N, int act, float beta,
                          asrx_stream_t stream);
/* the same with x stored fp32 (x_bf16 = 0) or bf16 (1: tgate.cs over a bf16-stored AbbyNormal output,
 * model.py:530) */
int asrx_small_linear_fwd2(const void* x, int x_bf16, const float* W, const float* b, float* y, int64_t rows,
                           int64_t K, int64_t N, int act, asrx_stream_t stream);
int asrx_small_linear_bwd2(const float* dy, const float* y, const void* x, int x_bf16, const float* W, float* dx,
                           float* dW, float* db, int64_t rows, int64_t K, int64_t N, int act, float beta,
                           asrx_stream_t stream);

/* ---- row L2 norms: torch.norm in rotary (model.py:201), F.normalize in v_gate (347). ---------- */
int asrx_rownorm(const float* x, float* n, int64_t rows, int64_t d, asrx_stream_t stream);
int asrx_rownorm_bwd(const float* dn, const float* x, const float* n, float* dx, int64_t rows, int64_t d,
                     asrx_stream_t stream);
/* acc == 0: dx = the |x| gradient (written); acc != 0: accumulated like asrx_rownorm_bwd. */
int asrx_rownorm_bwd2(const float* dn, const float* x, const float* n, float* dx, int64_t rows, int64_t d, int acc,
                      asrx_stream_t stream);
/* F.normalize(x, p=2, dim=-1) (v_gate's keys, model.py:347): y, n = max(|x|, 1e-12); backward
 * dx (+)= (dy - y (y.dy)) / n. */
int asrx_row_normalize(const float* x, float* y, float* n, int64_t rows, int64_t d, asrx_stream_t stream);
int asrx_row_normalize_bwd(const float* dy, const float* y, const float* n, float* dx, int64_t rows, int64_t d,
                           int acc, asrx_stream_t stream);
/* softmax over rows of N <= 8 (MPNet policy, model.py:385) and its backward. */
int asrx_softmax_small(const float* x, float* y, int64_t rows, int64_t N, asrx_stream_t stream);
int asrx_softmax_small_bwd(const float* g, const float* y, float* dx, int64_t rows, int64_t N, asrx_stream_t stream);
/* stream-ordered memset of device memory to zero */
int asrx_zero(void* p, int64_t bytes, asrx_stream_t stream);

/* ---- rotary (model.py:198-214) fused with the hd^-0.25 pre-scale (303-304); x (B,L,H*hd),
 *      m[B*L] = |src| rows, f[hd/2] float32 frequencies; dm accumulated in backward. ------------- */
int asrx_rotary_fwd(const float* x, const float* m, const float* f, float* y, int64_t BL, int64_t L, int64_t D,
                    int64_t hd, float scale, asrx_stream_t stream);
int asrx_rotary_bwd(const float* g, const float* x, const float* m, const float* f, float* dx, float* dm,
                    int64_t BL, int64_t L, int64_t D, int64_t hd, float scale, asrx_stream_t stream);
/* The same with the (cos, sin) table of asrx_rotary_table (tab: L x hd/2 float2, NULL = sincosf in the
   kernel): the angles depend only on (position, pair), so B samples x H heads share one table.  Results
   are bit-identical to the direct form. */
int asrx_rotary_table(const float* f, float* tab, int64_t L, int64_t hd, asrx_stream_t stream);
int asrx_rotary_fwd2(const float* x, const float* m, const float* f, const float* tab, float* y, int64_t BL, int64_t L,
                     int64_t D, int64_t hd, float scale, asrx_stream_t stream);
int asrx_rotary_bwd2(const float* g, const float* x, const float* m, const float* f, const float* tab, float* dx,
                     float* dm, int64_t BL, int64_t L, int64_t D, int64_t hd, float scale, asrx_stream_t stream);

/* ---- v_gate (model.py:346-351): S = x mkey_n^T, h = mlp[0](x) pre-activation from asrx_gemm. ---- */
int asrx_vgate_fwd(const float* S, const float* nx, const float* mval, const float* h, const float* w2,
                   const float* b2, const float* cw, const float* cb, const float* tx, float* ion, float* xval,
                   float* kv, float* m2, int64_t rows, int64_t M, int64_t Dh, float inv_sqrt_d,
                   asrx_stream_t stream);
int asrx_vgate_bwd(const float* dion, const float* S, const float* nx, const float* mval, const float* h,
                   const float* w2, const float* cw, const float* kv, const float* m2, float* dS, float* dnx,
                   float* dh, float* dmval, float* dw2, float* db2, float* dcw, float* dcb, int64_t rows, int64_t M,
                   int64_t Dh, float inv_sqrt_d, asrx_stream_t stream);

/* ---- fused MSheath layer rows (asrx/msheath.py; model.py:346-351, 452-461).  v_gate's projections
 *      as one GEMM against Wc = [normalize(mkey); mlp[0].weight] ((M+Dh) x D), bc = [0; mlp[0].bias]
 *      (asrx_vgate_weights; wb = bf16 Wc or NULL, mkn = key norms), giving SH = [S | h] (row stride
 *      ldsh).  asrx_msheath_row_fwd: per row px = LayerNorm(x), nx = |x|, g = sigmoid(px.gw + gb), the
 *      v_gate outputs (ion, kv, m2).  asrx_msheath_row_bwd: its backward with dx accumulated, dSH
 *      written and every parameter gradient accumulated; db1 is mlp[0].bias's gradient.  d in {128,
 *      256, 384, 512, 768, 1024}, M <= 64.  With next_i (L rows per sample), rows of samples with
 *      next_i[b] != layer are skipped (the reference never runs them): forward writes zeros, backward
 *      dSH = 0 rows. */
int asrx_vgate_weights(const float* mkey, const float* W1, const float* b1, float* Wc, float* bc, float* mkn,
                       unsigned short* wb, int64_t M, int64_t Dh, int64_t D, asrx_stream_t stream);
int asrx_msheath_row_fwd(const float* x, const float* lnw, const float* lnb, const float* gw, const float* gb,
                         const float* SH, int64_t ldsh, const float* mval, const float* w2, const float* b2,
                         const float* cw, const float* cb, const float* tx, float* px, float* mean, float* rstd,
                         float* nx, float* g, float* ion, float* kv, float* m2, int64_t rows, int64_t d, int64_t M,
                         int64_t Dh, float eps, float inv_sqrt_d, const float* next_i, int64_t layer, int64_t L,
                         asrx_stream_t stream);
/* px stored fp32 (px_bf16 = 0) or bf16 (1: on layers with an adapter px only feeds the adapter GEMM,
 * model.py:455-457) */
int asrx_msheath_row_fwd2(const float* x, const float* lnw, const float* lnb, const float* gw, const float* gb,
                          const float* SH, int64_t ldsh, const float* mval, const float* w2, const float* b2,
                          const float* cw, const float* cb, const float* tx, void* px, int px_bf16, float* mean,
                          float* rstd, float* nx, float* g, float* ion, float* kv, float* m2, int64_t rows, int64_t d,
                          int64_t M, int64_t Dh, float eps, float inv_sqrt_d, const float* next_i, int64_t layer,
                          int64_t L, asrx_stream_t stream);
/* asrx_msheath_row_fwd2 for a layer without adapter (px fp32, the update itself) that also forms x_new = x + g ion px
 * (model.py:461) into xnew (when non-null) and its per-sample 64-row chunk column sums into part (B x
 * asrx_mem_chunks(L) x d, zeros for a sample not at the layer) -- asrx_axpy_row2_colsum's work in the same pass.
 * rows = B L. */
int asrx_msheath_row_fwd3(const float* x, const float* lnw, const float* lnb, const float* gw, const float* gb,
                          const float* SH, int64_t ldsh, const float* mval, const float* w2, const float* b2,
                          const float* cw, const float* cb, const float* tx, float* px, float* mean, float* rstd,
                          float* nx, float* g, float* ion, float* kv, float* m2, float* xnew, float* part, int64_t rows,
                          int64_t d, int64_t M, int64_t Dh, float eps, float inv_sqrt_d, const float* next_i,
                          int64_t layer, int64_t L, asrx_stream_t stream);
int asrx_msheath_row_bwd(const float* dpx, const float* x, const float* lnw, const float* lnb, const float* mean,
                         const float* rstd, const float* dg, const float* g, const float* gw, const float* dion,
                         const float* SH, int64_t ldsh, const float* nx, const float* mval, const float* w2,
                         const float* cw, const float* kv, const float* m2, float* dx, float* dlnw, float* dlnb,
                         float* dgw, float* dgb, float* dSH, float* dmval, float* dw2, float* db2, float* dcw,
                         float* dcb, float* db1, int64_t rows, int64_t d, int64_t M, int64_t Dh, float inv_sqrt_d,
                         const float* next_i, int64_t layer, int64_t L, asrx_stream_t stream);

/* ---- tgate (model.py:532-535): G = sigmoid(x Wcat^T + b) (rows,3D) from asrx_gemm, c (rows,3). */
int asrx_tgate_fwd(const float* G, const float* c, float* out, int64_t rows, int64_t D, asrx_stream_t stream);
/* tgate combine with out stored bf16 (out_bf16 = 1: it only feeds mlp's Linear(D, 3D), model.py:573) */
int asrx_tgate_fwd2(const float* G, const float* c, void* out, int out_bf16, int64_t rows, int64_t D,
                    asrx_stream_t stream);
int asrx_tgate_bwd(const float* dout, const float* G, const float* c, float* dGz, float* dc, int64_t rows,
                   int64_t D, asrx_stream_t stream);

/* ---- MSheath updates (model.py:461, 489-505) and reductions ---------------------------------- */
int asrx_axpy_row(const float* x, const float* s, const float* y, float* out, int64_t rows, int64_t d,
                  asrx_stream_t stream);
int asrx_axpy_row_bwd(const float* g, const float* s, const float* y, float* dy, float* ds, int64_t rows,
                      int64_t d, asrx_stream_t stream);
/* as asrx_axpy_row_bwd, and dxc = g (x's pass-through gradient into a caller-owned buffer) */
int asrx_axpy_row_bwd2(const float* g, const float* s, const float* y, float* dy, float* ds, float* dxc,
                       int64_t rows, int64_t d, asrx_stream_t stream);
int asrx_jump_select(const float* xn, const float* orig, const float* xold, const float* act, const float* alpha,
                     const float* beta, const float* gam, float* out, int64_t B, int64_t L, int64_t d,
                     asrx_stream_t stream);
int asrx_jump_select_bwd(const float* g, const float* xn, const float* orig, const float* act, const float* alpha,
                         const float* beta, float* dxn, float* dorig, float* dxold, float* dalpha, float* dbeta,
                         float* dgam, int64_t B, int64_t L, int64_t d, asrx_stream_t stream);
/* MSheath per-layer control (model.py:461-501), batched with per-sample trajectories: potential,
 * gumbel-hard policy, action, alpha/beta/gam, mem_w update, next layer.  rec: B records of
 * asrx_msheath_rec_bytes() bytes saved for the backward.  g_mwo may be NULL. */
int asrx_msheath_ctrl_fwd(const float* policy, const float* gpol, int64_t ld_gpol, const float* ion,
                          const float* mem_v, const float* mem_w, const float* mem, const float* jump_s,
                          const float* next_i, int64_t layer_i, int64_t layers, int64_t B, int64_t L, int64_t D,
                          float* alpha, float* beta, float* gam, float* mem_w_out, float* active, float* next_out,
                          void* rec, asrx_stream_t stream);
int asrx_msheath_ctrl_bwd(const float* g_alpha, const float* g_beta, const float* g_gam, const float* g_mwo,
                          const float* mem_v, const float* mem_w, const float* mem, const float* jump_s,
                          const void* rec, int64_t layer_i, int64_t layers, int64_t B, int64_t D, float* g_policy,
                          float* g_mem_v, float* g_mem_w, float* g_mem, float* g_jump_s, asrx_stream_t stream);
int64_t asrx_msheath_rec_bytes(void);
/* ctrl with mem_w's row stride (0: the (1,1,D) parameter broadcast over samples) and a nullable
 * next_i (every sample at layer 0); backward with g_policy accumulated (acc_policy) and has_orig[b]
 * set when this layer's jump wrote orig's gradient (asrx_jump_select4_bwd_acc). */
int asrx_msheath_ctrl_fwd2(const float* policy, const float* gpol, int64_t ld_gpol, const float* ion,
                           const float* mem_v, const float* mem_w, int64_t ld_mem_w, const float* mem,
                           const float* jump_s, const float* next_i, int64_t layer_i, int64_t layers, int64_t B,
                           int64_t L, int64_t D, float* alpha, float* beta, float* gam, float* mem_w_out, float* active,
                           float* next_out, void* rec, asrx_stream_t stream);
int asrx_msheath_ctrl_bwd2(const float* g_alpha, const float* g_beta, const float* g_gam, const float* g_mwo,
                           const float* mem_v, const float* mem_w, int64_t ld_mem_w, const float* mem,
                           const float* jump_s, const void* rec, int64_t layer_i, int64_t layers, int64_t B, int64_t D,
                           float* g_policy, int acc_policy, float* g_mem_v, float* g_mem_w, float* g_mem,
                           float* g_jump_s, int* has_orig, asrx_stream_t stream);
/* ctrl with mem = (1/L) sum of the asrx_axpy_row2_colsum chunk partials mem_part (written to mem) and
 * mem_v = sigmoid(mem . mg_w + mg_b) computed in the kernel (mem_gate, model.py:464; written to
 * mem_v_out); backward with mem_v's gradient fused (g_mem += ..., g_mg_w / g_mg_b accumulated). */
int asrx_msheath_ctrl_fwd3(const float* policy, const float* gpol, int64_t ld_gpol, const float* ion,
                           const float* mg_w, const float* mg_b, float* mem_v_out, const float* mem_w,
                           int64_t ld_mem_w, const float* mem_part, float* mem, const float* jump_s,
                           const float* next_i, int64_t layer_i, int64_t layers, int64_t B, int64_t L, int64_t D,
                           float* alpha, float* beta, float* gam, float* mem_w_out, float* active, float* next_out,
                           void* rec, asrx_stream_t stream);
int asrx_msheath_ctrl_bwd3(const float* g_alpha, const float* g_beta, const float* g_gam, const float* g_mwo,
                           const float* mem_v, const float* mem_w, int64_t ld_mem_w, const float* mem,
                           const float* jump_s, const void* rec, int64_t layer_i, int64_t layers, int64_t B, int64_t D,
                           float* g_policy, int acc_policy, float* g_mem_w, float* g_mem, float* g_jump_s,
                           int* has_orig, const float* mg_w, float* g_mg_w, float* g_mg_b, asrx_stream_t stream);
/* x_new = x + s1 s2 y and per-sample column sums of x_new in row chunks of 64: part (B,
 * asrx_mem_chunks(L), d), no atomics (deterministic forward), d <= 1024. */
int64_t asrx_mem_chunks(int64_t L);
int asrx_axpy_row2_colsum(const float* x, const float* s1, const float* s2, const float* y, float* out, float* part,
                          int64_t B, int64_t L, int64_t d, const float* next_i, int64_t layer, asrx_stream_t stream);
/* MSheath fused backward (asrx/msheath.py): jump_select backward in accumulate form (active: dxn =
 * alpha g, orig's gradient (+)= beta g on a jump; inactive: dx = g), the x_new/mem backward writing
 * x's gradient for active samples (g' = dxn + gm/L), and the final dx += orig grad + u broadcast. */
int asrx_jump_select4_bwd_acc(const float* g, const float* xn, const float* orig, const float* act,
                              const float* alpha, const float* beta, const int* has_orig, float* dxn, float* dorig,
                              float* dx, float* dalpha, float* dbeta, float* dgam, int64_t B, int64_t L, int64_t d,
                              asrx_stream_t stream);
int asrx_axpy_row2_bwd_acc(const float* dxn, const float* gm, float invL, const float* act, const float* s1,
                           const float* s2, const float* y, float* dy, float* ds1, float* ds2, float* dx, int64_t B,
                           int64_t L, int64_t d, asrx_stream_t stream);
/* Deterministic pair (round 4): asrx_jump_select4_bwd_acc writing its per-sample sums (dalpha, dbeta,
 * dgam) as per-(128-row L chunk, 128-column chunk) partials into `part` (asrx_jump_bwd_part_floats(B, L,
 * d) floats, fully written, no memset), and asrx_msheath_ctrl_bwd3 reading them from `part`, summed in
 * chunk order -- no float atomics on the data gradient's path (model.py:489-501 backward). */
int64_t asrx_jump_bwd_part_floats(int64_t B, int64_t L, int64_t d);
int asrx_jump_select4_bwd_part(const float* g, const float* xn, const float* orig, const float* act,
                               const float* alpha, const float* beta, const int* has_orig, float* dxn, float* dorig,
                               float* dx, float* part, int64_t B, int64_t L, int64_t d, asrx_stream_t stream);
int asrx_msheath_ctrl_bwd4(const float* part, int64_t L, const float* g_mwo, const float* mem_v, const float* mem_w,
                           int64_t ld_mem_w, const float* mem, const float* jump_s, const void* rec, int64_t layer_i,
                           int64_t layers, int64_t B, int64_t D, float* g_policy, int acc_policy, float* g_mem_w,
                           float* g_mem, float* g_jump_s, int* has_orig, const float* mg_w, float* g_mg_w,
                           float* g_mg_b, asrx_stream_t stream);

int asrx_msheath_dx_final(float* dx, const float* dorig, const int* has_orig, const float* u, int64_t B, int64_t L,
                          int64_t d, asrx_stream_t stream);

/* ---- MSheath.forward without a backward in ONE call (model.py:429-507; the reference's dead blocks,
 *      model.py:617-626, eval and decoding): enqueues asrx/msheath.py forward(save=False)'s launches from C++
 *      -- policy (seg_colsum_det, MPNet GEMM, small_linear softmax), per layer row_tiles, the v_gate projection
 *      GEMM, msheath_row_fwd2, the adapter GEMM, axpy_row2_colsum, msheath_ctrl_fwd3, jump_axpy_inplace, then
 *      layernorm_fwd3, the two MLP GEMMs and axpy_row -- bit-identical to issuing them one by one.  bf16 perf
 *      mode (wide GEMM, bf16 weight copies N x K contiguous).  The plan holds the module's constant addresses
 *      (parameters, the bf16 copies, v_gate's combined projection from asrx_vgate_weights); x0, y (B, L, D)
 *      fp32 contiguous and distinct; gpol (B, layers, 3) policy noise with row stride ld_gpol floats; ws: a device
 *      workspace of asrx_msheath_fwd_ws_bytes(plan, B, L, D) bytes.  The plan and layer structs are HOST memory
 *      read during the call only. */
typedef struct asrx_msheath_layer {
  const float *ln_w, *ln_b, *gate_w, *gate_b, *mval, *vw2, *vb2, *cw, *cb, *tx, *bc;
  const unsigned short *wcb;   /* bf16 [normalize(mkey); v_gate.mlp[0].weight] (M + Dh, D) */
  const unsigned short *ad_wb; /* bf16 adapter weight (D, D); NULL on odd layers */
  const float *ad_b;
  int64_t M, Dh;
  float ln_eps;
  int32_t px_bf16;
} asrx_msheath_layer;
typedef struct asrx_msheath_plan {
  const unsigned short *p0_wb;
  const float *p0_b, *p2_w, *p2_b;
  int64_t p_hidden;
  const float *mem_w, *mg_w, *mg_b, *jump_s, *mln_w, *mln_b;
  float mln_eps;
  int32_t hln_bf16;
  const float *mgate_w, *mgate_b;
  const unsigned short *m0_wb;
  const float *m0_b;
  const unsigned short *m2_wb;
  const float *m2_b;
  int64_t H1;
  int32_t a1_bf16, n_layers;
  const asrx_msheath_layer* layers;
} asrx_msheath_plan;
int64_t asrx_msheath_plan_bytes(void);
int64_t asrx_msheath_layer_bytes(void);
int64_t asrx_msheath_fwd_ws_bytes(const asrx_msheath_plan* plan, int64_t B, int64_t L, int64_t D);
int asrx_msheath_fwd(const asrx_msheath_plan* plan, const float* x0, const float* gpol, int64_t ld_gpol, float* y,
                     void* ws, int64_t ws_bytes, int64_t B, int64_t L, int64_t D, asrx_stream_t stream);
/* out = x + s1[r] * s2[r] * y (s2 may be NULL), d % 4 == 0 (model.py:461: x + gate * ion * out). */
int asrx_axpy_row2(const float* x, const float* s1, const float* s2, const float* y, float* out, int64_t rows,
                   int64_t d, asrx_stream_t stream);
int asrx_axpy_row2_bwd(const float* g, const float* s1, const float* s2, const float* y, float* dy, float* ds1,
                       float* ds2, int64_t rows, int64_t d, asrx_stream_t stream);
/* float4 forms of asrx_jump_select(_bwd) for d % 4 == 0 (the backward zeroes dalpha/dbeta/dgam: one
 * memset when they are one block [dalpha | dbeta | dgam], as asrx_jump_select4_bwd_acc too). */
/* No-grad MSheath layer step (dead blocks, eval, decoding): for samples at this layer
 * xout = alpha (xin + s1 s2 y) + beta orig + gam (x_new, model.py:461, and the jump select, 489-501, in
 * one pass, x_new never stored); in place (xin == xout) other samples are untouched, else copied. */
int asrx_jump_axpy_inplace(const float* xin, float* xout, const float* s1, const float* s2, const float* y,
                           const float* orig, const float* act, const float* alpha, const float* beta, const float* gam,
                           int64_t B, int64_t L, int64_t d, asrx_stream_t stream);
int asrx_jump_select4(const float* xn, const float* orig, const float* xold, const float* act, const float* alpha,
                      const float* beta, const float* gam, float* out, int64_t B, int64_t L, int64_t d,
                      asrx_stream_t stream);
int asrx_jump_select4_bwd(const float* g, const float* xn, const float* orig, const float* act, const float* alpha,
                          const float* beta, float* dxn, float* dorig, float* dxold, float* dalpha, float* dbeta,
                          float* dgam, int64_t B, int64_t L, int64_t d, asrx_stream_t stream);
int asrx_seg_colsum(const float* x, float* out, int64_t B, int64_t L, int64_t d, float scale, int accumulate,
                    asrx_stream_t stream);
int asrx_colsum(const float* x, float* out, int64_t rows, int64_t d, asrx_stream_t stream);
/* out (B, d) = scale sum_l x[b, l, :] without atomics (deterministic); part: B ceil(L/64) d floats */
int asrx_seg_colsum_det(const float* x, float* part, float* out, int64_t B, int64_t L, int64_t d, float scale,
                        asrx_stream_t stream);
/* out[c] += sum_r x[r * ld + c] (a column block of a wider row-major tensor) */
int asrx_colsum_ld(const float* x, int64_t ld, float* out, int64_t rows, int64_t d, asrx_stream_t stream);
int asrx_add_rows(const float* x, const float* t, const float* u, float* out, int64_t B, int64_t L, int64_t d,
                  asrx_stream_t stream);
int asrx_lincomb(const float* x, const float* y, const float* z, float a, float b, float c, float* out, int64_t n,
                 asrx_stream_t stream);
/* MSheath policy gumbel noise (model.py:476): out (B, layers, 3). */
int asrx_policy_noise(float* out, int64_t B, int64_t layers, int64_t sid_base, uint32_t key,
                      asrx_stream_t stream);

/* ---- encoder elementwise / conv pieces (model.py:93-147), channels-last (B, T, C) ------------- */
int asrx_act_fwd(const float* x, float* y, int64_t n, int act, asrx_stream_t stream);
int asrx_act_bwd(const float* g, const float* x, float* dx, int64_t n, int act, asrx_stream_t stream);
int asrx_glu_fwd(const float* x, float* y, int64_t rows, int64_t C, asrx_stream_t stream);
int asrx_glu_bwd(const float* g, const float* x, float* dx, int64_t rows, int64_t C, asrx_stream_t stream);
int asrx_dropout(const float* x, float* y, int64_t B, int64_t T, int64_t C, int64_t sid_base, uint32_t key,
                 float p, asrx_stream_t stream);
/* act then nn.Dropout(p) then act2 fused (encoder layer tail GELU -> Dropout, model.py:147, and the
 * next layer's leading GELU, model.py:143; act2 = 0 for none): y = act2(act(z) masked and scaled with
 * asrx_dropout's keyed mask) [+ res when res != NULL: ConvLite's residual, model.py:118];
 * bwd dz = g * act2'(.) * mask / (1 - p) * act'(z) (the residual's gradient is g itself).  C % 4 == 0. */
int asrx_act_dropout_fwd(const float* z, const float* res, float* y, int64_t B, int64_t T, int64_t C,
                         int64_t sid_base, uint32_t key, float p, int act, int act2, asrx_stream_t stream);
int asrx_act_dropout_bwd(const float* g, const float* z, float* dz, int64_t B, int64_t T, int64_t C,
                         int64_t sid_base, uint32_t key, float p, int act, int act2, asrx_stream_t stream);
int asrx_dwconv_fwd(const float* x, const float* w, const float* b, float* y, int64_t B, int64_t T, int64_t C,
                    int64_t K, asrx_stream_t stream);
int asrx_dwconv_bwd(const float* g, const float* x, const float* w, float* dx, float* dw, float* db, int64_t B,
                    int64_t T, int64_t C, int64_t K, asrx_stream_t stream);
int asrx_bn_fwd(const float* x, const float* w, const float* b, float* y, float* mean, float* rstd, int64_t B,
                int64_t T, int64_t C, float eps, int use_batch_stats, asrx_stream_t stream);
int asrx_bn_bwd(const float* g, const float* x, const float* mean, const float* rstd, const float* w, float* sg_ws,
                float* sgx_ws, float* dx, float* dw, float* db, int64_t B, int64_t T, int64_t C,
                asrx_stream_t stream);
int asrx_stem1_fwd(const float* x, const float* W, const float* bias, float* y, int64_t B, int64_t T, int64_t D,
                   asrx_stream_t stream);
int asrx_stem1_bwd(const float* g, const float* x, float* dW, float* db, int64_t B, int64_t T, int64_t D,
                   asrx_stream_t stream);

/* ---- token embedding (model.py:592, 606) and tied-logits cross entropy (model.py:629, 670) ---- */
int asrx_embed_fwd(const int64_t* ids, const float* E, float* y, int64_t rows, int64_t d, asrx_stream_t stream);
int asrx_embed_bwd(const int64_t* ids, const float* g, float* dE, int64_t rows, int64_t d, asrx_stream_t stream);
int asrx_ce_fwd(const float* z, const int64_t* labels, float* loss, float* lse, int64_t rows, int64_t V,
                asrx_stream_t stream);
int asrx_ce_bwd(const float* z, const int64_t* labels, const float* lse, const float* scale, float* dz,
                int64_t rows, int64_t V, asrx_stream_t stream);

/* ---- MaxFactor optimizer step: replaces MaxFactor.step, optimizerc.py:6-147 (the optimizer
 *      model.py:783-787 builds), for every parameter of the model in one call.  table: device array
 *      of np parameter records (layout and packing: asrx/optim.py; record size from
 *      asrx_maxfactor_param_bytes()); nrows / ncols / ncc / nmats: sizes of the flat row, (mat,
 *      col), (mat, col, 256-row chunk) and mat spaces; nitems: size of the wave-work-item space
 *      (each record's rows packed 64 / gsz to a wave); ws: float workspace of 4 np + 4 nrows +
 *      ncols + nmats.  Updates parameters and optimizer state in place. ----------------------------- */
int asrx_maxfactor_param_bytes(void);
int asrx_maxfactor_step(const void* table, int np, int64_t nrows, int64_t ncols, int64_t ncc, int64_t nmats,
                        int64_t nitems, float* ws, asrx_stream_t stream);


/* ---- step glue (csrc/stepops.hip): ops that ran as stock ATen kernels on the hot path ------------
 * Cross entropy (model.py:670, ignore_index 0): one-pass online log-sum-exp per row + on-device mean
 * (loss, count are device scalars); backward dz = (g/count)(softmax - onehot) with g the device
 * gradient of the loss, dz may alias z. */
int asrx_ce_fwd1(const float* z, const int64_t* labels, float* loss_r, float* lse, float* loss, float* count,
                 int64_t rows, int64_t V, asrx_stream_t stream);
int asrx_ce_bwd2(const float* z, const int64_t* labels, const float* lse, const float* g, const float* count, float* dz,
                 int64_t rows, int64_t V, asrx_stream_t stream);
/* Fused tied logits + cross entropy (perf mode; model.py:629 logits, model.py:670 F.cross_entropy):
 * asrx_gemm_wn_ce (csrc/gemm_wn.hip) writes the logits bf16 and per row / 128*nj-column tile the
 * (max, sum exp) of the tile's bf16 logits (part: rows x nparts float2, nparts = ceil(V / (128 nj)));
 * asrx_ce_part_fwd merges them into lse and the loss (reads the label's logit only); asrx_ce_bwd_bf16
 * writes dz = (g/count)(softmax - onehot) bf16 from the bf16 logits.  A label outside [0, V) gives a
 * NaN loss / gradient (the reference raises). */
int asrx_gemm_wn_ce(const void* A, int64_t lda, const unsigned short* W, int64_t ldw, unsigned short* Zb, int64_t ldc,
                    float* part, int64_t M, int64_t N, int64_t K, int nj, asrx_stream_t stream);
int asrx_ce_part_fwd(const float* part, int64_t nparts, const unsigned short* zb, const int64_t* labels, float* loss_r,
                     float* lse, float* loss, float* count, int64_t rows, int64_t V, asrx_stream_t stream);
int asrx_ce_bwd_bf16(const unsigned short* zb, const int64_t* labels, const float* lse, const float* g,
                     const float* count, unsigned short* dzb, int64_t rows, int64_t V, asrx_stream_t stream);
/* The same with the logits stored fp32 (the drop-in boundary's logits dtype, model.py:629 .float(); the
 * default of Model.forward): statistics of the fp32 values, the label's fp32 logit, dz from fp32 logits.
 * The loss is NaN when every label is ignored (F.cross_entropy's mean over zero rows, model.py:670);
 * ignored rows get a zero gradient. */
int asrx_gemm_wn_ce_f32(const void* A, int64_t lda, const unsigned short* W, int64_t ldw, float* Zf, int64_t ldc,
                        float* part, int64_t M, int64_t N, int64_t K, int nj, asrx_stream_t stream);
int asrx_ce_part_fwd_f32(const float* part, int64_t nparts, const float* zf, const int64_t* labels, float* loss_r,
                         float* lse, float* loss, float* count, int64_t rows, int64_t V, asrx_stream_t stream);
int asrx_ce_bwd_f32in(const float* zf, const int64_t* labels, const float* lse, const float* g, const float* count,
                      unsigned short* dzb, int64_t rows, int64_t V, asrx_stream_t stream);
/* out projection with its residual add (model.py:578-580): C = R + A W^T + bias; A, C, R fp32, R != C,
 * 16-byte aligned rows, nj 1 or 3. */
/* Backward of y = act(A W^T + bias), act gelu (1) / silu (2) / sigmoid (3), whose forward kept no pre-activation:
   the GEMM recomputes z with the forward's tile width (nj 3) and writes gz = bf16(G * act'(z)) (M x N, ldc) from
   the output gradient G (fp32, row stride ldg), adding gz's column sums into db when non-NULL.  A fp32
   (a_bf16 = 0) or bf16 (1).  Replaces storing z in the forward and re-reading it (asrx_act_bwd_bias). */
int asrx_gemm_wn_gact(const void* A, int a_bf16, int64_t lda, const unsigned short* W, int64_t ldw, const float* bias,
                      const float* G, int64_t ldg, unsigned short* gz, int64_t ldc, float* db, int64_t M, int64_t N,
                      int64_t K, int act, int nj, asrx_stream_t stream);
/* q / k projection with its rotary fused (model.py:242-245 / 261, then model.py:198-214 with the hd^-0.25 scale of
 * model.py:303-304): C = rot(A W^T + bias) -- each head's pairs (2j, 2j+1) times polar(scale * m[row],
 * angle(row % L, j)) from tab ((positions >= L) x hd/2 float2 (cos, sin), asrx_rotary_table); bit-identical to
 * asrx_gemm_wn_ex followed by asrx_rotary_fwd2.  Z (nullable) receives the unrotated product.  A fp32 (a_bf16 = 0)
 * or bf16 (1); C, Z, tab 16-byte aligned; N % hd == 0, hd % 4 == 0; nj 1 or 3.  Replaces the rotary pass over
 * the projection's output (its fp32 write and re-read). */
int asrx_gemm_wn_rot(const void* A, int a_bf16, int64_t lda, const unsigned short* W, int64_t ldw, float* C, float* Z,
                     int64_t ldc, const float* bias, const float* m, const float* tab, int64_t L, int64_t hd,
                     float scale, int64_t M, int64_t N, int64_t K, int nj, asrx_stream_t stream);
/* Plain bf16 product on the vendor GEMM library (hipBLASLt; round 6): Y (M x N, ldc; fp32, or bf16 with c_bf16) =
 * alpha A W^T + bias + beta Y for a bf16-stored activation A (M x K, lda) and bf16 weight W (N x K, ldw), bias fp32
 * or NULL -- no other epilogue.  asrx/gemm.py routes the shapes where the library measured faster than the wide GEMM
 * (K >= 768, >= 16384 rows; profiles/r06_blaslt_vs_wide.txt).  Replaces nn.Linear's forward / input gradient at
 * those shapes (model.py:573-574 MLP down projection, 505 MSheath MLP, their input gradients). */
int asrx_gemm_lt(const void* A, int64_t lda, const unsigned short* W, int64_t ldw, void* C, int c_bf16, int64_t ldc,
                 const float* bias, int64_t M, int64_t N, int64_t K, float alpha, float beta, asrx_stream_t stream);
int asrx_gemm_wn_res(const float* A, int64_t lda, const unsigned short* W, int64_t ldw, float* C, int64_t ldc,
                     const float* bias, const float* R, int64_t ldr, int64_t M, int64_t N, int64_t K, int nj,
                     asrx_stream_t stream);
/* act(x W^T + b) backward in perf mode (model.py:147, 505, 573): gz = g * act'(z) stored bf16 (rows x N,
 * it only feeds the gradient GEMMs) and db += column sums of gz (fp32; db may be NULL); act gelu /
 * silu / sigmoid, N % 4 == 0. */
int asrx_act_bwd_bias(const float* g, const float* z, unsigned short* gz, float* db, int64_t rows, int64_t N, int act,
                      asrx_stream_t stream);
/* asrx_wgrad_bf16 with dY stored bf16 (M, lda % 8) and X stored fp32 (b_bf16 = 0) or bf16 (1: N, ldb % 8):
 * the tied token embedding's gradient from the bf16 logits gradient, weight gradients under an
 * activation (asrx_act_bwd_bias). */
int asrx_wgrad_bf16_ab(const void* A, int64_t lda, const void* B, int b_bf16, int64_t ldb, float* C, int64_t ldc,
                       int64_t M, int64_t N, int64_t R, int64_t splitk, asrx_stream_t stream);
/* dW += dY^T X and db += column sums of dY in one pass (bias gradient of y = x W^T + b, replacing the
 * nn.Linear backward's separate bias reduction; model.py Linear layers): dY fp32 (a_bf16 = 0) or bf16 (1),
 * X fp32 (b_bf16 = 0) or bf16 (1), shapes as asrx_wgrad_bf16_ex / _ab. */
int asrx_wgrad_bias(const void* A, int a_bf16, int64_t lda, const void* B, int b_bf16, int64_t ldb, float* C,
                    int64_t ldc, float* db, int64_t M, int64_t N, int64_t R, int64_t splitk, asrx_stream_t stream);
/* BatchNorm1d running statistics from per-clip (B, C) mean / rstd (ConvLite.bn, model.py:101);
 * nbt (num_batches_tracked, int64) may be NULL.  asrx_rsqrt_eps: eval-mode rstd. */
int asrx_bn_running(const float* mean, const float* rstd, float* rm, float* rv, int64_t* nbt, int64_t B, int64_t C,
                    int64_t T, float eps, float momentum, asrx_stream_t stream);
int asrx_rsqrt_eps(const float* v, float* out, int64_t n, float eps, asrx_stream_t stream);
/* k3 Conv1d weight (Co, Ci, 3), weight-normed when g != NULL (W = g v/|v|, model.py:140), into the
 * implicit-im2col GEMM layouts: Wt (Co, 3Ci) k-major and Wf (Ci, 3Co) flipped, fp32 and/or bf16 (each
 * may be NULL); nrm (Co) = |v| per channel.  Backward from dWt (Co, 3Ci): dg, dv accumulated. */
int asrx_conv3_weight(const float* g, const float* v, int64_t Co, int64_t Ci, float* Wt, unsigned short* Wtb, float* Wf,
                      unsigned short* Wfb, float* nrm, asrx_stream_t stream);
int asrx_conv3_weight_bwd(const float* dWt, const float* g, const float* v, const float* nrm, int64_t Co, int64_t Ci,
                          float* dg, float* dv, asrx_stream_t stream);
/* processor output blend (model.py:628): out = s d + (1-s) g, s = sigmoid(blend); backward writes dd,
 * dg (each may be NULL) and accumulates d blend. */
int asrx_blend_fwd(const float* d, const float* g, const float* blend, float* out, int64_t n, asrx_stream_t stream);
int asrx_blend_bwd(const float* go, const float* d, const float* g, const float* blend, float* dd, float* dg,
                   float* dblend, int64_t n, asrx_stream_t stream);
/* dst_k += src[k n .. (k+1) n) for k < nseg <= 3; asrx_cat3: out = [a; b; c] (c may be NULL). */
int asrx_add_segments(const float* src, int64_t n, float* d0, float* d1, float* d2, int64_t nseg, asrx_stream_t stream);
int asrx_cat3(const float* a, const float* b, const float* c, int64_t n, float* out, asrx_stream_t stream);


/* ---- pitch: pyworld dio + stonemask as extract_features calls them
 *      (essentials.py:451-455), float64 on the device over B equal-length float32 clips.  Filter
 *      taps and the band table come from asrx/pitch.py (lc: 2c+1 low-cut taps; nut: the bands' Nuttall
 *      windows, band i at nut_off[i] with nut_len[i] taps; nut_off / nut_len / bf0 are HOST arrays of
 *      nb entries).  Workspace: mean (B), hp (B, N+1+2c), f (B, N+1), ev (B, 4, cap), cand / score
 *      (B, nb, F), work (B, 3F); f0 (B, F) out, F = 1 + 1000 N / fs / fp.  stonemask refines f0 at the
 *      uniform frame times j fp / 1000. */
int asrx_pitch_dio(const float* x, int64_t ldx, int64_t B, int64_t N, double fs, double f0_floor, double f0_ceil,
                   double fp, double allowed_range, const double* lc, int64_t c, const double* nut,
                   const int64_t* nut_off, const int64_t* nut_len, const double* bf0, int64_t nb, double* mean,
                   double* hp, double* f, double* ev, int64_t cap, double* cand, double* score, double* work,
                   double* f0, int64_t F, asrx_stream_t stream);
int asrx_pitch_stonemask(const float* x, int64_t ldx, int64_t B, int64_t N, double fs, const double* f0, double fp,
                         int64_t F, double* out, asrx_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* ASRX_H */
