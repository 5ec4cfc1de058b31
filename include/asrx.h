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

/* ---- log-mel front end: replaces torchaudio MelSpectrogram + log10 + clip-max floor,
 *      essentials.py:469-491, and the waveform adaptive_avg_pool1d, essentials.py:493-510 -------- */
int asrx_mel_frames(int64_t n_samples); /* 1 + N/160 (host) */
/* wav (B,N) at row stride ld_wav; consts = window|tw512|tw1024 (see asrx/mel.py); fbw (128,32)
 * band weights and fbs[128] int32 start bins of the sparse HTK filterbank; out (B,F,128) when
 * layout==0 or (B,128,F) when layout==1, clip stride ld_out; clip_max_ws int32[B] workspace;
 * pool (B,T_pool) or NULL (needs N == 160*T_pool). */
int asrx_logmel(const float* wav, int64_t B, int64_t N, int64_t ld_wav, const float* consts,
                const float* fbw, const int* fbs, float* out, int layout, int64_t ld_out,
                int* clip_max_ws, float* pool, int64_t T_pool, asrx_stream_t stream);

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

#ifdef __cplusplus
}
#endif
#endif /* ASRX_H */
