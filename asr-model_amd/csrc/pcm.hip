// load_wave's scaling and peak normalisation (essentials.py:301-313) for a batch of decoded clips,
// on the GPU after one H2D copy of the packed int32 PCM (replaces the
// per-sample CPU normalisation + .to(cuda:0) inside the Dataset, essentials.py:491):
//   x = pcm * 2^-(bits-1)                       soundfile.read(path, dtype='float32')
//   mono:  x / max|x|            (if > 0)       essentials.py:310-312
//   multi: x[c] / max(x[c])      (if any > 0)   essentials.py:305-307 -- the per-channel MAX of x,
//                                               not of |x|, is the reference's own quirk, kept
// pcm (B, C, ld) int32 (decoded FLAC / integer PCM) or fp32 (is_float: float WAV, scale 1), lengths
// (B) int64, scale (B) float; out (B, C, ld_out) fp32, zero past each clip's length.  One workgroup per
// clip: a max reduction over its channels, then the scaled write.
#include "common.h"

namespace asrx {

constexpr int PCM_T = 256;

template <typename T>
__global__ __launch_bounds__(PCM_T) void pcm_normalize_kernel(const T* __restrict__ pcm, int64_t C, int64_t ld,
                                                              const int64_t* __restrict__ lengths,
                                                              const float* __restrict__ scale,
                                                              float* __restrict__ out, int64_t ld_out, int normalize) {
  __shared__ float red[PCM_T / 64];
  __shared__ float cmax[8];
  const int b = blockIdx.x;
  const int64_t n = lengths[b];
  const float s = scale[b];
  const T* src = pcm + (int64_t)b * C * ld;
  float* dst = out + (int64_t)b * C * ld_out;
  for (int c = 0; c < C; ++c) {
    float m = C == 1 ? 0.f : -INFINITY;
    for (int64_t i = threadIdx.x; i < n; i += PCM_T) {
      const float x = (float)src[c * ld + i] * s;
      m = C == 1 ? fmaxf(m, fabsf(x)) : fmaxf(m, x);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
      float t = red[0];
      for (int w = 1; w < PCM_T / 64; ++w) t = fmaxf(t, red[w]);
      cmax[c] = t;
    }
    __syncthreads();
  }
  bool any = false;
  for (int c = 0; c < C; ++c) any = any || cmax[c] > 0.f;
  for (int c = 0; c < C; ++c) {
    const float m = cmax[c];
    const bool div = normalize && any;
    for (int64_t i = threadIdx.x; i < ld_out; i += PCM_T) {
      float x = 0.f;
      if (i < n) {
        x = (float)src[c * ld + i] * s;
        if (div) x = x / m;
      }
      dst[c * ld_out + i] = x;
    }
  }
}

}  // namespace asrx

extern "C" int asrx_pcm_normalize(const void* pcm, int is_float, int64_t B, int64_t C, int64_t ld,
                                  const int64_t* lengths, const float* scale, float* out, int64_t ld_out, int normalize,
                                  hipStream_t stream) {
  ASRX_REQUIRE(C >= 1 && C <= 8, "asrx_pcm_normalize: 1..8 channels");
  ASRX_REQUIRE(ld_out >= 1 && ld >= 1, "asrx_pcm_normalize: empty rows");
  if (B == 0) return 0;
  if (is_float)
    asrx::pcm_normalize_kernel<float><<<(unsigned)B, asrx::PCM_T, 0, stream>>>(
        static_cast<const float*>(pcm), C, ld, lengths, scale, out, ld_out, normalize);
  else
    asrx::pcm_normalize_kernel<int><<<(unsigned)B, asrx::PCM_T, 0, stream>>>(
        static_cast<const int*>(pcm), C, ld, lengths, scale, out, ld_out, normalize);
  ASRX_LAUNCHED("asrx_pcm_normalize");
}
