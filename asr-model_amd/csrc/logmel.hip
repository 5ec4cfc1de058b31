// Log-mel front end, replacing the spectrogram and waveform branches of extract_features
// (essentials.py:469-491 and 493-510):
//
//   torchaudio MelSpectrogram(n_fft=1024, hop=160, periodic Hann, center=True zero pad 512,
//   power 2, 128 HTK mels 50-8000 Hz, norm=None)  ->  clamp(1e-10).log10()
//   -> maximum(x, max(x) - 8)  (max over the whole clip)  ->  (x + 4) / 4
//   adaptive_avg_pool1d(audio, N/160)  (exact 160-sample block means when 160 | N)
//
// Kernel 1 (logmel_frames): one workgroup = 4 waves = FPB consecutive frames of one clip.  The
// (FPB-1)*160 + 1024 samples those frames touch are staged once in LDS (each sample is re-used
// 6.4x by overlapping windows), so HBM sees every input byte once.  Each wave turns one frame at a
// time into a 512-point complex FFT (even/odd packing of the 1024 real samples), runs three radix-8
// Stockham passes through a per-wave LDS ping-pong, untangles the real spectrum, forms |X|^2 on the
// 513 bins and applies the sparse filterbank (<= 32 bins per band).  log10 values are staged in LDS
// and written with coalesced stores in either (B, F, 128) or (B, 128, F) layout; the per-clip max
// goes to an ordered-int atomicMax.  The fused waveform pool reads the same LDS samples.
// Kernel 2 (logmel_finalize): x -> (max(x, clipmax - 8) + 4) / 4 in place.
#include "common.h"
#include "fft.h"

using asrx_fft::cpx;

namespace asrx {

constexpr int MEL_NFFT = 1024, MEL_HOP = 160, MEL_NBINS = 513, MEL_BANDS = 128, MEL_FBW = 32;
constexpr int MEL_FPB = 32;  // frames per workgroup
constexpr int MEL_SAMP = (MEL_FPB - 1) * MEL_HOP + MEL_NFFT;

// consts layout (floats): window[1024] | tw512[512] (re,im) | tw1024[513] (re,im)
struct MelConsts {
  const float* win;
  const cpx* tw512;
  const cpx* tw1024;
};

__global__ __launch_bounds__(256) void logmel_frames_kernel(
    const float* __restrict__ wav, int64_t N, int64_t ld_wav, int64_t F, const float* __restrict__ consts,
    const float* __restrict__ fbw, const int* __restrict__ fbs, float* __restrict__ out, int layout,
    int64_t ld_out, int* __restrict__ clip_max, float* __restrict__ pool, int64_t T_pool) {
  __shared__ __attribute__((aligned(16))) float samp[MEL_SAMP];
  __shared__ __attribute__((aligned(16))) cpx fbuf[4][2][512];
  __shared__ float melst[MEL_FPB][MEL_BANDS + 1];
  __shared__ float red[4];

  const int b = blockIdx.y;
  const int64_t f0 = (int64_t)blockIdx.x * MEL_FPB;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const float* x = wav + b * ld_wav;
  MelConsts C{consts, reinterpret_cast<const cpx*>(consts + MEL_NFFT),
              reinterpret_cast<const cpx*>(consts + MEL_NFFT + 1024)};

  // 1. stage samples [f0*160 - 512, f0*160 - 512 + MEL_SAMP) (zero outside the clip)
  const int64_t g0 = f0 * MEL_HOP - MEL_NFFT / 2;
  for (int i = tid; i < MEL_SAMP; i += 256) {
    const int64_t g = g0 + i;
    samp[i] = (g >= 0 && g < N) ? x[g] : 0.f;
  }
  __syncthreads();

  // 2. fused waveform feature: exact 160-sample block means (pool index == frame index)
  if (pool) {
    for (int fi = wid; fi < MEL_FPB; fi += 4) {
      const int64_t f = f0 + fi;
      if (f >= T_pool) break;
      const int base = MEL_NFFT / 2 + fi * MEL_HOP;
      float s = samp[base + lane] + samp[base + lane + 64] + (lane < 32 ? samp[base + lane + 128] : 0.f);
      s = wave_sum(s);
      if (lane == 0) pool[b * T_pool + f] = s * (1.0f / MEL_HOP);
    }
  }

  float lmax = -3.0e38f;
  cpx* b0 = fbuf[wid][0];
  cpx* b1 = fbuf[wid][1];
  for (int fi = wid; fi < MEL_FPB; fi += 4) {
    const int64_t f = f0 + fi;  // wave-uniform
    const bool live = f < F;
    const int base = fi * MEL_HOP;
    // 3. pack windowed real frame as z[n] = x[2n] w[2n] + i x[2n+1] w[2n+1], lane j holds n = j + 64 r
    cpx v[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const int n = lane + 64 * r;
      const float2 s2 = *reinterpret_cast<const float2*>(&samp[base + 2 * n]);
      const float2 w2 = *reinterpret_cast<const float2*>(&C.win[2 * n]);
      v[r] = cpx{s2.x * w2.x, s2.y * w2.y};
    }
    // 4. three radix-8 Stockham passes
    asrx_fft::stockham_pass(lane, 1, v, b0, C.tw512);
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 8; ++r) v[r] = b0[lane + 64 * r];
    asrx_fft::stockham_pass(lane, 8, v, b1, C.tw512);
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 8; ++r) v[r] = b1[lane + 64 * r];
    asrx_fft::stockham_pass(lane, 64, v, b0, C.tw512);
    __syncthreads();
    // 5. real-FFT untangle + power spectrum into b1 (reused as float[513])
    float* pw = reinterpret_cast<float*>(b1);
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const int k = lane + 64 * r;
      const cpx zk = b0[k];
      const cpx zn = b0[(512 - k) & 511];
      // E = (Zk + conj(Zn)) / 2 ; O = (Zk - conj(Zn)) / (2i)
      const cpx e{0.5f * (zk.x + zn.x), 0.5f * (zk.y - zn.y)};
      const cpx o{0.5f * (zk.y + zn.y), -0.5f * (zk.x - zn.x)};
      const cpx t = asrx_fft::cmul(C.tw1024[k], o);
      const float re = e.x + t.x, im = e.y + t.y;
      pw[k] = re * re + im * im;
    }
    if (lane == 0) {
      const cpx z0 = b0[0];
      const float nyq = z0.x - z0.y;
      pw[512] = nyq * nyq;
    }
    __syncthreads();
    // 6. sparse filterbank (two bands per lane) + log10(clamp(., 1e-10))
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int m = lane + 64 * h;
      const int s = fbs[m];
      const float* w = fbw + m * MEL_FBW;
      float acc = 0.f;
#pragma unroll 8
      for (int i = 0; i < MEL_FBW; ++i) {
        const int bin = s + i;
        acc += w[i] * pw[bin < MEL_NBINS ? bin : MEL_NBINS - 1];
      }
      const float lv = (float)log10((double)fmaxf(acc, 1e-10f));  // correctly rounded like libm
      melst[fi][m] = lv;
      if (live) lmax = fmaxf(lmax, lv);
    }
    __syncthreads();
  }

  // 7. coalesced output of the staged log10 block
  if (layout == 0) {  // (B, F, 128): row f contiguous
    for (int i = tid; i < MEL_FPB * MEL_BANDS; i += 256) {
      const int fi = i / MEL_BANDS, m = i % MEL_BANDS;
      const int64_t f = f0 + fi;
      if (f < F) out[b * ld_out + f * MEL_BANDS + m] = melst[fi][m];
    }
  } else {  // (B, 128, F): each band's FPB frames contiguous
    for (int i = tid; i < MEL_FPB * MEL_BANDS; i += 256) {
      const int m = i / MEL_FPB, fi = i % MEL_FPB;
      const int64_t f = f0 + fi;
      if (f < F) out[b * ld_out + m * F + f] = melst[fi][m];
    }
  }
  lmax = wave_max(lmax);
  if (lane == 0) red[wid] = lmax;
  __syncthreads();
  if (tid == 0) {
    const float bm = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    atomicMax(clip_max + b, float_to_ordered(bm));
  }
}

__global__ void logmel_finalize_kernel(float* __restrict__ out, int64_t per_clip, int64_t ld_out,
                                       const int* __restrict__ clip_max) {
  const int b = blockIdx.y;
  const float floor_v = ordered_to_float(clip_max[b]) - 8.0f;
  float* o = out + b * ld_out;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < per_clip;
       i += (int64_t)gridDim.x * blockDim.x) {
    o[i] = (fmaxf(o[i], floor_v) + 4.0f) * 0.25f;
  }
}

__global__ void fill_int_kernel(int* p, int n, int v) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = v;
}

}  // namespace asrx

using namespace asrx;

// wav: (B, N) rows at stride ld_wav.  out: (B, F, 128) if layout == 0 else (B, 128, F), clip stride
// ld_out (>= 128*F).  clip_max_ws: int workspace of B entries (overwritten).  pool: (B, T_pool) or
// null; the fused pool requires N == 160 * T_pool.
extern "C" int asrx_logmel(const float* wav, int64_t B, int64_t N, int64_t ld_wav, const float* consts,
                           const float* fbw, const int* fbs, float* out, int layout, int64_t ld_out,
                           int* clip_max_ws, float* pool, int64_t T_pool, hipStream_t stream) {
  ASRX_REQUIRE(B > 0 && N > 0, "asrx_logmel: empty input");
  ASRX_REQUIRE(B < 65536, "asrx_logmel: too many clips");
  const int64_t F = 1 + N / MEL_HOP;
  ASRX_REQUIRE(ld_out >= F * MEL_BANDS, "asrx_logmel: ld_out too small");
  ASRX_REQUIRE(!pool || N == (int64_t)MEL_HOP * T_pool,
               "asrx_logmel: fused pool needs N == 160*T_pool (N=%ld T=%ld)", (long)N, (long)T_pool);
  fill_int_kernel<<<(unsigned)((B + 255) / 256), 256, 0, stream>>>(clip_max_ws, (int)B,
                                                                   float_to_ordered(-3.0e38f));
  dim3 g((unsigned)((F + MEL_FPB - 1) / MEL_FPB), (unsigned)B);
  logmel_frames_kernel<<<g, 256, 0, stream>>>(wav, N, ld_wav, F, consts, fbw, fbs, out, layout, ld_out,
                                              clip_max_ws, pool, T_pool);
  int64_t per_clip = F * MEL_BANDS;
  unsigned gx = (unsigned)std::min<int64_t>((per_clip + 255) / 256, 64);
  logmel_finalize_kernel<<<dim3(gx, (unsigned)B), 256, 0, stream>>>(out, per_clip, ld_out, clip_max_ws);
  ASRX_LAUNCHED("asrx_logmel");
}

extern "C" int asrx_mel_frames(int64_t N) { return (int)(1 + N / MEL_HOP); }
