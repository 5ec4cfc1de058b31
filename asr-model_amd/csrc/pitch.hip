// GPU pitch: the reference's extract_features(pitch=True) runs pyworld's
// dio + stonemask per clip on the CPU (essentials.py:451-455).  Here a batch of equal-length clips is
// processed in float64 on the device (oracle/pitch.py restates the algorithm and is the checker):
//   pitch_mean      DC of y = [x, 0] (y_length = N + 1, WORLD's layout)            one WG per clip
//   pitch_highpass  hp = y (*) zero-phase 50 Hz low-cut filter, on [-c, y_length + c)   LDS-tiled
//   per band:  pitch_lowpass  f = hp (*) Nuttall(4 h), delay 2 h compensated           LDS-tiled
//              pitch_band     negative / positive zero crossings, peaks, dips of f (block scan),
//                             interval series interpolated to the frame times, candidate + score
//   pitch_fix       best band per frame, FixF0Contour steps 1-4                      one WG per clip
//   stonemask       per frame: Blackman window of 3 periods + its central difference, DFT at the
//                   first min(fs/2/f0, 6) harmonic bins, instantaneous-frequency mean  one wave/frame
// WORLD filters by FFT products over a zero-padded buffer large enough that no circular wrap
// reaches the signal; the same filters are applied here as direct linear convolutions (equal up to
// float64 rounding).  Workspace is the caller's (asrx/pitch.py sizes it).
#include "common.h"

namespace asrx {

namespace {

constexpr int PT = 512;  // outputs per workgroup in the convolutions (256 threads, 2 each)

__device__ __forceinline__ double block_sum_d(double v, double* red) {
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  double t = 0.0;
  const int nw = (blockDim.x + 63) >> 6;
  for (int i = 0; i < nw; ++i) t += red[i];
  return t;
}

__device__ __forceinline__ int64_t mround(double x) { return x >= 0 ? (int64_t)floor(x + 0.5) : -(int64_t)floor(-x + 0.5); }

}  // namespace

__global__ __launch_bounds__(256) void pitch_mean_kernel(const float* __restrict__ x, int64_t ldx, int64_t N,
                                                         double* __restrict__ mean) {
  __shared__ double red[4];
  const float* xb = x + (int64_t)blockIdx.x * ldx;
  double s = 0.0;
  for (int64_t i = threadIdx.x; i < N; i += 256) s += (double)xb[i];
  s = block_sum_d(s, red);
  if (threadIdx.x == 0) mean[blockIdx.x] = s / (double)(N + 1);
}

// hp[b][m], m in [0, ext = y_length + 2c): n = m - c; hp = sum_{k=-c..c} h[k + c] y(n - k)
__global__ __launch_bounds__(256) void pitch_highpass_kernel(const float* __restrict__ x, int64_t ldx, int64_t N,
                                                             const double* __restrict__ mean,
                                                             const double* __restrict__ h, int c,
                                                             double* __restrict__ hp, int64_t ext) {
  extern __shared__ double sm[];
  double* seg = sm;                // PT + 2c samples of y starting at m0 - 2c
  double* hs = sm + PT + 2 * c;    // 2c + 1 taps
  const int b = blockIdx.y;
  const int64_t m0 = (int64_t)blockIdx.x * PT;
  const float* xb = x + (int64_t)b * ldx;
  const double mu = mean[b];
  for (int j = threadIdx.x; j < PT + 2 * c; j += 256) {
    const int64_t i = m0 - 2 * c + j;
    seg[j] = (i >= 0 && i < N) ? (double)xb[i] - mu : (i == N ? -mu : 0.0);
  }
  for (int j = threadIdx.x; j < 2 * c + 1; j += 256) hs[j] = h[j];
  __syncthreads();
  for (int t = threadIdx.x; t < PT; t += 256) {
    const int64_t m = m0 + t;
    if (m >= ext) break;
    double acc = 0.0;
    for (int k = -c; k <= c; ++k) acc += hs[k + c] * seg[t + c - k];
    hp[(int64_t)b * ext + m] = acc;
  }
}

// f[b][i] = sum_{k<L4} w[k] HP(i + h2 - k), HP(n) = hp[n + c] on [-c, ylen + c), 0 elsewhere
__global__ __launch_bounds__(256) void pitch_lowpass_kernel(const double* __restrict__ hp, int64_t ext, int c,
                                                            int64_t ylen, const double* __restrict__ w, int L4, int h2,
                                                            double* __restrict__ f) {
  extern __shared__ double sm[];
  double* seg = sm;               // PT + L4 - 1 values of HP starting at i0 + h2 - (L4 - 1)
  double* ws = sm + PT + L4 - 1;  // L4 taps
  const int b = blockIdx.y;
  const int64_t i0 = (int64_t)blockIdx.x * PT;
  const double* hb = hp + (int64_t)b * ext;
  const int64_t s0 = i0 + h2 - (L4 - 1);
  for (int j = threadIdx.x; j < PT + L4 - 1; j += 256) {
    const int64_t n = s0 + j;
    seg[j] = (n >= -c && n < ylen + c) ? hb[n + c] : 0.0;
  }
  for (int j = threadIdx.x; j < L4; j += 256) ws[j] = w[j];
  __syncthreads();
  for (int t = threadIdx.x; t < PT; t += 256) {
    const int64_t i = i0 + t;
    if (i >= ylen) break;
    double acc = 0.0;
    for (int k = 0; k < L4; ++k) acc += ws[k] * seg[t + (L4 - 1) - k];
    f[(int64_t)b * ylen + i] = acc;
  }
}

// Event series of one band (WORLD GetFourZeroCrossingIntervals + GetF0CandidateContour).  One
// workgroup per clip; ev holds 4 x cap fine edges per clip.
__device__ __forceinline__ bool pitch_event(const double* s, int64_t ylen, int type, int64_t i, double& fine) {
  // type 0: negative-going zero crossings of f; 1: of -f; 2: of d = f[i+1] - f[i] (peaks); 3: of -d
  double a, b;
  if (type < 2) {
    if (i + 1 >= ylen) return false;
    a = s[i];
    b = s[i + 1];
  } else {
    if (i + 2 >= ylen) return false;
    a = s[i + 1] - s[i];
    b = s[i + 2] - s[i + 1];
  }
  if (type & 1) {
    a = -a;
    b = -b;
  }
  if (!(0.0 < a && b <= 0.0)) return false;
  fine = (double)(i + 1) - a / (b - a);
  return true;
}

__global__ __launch_bounds__(1024) void pitch_band_kernel(const double* __restrict__ f, int64_t ylen, double fs,
                                                          double* __restrict__ ev, int64_t cap, int F, double fp,
                                                          double bf0, double f0_floor, double f0_ceil,
                                                          double* __restrict__ cand, double* __restrict__ score,
                                                          int band, int nb) {
  __shared__ int wsum[16];
  __shared__ int ncnt[4];
  const int b = blockIdx.x;
  const double* s = f + (int64_t)b * ylen;
  double* evb = ev + (int64_t)b * 4 * cap;
  const int64_t per = (ylen + 1023) / 1024;
  const int64_t i0 = (int64_t)threadIdx.x * per, i1 = min<int64_t>(i0 + per, ylen);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int type = 0; type < 4; ++type) {
    int cnt = 0;
    double fine;
    for (int64_t i = i0; i < i1; ++i) cnt += pitch_event(s, ylen, type, i, fine) ? 1 : 0;
    int v = cnt;  // inclusive wave scan, then across the 16 waves
    for (int o = 1; o < 64; o <<= 1) {
      const int u = __shfl_up(v, o);
      if (lane >= o) v += u;
    }
    if (lane == 63) wsum[wv] = v;
    __syncthreads();
    int off = v - cnt;
    for (int k = 0; k < wv; ++k) off += wsum[k];
    if (threadIdx.x == 0) {
      int tot = 0;
      for (int k = 0; k < 16; ++k) tot += wsum[k];
      ncnt[type] = tot;
    }
    double* dst = evb + type * cap;
    for (int64_t i = i0; i < i1 && off < cap; ++i)
      if (pitch_event(s, ylen, type, i, fine)) dst[off++] = fine;
    __syncthreads();
  }
  int n[4];
  bool ok = true;
  for (int type = 0; type < 4; ++type) {
    n[type] = (int)min<int64_t>(ncnt[type], cap);
    ok = ok && (n[type] - 1 - 2 > 0);  // CheckEvent(number_of_intervals - 2)
  }
  double* cb = cand + ((int64_t)b * nb + band) * F;
  double* sb = score + ((int64_t)b * nb + band) * F;
  for (int j = threadIdx.x; j < F; j += 1024) {
    if (!ok) {
      cb[j] = 0.0;
      sb[j] = 100000.0;
      continue;
    }
    const double t = (double)j * fp / 1000.0;
    double v[4];
    for (int type = 0; type < 4; ++type) {
      const double* fe = evb + type * cap;
      const int ni = n[type] - 1;  // intervals: loc[q] = (fe[q] + fe[q+1]) / 2 / fs, iv[q] = fs / (fe[q+1] - fe[q])
      // k = first q with loc[q] > t (searchsorted right), clamped to [1, ni - 1]
      int lo = 0, hi = ni;
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if ((fe[mid] + fe[mid + 1]) / 2.0 / fs <= t) lo = mid + 1;
        else hi = mid;
      }
      const int k = min(max(lo, 1), ni - 1);
      const double xa = (fe[k - 1] + fe[k]) / 2.0 / fs, xb = (fe[k] + fe[k + 1]) / 2.0 / fs;
      const double ya = fs / (fe[k] - fe[k - 1]), yb = fs / (fe[k + 1] - fe[k]);
      v[type] = ya + (t - xa) / (xb - xa) * (yb - ya);
    }
    double cm = (v[0] + v[1] + v[2] + v[3]) / 4.0;
    double sc = sqrt(((v[0] - cm) * (v[0] - cm) + (v[1] - cm) * (v[1] - cm) + (v[2] - cm) * (v[2] - cm) +
                      (v[3] - cm) * (v[3] - cm)) / 3.0);
    if (cm > bf0 || cm < bf0 / 2.0 || cm > f0_ceil || cm < f0_floor) {
      cm = 0.0;
      sc = 100000.0;
    }
    cb[j] = cm;
    sb[j] = sc;
  }
}

__device__ double pitch_select(double ref, const double* cand, int nb, int64_t F, int64_t j, double ar) {
  double best = 0.0, err = ar;
  for (int i = 0; i < nb; ++i) {
    const double c = cand[i * F + j];
    const double e = fabs(ref - c) / ref;
    if (e > err) continue;
    best = c;
    err = e;
  }
  return best;
}

// Best band per frame + FixF0Contour.  One workgroup per clip; s1..s4 are per-clip workspace rows.
__global__ __launch_bounds__(256) void pitch_fix_kernel(const double* __restrict__ cand,
                                                        const double* __restrict__ score, int nb, int F,
                                                        double fp, double f0_floor, double ar,
                                                        double* __restrict__ work, double* __restrict__ f0) {
  const int b = blockIdx.x;
  const double* cb = cand + (int64_t)b * nb * F;
  const double* sb = score + (int64_t)b * nb * F;
  double* best = work + (int64_t)b * 3 * F;
  double* s1 = best + F;
  double* s2 = s1 + F;
  double* out = f0 + (int64_t)b * F;
  for (int j = threadIdx.x; j < F; j += 256) {
    int bi = 0;
    double bs = sb[j];
    for (int i = 1; i < nb; ++i)
      if (bs > sb[(int64_t)i * F + j]) {
        bi = i;
        bs = sb[(int64_t)i * F + j];
      }
    best[j] = cb[(int64_t)bi * F + j];
  }
  __syncthreads();
  const int vmin = (int)(0.5 + 1000.0 / fp / f0_floor) * 2 + 1;
  if (F <= vmin) {
    for (int j = threadIdx.x; j < F; j += 256) out[j] = best[j];
    return;
  }
  auto base = [&](int i) { return (i < vmin || i >= F - vmin) ? 0.0 : best[i]; };
  for (int i = threadIdx.x; i < F; i += 256) {
    double v = 0.0;
    if (i >= vmin) {
      const double bi = base(i), bp = base(i - 1);
      v = fabs((bi - bp) / (1e-12 + bi)) < ar ? bi : 0.0;
    }
    s1[i] = v;
  }
  __syncthreads();
  const int c = (vmin - 1) / 2;
  for (int i = threadIdx.x; i < F; i += 256) {
    double v = s1[i];
    if (i >= c && i < F - c)
      for (int j = -c; j <= c; ++j)
        if (s1[i + j] == 0.0) {
          v = 0.0;
          break;
        }
    s2[i] = v;
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  // steps 3 / 4 walk the voiced sections sequentially (in place on `out`)
  for (int i = 0; i < F; ++i) out[i] = s2[i];
  // step 3: from each section's last voiced frame forwards (limit: the next section's end)
  int next_neg = -1;
  for (int i = 1; i < F; ++i) {
    if (!(s2[i] == 0.0 && s2[i - 1] != 0.0)) continue;
    const int start = i - 1;
    int nn = -1;
    for (int q = i + 1; q < F; ++q)
      if (s2[q] == 0.0 && s2[q - 1] != 0.0) {
        nn = q - 1;
        break;
      }
    const int limit = nn < 0 ? F - 1 : nn;
    for (int j = start; j < limit; ++j) {
      out[j + 1] = pitch_select(out[j], cb, nb, F, j + 1, ar);
      if (out[j + 1] == 0.0) break;
    }
    (void)next_neg;
  }
  // step 4: from each section's first voiced frame backwards, last section first
  int prev_pos = -1;
  for (int i = F - 1; i >= 1; --i) {
    if (!(s2[i - 1] == 0.0 && s2[i] != 0.0)) continue;
    int pp = -1;
    for (int q = i - 1; q >= 1; --q)
      if (s2[q - 1] == 0.0 && s2[q] != 0.0) {
        pp = q;
        break;
      }
    const int limit = pp < 0 ? 1 : pp;
    for (int j = i; j > limit; --j) {
      out[j - 1] = pitch_select(out[j], cb, nb, F, j - 1, ar);
      if (out[j - 1] == 0.0) break;
    }
    (void)prev_pos;
  }
}

// StoneMask: one wave per (clip, frame)
__global__ __launch_bounds__(256) void stonemask_kernel(const float* __restrict__ x, int64_t ldx, int64_t N, double fs,
                                                        const double* __restrict__ f0in, double fp, int F,
                                                        double* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t fr = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int b = blockIdx.y;
  if (fr >= F) return;
  const double f = f0in[(int64_t)b * F + fr];
  if (f <= 40.0 || f > fs / 12.0) {
    if (lane == 0) out[(int64_t)b * F + fr] = 0.0;
    return;
  }
  const float* xb = x + (int64_t)b * ldx;
  const double t = (double)fr * fp / 1000.0;
  const int half = (int)(1.5 * fs / f + 1.0);
  const int wl = 2 * half + 1;
  const double wlt = (2.0 * half + 1.0) / fs;
  const double fft = pow(2.0, 2.0 + (int)(log(half * 2.0 + 1.0) / log(2.0)));
  const int nh = min((int)(fs / 2.0 / f), 6);
  int64_t kb[6];
  for (int h = 0; h < 6; ++h) kb[h] = h < nh ? mround(f * fft / fs * (h + 1)) : 0;
  double mr[6], mi[6], dr[6], di[6];
  for (int h = 0; h < 6; ++h) mr[h] = mi[h] = dr[h] = di[h] = 0.0;
  auto mwin = [&](int n) {
    const double bt = (double)(n - half) / fs;
    return 0.42 + 0.5 * cos(2.0 * M_PI * bt / wlt) + 0.08 * cos(4.0 * M_PI * bt / wlt);
  };
  for (int n = lane; n < wl; n += 64) {
    const double bt = (double)(n - half) / fs;
    int64_t idx = mround((t + bt) * fs) - 1;
    idx = idx < 0 ? 0 : (idx > N - 1 ? N - 1 : idx);
    const double xv = (double)xb[idx];
    const double m = mwin(n);
    const double d = n == 0 ? -mwin(1) / 2.0 : (n == wl - 1 ? mwin(wl - 2) / 2.0 : -(mwin(n + 1) - mwin(n - 1)) / 2.0);
    for (int h = 0; h < nh; ++h) {
      double sn, cs;
      sincospi(2.0 * (double)((kb[h] * (int64_t)n) % (int64_t)fft) / fft, &sn, &cs);
      mr[h] += xv * m * cs;
      mi[h] -= xv * m * sn;
      dr[h] += xv * d * cs;
      di[h] -= xv * d * sn;
    }
  }
  for (int h = 0; h < nh; ++h)
    for (int o = 32; o >= 1; o >>= 1) {
      mr[h] += __shfl_xor(mr[h], o);
      mi[h] += __shfl_xor(mi[h], o);
      dr[h] += __shfl_xor(dr[h], o);
      di[h] += __shfl_xor(di[h], o);
    }
  if (lane != 0) return;
  double amp = 0.0, ifs = 0.0;
  for (int h = 0; h < nh; ++h) {
    const double pw = mr[h] * mr[h] + mi[h] * mi[h];
    const double num = mr[h] * di[h] - mi[h] * dr[h];
    const double inst = pw == 0.0 ? 0.0 : (double)kb[h] * fs / fft + num / pw * fs / 2.0 / M_PI;
    const double a = sqrt(pw);
    amp += a * (h + 1);
    ifs += a * inst;
  }
  const double mf = ifs / (amp + 1e-12);
  out[(int64_t)b * F + fr] = fabs(mf - f) > f * 0.2 ? f : mf;
}

}  // namespace asrx

using namespace asrx;

extern "C" {

// DIO over B equal-length clips x (B x N float32, row stride ldx) on the device.  taps: lc (2c+1
// low-cut taps), nut (concatenated Nuttall windows, band i at nut_off[i] with nut_len[i] taps,
// host arrays of nb entries), bf0 (nb boundary f0s, host).  Workspace: mean (B), hp (B, N + 1 + 2c),
// f (B, N + 1), ev (B, 4, cap), cand / score (B, nb, F), work (B, 3F) doubles.  f0 (B, F) out.
int asrx_pitch_dio(const float* x, int64_t ldx, int64_t B, int64_t N, double fs, double f0_floor, double f0_ceil,
                   double fp, double allowed_range, const double* lc, int64_t c, const double* nut,
                   const int64_t* nut_off, const int64_t* nut_len, const double* bf0, int64_t nb, double* mean,
                   double* hp, double* f, double* ev, int64_t cap, double* cand, double* score, double* work,
                   double* f0, int64_t F, hipStream_t stream) {
  if (B == 0 || N == 0) return 0;
  const int64_t ylen = N + 1, ext = ylen + 2 * c;
  ASRX_REQUIRE(c >= 0 && (PT + 4 * c + 1) * 8 <= 60000, "asrx_pitch_dio: low-cut filter too long");
  pitch_mean_kernel<<<(unsigned)B, 256, 0, stream>>>(x, ldx, N, mean);
  {
    dim3 g((unsigned)((ext + PT - 1) / PT), (unsigned)B);
    const size_t shm = (size_t)(PT + 2 * c + 2 * c + 1) * sizeof(double);
    pitch_highpass_kernel<<<g, 256, shm, stream>>>(x, ldx, N, mean, lc, (int)c, hp, ext);
  }
  for (int64_t i = 0; i < nb; ++i) {
    const int L4 = (int)nut_len[i];
    ASRX_REQUIRE((PT + 2 * L4) * 8 <= 160000, "asrx_pitch_dio: Nuttall window too long (f0_floor too low)");
    dim3 g((unsigned)((ylen + PT - 1) / PT), (unsigned)B);
    const size_t shm = (size_t)(PT + 2 * L4) * sizeof(double);
    if (shm > 65536) (void)hipFuncSetAttribute((const void*)pitch_lowpass_kernel,
                                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
    pitch_lowpass_kernel<<<g, 256, shm, stream>>>(hp, ext, (int)c, ylen, nut + nut_off[i], L4, L4 / 2, f);
    pitch_band_kernel<<<(unsigned)B, 1024, 0, stream>>>(f, ylen, fs, ev, cap, (int)F, fp, bf0[i], f0_floor, f0_ceil,
                                                        cand, score, (int)i, (int)nb);
  }
  pitch_fix_kernel<<<(unsigned)B, 256, 0, stream>>>(cand, score, (int)nb, (int)F, fp, f0_floor, allowed_range, work,
                                                    f0);
  ASRX_LAUNCHED("asrx_pitch_dio");
}

int asrx_pitch_stonemask(const float* x, int64_t ldx, int64_t B, int64_t N, double fs, const double* f0, double fp,
                         int64_t F, double* out, hipStream_t stream) {
  if (B == 0 || F == 0) return 0;
  dim3 g((unsigned)((F + 3) / 4), (unsigned)B);
  stonemask_kernel<<<g, 256, 0, stream>>>(x, ldx, N, fs, f0, fp, (int)F, out);
  ASRX_LAUNCHED("asrx_pitch_stonemask");
}

}  // extern "C"
