// Log-mel front end, replacing the spectrogram and waveform branches of extract_features
// (essentials.py:469-491 and 493-510):
//
//   torchaudio MelSpectrogram(n_fft=1024, hop=160, periodic Hann, center=True zero pad 512,
//   power 2, 128 HTK mels 50-8000 Hz, norm=None)  ->  clamp(1e-10).log10()
//   -> maximum(x, max(x) - 8)  (max over the whole clip)  ->  (x + 4) / 4
//   adaptive_avg_pool1d(audio, N/160)  (exact 160-sample block means when 160 | N)
//
// Kernel 1 (logmel_tiles): a tile is MEL_FPT consecutive frames of one clip; the (FPT-1)*160+1024
// samples a tile touches are staged once in LDS (each sample re-used 6.4x by the overlapping
// windows), so HBM sees every input byte about once.  Workgroups are persistent over a contiguous
// run of tiles (XCD-aware block order, so neighbouring tiles — which share 864 samples — stay in
// one XCD's L2) and prefetch the next tile's samples into registers while the current one is
// transformed.  Each wave owns one frame at a time and never synchronises with the other waves
// inside a frame: per frame it
//   * packs the windowed real frame as z[n] = x[2n] w[2n] + i x[2n+1] w[2n+1] (lane j holds
//     n = j + 64 r, r = 0..7; the window values are lane constants kept in VGPRs),
//   * runs a 512-point complex FFT as three radix-8 Stockham passes whose twiddles are lane
//     constants in VGPRs; the two inter-pass transposes go through a per-wave LDS buffer padded
//     with one slot every 8 (p(i) = i + i/8) so the stride-8 writes are bank-conflict free,
//   * untangles the real spectrum (lane j already holds Z[j + 64 r]; only the mirrored Z[512-k]
//     is read back) and forms 4|X_k|^2 (the factor 4 is folded into the filterbank weights),
//   * applies the sparse filterbank: lane m owns bands m (<= FB_LO taps) and m + 64 (<= FB_HI
//     taps) with the weights in VGPRs, reading the power bins by immediate LDS offsets,
//   * takes log10 as log2 * log10(2) (v_log_f32).
// Per tile the block stages the 128 x FPT log values in LDS, writes them with coalesced stores in
// (B, F, 128) or (B, 128, F) layout and folds its maximum into the clip's ordered-int atomicMax.
// The fused waveform pool reads the same LDS samples.
// Kernel 2 (logmel_finalize): x -> (max(x, clipmax - 8) + 4) / 4 in place, float4.
#include "../../../asr-model_amd/csrc/common.h"
#include "../../../asr-model_amd/csrc/fft.h"

using asrx_fft::cpx;

namespace asrx {

constexpr int MEL_NFFT = 1024, MEL_HOP = 160, MEL_NBINS = 513, MEL_BANDS = 128, MEL_FBW = 32;
constexpr int FB_A = 8, FB_B = 24;  // taps of a lane's two bands (see lane_filterbank in mel.py)
constexpr int FB_QUADS = (FB_A + FB_B) / 4;
constexpr int MEL_WAVES = 4;
constexpr int MEL_FPT = 16;  // frames per tile
constexpr int MEL_TSAMP = (MEL_FPT - 1) * MEL_HOP + MEL_NFFT;  // 3424 samples per tile
constexpr int MEL_TSAMP4 = MEL_TSAMP / 4;                      // 856 float4
constexpr int MEL_PF = (MEL_TSAMP4 + 255) / 256;               // prefetch float4 per thread
constexpr int FFT_SLOTS = 512 + 64 + 8;                        // padded cpx slots per wave
static_assert(MEL_TSAMP % 4 == 0, "tile samples must be float4 aligned");

__constant__ float kRot[8][2] = {
    {1.0f, 0.0f},
    {0.92387953251128674f, -0.38268343236508978f},
    {0.70710678118654757f, -0.70710678118654757f},
    {0.38268343236508984f, -0.92387953251128674f},
    {0.0f, -1.0f},
    {-0.38268343236508973f, -0.92387953251128674f},
    {-0.70710678118654746f, -0.70710678118654768f},
    {-0.92387953251128674f, -0.38268343236508989f}};

__device__ __forceinline__ int pidx(int i) { return i + (i >> 3); }

// Orders this wave's LDS accesses (the LDS unit executes one wave's DS instructions in order;
// this only stops the compiler from moving them across the exchange point).
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
}

// Explicit ds_read_b64 (2 LDS cycles per wave, 256 B/clk): left to itself the compiler merges pairs
// of these reads into ds_read2_b64 / ds_read2st64_b64, which the LDS services at half the rate
// (MI355X_MICROARCH.md LDS table).  The loads are issued back to back and completed by one
// lgkmcnt(0) wait that also names every destination, so no use can be scheduled before it.
typedef float f2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t lds_off(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}
template <int OFF>
__device__ __forceinline__ f2v ds_rd64(uint32_t a) {
  f2v r;
  asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(r) : "v"(a), "i"(OFF) : "memory");
  return r;
}
// eight b64 reads at base + OFF0 + r * STRIDE bytes, r = 0..7
template <int OFF0, int STRIDE>
__device__ __forceinline__ void ds_rd64x8(uint32_t a, f2v (&o)[8]) {
  o[0] = ds_rd64<OFF0>(a);
  o[1] = ds_rd64<OFF0 + STRIDE>(a);
  o[2] = ds_rd64<OFF0 + 2 * STRIDE>(a);
  o[3] = ds_rd64<OFF0 + 3 * STRIDE>(a);
  o[4] = ds_rd64<OFF0 + 4 * STRIDE>(a);
  o[5] = ds_rd64<OFF0 + 5 * STRIDE>(a);
  o[6] = ds_rd64<OFF0 + 6 * STRIDE>(a);
  o[7] = ds_rd64<OFF0 + 7 * STRIDE>(a);
  asm volatile("s_waitcnt lgkmcnt(0)"
               : "+v"(o[0]), "+v"(o[1]), "+v"(o[2]), "+v"(o[3]), "+v"(o[4]), "+v"(o[5]), "+v"(o[6]), "+v"(o[7])
               :
               : "memory");
}

template <int OFF0, int STRIDE>
__device__ __forceinline__ void ds_rd64x4(uint32_t a, f2v (&o)[4]) {
  o[0] = ds_rd64<OFF0>(a);
  o[1] = ds_rd64<OFF0 + STRIDE>(a);
  o[2] = ds_rd64<OFF0 + 2 * STRIDE>(a);
  o[3] = ds_rd64<OFF0 + 3 * STRIDE>(a);
  asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(o[0]), "+v"(o[1]), "+v"(o[2]), "+v"(o[3]) : : "memory");
}

__device__ __forceinline__ void dft8_tw(cpx (&v)[8], const cpx (&tw)[7]) {
#pragma unroll
  for (int r = 1; r < 8; ++r) v[r] = asrx_fft::cmul(v[r], tw[r - 1]);
  asrx_fft::dft8(v);
}

// contiguous run of tiles per workgroup; consecutive runs on one XCD (blocks are dealt to the 8
// XCDs round-robin by blockIdx)
__device__ __forceinline__ int xcd_block(int bid, int G) {
  const int per = G / 8, rem = G % 8, x = bid % 8, q = bid / 8;
  return (x < rem ? x * (per + 1) : rem * (per + 1) + (x - rem) * per) + q;
}

__global__ __launch_bounds__(256, 3) void logmel_tiles_kernel(
    const float* __restrict__ wav, int64_t N, int64_t ld_wav, int vec_ok, int64_t F, int tiles_per_clip,
    int64_t n_tiles, int tiles_per_block, const float* __restrict__ consts, const float* __restrict__ fbw,
    const int* __restrict__ fbs, float* __restrict__ out, int layout, int64_t ld_out,
    int* __restrict__ clip_max, float* __restrict__ pool, int64_t T_pool) {
  __shared__ __attribute__((aligned(16))) float samp[MEL_TSAMP];
  __shared__ __attribute__((aligned(16))) cpx fbuf[MEL_WAVES][FFT_SLOTS];
  __shared__ float melst[MEL_FPT][MEL_BANDS + 1];
  __shared__ float red[MEL_WAVES];
  __shared__ float4 fbw_s[FB_QUADS * 64];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int64_t t_begin = (int64_t)xcd_block(blockIdx.x, gridDim.x) * tiles_per_block;
  if (t_begin >= n_tiles) return;
  const int64_t t_end = t_begin + tiles_per_block < n_tiles ? t_begin + tiles_per_block : n_tiles;

  // ---- lane constants: window, pass-2/3 twiddles, untangle twiddles, filterbank rows
  const float* win = consts;
  const cpx* tw512 = reinterpret_cast<const cpx*>(consts + MEL_NFFT);
  const cpx* tw1024 = reinterpret_cast<const cpx*>(consts + MEL_NFFT + 1024);
  float2 wv[8];
  cpx t2[7], t3[7];
#pragma unroll
  for (int r = 0; r < 8; ++r) wv[r] = *reinterpret_cast<const float2*>(win + 2 * (lane + 64 * r));
  const cpx tu0 = tw1024[lane];
#pragma unroll
  for (int r = 1; r < 8; ++r) {
    t2[r - 1] = tw512[(r * (lane & 7) * 8) & 511];
    t3[r - 1] = tw512[(r * lane) & 511];
  }
  // lane-packed filterbank (asrx/mel.py lane_filterbank): lane m owns band_a (<= 8 taps from the
  // even bin sa) and band_b (<= 24 taps from the even bin sb); weights [tap/4][lane][4] in LDS
  const int band_a = fbs[lane], band_b = fbs[64 + lane];
  const int sa2 = fbs[128 + lane] >> 1, sb2 = fbs[192 + lane] >> 1;
  for (int i = tid; i < FB_QUADS * 64; i += 256) fbw_s[i] = reinterpret_cast<const float4*>(fbw)[i];

  cpx* S = fbuf[wid];
  float* P = reinterpret_cast<float*>(S);

  // ---- sample prefetch (registers) for tile t; the bounds test is per tile (wave-uniform)
  float4 pf[MEL_PF];
  auto prefetch = [&](int64_t t) {
    const int64_t b = t / tiles_per_clip;
    const int64_t f0 = (t - b * tiles_per_clip) * MEL_FPT;
    const int64_t g0 = f0 * MEL_HOP - MEL_NFFT / 2;
    const float* x = wav + b * ld_wav + g0;
    if (vec_ok && g0 >= 0 && g0 + MEL_TSAMP <= N) {
      const float4* x4 = reinterpret_cast<const float4*>(x);
#pragma unroll
      for (int q = 0; q < MEL_PF; ++q) {
        const int i4 = tid + 256 * q;
        pf[q] = i4 < MEL_TSAMP4 ? x4[i4] : make_float4(0.f, 0.f, 0.f, 0.f);
      }
    } else {
#pragma unroll
      for (int q = 0; q < MEL_PF; ++q) {
        const int i4 = tid + 256 * q;
        float e[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const int64_t g = g0 + 4 * i4 + c;
          e[c] = (i4 < MEL_TSAMP4 && g >= 0 && g < N) ? x[4 * i4 + c] : 0.f;
        }
        pf[q] = make_float4(e[0], e[1], e[2], e[3]);
      }
    }
  };
  prefetch(t_begin);

#pragma unroll 1
  for (int64_t t = t_begin; t < t_end; ++t) {
    const int64_t b = t / tiles_per_clip;
    const int64_t f0 = (t - b * tiles_per_clip) * MEL_FPT;
    __syncthreads();  // the previous tile's readers are done with samp / melst
#pragma unroll
    for (int q = 0; q < MEL_PF; ++q) {
      const int i4 = tid + 256 * q;
      if (i4 < MEL_TSAMP4) reinterpret_cast<float4*>(samp)[i4] = pf[q];
    }
    __syncthreads();
    if (t + 1 < t_end) prefetch(t + 1);

    // fused waveform feature: exact 160-sample block means (pool index == frame index)
    if (pool) {
      for (int fi = wid; fi < MEL_FPT; fi += MEL_WAVES) {
        const int64_t f = f0 + fi;
        if (f >= T_pool) break;
        const int base = MEL_NFFT / 2 + fi * MEL_HOP;
        float s = samp[base + lane] + samp[base + lane + 64] + (lane < 32 ? samp[base + lane + 128] : 0.f);
        s = wave_sum(s);
        if (lane == 0) pool[b * T_pool + f] = s * (1.0f / MEL_HOP);
      }
    }

    float lmax = -3.0e38f;
#pragma unroll 1
    for (int fi = wid; fi < MEL_FPT; fi += MEL_WAVES) {
      const bool live = f0 + fi < F;  // wave-uniform
      cpx v[8];
      {
        f2v sv[8];
        ds_rd64x8<0, 512>(lds_off(samp + fi * MEL_HOP + 2 * lane), sv);
#pragma unroll
        for (int r = 0; r < 8; ++r) v[r] = cpx{sv[r].x * wv[r].x, sv[r].y * wv[r].y};
      }
      // pass 1 (Ns = 1): out[8j + r]
      asrx_fft::dft8(v);
#pragma unroll
      for (int r = 0; r < 8; ++r) S[9 * lane + r] = v[r];
      wave_lds_sync();
      {
        f2v t[8];
        ds_rd64x8<0, 576>(lds_off(S + pidx(lane)), t);
#pragma unroll
        for (int r = 0; r < 8; ++r) v[r] = cpx{t[r].x, t[r].y};
      }
      wave_lds_sync();
      // pass 2 (Ns = 8): out[(j/8)*64 + j%8 + 8r]
      dft8_tw(v, t2);
#pragma unroll
      for (int r = 0; r < 8; ++r) S[72 * (lane >> 3) + (lane & 7) + 9 * r] = v[r];
      wave_lds_sync();
      {
        f2v t[8];
        ds_rd64x8<0, 576>(lds_off(S + pidx(lane)), t);
#pragma unroll
        for (int r = 0; r < 8; ++r) v[r] = cpx{t[r].x, t[r].y};
      }
      wave_lds_sync();
      // pass 3 (Ns = 64): out[j + 64 r] = Z[j + 64 r], kept in v
      dft8_tw(v, t3);
      // third exchange unpadded: the R-pattern writes and the mirrored reads are conflict-free
      // without padding (lane 0 also stores Z_0 at 512, the mirror of its r = 0 slot)
#pragma unroll
      for (int r = 0; r < 8; ++r) S[lane + 64 * r] = v[r];
      if (lane == 0) S[512] = v[0];
      wave_lds_sync();
      f2v zm[8];  // zm[r] = Z[(512 - lane - 64 r) & 511] = S[64 - lane + 64 (7 - r)]
      ds_rd64x8<0, 512>(lds_off(S + 64 - lane), zm);
      // real-FFT untangle: 2 X_k = (Z_k + conj Z_{512-k}) + W1024^k (-i)(Z_k - conj Z_{512-k})
      float pw[8];
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        const cpx zn{zm[7 - r].x, zm[7 - r].y};
        const cpx zk = v[r];
        const cpx e{zk.x + zn.x, zk.y - zn.y};
        const cpx o{zk.y + zn.y, zn.x - zk.x};
        // W1024^(j + 64 r) = W1024^j * exp(-i pi r / 8)
        const cpx tt = asrx_fft::cmul(asrx_fft::cmul(tu0, cpx{kRot[r][0], kRot[r][1]}), o);
        const float re = e.x + tt.x, im = e.y + tt.y;
        pw[r] = re * re + im * im;  // 4 |X_k|^2
      }
      wave_lds_sync();
#pragma unroll
      for (int r = 0; r < 8; ++r) P[lane + 64 * r] = pw[r];
      if (lane < 16) {
        const float nyq = 2.0f * (v[0].x - v[0].y);  // lane 0: 2 X_512 = 2 (Re Z0 - Im Z0)
        P[512 + lane] = lane == 0 ? nyq * nyq : 0.f;  // bins past 512 are zero pads for the taps
      }
      wave_lds_sync();
      // sparse filterbank (weights carry the 1/4; bins read in even-aligned pairs)
      static_assert(FB_A == 8 && FB_B == 24, "the filterbank reads below are written out for 8 + 24 taps");
      f2v pa[4], pb[8], pc[4];  // bins sa .. sa+7 | sb .. sb+15 | sb+16 .. sb+23
      ds_rd64x4<0, 8>(lds_off(P + 2 * sa2), pa);
      ds_rd64x8<0, 8>(lds_off(P + 2 * sb2), pb);
      ds_rd64x4<64, 8>(lds_off(P + 2 * sb2), pc);
      float acc_a = 0.f, acc_b = 0.f;
#pragma unroll
      for (int q = 0; q < FB_A / 4; ++q) {
        const float4 wq = fbw_s[q * 64 + lane];
        const f2v p0 = pa[2 * q], p1 = pa[2 * q + 1];
        acc_a = fmaf(wq.x, p0.x, fmaf(wq.y, p0.y, fmaf(wq.z, p1.x, fmaf(wq.w, p1.y, acc_a))));
      }
#pragma unroll
      for (int q = 0; q < FB_B / 4; ++q) {
        const float4 wq = fbw_s[(FB_A / 4 + q) * 64 + lane];
        const f2v p0 = q < 4 ? pb[2 * q] : pc[2 * (q - 4)], p1 = q < 4 ? pb[2 * q + 1] : pc[2 * (q - 4) + 1];
        acc_b = fmaf(wq.x, p0.x, fmaf(wq.y, p0.y, fmaf(wq.z, p1.x, fmaf(wq.w, p1.y, acc_b))));
      }
      wave_lds_sync();
      // clamp(1e-10).log10(): the clamped value maps to exactly -10 like the correctly rounded
      // library log10; elsewhere log2 * log10(2) is within a few ulp
      const float l_a = acc_a <= 1e-10f ? -10.0f : __builtin_amdgcn_logf(acc_a) * 0.30102999566398120f;
      const float l_b = acc_b <= 1e-10f ? -10.0f : __builtin_amdgcn_logf(acc_b) * 0.30102999566398120f;
      melst[fi][band_a] = l_a;
      melst[fi][band_b] = l_b;
      if (live) lmax = fmaxf(lmax, fmaxf(l_a, l_b));
    }
    lmax = wave_max(lmax);
    if (lane == 0) red[wid] = lmax;
    __syncthreads();

    // coalesced output of the staged block
    float* o = out + b * ld_out;
    if (layout == 0) {  // (B, F, 128): the tile is FPT contiguous rows of 128
      for (int i = tid; i < MEL_FPT * MEL_BANDS / 4; i += 256) {
        const int fi = i / (MEL_BANDS / 4), m4 = (i % (MEL_BANDS / 4)) * 4;
        if (f0 + fi < F) {
          const float* src = &melst[fi][m4];
          *reinterpret_cast<float4*>(o + (f0 + fi) * MEL_BANDS + m4) = make_float4(src[0], src[1], src[2], src[3]);
        }
      }
    } else {  // (B, 128, F): each band's FPT frames contiguous
      for (int i = tid; i < MEL_FPT * MEL_BANDS; i += 256) {
        const int m = i / MEL_FPT, fi = i % MEL_FPT;
        if (f0 + fi < F) o[m * F + f0 + fi] = melst[fi][m];
      }
    }
    if (tid == 0) {
      float bm = red[0];
#pragma unroll
      for (int w = 1; w < MEL_WAVES; ++w) bm = fmaxf(bm, red[w]);
      atomicMax(clip_max + b, float_to_ordered(bm));
    }
  }
}

__global__ void logmel_finalize_kernel(float* __restrict__ out, int64_t per_clip, int64_t ld_out,
                                       const int* __restrict__ clip_max, int vec) {
  const int b = blockIdx.y;
  const float floor_v = ordered_to_float(clip_max[b]) - 8.0f;
  float* o = out + b * ld_out;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  if (vec) {
    float4* o4 = reinterpret_cast<float4*>(o);
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < per_clip / 4; i += stride) {
      float4 v = o4[i];
      v.x = (fmaxf(v.x, floor_v) + 4.0f) * 0.25f;
      v.y = (fmaxf(v.y, floor_v) + 4.0f) * 0.25f;
      v.z = (fmaxf(v.z, floor_v) + 4.0f) * 0.25f;
      v.w = (fmaxf(v.w, floor_v) + 4.0f) * 0.25f;
      o4[i] = v;
    }
  } else {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < per_clip; i += stride)
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
// null; the fused pool requires N == 160 * T_pool.  fbw/fbs: the lane-packed filterbank of
// asrx/mel.py lane_filterbank: fbs = band_a[64] | band_b[64] | start_a[64] | start_b[64] (even
// starts), fbw = weights [8 tap quads][64 lanes][4] (taps 0-7 band_a, 8-31 band_b, x 1/4).
extern "C" int asrx_logmel(const float* wav, int64_t B, int64_t N, int64_t ld_wav, const float* consts,
                           const float* fbw, const int* fbs, float* out, int layout, int64_t ld_out,
                           int* clip_max_ws, float* pool, int64_t T_pool, hipStream_t stream) {
  ASRX_REQUIRE(B > 0 && N > 0, "asrx_logmel: empty input");
  ASRX_REQUIRE(B < (1 << 24), "asrx_logmel: too many clips");
  const int64_t F = 1 + N / MEL_HOP;
  ASRX_REQUIRE(ld_out >= F * MEL_BANDS, "asrx_logmel: ld_out too small");
  ASRX_REQUIRE(layout != 0 || (ld_out % 4 == 0 && (reinterpret_cast<uintptr_t>(out) & 15) == 0),
               "asrx_logmel: (B, F, 128) layout needs 16-byte aligned rows");
  ASRX_REQUIRE(!pool || N == (int64_t)MEL_HOP * T_pool,
               "asrx_logmel: fused pool needs N == 160*T_pool (N=%ld T=%ld)", (long)N, (long)T_pool);
  fill_int_kernel<<<(unsigned)((B + 255) / 256), 256, 0, stream>>>(clip_max_ws, (int)B,
                                                                   float_to_ordered(-3.0e38f));
  const int tiles_per_clip = (int)((F + MEL_FPT - 1) / MEL_FPT);
  const int64_t n_tiles = B * tiles_per_clip;
  // 3 resident workgroups per CU (168 VGPRs, 48.8 KB LDS) on 256 CUs; each takes a contiguous run
  const int64_t slots = 256 * 3;
  const int tiles_per_block = (int)std::max<int64_t>(1, (n_tiles + slots - 1) / slots);
  const int64_t grid = (n_tiles + tiles_per_block - 1) / tiles_per_block;
  const int vec_ok = (ld_wav % 4 == 0) && ((reinterpret_cast<uintptr_t>(wav) & 15) == 0);
  logmel_tiles_kernel<<<(unsigned)grid, 256, 0, stream>>>(wav, N, ld_wav, vec_ok, F, tiles_per_clip, n_tiles,
                                                          tiles_per_block, consts, fbw, fbs, out, layout, ld_out,
                                                          clip_max_ws, pool, T_pool);
  const int64_t per_clip = F * MEL_BANDS;
  const int vec = (ld_out % 4 == 0) && ((reinterpret_cast<uintptr_t>(out) & 15) == 0);
  const unsigned gx = (unsigned)std::min<int64_t>((per_clip / (vec ? 4 : 1) + 255) / 256, 96);
  logmel_finalize_kernel<<<dim3(gx, (unsigned)B), 256, 0, stream>>>(out, per_clip, ld_out, clip_max_ws, vec);
  ASRX_LAUNCHED("asrx_logmel");
}

extern "C" int asrx_mel_frames(int64_t N) { return (int)(1 + N / MEL_HOP); }

// ---------------------------------------------------------------------------------------------
// Waveform feature for any clip length (essentials.py:493-510): adaptive_avg_pool1d(audio, T) with
// T = int(N / 160) bins, bin i = mean of samples [floor(i N / T), ceil((i + 1) N / T)) -- the general
// case of the fused pool above (which needs 160 | N).  One wave per bin: the <= 161-sample window is
// read coalesced, summed in a wave reduction, and divided once.
namespace asrx {
__global__ __launch_bounds__(256) void wave_pool_kernel(const float* __restrict__ wav, int64_t N, int64_t ld_wav,
                                                        int64_t T, int64_t B, float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); w < B * T; w += nw) {
    const int64_t b = w / T, i = w % T;
    const int64_t s = (i * N) / T, e = ((i + 1) * N + T - 1) / T;
    const float* x = wav + b * ld_wav;
    float acc = 0.f;
    for (int64_t j = s + lane; j < e; j += 64) acc += x[j];
    acc = wave_sum(acc);
    if (lane == 0) out[w] = acc / (float)(e - s);
  }
}
}  // namespace asrx

extern "C" int asrx_wave_pool(const float* wav, int64_t B, int64_t N, int64_t ld_wav, int64_t T, float* out,
                              hipStream_t stream) {
  ASRX_REQUIRE(B > 0 && N > 0 && T > 0 && T <= N, "asrx_wave_pool: need 0 < T <= N (N=%ld T=%ld)", (long)N, (long)T);
  const int64_t waves = B * T;
  const unsigned grid = (unsigned)std::min<int64_t>((waves + 3) / 4, 65536);
  asrx::wave_pool_kernel<<<grid, 256, 0, stream>>>(wav, N, ld_wav, T, B, out);
  ASRX_LAUNCHED("asrx_wave_pool");
}
