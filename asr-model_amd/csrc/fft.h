// Radix-8 Stockham FFT building blocks shared by the log-mel kernel and its host-side unit test.
// A 512-point complex FFT is three radix-8 passes (Ns = 1, 8, 64) over 64 "lanes"; lane j reads
// in[j + 64 r] (r = 0..7), twiddles, does an 8-point DFT and writes
// out[(j / Ns) * Ns * 8 + (j % Ns) + r * Ns].  After the third pass `out` holds the transform in
// natural order.  Twiddles come from a table tw[m] = exp(-2*pi*i*m/512).
#pragma once
#ifndef __HIPCC__
#define __host__
#define __device__
#define __forceinline__ inline
#endif

namespace asrx_fft {

struct cpx {
  float x, y;
};

__host__ __device__ __forceinline__ cpx cadd(cpx a, cpx b) { return {a.x + b.x, a.y + b.y}; }
__host__ __device__ __forceinline__ cpx csub(cpx a, cpx b) { return {a.x - b.x, a.y - b.y}; }
__host__ __device__ __forceinline__ cpx cmul(cpx a, cpx b) {
  return {a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x};
}
__host__ __device__ __forceinline__ cpx cmul_negi(cpx a) { return {a.y, -a.x}; }  // a * (-i)

// In-register 8-point DFT, y[q] = sum_r x[r] exp(-2*pi*i*r*q/8), decimation in frequency.
__host__ __device__ __forceinline__ void dft8(cpx (&v)[8]) {
  const float h = 0.70710678118654752f;
  cpx a[4], b[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    a[r] = cadd(v[r], v[r + 4]);
    b[r] = csub(v[r], v[r + 4]);
  }
  b[1] = cmul(b[1], cpx{h, -h});
  b[2] = cmul_negi(b[2]);
  b[3] = cmul(b[3], cpx{-h, -h});
  // 4-point DFTs (DIF): p = x0+x2, x1+x3 ; q = x0-x2, (x1-x3)*(-i)
  cpx p0 = cadd(a[0], a[2]), p1 = cadd(a[1], a[3]);
  cpx q0 = csub(a[0], a[2]), q1 = cmul_negi(csub(a[1], a[3]));
  cpx s0 = cadd(b[0], b[2]), s1 = cadd(b[1], b[3]);
  cpx t0 = csub(b[0], b[2]), t1 = cmul_negi(csub(b[1], b[3]));
  v[0] = cadd(p0, p1);
  v[4] = csub(p0, p1);
  v[2] = cadd(q0, q1);
  v[6] = csub(q0, q1);
  v[1] = cadd(s0, s1);
  v[5] = csub(s0, s1);
  v[3] = cadd(t0, t1);
  v[7] = csub(t0, t1);
}

// One Stockham pass for lane j: v holds in[j + 64 r] on entry; writes the pass output to `out`.
__host__ __device__ __forceinline__ void stockham_pass(int j, int Ns, cpx (&v)[8], cpx* out,
                                                      const cpx* tw512) {
  const int k = j % Ns;
  if (Ns > 1) {
    const int step = 512 / (Ns * 8);  // exp(-2 pi i r k / (8 Ns)) = tw512[r*k*step]
#pragma unroll
    for (int r = 1; r < 8; ++r) v[r] = cmul(v[r], tw512[(r * k * step) & 511]);
  }
  dft8(v);
  const int base = (j / Ns) * Ns * 8 + k;
#pragma unroll
  for (int r = 0; r < 8; ++r) out[base + r * Ns] = v[r];
}

}  // namespace asrx_fft
