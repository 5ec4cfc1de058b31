// Log-mel front end, replacing the spectrogram and waveform branches of extract_features
// (essentials.py:469-491 and 493-510):
//
//   torchaudio MelSpectrogram(n_fft=1024, hop=160, periodic Hann, center=True zero pad 512,
//   power 2, 128 HTK mels 50-8000 Hz, norm=None)  ->  clamp(1e-10).log10()
//   -> maximum(x, max(x) - 8)  (max over the whole clip)  ->  (x + 4) / 4
//   adaptive_avg_pool1d(audio, N/160)  (exact 160-sample block means when 160 | N)
//
// Kernel 1 (logmel_tiles): a tile is MEL_FPT consecutive frames of one clip; the (FPT-1)*160+1024
// samples a tile touches land in LDS once (LDS-DMA; each sample is re-used 6.4x by the overlapping
// windows), so HBM sees every input byte about once.  Workgroups are persistent over a contiguous
// run of tiles (XCD-aware block order, so neighbouring tiles -- which share 864 samples -- stay in
// one XCD's L2).  Each wave owns one frame at a time and never synchronises with the other waves
// inside a frame: per frame it
//   * packs the windowed real frame as z[n] = x[2n] w[2n] + i x[2n+1] w[2n+1] (lane j holds
//     n = j + 64 r, r = 0..7, one complex value per aligned VGPR pair; the window values are lane
//     constants),
//   * runs the 512-point complex FFT as three radix-8 stages over the register index (n = j + 64 n2,
//     j = n0 + 8 n1): DFT over n2 and twiddle W512^(j kA); swap lane bits 3-5 with the register bits;
//     DFT over n1 and twiddle W64^(n0 kB); swap lane bits 0-2 with the register bits; DFT over n0.
//     The lane/register swaps never touch LDS: bits 5 and 4 are v_permlane32/16_swap, bits 3..0 one
//     v_cndmask_b32 with a DPP-read source per register (row_ror / quad_perm).  The complex arithmetic
//     is packed FP32 (v_pk_add/mul/fma_f32 with op_sel / neg modifiers for the swaps and signs),
//   * stores Z (digit-reversed in the lanes) to a padded per-wave LDS buffer in natural order, reads
//     the mirrored Z[512-k] back, untangles the real spectrum and forms 4|X_k|^2 (the factor 4 is
//     folded into the filterbank weights),
//   * applies the sparse filterbank: lane m owns bands m (<= FB_A taps) and m + 64 (<= FB_B taps),
//     weights re-read from LDS per frame, bins read by immediate LDS offsets, even and odd taps
//     accumulated in the two halves of a packed pair,
//   * takes log10 as log2 * log10(2) (v_log_f32) and stores (x + 4) / 4.
// Per tile the block writes its max and min log value (over live frames) to a workspace; the fused
// waveform pool reads the same LDS samples (16 threads per frame, DPP row sums).
// Kernel 2 (logmel_floor): the clip-max floor, max(x, clipmax - 8), on the (x + 4) / 4 values; a tile
// whose minimum is not below the floor is skipped.
#include "common.h"
#include "fft.h"

using asrx_fft::cpx;

namespace asrx {

constexpr int MEL_NFFT = 1024, MEL_HOP = 160, MEL_NBINS = 513, MEL_BANDS = 128, MEL_FBW = 32;
constexpr int FB_A = 8, FB_B = 24;  // taps of a lane's two bands (see lane_filterbank in mel.py)
constexpr int FB_QUADS = (FB_A + FB_B) / 4;
constexpr int MEL_WAVES = 4;
#ifndef MEL_WPS
#define MEL_WPS 3  // waves per SIMD (= resident 4-wave workgroups per CU)
#endif
#ifndef MEL_FPT_
#define MEL_FPT_ 16
#endif
#ifndef MEL_NBUF0
#define MEL_NBUF0 1  // sample buffers of the (B, F, 128) kernel (2: measured no faster, and 54 KB of LDS fits only 2 workgroups per CU)
#endif
#ifndef MEL_ILP
#define MEL_ILP 1  // frames per wave in flight at once
#endif
#ifndef MEL_ABL
#define MEL_ABL 0  // timing ablations (wrong results): 1 no sample loads, 2 no mirror exchange, 4 no filterbank
                   // reads, 8 no lane exchanges (64 only bits 5-4, 128 only bits 3-0), 16 no stores, 32 no pool
#endif
#ifndef MEL_STAGE0
#define MEL_STAGE0 0  // 1: (B, F, 128) output staged in LDS and stored as float4 rows
#endif
constexpr int MEL_FPT = MEL_FPT_;  // frames per tile
constexpr int MEL_TSAMP = (MEL_FPT - 1) * MEL_HOP + MEL_NFFT;  // 3424 samples per tile
constexpr int MEL_TSAMP4 = MEL_TSAMP / 4;                      // 856 float4
constexpr int MEL_PF = (MEL_TSAMP4 + 255) / 256;               // prefetch float4 per thread
constexpr int FFT_SLOTS = 512 + 64 + 1;                        // zpad(0..512) cpx slots per wave
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

// Z slot of bin i: two pad slots every 16 bins (slot(i + 64) = slot(i) + 72), which makes the
// digit-reversed Z stores conflict-free and leaves the mirrored reads 2-way
__device__ __forceinline__ int zpad(int i) { return i + 2 * (i >> 4); }

// 2 x 2 exchange between lane bit B and register bit: for every register pair (a, c) that differs
// only in that register bit, lanes with the lane bit clear keep a and take the partner's a into c,
// lanes with it set take the partner's c into a and keep c.  Bits 5 and 4 are one permlane swap per
// VGPR pair; bits 3..0 read the partner through DPP (row_ror by 8 or 4/12 inside a 16-lane row,
// quad_perm xor 2 / xor 1) and select.
template <int B>
__device__ __forceinline__ void xch_pair(float& a, float& c) {
  if constexpr (B == 5) {
    xrow32(a, c);
  } else {
    static_assert(B == 4, "bits 3..0 go through xch_dpp4");
    xrow16(a, c);
  }
}
// Bits 3..0, four register pairs at once: each output is one v_cndmask_b32 whose first source is
// read through DPP (the select and the partner read in one instruction):
//   c' = set ? c : partner(a)   with VCC = the lanes whose bit is set, DPP = UP
//   a' = set ? partner(c) : a   with VCC = the lanes whose bit is clear, DPP = DN
// UP: lane i reads lane i + 2^B (bit-clear lanes); DN: lane i - 2^B (bit-set lanes).  row_ror:n makes
// lane i read lane (i - n) mod 16 of its row, so i + 4 is row_ror:12 and i - 4 row_ror:4; bits 1 and
// 0 are quad_perm xor 2 / xor 1 both ways, bit 3 row_ror:8 both ways.  The leading s_nop 1 covers the
// VALU-write -> DPP-read hazard on the inputs; the outputs are fresh registers.
#define ASRX_XCH8(UPS, DNS)                                                                                    \
  asm("s_mov_b64 vcc, %[ms]\n\ts_nop 1\n\t"                                                                 \
      "v_cndmask_b32_dpp %[c0], %[a0i], %[c0i], vcc " UPS " row_mask:0xf bank_mask:0xf\n\t"   \
      "v_cndmask_b32_dpp %[c1], %[a1i], %[c1i], vcc " UPS " row_mask:0xf bank_mask:0xf\n\t"   \
      "v_cndmask_b32_dpp %[c2], %[a2i], %[c2i], vcc " UPS " row_mask:0xf bank_mask:0xf\n\t"   \
      "v_cndmask_b32_dpp %[c3], %[a3i], %[c3i], vcc " UPS " row_mask:0xf bank_mask:0xf\n\t"   \
      "v_cndmask_b32_dpp %[c4], %[a4i], %[c4i], vcc " UPS " row_mask:0xf bank_mask:0xf\n\t"   \
      "v_cndmask_b32_dpp %[c5], %[a5i], %[c5i], vcc " UPS " row_mask:0xf bank_mask:0xf\n\t"   \
      "v_cndmask_b32_dpp %[c6], %[a6i], %[c6i], vcc " UPS " row_mask:0xf bank_mask:0xf\n\t"   \
      "v_cndmask_b32_dpp %[c7], %[a7i], %[c7i], vcc " UPS " row_mask:0xf bank_mask:0xf\n\t"   \
      "s_mov_b64 vcc, %[mc]\n\t"                                                                             \
      "v_cndmask_b32_dpp %[a0], %[c0i], %[a0i], vcc " DNS " row_mask:0xf bank_mask:0xf\n\t"   \
      "v_cndmask_b32_dpp %[a1], %[c1i], %[a1i], vcc " DNS " row_mask:0xf bank_mask:0xf\n\t"   \
      "v_cndmask_b32_dpp %[a2], %[c2i], %[a2i], vcc " DNS " row_mask:0xf bank_mask:0xf\n\t"   \
      "v_cndmask_b32_dpp %[a3], %[c3i], %[a3i], vcc " DNS " row_mask:0xf bank_mask:0xf\n\t"   \
      "v_cndmask_b32_dpp %[a4], %[c4i], %[a4i], vcc " DNS " row_mask:0xf bank_mask:0xf\n\t"   \
      "v_cndmask_b32_dpp %[a5], %[c5i], %[a5i], vcc " DNS " row_mask:0xf bank_mask:0xf\n\t"   \
      "v_cndmask_b32_dpp %[a6], %[c6i], %[a6i], vcc " DNS " row_mask:0xf bank_mask:0xf\n\t"   \
      "v_cndmask_b32_dpp %[a7], %[c7i], %[a7i], vcc " DNS " row_mask:0xf bank_mask:0xf"   \
      : [a0] "=&v"(pa[0]), [a1] "=&v"(pa[1]), [a2] "=&v"(pa[2]), [a3] "=&v"(pa[3]), [a4] "=&v"(pa[4]), [a5] "=&v"(pa[5]), [a6] "=&v"(pa[6]), [a7] "=&v"(pa[7]), [c0] "=&v"(pc[0]), [c1] "=&v"(pc[1]), [c2] "=&v"(pc[2]), [c3] "=&v"(pc[3]), [c4] "=&v"(pc[4]), [c5] "=&v"(pc[5]), [c6] "=&v"(pc[6]), [c7] "=&v"(pc[7]) \
      : [a0i] "v"(ia[0]), [a1i] "v"(ia[1]), [a2i] "v"(ia[2]), [a3i] "v"(ia[3]), [a4i] "v"(ia[4]), [a5i] "v"(ia[5]), [a6i] "v"(ia[6]), [a7i] "v"(ia[7]), [c0i] "v"(ic[0]), [c1i] "v"(ic[1]), [c2i] "v"(ic[2]), [c3i] "v"(ic[3]), [c4i] "v"(ic[4]), [c5i] "v"(ic[5]), [c6i] "v"(ic[6]), [c7i] "v"(ic[7]), [ms] "s"(mset), [mc] "s"(~mset) \
      : "vcc")
// one stage, eight register pairs (x and y of four complex pairs) in one statement: two VCC loads and
// one s_nop per stage
template <int B>
__device__ __forceinline__ void xch_dpp8(float (&pa)[8], float (&pc)[8]) {
  constexpr uint64_t mset = B == 3 ? 0xFF00FF00FF00FF00ull
                          : B == 2 ? 0xF0F0F0F0F0F0F0F0ull
                          : B == 1 ? 0xCCCCCCCCCCCCCCCCull
                                   : 0xAAAAAAAAAAAAAAAAull;
  float ia[8], ic[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    ia[i] = pa[i];
    ic[i] = pc[i];
  }
  if constexpr (B == 3) ASRX_XCH8("row_ror:8", "row_ror:8");
  else if constexpr (B == 2) ASRX_XCH8("row_ror:12", "row_ror:4");
  else if constexpr (B == 1) ASRX_XCH8("quad_perm:[2,3,0,1]", "quad_perm:[2,3,0,1]");
  else ASRX_XCH8("quad_perm:[1,0,3,2]", "quad_perm:[1,0,3,2]");
}
#undef ASRX_XCH8
// lane bit B <-> register bit (B % 3): 5 and 2 pair registers r, r + 4; 4 and 1 pair r, r + 2; 3 and
// 0 pair r, r + 1
typedef float f2v __attribute__((ext_vector_type(2)));
template <int B>
__device__ __forceinline__ void xch_lanes(f2v (&v)[8]) {
  constexpr int RB = 1 << (B % 3);
  constexpr int R[4] = {0, RB == 1 ? 2 : 1, RB == 4 ? 2 : 4, RB == 1 ? 6 : RB == 2 ? 5 : 3};  // bit RB clear
  if constexpr (B >= 4) {
    // the eight swaps of the stage in one statement behind one s_nop (no swap reads another's output)
    float a[8], c[8];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      a[2 * i] = v[R[i]].x;
      a[2 * i + 1] = v[R[i]].y;
      c[2 * i] = v[R[i] + RB].x;
      c[2 * i + 1] = v[R[i] + RB].y;
    }
#define ASRX_SW(OP)                                                                                           \
  asm("s_nop 1\n\t" OP " %0, %8\n\t" OP " %1, %9\n\t" OP " %2, %10\n\t" OP " %3, %11\n\t" OP " %4, %12\n\t" OP  \
      " %5, %13\n\t" OP " %6, %14\n\t" OP " %7, %15"                                                             \
      : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7]), "+v"(c[0]), \
        "+v"(c[1]), "+v"(c[2]), "+v"(c[3]), "+v"(c[4]), "+v"(c[5]), "+v"(c[6]), "+v"(c[7]))
    if constexpr (B == 5) ASRX_SW("v_permlane32_swap_b32");
    else ASRX_SW("v_permlane16_swap_b32");
#undef ASRX_SW
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[R[i]] = f2v{a[2 * i], a[2 * i + 1]};
      v[R[i] + RB] = f2v{c[2 * i], c[2 * i + 1]};
    }
  } else {
    float a[8], c[8];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      a[2 * i] = v[R[i]].x;
      a[2 * i + 1] = v[R[i]].y;
      c[2 * i] = v[R[i] + RB].x;
      c[2 * i + 1] = v[R[i] + RB].y;
    }
    xch_dpp8<B>(a, c);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[R[i]] = f2v{a[2 * i], a[2 * i + 1]};
      v[R[i] + RB] = f2v{c[2 * i], c[2 * i + 1]};
    }
  }
}

// ---- packed complex arithmetic (a complex value is one aligned VGPR pair: x = re, y = im).  Each
// helper is one VOP3P instruction (v_pk_add_f32 / v_pk_mul_f32 / v_pk_fma_f32 with op_sel / neg
// modifiers doing the swaps and sign flips), two for the general product.
__device__ __forceinline__ f2v pk_cmul(f2v a, f2v b) {  // a b
  f2v t, r;
  asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]" : "=v"(t) : "v"(a), "v"(b));  // (ax bx, ax by)
  asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[1,0,0]"  // (-ay by, ay bx) + t
      : "=v"(r) : "v"(a), "v"(b), "v"(t));
  return r;
}
__device__ __forceinline__ f2v pk_add_negi(f2v q, f2v d) {  // q + (-i) d = (qx + dy, qy - dx)
  f2v r;
  asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]" : "=v"(r) : "v"(q), "v"(d));
  return r;
}
__device__ __forceinline__ f2v pk_sub_negi(f2v q, f2v d) {  // q - (-i) d = (qx - dy, qy + dx)
  f2v r;
  asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1]" : "=v"(r) : "v"(q), "v"(d));
  return r;
}
__device__ __forceinline__ f2v pk_conj_add(f2v a, f2v b) {  // a + conj b = (ax + bx, ay - by)
  f2v r;
  asm("v_pk_add_f32 %0, %1, %2 neg_hi:[0,1]" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ f2v pk_untangle_odd(f2v zk, f2v zn) {  // (-i)(zk - conj zn) = (zk.y + zn.y, zn.x - zk.x)
  f2v r;
  asm("v_pk_add_f32 %0, %1, %2 op_sel:[1,1] op_sel_hi:[0,0] neg_hi:[1,0]" : "=v"(r) : "v"(zk), "v"(zn));
  return r;
}
// 8-point DFT over the registers, y[q] = sum_r x[r] exp(-2 pi i r q / 8) -- asrx_fft::dft8's
// decimation-in-frequency graph on packed complex values (28 VOP3P instructions)
__device__ __forceinline__ void pk_dft8(f2v (&v)[8]) {
  const float h = 0.70710678118654752f;
  const f2v a0 = v[0] + v[4], a1 = v[1] + v[5], a2 = v[2] + v[6], a3 = v[3] + v[7];
  const f2v b0 = v[0] - v[4], b2 = v[2] - v[6];
  f2v b1 = v[1] - v[5], b3 = v[3] - v[7];
  {
    f2v t1, t3;  // b1 (h - ih) = h (b1x + b1y, b1y - b1x); b3 (-h - ih) = -h (b3x - b3y, b3y + b3x)
    asm("v_pk_add_f32 %0, %1, %1 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]" : "=v"(t1) : "v"(b1));
    asm("v_pk_add_f32 %0, %1, %1 op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1]" : "=v"(t3) : "v"(b3));
    b1 = t1 * f2v{h, h};
    b3 = t3 * f2v{-h, -h};
  }
  const f2v p0 = a0 + a2, p1 = a1 + a3, q0 = a0 - a2, d = a1 - a3;
  const f2v s0 = pk_add_negi(b0, b2), t0 = pk_sub_negi(b0, b2), s1 = b1 + b3, d2 = b1 - b3;
  v[0] = p0 + p1;
  v[4] = p0 - p1;
  v[2] = pk_add_negi(q0, d);
  v[6] = pk_sub_negi(q0, d);
  v[1] = s0 + s1;
  v[5] = s0 - s1;
  v[3] = pk_add_negi(t0, d2);
  v[7] = pk_sub_negi(t0, d2);
}

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

// the eight filterbank weight quads of this lane, re-read per frame (kept in VGPRs they would cost 32
// registers for the whole kernel and a wave per SIMD)
typedef float f4v __attribute__((ext_vector_type(4)));
template <int OFF>
__device__ __forceinline__ f4v ds_rd128(uint32_t a) {
  f4v r;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(a), "i"(OFF) : "memory");
  return r;
}

// the same reads without the wait: completed by lgkm_wait on every destination
template <int OFF0, int STRIDE>
__device__ __forceinline__ void ds_rd64x8_nw(uint32_t a, f2v (&o)[8]) {
  o[0] = ds_rd64<OFF0>(a);
  o[1] = ds_rd64<OFF0 + STRIDE>(a);
  o[2] = ds_rd64<OFF0 + 2 * STRIDE>(a);
  o[3] = ds_rd64<OFF0 + 3 * STRIDE>(a);
  o[4] = ds_rd64<OFF0 + 4 * STRIDE>(a);
  o[5] = ds_rd64<OFF0 + 5 * STRIDE>(a);
  o[6] = ds_rd64<OFF0 + 6 * STRIDE>(a);
  o[7] = ds_rd64<OFF0 + 7 * STRIDE>(a);
}
template <int OFF0, int STRIDE>
__device__ __forceinline__ void ds_rd64x4_nw(uint32_t a, f2v (&o)[4]) {
  o[0] = ds_rd64<OFF0>(a);
  o[1] = ds_rd64<OFF0 + STRIDE>(a);
  o[2] = ds_rd64<OFF0 + 2 * STRIDE>(a);
  o[3] = ds_rd64<OFF0 + 3 * STRIDE>(a);
}
// s_waitcnt lgkmcnt(0) naming every register of the arrays, so no use is scheduled before it
template <int N>
__device__ __forceinline__ void lgkm_wait8(f2v (&o)[N]) {
  static_assert(N == 8 || N == 4, "");
  if constexpr (N == 8)
    asm volatile("s_waitcnt lgkmcnt(0)"
                 : "+v"(o[0]), "+v"(o[1]), "+v"(o[2]), "+v"(o[3]), "+v"(o[4]), "+v"(o[5]), "+v"(o[6]), "+v"(o[7])
                 :
                 : "memory");
  else
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(o[0]), "+v"(o[1]), "+v"(o[2]), "+v"(o[3]) : : "memory");
}
template <int NQ, int N>
__device__ __forceinline__ void lgkm_wait(f2v (&o)[NQ][N]) {
  // the first call waits; the others only pin their registers behind it (lgkmcnt is already 0)
#pragma unroll
  for (int q = 0; q < NQ; ++q) lgkm_wait8(o[q]);
}

template <int OFF0, int STRIDE>
__device__ __forceinline__ void ds_rd64x4(uint32_t a, f2v (&o)[4]) {
  o[0] = ds_rd64<OFF0>(a);
  o[1] = ds_rd64<OFF0 + STRIDE>(a);
  o[2] = ds_rd64<OFF0 + 2 * STRIDE>(a);
  o[3] = ds_rd64<OFF0 + 3 * STRIDE>(a);
  asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(o[0]), "+v"(o[1]), "+v"(o[2]), "+v"(o[3]) : : "memory");
}

// contiguous run of tiles per workgroup; consecutive runs on one XCD (blocks are dealt to the 8
// XCDs round-robin by blockIdx)
__device__ __forceinline__ int xcd_block(int bid, int G) {
  const int per = G / 8, rem = G % 8, x = bid % 8, q = bid / 8;
  return (x < rem ? x * (per + 1) : rem * (per + 1) + (x - rem) * per) + q;
}

// LAYOUT 0 (B, F, 128): every lane stores its two bands straight into the frame's 512-byte row (L2
// merges the scattered dwords into whole lines), so no staging block is needed and the workgroup's
// LDS (40.6 KB) lets 4 of them share a CU.  LAYOUT 1 (B, 128, F) stages the tile in LDS for
// frame-contiguous stores.
template <int LAYOUT>
__global__ __launch_bounds__(256, MEL_WPS) void logmel_tiles_kernel(
    const float* __restrict__ wav, int64_t N, int64_t ld_wav, int vec_ok, int64_t F, int tiles_per_clip,
    int64_t n_tiles, int tiles_per_block, const float* __restrict__ consts, const float* __restrict__ fbw,
    const int* __restrict__ fbs, float* __restrict__ out, int64_t ld_out,
    float* __restrict__ tstat, float* __restrict__ pool, int64_t T_pool) {
  // (B, F, 128): two sample buffers, the next tile's samples land by LDS-DMA while this tile is
  // transformed; (B, 128, F) keeps one (its staging block takes the room)
  constexpr int NBUF = LAYOUT == 0 ? MEL_NBUF0 : 1;
  constexpr bool STAGED = LAYOUT == 1 || MEL_STAGE0;
  __shared__ __attribute__((aligned(16))) float samp_buf[NBUF][MEL_TSAMP];
  constexpr int NI = MEL_ILP;
  static_assert(MEL_FPT % (MEL_WAVES * NI) == 0, "frames per tile must split evenly over waves x NI");
  __shared__ __attribute__((aligned(16))) cpx fbuf[MEL_WAVES * NI][FFT_SLOTS];
  __shared__ float melst[STAGED ? MEL_FPT : 1][MEL_BANDS + 1];
  __shared__ float red[2][MEL_WAVES];
  __shared__ float4 fbw_s[FB_QUADS * 64];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int64_t t_begin = (int64_t)xcd_block(blockIdx.x, gridDim.x) * tiles_per_block;
  if (t_begin >= n_tiles) return;
  const int64_t t_end = t_begin + tiles_per_block < n_tiles ? t_begin + tiles_per_block : n_tiles;

  // ---- lane constants: window, pass-2/3 twiddles, untangle twiddles, filterbank rows
  const float* win = consts;
  const cpx* tw512 = reinterpret_cast<const cpx*>(consts + MEL_NFFT);
  const cpx* tw1024 = reinterpret_cast<const cpx*>(consts + MEL_NFFT + 1024);
  const f2v* tw512v = reinterpret_cast<const f2v*>(tw512);
  // the bin index lane j holds after the third stage: kj + 64 r, kj = (j >> 3) + 8 (j & 7)
  const int kj = (lane >> 3) + 8 * (lane & 7);
  f2v wv[8], twa[7], twb[7];
#pragma unroll
  for (int r = 0; r < 8; ++r) wv[r] = *reinterpret_cast<const f2v*>(win + 2 * (lane + 64 * r));
  const f2v tu0 = reinterpret_cast<const f2v*>(tw1024)[kj];
#pragma unroll
  for (int r = 1; r < 8; ++r) {
    twa[r - 1] = tw512v[(r * lane) & 511];            // W512^(j kA)
    twb[r - 1] = tw512v[(r * (lane & 7) * 8) & 511];  // W64^(n0 kB)
  }
  // lane-packed filterbank (asrx/mel.py lane_filterbank): lane m owns band_a (<= 8 taps from the
  // even bin sa) and band_b (<= 24 taps from the even bin sb); weights [tap/4][lane][4] in LDS
  const int band_a = fbs[lane], band_b = fbs[64 + lane];
  const int sa2 = fbs[128 + lane] >> 1, sb2 = fbs[192 + lane] >> 1;
  for (int i = tid; i < FB_QUADS * 64; i += 256) fbw_s[i] = reinterpret_cast<const float4*>(fbw)[i];


  // tile t's samples -> dst.  Interior tiles: LDS-DMA (global_load_lds_dwordx4, 1 KB per wave
  // instruction, no VGPRs held), completed by the s_waitcnt vmcnt(0) before the barrier that
  // publishes the buffer.  Tiles that touch a clip edge (the test is per tile, so workgroup-uniform):
  // element-wise with zero fill.
  auto stage = [&](int64_t t, float* dst) {
    const int64_t b = t / tiles_per_clip;
    const int64_t g0 = (t - b * tiles_per_clip) * MEL_FPT * MEL_HOP - MEL_NFFT / 2;
    const float* x = wav + b * ld_wav + g0;
    if (vec_ok && g0 >= 0 && g0 + MEL_TSAMP <= N) {
      const float4* x4 = reinterpret_cast<const float4*>(x);
#pragma unroll
      for (int q = 0; q < MEL_PF; ++q) {
        const int c0 = 256 * q + 64 * wid;  // this wave's float4 chunk (wave-uniform)
        if (c0 < MEL_TSAMP4 && c0 + lane < MEL_TSAMP4) glds16(x4 + c0 + lane, lds_addr(reinterpret_cast<float4*>(dst) + c0));
      }
    } else {
#pragma unroll 1
      for (int i = tid; i < MEL_TSAMP; i += 256) {
        const int64_t g = g0 + i;
        dst[i] = (g >= 0 && g < N) ? x[i] : 0.f;
      }
    }
  };
  if constexpr (NBUF == 2) stage(t_begin, samp_buf[0]);

#pragma unroll 1
  for (int64_t t = t_begin; t < t_end; ++t) {
    const int64_t b = t / tiles_per_clip;
    const int64_t f0 = (t - b * tiles_per_clip) * MEL_FPT;
    float* samp = samp_buf[NBUF == 2 ? (int)((t - t_begin) & 1) : 0];
    if constexpr (NBUF == 1) {
      __syncthreads();  // the previous tile's readers are done with samp / melst
#if !(MEL_ABL & 1)
      stage(t, samp);
#endif
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // samp published; with two buffers also: every wave is done with the other one
    if constexpr (NBUF == 2) {
      if (t + 1 < t_end) stage(t + 1, samp_buf[(int)((t + 1 - t_begin) & 1)]);
    }

    // fused waveform feature: exact 160-sample block means (pool index == frame index).  Sixteen
    // threads per frame, each summing 10 consecutive samples, then a DPP sum inside the 16-lane row
    // (quad_perm xor 1, xor 2, row_half_mirror, row_mirror): no LDS round trips
    static_assert(MEL_HOP == 16 * 10, "the pool splits a hop into 16 runs of 10 samples");
    if (pool && !(MEL_ABL & 32)) {
#pragma unroll 1
      for (int i = tid; i < MEL_FPT * 16; i += 256) {
        const int fi = i >> 4, part = i & 15;
        const float* q = samp + MEL_NFFT / 2 + fi * MEL_HOP + part * 10;
        float s = 0.f;
#pragma unroll
        for (int k = 0; k < 10; ++k) s += q[k];
        s += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, s), 0xB1, 0xF, 0xF, false));
        s += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, s), 0x4E, 0xF, 0xF, false));
        s += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, s), 0x141, 0xF, 0xF, false));
        s += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, s), 0x140, 0xF, 0xF, false));
        const int64_t f = f0 + fi;
        if (part == 0 && f < T_pool) pool[b * T_pool + f] = s * (1.0f / MEL_HOP);
      }
    }

    float lmax = -3.0e38f, lmin = 3.0e38f;
    // NI frames per wave at a time (frames fi0 + q * MEL_WAVES): their dependency chains interleave
#pragma unroll 1
    for (int fi0 = wid; fi0 < MEL_FPT; fi0 += MEL_WAVES * NI) {
      f2v v[NI][8];
#pragma unroll
      for (int q = 0; q < NI; ++q) ds_rd64x8_nw<0, 512>(lds_off(samp + (fi0 + q * MEL_WAVES) * MEL_HOP + 2 * lane), v[q]);
      lgkm_wait(v);
#pragma unroll
      for (int q = 0; q < NI; ++q) {
#pragma unroll
        for (int r = 0; r < 8; ++r) v[q][r] *= wv[r];
        // stage A: DFT over n2 (registers) -> kA, twiddle W512^(j kA)
        pk_dft8(v[q]);
#pragma unroll
        for (int r = 1; r < 8; ++r) v[q][r] = pk_cmul(v[q][r], twa[r - 1]);
      }
      // lane bits 3-5 (n1) <-> register bits 0-2 (kA): lane = n0 + 8 kA, registers n1
#pragma unroll
      for (int q = 0; q < NI; ++q) {
#if !(MEL_ABL & (8 | 64))
        xch_lanes<5>(v[q]);
        xch_lanes<4>(v[q]);
#endif
#if !(MEL_ABL & (8 | 128))
        xch_lanes<3>(v[q]);
#endif
      }
#pragma unroll
      for (int q = 0; q < NI; ++q) {
        // stage B: DFT over n1 -> kB, twiddle W64^(n0 kB)
        pk_dft8(v[q]);
#pragma unroll
        for (int r = 1; r < 8; ++r) v[q][r] = pk_cmul(v[q][r], twb[r - 1]);
      }
      // lane bits 0-2 (n0) <-> register bits 0-2 (kB): lane = kB + 8 kA, registers n0
#pragma unroll
      for (int q = 0; q < NI; ++q) {
#if !(MEL_ABL & (8 | 128))
        xch_lanes<2>(v[q]);
        xch_lanes<1>(v[q]);
        xch_lanes<0>(v[q]);
#endif
        // stage C: DFT over n0 -> kC; lane j register r now holds Z[kj + 64 r]
        pk_dft8(v[q]);
      }
      // the one LDS exchange per frame: Z in natural order (padded, zpad), Z_0 also at slot zpad(512)
      // for the mirror of lane 0's register 0
#pragma unroll
      for (int q = 0; q < NI; ++q) {
        f2v* Sv = reinterpret_cast<f2v*>(fbuf[wid * NI + q]);
#pragma unroll
        for (int r = 0; r < 8; ++r) Sv[zpad(kj) + 72 * r] = v[q][r];
        if (lane == 0) Sv[zpad(512)] = v[q][0];
      }
      wave_lds_sync();
      f2v zm[NI][8];  // zm[7 - r] = Z[(512 - kj - 64 r) & 511] = S[zpad(64 - kj) + 72 (7 - r)]
#if MEL_ABL & 2
#pragma unroll
      for (int q = 0; q < NI; ++q)
#pragma unroll
        for (int r = 0; r < 8; ++r) zm[q][r] = v[q][7 - r] * 0.5f;
#else
#pragma unroll
      for (int q = 0; q < NI; ++q) ds_rd64x8_nw<0, 576>(lds_off(fbuf[wid * NI + q] + zpad(64 - kj)), zm[q]);
      lgkm_wait(zm);
#endif
      // real-FFT untangle: 2 X_k = (Z_k + conj Z_{512-k}) + W1024^k (-i)(Z_k - conj Z_{512-k})
      // W1024^(kj + 64 r) = W1024^kj exp(-i pi r / 8) = u[r & 3] (-i)^(r >> 2)
      f2v u[4];
      u[0] = tu0;
#pragma unroll
      for (int r = 1; r < 4; ++r) u[r] = pk_cmul(tu0, f2v{kRot[r][0], kRot[r][1]});
      float pw[NI][8];
#pragma unroll
      for (int q = 0; q < NI; ++q)
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          const f2v zn = zm[q][7 - r], zk = v[q][r];
          const f2v e = pk_conj_add(zk, zn);                         // Z_k + conj Z_{512-k}
          const f2v w = pk_cmul(u[r & 3], pk_untangle_odd(zk, zn));  // W (-i)(Z_k - conj Z_{512-k}), W = u (-i)^(r>>2)
          const f2v x = r < 4 ? e + w : pk_add_negi(e, w);
          pw[q][r] = fmaf(x.x, x.x, x.y * x.y);  // 4 |X_k|^2
        }
      wave_lds_sync();
#pragma unroll
      for (int q = 0; q < NI; ++q) {
        float* P = reinterpret_cast<float*>(fbuf[wid * NI + q]);
#pragma unroll
        for (int r = 0; r < 8; ++r) P[kj + 64 * r] = pw[q][r];
        if (lane < 16) {
          const float nyq = 2.0f * (v[q][0].x - v[q][0].y);  // lane 0: 2 X_512 = 2 (Re Z0 - Im Z0)
          P[512 + lane] = lane == 0 ? nyq * nyq : 0.f;        // bins past 512 are zero pads for the taps
        }
      }
      wave_lds_sync();
      // sparse filterbank (weights carry the 1/4; bins read in even-aligned pairs), three read groups
      // (bins | weight quads), each drained before the next: band a (8 bins), band b taps 0-15, band b
      // taps 16-23; even and odd taps accumulate in the two halves of a packed pair
      static_assert(FB_A == 8 && FB_B == 24, "the filterbank reads below are written out for 8 + 24 taps");
      float acc_a[NI], acc_b[NI];
#if MEL_ABL & 4
#pragma unroll
      for (int q = 0; q < NI; ++q) {
        acc_a[q] = reinterpret_cast<float*>(fbuf[wid * NI + q])[lane];
        acc_b[q] = reinterpret_cast<float*>(fbuf[wid * NI + q])[lane + 64];
      }
#else
      const uint32_t wa = lds_off(fbw_s + lane);
      f2v sa[NI], sb[NI];
      {
        f2v p[NI][4];
#pragma unroll
        for (int q = 0; q < NI; ++q) ds_rd64x4_nw<0, 8>(lds_off(reinterpret_cast<float*>(fbuf[wid * NI + q]) + 2 * sa2), p[q]);
        f4v w0 = ds_rd128<0>(wa), w1 = ds_rd128<1024>(wa);
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(w0), "+v"(w1) : : "memory");
        lgkm_wait(p);
#pragma unroll
        for (int q = 0; q < NI; ++q) {
          sa[q] = w0.xy * p[q][0];
          sa[q] = __builtin_elementwise_fma(w0.zw, p[q][1], sa[q]);
          sa[q] = __builtin_elementwise_fma(w1.xy, p[q][2], sa[q]);
          sa[q] = __builtin_elementwise_fma(w1.zw, p[q][3], sa[q]);
        }
      }
      {
        f2v p[NI][8];
#pragma unroll
        for (int q = 0; q < NI; ++q) ds_rd64x8_nw<0, 8>(lds_off(reinterpret_cast<float*>(fbuf[wid * NI + q]) + 2 * sb2), p[q]);
        f4v w0 = ds_rd128<2048>(wa), w1 = ds_rd128<3072>(wa), w2 = ds_rd128<4096>(wa), w3 = ds_rd128<5120>(wa);
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(w0), "+v"(w1), "+v"(w2), "+v"(w3) : : "memory");
        lgkm_wait(p);
#pragma unroll
        for (int q = 0; q < NI; ++q) {
          sb[q] = w0.xy * p[q][0];
          sb[q] = __builtin_elementwise_fma(w0.zw, p[q][1], sb[q]);
          sb[q] = __builtin_elementwise_fma(w1.xy, p[q][2], sb[q]);
          sb[q] = __builtin_elementwise_fma(w1.zw, p[q][3], sb[q]);
          sb[q] = __builtin_elementwise_fma(w2.xy, p[q][4], sb[q]);
          sb[q] = __builtin_elementwise_fma(w2.zw, p[q][5], sb[q]);
          sb[q] = __builtin_elementwise_fma(w3.xy, p[q][6], sb[q]);
          sb[q] = __builtin_elementwise_fma(w3.zw, p[q][7], sb[q]);
        }
      }
      {
        f2v p[NI][4];
#pragma unroll
        for (int q = 0; q < NI; ++q) ds_rd64x4_nw<64, 8>(lds_off(reinterpret_cast<float*>(fbuf[wid * NI + q]) + 2 * sb2), p[q]);
        f4v w0 = ds_rd128<6144>(wa), w1 = ds_rd128<7168>(wa);
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(w0), "+v"(w1) : : "memory");
        lgkm_wait(p);
#pragma unroll
        for (int q = 0; q < NI; ++q) {
          sb[q] = __builtin_elementwise_fma(w0.xy, p[q][0], sb[q]);
          sb[q] = __builtin_elementwise_fma(w0.zw, p[q][1], sb[q]);
          sb[q] = __builtin_elementwise_fma(w1.xy, p[q][2], sb[q]);
          sb[q] = __builtin_elementwise_fma(w1.zw, p[q][3], sb[q]);
        }
      }
#pragma unroll
      for (int q = 0; q < NI; ++q) {
        acc_a[q] = sa[q].x + sa[q].y;
        acc_b[q] = sb[q].x + sb[q].y;
      }
#endif
      wave_lds_sync();
#pragma unroll
      for (int q = 0; q < NI; ++q) {
        const int fi = fi0 + q * MEL_WAVES;
        const bool live = f0 + fi < F;  // wave-uniform
        // clamp(1e-10).log10(): the clamped value maps to exactly -10 like the correctly rounded
        // library log10; elsewhere log2 * log10(2) is within a few ulp
        const float l_a = acc_a[q] <= 1e-10f ? -10.0f : __builtin_amdgcn_logf(acc_a[q]) * 0.30102999566398120f;
        const float l_b = acc_b[q] <= 1e-10f ? -10.0f : __builtin_amdgcn_logf(acc_b[q]) * 0.30102999566398120f;
        // (x + 4) / 4 here; the clip-max floor is applied afterwards, only to the tiles holding a value
        // below it (logmel_floor_kernel): (max(x, f) + 4) / 4 == max((x + 4) / 4, (f + 4) / 4) exactly,
        // as x -> fl(x + 4) is monotone and / 4 is exact
        const float y_a = (l_a + 4.0f) * 0.25f, y_b = (l_b + 4.0f) * 0.25f;
        if constexpr (!STAGED) {
          if (live && !(MEL_ABL & 16)) {
            float* orow = out + b * ld_out + (f0 + fi) * MEL_BANDS;
            orow[band_a] = y_a;
            orow[band_b] = y_b;
          }
        } else {
          melst[fi][band_a] = y_a;
          melst[fi][band_b] = y_b;
        }
        if (live) {
          lmax = fmaxf(lmax, fmaxf(l_a, l_b));
          lmin = fminf(lmin, fminf(l_a, l_b));
        }
      }
    }
    lmax = wave_max_dpp(lmax);
    lmin = -wave_max_dpp(-lmin);
    if (lane == 0) {
      red[0][wid] = lmax;
      red[1][wid] = lmin;
    }
    __syncthreads();

    // coalesced output of the staged block
    if constexpr (LAYOUT == 0 && STAGED) {  // (B, F, 128): the tile is FPT contiguous rows of 128
      float* o = out + b * ld_out;
      for (int i = tid; i < MEL_FPT * MEL_BANDS / 4; i += 256) {
        const int fi = i / (MEL_BANDS / 4), m4 = (i % (MEL_BANDS / 4)) * 4;
        if (f0 + fi < F) {
          const float* src = &melst[fi][m4];
          *reinterpret_cast<float4*>(o + (f0 + fi) * MEL_BANDS + m4) = make_float4(src[0], src[1], src[2], src[3]);
        }
      }
    }
    if constexpr (LAYOUT == 1) {  // (B, 128, F): each band's FPT frames contiguous
      float* o = out + b * ld_out;
      for (int i = tid; i < MEL_FPT * MEL_BANDS; i += 256) {
        const int m = i / MEL_FPT, fi = i % MEL_FPT;
        if (f0 + fi < F) o[m * F + f0 + fi] = melst[fi][m];
      }
    }
    if (tid == 0) {  // this tile's max and min log value over its live frames (no atomics, no init)
      float bm = red[0][0], bn = red[1][0];
#pragma unroll
      for (int w = 1; w < MEL_WAVES; ++w) {
        bm = fmaxf(bm, red[0][w]);
        bn = fminf(bn, red[1][w]);
      }
      tstat[t] = bm;
      tstat[n_tiles + t] = bn;
    }
  }
}

// Clip-max floor (maximum(x, max(x) - 8), essentials.py:485-488) on the (x + 4) / 4 values the tile
// kernel wrote.  One workgroup per tile: the clip max is the max of the clip's tile maxima; a tile
// whose minimum is not below the floor is left as it is (every value already final), any other is
// rewritten as max(y, (f + 4) / 4).
__global__ __launch_bounds__(256) void logmel_floor_kernel(float* __restrict__ out, int layout, int64_t F,
                                                           int64_t ld_out, int tiles_per_clip, int64_t n_tiles,
                                                           const float* __restrict__ tstat) {
  __shared__ float red[4];
  const int b = blockIdx.y, tl = blockIdx.x, tid = threadIdx.x;
  const float* tm = tstat + (int64_t)b * tiles_per_clip;
  float m = -3.0e38f;
  for (int i = tid; i < tiles_per_clip; i += 256) m = fmaxf(m, tm[i]);
  m = wave_max(m);
  if ((tid & 63) == 0) red[tid >> 6] = m;
  __syncthreads();
  const float floor_v = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3])) - 8.0f;
  if (!(tstat[n_tiles + (int64_t)b * tiles_per_clip + tl] < floor_v)) return;  // workgroup-uniform
  const float yf = (floor_v + 4.0f) * 0.25f;
  const int64_t f0 = (int64_t)tl * MEL_FPT;
  const int nf = (int)(F - f0 < MEL_FPT ? F - f0 : MEL_FPT);
  float* o = out + b * ld_out;
  if (layout == 0) {  // nf contiguous rows of 128
    float4* o4 = reinterpret_cast<float4*>(o + f0 * MEL_BANDS);
    for (int i = tid; i < nf * MEL_BANDS / 4; i += 256) {
      float4 v = o4[i];
      v.x = fmaxf(v.x, yf);
      v.y = fmaxf(v.y, yf);
      v.z = fmaxf(v.z, yf);
      v.w = fmaxf(v.w, yf);
      o4[i] = v;
    }
  } else {  // 128 runs of nf frames at stride F
    for (int i = tid; i < nf * MEL_BANDS; i += 256) {
      const int mb = i / nf, fi = i - mb * nf;
      float* q = o + mb * F + f0 + fi;
      *q = fmaxf(*q, yf);
    }
  }
}

}  // namespace asrx

using namespace asrx;

// wav: (B, N) rows at stride ld_wav.  out: (B, F, 128) if layout == 0 else (B, 128, F), clip stride
// ld_out (>= 128*F).  ws: float workspace of asrx_logmel_ws_bytes(B, N) bytes (per-tile max | min,
// overwritten).  pool: (B, T_pool) or null; the fused pool requires N == 160 * T_pool.  fbw/fbs: the
// lane-packed filterbank of asrx/mel.py lane_filterbank: fbs = band_a[64] | band_b[64] | start_a[64] |
// start_b[64] (even starts), fbw = weights [8 tap quads][64 lanes][4] (taps 0-7 band_a, 8-31 band_b,
// x 1/4).
static int64_t mel_tiles_per_clip(int64_t N) { return (1 + N / MEL_HOP + MEL_FPT - 1) / MEL_FPT; }

extern "C" int64_t asrx_logmel_ws_bytes(int64_t B, int64_t N) {
  return 2 * B * mel_tiles_per_clip(N) * (int64_t)sizeof(float);
}

extern "C" int asrx_logmel(const float* wav, int64_t B, int64_t N, int64_t ld_wav, const float* consts,
                           const float* fbw, const int* fbs, float* out, int layout, int64_t ld_out,
                           void* ws, float* pool, int64_t T_pool, hipStream_t stream) {
  ASRX_REQUIRE(B > 0 && N > 0, "asrx_logmel: empty input");
  ASRX_REQUIRE(B < 65536, "asrx_logmel: too many clips (grid y)");
  const int64_t F = 1 + N / MEL_HOP;
  ASRX_REQUIRE(ld_out >= F * MEL_BANDS, "asrx_logmel: ld_out too small");
  ASRX_REQUIRE(layout != 0 || (ld_out % 4 == 0 && (reinterpret_cast<uintptr_t>(out) & 15) == 0),
               "asrx_logmel: (B, F, 128) layout needs 16-byte aligned rows");
  ASRX_REQUIRE(!pool || N == (int64_t)MEL_HOP * T_pool,
               "asrx_logmel: fused pool needs N == 160*T_pool (N=%ld T=%ld)", (long)N, (long)T_pool);
  const int tiles_per_clip = (int)mel_tiles_per_clip(N);
  const int64_t n_tiles = B * tiles_per_clip;
  float* tstat = static_cast<float*>(ws);
  // MEL_WPS resident workgroups per CU (168 VGPRs; LDS 54 KB for (B, F, 128), 48.6 KB for (B, 128, F))
  // on 256 CUs; each takes a contiguous run
  const int64_t slots = 256 * MEL_WPS;
  const int tiles_per_block = (int)std::max<int64_t>(1, (n_tiles + slots - 1) / slots);
  const int64_t grid = (n_tiles + tiles_per_block - 1) / tiles_per_block;
  const int vec_ok = (ld_wav % 4 == 0) && ((reinterpret_cast<uintptr_t>(wav) & 15) == 0);
  auto kern = layout == 0 ? logmel_tiles_kernel<0> : logmel_tiles_kernel<1>;
  kern<<<(unsigned)grid, 256, 0, stream>>>(wav, N, ld_wav, vec_ok, F, tiles_per_clip, n_tiles, tiles_per_block,
                                           consts, fbw, fbs, out, ld_out, tstat, pool, T_pool);
  logmel_floor_kernel<<<dim3((unsigned)tiles_per_clip, (unsigned)B), 256, 0, stream>>>(
      out, layout, F, ld_out, tiles_per_clip, n_tiles, tstat);
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
