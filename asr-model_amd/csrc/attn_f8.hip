// Flash-attention forward with an fp8 (OCP e4m3) QK^T: the "fp8 attention" precision mode of
// SURVEY.md §8(b) (config 5: small model, fp8 attention, greedy decode).  Same SDPA contract as
// attn_mf.hip (model.py:307: head dim HD = 64 or 128, non-causal or top-left causal, Lq != Lk,
// ragged tails, fp32 (B, L, H, HD) q/k/v/o with arbitrary strides, natural-log lse).  HD = 128 keeps
// two 64-wide halves per tile (the attn_mf.hip layout) and issues one MX-rate MFMA per half.
//
// Workgroup = 8 waves = 256 query rows of one (b, h); wave = 32 rows; 64-key tiles, double-buffered.
//   Q and K are quantised per ROW to e4m3: x' = x / s, s = max|x_row| / 448 (the scale of a row
//     factors out of every dot product it enters, so S[key][q] = s_key * s_q * (K' Q'^T)[key][q]
//     exactly, up to the e4m3 rounding of K' and Q').  Q' rows live in registers, K' tiles in LDS
//     (64 B per key, 16-B chunks XOR-swizzled by key), the per-key scales in LDS beside them.
//   S^T = K' Q'^T  ONE v_mfma_scale_f32_32x32x64_f8f6f4 per 32-key block (the whole head dim in one
//     instruction, unit block scales): the MX-rate form, 2x the bf16 MFMA rate.  The reduction runs
//     over the 64 head dims in whatever order the hardware assigns to (lane>>5, byte); A and B are
//     laid out identically (lane = row, 32 consecutive dims of half lane>>5), so the order is
//     irrelevant.
//   softmax and O^T += V^T P^T are the bf16 path of attn_mf.hip unchanged (P in bf16, V^T by
//     ds_read_b64_tr_b16), so the fp8 rounding touches the scores only.
// Forward only: the backward of a model trained in this mode runs the bf16 kernels.
#include "common.h"

namespace asrx {

struct AttnStridesMF {
  int64_t b, l, h;
};

namespace af8 {

typedef int v8i32 __attribute__((ext_vector_type(8)));
typedef short v4i16 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4i16 lds_v4i16;

constexpr int QB = 256;
constexpr int KT = 64;
constexpr int NTHR = 512;
constexpr float LOG2E = 1.4426950408889634f;
constexpr float LN2 = 0.6931471805599453f;
constexpr float E4M3_MAX = 448.f;

__device__ __forceinline__ int vswz(int key) { return ((key >> 1) & 1) << 2; }
__device__ __forceinline__ int k8swz(int key) { return (key >> 2) & 3; }  // fp8 K rows: 4 chunks of 16 B

__device__ __forceinline__ unsigned pack2(float a, float b) {
  const unsigned lo = __builtin_bit_cast(unsigned short, (__bf16)a);
  const unsigned hi = __builtin_bit_cast(unsigned short, (__bf16)b);
  return lo | (hi << 16);
}

__device__ __forceinline__ bf16x8 pack8(const float (&v)[8]) {
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  u32x4 u = {pack2(v[0], v[1]), pack2(v[2], v[3]), pack2(v[4], v[5]), pack2(v[6], v[7])};
  return __builtin_bit_cast(bf16x8, u);
}

// four floats (already divided by the row scale, |x| <= 448) -> four e4m3 bytes, RNE
__device__ __forceinline__ unsigned f8x4(float a, float b, float c, float d) {
  int w = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
  w = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, w, true);
  return (unsigned)w;
}

__device__ __forceinline__ float amax4(const float4& x) {
  return fmaxf(fmaxf(fabsf(x.x), fabsf(x.y)), fmaxf(fabsf(x.z), fabsf(x.w)));
}

// one key row chunk (8 consecutive d) in fp32; rows past Lk read the last row and are zeroed
__device__ __forceinline__ void load8(const float* base, int64_t ld, int64_t key, int64_t Lk, int c, float4& a,
                                      float4& b) {
  const int64_t kc = key < Lk ? key : Lk - 1;
  const float* p = base + kc * ld + 8 * c;
  a = *reinterpret_cast<const float4*>(p);
  b = *reinterpret_cast<const float4*>(p + 4);
  if (key >= Lk) {
    a = make_float4(0.f, 0.f, 0.f, 0.f);
    b = a;
  }
}

// K chunks (8 consecutive d of every half) -> e4m3 in LDS with the key row's scale (the 8 threads
// of a key row are 8 consecutive lanes; each holds chunk c of every half)
template <int NH>
__device__ __forceinline__ void store_k8(unsigned char* Kt, float* ksc, int key, int c, const float4 (&a)[NH],
                                         const float4 (&b)[NH]) {
  float am = 0.f;
#pragma unroll
  for (int hf = 0; hf < NH; ++hf) am = fmaxf(am, fmaxf(amax4(a[hf]), amax4(b[hf])));
  am = fmaxf(am, __shfl_xor(am, 1));
  am = fmaxf(am, __shfl_xor(am, 2));
  am = fmaxf(am, __shfl_xor(am, 4));
  const float s = am > 0.f ? am / E4M3_MAX : 1.f;
  const float r = 1.f / s;
  const int chunk = (c >> 1) ^ k8swz(key);
#pragma unroll
  for (int hf = 0; hf < NH; ++hf) {
    uint2 u;
    u.x = f8x4(a[hf].x * r, a[hf].y * r, a[hf].z * r, a[hf].w * r);
    u.y = f8x4(b[hf].x * r, b[hf].y * r, b[hf].z * r, b[hf].w * r);
    *reinterpret_cast<uint2*>(Kt + hf * KT * 64 + key * 64 + 16 * chunk + 8 * (c & 1)) = u;
  }
  if (c == 0) ksc[key] = s;
}

__device__ __forceinline__ void store_v(unsigned short* tile, int key, int pc, const float4& a, const float4& b) {
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  u32x4 u = {pack2(a.x, a.y), pack2(a.z, a.w), pack2(b.x, b.y), pack2(b.z, b.w)};
  *reinterpret_cast<u32x4*>(tile + key * 64 + 8 * pc) = u;
}

template <int HD>
__global__ __launch_bounds__(NTHR, 1) void attn_fwd_f8_kernel(const float* __restrict__ q, const float* __restrict__ k,
                                                              const float* __restrict__ v, float* __restrict__ o,
                                                              float* __restrict__ lse, AttnStridesMF sq,
                                                              AttnStridesMF sk, AttnStridesMF sv, AttnStridesMF so,
                                                              int64_t H, int64_t Lq, int64_t Lk, int causal,
                                                              float scale) {
  constexpr int NH = HD / 64;
  __shared__ __attribute__((aligned(16))) unsigned char Ks[2][NH * KT * 64];
  __shared__ __attribute__((aligned(16))) float Kscale[2][KT];
  __shared__ __attribute__((aligned(16))) unsigned short Vs[2][NH * KT * 64];

  const int b = blockIdx.z, h = blockIdx.y;
  const int64_t q0 = (int64_t)blockIdx.x * QB;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int j = lane & 31, hi = lane >> 5;
  const int64_t qi = q0 + wid * 32 + j;
  const float* qb = q + b * sq.b + h * sq.h;
  const float* kb = k + b * sk.b + h * sk.h;
  const float* vb = v + b * sv.b + h * sv.h;

  // Q'^T (B operand): lane (q = j, hi) holds e4m3 Q[q][64 hf + 32 hi .. +31] / s_q, s_q over all HD
  v8i32 qf[NH];
  float sq_row;
  {
    float4 x[NH][8];
#pragma unroll
    for (int hf = 0; hf < NH; ++hf)
#pragma unroll
      for (int i = 0; i < 8; ++i) x[hf][i] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (qi < Lq) {
#pragma unroll
      for (int hf = 0; hf < NH; ++hf) {
        const float* p = qb + qi * sq.l + 64 * hf + 32 * hi;
#pragma unroll
        for (int i = 0; i < 8; ++i) x[hf][i] = *reinterpret_cast<const float4*>(p + 4 * i);
      }
    }
    float am = 0.f;
#pragma unroll
    for (int hf = 0; hf < NH; ++hf)
#pragma unroll
      for (int i = 0; i < 8; ++i) am = fmaxf(am, amax4(x[hf][i]));
    am = fmaxf(am, __shfl_xor(am, 32));
    sq_row = am > 0.f ? am / E4M3_MAX : 1.f;
    const float r = 1.f / sq_row;
#pragma unroll
    for (int hf = 0; hf < NH; ++hf)
#pragma unroll
      for (int i = 0; i < 8; ++i)
        qf[hf][i] = (int)f8x4(x[hf][i].x * r, x[hf][i].y * r, x[hf][i].z * r, x[hf][i].w * r);
  }
  const float c = scale * LOG2E;
  const float cq = c * sq_row;  // per-lane: score -> log2 domain, with the query's row scale folded in

  int64_t kend = Lk;
  if (causal) kend = min(Lk, q0 + QB);
  const int ntiles = (int)((kend + KT - 1) / KT);
  const int skey = tid >> 3, sc = tid & 7;

  float4 ka[NH], kb4[NH], va[NH], vb4[NH];
#pragma unroll
  for (int hf = 0; hf < NH; ++hf) {
    load8(kb + 64 * hf, sk.l, skey, Lk, sc, ka[hf], kb4[hf]);
    load8(vb + 64 * hf, sv.l, skey, Lk, sc, va[hf], vb4[hf]);
    store_v(Vs[0] + hf * KT * 64, skey, sc ^ vswz(skey), va[hf], vb4[hf]);
  }
  store_k8<NH>(Ks[0], Kscale[0], skey, sc, ka, kb4);
  __syncthreads();

  f32x16 oacc[HD / 32];
#pragma unroll
  for (int d = 0; d < HD / 32; ++d)
#pragma unroll
    for (int r = 0; r < 16; ++r) oacc[d][r] = 0.f;
  float m = -INFINITY;  // running max of (unscaled-by-c) scores
  float l = 0.f;

  for (int t = 0; t < ntiles; ++t) {
    const int buf = t & 1;
    const int64_t k0 = (int64_t)t * KT;
    if (t + 1 < ntiles) {
#pragma unroll
      for (int hf = 0; hf < NH; ++hf) {
        load8(kb + 64 * hf, sk.l, k0 + KT + skey, Lk, sc, ka[hf], kb4[hf]);
        load8(vb + 64 * hf, sv.l, k0 + KT + skey, Lk, sc, va[hf], vb4[hf]);
      }
    }
    const unsigned char* Kt = Ks[buf];
    const float* ksc = Kscale[buf];
    const unsigned short* Vt = Vs[buf];

    // ---- S^T = K' Q'^T, one MX-rate MFMA per 32-key block and half, then the per-key scale
    f32x16 sacc[2];
#pragma unroll
    for (int kb2 = 0; kb2 < 2; ++kb2) {
      const int key = 32 * kb2 + j;
#pragma unroll
      for (int r = 0; r < 16; ++r) sacc[kb2][r] = 0.f;
#pragma unroll
      for (int hf = 0; hf < NH; ++hf) {
        const unsigned char* row = Kt + hf * KT * 64 + key * 64;
        const uint4 a0 = *reinterpret_cast<const uint4*>(row + 16 * ((2 * hi) ^ k8swz(key)));
        const uint4 a1 = *reinterpret_cast<const uint4*>(row + 16 * ((2 * hi + 1) ^ k8swz(key)));
        const v8i32 a = {(int)a0.x, (int)a0.y, (int)a0.z, (int)a0.w, (int)a1.x, (int)a1.y, (int)a1.z, (int)a1.w};
        sacc[kb2] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, qf[hf], sacc[kb2], 0, 0, 0, 0, 0, 0);
      }
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {  // keys 32 kb2 + 8 g4 + 4 hi + (0..3)
        const float4 s4 = *reinterpret_cast<const float4*>(ksc + 32 * kb2 + 8 * g4 + 4 * hi);
        sacc[kb2][4 * g4] *= s4.x;
        sacc[kb2][4 * g4 + 1] *= s4.y;
        sacc[kb2][4 * g4 + 2] *= s4.z;
        sacc[kb2][4 * g4 + 3] *= s4.w;
      }
    }

    const bool need_mask = (k0 + KT > Lk) || (causal && k0 + KT - 1 > q0 + wid * 32);
    float tmax = -INFINITY;
#pragma unroll
    for (int kb2 = 0; kb2 < 2; ++kb2)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float x = sacc[kb2][r];
        if (need_mask) {
          const int64_t key = k0 + 32 * kb2 + (r & 3) + 8 * (r >> 2) + 4 * hi;
          if (key >= Lk || (causal && key > qi)) x = -INFINITY;
          sacc[kb2][r] = x;
        }
        tmax = fmaxf(tmax, x);
      }
    tmax = fmaxf(tmax, __shfl_xor(tmax, 32));
    // lazy rescale: the running max moves only when a score passes it by more than 2^8 in the exp2
    // domain (p <= 256 otherwise, exact in the fp32 sums and fine in bf16), so most tiles skip the
    // O / l rescale; m = -inf (nothing seen yet) moves on the first finite score
    const bool up = tmax * cq > m * cq + 8.f;
    if (__any(up)) {  // wave-uniform
      const float alpha = up ? __builtin_amdgcn_exp2f(m * cq - tmax * cq) : 1.f;  // m = -inf -> 0
      if (up) m = tmax;
      l *= alpha;
#pragma unroll
      for (int d = 0; d < HD / 32; ++d)
#pragma unroll
        for (int r = 0; r < 16; ++r) oacc[d][r] *= alpha;
    }
    const float mc = m == -INFINITY ? 0.f : m * cq;
    bf16x8 pb[2][2];
    float lsum = 0.f;
#pragma unroll
    for (int kb2 = 0; kb2 < 2; ++kb2)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        float pv[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          pv[e] = __builtin_amdgcn_exp2f(__builtin_fmaf(sacc[kb2][8 * s2 + e], cq, -mc));
          lsum += pv[e];
        }
        pb[kb2][s2] = pack8(pv);
      }
    l += lsum;

    // ---- O^T += V^T P^T (bf16, as attn_mf.hip)
    const int g = lane >> 4, gi = lane & 15;
    const int trow = gi >> 2, tcol = 4 * (gi & 3);
#pragma unroll
    for (int kb2 = 0; kb2 < 2; ++kb2)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const int kbase = 32 * kb2 + 16 * s2 + 4 * (g >> 1);
#pragma unroll
        for (int d = 0; d < HD / 32; ++d) {
          const unsigned short* Vh = Vt + (d >> 1) * KT * 64;
          const int col = 32 * (d & 1) + 16 * (g & 1) + tcol;
          const int key1 = kbase + trow, key2 = kbase + 8 + trow;
          const v4i16 t1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (lds_v4i16*)(Vh + key1 * 64 + 8 * ((col >> 3) ^ vswz(key1)) + (col & 7)));
          const v4i16 t2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (lds_v4i16*)(Vh + key2 * 64 + 8 * ((col >> 3) ^ vswz(key2)) + (col & 7)));
          typedef short v8i16 __attribute__((ext_vector_type(8)));
          const v8i16 a8 = {t1[0], t1[1], t1[2], t1[3], t2[0], t2[1], t2[2], t2[3]};
          oacc[d] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a8), pb[kb2][s2], oacc[d],
                                                              0, 0, 0);
        }
      }

    if (t + 1 < ntiles) {
      store_k8<NH>(Ks[buf ^ 1], Kscale[buf ^ 1], skey, sc, ka, kb4);
#pragma unroll
      for (int hf = 0; hf < NH; ++hf) store_v(Vs[buf ^ 1] + hf * KT * 64, skey, sc ^ vswz(skey), va[hf], vb4[hf]);
    }
    __syncthreads();
  }

  const float lt = l + __shfl_xor(l, 32);
  if (qi < Lq) {
    const float inv = 1.0f / lt;
    float* orow = o + b * so.b + h * so.h + qi * so.l;
#pragma unroll
    for (int d = 0; d < HD / 32; ++d)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int dd = 64 * (d >> 1) + 32 * (d & 1) + 8 * g4 + 4 * hi;
        *reinterpret_cast<float4*>(orow + dd) =
            make_float4(oacc[d][4 * g4] * inv, oacc[d][4 * g4 + 1] * inv, oacc[d][4 * g4 + 2] * inv,
                        oacc[d][4 * g4 + 3] * inv);
      }
    if (hi == 0) lse[((int64_t)b * H + h) * Lq + qi] = (m * cq + __builtin_amdgcn_logf(lt)) * LN2;
  }
}

}  // namespace af8

// fp8-QK^T flash-attention forward; called by asrx_attn_fwd for prec == PREC_FP8ATT.
int attn_fwd_f8(const float* q, const int64_t* sq, const float* k, const int64_t* sk, const float* v,
                const int64_t* sv, float* o, const int64_t* so, float* lse, int64_t B, int64_t H, int64_t Lq,
                int64_t Lk, int64_t hd, int causal, float scale, hipStream_t stream) {
  dim3 g((unsigned)((Lq + af8::QB - 1) / af8::QB), (unsigned)H, (unsigned)B);
  AttnStridesMF Sq{sq[0], sq[1], sq[2]}, Sk{sk[0], sk[1], sk[2]}, Sv{sv[0], sv[1], sv[2]}, So{so[0], so[1], so[2]};
  if (hd == 64)
    af8::attn_fwd_f8_kernel<64><<<g, af8::NTHR, 0, stream>>>(q, k, v, o, lse, Sq, Sk, Sv, So, H, Lq, Lk, causal, scale);
  else
    af8::attn_fwd_f8_kernel<128><<<g, af8::NTHR, 0, stream>>>(q, k, v, o, lse, Sq, Sk, Sv, So, H, Lq, Lk, causal, scale);
  return 0;
}

}  // namespace asrx
