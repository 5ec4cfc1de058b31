// asrx — MI355X (gfx950 / CDNA4) native kernels for the ASR hot path.
// Shared device helpers and the C-ABI error plumbing.
//
// Conventions (see include/asrx.h):
//   * every entry point is extern "C", takes raw device pointers, int64 sizes/strides and a
//     hipStream_t, launches on that stream and returns 0 on success or a nonzero code;
//   * kernels never allocate; the caller (PyTorch's caching allocator) owns every buffer;
//   * the last error message is thread-local and read back with asrx_last_error().
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>
#include <cstdio>
#include <cstdarg>

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;

namespace asrx {

// PREC_X3: fp32 storage with split-bf16 products (x = hi + lo, hi = bf16(x), lo = bf16(x - hi); a product is
// hi*hi + hi*lo + lo*hi on the bf16 MFMA, ~2^-16 relative per operand) -- asrx_gemm only
enum Prec : int { PREC_F32 = 0, PREC_BF16 = 1, PREC_X3 = 3 };

enum Act : int { ACT_NONE = 0, ACT_GELU = 1, ACT_SILU = 2, ACT_SIGMOID = 3, ACT_RELU = 4 };
// small_linear only: softmax over the N outputs of each row (forward only; the caller differentiates it)
constexpr int ACT_SOFTMAX = 16;

void set_error(const char* fmt, ...);
int check_launch(const char* what);

}  // namespace asrx

#define ASRX_NOISE_EPOCH_SETTER(NAME)                                                                      \
  extern "C" int NAME(uint32_t epoch, hipStream_t stream) {                                               \
    static uint32_t host_epoch[64];                                                                       \
    static unsigned slot = 0;                                                                             \
    uint32_t* src = &host_epoch[(slot++) & 63]; /* stays valid while the copy may still be pending */    \
    *src = epoch;                                                                                         \
    hipError_t e = hipMemcpyToSymbolAsync(HIP_SYMBOL(asrx::g_noise_epoch), src, sizeof(uint32_t), 0,      \
                                          hipMemcpyHostToDevice, stream);                                 \
    if (e != hipSuccess) {                                                                                \
      asrx::set_error("%s: %s", #NAME, hipGetErrorString(e));                                             \
      return (int)e;                                                                                      \
    }                                                                                                     \
    return 0;                                                                                             \
  }

#define ASRX_REQUIRE(cond, ...)            \
  do {                                     \
    if (!(cond)) {                         \
      asrx::set_error(__VA_ARGS__);        \
      return 2;                            \
    }                                      \
  } while (0)

#define ASRX_LAUNCHED(name) return asrx::check_launch(name)

// ---------------------------------------------------------------- device helpers
namespace asrx {

__device__ __forceinline__ float gelu_f(float x) {  // exact (erf) GELU, nn.GELU() default
  return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f));
}
// The activation derivatives are written without contractions in every translation unit (the row-kernel
// units build with -ffp-contract=off, the GEMM units do not): the backward's activation-gradient GEMM
// epilogue and asrx_act_bwd_bias then round identically.
__device__ __forceinline__ float gelu_grad(float x) {
#pragma clang fp contract(off)
  float cdf = 0.5f * (1.0f + erff(x * 0.70710678118654752f));
  float pdf = 0.39894228040143268f * __expf(-0.5f * x * x);
  return cdf + x * pdf;
}
// v_rcp_f32 (1 ulp) instead of an IEEE division: the epilogues apply this to every element of wide outputs
__device__ __forceinline__ float sigmoid_f(float x) { return __builtin_amdgcn_rcpf(1.0f + __expf(-x)); }
__device__ __forceinline__ float silu_f(float x) { return x * sigmoid_f(x); }
__device__ __forceinline__ float silu_grad(float x) {
#pragma clang fp contract(off)
  float s = sigmoid_f(x);
  return s * (1.0f + x * (1.0f - s));
}

__device__ __forceinline__ float apply_act(int act, float x) {
  switch (act) {
    case ACT_GELU: return gelu_f(x);
    case ACT_SILU: return silu_f(x);
    case ACT_SIGMOID: return sigmoid_f(x);
    case ACT_RELU: return x > 0.f ? x : 0.f;
    default: return x;
  }
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
// Cross-row exchanges on gfx950's v_permlane{16,32}_swap_b32 (VALU, no LDS round trip).  With both
// operands holding v, the 16-lane swap leaves rows (r0, r0, r2, r2) in one and (r1, r1, r3, r3) in the
// other, so a + b is v + v[lane ^ 16] in every lane; the 32-lane swap likewise pairs lane with lane ^ 32.
// Inline asm: the ROCm 7.2 compiler returns the first result for both members of the builtin's pair.
// The s_nop covers the VALU-write -> permlane-read hazard (the compiler cannot see into the asm).
__device__ __forceinline__ void xrow16(float& a, float& b) {
  asm("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(a), "+v"(b));
}
__device__ __forceinline__ void xrow32(float& a, float& b) {
  asm("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(a), "+v"(b));
}
// two / three independent swaps behind one s_nop (the second and third read registers no swap wrote)
__device__ __forceinline__ void xrow16x2(float& a0, float& b0, float& a1, float& b1) {
  asm("s_nop 1\n\tv_permlane16_swap_b32 %0, %1\n\tv_permlane16_swap_b32 %2, %3" : "+v"(a0), "+v"(b0), "+v"(a1), "+v"(b1));
}
__device__ __forceinline__ void xrow32x2(float& a0, float& b0, float& a1, float& b1) {
  asm("s_nop 1\n\tv_permlane32_swap_b32 %0, %1\n\tv_permlane32_swap_b32 %2, %3" : "+v"(a0), "+v"(b0), "+v"(a1), "+v"(b1));
}
__device__ __forceinline__ void xrow16x3(float& a0, float& b0, float& a1, float& b1, float& a2, float& b2) {
  asm("s_nop 1\n\tv_permlane16_swap_b32 %0, %1\n\tv_permlane16_swap_b32 %2, %3\n\tv_permlane16_swap_b32 %4, %5"
      : "+v"(a0), "+v"(b0), "+v"(a1), "+v"(b1), "+v"(a2), "+v"(b2));
}
__device__ __forceinline__ void xrow32x3(float& a0, float& b0, float& a1, float& b1, float& a2, float& b2) {
  asm("s_nop 1\n\tv_permlane32_swap_b32 %0, %1\n\tv_permlane32_swap_b32 %2, %3\n\tv_permlane32_swap_b32 %4, %5"
      : "+v"(a0), "+v"(b0), "+v"(a1), "+v"(b1), "+v"(a2), "+v"(b2));
}
__device__ __forceinline__ float dpp_row_sum(float v) {  // the 4 in-row DPP steps of wave_sum_dpp
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x141, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x140, 0xF, 0xF, false));
  return v;
}
// wave_sum_dpp of two / three independent values (each bit-identical to wave_sum_dpp of it), their chains
// interleaved and their cross-row swaps sharing one hazard s_nop
__device__ __forceinline__ void wave_sum2_dpp(float& x, float& y) {
  x = dpp_row_sum(x);
  y = dpp_row_sum(y);
  float a0 = x, b0 = x, a1 = y, b1 = y;
  xrow16x2(a0, b0, a1, b1);
  x = a0 + b0;
  y = a1 + b1;
  a0 = b0 = x;
  a1 = b1 = y;
  xrow32x2(a0, b0, a1, b1);
  x = a0 + b0;
  y = a1 + b1;
}
__device__ __forceinline__ void wave_sum3_dpp(float& x, float& y, float& z) {
  x = dpp_row_sum(x);
  y = dpp_row_sum(y);
  z = dpp_row_sum(z);
  float a0 = x, b0 = x, a1 = y, b1 = y, a2 = z, b2 = z;
  xrow16x3(a0, b0, a1, b1, a2, b2);
  x = a0 + b0;
  y = a1 + b1;
  z = a2 + b2;
  a0 = b0 = x;
  a1 = b1 = y;
  a2 = b2 = z;
  xrow32x3(a0, b0, a1, b1, a2, b2);
  x = a0 + b0;
  y = a1 + b1;
  z = a2 + b2;
}
// wave_sum_dpp of x beside wave_max_dpp of y (bit-identical to each alone), one hazard s_nop per swap pair
__device__ __forceinline__ void wave_sum_max_dpp(float& x, float& y) {
  x = dpp_row_sum(x);
  y = fmaxf(y, __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, y), 0xB1, 0xF, 0xF, false)));
  y = fmaxf(y, __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, y), 0x4E, 0xF, 0xF, false)));
  y = fmaxf(y, __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, y), 0x141, 0xF, 0xF, false)));
  y = fmaxf(y, __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, y), 0x140, 0xF, 0xF, false)));
  float a0 = x, b0 = x, a1 = y, b1 = y;
  xrow16x2(a0, b0, a1, b1);
  x = a0 + b0;
  y = fmaxf(a1, b1);
  a0 = b0 = x;
  a1 = b1 = y;
  xrow32x2(a0, b0, a1, b1);
  x = a0 + b0;
  y = fmaxf(a1, b1);
}
// Wave sum with the in-row steps on DPP: xor 1 and xor 2 by quad_perm, then the other quad of each 8
// (row_half_mirror) and the other 8 of each 16 (row_mirror); the two cross-row steps by permlane
// swaps.  Every lane ends with the full sum, bit-identical to the ds_bpermute (__shfl_xor) version
// (each step adds the same two values; float addition commutes).
__device__ __forceinline__ float wave_sum_dpp(float v) {
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x141, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x140, 0xF, 0xF, false));
  float a = v, b = v;
  xrow16(a, b);
  v = a + b;
  a = v;
  b = v;
  xrow32(a, b);
  return a + b;
}
// wave_sum_dpp's pattern with max (exact, so the result equals wave_max's)
__device__ __forceinline__ float wave_max_dpp(float v) {
  v = fmaxf(v, __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, false)));
  v = fmaxf(v, __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, false)));
  v = fmaxf(v, __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x141, 0xF, 0xF, false)));
  v = fmaxf(v, __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x140, 0xF, 0xF, false)));
  float a = v, b = v;
  xrow16(a, b);
  v = fmaxf(a, b);
  a = v;
  b = v;
  xrow32(a, b);
  return fmaxf(a, b);
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blockDim.x == NT (multiple of 64). `red` must hold NT/64 floats.
template <int NT>
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) t += red[i];
  return t;
}

// ------------------------------------------------------------ LDS-DMA from inline asm
// global -> LDS copies (global_load_lds_dword{,x4}) issued from inline asm.  The compiler's waitcnt
// model does not see them, so it neither drains them (vmcnt(0)) before every ds_read -- which is what
// it does for __builtin_amdgcn_global_load_lds, defeating any prefetch ring -- nor counts them:
// completion is tracked by hand with s_waitcnt vmcnt(N) + s_barrier.  M0 is written and restored
// inside the statement (MI355X guide, "LDS-DMA recipe").
typedef __attribute__((address_space(3))) char lds_char_t;
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(uintptr_t)(const lds_char_t*)p);
}
__device__ __forceinline__ void glds16(const void* gsrc, uint32_t lds_dst) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(gsrc), "s"(lds_dst) : "memory");
}
__device__ __forceinline__ void glds4(const void* gsrc, uint32_t lds_dst) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(gsrc), "s"(lds_dst) : "memory");
}
// s_waitcnt vmcnt(k) for the largest listed k <= n (waiting for more than needed is always safe).
__device__ __forceinline__ void wait_vm_le(int n) {
  if (n >= 48) asm volatile("s_waitcnt vmcnt(48)" ::: "memory");
  else if (n >= 40) asm volatile("s_waitcnt vmcnt(40)" ::: "memory");
  else if (n >= 32) asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
  else if (n >= 28) asm volatile("s_waitcnt vmcnt(28)" ::: "memory");
  else if (n >= 24) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
  else if (n >= 20) asm volatile("s_waitcnt vmcnt(20)" ::: "memory");
  else if (n >= 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  else if (n >= 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  else if (n >= 10) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
  else if (n >= 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if (n >= 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else if (n >= 5) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
  else if (n >= 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if (n >= 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
  else if (n >= 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else if (n >= 1) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// Ordered-int encoding so that atomicMax on int works for any float.
__host__ __device__ __forceinline__ int float_to_ordered(float f) {
  int i = __builtin_bit_cast(int, f);
  return i >= 0 ? i : i ^ 0x7fffffff;
}
__host__ __device__ __forceinline__ float ordered_to_float(int i) {
  return __builtin_bit_cast(float, i >= 0 ? i : i ^ 0x7fffffff);
}

// ------------------------------------------------------------ counter-based noise
// The reference draws torch Exp(1) noise inside F.gumbel_softmax (essentials.py:170,
// model.py:476) and Bernoulli masks inside nn.Dropout (model.py:107,147). Here noise is a pure
// function of (site key, logical element index): u = ((mix(mix(idx ^ k0) + k1) >> 9) + 0.5) / 2^23,
// so 2^-24 <= u <= 1 - 2^-24 exactly in fp32 (u never rounds to 0 or 1, gumbel noise stays finite),
// restated bit-for-bit in oracle/noise.py so the oracle sees the same draws.
__host__ __device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}
// Noise epoch: a device-side word mixed into every site key when nonzero.  A captured HIP graph bakes
// the host-computed site keys (seed, step, site) into its launches; bumping the epoch between replays
// (asrx_set_noise_epoch, a stream-ordered copy outside the graph) gives every replayed step fresh
// dropout masks and gumbel draws.  Epoch 0 (the default, and what every eager step uses) leaves the
// keys exactly as oracle/keys.py computes them.  One copy per translation unit (no relocatable
// device code); each noise-drawing TU exports its setter (ASRX_NOISE_EPOCH_SETTER).
static __device__ uint32_t g_noise_epoch;
// The site key with the epoch mixed in.  Row / element loops take it once before the loop: read per
// draw, the epoch was a global load inside the loop whose wait (vmcnt counts in order) drained every
// prefetch in flight on each row.  Read through the constant address space: a scalar load.
__device__ __forceinline__ uint32_t noise_key(uint32_t key) {
  const uint32_t ep = *(const __attribute__((address_space(4))) uint32_t*)&g_noise_epoch;
  if (ep != 0u) key ^= mix32(ep * 0x9E3779B9U + 0x7F4A7C15U);
  return key;
}
// draws from a key already passed through noise_key
__device__ __forceinline__ float noise_uniform_k(uint32_t key, uint32_t idx) {
  uint32_t h = mix32(mix32(idx ^ key) + (key * 0x9E3779B9U + 0x632BE5ABU));
  return ((float)(h >> 9) + 0.5f) * (1.0f / 8388608.0f);
}
__device__ __forceinline__ float noise_uniform(uint32_t key, uint32_t idx) {
  return noise_uniform_k(noise_key(key), idx);
}
// Gumbel(0,1) sample g = -log(E), E = -log(u) ~ Exp(1).
__device__ __forceinline__ float noise_gumbel_k(uint32_t key, uint32_t idx) {
  float u = noise_uniform_k(key, idx);
  return -logf(-logf(u));
}
__device__ __forceinline__ float noise_gumbel(uint32_t key, uint32_t idx) { return noise_gumbel_k(noise_key(key), idx); }

}  // namespace asrx

#define ASRX_NOISE_EPOCH_SETTER(NAME)                                                                      \
  extern "C" int NAME(uint32_t epoch, hipStream_t stream) {                                               \
    static uint32_t host_epoch[64];                                                                       \
    static unsigned slot = 0;                                                                             \
    uint32_t* src = &host_epoch[(slot++) & 63]; /* stays valid while the copy may still be pending */    \
    *src = epoch;                                                                                         \
    hipError_t e = hipMemcpyToSymbolAsync(HIP_SYMBOL(asrx::g_noise_epoch), src, sizeof(uint32_t), 0,      \
                                          hipMemcpyHostToDevice, stream);                                 \
    if (e != hipSuccess) {                                                                                \
      asrx::set_error("%s: %s", #NAME, hipGetErrorString(e));                                             \
      return (int)e;                                                                                      \
    }                                                                                                     \
    return 0;                                                                                             \
  }
