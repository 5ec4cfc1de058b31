// MSheath (model.py:387-507) per-sample control flow and its row updates, batched with batch-1
// semantics per sample.  The reference runs a Python while-loop with `.item()` branches per layer;
// here every sample's trajectory is device state and each layer step is three launches:
//   x_new = x + g * ion * out               axpy_row2 (model.py:461)
//   control: potential, gumbel policy, action, alpha/beta/gam, mem_w, next layer  msheath_ctrl
//   x = act ? alpha*x_new + beta*orig + gam : x                                     jump_select
// instead of ~25 small tensor ops forward and ~40 backward.
#include <type_traits>
#include "common.h"

namespace asrx {

// Per-sample record saved by the control forward for its backward.
struct CtrlRec {
  float ys[3];    // softmax(policy + gumbel) of this layer
  float action;   // 0, 1, 2 (model.py:478-482)
  float low;      // potential < 0.1 forced action 1 (model.py:480)
  float jump_g;   // the STE-gathered jump weight (1 when low or last layer)
  float cg;       // gam coefficient (1 - jw) * jump_g when jumped, else 0
  float act;      // sample was at this layer
};

// Forward.  grid B, 256 threads.  policy (B,3), gpol (B,3) with row stride ld_gpol (the noise of
// this layer), ion (B,L) the v_gate output, mem_v (B) sigmoid(mem_gate(mem)), mem_w / mem (B,D),
// jump_s (3), next_i (B) float layer index.  Outputs alpha, beta (B), gam (B,D), mem_w_out (B,D),
// active (B), next_out (B), rec (B).
// CT: threads of the forward control kernel (one workgroup per sample): above D = 512 the mem-partial loads of 512
// threads take half the dependent trips of 256 (8.6 vs 11.2 us at B = 8, L = 6002, D = 768); at D <= 512 the
// 256-thread kernel is as fast or faster (7.8 vs 8.6 us at B = 32, D = 384; profiles/r06_ctrl_ab.txt)
template <int CT>
__global__ __launch_bounds__(CT) void msheath_ctrl_fwd_kernel(
    const float* __restrict__ policy, const float* __restrict__ gpol, int64_t ld_gpol, const float* __restrict__ ion,
    const float* __restrict__ mem_v, const float* __restrict__ mem_w, const float* __restrict__ mem,
    const float* __restrict__ jump_s, const float* __restrict__ next_i, int layer_i, int layers, int64_t L, int D,
    float* __restrict__ alpha, float* __restrict__ beta, float* __restrict__ gam, float* __restrict__ mem_w_out,
    float* __restrict__ active, float* __restrict__ next_out, CtrlRec* __restrict__ rec, int64_t ld_mem_w,
    const float* __restrict__ mg_w, const float* __restrict__ mg_b, float* __restrict__ mem_v_out,
    const float* __restrict__ mem_part, int nchunk, float* __restrict__ mem_out) {
  __shared__ float red[CT / 64];
  const int64_t b = blockIdx.x;
  // the sample's ion values (L <= 12 * 512: the configurations' 3001 / 6002 frames) are requested first, so
  // their loads are in flight together with the mem partials' instead of after them
  constexpr int IQ = 6144 / CT;
  const float* ib = ion + b * L;
  const bool ion_pre = L <= (int64_t)IQ * CT;
  float iv[IQ];
  if (ion_pre) {
#pragma unroll
    for (int j = 0; j < IQ; ++j) iv[j] = ib[min<int64_t>(threadIdx.x + CT * j, L - 1)];
  }
  if (mem_part) {  // mem = (1/L) sum over the row chunks of x_new, in chunk order (deterministic)
    // the chunk partials are loaded 16 at a time before they are added (in chunk order, so the sum
    // is bit-identical to the sequential loop): a dependent load-add chain over ~47 chunks left
    // every load's latency exposed (24 us per launch at B = 32)
    // (a thread's two columns c0 and c0 + CT in flight together, and the last partial group loaded from
    // clamped addresses like the full ones: its serial remainder loop and the second column's separate pass
    // exposed ~20 load latencies per launch)
    const float* mp = mem_part + (int64_t)b * nchunk * D;
    for (int c0 = threadIdx.x; c0 < D; c0 += 2 * CT) {
      const int c1 = c0 + CT;
      const bool two = c1 < D;
      const int c1c = two ? c1 : c0;
      float t0 = 0.f, t1 = 0.f;
      for (int k = 0; k < nchunk; k += 16) {
        float v0[16], v1[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          const int64_t kk = min(k + j, nchunk - 1);
          v0[j] = mp[kk * D + c0];
          v1[j] = mp[kk * D + c1c];
        }
#pragma unroll
        for (int j = 0; j < 16; ++j)
          if (k + j < nchunk) {
            t0 += v0[j];
            t1 += v1[j];
          }
      }
      mem_out[b * D + c0] = t0 * (1.0f / (float)L);
      if (two) mem_out[b * D + c1] = t1 * (1.0f / (float)L);
    }
    __syncthreads();
    mem = mem_out;
  }
  float s = 0.f;
  if (ion_pre) {  // the thread's values in the order of the loop below
#pragma unroll
    for (int j = 0; j < IQ; ++j)
      if (threadIdx.x + CT * j < L) s += iv[j];
  } else {
    for (int64_t l = threadIdx.x; l < L; l += 8 * CT) {  // 8 loads in flight (the tail's from clamped
      float v[8];                                          // addresses), added in the same order
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = ib[min<int64_t>(l + CT * j, L - 1)];
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (l + CT * j < L) s += v[j];
    }
  }
  const float potential = block_sum<CT>(s, red) / (float)L;  // ion.mean(dim=1), model.py:466
  float mv;
  if (mg_w) {  // mem_v = sigmoid(mem_gate(mem)) computed here (model.py:464)
    float t = 0.f;
    for (int c = threadIdx.x; c < D; c += CT) t += mem[b * D + c] * mg_w[c];
    mv = sigmoid_f(block_sum<CT>(t, red) + mg_b[0]);
    if (threadIdx.x == 0) mem_v_out[b] = mv;
  } else {
    mv = mem_v[b];
  }
  const float ni = next_i ? next_i[b] : 0.f;  // null: every sample starts at layer 0
  const float act = ni == (float)layer_i ? 1.f : 0.f;
  float ys[3] = {0.f, 0.f, 0.f};
  int action;
  float jump_g, low = 0.f;
  if (layer_i < layers - 1) {
    // F.gumbel_softmax(policy, tau=1, hard=True) (model.py:475-477) with keyed gumbel noise
    float z[3], m = -INFINITY;
    for (int k = 0; k < 3; ++k) {
      z[k] = policy[b * 3 + k] + gpol[b * ld_gpol + k];
      m = fmaxf(m, z[k]);
    }
    float den = 0.f;
    for (int k = 0; k < 3; ++k) {
      ys[k] = expf(z[k] - m);
      den += ys[k];
    }
    int a = 0;
    for (int k = 0; k < 3; ++k) {
      ys[k] /= den;
      if (ys[k] > ys[a]) a = k;
    }
    const float jg = (1.f - ys[a]) + ys[a];  // (y_hard - y.detach() + y)[a]
    low = potential < 0.1f ? 1.f : 0.f;
    action = low != 0.f ? 1 : a;
    jump_g = low != 0.f ? 1.f : jg;
  } else {
    action = 0;
    jump_g = 1.f;
  }
  const bool jumped = action > 0;
  const float jw = jump_s[min(max(action - 1, 0), 2)];
  const float al = jumped ? 1.f : jump_g;
  const float be = jumped ? jw * jump_g : 0.f;
  const float cg = jumped ? (1.f - jw) * jump_g : 0.f;
  for (int c = threadIdx.x; c < D; c += CT) {
    const float mw = mem_w[b * ld_mem_w + c];                 // ld 0: the (1, 1, D) parameter broadcast
    const float mwn = mv * mw + (1.f - mv) * mem[b * D + c];  // model.py:464
    gam[b * D + c] = cg * mwn;
    mem_w_out[b * D + c] = act != 0.f ? mwn : mw;
  }
  if (threadIdx.x == 0) {
    alpha[b] = al;
    beta[b] = be;
    active[b] = act;
    const float step = jumped ? (float)min(layer_i + action + 1, layers) : (float)(layer_i + 1);
    next_out[b] = act != 0.f ? step : ni;
    CtrlRec r;
    r.ys[0] = ys[0];
    r.ys[1] = ys[1];
    r.ys[2] = ys[2];
    r.action = (float)action;
    r.low = low;
    r.jump_g = jump_g;
    r.cg = cg;
    r.act = act;
    rec[b] = r;
  }
}

// Backward.  g_mwo may be null (mem_w of the last layer is not used).  Writes g_policy (B,3),
// g_mem_v (B), g_mem_w (B,D), g_mem (B,D); accumulates g_jump_s (3) with atomics.
__global__ __launch_bounds__(256) void msheath_ctrl_bwd_kernel(
    const float* __restrict__ g_alpha, const float* __restrict__ g_beta, const float* __restrict__ g_gam,
    const float* __restrict__ g_mwo, const float* __restrict__ mem_v, const float* __restrict__ mem_w,
    const float* __restrict__ mem, const float* __restrict__ jump_s, const CtrlRec* __restrict__ rec, int layer_i,
    int layers, int D, float* __restrict__ g_policy, float* __restrict__ g_mem_v, float* __restrict__ g_mem_w,
    float* __restrict__ g_mem, float* __restrict__ g_jump_s, int64_t ld_mem_w, int* __restrict__ has_orig,
    int acc_policy, const float* __restrict__ mg_w, float* __restrict__ g_mg_w, float* __restrict__ g_mg_b,
    const float2* __restrict__ part_ab = nullptr, const float* __restrict__ part_g = nullptr, int nlc = 0,
    int ncc = 0) {
  __shared__ float red[4];
  const int64_t b = blockIdx.x;
  const CtrlRec r = rec[b];
  const float mv = mem_v[b];
  const bool act = r.act != 0.f;
  float s_cg = 0.f, s_mv = 0.f;
  for (int c = threadIdx.x; c < D; c += 256) {
    const float mw = mem_w[b * ld_mem_w + c], me = mem[b * D + c];
    const float mwn = mv * mw + (1.f - mv) * me;
    float gg;
    if (part_g) {  // the jump-select backward's L-chunk partials, added in chunk order (deterministic;
      gg = 0.f;      // 16 loads in flight, the last group's from clamped addresses)
      for (int k = 0; k < nlc; k += 16) {
        float v[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) v[j] = part_g[(b * nlc + min(k + j, nlc - 1)) * D + c];
#pragma unroll
        for (int j = 0; j < 16; ++j)
          if (k + j < nlc) gg += v[j];
      }
    } else {
      gg = g_gam[b * D + c];
    }
    const float go = g_mwo ? g_mwo[b * D + c] : 0.f;
    const float gmwn = gg * r.cg + (act ? go : 0.f);
    s_cg += gg * mwn;
    s_mv += gmwn * (mw - me);
    g_mem_w[b * D + c] = gmwn * mv + (act ? 0.f : go);
    g_mem[b * D + c] = gmwn * (1.f - mv);
  }
  s_cg = block_sum<256>(s_cg, red);
  s_mv = block_sum<256>(s_mv, red);
  if (mg_w) {  // mem_v = sigmoid(mem . mg_w + mg_b): its backward onto mem and the gate parameters
    const float gz = s_mv * mv * (1.f - mv);
    for (int c = threadIdx.x; c < D; c += 256) {
      g_mem[b * D + c] += gz * mg_w[c];
      atomicAdd(g_mg_w + c, gz * mem[b * D + c]);
    }
    if (threadIdx.x == 0) atomicAdd(g_mg_b, gz);
  }
  if (threadIdx.x == 0) {
    if (g_mem_v) g_mem_v[b] = s_mv;
    const int action = (int)r.action;
    const bool jumped = action > 0;
    float ga, gb;
    if (part_ab) {  // in order, 16 loads in flight (a dependent chain of ~100 loads cost ~10 us per launch)
      ga = 0.f, gb = 0.f;
      const int n = nlc * ncc;
      const float2* pb = part_ab + b * n;
      for (int k = 0; k < n; k += 16) {
        float2 v[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) v[j] = pb[min(k + j, n - 1)];
#pragma unroll
        for (int j = 0; j < 16; ++j)
          if (k + j < n) {
            ga += v[j].x;
            gb += v[j].y;
          }
      }
    } else {
      ga = g_alpha[b], gb = g_beta[b];
    }
    const int widx = min(max(action - 1, 0), 2);
    const float jw = jump_s[widx];
    const float g_jump = jumped ? jw * gb + (1.f - jw) * s_cg : ga;
    if (jumped) atomicAdd(g_jump_s + widx, r.jump_g * (gb - s_cg));
    float gp[3] = {0.f, 0.f, 0.f};
    if (layer_i < layers - 1 && r.low == 0.f) {
      // d jump_g / d ys[a] = 1 (straight-through), then softmax backward to the policy logits
      int a = 0;
      for (int k = 1; k < 3; ++k)
        if (r.ys[k] > r.ys[a]) a = k;
      for (int k = 0; k < 3; ++k) gp[k] = r.ys[k] * ((k == a ? 1.f : 0.f) - r.ys[a]) * g_jump;
    }
    for (int k = 0; k < 3; ++k) g_policy[b * 3 + k] = (acc_policy ? g_policy[b * 3 + k] : 0.f) + gp[k];
    // jump_select4_bwd_acc of this layer wrote orig's gradient for a jumping active sample
    if (has_orig && act && jumped && jw * r.jump_g != 0.f) has_orig[b] = 1;
  }
}

// out = x + s1[r] * s2[r] * y  (s2 may be null) -- model.py:461 with s1 = gate, s2 = ion.
__global__ void axpy_row2_kernel(const float4* __restrict__ x, const float* __restrict__ s1,
                                 const float* __restrict__ s2, const float4* __restrict__ y, float4* __restrict__ out,
                                 int64_t rows, int d4) {
  const int64_t total = rows * d4;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / d4;
    const float sc = s1[r] * (s2 ? s2[r] : 1.f);
    const float4 a = x[i], v = y[i];
    out[i] = make_float4(a.x + sc * v.x, a.y + sc * v.y, a.z + sc * v.z, a.w + sc * v.w);
  }
}

// x_new = x + s1 s2 y (model.py:461) and the per-sample column sums for mem = mean_l x_new (463) in
// one pass.  grid (B, ceil(L / 64)); the 256 threads are nrl = 256 / d4 row lanes x d4 float4 columns
// (d4 <= 256), each keeping its column's partial sum in registers; the workgroup's sums go to
// part[b][chunk][:] (no atomics: the control kernel adds the chunks in a fixed order, so the forward
// is deterministic -- its hard decisions must not depend on atomic ordering).
constexpr int MEM_CHUNK = 64;
__global__ __launch_bounds__(256) void axpy_row2_colsum_kernel(const float4* __restrict__ x, const float* __restrict__ s1,
                                                               const float* __restrict__ s2, const float4* __restrict__ y,
                                                               float4* __restrict__ out, float4* __restrict__ part,
                                                               int64_t L, int d4, const float* __restrict__ next_i,
                                                               int layer) {
  __shared__ float4 red[256];
  const int nrl = 256 / d4;
  const int c = threadIdx.x % d4, rl = threadIdx.x / d4;
  const int64_t b = blockIdx.x;
  if (next_i && next_i[b] != (float)layer) {  // sample not at this layer: x_new unused, mem = 0
    if (rl == 0) part[((int64_t)b * gridDim.y + blockIdx.y) * d4 + c] = make_float4(0.f, 0.f, 0.f, 0.f);
    return;
  }
  const int64_t l0 = (int64_t)blockIdx.y * MEM_CHUNK, l1 = min<int64_t>(L, l0 + MEM_CHUNK);
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  auto one = [&](float sc, float4 a, float4 v, int64_t i) __attribute__((always_inline)) {
    const float4 o = make_float4(__builtin_fmaf(sc, v.x, a.x), __builtin_fmaf(sc, v.y, a.y),
                                 __builtin_fmaf(sc, v.z, a.z), __builtin_fmaf(sc, v.w, a.w));
    if (out) out[i] = o;  // null: column sums only (the in-place no-grad MSheath recomputes x_new)
    acc.x += o.x; acc.y += o.y; acc.z += o.z; acc.w += o.w;
  };
  if (rl < nrl) {
    int64_t l = l0 + rl;
    // U of the thread's rows per trip, every load issued first (one row per trip exposed a full load
    // latency per row; most launches have few samples at the layer, so few waves per SIMD, and the
    // bytes in flight per wave set the rate); the sums keep the row order, so the results are unchanged
    auto trips = [&](auto UC) __attribute__((always_inline)) {
      constexpr int U = decltype(UC)::value;
      for (; l + (U - 1) * nrl < l1; l += U * nrl) {
        float sc[U];
        float4 a[U], v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int64_t r = b * L + l + u * nrl;
          sc[u] = s1[r] * s2[r];
          a[u] = x[r * d4 + c];
          v[u] = y[r * d4 + c];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) one(sc[u], a[u], v[u], (b * L + l + u * nrl) * d4 + c);
      }
    };
    trips(std::integral_constant<int, 8>{});
    trips(std::integral_constant<int, 4>{});
    for (; l < l1; l += nrl) {
      const int64_t r = b * L + l;
      one(s1[r] * s2[r], x[r * d4 + c], y[r * d4 + c], r * d4 + c);
    }
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  if (rl == 0) {
    for (int k = 1; k < nrl; ++k) {
      const float4 t = red[k * d4 + c];
      acc.x += t.x; acc.y += t.y; acc.z += t.z; acc.w += t.w;
    }
    part[((int64_t)b * gridDim.y + blockIdx.y) * d4 + c] = acc;
  }
}

// dy = s1 s2 g ; t = sum_j g y ; ds1 = s2 t ; ds2 = s1 t.  One wave per row.
__global__ __launch_bounds__(256) void axpy_row2_bwd_kernel(const float4* __restrict__ g, const float* __restrict__ s1,
                                                            const float* __restrict__ s2, const float4* __restrict__ y,
                                                            float4* __restrict__ dy, float* __restrict__ ds1,
                                                            float* __restrict__ ds2, int64_t rows, int d4) {
  const int lane = threadIdx.x & 63;
  for (int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); r < rows; r += (int64_t)gridDim.x * 4) {
    const float a = s1[r], c = s2 ? s2[r] : 1.f;
    const float sc = a * c;
    float t = 0.f;
    for (int j = lane; j < d4; j += 64) {
      const float4 gv = g[r * d4 + j], yv = y[r * d4 + j];
      t += gv.x * yv.x + gv.y * yv.y + gv.z * yv.z + gv.w * yv.w;
      dy[r * d4 + j] = make_float4(sc * gv.x, sc * gv.y, sc * gv.z, sc * gv.w);
    }
    t = wave_sum(t);
    if (lane == 0) {
      ds1[r] = c * t;
      if (ds2) ds2[r] = a * t;
    }
  }
}

// jump_select forward, float4: out = act ? alpha*xn + beta*orig + gam : xold.  grid (chunks, B).
__global__ void jump_select4_kernel(const float4* __restrict__ xn, const float4* __restrict__ orig,
                                    const float4* __restrict__ xold, const float* __restrict__ act,
                                    const float* __restrict__ alpha, const float* __restrict__ beta,
                                    const float4* __restrict__ gam, float4* __restrict__ out, int64_t L, int d4) {
  const int64_t b = blockIdx.y;
  const int64_t n = L * d4;
  const int64_t base = b * n;
  const bool a = act[b] != 0.f;
  const float al = alpha[b], be = beta[b];
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    if (a) {
      const float4 u = xn[base + i], v = orig[base + i], w = gam[b * d4 + i % d4];
      out[base + i] = make_float4(__builtin_fmaf(al, u.x, __builtin_fmaf(be, v.x, w.x)),
                                  __builtin_fmaf(al, u.y, __builtin_fmaf(be, v.y, w.y)),
                                  __builtin_fmaf(al, u.z, __builtin_fmaf(be, v.z, w.z)),
                                  __builtin_fmaf(al, u.w, __builtin_fmaf(be, v.w, w.w)));
    } else {
      out[base + i] = xold[base + i];
    }
  }
}

// No-grad MSheath layer step (the reference's dead blocks, eval, decoding: nothing is saved for a
// backward): for a sample at this layer xout <- alpha (xin + s1 s2 y) + beta orig + gam, i.e. x_new
// (model.py:461) and the jump select (489-501) in one pass without materialising x_new.  In place
// (xin == xout) a sample not at the layer is not touched -- its x already is the layer's output; otherwise
// it is copied.  Same arithmetic as axpy_row2_colsum + jump_select4 (explicit fma): bit-identical.
__global__ void jump_axpy_inplace_kernel(const float4* xin, float4* xout, const float* __restrict__ s1,
                                         const float* __restrict__ s2, const float4* __restrict__ y,
                                         const float4* __restrict__ orig, const float* __restrict__ act,
                                         const float* __restrict__ alpha, const float* __restrict__ beta,
                                         const float4* __restrict__ gam, int64_t L, int d4) {
  const int64_t b = blockIdx.y;
  const int64_t n = L * d4;
  const int64_t base = b * n;
  if (act[b] == 0.f) {
    if (xin != xout)
      for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        xout[base + i] = xin[base + i];
    return;
  }
  const float al = alpha[b], be = beta[b];
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = b * L + i / d4;
    const float sc = s1[r] * s2[r];
    const float4 a = xin[base + i], v = y[base + i], o = orig[base + i], w = gam[b * d4 + i % d4];
    const float4 u = make_float4(__builtin_fmaf(sc, v.x, a.x), __builtin_fmaf(sc, v.y, a.y), __builtin_fmaf(sc, v.z, a.z),
                                 __builtin_fmaf(sc, v.w, a.w));
    xout[base + i] = make_float4(__builtin_fmaf(al, u.x, __builtin_fmaf(be, o.x, w.x)),
                                 __builtin_fmaf(al, u.y, __builtin_fmaf(be, o.y, w.y)),
                                 __builtin_fmaf(al, u.z, __builtin_fmaf(be, o.z, w.z)),
                                 __builtin_fmaf(al, u.w, __builtin_fmaf(be, o.w, w.w)));
  }
}

// jump_select backward, float4: a 256-thread workgroup per (sample, 32 float4 columns, L chunk):
// 8 row groups of 32 lanes; per-sample sums leave as atomics (dalpha, dbeta, dgam zeroed by the
// launcher).  Inactive samples only copy g to dxold.
__global__ __launch_bounds__(256) void jump_select4_bwd_kernel(
    const float4* __restrict__ g, const float4* __restrict__ xn, const float4* __restrict__ orig,
    const float* __restrict__ act, const float* __restrict__ alpha, const float* __restrict__ beta,
    float4* __restrict__ dxn, float4* __restrict__ dorig, float4* __restrict__ dxold, float* __restrict__ dalpha,
    float* __restrict__ dbeta, float* __restrict__ dgam, int64_t L, int d4, int lchunk) {
  __shared__ float4 sg_s[8][32];
  __shared__ float red[2][4];
  const int lane = threadIdx.x & 31, grp = threadIdx.x >> 5;
  const int cchunks = (d4 + 31) / 32;
  const int cc = blockIdx.x % cchunks;
  const int64_t b = blockIdx.y;
  const int64_t l0 = (int64_t)(blockIdx.x / cchunks) * lchunk;
  const int64_t l1 = min(L, l0 + lchunk);
  const int c4 = cc * 32 + lane;
  const bool a = act[b] != 0.f;
  const float al = alpha[b], be = beta[b];
  float sa = 0.f, sb = 0.f;
  float4 sgv = make_float4(0.f, 0.f, 0.f, 0.f);
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
  if (c4 < d4) {
    for (int64_t l = l0 + grp; l < l1; l += 8) {
      const int64_t i = (b * L + l) * d4 + c4;
      const float4 gv = g[i];
      if (a) {
        const float4 u = xn[i], v = orig[i];
        sa += gv.x * u.x + gv.y * u.y + gv.z * u.z + gv.w * u.w;
        sb += gv.x * v.x + gv.y * v.y + gv.z * v.z + gv.w * v.w;
        sgv.x += gv.x; sgv.y += gv.y; sgv.z += gv.z; sgv.w += gv.w;
        dxn[i] = make_float4(al * gv.x, al * gv.y, al * gv.z, al * gv.w);
        dorig[i] = make_float4(be * gv.x, be * gv.y, be * gv.z, be * gv.w);
        dxold[i] = z4;
      } else {
        dxn[i] = z4;
        dorig[i] = z4;
        dxold[i] = gv;
      }
    }
  }
  if (!a) return;  // uniform per workgroup
  sg_s[grp][lane] = sgv;
  sa = wave_sum(sa);
  sb = wave_sum(sb);
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = sa;
    red[1][threadIdx.x >> 6] = sb;
  }
  __syncthreads();
  if (threadIdx.x < 128) {  // 32 float4 columns x 4 components
    const int cl = threadIdx.x >> 2, q = threadIdx.x & 3;
    const int c4b = cc * 32 + cl;
    if (c4b < d4) {
      float t = 0.f;
      for (int g2 = 0; g2 < 8; ++g2) {
        const float4 v = sg_s[g2][cl];
        t += q == 0 ? v.x : q == 1 ? v.y : q == 2 ? v.z : v.w;
      }
      atomicAdd(dgam + b * 4 * d4 + 4 * c4b + q, t);
    }
  } else if (threadIdx.x == 128) {
    atomicAdd(dalpha + b, red[0][0] + red[0][1] + red[0][2] + red[0][3]);
    atomicAdd(dbeta + b, red[1][0] + red[1][1] + red[1][2] + red[1][3]);
  }
}

// ---------------------------------------------------------------------------------------------
// Fused-backward variants (asrx/msheath.py MSheathFn): every gradient contribution to a layer's input
// x_i lands in ONE buffer -- written by the first producer, accumulated by the rest -- instead of
// separate tensors that autograd sums with extra add kernels.
//
// jump_select backward, accumulate form.  Active samples: dxn = alpha g; orig's gradient
// dorig (+)= beta g only when beta != 0 (a jump), the first jumping layer of a sample writing
// (has_orig[b] == 0, set afterwards by msheath_ctrl_bwd); x_i's gradient is left to
// axpy_row2_bwd_acc.  Inactive samples: dx = g (the pass-through), nothing else.
__global__ __launch_bounds__(256) void jump_select4_bwd_acc_kernel(
    const float4* __restrict__ g, const float4* __restrict__ xn, const float4* __restrict__ orig,
    const float* __restrict__ act, const float* __restrict__ alpha, const float* __restrict__ beta,
    const int* __restrict__ has_orig, float4* __restrict__ dxn, float4* __restrict__ dorig, float4* __restrict__ dx,
    float* __restrict__ dalpha, float* __restrict__ dbeta, float* __restrict__ dgam, int64_t L, int d4, int lchunk,
    float2* __restrict__ part_ab = nullptr, float* __restrict__ part_g = nullptr) {
  __shared__ float4 sg_s[8][32];
  __shared__ float red[2][4];
  const int lane = threadIdx.x & 31, grp = threadIdx.x >> 5;
  const int cchunks = (d4 + 31) / 32;
  const int cc = blockIdx.x % cchunks;
  const int lc = blockIdx.x / cchunks, nlc = gridDim.x / cchunks;
  const int64_t b = blockIdx.y;
  const int64_t l0 = (int64_t)lc * lchunk;
  const int64_t l1 = min(L, l0 + lchunk);
  const int c4 = cc * 32 + lane;
  const bool a = act[b] != 0.f;
  const float al = alpha[b], be = beta[b];
  const bool jo = be != 0.f, acc_o = has_orig[b] != 0;
  float sa = 0.f, sb = 0.f;
  float4 sgv = make_float4(0.f, 0.f, 0.f, 0.f);
  if (c4 < d4) {
    for (int64_t l = l0 + grp; l < l1; l += 8) {
      const int64_t i = (b * L + l) * d4 + c4;
      const float4 gv = g[i];
      if (a) {
        const float4 u = xn[i], v = orig[i];
        sa += gv.x * u.x + gv.y * u.y + gv.z * u.z + gv.w * u.w;
        sb += gv.x * v.x + gv.y * v.y + gv.z * v.z + gv.w * v.w;
        sgv.x += gv.x; sgv.y += gv.y; sgv.z += gv.z; sgv.w += gv.w;
        dxn[i] = make_float4(al * gv.x, al * gv.y, al * gv.z, al * gv.w);
        if (jo) {
          float4 o = make_float4(be * gv.x, be * gv.y, be * gv.z, be * gv.w);
          if (acc_o) {
            const float4 p = dorig[i];
            o.x += p.x; o.y += p.y; o.z += p.z; o.w += p.w;
          }
          dorig[i] = o;
        }
      } else {
        dx[i] = gv;
      }
    }
  }
  // partial mode writes every (sample, L chunk, column chunk) slot, zeros for an inactive sample
  if (!a && !part_g) return;  // uniform per workgroup
  sg_s[grp][lane] = sgv;
  sa = wave_sum(sa);
  sb = wave_sum(sb);
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = sa;
    red[1][threadIdx.x >> 6] = sb;
  }
  __syncthreads();
  if (threadIdx.x < 128) {
    const int cl = threadIdx.x >> 2, q = threadIdx.x & 3;
    const int c4b = cc * 32 + cl;
    if (c4b < d4) {
      float t = 0.f;
      for (int g2 = 0; g2 < 8; ++g2) {
        const float4 v = sg_s[g2][cl];
        t += q == 0 ? v.x : q == 1 ? v.y : q == 2 ? v.z : v.w;
      }
      if (part_g)
        part_g[(b * nlc + lc) * 4 * d4 + 4 * c4b + q] = t;
      else
        atomicAdd(dgam + b * 4 * d4 + 4 * c4b + q, t);
    }
  } else if (threadIdx.x == 128) {
    const float A = red[0][0] + red[0][1] + red[0][2] + red[0][3];
    const float Bv = red[1][0] + red[1][1] + red[1][2] + red[1][3];
    if (part_ab) {
      part_ab[(b * nlc + lc) * cchunks + cc] = make_float2(A, Bv);
    } else {
      atomicAdd(dalpha + b, A);
      atomicAdd(dbeta + b, Bv);
    }
  }
}

// x_new = x + s1 s2 y (model.py:461) and mem = mean_l x_new (model.py:463) backward, for active
// samples: g' = dxn + gm[b] / L (the seg-mean broadcast folded in), dy = s1 s2 g', ds1 = s2 g'.y,
// ds2 = s1 g'.y, and dx = g' -- the first contribution to x_i of an active sample.  Inactive
// samples: dy = 0, ds = 0, dx untouched (jump_select4_bwd_acc wrote the pass-through).
__global__ __launch_bounds__(256) void axpy_row2_bwd_acc_kernel(const float4* __restrict__ dxn,
                                                                const float* __restrict__ gm, float invL,
                                                                const float* __restrict__ act,
                                                                const float* __restrict__ s1, const float* __restrict__ s2,
                                                                const float4* __restrict__ y, float4* __restrict__ dy,
                                                                float* __restrict__ ds1, float* __restrict__ ds2,
                                                                float4* __restrict__ dx, int64_t rows, int64_t L, int d4) {
  const int lane = threadIdx.x & 63;
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); r < rows; r += (int64_t)gridDim.x * 4) {
    const int64_t b = r / L;
    if (act[b] == 0.f) {
      for (int j = lane; j < d4; j += 64) dy[r * d4 + j] = z4;
      if (lane == 0) {
        ds1[r] = 0.f;
        if (ds2) ds2[r] = 0.f;
      }
      continue;
    }
    const float a = s1[r], c = s2 ? s2[r] : 1.f;
    const float sc = a * c;
    const float4* gm4 = reinterpret_cast<const float4*>(gm + b * 4 * d4);
    float t = 0.f;
    for (int j = lane; j < d4; j += 64) {
      float4 gv = dxn[r * d4 + j];
      if (gm) {
        const float4 m = gm4[j];
        gv.x += m.x * invL; gv.y += m.y * invL; gv.z += m.z * invL; gv.w += m.w * invL;
      }
      const float4 yv = y[r * d4 + j];
      t += gv.x * yv.x + gv.y * yv.y + gv.z * yv.z + gv.w * yv.w;
      dy[r * d4 + j] = make_float4(sc * gv.x, sc * gv.y, sc * gv.z, sc * gv.w);
      dx[r * d4 + j] = gv;
    }
    t = wave_sum(t);
    if (lane == 0) {
      ds1[r] = c * t;
      if (ds2) ds2[r] = a * t;
    }
  }
}

// dx += (has_orig[b] ? dorig : 0) + u[b, :]   (orig's jump gradient and the pooled-mean broadcast of
// the MSheath input, model.py:432-435, 497)
__global__ void msheath_dx_final_kernel(float4* __restrict__ dx, const float4* __restrict__ dorig,
                                        const int* __restrict__ has_orig, const float4* __restrict__ u, int64_t B,
                                        int64_t L, int d4) {
  const int64_t total = B * L * d4;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = i / (L * d4);
    float4 v = dx[i];
    if (u) {
      const float4 w = u[b * d4 + i % d4];
      v.x += w.x; v.y += w.y; v.z += w.z; v.w += w.w;
    }
    if (has_orig[b]) {
      const float4 w = dorig[i];
      v.x += w.x; v.y += w.y; v.z += w.z; v.w += w.w;
    }
    dx[i] = v;
  }
}

}  // namespace asrx

using namespace asrx;


// the forward control kernel at its thread count for D (CT above)
template <typename... A>
static void ctrl_fwd_launch(int64_t D, int64_t B, hipStream_t stream, A... a) {
  if (D > 512) msheath_ctrl_fwd_kernel<512><<<(unsigned)B, 512, 0, stream>>>(a...);
  else msheath_ctrl_fwd_kernel<256><<<(unsigned)B, 256, 0, stream>>>(a...);
}

extern "C" {

int asrx_jump_select4_bwd_acc(const float* g, const float* xn, const float* orig, const float* act,
                              const float* alpha, const float* beta, const int* has_orig, float* dxn, float* dorig,
                              float* dx, float* dalpha, float* dbeta, float* dgam, int64_t B, int64_t L, int64_t d,
                              hipStream_t stream) {
  ASRX_REQUIRE(d % 4 == 0, "asrx_jump_select4_bwd_acc: d % 4 != 0");
  if (B * L == 0) return 0;
  if (dbeta == dalpha + B && dgam == dalpha + 2 * B) {  // one block [dalpha | dbeta | dgam]
    (void)hipMemsetAsync(dalpha, 0, B * (2 + d) * sizeof(float), stream);
  } else {
    (void)hipMemsetAsync(dalpha, 0, B * sizeof(float), stream);
    (void)hipMemsetAsync(dbeta, 0, B * sizeof(float), stream);
    (void)hipMemsetAsync(dgam, 0, B * d * sizeof(float), stream);
  }
  const int d4 = (int)(d / 4);
  const int lchunk = 128;
  dim3 grid((unsigned)(((d4 + 31) / 32) * ((L + lchunk - 1) / lchunk)), (unsigned)B);
  jump_select4_bwd_acc_kernel<<<grid, 256, 0, stream>>>((const float4*)g, (const float4*)xn, (const float4*)orig, act,
                                                        alpha, beta, has_orig, (float4*)dxn, (float4*)dorig,
                                                        (float4*)dx, dalpha, dbeta, dgam, L, d4, lchunk);
  ASRX_LAUNCHED("asrx_jump_select4_bwd_acc");
}

// Deterministic form of asrx_jump_select4_bwd_acc: the per-sample sums (dalpha, dbeta, dgam) leave as
// per-(L chunk, column chunk) partials in `part` (asrx_jump_bwd_part_floats floats, no memset needed),
// which asrx_msheath_ctrl_bwd4 adds in a fixed order -- no float atomics on the data gradient's path,
// so a backward is bit-reproducible run to run.
int64_t asrx_jump_bwd_part_floats(int64_t B, int64_t L, int64_t d) {
  const int64_t nlc = (L + 127) / 128, ncc = (d / 4 + 31) / 32;
  return B * nlc * (2 * ncc + d);
}

int asrx_jump_select4_bwd_part(const float* g, const float* xn, const float* orig, const float* act,
                               const float* alpha, const float* beta, const int* has_orig, float* dxn, float* dorig,
                               float* dx, float* part, int64_t B, int64_t L, int64_t d, hipStream_t stream) {
  ASRX_REQUIRE(d % 4 == 0, "asrx_jump_select4_bwd_part: d % 4 != 0");
  if (B * L == 0) return 0;
  const int d4 = (int)(d / 4);
  const int lchunk = 128;
  const int64_t nlc = (L + lchunk - 1) / lchunk, ncc = (d4 + 31) / 32;
  float2* part_ab = reinterpret_cast<float2*>(part);
  float* part_g = part + 2 * B * nlc * ncc;
  dim3 grid((unsigned)(ncc * nlc), (unsigned)B);
  jump_select4_bwd_acc_kernel<<<grid, 256, 0, stream>>>((const float4*)g, (const float4*)xn, (const float4*)orig, act,
                                                        alpha, beta, has_orig, (float4*)dxn, (float4*)dorig,
                                                        (float4*)dx, nullptr, nullptr, nullptr, L, d4, lchunk,
                                                        part_ab, part_g);
  ASRX_LAUNCHED("asrx_jump_select4_bwd_part");
}

int asrx_axpy_row2_bwd_acc(const float* dxn, const float* gm, float invL, const float* act, const float* s1,
                           const float* s2, const float* y, float* dy, float* ds1, float* ds2, float* dx, int64_t B,
                           int64_t L, int64_t d, hipStream_t stream) {
  ASRX_REQUIRE(d % 4 == 0, "asrx_axpy_row2_bwd_acc: d % 4 != 0");
  const int64_t rows = B * L;
  if (rows == 0) return 0;
  axpy_row2_bwd_acc_kernel<<<(unsigned)std::min<int64_t>((rows + 3) / 4, 8192), 256, 0, stream>>>(
      (const float4*)dxn, gm, invL, act, s1, s2, (const float4*)y, (float4*)dy, ds1, ds2, (float4*)dx, rows, L,
      (int)(d / 4));
  ASRX_LAUNCHED("asrx_axpy_row2_bwd_acc");
}

int asrx_msheath_dx_final(float* dx, const float* dorig, const int* has_orig, const float* u, int64_t B, int64_t L,
                          int64_t d, hipStream_t stream) {
  ASRX_REQUIRE(d % 4 == 0, "asrx_msheath_dx_final: d % 4 != 0");
  if (B * L == 0) return 0;
  const int64_t n = B * L * d / 4;
  msheath_dx_final_kernel<<<(unsigned)std::min<int64_t>((n + 255) / 256, 16384), 256, 0, stream>>>(
      (float4*)dx, (const float4*)dorig, has_orig, (const float4*)u, B, L, (int)(d / 4));
  ASRX_LAUNCHED("asrx_msheath_dx_final");
}

int asrx_msheath_ctrl_fwd(const float* policy, const float* gpol, int64_t ld_gpol, const float* ion,
                          const float* mem_v, const float* mem_w, const float* mem, const float* jump_s,
                          const float* next_i, int64_t layer_i, int64_t layers, int64_t B, int64_t L, int64_t D,
                          float* alpha, float* beta, float* gam, float* mem_w_out, float* active, float* next_out,
                          void* rec, hipStream_t stream) {
  if (B == 0) return 0;
  ctrl_fwd_launch(D, B, stream, policy, gpol, ld_gpol, ion, mem_v, mem_w, mem, jump_s,
                                                           next_i, (int)layer_i, (int)layers, L, (int)D, alpha, beta,
                                                           gam, mem_w_out, active, next_out, (CtrlRec*)rec, D, nullptr,
                                                           nullptr, nullptr, nullptr, 0, nullptr);
  ASRX_LAUNCHED("asrx_msheath_ctrl_fwd");
}

// As asrx_msheath_ctrl_fwd with mem_w's row stride (0 = the parameter broadcast over samples) and a
// nullable next_i (all samples at layer 0).
int asrx_msheath_ctrl_fwd2(const float* policy, const float* gpol, int64_t ld_gpol, const float* ion,
                           const float* mem_v, const float* mem_w, int64_t ld_mem_w, const float* mem,
                           const float* jump_s, const float* next_i, int64_t layer_i, int64_t layers, int64_t B,
                           int64_t L, int64_t D, float* alpha, float* beta, float* gam, float* mem_w_out, float* active,
                           float* next_out, void* rec, hipStream_t stream) {
  if (B == 0) return 0;
  ctrl_fwd_launch(D, B, stream, policy, gpol, ld_gpol, ion, mem_v, mem_w, mem, jump_s,
                                                           next_i, (int)layer_i, (int)layers, L, (int)D, alpha, beta,
                                                           gam, mem_w_out, active, next_out, (CtrlRec*)rec, ld_mem_w,
                                                           nullptr, nullptr, nullptr, nullptr, 0, nullptr);
  ASRX_LAUNCHED("asrx_msheath_ctrl_fwd2");
}

// As asrx_msheath_ctrl_fwd2 with mem = (1/L) sum of the asrx_axpy_row2_colsum chunk partials
// (written to mem) and mem_v = sigmoid(mem . mg_w + mg_b) computed in the kernel (written to
// mem_v_out for the backward).
int asrx_msheath_ctrl_fwd3(const float* policy, const float* gpol, int64_t ld_gpol, const float* ion,
                           const float* mg_w, const float* mg_b, float* mem_v_out, const float* mem_w,
                           int64_t ld_mem_w, const float* mem_part, float* mem, const float* jump_s,
                           const float* next_i, int64_t layer_i, int64_t layers, int64_t B, int64_t L, int64_t D,
                           float* alpha, float* beta, float* gam, float* mem_w_out, float* active, float* next_out,
                           void* rec, hipStream_t stream) {
  if (B == 0) return 0;
  const int nchunk = (int)((L + MEM_CHUNK - 1) / MEM_CHUNK);
  ctrl_fwd_launch(D, B, stream, policy, gpol, ld_gpol, ion, nullptr, mem_w, mem, jump_s,
                                                           next_i, (int)layer_i, (int)layers, L, (int)D, alpha, beta,
                                                           gam, mem_w_out, active, next_out, (CtrlRec*)rec, ld_mem_w,
                                                           mg_w, mg_b, mem_v_out, mem_part, nchunk, mem);
  ASRX_LAUNCHED("asrx_msheath_ctrl_fwd3");
}

int asrx_msheath_ctrl_bwd(const float* g_alpha, const float* g_beta, const float* g_gam, const float* g_mwo,
                          const float* mem_v, const float* mem_w, const float* mem, const float* jump_s,
                          const void* rec, int64_t layer_i, int64_t layers, int64_t B, int64_t D, float* g_policy,
                          float* g_mem_v, float* g_mem_w, float* g_mem, float* g_jump_s, hipStream_t stream) {
  if (B == 0) return 0;
  msheath_ctrl_bwd_kernel<<<(unsigned)B, 256, 0, stream>>>(g_alpha, g_beta, g_gam, g_mwo, mem_v, mem_w, mem, jump_s,
                                                           (const CtrlRec*)rec, (int)layer_i, (int)layers, (int)D,
                                                           g_policy, g_mem_v, g_mem_w, g_mem, g_jump_s, D, nullptr, 0,
                                                           nullptr, nullptr, nullptr);
  ASRX_LAUNCHED("asrx_msheath_ctrl_bwd");
}

// As asrx_msheath_ctrl_bwd with mem_w's row stride, g_policy accumulated when acc_policy != 0, and
// has_orig[b] set when this layer's jump wrote orig's gradient (see jump_select4_bwd_acc).
int asrx_msheath_ctrl_bwd2(const float* g_alpha, const float* g_beta, const float* g_gam, const float* g_mwo,
                           const float* mem_v, const float* mem_w, int64_t ld_mem_w, const float* mem,
                           const float* jump_s, const void* rec, int64_t layer_i, int64_t layers, int64_t B, int64_t D,
                           float* g_policy, int acc_policy, float* g_mem_v, float* g_mem_w, float* g_mem,
                           float* g_jump_s, int* has_orig, hipStream_t stream) {
  if (B == 0) return 0;
  msheath_ctrl_bwd_kernel<<<(unsigned)B, 256, 0, stream>>>(g_alpha, g_beta, g_gam, g_mwo, mem_v, mem_w, mem, jump_s,
                                                           (const CtrlRec*)rec, (int)layer_i, (int)layers, (int)D,
                                                           g_policy, g_mem_v, g_mem_w, g_mem, g_jump_s, ld_mem_w,
                                                           has_orig, acc_policy, nullptr, nullptr, nullptr);
  ASRX_LAUNCHED("asrx_msheath_ctrl_bwd2");
}

// As asrx_msheath_ctrl_bwd2 with mem_v's gate backward fused: g_mem also receives
// g_mem_v mv (1 - mv) mg_w, and g_mg_w / g_mg_b accumulate its parameter gradients (atomics).
int asrx_msheath_ctrl_bwd3(const float* g_alpha, const float* g_beta, const float* g_gam, const float* g_mwo,
                           const float* mem_v, const float* mem_w, int64_t ld_mem_w, const float* mem,
                           const float* jump_s, const void* rec, int64_t layer_i, int64_t layers, int64_t B, int64_t D,
                           float* g_policy, int acc_policy, float* g_mem_w, float* g_mem, float* g_jump_s,
                           int* has_orig, const float* mg_w, float* g_mg_w, float* g_mg_b, hipStream_t stream) {
  if (B == 0) return 0;
  msheath_ctrl_bwd_kernel<<<(unsigned)B, 256, 0, stream>>>(g_alpha, g_beta, g_gam, g_mwo, mem_v, mem_w, mem, jump_s,
                                                           (const CtrlRec*)rec, (int)layer_i, (int)layers, (int)D,
                                                           g_policy, nullptr, g_mem_w, g_mem, g_jump_s, ld_mem_w,
                                                           has_orig, acc_policy, mg_w, g_mg_w, g_mg_b);
  ASRX_LAUNCHED("asrx_msheath_ctrl_bwd3");
}

// asrx_msheath_ctrl_bwd3 reading (dalpha, dbeta, dgam) as the partials of asrx_jump_select4_bwd_part
// (same B, L, D), summed in chunk order.
int asrx_msheath_ctrl_bwd4(const float* part, int64_t L, const float* g_mwo, const float* mem_v, const float* mem_w,
                           int64_t ld_mem_w, const float* mem, const float* jump_s, const void* rec, int64_t layer_i,
                           int64_t layers, int64_t B, int64_t D, float* g_policy, int acc_policy, float* g_mem_w,
                           float* g_mem, float* g_jump_s, int* has_orig, const float* mg_w, float* g_mg_w,
                           float* g_mg_b, hipStream_t stream) {
  ASRX_REQUIRE(D % 4 == 0, "asrx_msheath_ctrl_bwd4: D % 4 != 0");
  if (B == 0) return 0;
  const int64_t nlc = (L + 127) / 128, ncc = (D / 4 + 31) / 32;
  const float2* part_ab = reinterpret_cast<const float2*>(part);
  const float* part_g = part + 2 * B * nlc * ncc;
  msheath_ctrl_bwd_kernel<<<(unsigned)B, 256, 0, stream>>>(nullptr, nullptr, nullptr, g_mwo, mem_v, mem_w, mem,
                                                           jump_s, (const CtrlRec*)rec, (int)layer_i, (int)layers,
                                                           (int)D, g_policy, nullptr, g_mem_w, g_mem, g_jump_s,
                                                           ld_mem_w, has_orig, acc_policy, mg_w, g_mg_w, g_mg_b,
                                                           part_ab, part_g, (int)nlc, (int)ncc);
  ASRX_LAUNCHED("asrx_msheath_ctrl_bwd4");
}

int64_t asrx_mem_chunks(int64_t L) { return (L + MEM_CHUNK - 1) / MEM_CHUNK; }

int asrx_axpy_row2_colsum(const float* x, const float* s1, const float* s2, const float* y, float* out, float* part,
                          int64_t B, int64_t L, int64_t d, const float* next_i, int64_t layer, hipStream_t stream) {
  ASRX_REQUIRE(d % 4 == 0 && d <= 1024, "asrx_axpy_row2_colsum: d %% 4 == 0 and d <= 1024 required");
  ASRX_REQUIRE(s2 != nullptr, "asrx_axpy_row2_colsum: s2 required");
  if (B * L == 0) return 0;
  const int d4 = (int)(d / 4);
  dim3 grid((unsigned)B, (unsigned)asrx_mem_chunks(L));
  axpy_row2_colsum_kernel<<<grid, 256, 0, stream>>>((const float4*)x, s1, s2, (const float4*)y, (float4*)out,
                                                    (float4*)part, L, d4, next_i, (int)layer);
  ASRX_LAUNCHED("asrx_axpy_row2_colsum");
}

int64_t asrx_msheath_rec_bytes(void) { return (int64_t)sizeof(CtrlRec); }

int asrx_axpy_row2(const float* x, const float* s1, const float* s2, const float* y, float* out, int64_t rows,
                   int64_t d, hipStream_t stream) {
  ASRX_REQUIRE(d % 4 == 0, "asrx_axpy_row2: d % 4 != 0");
  if (rows == 0) return 0;
  const int64_t n = rows * d / 4;
  axpy_row2_kernel<<<(unsigned)std::min<int64_t>((n + 255) / 256, 16384), 256, 0, stream>>>(
      (const float4*)x, s1, s2, (const float4*)y, (float4*)out, rows, (int)(d / 4));
  ASRX_LAUNCHED("asrx_axpy_row2");
}

int asrx_axpy_row2_bwd(const float* g, const float* s1, const float* s2, const float* y, float* dy, float* ds1,
                       float* ds2, int64_t rows, int64_t d, hipStream_t stream) {
  ASRX_REQUIRE(d % 4 == 0, "asrx_axpy_row2_bwd: d % 4 != 0");
  if (rows == 0) return 0;
  axpy_row2_bwd_kernel<<<(unsigned)std::min<int64_t>((rows + 3) / 4, 8192), 256, 0, stream>>>(
      (const float4*)g, s1, s2, (const float4*)y, (float4*)dy, ds1, ds2, rows, (int)(d / 4));
  ASRX_LAUNCHED("asrx_axpy_row2_bwd");
}

int asrx_jump_axpy_inplace(const float* xin, float* xout, const float* s1, const float* s2, const float* y,
                           const float* orig, const float* act, const float* alpha, const float* beta, const float* gam,
                           int64_t B, int64_t L, int64_t d, hipStream_t stream) {
  ASRX_REQUIRE(d % 4 == 0, "asrx_jump_axpy_inplace: d % 4 != 0");
  ASRX_REQUIRE(xout != orig, "asrx_jump_axpy_inplace: xout must not alias orig");
  if (B * L == 0) return 0;
  ASRX_REQUIRE(d / 4 <= 256, "asrx_jump_axpy_inplace: d <= 1024 required");
  // flat grid-stride (measured faster than 64- or 16-row chunk grids: profiles/r04_jump_ab.txt)
  dim3 grid((unsigned)std::min<int64_t>((L * (d / 4) + 255) / 256, 512), (unsigned)B);
  jump_axpy_inplace_kernel<<<grid, 256, 0, stream>>>((const float4*)xin, (float4*)xout, s1, s2, (const float4*)y,
                                                     (const float4*)orig, act, alpha, beta, (const float4*)gam, L,
                                                     (int)(d / 4));
  ASRX_LAUNCHED("asrx_jump_axpy_inplace");
}

int asrx_jump_select4(const float* xn, const float* orig, const float* xold, const float* act, const float* alpha,
                      const float* beta, const float* gam, float* out, int64_t B, int64_t L, int64_t d,
                      hipStream_t stream) {
  ASRX_REQUIRE(d % 4 == 0 && d <= 1024, "asrx_jump_select4: d % 4 != 0 or d > 1024");
  if (B * L == 0) return 0;
  // flat grid-stride (measured faster than 64- or 16-row chunk grids: profiles/r04_jump_ab.txt)
  dim3 grid((unsigned)std::min<int64_t>((L * (d / 4) + 255) / 256, 512), (unsigned)B);
  jump_select4_kernel<<<grid, 256, 0, stream>>>((const float4*)xn, (const float4*)orig, (const float4*)xold, act,
                                                alpha, beta, (const float4*)gam, (float4*)out, L, (int)(d / 4));
  ASRX_LAUNCHED("asrx_jump_select4");
}

int asrx_jump_select4_bwd(const float* g, const float* xn, const float* orig, const float* act, const float* alpha,
                          const float* beta, float* dxn, float* dorig, float* dxold, float* dalpha, float* dbeta,
                          float* dgam, int64_t B, int64_t L, int64_t d, hipStream_t stream) {
  ASRX_REQUIRE(d % 4 == 0, "asrx_jump_select4_bwd: d % 4 != 0");
  if (B * L == 0) return 0;
  (void)hipMemsetAsync(dalpha, 0, B * sizeof(float), stream);
  (void)hipMemsetAsync(dbeta, 0, B * sizeof(float), stream);
  (void)hipMemsetAsync(dgam, 0, B * d * sizeof(float), stream);
  const int d4 = (int)(d / 4);
  const int lchunk = 128;
  dim3 grid((unsigned)(((d4 + 31) / 32) * ((L + lchunk - 1) / lchunk)), (unsigned)B);
  jump_select4_bwd_kernel<<<grid, 256, 0, stream>>>((const float4*)g, (const float4*)xn, (const float4*)orig, act,
                                                    alpha, beta, (float4*)dxn, (float4*)dorig, (float4*)dxold, dalpha,
                                                    dbeta, dgam, L, d4, lchunk);
  ASRX_LAUNCHED("asrx_jump_select4_bwd");
}

}  // extern "C"
