// Shared helpers for the ssq HIP kernels (gfx950 / CDNA4).
//
// Numerics contract (see DESIGN.md "bit-exactness"): every kernel reproduces the
// reference's fp32 operation order with IEEE division (hipcc default: correctly
// rounded fp32 divide), round-half-even (rintf), and no FMA contraction
// (-ffp-contract=off on the build line, plus explicit __fmul_rn/__fadd_rn where the
// reference does separate tensor ops).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>

#include "../../include/ssq.h"

namespace ssq {

typedef float f32x4 __attribute__((ext_vector_type(4)));  // native 16-B vector

constexpr int kWave = 64;          // CDNA wavefront
constexpr int kBlock = 256;        // 4 waves per workgroup
constexpr float kGamma = -0.1f;    // channelQuant.py:35 (gamma, zeta) = (-0.1, 1.1)
constexpr float kZmG = 1.2f;       // fp32((1.1) - (-0.1)) = fp32(1.2000000000000002)

// ---------------------------------------------------------------- error plumbing
void set_error(const char* fmt, ...);
int check_launch(const char* what);

#define SSQ_REQUIRE(cond, code, ...)         \
  do {                                       \
    if (!(cond)) {                           \
      ::ssq::set_error(__VA_ARGS__);         \
      return (code);                         \
    }                                        \
  } while (0)

inline int grid_for(int64_t work_items, int block, int max_blocks = 4096) {
  int64_t g = (work_items + block - 1) / block;
  if (g < 1) g = 1;
  if (g > max_blocks) g = max_blocks;
  return (int)g;
}

// Streaming loads/stores: NT=true uses the non-temporal (streaming) cache policy.
template <bool NT>
__device__ __forceinline__ f32x4 ld4(const f32x4* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}
template <bool NT>
__device__ __forceinline__ void st4(f32x4 v, f32x4* p) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

// n / d for 0 <= n < 2^31 as (umulhi(n, m) + n) >> s (round-up magic number, exact;
// d >= 1).  Replaces 32/64-bit integer divides in per-element index math.
struct FastDiv {
  uint32_t m, s;
};
inline FastDiv make_fastdiv(uint32_t d) {
  uint32_t s = 0;
  while (s < 32 && (1ull << s) < d) ++s;
  const uint64_t m = ((1ull << 32) * ((1ull << s) - d)) / d + 1;
  return FastDiv{(uint32_t)m, s};
}
__device__ __forceinline__ uint32_t fdiv(uint32_t n, FastDiv f) {
  return (__umulhi(n, f.m) + n) >> f.s;
}

// ---------------------------------------------------------------- activations
// Activation codes of the fused epilogues (ABI int `relu`): 0 none, 1 ReLU, 2 ReLU6.
// Forward as torch's clamp (t < lo -> lo keeps -0.0 and NaN); the gradient passes unless
// the activation's output sits on / beyond a clamp edge -- threshold_backward (out <= 0)
// for ReLU, hardtanh_backward (x <= 0 || x >= 6, NaN passes) for ReLU6, evaluated on the
// output, which equals the input strictly inside the edges.
template <int ACT>
__device__ __forceinline__ float act_fwd(float t) {
  if (ACT >= 1) t = t < 0.0f ? 0.0f : t;
  if (ACT == 2) t = t > 6.0f ? 6.0f : t;
  return t;
}
template <int ACT>
__device__ __forceinline__ bool act_pass(float o) {
  if (ACT == 1) return !(o <= 0.0f);
  if (ACT == 2) return !(o <= 0.0f || o >= 6.0f);
  return true;
}

// ---------------------------------------------------------------- device math
// Division by a loop-invariant d without the per-element divide sequence.  With
// r = RN(1/d) (computed once), q0 = x*r is within 1.5 ulp of x/d, one fma residual /
// correction makes it faithful, and a second one returns RN(x/d) -- Markstein's theorem
// (r within 1/2 ulp of 1/d, q1 faithful => RN(q1 + RN(x - d*q1)*r) = RN(x/d)), the same
// correction the compiler's IEEE divide ends with.  The premise needs every residual
// normal: |d| and nonzero |x| in [2^-60, 2^60].  recip_for_div returns 0 for a d outside
// that range and div_fast_ok tests x; callers take the IEEE divide when either fails.
// x = +-0 returns x*r, the correctly signed zero.  Validated against the IEEE divide on
// 3.4e9 random pairs (tools/divcheck.c) in addition to the boundary tests.
__device__ __forceinline__ float recip_for_div(float d) {
  const float a = fabsf(d);
  return (a >= 0x1p-60f && a <= 0x1p60f) ? 1.0f / d : 0.0f;
}
__device__ __forceinline__ bool div_fast_ok(float x) {
  const uint32_t b = __float_as_uint(x) & 0x7fffffffu;
  return b == 0u || (b - 0x21800000u) <= (0x5d800000u - 0x21800000u);
}
__device__ __forceinline__ float div_fast(float x, float d, float r) {
  const float q0 = __fmul_rn(x, r);
  const float q1 = __fmaf_rn(__fmaf_rn(-q0, d, x), r, q0);
  const float q2 = __fmaf_rn(__fmaf_rn(-q1, d, x), r, q1);
  return x == 0.0f ? q0 : q2;
}

__device__ __forceinline__ float clampf(float v, float lo, float hi) {
  // torch.clamp: min(max(v, lo), hi) with a NaN input kept NaN (fminf / fmaxf would
  // return the bound): IEEE 754-2019 maximum / minimum, v_maximum3_f32 / v_minimum3_f32
  // on gfx950 -- two instructions, as many as the bound-returning form
  return __builtin_elementwise_minimum(__builtin_elementwise_maximum(v, lo), hi);
}

// torch.sigmoid in fp32 (1 / (1 + exp(-x))).
__device__ __forceinline__ float sigmoidf(float x) { return 1.0f / (1.0f + expf(-x)); }

// rectified sigmoid h(v) = clamp(sigmoid(v)*(zeta-gamma) + gamma, 0, 1)
// (channelQuant.py:123-127, adaptive_rounding.py:63-64)
__device__ __forceinline__ float rect_sigmoid(float v) {
  return clampf(__fadd_rn(__fmul_rn(sigmoidf(v), kZmG), kGamma), 0.0f, 1.0f);
}

// d h / d v  (clamp mask inclusive) * upstream
// The reference's autograd order: clamp backward (0 outside, NaN u -> 0), * (zeta-gamma),
// sigmoid backward g*(1-s)*s -- so a NaN v gives NaN even under a zero upstream, and an
// outside-the-clamp finite v gives +0 as before.
__device__ __forceinline__ float rect_sigmoid_grad(float v, float g) {
  float s = sigmoidf(v);
  float u = __fadd_rn(__fmul_rn(s, kZmG), kGamma);
  const float gu = (u >= 0.0f && u <= 1.0f) ? g : 0.0f;
  return __fmul_rn(__fmul_rn(__fmul_rn(gu, kZmG), __fsub_rn(1.0f, s)), s);
}

// p = clamp(softmax(a)*(zeta-gamma)+gamma, 0, 1) over S logits (channelQuant.py:120-121)
template <int MAXS>
__device__ __forceinline__ void soft_targets(const float* a, int S, float* s_out, float* p_out) {
  float m = a[0];
  for (int i = 1; i < S; ++i) m = fmaxf(m, a[i]);
  float e[MAXS];
  float sum = 0.0f;
  for (int i = 0; i < S; ++i) {
    e[i] = expf(__fsub_rn(a[i], m));
    sum = __fadd_rn(sum, e[i]);
  }
  for (int i = 0; i < S; ++i) {
    float s = e[i] / sum;
    if (s_out) s_out[i] = s;
    p_out[i] = clampf(__fadd_rn(__fmul_rn(s, kZmG), kGamma), 0.0f, 1.0f);
  }
}

// first index of the maximum (torch.argmax tie rule)
__device__ __forceinline__ int argmax_first(const float* p, int S) {
  int best = 0;
  for (int i = 1; i < S; ++i)
    if (p[i] > p[best]) best = i;
  return best;
}

// ---------------------------------------------------------------- wave / block reductions
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}
__device__ __forceinline__ float wave_min(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o, kWave));
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, kWave));
  return v;
}

// Deterministic block sum of one double per thread (blockDim multiple of 64, <= 1024).
__device__ __forceinline__ double block_sum(double v, double* lds /* >= 16 */) {
  v = wave_sum(v);
  const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
  __syncthreads();
  if (lane == 0) lds[w] = v;
  __syncthreads();
  double t = 0.0;
  const int nw = blockDim.x / kWave;
  if (threadIdx.x == 0) {
    for (int i = 0; i < nw; ++i) t += lds[i];
    lds[0] = t;
  }
  __syncthreads();
  return lds[0];
}

// ---------------------------------------------------------------- last-arriver hand-off
// One launch instead of a partials kernel + a 1-workgroup finalize kernel
// (cdna_hip_programming.md Guideline 16, counter form with write-through partials): every
// workgroup stores its partials write-through (sc1, agent scope: no release fence), drains
// them (every wave s_waitcnt vmcnt(0), then the barrier), and one lane takes a ticket
// (relaxed agent-scope fetch_add on a per-reduction counter); the workgroup that draws
// the last ticket reads every partial with sc1 loads (each of them: no acquire fence
// needed) in a fixed order -- deterministic -- and resets the counter for the next
// launch.  The one counter (fin_epi's act-delta reduction) is a word of the calling launch's
// own workspace, zeroed by the launch that writes the partials it counts, so two launches in
// flight with different workspaces -- e.g. on two streams -- never share one; no counter is a
// device global.
typedef __attribute__((address_space(1))) unsigned long long gu64_t;
typedef __attribute__((address_space(1))) unsigned int gu32_t;

__device__ __forceinline__ void st_sc1(double* p, double v) {
  __hip_atomic_store((gu64_t*)p, (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_sc1(const double* p) {
  return __longlong_as_double(
      (long long)__hip_atomic_load((gu64_t*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
// Every thread of the workgroup calls it after its partial stores; true in every thread of
// the last-arriving workgroup of `nblocks` sharing `ticket`.  `flag`: one LDS word.
__device__ __forceinline__ bool arrive_last(unsigned* ticket, unsigned nblocks, int* flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned t = __hip_atomic_fetch_add((gu32_t*)ticket, 1u, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
    *flag = t == nblocks - 1;
  }
  __syncthreads();
  const bool last = *flag != 0;
  if (last && threadIdx.x == 0)
    __hip_atomic_store((gu32_t*)ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // keep the sc1 loads below
  return last;
}

// round_ste's forward (quant_layer.py:18-22) plus the zero point: ((round(t) - t) + t) + zp.
// (round(t) - t) + t is round(t) for every finite t (round(t) - t is a multiple of ulp(t)
// no larger than 1/2: both operations are exact) and NaN at t = +-inf, where torch.round
// alone returns +-inf.  Evaluated as v = round(t) + zp, then fma(v, 0, v): v for every
// finite v (the product is a signed zero), NaN for an infinite one -- one instruction.
// Only the sign of a zero v can differ from the reference's order, and (q - zp) * delta
// maps both signs to the same dequantized value.
__device__ __forceinline__ float round_ste_zp(float t, float z) {
  const float v = __fadd_rn(rintf(t), z);
  return __fmaf_rn(v, 0.0f, v);
}

// one element of the uniform affine fake-quant (quant_layer.py:92-98).  STE: the
// UniformAffineQuantizer's round_ste; !STE: plain torch.round (ChannelQuant 'none',
// ChannelQuantAct 'none', AdaRound 'nearest'): the two differ only where x / delta is
// +-inf (NaN vs a clamped edge).
struct QParams {
  float d, z, lo, hi;
};

template <bool FAST = false, bool STE = true>
__device__ __forceinline__ float fq1(float x, const QParams& p, float* qout, float r = 0.0f) {
  // x / delta: IEEE fp32 divide, or its bit-identical reciprocal form (div_fast)
  float t = FAST ? div_fast(x, p.d, r) : x / p.d;
  const float v = STE ? round_ste_zp(t, p.z) : __fadd_rn(rintf(t), p.z);  // + zp
  float q = clampf(v, p.lo, p.hi);         // clamp(x_int, lo, hi): NaN stays NaN
  *qout = q;
  return __fmul_rn(__fsub_rn(q, p.z), p.d);  // (x_quant - zp) * delta
}

// ---------------------------------------------------------------- loss / regulariser terms
// (lp_loss_kernel and the fused tail in recon.hip, the fused fc iteration in fc_recon.hip)
// |d|^p and its derivative p*|d|^(p-1) for one element.
template <int PMODE>  // 0: p == 2, 1: p == 1, 2: general p
__device__ __forceinline__ void lp_term(float a, float p, float& pw, float& dp) {
  if (PMODE == 0) {
    pw = __fmul_rn(a, a);
    dp = __fmul_rn(2.0f, a);
  } else if (PMODE == 1) {
    pw = a;
    dp = 1.0f;
  } else {
    // both powers from one hardware log2 and two hardware exp2 (about 1e-6 relative; the
    // loss and gradient tolerance is 1e-5).  No divide and no ocml powf: those made this
    // pass VALU-bound.  a == 0: log2 = -inf gives pow's own values (0 for p > 1; inf for
    // p - 1 < 0, so the gradient is inf * sgn(0) = NaN, as torch's)
    const float l = __builtin_amdgcn_logf(a);
    pw = __builtin_amdgcn_exp2f(__fmul_rn(p, l));
    dp = __fmul_rn(p, __builtin_amdgcn_exp2f(__fmul_rn(__fsub_rn(p, 1.0f), l)));
  }
}

template <int PMODE>
__device__ __forceinline__ float lp_elem(float x, float t, float p, float inv_m, float gs,
                                         int relu_mask, double& acc) {
  const float d = __fsub_rn(x, t);
  float pw, dp;
  lp_term<PMODE>(fabsf(d), p, pw, dp);
  acc += (double)pw;
  const float sg = d > 0.0f ? 1.0f : (d < 0.0f ? -1.0f : 0.0f);
  const float gv = __fmul_rn(__fmul_rn(__fmul_rn(inv_m, dp), sg), gs);
  // relu_mask: pred is a ReLU output; the gradient is written at the ReLU's input
  // (torch threshold_backward: out <= 0 -> 0)
  return (relu_mask && x <= 0.0f) ? 0.0f : gv;
}

// d/dv of the rounding regulariser lambda*(1-|2h(v)-1|^b) (round_reg_kernel's gradient)
__device__ __forceinline__ float round_reg_grad(float v, float lambda, float b) {
  if (lambda == 0.0f || b == 0.0f) return 0.0f;
  const float h = rect_sigmoid(v);
  const float r = __fmul_rn(fabsf(__fsub_rn(h, 0.5f)), 2.0f);
  const float sg = h > 0.5f ? 1.0f : (h < 0.5f ? -1.0f : 0.0f);
  const float gh = -lambda * b * powf(r, b - 1.0f) * 2.0f * sg;
  return rect_sigmoid_grad(v, gh);
}

}  // namespace ssq
