// K5-K9, K12: ChannelQuant / AdaRound kernels.
//
// A weight is viewed as (Co, Ci, K), K = kh*kw (1 for Linear).  Shift-candidate floors
// F_i = floor(W / (delta[co]*s_i)) are recomputed from W in every kernel instead of being
// materialized as S W-sized tensors (the reference's self.x_q list, channelQuant.py:284-286),
// so the adaShift forward reads W + beta (8 B/elem) and writes What (4 B/elem).
//
// Conv kernels are column-tiled (see "column-tiled conv kernels"): the softmax of an
// input channel's alpha row is computed once per thread, rows are coalesced sweeps, and
// the alpha-gradient reductions over (Co, K) are two fixed-order stages (deterministic).
#include "adashift_common.h"

namespace ssq {

// ------------------------------------------------------------------ adaShift forward
__global__ __launch_bounds__(kBlock) void adashift_fwd_kernel(
    const float* __restrict__ W, const float* __restrict__ alpha, const float* __restrict__ beta,
    const float* __restrict__ delta, const float* __restrict__ zp, Shifts sh, Geo g, uint32_t n,
    int hard_t, int hard_r, float lo, float hi, float* __restrict__ What,
    uint8_t* __restrict__ codes) {
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t e = blockIdx.x * blockDim.x + threadIdx.x; e < n; e += stride) {
    uint32_t co, ci;
    decompose(e, g, co, ci);
    float a[kMaxS], p[kMaxS], F[kMaxS];
    load_row(alpha, alpha_row(g, co, ci), sh.n, a);
    soft_targets<kMaxS>(a, sh.n, nullptr, p);
    const float d = delta[co], z = zp[co], w = W[e];
    float xf;
    if (hard_t) {
      const int sel = argmax_first(p, sh.n);
      xf = floorf(w / __fmul_rn(d, sh.s[sel]));
    } else {
      xf = soft_floor(w, d, sh, sh.n, p, F);
    }
    const float b = beta[e];
    const float hr = hard_r ? (b >= 0.0f ? 1.0f : 0.0f) : rect_sigmoid(b);
    const float q = clampf(__fadd_rn(__fadd_rn(xf, hr), z), lo, hi);
    What[e] = __fmul_rn(__fsub_rn(q, z), __fmul_rn(d, 1.0f));
    if (codes) codes[e] = (uint8_t)((int)q & 0xff);
  }
}

// ------------------------------------------------------------------ adaShift backward
// MODE 0: adaShift (floors), MODE 1: learned_hard_sigmoid (dequantized 'none' candidates)
template <int MODE>
__device__ __forceinline__ float cand_value(float w, float d, float z, float s, float lo, float hi) {
  if (MODE == 0) return floorf(w / __fmul_rn(d, s));
  const float ds = __fmul_rn(d, s);
  const float q = clampf(__fadd_rn(rintf(w / ds), z), lo, hi);
  return __fmul_rn(__fsub_rn(q, z), ds);
}

// Linear: alpha is per element, no reduction.
template <int MODE>
__global__ __launch_bounds__(kBlock) void alpha_grad_fc(
    const float* __restrict__ gWhat, const float* __restrict__ W, const float* __restrict__ alpha,
    const float* __restrict__ beta, const float* __restrict__ delta, const float* __restrict__ zp,
    Shifts sh, Geo g, uint32_t n, int hard_r, float lo, float hi, float reg_lambda, float reg_b,
    const float* __restrict__ reg_dev, float* __restrict__ galpha, float* __restrict__ gbeta,
    float* __restrict__ reg_vals) {
  if (reg_dev) {
    reg_lambda = reg_dev[0];
    reg_b = reg_dev[1];
  }
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t e = blockIdx.x * blockDim.x + threadIdx.x; e < n; e += stride) {
    const uint32_t co = e / g.CiK;
    float a[kMaxS], p[kMaxS], F[kMaxS], ga[kMaxS];
    load_row(alpha, e, sh.n, a);
    soft_targets<kMaxS>(a, sh.n, nullptr, p);
    const float w = W[e], d = delta[co], z = zp[co], gy = gWhat[e];
    float gi;
    if (MODE == 0) {
      const float xf = soft_floor(w, d, sh, sh.n, p, F);
      const float b = beta[e];
      const float hr = hard_r ? (b >= 0.0f ? 1.0f : 0.0f) : rect_sigmoid(b);
      const float u = __fadd_rn(__fadd_rn(xf, hr), z);
      gi = (u >= lo && u <= hi) ? __fmul_rn(gy, __fmul_rn(d, 1.0f)) : 0.0f;
      if (gbeta) gbeta[e] = hard_r ? 0.0f : rect_sigmoid_grad(b, gi);
    } else {
      for (int i = 0; i < sh.n; ++i) F[i] = cand_value<1>(w, d, z, sh.s[i], lo, hi);
      gi = gy;
    }
    double gp[kMaxS];
    for (int i = 0; i < sh.n; ++i) gp[i] = (double)gi * (double)F[i];
    const float reg = alpha_chain(a, sh.n, gp, reg_lambda, reg_b, 0, ga);
    for (int i = 0; i < sh.n; ++i) galpha[(size_t)e * sh.n + i] = ga[i];
    if (reg_vals) reg_vals[e] = reg;
  }
}

// ------------------------------------------------------------------ shift regulariser alone
__global__ __launch_bounds__(kBlock) void shift_reg_kernel(const float* __restrict__ alpha, int S,
                                                           uint32_t rows, int mode, float lambda,
                                                           float b, float* __restrict__ galpha,
                                                           float* __restrict__ reg_vals) {
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= rows) return;
  float a[kMaxS], ga[kMaxS];
  double gp[kMaxS];
  load_row(alpha, r, S, a);
  for (int i = 0; i < S; ++i) gp[i] = 0.0;
  const float reg = alpha_chain(a, S, gp, lambda, b, mode, ga);
  if (galpha)
    for (int i = 0; i < S; ++i) galpha[(size_t)r * S + i] += ga[i];
  if (reg_vals) reg_vals[r] = reg;
}

// ------------------------------------------------------------------ learned_hard_sigmoid fwd
__global__ __launch_bounds__(kBlock) void lhs_fwd_kernel(
    const float* __restrict__ W, const float* __restrict__ alpha, const float* __restrict__ delta,
    const float* __restrict__ zp, Shifts sh, Geo g, uint32_t n, int hard_t, float lo, float hi,
    float* __restrict__ What) {
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t e = blockIdx.x * blockDim.x + threadIdx.x; e < n; e += stride) {
    uint32_t co, ci;
    decompose(e, g, co, ci);
    float a[kMaxS], p[kMaxS];
    load_row(alpha, alpha_row(g, co, ci), sh.n, a);
    soft_targets<kMaxS>(a, sh.n, nullptr, p);
    const float w = W[e], d = delta[co], z = zp[co];
    float out;
    if (hard_t) {
      out = cand_value<1>(w, d, z, sh.s[argmax_first(p, sh.n)], lo, hi);
    } else {
      out = 0.0f;
      for (int i = 0; i < sh.n; ++i) {
        const float t = __fmul_rn(cand_value<1>(w, d, z, sh.s[i], lo, hi), p[i]);
        out = i == 0 ? t : __fadd_rn(out, t);
      }
    }
    What[e] = out;
  }
}

// ------------------------------------------------------------------ adaround fwd / bwd
__device__ __forceinline__ float delta_at(const float* delta, int per_ci, const Geo& g,
                                          uint32_t co, uint32_t ci) {
  return per_ci ? delta[(size_t)co * g.Ci + ci] : delta[co];
}

__global__ __launch_bounds__(kBlock) void adaround_fwd_kernel(
    const float* __restrict__ W, const float* __restrict__ beta, const float* __restrict__ delta,
    int per_ci, const float* __restrict__ zp, float scale, Geo g, uint32_t n, int hard_r, float lo,
    float hi, float* __restrict__ What, uint8_t* __restrict__ codes) {
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t e = blockIdx.x * blockDim.x + threadIdx.x; e < n; e += stride) {
    uint32_t co, ci;
    decompose(e, g, co, ci);
    const float d = __fmul_rn(delta_at(delta, per_ci, g, co, ci), scale), z = zp[co];
    const float b = beta[e];
    const float hr = hard_r ? (b >= 0.0f ? 1.0f : 0.0f) : rect_sigmoid(b);
    const float q = clampf(__fadd_rn(__fadd_rn(floorf(W[e] / d), hr), z), lo, hi);
    What[e] = __fmul_rn(__fsub_rn(q, z), d);
    if (codes) codes[e] = (uint8_t)((int)q & 0xff);
  }
}

// reg_dev != null: the rounding regulariser's gradient (lambda, b = reg_dev[0..1]) is added
// (BRECQ's round loss, block_recon.py:171-174, folded into this backward).
__global__ __launch_bounds__(kBlock) void adaround_bwd_kernel(
    const float* __restrict__ gWhat, const float* __restrict__ W, const float* __restrict__ beta,
    const float* __restrict__ delta, int per_ci, const float* __restrict__ zp, float scale, Geo g,
    uint32_t n, float lo, float hi, float reg_lambda, float reg_b,
    const float* __restrict__ reg_dev, float* __restrict__ gbeta) {
  if (reg_dev) {
    reg_lambda = reg_dev[0];
    reg_b = reg_dev[1];
  }
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t e = blockIdx.x * blockDim.x + threadIdx.x; e < n; e += stride) {
    uint32_t co, ci;
    decompose(e, g, co, ci);
    const float d = __fmul_rn(delta_at(delta, per_ci, g, co, ci), scale), z = zp[co];
    const float b = beta[e];
    const float u = __fadd_rn(__fadd_rn(floorf(W[e] / d), rect_sigmoid(b)), z);
    const float gi = (u >= lo && u <= hi) ? __fmul_rn(gWhat[e], d) : 0.0f;
    const float ga = rect_sigmoid_grad(b, gi);
    gbeta[e] = reg_lambda != 0.0f ? __fadd_rn(ga, round_reg_grad(b, reg_lambda, reg_b)) : ga;
  }
}

// Several weights in one launch (the AdaRound quantizers of a block, BRECQ's weight phase):
// a table of segments, each a contiguous run of kAdaTile-element tiles; every element runs
// the single-weight kernels' exact ops, so the results are bit-identical to one launch per
// weight.
constexpr int kMaxAdaSeg = 8;
constexpr uint32_t kAdaTile = 512;   // 2 elements per thread: as many workgroups as the single launches
struct AdaSeg {
  const float* W;
  const float* beta;
  const float* delta;
  const float* zp;
  const float* gWhat;   // backward
  float* out;           // forward: What; backward: gbeta
  Geo g;
  uint32_t n, blk0;
  int per_ci;
  float scale, lo, hi;
};
struct AdaTable {
  AdaSeg s[kMaxAdaSeg];
  int nseg;
};

__device__ __forceinline__ const AdaSeg& ada_seg(const AdaTable& tab, uint32_t& t0, uint32_t& t1) {
  int si = 0;
  while (si + 1 < tab.nseg && blockIdx.x >= tab.s[si + 1].blk0) ++si;
  const AdaSeg& sg = tab.s[si];
  t0 = (blockIdx.x - sg.blk0) * kAdaTile;
  t1 = min(t0 + kAdaTile, sg.n);
  return sg;
}

__global__ __launch_bounds__(kBlock) void adaround_fwd_multi_kernel(AdaTable tab, int hard_r) {
  uint32_t t0, t1;
  const AdaSeg& sg = ada_seg(tab, t0, t1);
  for (uint32_t e = t0 + threadIdx.x; e < t1; e += kBlock) {
    uint32_t co, ci;
    decompose(e, sg.g, co, ci);
    const float d = __fmul_rn(delta_at(sg.delta, sg.per_ci, sg.g, co, ci), sg.scale), z = sg.zp[co];
    const float b = sg.beta[e];
    const float hr = hard_r ? (b >= 0.0f ? 1.0f : 0.0f) : rect_sigmoid(b);
    const float q = clampf(__fadd_rn(__fadd_rn(floorf(sg.W[e] / d), hr), z), sg.lo, sg.hi);
    sg.out[e] = __fmul_rn(__fsub_rn(q, z), d);
  }
}

__global__ __launch_bounds__(kBlock) void adaround_bwd_multi_kernel(AdaTable tab, float reg_lambda,
                                                                    float reg_b,
                                                                    const float* __restrict__ reg_dev) {
  if (reg_dev) {
    reg_lambda = reg_dev[0];
    reg_b = reg_dev[1];
  }
  uint32_t t0, t1;
  const AdaSeg& sg = ada_seg(tab, t0, t1);
  for (uint32_t e = t0 + threadIdx.x; e < t1; e += kBlock) {
    uint32_t co, ci;
    decompose(e, sg.g, co, ci);
    const float d = __fmul_rn(delta_at(sg.delta, sg.per_ci, sg.g, co, ci), sg.scale), z = sg.zp[co];
    const float b = sg.beta[e];
    const float u = __fadd_rn(__fadd_rn(floorf(sg.W[e] / d), rect_sigmoid(b)), z);
    const float gi = (u >= sg.lo && u <= sg.hi) ? __fmul_rn(sg.gWhat[e], d) : 0.0f;
    const float ga = rect_sigmoid_grad(b, gi);
    sg.out[e] = reg_lambda != 0.0f ? __fadd_rn(ga, round_reg_grad(b, reg_lambda, reg_b)) : ga;
  }
}

// ------------------------------------------------------------------ inits
// -log((zeta-gamma)/(rest-gamma) - 1); python_float/tensor == reciprocal(tensor)*float
__device__ __forceinline__ float rect_inverse(float w, float d) {
  const float t = w / d;
  const float rest = __fsub_rn(t, floorf(t));
  const float r = __fmul_rn(1.0f / __fsub_rn(rest, kGamma), kZmG);
  return -logf(__fsub_rn(r, 1.0f));
}

__global__ __launch_bounds__(kBlock) void rect_init_kernel(const float* __restrict__ W,
                                                           const float* __restrict__ delta,
                                                           int per_ci, Geo g, uint32_t n,
                                                           float* __restrict__ beta) {
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t e = blockIdx.x * blockDim.x + threadIdx.x; e < n; e += stride) {
    uint32_t co, ci;
    decompose(e, g, co, ci);
    beta[e] = rect_inverse(W[e], delta_at(delta, per_ci, g, co, ci));
  }
}

__device__ __forceinline__ float delta_sel(const float* __restrict__ alpha, const float* delta,
                                           const Shifts& sh, const Geo& g, uint32_t co,
                                           uint32_t ci) {
  float a[kMaxS], p[kMaxS];
  load_row(alpha, alpha_row(g, co, ci), sh.n, a);
  soft_targets<kMaxS>(a, sh.n, nullptr, p);
  return __fmul_rn(delta[co], sh.s[argmax_first(p, sh.n)]);
}

__global__ __launch_bounds__(kBlock) void get_delta_kernel(const float* __restrict__ delta,
                                                           const float* __restrict__ alpha,
                                                           Shifts sh, Geo g,
                                                           float* __restrict__ out) {
  const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= g.Co * g.Ci) return;
  const uint32_t co = e / g.Ci, ci = e - co * g.Ci;
  out[e] = delta_sel(alpha, delta, sh, g, co, ci);
}

__global__ __launch_bounds__(kBlock) void beta_from_alpha_kernel(const float* __restrict__ W,
                                                                 const float* __restrict__ delta,
                                                                 const float* __restrict__ alpha,
                                                                 Shifts sh, Geo g, uint32_t n,
                                                                 float* __restrict__ beta) {
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t e = blockIdx.x * blockDim.x + threadIdx.x; e < n; e += stride) {
    uint32_t co, ci;
    decompose(e, g, co, ci);
    beta[e] = rect_inverse(W[e], delta_sel(alpha, delta, sh, g, co, ci));
  }
}

// init_alpha (channelQuant.py:158-199) from per-row squared errors.
__device__ __forceinline__ void init_alpha_row(const double* mse, int S, float* a_out) {
  int mi = 0;
  for (int i = 1; i < S; ++i)
    if (mse[i] < mse[mi]) mi = i;  // torch.min(dim) -> first index of the minimum
  const float clip = S == 1 ? 1.0f : 0.33f;
  const float remain = S == 1 ? 0.0f : (float)((1.0 - 0.33) / (double)(S - 1));
  float lg[kMaxS];
  float sum = 0.0f;
  for (int i = 0; i < S; ++i) {
    const float pr = i == mi ? clip : remain;
    const float x = __fsub_rn(pr, kGamma) / kZmG;   // (x - gamma) / (zeta - gamma)
    lg[i] = logf(x);
    sum = i == 0 ? lg[i] : __fadd_rn(sum, lg[i]);
  }
  const float avg = __fmul_rn(sum, 1.0f / (float)S);  // torch mean: sum * (1/N)
  for (int i = 0; i < S; ++i) a_out[i] = __fsub_rn(lg[i], avg);
}

// Candidate error w - X_i for init_alpha: mode 0 (init_v_beta) X_i = floor(w/(d*s_i))
// (integer floors, the reference's quirk, channelQuant.py:286); mode 1 (init_v) X_i =
// the dequantized 'none'-mode value at d*s_i (channelQuant.py:206-208).
struct CandCfg {
  const float* zp;
  int mode;
  float lo, hi;
};
__device__ __forceinline__ float cand_err(float w, float d, uint32_t co, float s,
                                          const CandCfg& c) {
  const float x = c.mode == 0 ? floorf(w / __fmul_rn(d, s))
                              : cand_value<1>(w, d, c.zp[co], s, c.lo, c.hi);
  const float r = __fsub_rn(w, x);
  return __fmul_rn(r, r);
}

__global__ __launch_bounds__(kBlock) void shift_init_fc(const float* __restrict__ W,
                                                        const float* __restrict__ delta, Shifts sh,
                                                        Geo g, uint32_t n, CandCfg cc,
                                                        float* __restrict__ alpha,
                                                        float* __restrict__ mse_out) {
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t e = blockIdx.x * blockDim.x + threadIdx.x; e < n; e += stride) {
    const uint32_t co = e / g.CiK;
    const float w = W[e], d = delta[co];
    double m[kMaxS];
    for (int i = 0; i < sh.n; ++i) m[i] = (double)cand_err(w, d, co, sh.s[i], cc);
    float a[kMaxS];
    init_alpha_row(m, sh.n, a);
    for (int i = 0; i < sh.n; ++i) {
      alpha[(size_t)e * sh.n + i] = a[i];
      if (mse_out) mse_out[(size_t)e * sh.n + i] = (float)m[i];
    }
  }
}

// ------------------------------------------------------------------ rounding regulariser
__global__ __launch_bounds__(kBlock) void round_reg_kernel(const float* __restrict__ v, int64_t n,
                                                           float lambda, float b,
                                                           float* __restrict__ gv,
                                                           double* __restrict__ part) {
  __shared__ double red[16];
  double acc = 0.0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += stride) {
    const float h = rect_sigmoid(v[e]);
    const float r = __fmul_rn(fabsf(__fsub_rn(h, 0.5f)), 2.0f);
    acc += 1.0 - (double)powf(r, b);
    if (gv && b != 0.0f) {
      const float sg = h > 0.5f ? 1.0f : (h < 0.5f ? -1.0f : 0.0f);
      const float gh = -lambda * b * powf(r, b - 1.0f) * 2.0f * sg;
      gv[e] += rect_sigmoid_grad(v[e], gh);
    }
  }
  acc = block_sum(acc, red);
  if (threadIdx.x == 0) part[blockIdx.x] = acc;
}

__global__ void reduce_partials(const double* __restrict__ part, int nblk, double scale,
                                float* __restrict__ out) {
  __shared__ double red[16];
  double a = 0.0;
  for (int i = threadIdx.x; i < nblk; i += blockDim.x) a += part[i];
  a = block_sum(a, red);
  if (threadIdx.x == 0) out[0] = (float)(a * scale);
}

}  // namespace ssq

using namespace ssq;

// Rows are processed RB at a time with every load of the batch issued before any math
// (the row stride is Ci*K floats, so each load is its own cache line: latency, not
// bandwidth, bounds a row-at-a-time loop).  NS > 0 fixes the shift count at compile time
// so the per-shift loops unroll; NS == 0 takes it from sh.n.
constexpr int kRB = 4;

// MODE 0: adaShift forward (floors + h(beta)); MODE 1: learned_hard_sigmoid forward.
template <int MODE, int NS>
__global__ __launch_bounds__(1024) void shift_fwd_col(
    const float* __restrict__ W, const float* __restrict__ alpha, const float* __restrict__ beta,
    const float* __restrict__ delta, const float* __restrict__ zp, Shifts sh, Geo g,
    ColTiling tl, int hard_t, int hard_r, float lo, float hi, float* __restrict__ What,
    uint8_t* __restrict__ codes) {
  const int S = NS > 0 ? NS : sh.n;
  const uint32_t ci0 = blockIdx.x * tl.ncb;
  const uint32_t nci = min(tl.ncb, g.Ci - ci0);
  const uint32_t t = threadIdx.x;
  if (t >= nci * g.K) return;
  const uint32_t ci = ci0 + t / g.K, j = ci0 * g.K + t;
  float a[kMaxS], p[kMaxS];
  load_row(alpha, ci, S, a);
  soft_targets<kMaxS>(a, S, nullptr, p);
  const float s_sel = sh.s[argmax_first(p, S)];
  const uint32_t co0 = blockIdx.y * tl.R, co1 = min(co0 + tl.R, g.Co);
  auto one = [&](uint32_t co, float w, float d, float z, float b) {
    const uint32_t e = co * g.CiK + j;
    float F[kMaxS];
    if (MODE == 0) {
      const float xf = hard_t ? floorf(w / __fmul_rn(d, s_sel)) : soft_floor(w, d, sh, S, p, F);
      const float hr = hard_r ? (b >= 0.0f ? 1.0f : 0.0f) : rect_sigmoid(b);
      const float q = clampf(__fadd_rn(__fadd_rn(xf, hr), z), lo, hi);
      What[e] = __fmul_rn(__fsub_rn(q, z), __fmul_rn(d, 1.0f));
      if (codes) codes[e] = (uint8_t)((int)q & 0xff);
    } else {
      float out;
      if (hard_t) {
        out = cand_value<1>(w, d, z, s_sel, lo, hi);
      } else {
        out = 0.0f;
        for (int i = 0; i < S; ++i) {
          const float v = __fmul_rn(cand_value<1>(w, d, z, sh.s[i], lo, hi), p[i]);
          out = i == 0 ? v : __fadd_rn(out, v);
        }
      }
      What[e] = out;
    }
  };
  uint32_t co = co0;
  for (; co + kRB <= co1; co += kRB) {
    float w[kRB], d[kRB], z[kRB], b[kRB];
#pragma unroll
    for (int r = 0; r < kRB; ++r) {
      const uint32_t e = (co + r) * g.CiK + j;
      w[r] = W[e];
      d[r] = delta[co + r];
      z[r] = zp[co + r];
      b[r] = MODE == 0 ? beta[e] : 0.0f;
    }
#pragma unroll
    for (int r = 0; r < kRB; ++r) one(co + r, w[r], d[r], z[r], b[r]);
  }
  for (; co < co1; ++co) {
    const uint32_t e = co * g.CiK + j;
    one(co, W[e], delta[co], zp[co], MODE == 0 ? beta[e] : 0.0f);
  }
}

// Stage 1 of the per-input-channel reductions over (Co, K):
//   MODE 0: adaShift backward   sum g_int * F_i   (and gbeta, elementwise)
//   MODE 1: lhs backward        sum gy * Xq_i
//   MODE 2: shift init          sum (w - X_i)^2   (cc.mode selects X_i)
// part[(chunk*Ci + ci)*S + i] = this chunk's sum, accumulated in double in a fixed order.
template <int MODE, int NS>
__global__ __launch_bounds__(1024) void alpha_col_stage1(
    const float* __restrict__ gWhat, const float* __restrict__ W, const float* __restrict__ alpha,
    const float* __restrict__ beta, const float* __restrict__ delta, const float* __restrict__ zp,
    Shifts sh, Geo g, ColTiling tl, int hard_r, float lo, float hi, CandCfg cc,
    float* __restrict__ gbeta, double* __restrict__ part) {
  extern __shared__ double red[];  // [threads][S]
  const int S = NS > 0 ? NS : sh.n;
  const uint32_t ci0 = blockIdx.x * tl.ncb;
  const uint32_t nci = min(tl.ncb, g.Ci - ci0);
  const uint32_t t = threadIdx.x;
  const bool active = t < nci * g.K;
  double acc[kMaxS];
  for (int i = 0; i < S; ++i) acc[i] = 0.0;
  if (active) {
    const uint32_t ci = ci0 + t / g.K, j = ci0 * g.K + t;
    float p[kMaxS];
    if (MODE == 0) {
      float a[kMaxS];
      load_row(alpha, ci, S, a);
      soft_targets<kMaxS>(a, S, nullptr, p);
    }
    auto one = [&](uint32_t co, float w, float d, float z, float b, float gy) {
      if (MODE == 0) {
        float F[kMaxS];
        const float xf = soft_floor(w, d, sh, S, p, F);
        const float hr = hard_r ? (b >= 0.0f ? 1.0f : 0.0f) : rect_sigmoid(b);
        const float u = __fadd_rn(__fadd_rn(xf, hr), z);
        const float gi = (u >= lo && u <= hi) ? __fmul_rn(gy, __fmul_rn(d, 1.0f)) : 0.0f;
        if (gbeta) gbeta[co * g.CiK + j] = hard_r ? 0.0f : rect_sigmoid_grad(b, gi);
        for (int i = 0; i < S; ++i) acc[i] += (double)gi * (double)F[i];
      } else if (MODE == 1) {
        for (int i = 0; i < S; ++i)
          acc[i] += (double)gy * (double)cand_value<1>(w, d, z, sh.s[i], lo, hi);
      } else {
        for (int i = 0; i < S; ++i) acc[i] += (double)cand_err(w, d, co, sh.s[i], cc);
      }
    };
    const uint32_t co0 = blockIdx.y * tl.R, co1 = min(co0 + tl.R, g.Co);
    uint32_t co = co0;
    for (; co + kRB <= co1; co += kRB) {
      float w[kRB], d[kRB], z[kRB], b[kRB], gy[kRB];
#pragma unroll
      for (int r = 0; r < kRB; ++r) {
        const uint32_t e = (co + r) * g.CiK + j;
        w[r] = W[e];
        d[r] = delta[co + r];
        z[r] = MODE != 2 ? zp[co + r] : 0.0f;
        b[r] = MODE == 0 ? beta[e] : 0.0f;
        gy[r] = MODE != 2 ? gWhat[e] : 0.0f;
      }
#pragma unroll
      for (int r = 0; r < kRB; ++r) one(co + r, w[r], d[r], z[r], b[r], gy[r]);
    }
    for (; co < co1; ++co) {
      const uint32_t e = co * g.CiK + j;
      one(co, W[e], delta[co], MODE != 2 ? zp[co] : 0.0f, MODE == 0 ? beta[e] : 0.0f,
          MODE != 2 ? gWhat[e] : 0.0f);
    }
  }
  for (int i = 0; i < S; ++i) red[t * S + i] = acc[i];
  __syncthreads();
  if (t < nci) {
    for (int i = 0; i < S; ++i) {
      double sum = 0.0;
      for (uint32_t k = 0; k < g.K; ++k) sum += red[(t * g.K + k) * S + i];
      part[((size_t)blockIdx.y * g.Ci + ci0 + t) * S + i] = sum;
    }
  }
}

// Stage 2: one wave per input channel -- lane c loads chunk c's partials (one round of
// loads), a fixed shuffle tree sums them (deterministic), and lane 0 applies the
// softmax/clamp chain (+ regulariser, MODE 0) or the init_alpha logits (MODE 2).
template <int MODE, int NS>
__global__ __launch_bounds__(kBlock) void alpha_col_stage2(
    const double* __restrict__ part, uint32_t nchunk, const float* __restrict__ alpha, Shifts sh,
    Geo g, float reg_lambda, float reg_b, const float* __restrict__ reg_dev,
    float* __restrict__ out_alpha, float* __restrict__ side) {
  const int S = NS > 0 ? NS : sh.n;
  const uint32_t ci = blockIdx.x * (blockDim.x / kWave) + threadIdx.x / kWave;
  const uint32_t lane = threadIdx.x & (kWave - 1);
  if (ci >= g.Ci) return;
  // every load this wave needs is issued up front, so their latencies overlap
  float a[kMaxS];
  if (MODE != 2) {
    load_row(alpha, ci, S, a);
    if (reg_dev) {
      reg_lambda = reg_dev[0];
      reg_b = reg_dev[1];
    }
  }
  double tot[kMaxS];
  {
    double v[kMaxChunks / kWave][kMaxS];
#pragma unroll
    for (uint32_t r = 0; r < kMaxChunks / kWave; ++r) {
      const uint32_t c = lane + r * kWave;
      for (int i = 0; i < S; ++i) v[r][i] = c < nchunk ? part[((size_t)c * g.Ci + ci) * S + i] : 0.0;
    }
    for (int i = 0; i < S; ++i) {
      tot[i] = v[0][i];
#pragma unroll
      for (uint32_t r = 1; r < kMaxChunks / kWave; ++r) tot[i] += v[r][i];
    }
  }
  // MODE 0: lane i < S evaluates shift i's regulariser term while the partials are in
  // flight; lane 0 gathers them (same values, same summation order as alpha_chain)
  float sm[kMaxS], p[kMaxS];
  double rv = 0.0, rg = 0.0;
  if (MODE != 2) {
    soft_targets<kMaxS>(a, S, sm, p);
    if (MODE == 0 && reg_lambda != 0.0f && lane < (uint32_t)S) {
      float pl = p[0];
      for (int i = 1; i < S; ++i)
        if ((uint32_t)i == lane) pl = p[i];
      reg_term(pl, reg_lambda, reg_b, 0, rv, rg);
    }
  }
  for (int i = 0; i < S; ++i) tot[i] = wave_sum(tot[i]);
  double rvs[kMaxS], rgs[kMaxS];
  for (int i = 0; i < S; ++i) {
    rvs[i] = __shfl(rv, i, kWave);
    rgs[i] = __shfl(rg, i, kWave);
  }
  if (lane != 0) return;
  if (MODE == 2) {
    float a[kMaxS];
    init_alpha_row(tot, S, a);
    for (int i = 0; i < S; ++i) {
      out_alpha[(size_t)ci * S + i] = a[i];
      if (side) side[(size_t)ci * S + i] = (float)tot[i];
    }
    return;
  }
  float ga[kMaxS], reg = 0.0f;
  if (MODE == 0 && reg_lambda != 0.0f) {
    double acc = 0.0;
    for (int i = 0; i < S; ++i) {
      acc += rvs[i];
      tot[i] += rgs[i];
    }
    reg = (float)((double)reg_lambda * acc);
  }
  softmax_clamp_bwd(sm, S, tot, ga);
  for (int i = 0; i < S; ++i) out_alpha[(size_t)ci * S + i] = ga[i];
  if (side && MODE == 0) side[ci] = reg;
}

template <int MODE>
static int launch_alpha_col(const Geo& g, const Shifts& sh, const float* gWhat, const float* W,
                            const float* alpha, const float* beta, const float* delta,
                            const float* zp, int hard_r, float lo, float hi, const CandCfg& cc,
                            float reg_lambda, float reg_b, const float* reg_dev, float* out_alpha,
                            float* gbeta, float* side, void* ws, size_t ws_bytes, hipStream_t s,
                            const char* what) {
  const ColTiling tl = col_tiling(g);
  SSQ_REQUIRE(tl.threads <= 1024, SSQ_E_ARG, "%s: kernel window K > 1024 unsupported", what);
  SSQ_REQUIRE(ws && ws_bytes >= col_ws_bytes(g, sh.n), SSQ_E_WS, "%s: workspace too small", what);
  const size_t lds = (size_t)tl.threads * sh.n * sizeof(double);
#define SSQ_STAGE1(NS)                                                                        \
  hipLaunchKernelGGL((alpha_col_stage1<MODE, NS>), dim3(tl.ncolblk, tl.nchunk), dim3(tl.threads), \
                     lds, s, gWhat, W, alpha, beta, delta, zp, sh, g, tl, hard_r, lo, hi, cc,      \
                     gbeta, (double*)ws)
  switch (sh.n) {
    case 1: SSQ_STAGE1(1); break;
    case 2: SSQ_STAGE1(2); break;
    case 3: SSQ_STAGE1(3); break;
    case 4: SSQ_STAGE1(4); break;
    default: SSQ_STAGE1(0); break;
  }
#undef SSQ_STAGE1
  const unsigned waves = kBlock / kWave;
  const unsigned blocks2 = (g.Ci + waves - 1) / waves;
#define SSQ_STAGE2(NS)                                                                         \
  hipLaunchKernelGGL((alpha_col_stage2<MODE, NS>), dim3(blocks2), dim3(kBlock), 0, s,             \
                     (const double*)ws, tl.nchunk, alpha, sh, g, reg_lambda, reg_b, reg_dev,     \
                     out_alpha, side)
  switch (sh.n) {
    case 1: SSQ_STAGE2(1); break;
    case 2: SSQ_STAGE2(2); break;
    case 3: SSQ_STAGE2(3); break;
    case 4: SSQ_STAGE2(4); break;
    default: SSQ_STAGE2(0); break;
  }
#undef SSQ_STAGE2
  return check_launch(what);
}

template <int MODE>
static void launch_shift_fwd_col(const Geo& g, const Shifts& sh, const ColTiling& tl,
                                 const float* W, const float* alpha, const float* beta,
                                 const float* delta, const float* zp, int hard_t, int hard_r,
                                 float lo, float hi, float* What, uint8_t* codes, hipStream_t s) {
#define SSQ_FWD(NS)                                                                         \
  hipLaunchKernelGGL((shift_fwd_col<MODE, NS>), dim3(tl.ncolblk, tl.nchunk), dim3(tl.threads), 0, \
                     s, W, alpha, beta, delta, zp, sh, g, tl, hard_t, hard_r, lo, hi, What, codes)
  switch (sh.n) {
    case 1: SSQ_FWD(1); break;
    case 2: SSQ_FWD(2); break;
    case 3: SSQ_FWD(3); break;
    case 4: SSQ_FWD(4); break;
    default: SSQ_FWD(0); break;
  }
#undef SSQ_FWD
}

extern "C" int ssq_adashift_fwd(const float* W, const float* alpha, const float* beta,
                                const float* delta, const float* zp, const float* shifts, int S,
                                int64_t Co, int64_t Ci, int64_t K, int is_fc, int hard_targets,
                                int hard_round, int qmin, int qmax, float* What, void* codes,
                                ssq_stream_t stream) {
  SSQ_GEO(Co, Ci, K, is_fc, g);
  SSQ_SHIFTS(shifts, S, sh);
  SSQ_REQUIRE(W && alpha && beta && delta && zp && What, SSQ_E_ARG, "ssq_adashift_fwd: null");
  const uint32_t n = g.Co * g.CiK;
  if (is_fc) {
    hipLaunchKernelGGL(adashift_fwd_kernel, dim3(grid_for(n, kBlock)), dim3(kBlock), 0,
                       (hipStream_t)stream, W, alpha, beta, delta, zp, sh, g, n, hard_targets,
                       hard_round, (float)qmin, (float)qmax, What, (uint8_t*)codes);
  } else {
    const ColTiling tl = col_tiling(g, (g.Co + 3) / 4);
    SSQ_REQUIRE(tl.threads <= 1024, SSQ_E_ARG, "ssq_adashift_fwd: kernel window K > 1024");
    launch_shift_fwd_col<0>(g, sh, tl, W, alpha, beta, delta, zp, hard_targets, hard_round,
                            (float)qmin, (float)qmax, What, (uint8_t*)codes, (hipStream_t)stream);
  }
  return check_launch("ssq_adashift_fwd");
}

extern "C" size_t ssq_adashift_bwd_workspace_size(int64_t Co, int64_t Ci, int64_t K, int S,
                                                  int is_fc) {
  Geo g;
  if (is_fc || S < 1 || S > kMaxS || make_geo(Co, Ci, K, 0, g) != SSQ_OK) return 0;
  return col_ws_bytes(g, S);
}

extern "C" int ssq_adashift_bwd(const float* gWhat, const float* W, const float* alpha,
                                const float* beta, const float* delta, const float* zp,
                                const float* shifts, int S, int64_t Co, int64_t Ci, int64_t K,
                                int is_fc, int hard_round, int qmin, int qmax, float reg_lambda,
                                float reg_b, const float* reg_dev, float* galpha, float* gbeta,
                                float* reg_vals, void* ws, size_t ws_bytes,
                                ssq_stream_t stream) {
  SSQ_GEO(Co, Ci, K, is_fc, g);
  SSQ_SHIFTS(shifts, S, sh);
  SSQ_REQUIRE(gWhat && W && alpha && beta && delta && zp && galpha, SSQ_E_ARG,
              "ssq_adashift_bwd: null");
  hipStream_t s = (hipStream_t)stream;
  const uint32_t n = g.Co * g.CiK;
  if (is_fc) {
    hipLaunchKernelGGL(alpha_grad_fc<0>, dim3(grid_for(n, kBlock)), dim3(kBlock), 0, s, gWhat, W,
                       alpha, beta, delta, zp, sh, g, n, hard_round, (float)qmin, (float)qmax,
                       reg_lambda, reg_b, reg_dev, galpha, gbeta, reg_vals);
    return check_launch("ssq_adashift_bwd(fc)");
  }
  const CandCfg cc{nullptr, 0, 0.0f, 0.0f};
  return launch_alpha_col<0>(g, sh, gWhat, W, alpha, beta, delta, zp, hard_round, (float)qmin,
                             (float)qmax, cc, reg_lambda, reg_b, reg_dev, galpha, gbeta, reg_vals,
                             ws, ws_bytes, s, "ssq_adashift_bwd");
}

extern "C" int ssq_shift_reg(const float* alpha, int S, int64_t rows, int mode, float lambda,
                             float b, float* galpha, float* reg_vals, ssq_stream_t stream) {
  SSQ_REQUIRE(alpha && rows >= 1 && S >= 1 && S <= kMaxS && (mode == 0 || mode == 1), SSQ_E_ARG,
              "ssq_shift_reg: bad args");
  hipLaunchKernelGGL(shift_reg_kernel, dim3((unsigned)((rows + kBlock - 1) / kBlock)),
                     dim3(kBlock), 0, (hipStream_t)stream, alpha, S, (uint32_t)rows, mode, lambda,
                     b, galpha, reg_vals);
  return check_launch("ssq_shift_reg");
}

extern "C" int ssq_lhs_fwd(const float* W, const float* alpha, const float* delta,
                           const float* zp, const float* shifts, int S, int64_t Co, int64_t Ci,
                           int64_t K, int is_fc, int hard_targets, int qmin, int qmax,
                           float* What, ssq_stream_t stream) {
  SSQ_GEO(Co, Ci, K, is_fc, g);
  SSQ_SHIFTS(shifts, S, sh);
  SSQ_REQUIRE(W && alpha && delta && zp && What, SSQ_E_ARG, "ssq_lhs_fwd: null");
  const uint32_t n = g.Co * g.CiK;
  if (is_fc) {
    hipLaunchKernelGGL(lhs_fwd_kernel, dim3(grid_for(n, kBlock)), dim3(kBlock), 0,
                       (hipStream_t)stream, W, alpha, delta, zp, sh, g, n, hard_targets,
                       (float)qmin, (float)qmax, What);
  } else {
    const ColTiling tl = col_tiling(g, (g.Co + 3) / 4);
    SSQ_REQUIRE(tl.threads <= 1024, SSQ_E_ARG, "ssq_lhs_fwd: kernel window K > 1024");
    launch_shift_fwd_col<1>(g, sh, tl, W, alpha, nullptr, delta, zp, hard_targets, 0,
                            (float)qmin, (float)qmax, What, nullptr, (hipStream_t)stream);
  }
  return check_launch("ssq_lhs_fwd");
}

extern "C" int ssq_lhs_bwd(const float* gWhat, const float* W, const float* alpha,
                           const float* delta, const float* zp, const float* shifts, int S,
                           int64_t Co, int64_t Ci, int64_t K, int is_fc, int qmin, int qmax,
                           float* galpha, void* ws, size_t ws_bytes, ssq_stream_t stream) {
  SSQ_GEO(Co, Ci, K, is_fc, g);
  SSQ_SHIFTS(shifts, S, sh);
  SSQ_REQUIRE(gWhat && W && alpha && delta && zp && galpha, SSQ_E_ARG, "ssq_lhs_bwd: null");
  hipStream_t s = (hipStream_t)stream;
  const uint32_t n = g.Co * g.CiK;
  if (is_fc) {
    hipLaunchKernelGGL(alpha_grad_fc<1>, dim3(grid_for(n, kBlock)), dim3(kBlock), 0, s, gWhat, W,
                       alpha, nullptr, delta, zp, sh, g, n, 0, (float)qmin, (float)qmax, 0.0f,
                       0.0f, nullptr, galpha, nullptr, nullptr);
    return check_launch("ssq_lhs_bwd(fc)");
  }
  const CandCfg cc{nullptr, 0, 0.0f, 0.0f};
  return launch_alpha_col<1>(g, sh, gWhat, W, alpha, nullptr, delta, zp, 0, (float)qmin,
                             (float)qmax, cc, 0.0f, 0.0f, nullptr, galpha, nullptr, nullptr, ws,
                             ws_bytes, s, "ssq_lhs_bwd");
}

extern "C" int ssq_adaround_fwd(const float* W, const float* beta, const float* delta,
                                int delta_per_ci, const float* zp, float scale, int64_t Co,
                                int64_t Ci, int64_t K, int hard_round, int qmin, int qmax,
                                float* What, void* codes, ssq_stream_t stream) {
  SSQ_GEO(Co, Ci, K, 0, g);
  SSQ_REQUIRE(W && beta && delta && zp && What, SSQ_E_ARG, "ssq_adaround_fwd: null");
  const uint32_t n = g.Co * g.CiK;
  hipLaunchKernelGGL(adaround_fwd_kernel, dim3(grid_for(n, kBlock)), dim3(kBlock), 0,
                     (hipStream_t)stream, W, beta, delta, delta_per_ci, zp, scale, g, n,
                     hard_round, (float)qmin, (float)qmax, What, (uint8_t*)codes);
  return check_launch("ssq_adaround_fwd");
}

extern "C" int ssq_adaround_bwd(const float* gWhat, const float* W, const float* beta,
                                const float* delta, int delta_per_ci, const float* zp, float scale,
                                int64_t Co, int64_t Ci, int64_t K, int qmin, int qmax,
                                float reg_lambda, float reg_b, const float* reg_dev, float* gbeta,
                                ssq_stream_t stream) {
  SSQ_GEO(Co, Ci, K, 0, g);
  SSQ_REQUIRE(gWhat && W && beta && delta && zp && gbeta, SSQ_E_ARG, "ssq_adaround_bwd: null");
  const uint32_t n = g.Co * g.CiK;
  hipLaunchKernelGGL(adaround_bwd_kernel, dim3(grid_for(n, kBlock)), dim3(kBlock), 0,
                     (hipStream_t)stream, gWhat, W, beta, delta, delta_per_ci, zp, scale, g, n,
                     (float)qmin, (float)qmax, reg_lambda, reg_b, reg_dev, gbeta);
  return check_launch("ssq_adaround_bwd");
}

static int ada_table(const char* what, int nseg, const float* const* gWhat, const float* const* W,
                     const float* const* beta, const float* const* delta,
                     const int* delta_per_ci, const float* const* zp, const float* scale,
                     const int64_t* Co, const int64_t* Ci, const int64_t* K, const int* qmin,
                     const int* qmax, float* const* out, AdaTable& tab, uint32_t& nblk) {
  SSQ_REQUIRE(nseg >= 1 && nseg <= kMaxAdaSeg, SSQ_E_ARG, "%s: 1 <= nseg <= %d", what, kMaxAdaSeg);
  SSQ_REQUIRE(W && beta && delta && delta_per_ci && zp && scale && Co && Ci && K && qmin && qmax &&
              out, SSQ_E_ARG, "%s: null array", what);
  tab.nseg = nseg;
  int64_t blk = 0;
  for (int i = 0; i < nseg; ++i) {
    AdaSeg& sg = tab.s[i];
    {
      const int r = make_geo(Co[i], Ci[i], K[i], 0, sg.g);
      if (r) return r;
    }
    SSQ_REQUIRE(W[i] && beta[i] && delta[i] && zp[i] && out[i] && (!gWhat || gWhat[i]), SSQ_E_ARG,
                "%s: segment %d has a null pointer", what, i);
    sg.W = W[i];
    sg.beta = beta[i];
    sg.delta = delta[i];
    sg.zp = zp[i];
    sg.gWhat = gWhat ? gWhat[i] : nullptr;
    sg.out = out[i];
    sg.n = sg.g.Co * sg.g.CiK;
    sg.blk0 = (uint32_t)blk;
    sg.per_ci = delta_per_ci[i];
    sg.scale = scale[i];
    sg.lo = (float)qmin[i];
    sg.hi = (float)qmax[i];
    blk += (sg.n + kAdaTile - 1) / kAdaTile;
  }
  SSQ_REQUIRE(blk < (1ll << 31), SSQ_E_ARG, "%s: too many tiles", what);
  nblk = (uint32_t)blk;
  return SSQ_OK;
}

extern "C" int ssq_adaround_fwd_multi(int nseg, const float* const* W, const float* const* beta,
                                      const float* const* delta, const int* delta_per_ci,
                                      const float* const* zp, const float* scale,
                                      const int64_t* Co, const int64_t* Ci, const int64_t* K,
                                      int hard_round, const int* qmin, const int* qmax,
                                      float* const* What, ssq_stream_t stream) {
  AdaTable tab;
  uint32_t nblk = 0;
  const int rc = ada_table("ssq_adaround_fwd_multi", nseg, nullptr, W, beta, delta, delta_per_ci,
                           zp, scale, Co, Ci, K, qmin, qmax, What, tab, nblk);
  if (rc) return rc;
  hipLaunchKernelGGL(adaround_fwd_multi_kernel, dim3(nblk), dim3(kBlock), 0, (hipStream_t)stream,
                     tab, hard_round);
  return check_launch("ssq_adaround_fwd_multi");
}

extern "C" int ssq_adaround_bwd_multi(int nseg, const float* const* gWhat, const float* const* W,
                                      const float* const* beta, const float* const* delta,
                                      const int* delta_per_ci, const float* const* zp,
                                      const float* scale, const int64_t* Co, const int64_t* Ci,
                                      const int64_t* K, const int* qmin, const int* qmax,
                                      float reg_lambda, float reg_b, const float* reg_dev,
                                      float* const* gbeta, ssq_stream_t stream) {
  SSQ_REQUIRE(gWhat, SSQ_E_ARG, "ssq_adaround_bwd_multi: null gWhat");
  AdaTable tab;
  uint32_t nblk = 0;
  const int rc = ada_table("ssq_adaround_bwd_multi", nseg, gWhat, W, beta, delta, delta_per_ci,
                           zp, scale, Co, Ci, K, qmin, qmax, gbeta, tab, nblk);
  if (rc) return rc;
  hipLaunchKernelGGL(adaround_bwd_multi_kernel, dim3(nblk), dim3(kBlock), 0, (hipStream_t)stream,
                     tab, reg_lambda, reg_b, reg_dev);
  return check_launch("ssq_adaround_bwd_multi");
}

extern "C" int ssq_rect_init(const float* W, const float* delta, int delta_per_ci, int64_t Co,
                             int64_t Ci, int64_t K, float* beta, ssq_stream_t stream) {
  SSQ_GEO(Co, Ci, K, 0, g);
  SSQ_REQUIRE(W && delta && beta, SSQ_E_ARG, "ssq_rect_init: null");
  const uint32_t n = g.Co * g.CiK;
  hipLaunchKernelGGL(rect_init_kernel, dim3(grid_for(n, kBlock)), dim3(kBlock), 0,
                     (hipStream_t)stream, W, delta, delta_per_ci, g, n, beta);
  return check_launch("ssq_rect_init");
}

extern "C" int ssq_get_delta(const float* delta, const float* alpha, const float* shifts, int S,
                             int64_t Co, int64_t Ci, int is_fc, float* out, ssq_stream_t stream) {
  SSQ_GEO(Co, Ci, 1, is_fc, g);
  SSQ_SHIFTS(shifts, S, sh);
  SSQ_REQUIRE(delta && alpha && out, SSQ_E_ARG, "ssq_get_delta: null");
  hipLaunchKernelGGL(get_delta_kernel, dim3((g.Co * g.Ci + kBlock - 1) / kBlock), dim3(kBlock), 0,
                     (hipStream_t)stream, delta, alpha, sh, g, out);
  return check_launch("ssq_get_delta");
}

extern "C" size_t ssq_shift_init_workspace_size(int64_t Co, int64_t Ci, int64_t K, int S,
                                                int is_fc) {
  return ssq_adashift_bwd_workspace_size(Co, Ci, K, S, is_fc);
}

extern "C" int ssq_shift_init(const float* W, const float* delta, const float* zp,
                              const float* shifts, int S, int64_t Co, int64_t Ci, int64_t K,
                              int is_fc, int mode, int qmin, int qmax, float* alpha, float* beta,
                              float* mse_out, void* ws, size_t ws_bytes, ssq_stream_t stream) {
  SSQ_GEO(Co, Ci, K, is_fc, g);
  SSQ_SHIFTS(shifts, S, sh);
  SSQ_REQUIRE(W && delta && alpha && (mode == 0 || mode == 1), SSQ_E_ARG, "ssq_shift_init: args");
  SSQ_REQUIRE(mode == 0 || zp, SSQ_E_ARG, "ssq_shift_init: mode 1 needs zero_point");
  hipStream_t s = (hipStream_t)stream;
  const uint32_t n = g.Co * g.CiK;
  const CandCfg cc{zp, mode, (float)qmin, (float)qmax};
  if (is_fc) {
    hipLaunchKernelGGL(shift_init_fc, dim3(grid_for(n, kBlock)), dim3(kBlock), 0, s, W, delta, sh,
                       g, n, cc, alpha, mse_out);
  } else {
    const int rc = launch_alpha_col<2>(g, sh, nullptr, W, nullptr, nullptr, delta, nullptr, 0, 0.0f,
                                       0.0f, cc, 0.0f, 0.0f, nullptr, alpha, nullptr, mse_out, ws,
                                       ws_bytes, s, "ssq_shift_init");
    if (rc) return rc;
  }
  if (beta)  // init_v_beta: beta from delta * s[argmax p(alpha)] (channelQuant.py:289-292)
    hipLaunchKernelGGL(beta_from_alpha_kernel, dim3(grid_for(n, kBlock)), dim3(kBlock), 0, s, W,
                       delta, alpha, sh, g, n, beta);
  return check_launch("ssq_shift_init");
}

extern "C" size_t ssq_round_reg_workspace_size(int64_t n) {
  (void)n;
  return 1024 * sizeof(double);
}

extern "C" int ssq_round_reg(const float* v, int64_t n, float lambda, float b, float* loss_out,
                             float* gv, void* ws, size_t ws_bytes, ssq_stream_t stream) {
  SSQ_REQUIRE(v && n >= 1 && loss_out, SSQ_E_ARG, "ssq_round_reg: bad args");
  SSQ_REQUIRE(ws && ws_bytes >= ssq_round_reg_workspace_size(n), SSQ_E_WS,
              "ssq_round_reg: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  const int grid = grid_for(n, kBlock, 1024);
  hipLaunchKernelGGL(round_reg_kernel, dim3(grid), dim3(kBlock), 0, s, v, n, lambda, b, gv,
                     (double*)ws);
  hipLaunchKernelGGL(reduce_partials, dim3(1), dim3(kBlock), 0, s, (const double*)ws, grid,
                     (double)lambda, loss_out);
  return check_launch("ssq_round_reg");
}
