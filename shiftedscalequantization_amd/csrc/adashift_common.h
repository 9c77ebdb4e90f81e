// Shared types and helpers of the ChannelQuant kernels (adashift.hip: recomputing
// K5-K9 kernels; adashift_prep.hip: the prepared multi-segment K5p/K6p kernels).
#pragma once

#include "ssq_common.h"

namespace ssq {

constexpr int kMaxS = 8;

struct Shifts {
  float s[kMaxS];
  int n;
};

struct Geo {
  uint32_t Co, Ci, K, CiK;
  int is_fc;
};

__device__ __forceinline__ void decompose(uint32_t e, const Geo& g, uint32_t& co, uint32_t& ci) {
  co = e / g.CiK;
  ci = (e - co * g.CiK) / g.K;
}

__device__ __forceinline__ uint32_t alpha_row(const Geo& g, uint32_t co, uint32_t ci) {
  return g.is_fc ? co * g.Ci + ci : ci;
}

__device__ __forceinline__ void load_row(const float* __restrict__ a, uint32_t row, int S,
                                         float* out) {
  for (int i = 0; i < S; ++i) out[i] = a[(size_t)row * S + i];
}

// soft shifted floor  sum_i F_i * p_i  (x_out = x_q0*p0; x_out += x_q1*p1; ...)
__device__ __forceinline__ float soft_floor(float w, float d, const Shifts& sh, int S,
                                            const float* p, float* F) {
  float acc = 0.0f;
  for (int i = 0; i < S; ++i) {
    F[i] = floorf(w / __fmul_rn(d, sh.s[i]));
    const float t = __fmul_rn(F[i], p[i]);
    acc = i == 0 ? t : __fadd_rn(acc, t);
  }
  return acc;
}

// ------------------------------------------------------------------ shared stage-2 helper
// Backward through p = clamp(softmax(a)*c + gamma, 0, 1), plus the optional shift
// regulariser lambda*sum(1-|2p-1|^b) (value returned, gradient folded into g_p).
// One shift's regulariser term and its gradient wrt p_i, in fp32 like the reference's
// tensor ops (pow / log and their autograd): mode 0 = lambda * (1 - |2p-1|^b) (without
// lambda in the value), mode 1 = entropy -p log(p + 1e-10).
__device__ __forceinline__ void reg_term(float p, float reg_lambda, float reg_b, int reg_mode,
                                         double& val, double& grad) {
  if (reg_mode == 0) {  // lambda * sum(1 - ((p - 0.5).abs() * 2).pow(b))
    const float r = __fmul_rn(fabsf(__fsub_rn(p, 0.5f)), 2.0f);
    val = (double)__fsub_rn(1.0f, powf(r, reg_b));
    grad = 0.0;
    if (reg_b != 0.0f) {
      const float sg = p > 0.5f ? 1.0f : (p < 0.5f ? -1.0f : 0.0f);
      const float gr = __fmul_rn(__fmul_rn(-reg_lambda, reg_b), powf(r, __fsub_rn(reg_b, 1.0f)));
      grad = (double)__fmul_rn(__fmul_rn(gr, 2.0f), sg);
    }
  } else {
    const float lg = logf(__fadd_rn(p, 1e-10f));
    val = -(double)__fmul_rn(p, lg);
    grad = (double)(-reg_lambda * __fadd_rn(lg, p / __fadd_rn(p, 1e-10f)));
  }
}

// Backward through p = clamp(softmax(a)*c + gamma, 0, 1) given d/dp in g_p (double).
__device__ __forceinline__ void softmax_clamp_bwd(const float* s, int S, const double* g_p,
                                                  float* ga_out) {
  double gs[kMaxS], dot = 0.0;
  for (int i = 0; i < S; ++i) {
    const float u = __fadd_rn(__fmul_rn(s[i], kZmG), kGamma);
    gs[i] = (u >= 0.0f && u <= 1.0f) ? g_p[i] * (double)kZmG : 0.0;
    dot += gs[i] * (double)s[i];
  }
  for (int i = 0; i < S; ++i) ga_out[i] = (float)((double)s[i] * (gs[i] - dot));
}

// g_p += regulariser gradient; returns the regulariser value (summed in double, fixed
// order); then the softmax/clamp backward into ga_out.
__device__ __forceinline__ float alpha_chain(const float* a, int S, double* g_p, float reg_lambda,
                                             float reg_b, int reg_mode, float* ga_out) {
  float s[kMaxS], p[kMaxS];
  soft_targets<kMaxS>(a, S, s, p);
  float reg = 0.0f;
  if (reg_lambda != 0.0f) {
    double acc = 0.0;
    for (int i = 0; i < S; ++i) {
      double v, gr;
      reg_term(p[i], reg_lambda, reg_b, reg_mode, v, gr);
      acc += v;
      g_p[i] += gr;
    }
    reg = (float)((double)reg_lambda * acc);
  }
  softmax_clamp_bwd(s, S, g_p, ga_out);
  return reg;
}

// ------------------------------------------------------------------ host helpers
static inline int make_geo(int64_t Co, int64_t Ci, int64_t K, int is_fc, Geo& g) {
  SSQ_REQUIRE(Co >= 1 && Ci >= 1 && K >= 1, SSQ_E_ARG, "bad geometry (%lld,%lld,%lld)",
              (long long)Co, (long long)Ci, (long long)K);
  SSQ_REQUIRE(Co * Ci * K < (1ll << 31), SSQ_E_ARG, "weight too large for 32-bit indexing");
  SSQ_REQUIRE(!is_fc || K == 1, SSQ_E_ARG, "Linear weights must have K == 1");
  g.Co = (uint32_t)Co;
  g.Ci = (uint32_t)Ci;
  g.K = (uint32_t)K;
  g.CiK = (uint32_t)(Ci * K);
  g.is_fc = is_fc;
  return SSQ_OK;
}

static inline int make_shifts(const float* shifts, int S, Shifts& sh) {
  SSQ_REQUIRE(S >= 1 && S <= kMaxS && shifts, SSQ_E_ARG, "1 <= S <= %d shifts required", kMaxS);
  sh.n = S;
  for (int i = 0; i < kMaxS; ++i) sh.s[i] = i < S ? shifts[i] : 1.0f;
  return SSQ_OK;
}

// ------------------------------------------------------------------ column-tiled conv kernels
// A conv weight (Co, Ci, K) is tiled as [chunk of R output channels] x [column block of
// ncb whole input channels = ncb*K contiguous columns].  Thread t owns column
// j = ci0*K + t of every row of the chunk, so its input channel ci = ci0 + t/K is fixed:
// the softmax p(alpha[ci]) is computed once per thread (not once per element), and each
// row is one coalesced sweep of ncb*K contiguous floats.  delta/zp are per row (wave
// uniform).  The alpha reductions write one fixed-order partial per (chunk, ci) and a
// second launch sums the chunks with one wave per input channel (fixed shuffle tree):
// deterministic, no atomics.
struct ColTiling {
  uint32_t ncb, ncolblk, R, nchunk, threads;
  uint32_t whole;   // prepared alpha backward: one chunk, finalised in the workgroup
  uint32_t form;    // prepared alpha backward: 0 thread-column (+ stage 2), 3 one workgroup per ci
};
constexpr uint32_t kMaxChunks = 256;  // stage 2: lane c sums chunks c, c+64, ... in order

// max_chunks: kMaxChunks for the reductions (stage 2 has one lane per chunk); the
// forward has no second stage and takes as many row chunks as keep ~8 workgroups per CU
// (down to 4 rows = one load batch per thread: its time is load latency, not bandwidth).
static inline ColTiling col_tiling(const Geo& g, uint32_t max_chunks = kMaxChunks) {
  ColTiling t;
  t.ncb = g.K >= (uint32_t)kBlock ? 1u : (uint32_t)kBlock / g.K;
  if (t.ncb > g.Ci) t.ncb = g.Ci;
  t.ncolblk = (g.Ci + t.ncb - 1) / t.ncb;
  t.threads = (t.ncb * g.K + kWave - 1) / kWave * kWave;
  uint32_t want = 2048 / t.ncolblk;  // ~8 workgroups per CU
  if (want < 1) want = 1;
  if (want > max_chunks) want = max_chunks;
  if (want > g.Co) want = g.Co;
  t.R = (g.Co + want - 1) / want;
  t.nchunk = (g.Co + t.R - 1) / t.R;
  t.whole = 0;
  t.form = 0;
  return t;
}
static inline size_t col_ws_bytes(const Geo& g, int S) {
  const ColTiling t = col_tiling(g);
  return (size_t)t.nchunk * g.Ci * S * sizeof(double);
}

}  // namespace ssq

#define SSQ_GEO(Co, Ci, K, fc, g)                      \
  Geo g;                                               \
  {                                                    \
    int _r = make_geo(Co, Ci, K, fc, g);               \
    if (_r) return _r;                                 \
  }
#define SSQ_SHIFTS(p, S, sh)                           \
  Shifts sh;                                           \
  {                                                    \
    int _r = make_shifts(p, S, sh);                    \
    if (_r) return _r;                                 \
  }
