// K11: reconstruction loss value + gradient in one pass, and K14: the batch gather of
// the reconstruction loop (layer_recon_fused_shiftedScale.py:94-102).
//
// lp_loss (quant_layer.py:25-32) is five eager launches plus five more in autograd; here
// one pass reads pred and tgt and writes d loss/d pred (12 B/elem), with a deterministic
// reduction of the loss value (workgroup partials summed in index order by a 1-workgroup
// finalize launch, or by a finalize task riding on a later launch: fin_tasks.h).  For p == 2
// the gradient is bit-identical to PyTorch's: (1/M) * (2*|d|) * sgn(d).
#include <stdlib.h>

#include <type_traits>

#include "fin_tasks.h"
#include "prep_ride.h"
#include "ssq_common.h"

namespace ssq {

// Target rows: tgt itself, or (GATHER) rows idx[r] of a [N, row] cache, r = i / row, so the
// loop's batch target is never materialised.
struct TgtRows {
  const int64_t* idx;
  uint32_t row;
  FastDiv div_row;
};

template <bool GATHER>
__device__ __forceinline__ int64_t tgt_index(uint32_t i, const TgtRows& tr) {
  if (!GATHER) return i;
  const uint32_t r = fdiv(i, tr.div_row);
  return tr.idx[r] * (int64_t)tr.row + (i - r * tr.row);
}

// float4 body over the first n & ~3 elements (when aligned), scalar tail; one double
// partial per block.  GATHER: tr is in float4 units in the body, in elements in the tail.
template <int PMODE, bool GATHER>
__global__ __launch_bounds__(kBlock) void lp_loss_kernel(const float* __restrict__ pred,
                                                         const float* __restrict__ tgt, int64_t n,
                                                         float p, float inv_m,
                                                         float* __restrict__ grad,
                                                         const float* __restrict__ gscale,
                                                         int relu_mask, int vec, TgtRows tr4,
                                                         TgtRows tr1,
                                                         double* __restrict__ part) {
  __shared__ double red[16];
  double acc = 0.0;
  const float gs = gscale ? gscale[0] : 1.0f;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t n4 = vec ? n >> 2 : 0;  // vec: every pointer 16-B aligned
  const f32x4* P = (const f32x4*)pred;
  const f32x4* T = (const f32x4*)tgt;
  f32x4* G = (f32x4*)grad;
  for (int64_t i = tid; i < n4; i += stride) {
    const f32x4 x = __builtin_nontemporal_load(P + i);
    const f32x4 t = __builtin_nontemporal_load(T + tgt_index<GATHER>((uint32_t)i, tr4));
    f32x4 g;
    g.x = lp_elem<PMODE>(x.x, t.x, p, inv_m, gs, relu_mask, acc);
    g.y = lp_elem<PMODE>(x.y, t.y, p, inv_m, gs, relu_mask, acc);
    g.z = lp_elem<PMODE>(x.z, t.z, p, inv_m, gs, relu_mask, acc);
    g.w = lp_elem<PMODE>(x.w, t.w, p, inv_m, gs, relu_mask, acc);
    if (grad) __builtin_nontemporal_store(g, G + i);
  }
  for (int64_t i = (n4 << 2) + tid; i < n; i += stride) {
    const float g = lp_elem<PMODE>(pred[i], tgt[tgt_index<GATHER>((uint32_t)i, tr1)], p, inv_m, gs,
                                   relu_mask, acc);
    if (grad) grad[i] = g;
  }
  if (!part) return;
  acc = block_sum(acc, red);
  if (threadIdx.x == 0) part[blockIdx.x] = acc;   // lp_loss_finalize / a finalize task sums them
}

// the block partials summed in index order (every load issued first)
__global__ void lp_loss_finalize(const double* __restrict__ part, int nblk, double m,
                                 float* __restrict__ out) {
  fin_loss(part, nblk, m, out);
}

// ------------------------------------------------------------------ K13 fused epilogue
// out = act(y + bias[c] (+ res)),  c = (i / hw) % C, in the reference's op order (conv
// bias add, residual add, ReLU: three separate fp32 roundings -> bit-identical to the
// eager sequence), one pass instead of three.  yrows (optional): y is a cache of per-sample
// [C, hw] rows and sample n of this batch is its row yrows[n] (BRECQ's act phase reads the
// frozen conv's precomputed outputs in place instead of a gathered copy).
template <bool RES, int ACT, bool QUANT, bool AFFINE>
__global__ __launch_bounds__(kBlock) void bias_act_kernel(const float* __restrict__ y,
                                                          const float* __restrict__ bias,
                                                          const float* __restrict__ res,
                                                          float* __restrict__ out, uint32_t n,
                                                          FastDiv div_hw, FastDiv div_c,
                                                          uint32_t C, int vec,
                                                          float* __restrict__ yq,
                                                          const float* __restrict__ qdelta,
                                                          const float* __restrict__ qzp,
                                                          float qlo, float qhi,
                                                          const float* __restrict__ gamma,
                                                          const float* __restrict__ phi,
                                                          const int64_t* __restrict__ yrows,
                                                          const int64_t* __restrict__ rrows,
                                                          uint32_t chw,
                                                          const int64_t* __restrict__ stage_src,
                                                          int64_t* __restrict__ stage_dst,
                                                          uint32_t stage_n) {
  const uint32_t stride = gridDim.x * blockDim.x;
  // the iteration's device words (a chunk ring row) copied into the loop's static slot, which
  // the iteration's later launches read (this launch reads its row maps from the ring row)
  if (stage_dst && blockIdx.x == 0)
    for (uint32_t k = threadIdx.x; k < stage_n; k += blockDim.x) stage_dst[k] = stage_src[k];
  QParams qp{1.0f, 0.0f, qlo, qhi};
  // element i of the batch -> its offset in y / res (a row map: sample n = i / chw is row
  // map[n] of the cache)
  auto off = [&](const int64_t* map, uint32_t i) -> int64_t {
    if (!map) return (int64_t)i;
    const uint32_t nn = fdiv(fdiv(i, div_hw), div_c);
    return map[nn] * (int64_t)chw + (int64_t)(i - nn * chw);
  };
  if (QUANT) {
    qp.d = qdelta[0];
    qp.z = qzp[0];
  }
  // channel c's operands applied to one element (the reference's op order)
  auto epi = [&](float v, float rv, float bc, float gc, float pc) {
    float t = bias ? __fadd_rn(v, bc) : v;
    if (AFFINE) t = __fadd_rn(__fmul_rn(t, gc), pc);  // out*alpha_out + beta_out
    if (RES) t = __fadd_rn(t, rv);
    return act_fwd<ACT>(t);  // torch clamp: keeps -0 and NaN
  };
  auto one = [&](uint32_t i, float v, float rv) {
    const uint32_t q = fdiv(i, div_hw);
    const uint32_t c = q - fdiv(q, div_c) * C;
    return epi(v, rv, bias ? bias[c] : 0.0f, AFFINE ? gamma[c] : 1.0f, AFFINE ? phi[c] : 0.0f);
  };
  auto fq = [&](float t) {
    float q;
    return fq1(t, qp, &q);
  };
  if (vec == 2) {
    // hw % 4 == 0: a float4 lies in one (n, c) plane -- one channel lookup, one row-map
    // lookup and one set of channel operands per float4 instead of per element (the
    // act-quant form of this pass is VALU-bound: the divide of the fake quant)
    const uint32_t n4 = n / 4;
    for (uint32_t v = blockIdx.x * blockDim.x + threadIdx.x; v < n4; v += stride) {
      const uint32_t i = 4 * v, q = fdiv(i, div_hw), nn = fdiv(q, div_c), c = q - nn * C;
      const uint32_t inrow = i - nn * chw;
      const f32x4 a = *(const f32x4*)(y + (yrows ? yrows[nn] * (int64_t)chw + inrow : (int64_t)i));
      f32x4 rr = {0.0f, 0.0f, 0.0f, 0.0f};
      if (RES) rr = *(const f32x4*)(res + (rrows ? rrows[nn] * (int64_t)chw + inrow : (int64_t)i));
      const float bc = bias ? bias[c] : 0.0f;
      const float gc = AFFINE ? gamma[c] : 1.0f, pc = AFFINE ? phi[c] : 0.0f;
      f32x4 o;
      o.x = epi(a.x, rr.x, bc, gc, pc);
      o.y = epi(a.y, rr.y, bc, gc, pc);
      o.z = epi(a.z, rr.z, bc, gc, pc);
      o.w = epi(a.w, rr.w, bc, gc, pc);
      if (!QUANT || out) ((f32x4*)out)[v] = o;
      if (QUANT) {
        f32x4 r;
        r.x = fq(o.x);
        r.y = fq(o.y);
        r.z = fq(o.z);
        r.w = fq(o.w);
        ((f32x4*)yq)[v] = r;
      }
    }
  } else if (vec) {
    const uint32_t n4 = n / 4;
    for (uint32_t v = blockIdx.x * blockDim.x + threadIdx.x; v < n4; v += stride) {
      const f32x4 a = *(const f32x4*)(y + off(yrows, 4 * v));   // hw % 4 == 0 with a map
      f32x4 rr = {0.0f, 0.0f, 0.0f, 0.0f};
      if (RES) rr = *(const f32x4*)(res + off(rrows, 4 * v));
      f32x4 o;
      o.x = one(4 * v, a.x, rr.x);
      o.y = one(4 * v + 1, a.y, rr.y);
      o.z = one(4 * v + 2, a.z, rr.z);
      o.w = one(4 * v + 3, a.w, rr.w);
      if (!QUANT || out) ((f32x4*)out)[v] = o;
      if (QUANT) {
        f32x4 r;
        r.x = fq(o.x);
        r.y = fq(o.y);
        r.z = fq(o.z);
        r.w = fq(o.w);
        ((f32x4*)yq)[v] = r;
      }
    }
  } else {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
      const float t = one(i, y[off(yrows, i)], RES ? res[off(rrows, i)] : 0.0f);
      if (!QUANT || out) out[i] = t;
      if (QUANT) yq[i] = fq(t);
    }
  }
}

// Activation backward from the output (act_pass): ReLU = torch threshold_backward
// (out <= 0 -> 0; a NaN output passes its gradient), ReLU6 = hardtanh_backward.
template <int ACT>
__global__ __launch_bounds__(kBlock) void relu_bwd_kernel(const f32x4* __restrict__ g,
                                                          const f32x4* __restrict__ out,
                                                          f32x4* __restrict__ gin, uint32_t n4) {
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t v = blockIdx.x * blockDim.x + threadIdx.x; v < n4; v += stride) {
    const f32x4 a = g[v], o = out[v];
    f32x4 r;
    r.x = act_pass<ACT>(o.x) ? a.x : 0.0f;
    r.y = act_pass<ACT>(o.y) ? a.y : 0.0f;
    r.z = act_pass<ACT>(o.z) ? a.z : 0.0f;
    r.w = act_pass<ACT>(o.w) ? a.w : 0.0f;
    gin[v] = r;
  }
}
template <int ACT>
__global__ __launch_bounds__(kBlock) void relu_bwd_tail(const float* __restrict__ g,
                                                        const float* __restrict__ out,
                                                        float* __restrict__ gin, uint32_t start,
                                                        uint32_t n) {
  const uint32_t i = start + blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) gin[i] = act_pass<ACT>(out[i]) ? g[i] : 0.0f;
}

// ------------------------------------------------------------------ Adam step
// torch.optim.Adam's single-tensor update (the reference's optimizer) for several
// parameter tensors in one launch, op for op in fp32:
//   m = m + (1-b1)*(g - m)                       exp_avg.lerp_(grad, 1-beta1)
//   v = v*b2 + ((1-b2)*g)*g                      exp_avg_sq.mul_(beta2).addcmul_(g, g, 1-beta2)
//   p = p + (nss*m) / (sqrt(v)/bc2s + eps)       param.addcdiv_(exp_avg, denom, -step_size)
// nss = -lr/(1-b1^t) and bc2s = sqrt(1-b2^t) are host doubles rounded to fp32, read from
// `hyper` (device) when given so that a captured graph picks up each step's values.
struct AdamSeg {
  float* p;
  const float* g;
  float* m;
  float* v;
  uint32_t n, blk0;
};
constexpr int kMaxAdamSeg = 48;
constexpr int kAdamTile = 2048;
struct AdamTable {
  AdamSeg s[kMaxAdamSeg];
  int nseg;
};

__global__ __launch_bounds__(kBlock) void adam_kernel(AdamTable tab, float w1, float b2, float w2,
                                                      float eps, const float* __restrict__ hyper,
                                                      float nss, float bc2s, FinTable fin) {
  // queued finalize tasks that write none of the gradients read here ride on the launch
  // (its first workgroups; ssq_adam)
  if (blockIdx.x < fin.nwg) {
    run_fin(fin, blockIdx.x);
    return;
  }
  const uint32_t bid = blockIdx.x - fin.nwg;
  if (hyper) {
    nss = hyper[0];
    bc2s = hyper[1];
  }
  int si = 0;
  while (si + 1 < tab.nseg && bid >= tab.s[si + 1].blk0) ++si;
  const AdamSeg& sg = tab.s[si];
  const uint32_t t0 = (bid - sg.blk0) * (uint32_t)kAdamTile;
  const uint32_t t1 = min(t0 + (uint32_t)kAdamTile, sg.n);
  for (uint32_t e = t0 + threadIdx.x; e < t1; e += blockDim.x) {
    const float g = sg.g[e];
    float m = sg.m[e], v = sg.v[e];
    m = __fadd_rn(m, __fmul_rn(w1, __fsub_rn(g, m)));
    v = __fadd_rn(__fmul_rn(v, b2), __fmul_rn(__fmul_rn(w2, g), g));
    const float denom = __fadd_rn(__fdiv_rn(__fsqrt_rn(v), bc2s), eps);
    sg.p[e] = __fadd_rn(sg.p[e], __fdiv_rn(__fmul_rn(nss, m), denom));
    sg.m[e] = m;
    sg.v[e] = v;
  }
}

// One element of the epilogue backward (the pass below): the forward recomputed from y with
// the forward's fp32 operations, then dL/d(pre-activation) and the per-row sums.
struct EpiRow {
  float b, ga, ph;                                   // bias[c], gamma[c], phi[c]
  float rb, rga, rph;                                // RES 2: the residual's own epilogue
  double sg = 0, sp = 0, a0 = 0, a1 = 0, a2 = 0, a3 = 0, la = 0, sgr = 0, spr = 0;
};
// Residual epilogue (RES 2): the residual is the raw output of the block's downsample conv,
// and its own K13 epilogue -- bias add, gamma^z/phi^z, no activation, the ops of
// bias_act_kernel<false, 0, false, *> -- is applied here (rbias / raffine: which of them the
// downsample has, uniform).
struct ResEpi {
  const float* bias;
  const float* gamma;
  const float* phi;
};
template <int RES, int ACT, bool QUANT, bool AFFINE, int LOSS, bool BIAS>
__device__ __forceinline__ void epi_elem(EpiRow& w, float d, float z, float lo, float hi,
                                         float inv_m, float lp, bool rbias, bool raffine,
                                         float yv, float gv_or_tgt, float rv, float& oy,
                                         float& orr) {
  const float pre = BIAS ? __fadd_rn(yv, w.b) : yv;
  float t = AFFINE ? __fadd_rn(__fmul_rn(pre, w.ga), w.ph) : pre;
  float prer = rv;
  if (RES == 2) {
    prer = rbias ? __fadd_rn(rv, w.rb) : rv;
    rv = raffine ? __fadd_rn(__fmul_rn(prer, w.rga), w.rph) : prer;
  }
  if (RES) t = __fadd_rn(t, rv);
  t = act_fwd<ACT>(t);
  float tq = 0.0f, q = 0.0f;
  bool m = true;
  if (QUANT) {
    tq = t / d;
    const float v = round_ste_zp(tq, z);                // the act quantizer's round_ste
    m = (v >= lo) && (v <= hi);
    q = clampf(v, lo, hi);
  }
  float gv = gv_or_tgt;
  if (LOSS) {   // the forward's output (fq1's dequant), then the loss gradient wrt it
    const float o = QUANT ? __fmul_rn(__fsub_rn(q, z), d) : t;
    gv = lp_elem<LOSS == 1 ? 0 : 2>(o, gv_or_tgt, LOSS == 1 ? 2.0f : lp, inv_m, 1.0f, 0, w.la);
  }
  float gt = gv;
  if (QUANT) {
    const float gq = __fmul_rn(gv, d);
    const float gi = m ? gq : 0.0f;
    gt = gi / d;
    w.a0 += (double)gv * (double)__fsub_rn(q, z);
    w.a1 += (double)gi * (double)(tq / d);
    w.a2 += (double)gi;
    w.a3 += (double)gq;
  }
  if (ACT) gt = act_pass<ACT>(t) ? gt : 0.0f;
  oy = AFFINE ? __fmul_rn(gt, w.ga) : gt;
  orr = gt;
  w.sg += (double)gt * (double)pre;
  w.sp += (double)gt;
  if (RES == 2) {   // the residual epilogue's backward (epi_elem<false, 0, false, *> of g_t)
    if (raffine) orr = __fmul_rn(gt, w.rga);
    w.sgr += (double)gt * (double)prer;
    w.spr += (double)gt;
  }
}

// the row's sums over the wave (fixed shuffle tree), written by lane 0 to its kEpiParts slots
template <bool QUANT, int LOSS, int RES>
__device__ __forceinline__ void epi_row_sums(EpiRow& w, uint32_t lane, double* __restrict__ o) {
  w.sg = wave_sum(w.sg);
  w.sp = wave_sum(w.sp);
  if (RES == 2) {
    w.sgr = wave_sum(w.sgr);
    w.spr = wave_sum(w.spr);
  }
  if (QUANT) {
    w.a0 = wave_sum(w.a0);
    w.a1 = wave_sum(w.a1);
    w.a2 = wave_sum(w.a2);
    w.a3 = wave_sum(w.a3);
  }
  if (LOSS) w.la = wave_sum(w.la);
  if (lane == 0) {
    o[0] = w.sg;
    o[1] = w.sp;
    o[2] = w.a0;
    o[3] = w.a1;
    o[4] = w.a2;
    o[5] = w.a3;
    o[6] = w.la;
    if (RES == 2) {
      o[7] = w.sgr;
      o[8] = w.spr;
    }
  }
}

// Small planes (<= 64 elements or float4s per row: ResNet layer3 / layer4, 14x14 / 7x7):
// 4 rows per wave, 16 lanes per row (RPW = kG16).  Each lane sums its elements of the row in
// order (j = l16, l16 + 16, ...), then the 16 lanes of a row are added by one xor tree
// (8, 4, 2, 1) that reduces the wave's 4 rows at once -- 4 shuffle steps per quantity for 4
// rows, where a row per wave takes 6 for 1.  Every path that produces these rows' records
// (the plain backward, the fused tail) takes this form for the same shape, so they agree bit
// for bit; the order differs from the row-per-wave form's only in how the doubles are
// grouped.
constexpr int kG16 = 16;
__device__ __forceinline__ double group16_sum(double v) {
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}
template <bool QUANT, int LOSS, int RES>
__device__ __forceinline__ void epi_row_sums16(EpiRow& w, bool writer, double* __restrict__ o) {
  w.sg = group16_sum(w.sg);
  w.sp = group16_sum(w.sp);
  if (RES == 2) {
    w.sgr = group16_sum(w.sgr);
    w.spr = group16_sum(w.spr);
  }
  if (QUANT) {
    w.a0 = group16_sum(w.a0);
    w.a1 = group16_sum(w.a1);
    w.a2 = group16_sum(w.a2);
    w.a3 = group16_sum(w.a3);
  }
  if (LOSS) w.la = group16_sum(w.la);
  if (writer) {
    o[0] = w.sg;
    o[1] = w.sp;
    o[2] = w.a0;
    o[3] = w.a1;
    o[4] = w.a2;
    o[5] = w.a3;
    o[6] = w.la;
    if (RES == 2) {
      o[7] = w.sgr;
      o[8] = w.spr;
    }
  }
}

// Backward of the K13 epilogue (optionally with gamma^z/phi^z and the act quantizer):
// t = (y + bias[c]) [*gamma[c] + phi[c]] [+ res] [-> ReLU] [-> fq]; given g = dL/d(output)
//   g_t = dL/d(pre-ReLU t): the STE of the act quantizer (fq_bwd_pt's formulas), then the
//         ReLU mask (relu output <= 0 -> 0, torch threshold_backward);
//   gy  = g_t * gamma[c] (mul backward) or g_t;   gres = g_t;
//   per row (n, c): sum g_t*(y + bias[c]) -> dL/dgamma[c],  sum g_t -> dL/dphi[c],
//   and the act quantizer's four sums -> dL/ddelta, dL/dzp.
// A wave owns RPW (n, c) rows: RPW = 1 walks a row of any length in 64-lane strides; RPW = 4
// (rows of <= 64 elements or float4s: ResNet-18 layer3 / layer4 planes) gives each lane one
// element (float4) of each of 4 consecutive rows, every load of the 4 rows issued before any
// math -- the same per-lane values and order as RPW = 1, so the same bits, with a quarter of
// the waves.  The pre-activation values are recomputed from y with the forward's fp32
// operations (bit-identical masks), nothing of the forward is stored.
// LOSS (the fused tail, ssq_epilogue_loss_bwd): g is the cache of target rows instead of
// dL/d(output); the output is recomputed (the forward's ops) and dL/d(output) is the
// lp_loss gradient of K11 (lp_elem, identical ops: LOSS 1 for p = 2, 2 for a general p such
// as the act phase's 2.4), the loss partial goes to slot 6.
// RES 2 (fused tail only): res is the downsample conv's raw output and re its epilogue; gres
// then receives dL/d(that raw output) and the row records' slots 7 / 8 its gamma / phi sums.
// The wave's RPW rows (bid: the workgroup among the launch's main ones); returns the wave's
// loss sum (LOSS: its rows' totals in row order), 0 for a wave past the last row.
template <int RES, int ACT, bool QUANT, bool AFFINE, bool VEC, int LOSS, int RPW>
__device__ __forceinline__ double epilogue_rows_body(
    const float* __restrict__ g, const float* __restrict__ y, const float* __restrict__ bias,
    const float* __restrict__ gamma, const float* __restrict__ phi, const float* __restrict__ res,
    uint32_t rows, uint32_t C, uint32_t hw, const float* __restrict__ qdelta,
    const float* __restrict__ qzp, float lo, float hi, float* __restrict__ gy,
    float* __restrict__ gres, double* __restrict__ part, const int64_t* __restrict__ lidx,
    float inv_m, float lp, const ResEpi& re, uint32_t bid, const int64_t* __restrict__ yrows,
    const int64_t* __restrict__ rrows) {
  const uint32_t lane = threadIdx.x & (kWave - 1);
  constexpr uint32_t kRows = RPW == kG16 ? 4u : (uint32_t)RPW;     // rows per wave
  const uint32_t r0 = (bid * (kBlock / kWave) + threadIdx.x / kWave) * kRows;
  if (r0 >= rows) return 0.0;
  const float d = QUANT ? qdelta[0] : 1.0f, z = QUANT ? qzp[0] : 0.0f;
  const bool rbias = RES == 2 && re.bias, raffine = RES == 2 && re.gamma;
  // per-row constants of the row-per-wave / 4-rows forms (the 16-lane form loads its own)
  constexpr int kW = RPW == kG16 ? 1 : RPW;
  EpiRow w[kW];
#pragma unroll
  for (int k = 0; k < kW; ++k) {
    if (RPW == kG16) break;
    const uint32_t c = (r0 + k) % C;
    const bool ok = r0 + k < rows;
    w[k].b = (bias && ok) ? bias[c] : 0.0f;
    w[k].ga = (AFFINE && ok) ? gamma[c] : 1.0f;
    w[k].ph = (AFFINE && ok) ? phi[c] : 0.0f;
    w[k].rb = (rbias && ok) ? re.bias[c] : 0.0f;
    w[k].rga = (raffine && ok) ? re.gamma[c] : 1.0f;
    w[k].rph = (raffine && ok) ? re.phi[c] : 0.0f;
  }
  auto elem = [&](EpiRow& wr, float yv, float gv, float rv, float& oy, float& orr) {
    if (bias) epi_elem<RES, ACT, QUANT, AFFINE, LOSS, true>(wr, d, z, lo, hi, inv_m, lp, rbias, raffine, yv, gv, rv, oy, orr);
    else epi_elem<RES, ACT, QUANT, AFFINE, LOSS, false>(wr, d, z, lo, hi, inv_m, lp, rbias, raffine, yv, gv, rv, oy, orr);
  };
  // row r = (n, c) of a [*, C, hw] cache read through a row map: row c of cached sample
  // map[n] (LOSS: the target; yrows / rrows: y / res read in place from a cache)
  auto mapped = [&](const int64_t* map, uint32_t r) -> int64_t {
    return map ? (map[r / C] * (int64_t)C + r % C) * hw : (int64_t)r * hw;
  };
  auto gbase_of = [&](uint32_t r) -> int64_t { return mapped(LOSS ? lidx : nullptr, r); };
  if (RPW == kG16) {
    // row r0 + (lane >> 4), this lane's elements l16, l16 + 16, ... (<= 4 of them: every
    // load issued before any math)
    const uint32_t l16 = lane & 15, r = r0 + (lane >> 4);
    const bool ok = r < rows;
    const uint32_t rr = ok ? r : r0;
    const uint32_t c = rr % C;
    EpiRow wr;
    wr.b = bias ? bias[c] : 0.0f;
    wr.ga = AFFINE ? gamma[c] : 1.0f;
    wr.ph = AFFINE ? phi[c] : 0.0f;
    wr.rb = rbias ? re.bias[c] : 0.0f;
    wr.rga = raffine ? re.gamma[c] : 1.0f;
    wr.rph = raffine ? re.phi[c] : 0.0f;
    const int64_t base = (int64_t)rr * hw, gbase = gbase_of(rr);
    const int64_t ybase = mapped(yrows, rr), rbase = mapped(rrows, rr);
    const uint32_t nv = VEC ? hw / 4 : hw;     // <= 64 (host-checked)
    if (VEC) {
      f32x4 yv[4], gv[4], rv[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t v = l16 + 16 * k;
        yv[k] = gv[k] = rv[k] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
        if (ok && v < nv) {
          yv[k] = ((const f32x4*)(y + ybase))[v];
          gv[k] = ((const f32x4*)(g + gbase))[v];
          if (RES) rv[k] = ((const f32x4*)(res + rbase))[v];
        }
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t v = l16 + 16 * k;
        if (!(ok && v < nv)) continue;
        float oy[4], orr[4];
        elem(wr, yv[k].x, gv[k].x, rv[k].x, oy[0], orr[0]);
        elem(wr, yv[k].y, gv[k].y, rv[k].y, oy[1], orr[1]);
        elem(wr, yv[k].z, gv[k].z, rv[k].z, oy[2], orr[2]);
        elem(wr, yv[k].w, gv[k].w, rv[k].w, oy[3], orr[3]);
        if (gy) ((f32x4*)(gy + base))[v] = f32x4{oy[0], oy[1], oy[2], oy[3]};
        if (gres) ((f32x4*)(gres + base))[v] = f32x4{orr[0], orr[1], orr[2], orr[3]};
      }
    } else {
      float yv[4], gv[4], rv[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t j = l16 + 16 * k;
        yv[k] = gv[k] = rv[k] = 0.0f;
        if (ok && j < nv) {
          yv[k] = y[ybase + j];
          gv[k] = g[gbase + j];
          if (RES) rv[k] = res[rbase + j];
        }
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t j = l16 + 16 * k;
        if (!(ok && j < nv)) continue;
        float oy, orr;
        elem(wr, yv[k], gv[k], rv[k], oy, orr);
        if (gy) gy[base + j] = oy;
        if (gres) gres[base + j] = orr;
      }
    }
    epi_row_sums16<QUANT, LOSS, RES>(wr, ok && l16 == 0, part + (int64_t)rr * kEpiParts);
    // the wave's loss sum: its rows' totals in row order (lane 0's value is the one used)
    double wl = 0.0;
    if (LOSS) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const double t = __shfl(wr.la, 16 * k, kWave);
        if (r0 + k < rows) wl += t;
      }
    }
    return wl;
  }
  if (RPW == 1) {
    EpiRow& wr = w[0];
    const int64_t base = (int64_t)r0 * hw, gbase = gbase_of(r0);
    const int64_t ybase = mapped(yrows, r0), rbase = mapped(rrows, r0);
    if (VEC) {
      const f32x4* Y = (const f32x4*)(y + ybase);
      const f32x4* G = (const f32x4*)(g + gbase);
      const f32x4* R = RES ? (const f32x4*)(res + rbase) : nullptr;
      f32x4* GY = gy ? (f32x4*)(gy + base) : nullptr;
      f32x4* GR = gres ? (f32x4*)(gres + base) : nullptr;
      for (uint32_t v = lane; v < hw / 4; v += kWave) {
        const f32x4 yv = Y[v], gv = G[v];
        f32x4 rv = {0.0f, 0.0f, 0.0f, 0.0f};
        if (RES) rv = R[v];
        float oy[4], orr[4];
        elem(wr, yv.x, gv.x, rv.x, oy[0], orr[0]);
        elem(wr, yv.y, gv.y, rv.y, oy[1], orr[1]);
        elem(wr, yv.z, gv.z, rv.z, oy[2], orr[2]);
        elem(wr, yv.w, gv.w, rv.w, oy[3], orr[3]);
        if (GY) GY[v] = f32x4{oy[0], oy[1], oy[2], oy[3]};
        if (GR) GR[v] = f32x4{orr[0], orr[1], orr[2], orr[3]};
      }
    } else {
      for (uint32_t j = lane; j < hw; j += kWave) {
        float oy, orr;
        elem(wr, y[ybase + j], g[gbase + j], RES ? res[rbase + j] : 0.0f, oy, orr);
        if (gy) gy[base + j] = oy;
        if (gres) gres[base + j] = orr;
      }
    }
    epi_row_sums<QUANT, LOSS, RES>(wr, lane, part + (int64_t)r0 * kEpiParts);
    return wr.la;
  }
  // RPW rows, one element (float4) per lane and row, all loads first
  double wl = 0.0;
  const uint32_t nv = VEC ? hw / 4 : hw;     // <= 64 (host-checked)
  const bool on = lane < nv;
  if (VEC) {
    f32x4 yv[RPW], gv[RPW], rv[RPW];
#pragma unroll
    for (int k = 0; k < RPW; ++k) {
      yv[k] = gv[k] = rv[k] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
      if (on && r0 + k < rows) {
        yv[k] = ((const f32x4*)(y + mapped(yrows, r0 + k)))[lane];
        gv[k] = ((const f32x4*)(g + gbase_of(r0 + k)))[lane];
        if (RES) rv[k] = ((const f32x4*)(res + mapped(rrows, r0 + k)))[lane];
      }
    }
#pragma unroll
    for (int k = 0; k < RPW; ++k) {
      if (r0 + k >= rows) break;             // wave-uniform
      if (on) {
        float oy[4], orr[4];
        elem(w[k], yv[k].x, gv[k].x, rv[k].x, oy[0], orr[0]);
        elem(w[k], yv[k].y, gv[k].y, rv[k].y, oy[1], orr[1]);
        elem(w[k], yv[k].z, gv[k].z, rv[k].z, oy[2], orr[2]);
        elem(w[k], yv[k].w, gv[k].w, rv[k].w, oy[3], orr[3]);
        const int64_t base = (int64_t)(r0 + k) * hw;
        if (gy) ((f32x4*)(gy + base))[lane] = f32x4{oy[0], oy[1], oy[2], oy[3]};
        if (gres) ((f32x4*)(gres + base))[lane] = f32x4{orr[0], orr[1], orr[2], orr[3]};
      }
      epi_row_sums<QUANT, LOSS, RES>(w[k], lane, part + (int64_t)(r0 + k) * kEpiParts);
      wl += w[k].la;
    }
  } else {
    float yv[RPW], gv[RPW], rv[RPW];
#pragma unroll
    for (int k = 0; k < RPW; ++k) {
      yv[k] = gv[k] = rv[k] = 0.0f;
      if (on && r0 + k < rows) {
        yv[k] = y[mapped(yrows, r0 + k) + lane];
        gv[k] = g[gbase_of(r0 + k) + lane];
        if (RES) rv[k] = res[mapped(rrows, r0 + k) + lane];
      }
    }
#pragma unroll
    for (int k = 0; k < RPW; ++k) {
      if (r0 + k >= rows) break;             // wave-uniform
      if (on) {
        float oy, orr;
        elem(w[k], yv[k], gv[k], rv[k], oy, orr);
        const int64_t base = (int64_t)(r0 + k) * hw;
        if (gy) gy[base + lane] = oy;
        if (gres) gres[base + lane] = orr;
      }
      epi_row_sums<QUANT, LOSS, RES>(w[k], lane, part + (int64_t)(r0 + k) * kEpiParts);
      wl += w[k].la;
    }
  }
  return wl;
}

template <int RES, int ACT, bool QUANT, bool AFFINE, bool VEC, int LOSS, int RPW>
__global__ __launch_bounds__(kBlock) void epilogue_bwd_rows(
    const float* __restrict__ g, const float* __restrict__ y, const float* __restrict__ bias,
    const float* __restrict__ gamma, const float* __restrict__ phi, const float* __restrict__ res,
    uint32_t rows, uint32_t C, uint32_t hw, const float* __restrict__ qdelta,
    const float* __restrict__ qzp, float lo, float hi, float* __restrict__ gy,
    float* __restrict__ gres, double* __restrict__ part, FinTable fin, uint32_t nmain,
    const int64_t* __restrict__ lidx, float inv_m, float lp, ResEpi re,
    const int64_t* __restrict__ yrows, const int64_t* __restrict__ rrows) {
  // queued finalize tasks ride on this launch: its first workgroups (dispatched first, so
  // they run beside the main work instead of after it)
  (void)nmain;
  if (blockIdx.x < fin.nwg) {
    run_fin(fin, blockIdx.x);
    return;
  }
  const uint32_t bid = blockIdx.x - fin.nwg;
  // the act quantizer's delta reduction (fin_epi, a later launch) counts its workgroups in
  // this call's workspace: start it at zero
  if (QUANT && bid == 0 && threadIdx.x == 0)
    __hip_atomic_store((gu32_t*)(part + delta_ticket_offset(rows)), 0u, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  const double wl = epilogue_rows_body<RES, ACT, QUANT, AFFINE, VEC, LOSS, RPW>(
      g, y, bias, gamma, phi, res, rows, C, hw, qdelta, qzp, lo, hi, gy, gres, part, lidx, inv_m,
      lp, re, bid, yrows, rrows);
  if (!LOSS) return;
  // the fused tail's loss: one partial per workgroup (its waves in order) after the rows'
  // records, so the finalize sums rows / (4 RPW) values instead of every row's
  __shared__ double sl[kBlock / kWave];
  if ((threadIdx.x & (kWave - 1)) == 0) sl[threadIdx.x / kWave] = wl;
  __syncthreads();
  if (threadIdx.x == 0) {
    double a = sl[0];
#pragma unroll
    for (int k = 1; k < kBlock / kWave; ++k) a += sl[k];
    part[(int64_t)rows * kEpiParts + bid] = a;
  }
}

// blocks [0, nb): per-channel gamma / phi gradients (sum over n in order); block nb (when
// launched): the act quantizer's delta / zp gradients (rows in a fixed order, as
// fq_bwd_finalize).
__global__ __launch_bounds__(kBlock) void epilogue_bwd_finalize(
    const double* __restrict__ part, uint32_t N, uint32_t C, uint32_t nb,
    float* __restrict__ ggamma, float* __restrict__ gphi, float* __restrict__ gdelta,
    float* __restrict__ gzp) {
  const AdamRef none[3] = {AdamRef{}, AdamRef{}, AdamRef{}};
  fin_epi(blockIdx.x, part, N, C, nb, gridDim.x - nb, 0, ggamma, gphi, gdelta, gzp, AdamConst{},
          none);
}

// the queued finalize tasks of a stream as one standalone launch
__global__ __launch_bounds__(kBlock) void fin_tasks_kernel(FinTable fin) {
  run_fin(fin, blockIdx.x);
}

// ------------------------------------------------------------------ finalize queue (host)
static bool g_fin_defer = false;
struct PendingFin {
  hipStream_t s;
  FinTask t;
};
constexpr int kMaxPendingFin = 16;
static PendingFin g_fin_pending[kMaxPendingFin];
static int g_fin_npending = 0;

bool fin_defer_on() { return g_fin_defer; }

FinTable fin_take(hipStream_t s) {
  FinTable ft{};
  ft.n = 0;
  ft.nwg = 0;
  int keep = 0;
  for (int i = 0; i < g_fin_npending; ++i) {
    if (g_fin_pending[i].s == s && ft.n < kMaxFin) {
      ft.t[ft.n++] = g_fin_pending[i].t;
      ft.nwg += g_fin_pending[i].t.nwg;
    } else {
      g_fin_pending[keep++] = g_fin_pending[i];
    }
  }
  g_fin_npending = keep;
  return ft;
}

int fin_flush(hipStream_t s) {
  for (;;) {
    const FinTable ft = fin_take(s);
    if (ft.n == 0) return SSQ_OK;
    hipLaunchKernelGGL(fin_tasks_kernel, dim3(ft.nwg), dim3(kBlock), 0, s, ft);
    const int rc = check_launch("ssq finalize tasks");
    if (rc) return rc;
  }
}

int fin_push(hipStream_t s, const FinTask& t) {
  int mine = 0;
  for (int i = 0; i < g_fin_npending; ++i) mine += g_fin_pending[i].s == s;
  if (mine >= kMaxFin || g_fin_npending >= kMaxPendingFin) {
    const int rc = fin_flush(s);
    if (rc) return rc;
    if (g_fin_npending >= kMaxPendingFin) {   // other streams' tasks: launch them too
      while (g_fin_npending) {
        const int r2 = fin_flush(g_fin_pending[0].s);
        if (r2) return r2;
      }
    }
  }
  g_fin_pending[g_fin_npending++] = PendingFin{s, t};
  return SSQ_OK;
}

// ------------------------------------------------------------------ armed optimizer step
// ssq_adam_arm records the loop's Adam parameters; the epilogue backward entry points log
// the gradient tensors they produce for armed gamma^z / phi^z (gradient pointer per
// parameter pointer); the next alpha-backward launch of the stream attaches the whole step
// (adam_attach) or nothing; ssq_adam_take reports which.
constexpr int kMaxArmed = 32;
constexpr uint32_t kMaxRideAdam = 4096;   // elements of a final gradient a kind-3 task takes
struct ArmedAdam {
  bool on, consumed;
  hipStream_t s;
  int n;
  float* p[kMaxArmed];
  float* m[kMaxArmed];
  float* v[kMaxArmed];
  int64_t len[kMaxArmed];
  const float* g[kMaxArmed];    // logged final gradient (gamma^z / phi^z), or null
  AdamConst c;
};
static ArmedAdam g_armed{};

static int armed_index(const void* p) {
  for (int k = 0; k < g_armed.n; ++k)
    if (g_armed.p[k] == p) return k;
  return -1;
}

// an epilogue backward on stream s produces the gradients of (gamma, phi)
static void adam_log(hipStream_t s, const float* gamma, const float* phi, const float* ggamma,
                     const float* gphi) {
  if (!g_armed.on || g_armed.s != s) return;
  const int kg = gamma && ggamma ? armed_index(gamma) : -1;
  const int kp = phi && gphi ? armed_index(phi) : -1;
  if (kg >= 0) g_armed.g[kg] = ggamma;
  if (kp >= 0) g_armed.g[kp] = gphi;
}

bool adam_attach(hipStream_t s, int nseg, const float* const* alpha, const int64_t* len,
                 AdamRef* refs, FinTable& ft, AdamConst* ac) {
  if (!g_armed.on || g_armed.s != s || g_armed.consumed || nseg > kMaxAdamSegs) return false;
  bool covered[kMaxArmed] = {};
  int seg_k[kMaxAdamSegs];
  for (int i = 0; i < nseg; ++i) {
    const int k = armed_index(alpha[i]);
    seg_k[i] = k;
    if (k >= 0 && g_armed.len[k] == len[i]) covered[k] = true;
    else seg_k[i] = -1;
  }
  int ride_k[kMaxFin][2];
  for (int t = 0; t < ft.n; ++t) {
    ride_k[t][0] = ride_k[t][1] = -1;
    if (ft.t[t].kind != 1) continue;
    for (int j = 0; j < 2; ++j) {
      const float* gout = ft.t[t].o[j];
      for (int k = 0; k < g_armed.n && gout; ++k)
        if (g_armed.g[k] == gout) {
          ride_k[t][j] = k;
          covered[k] = true;
        }
    }
  }
  int extra[kMaxArmed], ne = 0;
  for (int k = 0; k < g_armed.n; ++k) {
    if (covered[k]) continue;
    if (!g_armed.g[k] || g_armed.len[k] > (int64_t)kMaxRideAdam) return false;
    extra[ne++] = k;
  }
  if (ft.n + ne > kMaxFin) return false;
  // every armed parameter is covered: attach
  for (int i = 0; i < nseg; ++i) {
    const int k = seg_k[i];
    refs[i] = k >= 0 ? AdamRef{g_armed.p[k], g_armed.m[k], g_armed.v[k]} : AdamRef{};
  }
  for (int t = 0; t < ft.n; ++t)
    for (int j = 0; j < 2; ++j) {
      const int k = ft.t[t].kind == 1 ? ride_k[t][j] : -1;
      ft.t[t].ad[j] = k >= 0 ? AdamRef{g_armed.p[k], g_armed.m[k], g_armed.v[k]} : AdamRef{};
    }
  for (int e = 0; e < ne; ++e) {
    const int k = extra[e];
    FinTask t{};
    t.kind = 3;
    t.nwg = 1;
    t.a = (uint32_t)g_armed.len[k];
    t.o[0] = (float*)g_armed.g[k];
    t.ad[0] = AdamRef{g_armed.p[k], g_armed.m[k], g_armed.v[k]};
    ft.t[ft.n++] = t;
    ft.nwg += 1;
  }
  ft.ac = g_armed.c;
  *ac = g_armed.c;
  g_armed.consumed = true;
  return true;
}

// A host launch about to write [w0, w0 + wn): tasks that read it are launched standalone
// first; the rest are handed to the host.
static FinTable fin_take_for_host(hipStream_t s, const void* w0, size_t wn, int* rc) {
  *rc = SSQ_OK;
  for (int i = 0; i < g_fin_npending; ++i) {
    const PendingFin& pf = g_fin_pending[i];
    if (pf.s != s || !w0) continue;
    const char* a = (const char*)pf.t.part;
    if (a >= (const char*)w0 && a < (const char*)w0 + wn) {
      *rc = fin_flush(s);
      FinTable none{};
      none.n = 0;
      none.nwg = 0;
      return none;
    }
  }
  return fin_take(s);
}

}  // namespace ssq

using namespace ssq;

extern "C" size_t ssq_lp_loss_workspace_size(int64_t n) {
  (void)n;
  return kLossBlocks * sizeof(double);
}

static int lp_loss(const char* what, const float* pred, const float* tgt, const int64_t* idx,
                   int64_t row, int64_t n, int64_t M, float p, float* loss_out, float* grad,
                   const float* gscale, int relu_mask, void* ws, size_t ws_bytes, hipStream_t s) {
  SSQ_REQUIRE(pred && tgt && n >= 1 && M >= 1 && (loss_out || grad), SSQ_E_ARG, "%s: bad args",
              what);
  SSQ_REQUIRE(!loss_out || (ws && ws_bytes >= ssq_lp_loss_workspace_size(n)), SSQ_E_WS,
              "%s: workspace too small", what);
  const bool gather = idx != nullptr;
  SSQ_REQUIRE(!gather || (row >= 1 && n % row == 0 && n < (1ll << 31)), SSQ_E_ARG,
              "%s: n must be a whole number of target rows (< 2^31 elements)", what);
  {  // a queued loss task reads the workspace this launch is about to overwrite
    const int rc = fin_flush(s);
    if (rc) return rc;
  }
  const int grid = grid_for(n, kBlock * 4, kLossBlocks);
  const float inv_m = 1.0f / (float)M;  // mean backward: 1.0 / numel in fp32
  double* part = loss_out ? (double*)ws : nullptr;
  int vec = ((((uintptr_t)pred) | ((uintptr_t)tgt) | ((uintptr_t)grad)) & 15) == 0;
  if (gather && row % 4 != 0) vec = 0;  // float4s must not straddle target rows
  TgtRows tr4{idx, 1, make_fastdiv(1)}, tr1 = tr4;
  if (gather) {
    tr1 = TgtRows{idx, (uint32_t)row, make_fastdiv((uint32_t)row)};
    if (vec) tr4 = TgtRows{idx, (uint32_t)(row / 4), make_fastdiv((uint32_t)(row / 4))};
  }
  auto k = gather ? (p == 2.0f ? lp_loss_kernel<0, true>
                               : (p == 1.0f ? lp_loss_kernel<1, true> : lp_loss_kernel<2, true>))
                  : (p == 2.0f ? lp_loss_kernel<0, false>
                               : (p == 1.0f ? lp_loss_kernel<1, false> : lp_loss_kernel<2, false>));
  hipLaunchKernelGGL(k, dim3(grid), dim3(kBlock), 0, s, pred, tgt, n, p, inv_m, grad, gscale,
                     relu_mask, vec, tr4, tr1, part);
  if (loss_out) {
    if (fin_defer_on()) {
      FinTask t{};
      t.kind = 0;
      t.nwg = 1;
      t.part = part;
      t.a = (uint32_t)grid;
      t.m = (double)M;
      t.o[0] = loss_out;
      const int rc = check_launch(what);
      return rc ? rc : fin_push(s, t);
    }
    hipLaunchKernelGGL(lp_loss_finalize, dim3(1), dim3(kBlock), 0, s, (const double*)part, grid,
                       (double)M, loss_out);
  }
  return check_launch(what);
}

extern "C" int ssq_lp_loss(const float* pred, const float* tgt, int64_t n, int64_t M, float p,
                           float* loss_out, float* grad, const float* gscale, int relu_mask,
                           void* ws, size_t ws_bytes, ssq_stream_t stream) {
  return lp_loss("ssq_lp_loss", pred, tgt, nullptr, 0, n, M, p, loss_out, grad, gscale,
                 relu_mask, ws, ws_bytes, (hipStream_t)stream);
}

extern "C" int ssq_lp_loss_rows(const float* pred, const float* tgt_cache, const int64_t* idx,
                                int64_t row, int64_t n, int64_t M, float p, float* loss_out,
                                float* grad, const float* gscale, int relu_mask, void* ws,
                                size_t ws_bytes, ssq_stream_t stream) {
  SSQ_REQUIRE(idx, SSQ_E_ARG, "ssq_lp_loss_rows: idx is required");
  return lp_loss("ssq_lp_loss_rows", pred, tgt_cache, idx, row, n, M, p, loss_out, grad, gscale,
                 relu_mask, ws, ws_bytes, (hipStream_t)stream);
}

static int gather_rows2(const float* src0, float* dst0, int64_t row0, const float* src1,
                        float* dst1, int64_t row1, const int64_t* idx, int64_t nidx,
                        int64_t* stage_dst, int64_t stage_n, hipStream_t stream) {
  SSQ_REQUIRE(src0 && dst0 && idx && row0 >= 1 && nidx >= 1, SSQ_E_ARG,
              "ssq_gather_rows2: bad args");
  SSQ_REQUIRE(!src1 || (dst1 && row1 >= 1), SSQ_E_ARG, "ssq_gather_rows2: bad second source");
  SSQ_REQUIRE(nidx <= 65535, SSQ_E_ARG, "ssq_gather_rows2: at most 65535 rows per call");
  auto al = [](const void* q) { return ((uintptr_t)q & 15u) == 0; };
  const bool vec = row0 % 4 == 0 && al(src0) && al(dst0) &&
                   (!src1 || (row1 % 4 == 0 && al(src1) && al(dst1)));
  const int64_t per = (row0 > row1 ? row0 : row1) / (vec ? 4 : 1);
  int64_t gx = 2048 / nidx;  // ~8 workgroups per CU in all
  const int64_t need = (per + kBlock - 1) / kBlock;
  if (gx > need) gx = need;
  if (gx < 1) gx = 1;
  GatherArgs a{src0, dst0, row0, src1, dst1, row1, idx, (uint32_t)gx, (uint32_t)nidx,
               stage_dst, (uint32_t)stage_n};
  const int rc = launch_gather(stream, a, vec);
  if (rc) return rc;
  return check_launch("ssq_gather_rows2");
}

extern "C" int ssq_gather_rows2(const float* src0, float* dst0, int64_t row0, const float* src1,
                                float* dst1, int64_t row1, const int64_t* idx, int64_t nidx,
                                ssq_stream_t stream) {
  return gather_rows2(src0, dst0, row0, src1, dst1, row1, idx, nidx, nullptr, 0,
                      (hipStream_t)stream);
}

extern "C" int ssq_gather_rows2_staged(const float* src0, float* dst0, int64_t row0,
                                       const float* src1, float* dst1, int64_t row1,
                                       const int64_t* slot, int64_t nidx, int64_t* stage_dst,
                                       int64_t stage_words, ssq_stream_t stream) {
  SSQ_REQUIRE(slot && stage_dst && stage_words >= nidx && stage_words <= 65536, SSQ_E_ARG,
              "ssq_gather_rows2_staged: the slot holds the nidx indices first, <= 65536 words");
  SSQ_REQUIRE(stage_dst + stage_words <= slot || slot + stage_words <= stage_dst, SSQ_E_ARG,
              "ssq_gather_rows2_staged: slot and stage_dst overlap");
  return gather_rows2(src0, dst0, row0, src1, dst1, row1, slot, nidx, stage_dst, stage_words,
                      (hipStream_t)stream);
}

// A/B knob SSQ_EPI_MULTI_ROW: 4 rows per wave on small planes for the epilogue backward
// (1, the default), also for its fused-tail form (2), or never (0)
static bool epi_g16() {
  static const bool on = [] {
    const char* e = getenv("SSQ_EPI_G16");
    return !(e && *e && atoi(e) == 0);
  }();
  return on;
}

static int epi_multi_row() {
  static const int mode = [] {
    const char* e = getenv("SSQ_EPI_MULTI_ROW");
    return e && *e ? atoi(e) : 1;
  }();
  return mode;
}

static int bias_act(const char* what, const float* y, const float* bias, const float* res,
                    float* out, float* yq, int64_t n, int64_t hw, int64_t C, int relu,
                    const float* qdelta, const float* qzp, int qmin, int qmax, hipStream_t s,
                    const float* gamma = nullptr, const float* phi = nullptr,
                    const int64_t* yrows = nullptr, const int64_t* rrows = nullptr,
                    const int64_t* stage_src = nullptr, int64_t* stage_dst = nullptr,
                    int64_t stage_n = 0) {
  SSQ_REQUIRE(!gamma == !phi, SSQ_E_ARG, "%s: gamma and phi go together", what);
  SSQ_REQUIRE(y && n >= 0 && hw >= 1 && C >= 1, SSQ_E_ARG, "%s: bad args", what);
  SSQ_REQUIRE(yq ? (qdelta && qzp && qmin < qmax) : out != nullptr, SSQ_E_ARG, "%s: bad outputs",
              what);
  SSQ_REQUIRE(n < (1ll << 31) && hw < (1ll << 31) && C < (1ll << 31), SSQ_E_ARG,
              "%s: tensor exceeds 2^31 elements", what);
  if (n == 0 && !stage_dst) return SSQ_OK;
  auto al = [](const void* q) { return ((uintptr_t)q & 15u) == 0; };
  SSQ_REQUIRE((!yrows && !rrows) || n % (hw * C) == 0, SSQ_E_ARG,
              "%s: row maps need whole [C, hw] samples", what);
  SSQ_REQUIRE(!rrows || res, SSQ_E_ARG, "%s: res_rows without res", what);
  SSQ_REQUIRE(!stage_dst || (stage_src && stage_n > 0 && stage_n <= 4096), SSQ_E_ARG,
              "%s: staging needs a source and 1..4096 words", what);
  // vec 2: float4s that never straddle an (n, c) plane (SSQ_K13_PLANE4=0: the per-element
  // channel form, for A/B)
  static const bool kPlane4 = !getenv("SSQ_K13_PLANE4") || atoi(getenv("SSQ_K13_PLANE4")) != 0;
  int vec = n % 4 == 0 && al(y) && (!out || al(out)) && (!res || al(res)) &&
            (!yq || al(yq)) && ((!yrows && !rrows) || hw % 4 == 0);
  if (vec && hw % 4 == 0 && kPlane4) vec = 2;
  const FastDiv dh = make_fastdiv((uint32_t)hw), dc = make_fastdiv((uint32_t)C);
  const dim3 grid(grid_for(vec ? n / 4 : n, kBlock, 2048));
  const float lo = (float)qmin, hi = (float)qmax;
#define SSQ_BA(R, A, Q, F)                                                                    \
  hipLaunchKernelGGL((bias_act_kernel<R, A, Q, F>), grid, dim3(kBlock), 0, s, y, bias, res, out, \
                     (uint32_t)n, dh, dc, (uint32_t)C, vec, yq, qdelta, qzp, lo, hi, gamma, phi, \
                     yrows, rrows, (uint32_t)(C * hw), stage_src, stage_dst, (uint32_t)stage_n)
#define SSQ_BA1(R, A, Q) \
  if (gamma) SSQ_BA(R, A, Q, true); else SSQ_BA(R, A, Q, false);
#define SSQ_BA2(R, A) \
  if (yq) { SSQ_BA1(R, A, true) } else { SSQ_BA1(R, A, false) }
  SSQ_REQUIRE(relu >= 0 && relu <= 2, SSQ_E_ARG, "%s: activation code %d (0/1/2)", what, relu);
  if (res) {
    if (relu == 2) { SSQ_BA2(true, 2) } else if (relu) { SSQ_BA2(true, 1) } else { SSQ_BA2(true, 0) }
  } else {
    if (relu == 2) { SSQ_BA2(false, 2) } else if (relu) { SSQ_BA2(false, 1) } else { SSQ_BA2(false, 0) }
  }
#undef SSQ_BA2
#undef SSQ_BA1
#undef SSQ_BA
  return check_launch(what);
}

extern "C" int ssq_bias_act(const float* y, const float* bias, const float* res, float* out,
                            int64_t n, int64_t hw, int64_t C, int relu, ssq_stream_t stream) {
  return bias_act("ssq_bias_act", y, bias, res, out, nullptr, n, hw, C, relu, nullptr, nullptr,
                  0, 1, (hipStream_t)stream);
}

extern "C" int ssq_bias_act_fq(const float* y, const float* bias, const float* res, float* out,
                               float* yq, int64_t n, int64_t hw, int64_t C, int relu,
                               const float* delta, const float* zp, int qmin, int qmax,
                               ssq_stream_t stream) {
  SSQ_REQUIRE(yq, SSQ_E_ARG, "ssq_bias_act_fq: yq is required");
  return bias_act("ssq_bias_act_fq", y, bias, res, out, yq, n, hw, C, relu, delta, zp, qmin, qmax,
                  (hipStream_t)stream);
}

extern "C" int ssq_epilogue_fwd(const float* y, const float* bias, const float* gamma,
                                const float* phi, const float* res, float* out, float* yq,
                                int64_t n, int64_t hw, int64_t C, int relu, const float* delta,
                                const float* zp, int qmin, int qmax, ssq_stream_t stream) {
  return bias_act("ssq_epilogue_fwd", y, bias, res, out, yq, n, hw, C, relu, delta, zp, qmin,
                  qmax, (hipStream_t)stream, gamma, phi);
}

extern "C" int ssq_epilogue_fwd_rows(const float* y, const int64_t* y_rows, const float* bias,
                                     const float* gamma, const float* phi, const float* res,
                                     const int64_t* res_rows, float* out, float* yq, int64_t n,
                                     int64_t hw, int64_t C, int relu, const float* delta,
                                     const float* zp, int qmin, int qmax,
                                     const int64_t* stage_src, int64_t* stage_dst,
                                     int64_t stage_n, ssq_stream_t stream) {
  return bias_act("ssq_epilogue_fwd_rows", y, bias, res, out, yq, n, hw, C, relu, delta, zp,
                  qmin, qmax, (hipStream_t)stream, gamma, phi, y_rows, res_rows, stage_src,
                  stage_dst, stage_n);
}

extern "C" size_t ssq_epilogue_bwd_workspace_size(int64_t rows) {
  // the rows' records, then (fused tail) one loss partial per workgroup: <= ceil(rows / 4),
  // then the delta reduction's workgroup partials and its counter (fin_epi)
  return (delta_ticket_offset((size_t)rows) + 1) * sizeof(double);
}

// ssq_epilogue_bwd (g = dL/d(output)) and its fused-tail form ssq_epilogue_loss_bwd
// (tgt = the cache of target rows, idx = this batch's rows: dL/d(output) of the lp_loss
// (power lp) computed in the pass, its value finalised into loss_out).
static int epilogue_bwd(const char* what, const float* g, const float* y, const float* bias,
                        const float* gamma, const float* phi, const float* res, const ResEpi& re,
                        int64_t N, int64_t C, int64_t hw, int relu, const float* delta,
                        const float* zp, int qmin, int qmax, const int64_t* lidx, int64_t M,
                        float lp, float* loss_out, float* gy, float* gres, float* ggamma,
                        float* gphi, float* grgamma, float* grphi, float* gdelta, float* gzp,
                        void* ws, size_t ws_bytes, hipStream_t s,
                        const int64_t* yrows = nullptr, const int64_t* rrows = nullptr) {
  const bool loss = lidx != nullptr;
  // the residual's own epilogue folded in (fused tail only)
  const bool res2 = res && (re.bias || re.gamma);
  SSQ_REQUIRE(!re.gamma == !re.phi && (!(grgamma || grphi) || re.gamma), SSQ_E_ARG,
              "%s: residual gamma/phi go together (and their gradients need them)", what);
  SSQ_REQUIRE(!(re.bias || re.gamma) || (res && loss && relu <= 1), SSQ_E_ARG,
              "%s: a residual epilogue needs the residual, the fused loss and ReLU / identity",
              what);
  // gy may be null: dL/dy not wanted (the conv's weight and input are frozen, e.g. the first
  // conv of a block in BRECQ's act phase) -- only the per-row sums are produced
  SSQ_REQUIRE(g && y && N >= 1 && C >= 1 && hw >= 1, SSQ_E_ARG, "%s: bad args", what);
  SSQ_REQUIRE(!loss || (loss_out && M >= 1), SSQ_E_ARG, "%s: loss_out and M required", what);
  SSQ_REQUIRE(!loss || lp > 0.0f, SSQ_E_ARG, "%s: loss power p must be > 0", what);
  const bool lp2 = lp == 2.0f;
  SSQ_REQUIRE(!gamma == !phi && (!(ggamma || gphi) || gamma), SSQ_E_ARG,
              "%s: gamma/phi gradients need gamma and phi", what);
  SSQ_REQUIRE(!delta || (zp && qmin < qmax), SSQ_E_ARG, "%s: act quantizer", what);
  SSQ_REQUIRE(!(gdelta || gzp) || delta, SSQ_E_ARG, "%s: delta/zp grads need delta", what);
  SSQ_REQUIRE(N * C * hw < (1ll << 31) && N * C < (1ll << 31), SSQ_E_ARG,
              "%s: tensor exceeds 2^31 elements", what);
  const int64_t rows = N * C;
  SSQ_REQUIRE(ws && ws_bytes >= ssq_epilogue_bwd_workspace_size(rows), SSQ_E_WS,
              "%s: workspace too small", what);
  auto al = [](const void* q) { return ((uintptr_t)q & 15u) == 0; };
  const bool vec = hw % 4 == 0 && al(g) && al(y) && (!gy || al(gy)) && (!res || al(res)) &&
                   (!gres || al(gres));
  SSQ_REQUIRE(relu >= 0 && relu <= 2, SSQ_E_ARG, "%s: activation code %d", what, relu);
  // small planes (<= 64 elements or float4s per row): 4 rows per wave (same bits); not with
  // the act quantizer's four extra sums per row (3-4 waves per SIMD instead of 7-8)
  // rows of <= 64 elements or float4s: 4 rows per wave, 16 lanes each (kG16; every variant,
  // the same form for the plain backward and the fused tail); SSQ_EPI_G16=0 for A/B: the r4
  // forms (4 rows per wave with a lane per element where the registers allow, else a row
  // per wave)
  const bool small = (vec ? hw / 4 : hw) <= kWave;
  const bool g16 = small && epi_g16();
  const bool multi = !g16 && small && !delta && !res2 && epi_multi_row() >= (loss ? 2 : 1);
  const int64_t rpw = (g16 || multi) ? 4 : 1;
  const int64_t waves = (rows + rpw - 1) / rpw;
  const uint32_t nmain = (uint32_t)((waves + kBlock / kWave - 1) / (kBlock / kWave));
  int frc = SSQ_OK;
  const FinTable fin = fin_take_for_host(s, ws, ws_bytes, &frc);
  if (frc) return frc;
  const dim3 grid(nmain + fin.nwg);
  const float lo = (float)qmin, hi = (float)qmax;
  const float inv_m = loss ? 1.0f / (float)M : 0.0f;   // mean backward, as lp_loss
  double* part = (double*)ws;
#define SSQ_EB0(R, A, Q, F, V, L, P)                                                              \
  hipLaunchKernelGGL((epilogue_bwd_rows<R, A, Q, F, V, L, P>), grid, dim3(kBlock), 0, s, g, y,    \
                     bias, gamma, phi, res, (uint32_t)rows, (uint32_t)C, (uint32_t)hw, delta, zp, \
                     lo, hi, gy, gres, part, fin, nmain, lidx, inv_m, lp, re2, yrows, rrows)
#define SSQ_EB(R, A, Q, F, V, L) \
  if (g16) SSQ_EB0(R, A, Q, F, V, L, kG16); \
  else if (multi) SSQ_EB0(R, A, Q, F, V, L, ((Q) ? 1 : 4)); else SSQ_EB0(R, A, Q, F, V, L, 1);
#define SSQ_EBL(R, A, Q, F, V) \
  if (lp2) { SSQ_EB(R, A, Q, F, V, 1) } else { SSQ_EB(R, A, Q, F, V, 2) }
#define SSQ_EB1(R, A, Q, F) \
  if (loss) { if (vec) { SSQ_EBL(R, A, Q, F, true) } else { SSQ_EBL(R, A, Q, F, false) } } \
  else if (vec) { SSQ_EB(R, A, Q, F, true, 0) } else { SSQ_EB(R, A, Q, F, false, 0) }
#define SSQ_EB2(R, A, Q) \
  if (gamma) { SSQ_EB1(R, A, Q, true) } else { SSQ_EB1(R, A, Q, false) }
#define SSQ_EB3(R, A) \
  if (delta) { SSQ_EB2(R, A, true) } else { SSQ_EB2(R, A, false) }
// RES 2: the fused tail only, ReLU / identity, one row per wave
#define SSQ_EBLR(A, Q, F, V) \
  if (g16) { if (lp2) { SSQ_EB0(2, A, Q, F, V, 1, kG16); } else { SSQ_EB0(2, A, Q, F, V, 2, kG16); } } \
  else if (lp2) { SSQ_EB0(2, A, Q, F, V, 1, 1); } else { SSQ_EB0(2, A, Q, F, V, 2, 1); }
#define SSQ_EBR1(A, Q, F) \
  if (vec) { SSQ_EBLR(A, Q, F, true) } else { SSQ_EBLR(A, Q, F, false) }
#define SSQ_EBR2(A, Q) \
  if (gamma) { SSQ_EBR1(A, Q, true) } else { SSQ_EBR1(A, Q, false) }
#define SSQ_EBR3(A) \
  if (delta) { SSQ_EBR2(A, true) } else { SSQ_EBR2(A, false) }
  const ResEpi re2 = res2 ? re : ResEpi{nullptr, nullptr, nullptr};
  if (res2) {
    if (relu) { SSQ_EBR3(1) } else { SSQ_EBR3(0) }
  } else if (res) {
    if (relu == 2) { SSQ_EB3(true, 2) } else if (relu) { SSQ_EB3(true, 1) } else { SSQ_EB3(true, 0) }
  } else {
    if (relu == 2) { SSQ_EB3(false, 2) } else if (relu) { SSQ_EB3(false, 1) } else { SSQ_EB3(false, 0) }
  }
#undef SSQ_EBR3
#undef SSQ_EBR2
#undef SSQ_EBR1
#undef SSQ_EBLR
#undef SSQ_EB3
#undef SSQ_EB2
#undef SSQ_EB1
#undef SSQ_EBL
#undef SSQ_EB
#undef SSQ_EB0
  int rc = check_launch(what);
  if (rc) return rc;
  if (loss) {
    FinTask t{};
    t.kind = 2;
    t.nwg = 1;
    t.part = part + (size_t)rows * kEpiParts;   // the launch's workgroup partials
    t.a = nmain;
    t.m = (double)M;
    t.o[0] = loss_out;
    if (fin_defer_on()) {
      rc = fin_push(s, t);
    } else {
      FinTable one{};
      one.t[0] = t;
      one.n = 1;
      one.nwg = 1;
      hipLaunchKernelGGL(fin_tasks_kernel, dim3(1), dim3(kBlock), 0, s, one);
      rc = check_launch(what);
    }
    if (rc) return rc;
  }
  adam_log(s, gamma, phi, ggamma, gphi);
  if (res2 && (grgamma || grphi)) {
    // the residual epilogue's gamma / phi: its own finalize task over slots 7 / 8
    adam_log(s, re.gamma, re.phi, grgamma, grphi);
    FinTask t{};
    t.kind = 1;
    t.nwg = (unsigned)((C + kEpiChan - 1) / kEpiChan);
    t.part = part;
    t.a = (uint32_t)N;
    t.b = (uint32_t)C;
    t.c = t.nwg;
    t.s0 = 7;
    t.o[0] = grgamma;
    t.o[1] = grphi;
    if (fin_defer_on()) {
      rc = fin_push(s, t);
    } else {
      FinTable one{};
      one.t[0] = t;
      one.n = 1;
      one.nwg = t.nwg;
      hipLaunchKernelGGL(fin_tasks_kernel, dim3(one.nwg), dim3(kBlock), 0, s, one);
      rc = check_launch(what);
    }
    if (rc) return rc;
  }
  if (ggamma || gphi || gdelta || gzp) {
    // blocks [0, nb) only when gamma / phi are wanted; blocks [nb, nb + nq) (the act
    // quantizer's four sums over every row, kDeltaRows rows per workgroup) only when delta /
    // zp are
    const unsigned nb = (ggamma || gphi) ? (unsigned)((C + kEpiChan - 1) / kEpiChan) : 0u;
    const unsigned nq = (gdelta || gzp) ? delta_wgs((uint32_t)rows) : 0u;
    if (fin_defer_on()) {
      FinTask t{};
      t.kind = 1;
      t.nwg = nb + nq;
      t.part = part;
      t.a = (uint32_t)N;
      t.b = (uint32_t)C;
      t.c = nb;
      t.o[0] = ggamma;
      t.o[1] = gphi;
      t.o[2] = gdelta;
      t.o[3] = gzp;
      return fin_push(s, t);
    }
    hipLaunchKernelGGL(epilogue_bwd_finalize, dim3(nb + nq), dim3(kBlock), 0, s,
                       (const double*)part, (uint32_t)N, (uint32_t)C, nb, ggamma, gphi, gdelta,
                       gzp);
  }
  return check_launch(what);
}

extern "C" int ssq_epilogue_bwd(const float* g, const float* y, const float* bias,
                                const float* gamma, const float* phi, const float* res,
                                int64_t N, int64_t C, int64_t hw, int relu, const float* delta,
                                const float* zp, int qmin, int qmax, float* gy, float* gres,
                                float* ggamma, float* gphi, float* gdelta, float* gzp, void* ws,
                                size_t ws_bytes, ssq_stream_t stream) {
  return epilogue_bwd("ssq_epilogue_bwd", g, y, bias, gamma, phi, res,
                      ResEpi{nullptr, nullptr, nullptr}, N, C, hw, relu, delta, zp, qmin, qmax,
                      nullptr, 0, 2.0f, nullptr, gy, gres, ggamma, gphi, nullptr, nullptr, gdelta,
                      gzp, ws, ws_bytes, (hipStream_t)stream);
}

extern "C" int ssq_epilogue_loss_bwd(const float* tgt_cache, const int64_t* idx, int64_t M,
                                     float p, float* loss_out, const float* y, const float* bias,
                                     const float* gamma, const float* phi, const float* res,
                                     const float* res_bias, const float* res_gamma,
                                     const float* res_phi, int64_t N, int64_t C, int64_t hw,
                                     int relu, const float* delta, const float* zp, int qmin,
                                     int qmax, float* gy, float* gres, float* ggamma, float* gphi,
                                     float* gres_gamma, float* gres_phi, float* gdelta,
                                     float* gzp, void* ws, size_t ws_bytes, ssq_stream_t stream) {
  SSQ_REQUIRE(idx, SSQ_E_ARG, "ssq_epilogue_loss_bwd: idx is required");
  return epilogue_bwd("ssq_epilogue_loss_bwd", tgt_cache, y, bias, gamma, phi, res,
                      ResEpi{res_bias, res_gamma, res_phi}, N, C, hw, relu, delta, zp, qmin, qmax,
                      idx, M, p, loss_out, gy, gres, ggamma, gphi, gres_gamma, gres_phi, gdelta,
                      gzp, ws, ws_bytes, (hipStream_t)stream);
}

// the two above with y and / or res read in place from per-sample row caches (y_rows /
// res_rows: this batch's rows of y / res; either may be null = y / res are the batch itself)
extern "C" int ssq_epilogue_bwd_rows(const float* g, const float* y, const int64_t* y_rows,
                                     const float* bias, const float* gamma, const float* phi,
                                     const float* res, const int64_t* res_rows, int64_t N,
                                     int64_t C, int64_t hw, int relu, const float* delta,
                                     const float* zp, int qmin, int qmax, float* gy, float* gres,
                                     float* ggamma, float* gphi, float* gdelta, float* gzp,
                                     void* ws, size_t ws_bytes, ssq_stream_t stream) {
  SSQ_REQUIRE(!res_rows || res, SSQ_E_ARG, "ssq_epilogue_bwd_rows: res_rows without res");
  return epilogue_bwd("ssq_epilogue_bwd_rows", g, y, bias, gamma, phi, res,
                      ResEpi{nullptr, nullptr, nullptr}, N, C, hw, relu, delta, zp, qmin, qmax,
                      nullptr, 0, 2.0f, nullptr, gy, gres, ggamma, gphi, nullptr, nullptr, gdelta,
                      gzp, ws, ws_bytes, (hipStream_t)stream, y_rows, res_rows);
}

extern "C" int ssq_epilogue_loss_bwd_rows(
    const float* tgt_cache, const int64_t* idx, int64_t M, float p, float* loss_out,
    const float* y, const int64_t* y_rows, const float* bias, const float* gamma,
    const float* phi, const float* res, const int64_t* res_rows, const float* res_bias,
    const float* res_gamma, const float* res_phi, int64_t N, int64_t C, int64_t hw, int relu,
    const float* delta, const float* zp, int qmin, int qmax, float* gy, float* gres,
    float* ggamma, float* gphi, float* gres_gamma, float* gres_phi, float* gdelta, float* gzp,
    void* ws, size_t ws_bytes, ssq_stream_t stream) {
  SSQ_REQUIRE(idx, SSQ_E_ARG, "ssq_epilogue_loss_bwd_rows: idx is required");
  SSQ_REQUIRE(!res_rows || res, SSQ_E_ARG, "ssq_epilogue_loss_bwd_rows: res_rows without res");
  return epilogue_bwd("ssq_epilogue_loss_bwd_rows", tgt_cache, y, bias, gamma, phi, res,
                      ResEpi{res_bias, res_gamma, res_phi}, N, C, hw, relu, delta, zp, qmin, qmax,
                      idx, M, p, loss_out, gy, gres, ggamma, gphi, gres_gamma, gres_phi, gdelta,
                      gzp, ws, ws_bytes, (hipStream_t)stream, y_rows, res_rows);
}

template <int ACT>
static int act_bwd(const char* what, const float* g, const float* out, float* gin, int64_t n,
                   hipStream_t s) {
  SSQ_REQUIRE(g && out && gin && n >= 0 && n < (1ll << 31), SSQ_E_ARG, "%s: bad args", what);
  if (n == 0) return SSQ_OK;
  auto al = [](const void* q) { return ((uintptr_t)q & 15u) == 0; };
  const bool vec = al(g) && al(out) && al(gin);
  const int64_t n4 = vec ? n / 4 : 0;
  if (n4 > 0)
    hipLaunchKernelGGL(relu_bwd_kernel<ACT>, dim3(grid_for(n4, kBlock, 2048)), dim3(kBlock), 0, s,
                       (const f32x4*)g, (const f32x4*)out, (f32x4*)gin, (uint32_t)n4);
  const int64_t start = n4 * 4;
  if (start < n)
    hipLaunchKernelGGL(relu_bwd_tail<ACT>, dim3((unsigned)((n - start + kBlock - 1) / kBlock)),
                       dim3(kBlock), 0, s, g, out, gin, (uint32_t)start, (uint32_t)n);
  return check_launch(what);
}

extern "C" int ssq_relu_bwd(const float* g, const float* out, float* gin, int64_t n,
                            ssq_stream_t stream) {
  return act_bwd<1>("ssq_relu_bwd", g, out, gin, n, (hipStream_t)stream);
}

extern "C" int ssq_relu6_bwd(const float* g, const float* out, float* gin, int64_t n,
                             ssq_stream_t stream) {
  return act_bwd<2>("ssq_relu6_bwd", g, out, gin, n, (hipStream_t)stream);
}

extern "C" int ssq_adam_arm(int nseg, float* const* p, float* const* m, float* const* v,
                            const int64_t* n, float one_minus_beta1, float beta2,
                            float one_minus_beta2, float eps, const float* hyper,
                            ssq_stream_t stream) {
  SSQ_REQUIRE(nseg >= 1 && nseg <= kMaxArmed && p && m && v && n && hyper, SSQ_E_ARG,
              "ssq_adam_arm: 1 <= nseg <= %d, non-null arrays and device hyper required",
              kMaxArmed);
  ArmedAdam a{};
  a.on = true;
  a.s = (hipStream_t)stream;
  a.n = nseg;
  for (int k = 0; k < nseg; ++k) {
    SSQ_REQUIRE(p[k] && m[k] && v[k] && n[k] >= 1, SSQ_E_ARG, "ssq_adam_arm: segment %d", k);
    a.p[k] = p[k];
    a.m[k] = m[k];
    a.v[k] = v[k];
    a.len[k] = n[k];
  }
  a.c = AdamConst{one_minus_beta1, beta2, one_minus_beta2, eps, hyper};
  g_armed = a;
  return SSQ_OK;
}

extern "C" int ssq_adam_take(ssq_stream_t stream) {
  const bool mine = g_armed.on && g_armed.s == (hipStream_t)stream;
  const int done = mine && g_armed.consumed ? 1 : 0;
  if (mine) g_armed = ArmedAdam{};
  return done;
}

// ssq_adam's update riding on the stream's pending finalize tasks (fin_tasks.h): every
// segment's step is attached where its gradient is finalised (a kind-1 task's gamma / phi /
// delta output) or, for a gradient some earlier launch finished, as a kind-3 task; the table
// is then launched as one kernel.  False (nothing launched, nothing taken) when a segment
// cannot ride: no device hyper, no pending task, a gradient too large for a kind-3 task, or
// a full table.
static bool adam_ride(hipStream_t s, int nseg, float* const* p, const float* const* g,
                      float* const* m, float* const* v, const int64_t* n, const AdamConst& c) {
  if (!c.hyper) return false;
  int npend = 0;
  for (int i = 0; i < g_fin_npending; ++i) npend += g_fin_pending[i].s == s;
  if (npend == 0 || npend > kMaxFin) return false;
  FinTable ft = fin_take(s);
  const int nt = ft.n;
  bool ok = true;
  for (int i = 0; i < nseg && ok; ++i) {
    const AdamRef r{p[i], m[i], v[i]};
    bool placed = false;
    for (int t = 0; t < nt && !placed; ++t) {
      FinTask& k = ft.t[t];
      if (k.kind != 1) continue;
      for (int j = 0; j < 4 && !placed && ok; ++j) {
        if (!k.o[j] || k.o[j] != g[i]) continue;
        if (j < 3 && (j < 2 ? n[i] == (int64_t)k.b : n[i] == 1)) {
          k.ad[j] = r;
          placed = true;
        } else {
          ok = false;
        }
      }
    }
    if (placed || !ok) continue;
    // a gradient none of the pending tasks writes: final already
    if (n[i] > (int64_t)kMaxRideAdam || ft.n >= kMaxFin) {
      ok = false;
      break;
    }
    FinTask t{};
    t.kind = 3;
    t.nwg = 1;
    t.a = (uint32_t)n[i];
    t.o[0] = (float*)g[i];
    t.ad[0] = r;
    ft.t[ft.n++] = t;
    ft.nwg += 1;
  }
  if (!ok) {
    // put the pending tasks back untouched (same order) for the plain path
    for (int t = 0; t < nt; ++t) {
      FinTask k = ft.t[t];
      k.ad[0] = k.ad[1] = k.ad[2] = AdamRef{};
      g_fin_pending[g_fin_npending++] = PendingFin{s, k};
    }
    return false;
  }
  ft.ac = c;
  hipLaunchKernelGGL(fin_tasks_kernel, dim3(ft.nwg), dim3(kBlock), 0, s, ft);
  return true;
}

extern "C" int ssq_adam(int nseg, float* const* p, const float* const* g, float* const* m,
                        float* const* v, const int64_t* n, float one_minus_beta1, float beta2,
                        float one_minus_beta2, float eps, const float* hyper, float neg_step_size,
                        float bias_correction2_sqrt, ssq_stream_t stream) {
  SSQ_REQUIRE(nseg >= 1 && p && g && m && v && n, SSQ_E_ARG, "ssq_adam: bad arrays");
  for (int i = 0; i < nseg; ++i)
    SSQ_REQUIRE(p[i] && g[i] && m[i] && v[i] && n[i] >= 1 && n[i] < (1ll << 31), SSQ_E_ARG,
                "ssq_adam: bad segment %d", i);
  if (adam_ride((hipStream_t)stream, nseg, p, g, m, v, n,
                AdamConst{one_minus_beta1, beta2, one_minus_beta2, eps, hyper}))
    return check_launch("ssq_adam (riding on the pending finalizes)");
  // queued finalizes: those that write a gradient read here (gamma / phi / delta) must land
  // before the update -- launched first, standalone; the others (e.g. the loss value) ride
  // on the update's first launch
  FinTable ride{};
  {
    bool disjoint = true;
    for (int t = 0; t < g_fin_npending && disjoint; ++t) {
      const PendingFin& pf = g_fin_pending[t];
      if (pf.s != (hipStream_t)stream) continue;
      for (int j = 0; j < 4; ++j) {
        if (!pf.t.o[j]) continue;
        // what the task writes: gamma / phi gradients (C floats) or one float
        const int64_t len = (pf.t.kind == 1 && j < 2) ? (int64_t)pf.t.b
                            : (pf.t.kind == 3 ? (int64_t)pf.t.a : 1);
        const float* lo = pf.t.o[j];
        for (int i = 0; i < nseg; ++i)
          if (lo < g[i] + n[i] && g[i] < lo + len) disjoint = false;
      }
    }
    int npend = 0;
    for (int t = 0; t < g_fin_npending; ++t) npend += g_fin_pending[t].s == (hipStream_t)stream;
    if (disjoint && npend <= kMaxFin) {
      ride = fin_take((hipStream_t)stream);
    } else {
      const int rc = fin_flush((hipStream_t)stream);
      if (rc) return rc;
    }
  }
  for (int base = 0; base < nseg; base += kMaxAdamSeg) {
    AdamTable tab;
    tab.nseg = nseg - base < kMaxAdamSeg ? nseg - base : kMaxAdamSeg;
    int64_t blk = 0;
    for (int k = 0; k < tab.nseg; ++k) {
      const int i = base + k;
      SSQ_REQUIRE(p[i] && g[i] && m[i] && v[i] && n[i] >= 1 && n[i] < (1ll << 31), SSQ_E_ARG,
                  "ssq_adam: bad segment %d", i);
      tab.s[k] = AdamSeg{p[i], g[i], m[i], v[i], (uint32_t)n[i], (uint32_t)blk};
      blk += (n[i] + kAdamTile - 1) / kAdamTile;
    }
    SSQ_REQUIRE(blk < (1ll << 31), SSQ_E_ARG, "ssq_adam: too many tiles");
    hipLaunchKernelGGL(adam_kernel, dim3((unsigned)(blk + ride.nwg)), dim3(kBlock), 0,
                       (hipStream_t)stream, tab, one_minus_beta1, beta2, one_minus_beta2, eps, hyper,
                       neg_step_size, bias_correction2_sqrt, ride);
    const int rc = check_launch("ssq_adam");
    if (rc) return rc;
    ride = FinTable{};
  }
  return SSQ_OK;
}

extern "C" int ssq_set_deferred_finalize(int on) {
  const int prev = g_fin_defer ? 1 : 0;
  g_fin_defer = on != 0;
  return prev;
}

extern "C" int ssq_flush_finalize(ssq_stream_t stream) {
  return fin_flush((hipStream_t)stream);
}

// ------------------------------------------------------------------ stem max-pool
// F.max_pool2d forward (NCHW fp32, kernel K x K <= 7 x 7, stride, zero-free padding, no
// dilation, floor mode): the ResNet stem's 3x3 / s2 / p1 pool that follows the stem's K13
// epilogue in validation (torch's kernel ran at 1.8 TB/s there).  One output per thread
// (2x2 / 3x3 windows: every tap loaded at once), the window walked row-major with torch's
// rule (a larger value or a NaN replaces the running max; ties keep the first), so the
// result is bit-identical to torch's.
// The stem's 3x3 / s2 / p1 pool with W and OW even: two adjacent outputs per thread, their
// 5 input columns per row read as one scalar (column 2*ow0 - 1) and two float2s (columns
// 2*ow0 .. 2*ow0 + 3): 9 loads for 2 outputs instead of 18; same taps, same order, same
// rule as maxpool2d_kernel.
__global__ __launch_bounds__(kBlock) void maxpool3s2_pair_kernel(
    const float* __restrict__ x, float* __restrict__ y, uint32_t total2, uint32_t H, uint32_t W,
    uint32_t OH, uint32_t OW, FastDiv dOW2, FastDiv dOH) {
  typedef float f32x2v __attribute__((ext_vector_type(2)));
  const uint32_t OW2 = OW / 2, stride = gridDim.x * blockDim.x;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < total2; i += stride) {
    const uint32_t q1 = fdiv(i, dOW2), ow0 = 2 * (i - q1 * OW2);
    const uint32_t nc = fdiv(q1, dOH), oh = q1 - nc * OH;
    const float* __restrict__ xp = x + (size_t)nc * H * W;
    const int h0 = 2 * (int)oh - 1, c0 = 2 * (int)ow0;   // window columns c0-1 .. c0+3
    float v[3][5];
    bool rok[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      const int h = h0 + r;
      rok[r] = h >= 0 && h < (int)H;
      const float* row = xp + (size_t)min(max(h, 0), (int)H - 1) * W;
      v[r][0] = row[max(c0 - 1, 0)];
      const f32x2v a = *(const f32x2v*)(row + c0);
      v[r][1] = a.x;
      v[r][2] = a.y;
      const int c2 = min(c0 + 2, (int)W - 2);          // W even: c0 + 2 <= W - 2 unless edge
      const f32x2v b = *(const f32x2v*)(row + c2);
      v[r][3] = b.x;
      v[r][4] = b.y;
    }
    const bool left = c0 >= 1, right = c0 + 2 < (int)W;  // column c0-1 / c0+2 in the plane
    float m0 = -__builtin_inff(), m1 = -__builtin_inff();
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      if (!rok[r]) continue;
      // output ow0: columns c0-1, c0, c0+1 ; output ow0+1: columns c0+1, c0+2, c0+3
      if (left && (v[r][0] > m0 || __builtin_isnan(v[r][0]))) m0 = v[r][0];
      if (v[r][1] > m0 || __builtin_isnan(v[r][1])) m0 = v[r][1];
      if (v[r][2] > m0 || __builtin_isnan(v[r][2])) m0 = v[r][2];
      if (v[r][2] > m1 || __builtin_isnan(v[r][2])) m1 = v[r][2];
      if (right && (v[r][3] > m1 || __builtin_isnan(v[r][3]))) m1 = v[r][3];
      if (right && c0 + 3 < (int)W && (v[r][4] > m1 || __builtin_isnan(v[r][4]))) m1 = v[r][4];
    }
    *(f32x2v*)(y + (size_t)q1 * OW + ow0) = f32x2v{m0, m1};
  }
}

template <int KT>   // KT > 0: the window size at compile time (every load issued at once)
__global__ __launch_bounds__(kBlock) void maxpool2d_kernel(const float* __restrict__ x,
                                                           float* __restrict__ y, uint32_t total,
                                                           uint32_t H, uint32_t W, uint32_t OH,
                                                           uint32_t OW, uint32_t Kr, uint32_t st,
                                                           int pad, FastDiv dOW, FastDiv dOH) {
  const uint32_t K = KT > 0 ? (uint32_t)KT : Kr;
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    const uint32_t q1 = fdiv(i, dOW), ow = i - q1 * OW;
    const uint32_t nc = fdiv(q1, dOH), oh = q1 - nc * OH;
    const float* __restrict__ xp = x + (size_t)nc * H * W;
    const int h0 = (int)(oh * st) - pad, w0 = (int)(ow * st) - pad;
    float m = -__builtin_inff();
    if constexpr (KT > 0) {
      // in-range taps loaded (out-of-range ones read a clamped in-plane address and are
      // skipped), then the row-major max
      float v[KT * KT];
      bool ok[KT * KT];
#pragma unroll
      for (int r = 0; r < KT; ++r)
#pragma unroll
        for (int s2 = 0; s2 < KT; ++s2) {
          const int h = h0 + r, w = w0 + s2;
          ok[r * KT + s2] = h >= 0 && h < (int)H && w >= 0 && w < (int)W;
          const int hc = min(max(h, 0), (int)H - 1), wc = min(max(w, 0), (int)W - 1);
          v[r * KT + s2] = xp[(size_t)hc * W + wc];
        }
#pragma unroll
      for (int t = 0; t < KT * KT; ++t)
        if (ok[t] && (v[t] > m || __builtin_isnan(v[t]))) m = v[t];
    } else {
      for (uint32_t r = 0; r < K; ++r) {
        const int h = h0 + (int)r;
        if (h < 0 || h >= (int)H) continue;
        for (uint32_t s2 = 0; s2 < K; ++s2) {
          const int w = w0 + (int)s2;
          if (w < 0 || w >= (int)W) continue;
          const float v = xp[(size_t)h * W + w];
          if (v > m || __builtin_isnan(v)) m = v;
        }
      }
    }
    y[i] = m;
  }
}

// A/B knob SSQ_POOL_PAIR=0: the one-output-per-thread pool for the stem's shape too
static bool pair_pool() {
  static const bool on = [] {
    const char* e = getenv("SSQ_POOL_PAIR");
    return !(e && *e && atoi(e) == 0);
  }();
  return on;
}

extern "C" int ssq_maxpool2d_fwd(const float* x, float* y, int64_t N, int64_t C, int64_t H,
                                 int64_t W, int64_t K, int64_t stride, int64_t pad,
                                 ssq_stream_t s) {
  SSQ_REQUIRE(x && y, SSQ_E_ARG, "ssq_maxpool2d_fwd: null pointer");
  SSQ_REQUIRE(N >= 1 && C >= 1 && H >= 1 && W >= 1 && K >= 1 && K <= 7 && stride >= 1 &&
                  pad >= 0 && 2 * pad <= K, SSQ_E_ARG,
              "ssq_maxpool2d_fwd: bad geometry (K <= 7, pad <= K / 2)");
  const int64_t OH = (H + 2 * pad - K) / stride + 1, OW = (W + 2 * pad - K) / stride + 1;
  SSQ_REQUIRE(OH >= 1 && OW >= 1, SSQ_E_ARG, "ssq_maxpool2d_fwd: empty output");
  const int64_t total = N * C * OH * OW;
  SSQ_REQUIRE(total < (1ll << 31) && N * C * H * W < (1ll << 31), SSQ_E_ARG,
              "ssq_maxpool2d_fwd: tensor exceeds 2^31 elements");
  const bool al8 = ((uintptr_t)x & 7u) == 0 && ((uintptr_t)y & 7u) == 0;
  if (K == 3 && stride == 2 && pad == 1 && W % 2 == 0 && OW % 2 == 0 && al8 && pair_pool()) {
    const int64_t total2 = total / 2;
    hipLaunchKernelGGL(maxpool3s2_pair_kernel, dim3(grid_for(total2, kBlock, 8192)),
                       dim3(kBlock), 0, (hipStream_t)s, x, y, (uint32_t)total2, (uint32_t)H,
                       (uint32_t)W, (uint32_t)OH, (uint32_t)OW,
                       make_fastdiv((uint32_t)(OW / 2)), make_fastdiv((uint32_t)OH));
    return check_launch("ssq_maxpool2d_fwd");
  }
  const dim3 grid(grid_for(total, kBlock, 8192));
#define SSQ_MP(KT)                                                                         \
  hipLaunchKernelGGL(maxpool2d_kernel<KT>, grid, dim3(kBlock), 0, (hipStream_t)s, x, y,      \
                     (uint32_t)total, (uint32_t)H, (uint32_t)W, (uint32_t)OH, (uint32_t)OW, \
                     (uint32_t)K, (uint32_t)stride, (int)pad, make_fastdiv((uint32_t)OW),    \
                     make_fastdiv((uint32_t)OH))
  if (K == 3) SSQ_MP(3);
  else if (K == 2) SSQ_MP(2);
  else SSQ_MP(0);
#undef SSQ_MP
  return check_launch("ssq_maxpool2d_fwd");
}
