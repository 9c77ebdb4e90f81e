// K19: one BRECQ AdaRound iteration of a Linear layer in two launches.
//
// The end-to-end flow reconstructs the network's last layer (ResNet-18's fc, 512 -> 1000)
// with BRECQ's layer loop, 20000 iterations at batch 32 (layer_recon.py:10-104, called from
// main_imagenet.py for the fc).  Per iteration the reference gathers the batch
// (cached[randperm(N)[:32]]), runs the quantized layer (AdaRoundQuantizer soft rounding,
// adaptive_rounding.py:38-67, then F.linear), the loss (lp_loss p = 2 + the rounding
// regulariser, block_recon.py:119-182 / layer_recon.py:107-170), its backward and Adam.
// Each of those is microseconds of GPU work on this layer, so as separate launches the loop
// is bound by launch boundaries (r4: 9 launches, 45 us of GPU time per iteration).  Here:
//
//   fc_fwd_loss  (one workgroup per 32 output channels): the batch rows x[idx[r]] staged in
//     LDS, W^ = AdaRound(W, V) of the workgroup's rows computed on the fly into LDS (the
//     adaround_fwd_kernel ops), y = x W^T + bias (fp32 FMA, ci in order), the lp_loss p = 2
//     term and gradient of every output (lp_elem: the lp_loss_kernel ops) -> g = dL/dy and
//     one double loss partial per workgroup;
//   fc_bwd_adam  (one workgroup per 8 output channels): dW = g^T x (r in order), AdaRound's
//     backward with the rounding regulariser folded in (the adaround_bwd_kernel ops, lambda
//     and b from the iteration's device words), and the Adam step of V (ssq_adam's ops);
//     workgroup 0 also sums the loss partials in order (the loss value).
//
// The batch indices and the iteration's scalars are read from one device slot (the
// BatchFeeder's words: idx, then (lambda, b), then Adam's (-lr/bc1, sqrt(bc2))), so a
// graph of several iterations reads one slot each (quant/block_recon.py ChunkGraph).
// Deterministic: fixed summation orders, no atomics.  The GEMMs' summation order is this
// kernel's, not hipBLASLt's: values agree with the unfused path to fp32 rounding
// (tests/test_recon_gpu.py::test_fc_fused_iteration_matches_unfused).
#include "fin_tasks.h"
#include "ssq_common.h"

namespace ssq {

constexpr uint32_t kFcCo = 32;        // output channels per forward workgroup
constexpr uint32_t kFcRows = 64;      // max batch rows
constexpr uint32_t kFcCi = 128;       // ci chunk staged per step (forward)
constexpr uint32_t kFcBwdCo = 8;      // output channels per backward workgroup
constexpr uint32_t kFcMaxCi = 4096;   // x rows staged whole in the backward (LDS)

// W^ of one element: adaround_fwd_kernel's ops (per-row delta, scale 1)
__device__ __forceinline__ float fc_what(float w, float v, float d, float z, float lo, float hi) {
  const float q = clampf(__fadd_rn(__fadd_rn(floorf(w / d), rect_sigmoid(v)), z), lo, hi);
  return __fmul_rn(__fsub_rn(q, z), d);
}

// Forward: workgroup b owns output channels [b*32, b*32+32); thread t -> channel t % 32,
// rows (t / 32) + 8 j.  Every output's dot product runs ci = 0, 1, ... in order.
__global__ __launch_bounds__(kBlock) void fc_fwd_loss(
    const float* __restrict__ x, const int64_t* __restrict__ slot, uint32_t bs,
    const float* __restrict__ W, const float* __restrict__ V, const float* __restrict__ delta,
    const float* __restrict__ zp, float lo, float hi, const float* __restrict__ bias,
    uint32_t Co, uint32_t Ci, const float* __restrict__ tgt, float inv_m, float* __restrict__ g,
    double* __restrict__ part) {
  __shared__ float xs[kFcRows][kFcCi + 1];
  __shared__ float ws[kFcCo][kFcCi + 1];
  __shared__ double red[kBlock / kWave];
  const uint32_t t = threadIdx.x, cl = t % kFcCo, rg = t / kFcCo;   // rg in [0, 8)
  const uint32_t co0 = blockIdx.x * kFcCo, co = co0 + cl;
  constexpr uint32_t kRpt = kFcRows / (kBlock / kFcCo);             // 8 rows per thread
  float acc[kRpt];
#pragma unroll
  for (uint32_t j = 0; j < kRpt; ++j) acc[j] = 0.0f;
  for (uint32_t c0 = 0; c0 < Ci; c0 += kFcCi) {
    const uint32_t nc = min(kFcCi, Ci - c0);
    // stage x[idx[r], c0:c0+nc] and W^[co0:co0+32, c0:c0+nc]
    for (uint32_t e = t; e < bs * kFcCi; e += kBlock) {
      const uint32_t r = e / kFcCi, c = e % kFcCi;
      xs[r][c] = c < nc ? x[slot[r] * (int64_t)Ci + c0 + c] : 0.0f;
    }
    for (uint32_t e = t; e < kFcCo * kFcCi; e += kBlock) {
      const uint32_t r = e / kFcCi, c = e % kFcCi, o = co0 + r;
      float wv = 0.0f;
      if (o < Co && c < nc) {
        const int64_t i = (int64_t)o * Ci + c0 + c;
        wv = fc_what(W[i], V[i], delta[o], zp[o], lo, hi);
      }
      ws[r][c] = wv;
    }
    __syncthreads();
    for (uint32_t c = 0; c < nc; ++c) {
      const float wv = ws[cl][c];
#pragma unroll
      for (uint32_t j = 0; j < kRpt; ++j) acc[j] = __fmaf_rn(xs[rg + 8 * j][c], wv, acc[j]);
    }
    __syncthreads();
  }
  double la = 0.0;
  if (co < Co) {
    const float b = bias ? bias[co] : 0.0f;
#pragma unroll
    for (uint32_t j = 0; j < kRpt; ++j) {
      const uint32_t r = rg + 8 * j;
      if (r < bs) {
        const float y = bias ? __fadd_rn(acc[j], b) : acc[j];
        g[(int64_t)r * Co + co] = lp_elem<0>(y, tgt[slot[r] * (int64_t)Co + co], 2.0f, inv_m,
                                             1.0f, 0, la);
      }
    }
  }
  la = wave_sum(la);
  if ((t & (kWave - 1)) == 0) red[t / kWave] = la;
  __syncthreads();
  if (t == 0) {
    double s = red[0];
#pragma unroll
    for (int k = 1; k < kBlock / kWave; ++k) s += red[k];
    part[blockIdx.x] = s;
  }
}

// Backward + Adam: workgroup b owns output channels [b*8, b*8+8) x every ci; the batch's x
// rows and g columns staged in LDS; thread t walks elements t, t + 256, ... of the tile.
__global__ __launch_bounds__(kBlock) void fc_bwd_adam(
    const float* __restrict__ x, const int64_t* __restrict__ slot, uint32_t bs,
    const float* __restrict__ g, const float* __restrict__ W, float* __restrict__ V,
    const float* __restrict__ delta, const float* __restrict__ zp, float lo, float hi,
    uint32_t Co, uint32_t Ci, const float* __restrict__ regp, AdamConst ac,
    float* __restrict__ m, float* __restrict__ v, float* __restrict__ gv_out,
    const double* __restrict__ part, uint32_t nparts, double M, float* __restrict__ loss_out) {
  extern __shared__ float sm[];
  float* xs = sm;                        // [bs][Ci]
  float* gs = sm + (size_t)bs * Ci;      // [bs][8]
  const uint32_t t = threadIdx.x;
  if (blockIdx.x == 0 && t == 0) {
    // the loss value: the forward's workgroup partials in order
    double s = 0.0;
    for (uint32_t k = 0; k < nparts; ++k) s += part[k];
    loss_out[0] = (float)(s / M);
  }
  const uint32_t co0 = blockIdx.x * kFcBwdCo;
  for (uint32_t e = t; e < bs * Ci; e += kBlock) {
    const uint32_t r = e / Ci, c = e - r * Ci;
    xs[e] = x[slot[r] * (int64_t)Ci + c];
  }
  for (uint32_t e = t; e < bs * kFcBwdCo; e += kBlock) {
    const uint32_t r = e / kFcBwdCo, o = co0 + e % kFcBwdCo;
    gs[e] = o < Co ? g[(int64_t)r * Co + o] : 0.0f;
  }
  __syncthreads();
  const float lam = regp[0], rb = regp[1];
  const AdamRef ar{V, m, v};
  for (uint32_t e = t; e < kFcBwdCo * Ci; e += kBlock) {
    const uint32_t ol = e / Ci, c = e - ol * Ci, o = co0 + ol;
    if (o >= Co) continue;
    float dw = 0.0f;
    for (uint32_t r = 0; r < bs; ++r) dw = __fmaf_rn(gs[r * kFcBwdCo + ol], xs[r * Ci + c], dw);
    const int64_t i = (int64_t)o * Ci + c;
    const float d = delta[o], z = zp[o], b = V[i];
    // adaround_bwd_kernel's ops
    const float u = __fadd_rn(__fadd_rn(floorf(W[i] / d), rect_sigmoid(b)), z);
    const float gi = (u >= lo && u <= hi) ? __fmul_rn(dw, d) : 0.0f;
    const float ga = rect_sigmoid_grad(b, gi);
    const float gb = lam != 0.0f ? __fadd_rn(ga, round_reg_grad(b, lam, rb)) : ga;
    if (gv_out) gv_out[i] = gb;
    adam_apply_loaded(ac, ar, (uint32_t)i, gb, b, m[i], v[i]);
  }
}

}  // namespace ssq

using namespace ssq;

extern "C" size_t ssq_fc_recon_workspace_size(int64_t Co, int64_t Ci, int64_t bs) {
  (void)Ci;
  (void)bs;
  const size_t nwg = (size_t)((Co + kFcCo - 1) / kFcCo);
  return nwg * sizeof(double);
}

extern "C" int ssq_fc_recon_iter(const float* x_cache, const float* tgt_cache,
                                 const int64_t* slot, int64_t bs, const float* W, float* V,
                                 const float* delta, const float* zp, int qmin, int qmax,
                                 const float* bias, int64_t Co, int64_t Ci, float one_minus_beta1,
                                 float beta2, float one_minus_beta2, float eps, float* exp_avg,
                                 float* exp_avg_sq, float* g, float* gv_out, float* loss_out,
                                 void* ws, size_t ws_bytes, ssq_stream_t stream) {
  SSQ_REQUIRE(x_cache && tgt_cache && slot && W && V && delta && zp && exp_avg && exp_avg_sq && g &&
                  loss_out, SSQ_E_ARG, "ssq_fc_recon_iter: null pointer");
  SSQ_REQUIRE(bs >= 1 && bs <= (int64_t)kFcRows && Co >= 1 && Ci >= 1 && Ci <= (int64_t)kFcMaxCi &&
                  Co * Ci < (1ll << 31) && qmin < qmax, SSQ_E_ARG,
              "ssq_fc_recon_iter: 1 <= batch <= %u, Ci <= %u", kFcRows, kFcMaxCi);
  SSQ_REQUIRE(ws && ws_bytes >= ssq_fc_recon_workspace_size(Co, Ci, bs), SSQ_E_WS,
              "ssq_fc_recon_iter: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  const uint32_t nf = (uint32_t)((Co + kFcCo - 1) / kFcCo);
  double* part = (double*)ws;
  // the slot: bs indices, then (lambda, b) and Adam's (-lr/bc1, sqrt(bc2)) as fp32 pairs
  const float* words = (const float*)(slot + bs);
  hipLaunchKernelGGL(fc_fwd_loss, dim3(nf), dim3(kBlock), 0, s, x_cache, slot, (uint32_t)bs, W, V,
                     delta, zp, (float)qmin, (float)qmax, bias, (uint32_t)Co, (uint32_t)Ci,
                     tgt_cache, 1.0f / (float)bs, g, part);
  int rc = check_launch("ssq_fc_recon_iter (forward)");
  if (rc) return rc;
  const uint32_t nb = (uint32_t)((Co + kFcBwdCo - 1) / kFcBwdCo);
  const size_t lds = ((size_t)bs * Ci + (size_t)bs * kFcBwdCo) * sizeof(float);
  SSQ_REQUIRE(lds <= 160 * 1024, SSQ_E_ARG, "ssq_fc_recon_iter: batch x Ci exceeds the LDS");
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)fc_bwd_adam, hipFuncAttributeMaxDynamicSharedMemorySize,
                        160 * 1024);
    attr = true;
  }
  const AdamConst ac{one_minus_beta1, beta2, one_minus_beta2, eps, words + 2};
  hipLaunchKernelGGL(fc_bwd_adam, dim3(nb), dim3(kBlock), lds, s, x_cache, slot, (uint32_t)bs, g, W,
                     V, delta, zp, (float)qmin, (float)qmax, (uint32_t)Co, (uint32_t)Ci, words, ac,
                     exp_avg, exp_avg_sq, gv_out, part, nf, (double)bs, loss_out);
  return check_launch("ssq_fc_recon_iter (backward + Adam)");
}
