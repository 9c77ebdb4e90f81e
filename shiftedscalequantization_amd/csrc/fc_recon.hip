// K19: one BRECQ AdaRound iteration of a Linear layer in two launches.
//
// The end-to-end flow reconstructs the network's last layer (ResNet-18's fc, 512 -> 1000)
// with BRECQ's layer loop, 20000 iterations at batch 32 (layer_recon.py:10-104, called from
// main_imagenet.py for the fc).  Per iteration the reference gathers the batch
// (cached[randperm(N)[:32]]), runs the quantized layer (AdaRoundQuantizer soft rounding,
// adaptive_rounding.py:38-67, then F.linear), the loss (lp_loss p = 2 + the rounding
// regulariser, block_recon.py:119-182 / layer_recon.py:107-170), its backward and Adam.
// Each of those is microseconds of GPU work on this layer, so as separate launches the loop
// is bound by dependent-launch boundaries (8 launches: 32 us per iteration replayed back to
// back; in two launches 19.5 us, profiles/r5_fc_replay_probe.txt).  Here:
//
//   fc_fwd_loss  (one workgroup per 16 x 16 tile of y, 8 waves splitting C_in): y = x W^T
//     + bias on fp32 MFMA (v_mfma_f32_16x16x4_f32, every operand load of a wave issued
//     before its first MFMA), the 8 partial tiles added in wave order, then the lp_loss
//     p = 2 term and gradient of every output (lp_elem: the lp_loss_kernel ops) -> g = dL/dy
//     and one double loss partial per workgroup;
//   fc_bwd_adam  (one workgroup per 16 x 16 tile of dW): dW = g^T x on the same MFMA, then
//     per element (one a thread) AdaRound's backward with the rounding regulariser folded in
//     (the adaround_bwd_kernel ops, lambda and b from the iteration's device words), V's Adam step
//     (ssq_adam's ops), and W^ of the NEXT iteration from the updated V (the
//     adaround_fwd_kernel ops) -- so the forward reads W^ instead of evaluating the soft
//     rounding (a divide and an exp per weight) itself; workgroup 0 also sums the loss
//     partials.
//
// W^ of the first iteration comes from ssq_adaround_fwd (the caller's).  The batch indices
// and the iteration's scalars are read from one device slot (BatchFeeder's words: idx, then
// (lambda, b), then Adam's (-lr/bc1, sqrt(bc2))), so a graph of several iterations reads one
// slot each (quant/block_recon.py ChunkGraph).  Deterministic: fixed summation orders, no
// atomics.  The GEMMs' summation order is this kernel's, not hipBLASLt's: values agree with
// the unfused launches to fp32 rounding (tests/test_recon_gpu.py).
#include "fin_tasks.h"
#include "ssq_common.h"

namespace ssq {

constexpr uint32_t kFcRows = 64;      // max batch rows
constexpr uint32_t kFcMaxCi = 4096;
constexpr uint32_t kFcKW = 8;         // forward: waves per output tile = K chunks
constexpr uint32_t kFcBwdW = 4;       // backward: waves per workgroup (one 16x16 dW tile)

// W^ of one element: adaround_fwd_kernel's ops (per-row delta, scale 1)
__device__ __forceinline__ float fc_what(float w, float v, float d, float z, float lo, float hi) {
  const float q = clampf(__fadd_rn(__fadd_rn(floorf(w / d), rect_sigmoid(v)), z), lo, hi);
  return __fmul_rn(__fsub_rn(q, z), d);
}

// 16 consecutive floats (4 x 16 B) from a 16-B aligned row, or zeros
__device__ __forceinline__ void ld16(const float* p, bool ok, f32x4* v) {
#pragma unroll
  for (int u = 0; u < 4; ++u) v[u] = ok ? ((const f32x4*)p)[u] : f32x4{0.0f, 0.0f, 0.0f, 0.0f};
}

// Forward: workgroup = one 16 x 16 tile of y (rows r0.., columns o0..), 8 waves; wave w
// sums k in its chunk [w*ck, (w+1)*ck) with v_mfma_f32_16x16x4_f32 (A = x rows, B = W^^T),
// 64 k per round: lane l (k slot q = l >> 4) feeds k = k0 + 16 q + s at step s, so its 16
// A and 16 B values are 4 float4 loads each, all issued before the first MFMA.  The 8
// partial tiles are added in wave order through LDS, then the epilogue: bias, the lp_loss
// p = 2 term and gradient (lp_elem), one loss partial per workgroup.
__global__ __launch_bounds__(kBlock * 2) void fc_fwd_loss(
    const float* __restrict__ x, const int64_t* __restrict__ slot, uint32_t bs,
    const float* __restrict__ what, const float* __restrict__ bias, uint32_t Co, uint32_t Ci,
    uint32_t ck, const float* __restrict__ tgt, float inv_m, float* __restrict__ g,
    double* __restrict__ part) {
  __shared__ f32x4 red[kFcKW][kWave];
  __shared__ double lred[kWave];
  const uint32_t lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
  const uint32_t i16 = lane & 15, q = lane >> 4;
  const uint32_t o0 = blockIdx.x * 16, r0 = blockIdx.y * 16;
  const uint32_t ra = r0 + i16, ob = o0 + i16;          // this lane's A row / B column
  const bool aok = ra < bs, bok = ob < Co;
  const float* xr = x + (aok ? slot[ra] : 0) * (int64_t)Ci;
  const float* wr = what + (int64_t)(bok ? ob : 0) * Ci;
  f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
  const uint32_t k1 = min(Ci, (w + 1) * ck);
  for (uint32_t k0 = w * ck; k0 < k1; k0 += 64) {
    const uint32_t kq = k0 + 16 * q;
    const bool in = kq < k1;                          // Ci % 64 == 0 -> whole 16-runs
    f32x4 av[4], bv[4];
    ld16(xr + kq, aok && in, av);
    ld16(wr + kq, bok && in, bv);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u].x, bv[u].x, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u].y, bv[u].y, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u].z, bv[u].z, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u].w, bv[u].w, acc, 0, 0, 0);
    }
  }
  red[w][lane] = acc;
  __syncthreads();
  if (w != 0) return;
  f32x4 y = red[0][lane];
#pragma unroll
  for (uint32_t k = 1; k < kFcKW; ++k) {
    const f32x4 t = red[k][lane];
    y.x = __fadd_rn(y.x, t.x);
    y.y = __fadd_rn(y.y, t.y);
    y.z = __fadd_rn(y.z, t.z);
    y.w = __fadd_rn(y.w, t.w);
  }
  // D layout: column o = o0 + (lane & 15), rows r0 + 4 (lane >> 4) + v
  const uint32_t o = o0 + i16;
  double la = 0.0;
  if (o < Co) {
    const float b = bias ? bias[o] : 0.0f;
    float yv[4] = {y.x, y.y, y.z, y.w};
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const uint32_t r = r0 + 4 * q + v;
      if (r < bs) {
        const float yy = bias ? __fadd_rn(yv[v], b) : yv[v];
        g[(int64_t)r * Co + o] = lp_elem<0>(yy, tgt[slot[r] * (int64_t)Co + o], 2.0f, inv_m, 1.0f, 0,
                                            la);
      }
    }
  }
  la = wave_sum(la);
  if (lane == 0) part[blockIdx.y * gridDim.x + blockIdx.x] = la;
}

// Backward + Adam + the next W^: workgroup = one 16 x 16 tile of dW (rows o0.., columns
// c0..), 4 waves.  Wave 0 forms dW = g^T x over the batch rows with v_mfma_f32_16x16x4_f32
// (lane slot q feeds rows r = 4 s + q in a fixed order) and puts the tile in LDS; then each
// of the 4 waves takes 4 of its rows, one element per lane: AdaRound's backward with the
// rounding regulariser (adaround_bwd_kernel's ops, lambda and b from the iteration's words),
// V's Adam step (ssq_adam's ops) and W^ of the updated V (adaround_fwd_kernel's ops) for the
// next iteration.  The per-element math (a divide, two exps, a pow, a sqrt, Adam's divides)
// is most of the kernel, so it is spread over 4x the waves of a wave-per-tile form (traced on
// the ResNet-18 fc: 13.1-15.1 -> 11.7-13.1 us, profiles/r5_fc_anatomy_wavetile.txt vs
// r5_fc_anatomy.txt).  Every load of a wave is issued before its first use.
// Workgroup 0 also sums the forward's loss partials in order.
__global__ __launch_bounds__(kBlock) void fc_bwd_adam(
    const float* __restrict__ x, const int64_t* __restrict__ slot, uint32_t bs,
    const float* __restrict__ g, const float* __restrict__ W, float* __restrict__ V,
    const float* __restrict__ delta, const float* __restrict__ zp, float lo, float hi,
    uint32_t Co, uint32_t Ci, const float* __restrict__ regp, AdamConst ac,
    float* __restrict__ m, float* __restrict__ v, float* __restrict__ gv_out,
    float* __restrict__ what, const double* __restrict__ part, uint32_t nparts, double M,
    float* __restrict__ loss_out) {
  __shared__ float tile_dw[16][17];
  const uint32_t lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    // the loss value: the forward's workgroup partials in order
    double s = 0.0;
    for (uint32_t k = 0; k < nparts; ++k) s += part[k];
    loss_out[0] = (float)(s / M);
  }
  const uint32_t nct = Ci / 16;                       // column tiles (Ci % 16 == 0)
  const uint32_t o0 = (blockIdx.x / nct) * 16, c0 = (blockIdx.x % nct) * 16;
  const uint32_t i16 = lane & 15, q = lane >> 4;
  // this thread's element: row o = o0 + 4 w + q, column c = c0 + i16
  const uint32_t o = o0 + 4 * w + q, c = c0 + i16;
  const bool ok = o < Co;
  const int64_t i = (int64_t)(ok ? o : 0) * Ci + c;
  const float wv = ok ? W[i] : 0.0f, b = ok ? V[i] : 0.0f;
  const float mv = ok ? m[i] : 0.0f, vv = ok ? v[i] : 0.0f;
  const float d = ok ? delta[o] : 1.0f, z = ok ? zp[o] : 0.0f;
  const float lam = regp[0], rb = regp[1];
  if (w == 0) {
    // the operands: A[i][k] = g[r][o0 + i], B[k][j] = x[idx[r]][c0 + j], r = 4 s + q over
    // the 16 steps (bs <= 64)
    float av[16], bv[16];
    const uint32_t oa = o0 + i16;
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const uint32_t r = 4 * s + q;
      const bool rk = r < bs;
      av[s] = (rk && oa < Co) ? g[(int64_t)r * Co + oa] : 0.0f;
      bv[s] = rk ? x[slot[r] * (int64_t)Ci + c0 + i16] : 0.0f;
    }
    f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
    const uint32_t steps = (bs + 3) / 4;               // uniform
    for (uint32_t s = 0; s < 16; ++s)
      if (s < steps) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[s], bv[s], acc, 0, 0, 0);
    // D layout: column i16, rows 4 q + e
    tile_dw[4 * q + 0][i16] = acc.x;
    tile_dw[4 * q + 1][i16] = acc.y;
    tile_dw[4 * q + 2][i16] = acc.z;
    tile_dw[4 * q + 3][i16] = acc.w;
  }
  __syncthreads();
  if (!ok) return;
  const float dwv = tile_dw[4 * w + q][i16];
  // adaround_bwd_kernel's ops
  const float u0 = __fadd_rn(__fadd_rn(floorf(wv / d), rect_sigmoid(b)), z);
  const float gi = (u0 >= lo && u0 <= hi) ? __fmul_rn(dwv, d) : 0.0f;
  const float ga = rect_sigmoid_grad(b, gi);
  const float gb = lam != 0.0f ? __fadd_rn(ga, round_reg_grad(b, lam, rb)) : ga;
  if (gv_out) gv_out[i] = gb;
  float pn = b, mn = mv, vn = vv;
  adam_update(ac, gb, pn, mn, vn);            // ssq_adam's ops
  V[i] = pn;
  m[i] = mn;
  v[i] = vn;
  // the next iteration's W^ from the updated V (adaround_fwd_kernel's ops)
  what[i] = fc_what(wv, pn, d, z, lo, hi);
}

}  // namespace ssq

using namespace ssq;

extern "C" size_t ssq_fc_recon_workspace_size(int64_t Co, int64_t Ci, int64_t bs) {
  (void)Ci;
  const size_t nwg = (size_t)((Co + 15) / 16) * (size_t)((bs + 15) / 16);
  return nwg * sizeof(double);
}

extern "C" int ssq_fc_recon_iter(const float* x_cache, const float* tgt_cache,
                                 const int64_t* slot, int64_t bs, const float* W, float* V,
                                 float* What, const float* delta, const float* zp, int qmin,
                                 int qmax, const float* bias, int64_t Co, int64_t Ci,
                                 float one_minus_beta1, float beta2, float one_minus_beta2,
                                 float eps, float* exp_avg, float* exp_avg_sq, float* g,
                                 float* gv_out, float* loss_out, void* ws, size_t ws_bytes,
                                 ssq_stream_t stream) {
  SSQ_REQUIRE(x_cache && tgt_cache && slot && W && V && What && delta && zp && exp_avg &&
                  exp_avg_sq && g && loss_out, SSQ_E_ARG, "ssq_fc_recon_iter: null pointer");
  SSQ_REQUIRE(bs >= 1 && bs <= (int64_t)kFcRows && Co >= 1 && Ci >= 64 && Ci % 64 == 0 &&
                  Ci <= (int64_t)kFcMaxCi && Co * Ci < (1ll << 31) && qmin < qmax, SSQ_E_ARG,
              "ssq_fc_recon_iter: 1 <= batch <= %u, 64 <= C_in <= %u, C_in %% 64 == 0", kFcRows,
              kFcMaxCi);
  auto al = [](const void* p) { return ((uintptr_t)p & 15u) == 0; };
  SSQ_REQUIRE(al(x_cache) && al(What), SSQ_E_ARG, "ssq_fc_recon_iter: 16-B aligned x / W^");
  SSQ_REQUIRE(ws && ws_bytes >= ssq_fc_recon_workspace_size(Co, Ci, bs), SSQ_E_WS,
              "ssq_fc_recon_iter: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  // K chunk per wave: C_in / 8 rounded up to whole 64-k rounds
  const uint32_t ck = (uint32_t)(((Ci + kFcKW - 1) / kFcKW + 63) / 64 * 64);
  const dim3 gf((unsigned)((Co + 15) / 16), (unsigned)((bs + 15) / 16));
  double* part = (double*)ws;
  // the slot: bs indices, then (lambda, b) and Adam's (-lr/bc1, sqrt(bc2)) as fp32 pairs
  const float* words = (const float*)(slot + bs);
  hipLaunchKernelGGL(fc_fwd_loss, gf, dim3(kWave * kFcKW), 0, s, x_cache, slot, (uint32_t)bs,
                     What, bias, (uint32_t)Co, (uint32_t)Ci, ck, tgt_cache, 1.0f / (float)bs, g,
                     part);
  int rc = check_launch("ssq_fc_recon_iter (forward)");
  if (rc) return rc;
  const uint32_t ntile = (uint32_t)(((Co + 15) / 16) * (Ci / 16));
  const AdamConst ac{one_minus_beta1, beta2, one_minus_beta2, eps, words + 2};
  hipLaunchKernelGGL(fc_bwd_adam, dim3(ntile), dim3(kWave * kFcBwdW), 0,
                     s, x_cache, slot, (uint32_t)bs, g, W, V, delta, zp, (float)qmin, (float)qmax,
                     (uint32_t)Co, (uint32_t)Ci, words, ac, exp_avg, exp_avg_sq, gv_out, What,
                     part, gf.x * gf.y, (double)bs, loss_out);
  return check_launch("ssq_fc_recon_iter (backward + Adam + next W^)");
}
