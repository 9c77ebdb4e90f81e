// K11: reconstruction loss value + gradient in one pass, and K14: the batch gather of
// the reconstruction loop (layer_recon_fused_shiftedScale.py:94-102).
//
// lp_loss (quant_layer.py:25-32) is five eager launches plus five more in autograd; here
// one pass reads pred and tgt and writes d loss/d pred (12 B/elem), with a deterministic
// two-stage reduction of the loss value.  For p == 2 the gradient is bit-identical to
// PyTorch's: (1/M) * (2*|d|) * sgn(d).
#include "ssq_common.h"

namespace ssq {

constexpr int kLossBlocks = 1024;

template <int PMODE>  // 0: p == 2, 1: p == 1, 2: general p
__global__ __launch_bounds__(kBlock) void lp_loss_kernel(const float* __restrict__ pred,
                                                         const float* __restrict__ tgt, int64_t n,
                                                         float p, float inv_m,
                                                         float* __restrict__ grad,
                                                         const float* __restrict__ gscale,
                                                         double* __restrict__ part) {
  __shared__ double red[16];
  double acc = 0.0;
  const float gs = gscale ? gscale[0] : 1.0f;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const float d = __fsub_rn(pred[i], tgt[i]);
    const float a = fabsf(d);
    float pw, dp;  // |d|^p and p*|d|^(p-1)
    if (PMODE == 0) {
      pw = __fmul_rn(a, a);
      dp = __fmul_rn(2.0f, a);
    } else if (PMODE == 1) {
      pw = a;
      dp = 1.0f;
    } else {
      pw = powf(a, p);
      dp = __fmul_rn(p, powf(a, p - 1.0f));
    }
    acc += (double)pw;
    if (grad) {
      const float sg = d > 0.0f ? 1.0f : (d < 0.0f ? -1.0f : 0.0f);
      grad[i] = __fmul_rn(__fmul_rn(__fmul_rn(inv_m, dp), sg), gs);
    }
  }
  if (!part) return;
  acc = block_sum(acc, red);
  if (threadIdx.x == 0) part[blockIdx.x] = acc;
}

__global__ void lp_loss_finalize(const double* __restrict__ part, int nblk, double m,
                                 float* __restrict__ out) {
  __shared__ double red[16];
  double a = 0.0;
  for (int i = threadIdx.x; i < nblk; i += blockDim.x) a += part[i];
  a = block_sum(a, red);
  if (threadIdx.x == 0) out[0] = (float)(a / m);
}

// dst_k[r, :] = src_k[idx[r], :], 16-B vectors when rows allow it.
template <bool VEC>
__global__ __launch_bounds__(kBlock) void gather2_kernel(const float* __restrict__ s0,
                                                         float* __restrict__ d0, int64_t row0,
                                                         const float* __restrict__ s1,
                                                         float* __restrict__ d1, int64_t row1,
                                                         const int64_t* __restrict__ idx,
                                                         int64_t nidx) {
  const int64_t w = VEC ? 4 : 1;
  const int64_t r0 = row0 / w, r1 = s1 ? row1 / w : 0;
  const int64_t per = r0 + r1;
  const int64_t total = per * nidx;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += stride) {
    const int64_t r = e / per, k = e - r * per;
    const int64_t src_row = idx[r];
    if (VEC) {
      if (k < r0)
        ((f32x4*)d0)[r * r0 + k] = ((const f32x4*)s0)[src_row * r0 + k];
      else
        ((f32x4*)d1)[r * r1 + (k - r0)] = ((const f32x4*)s1)[src_row * r1 + (k - r0)];
    } else {
      if (k < r0)
        d0[r * r0 + k] = s0[src_row * r0 + k];
      else
        d1[r * r1 + (k - r0)] = s1[src_row * r1 + (k - r0)];
    }
  }
}

}  // namespace ssq

using namespace ssq;

extern "C" size_t ssq_lp_loss_workspace_size(int64_t n) {
  (void)n;
  return kLossBlocks * sizeof(double);
}

extern "C" int ssq_lp_loss(const float* pred, const float* tgt, int64_t n, int64_t M, float p,
                           float* loss_out, float* grad, const float* gscale, void* ws,
                           size_t ws_bytes, ssq_stream_t stream) {
  SSQ_REQUIRE(pred && tgt && n >= 1 && M >= 1 && (loss_out || grad), SSQ_E_ARG,
              "ssq_lp_loss: bad args");
  SSQ_REQUIRE(!loss_out || (ws && ws_bytes >= ssq_lp_loss_workspace_size(n)), SSQ_E_WS,
              "ssq_lp_loss: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  const int grid = grid_for(n, kBlock * 4, kLossBlocks);
  const float inv_m = 1.0f / (float)M;  // mean backward: 1.0 / numel in fp32
  double* part = loss_out ? (double*)ws : nullptr;
  if (p == 2.0f)
    hipLaunchKernelGGL(lp_loss_kernel<0>, dim3(grid), dim3(kBlock), 0, s, pred, tgt, n, p, inv_m,
                       grad, gscale, part);
  else if (p == 1.0f)
    hipLaunchKernelGGL(lp_loss_kernel<1>, dim3(grid), dim3(kBlock), 0, s, pred, tgt, n, p, inv_m,
                       grad, gscale, part);
  else
    hipLaunchKernelGGL(lp_loss_kernel<2>, dim3(grid), dim3(kBlock), 0, s, pred, tgt, n, p, inv_m,
                       grad, gscale, part);
  if (loss_out)
    hipLaunchKernelGGL(lp_loss_finalize, dim3(1), dim3(kBlock), 0, s, (const double*)part, grid,
                       (double)M, loss_out);
  return check_launch("ssq_lp_loss");
}

extern "C" int ssq_gather_rows2(const float* src0, float* dst0, int64_t row0, const float* src1,
                                float* dst1, int64_t row1, const int64_t* idx, int64_t nidx,
                                ssq_stream_t stream) {
  SSQ_REQUIRE(src0 && dst0 && idx && row0 >= 1 && nidx >= 1, SSQ_E_ARG,
              "ssq_gather_rows2: bad args");
  SSQ_REQUIRE(!src1 || (dst1 && row1 >= 1), SSQ_E_ARG, "ssq_gather_rows2: bad second source");
  auto al = [](const void* q) { return ((uintptr_t)q & 15u) == 0; };
  const bool vec = row0 % 4 == 0 && al(src0) && al(dst0) &&
                   (!src1 || (row1 % 4 == 0 && al(src1) && al(dst1)));
  const int64_t total = (row0 + (src1 ? row1 : 0)) * nidx / (vec ? 4 : 1);
  const dim3 grid(grid_for(total, kBlock, 8192));
  if (vec)
    hipLaunchKernelGGL(gather2_kernel<true>, grid, dim3(kBlock), 0, (hipStream_t)stream, src0,
                       dst0, row0, src1, dst1, row1, idx, nidx);
  else
    hipLaunchKernelGGL(gather2_kernel<false>, grid, dim3(kBlock), 0, (hipStream_t)stream, src0,
                       dst0, row0, src1, dst1, row1, idx, nidx);
  return check_launch("ssq_gather_rows2");
}
