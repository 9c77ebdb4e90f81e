// K3/K4: UniformAffineQuantizer.init_quantization_scale (quant_layer.py:100-166) and
// K10: ChannelQuantMSE.init_scale / forward (channelQuantMSE.py:203-276).
//
// The reference runs a Python loop over channels with two .item() host syncs per
// channel ('max') or 80 x (quantize + Lp loss) eager launches per channel ('mse').
// Here every row is reduced on the device:
//   stage A  per (row, slice): fp32 min / max                      (4 B/elem)
//   stage B  per (row, slice): the slice is staged in LDS once and each wave scores a
//            strided subset of the 80 shrink candidates from LDS   (4 B/elem HBM)
//   stage C  per row: fixed-order sum of slice partials, first strict minimum, and the
//            fp64 finalize that the host Python performs ('max').
#include "ssq_common.h"

namespace ssq {

constexpr int kCand = 80;
constexpr int kSlice = 8192;  // elements of one row handled by one workgroup (32 KB LDS)

// torch.min / torch.max propagate NaN (the reference's x.min() / x.max(),
// quant_layer.py:124-125,145-146): IEEE 754-2019 minimum / maximum, not fminf / fmaxf
__device__ __forceinline__ float nan_min(float a, float b) { return __builtin_elementwise_minimum(a, b); }
__device__ __forceinline__ float nan_max(float a, float b) { return __builtin_elementwise_maximum(a, b); }
__device__ __forceinline__ float wave_nan_min(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = nan_min(v, __shfl_xor(v, o, kWave));
  return v;
}
__device__ __forceinline__ float wave_nan_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = nan_max(v, __shfl_xor(v, o, kWave));
  return v;
}

__global__ __launch_bounds__(kBlock) void minmax_stage(const float* __restrict__ x, int64_t inner,
                                                       int nslice, float* __restrict__ pmin,
                                                       float* __restrict__ pmax) {
  __shared__ float smin[kBlock / kWave], smax[kBlock / kWave];
  const int64_t row = blockIdx.y;
  const int64_t s0 = (int64_t)blockIdx.x * kSlice, s1 = min(s0 + (int64_t)kSlice, inner);
  const float* r = x + row * inner;
  float mn = INFINITY, mx = -INFINITY;
  for (int64_t k = s0 + threadIdx.x; k < s1; k += blockDim.x) {
    const float v = r[k];
    mn = nan_min(mn, v);
    mx = nan_max(mx, v);
  }
  mn = wave_nan_min(mn);
  mx = wave_nan_max(mx);
  const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
  if (lane == 0) {
    smin[w] = mn;
    smax[w] = mx;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < kBlock / kWave; ++i) {
      mn = nan_min(mn, smin[i]);
      mx = nan_max(mx, smax[i]);
    }
    mn = nan_min(smin[0], mn);
    mx = nan_max(smax[0], mx);
    pmin[row * nslice + blockIdx.x] = mn;
    pmax[row * nslice + blockIdx.x] = mx;
  }
}

__device__ __forceinline__ void row_minmax(const float* pmin, const float* pmax, int64_t row,
                                           int nslice, float& mn, float& mx) {
  mn = pmin[row * nslice];
  mx = pmax[row * nslice];
  for (int i = 1; i < nslice; ++i) {
    mn = nan_min(mn, pmin[row * nslice + i]);
    mx = nan_max(mx, pmax[row * nslice + i]);
  }
}

// 'max' finalize: host Python fp64 arithmetic (quant_layer.py:124-142).  A row the
// reference cannot initialise -- a NaN extremum, or x_min = -inf, where its
// round(-x_min / delta) is round(nan) and raises ValueError (:140) -- gets delta = zp =
// raw_zp = NaN, which the host layer turns into that error (kernels.scale_init).
__global__ void finalize_max(const float* __restrict__ pmin, const float* __restrict__ pmax,
                             int64_t rows, int nslice, int n_bits, int sym, int scale_flag,
                             float* __restrict__ delta, float* __restrict__ zp,
                             float* __restrict__ raw_zp) {
  const int64_t row = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (row >= rows) return;
  float fmn, fmx;
  row_minmax(pmin, pmax, row, nslice, fmn, fmx);
  double x_min = fmin((double)fmn, 0.0), x_max = fmax((double)fmx, 0.0);
  if (scale_flag) {
    x_min = x_min * (double)(n_bits + 2) / 8.0;
    x_max = x_max * (double)(n_bits + 2) / 8.0;
  }
  if (sym) {
    const double a = fmax(fabs(x_min), x_max);
    x_min = x_min < 0 ? -a : 0.0;
    x_max = a;
  }
  double d = (x_max - x_min) / (double)((1 << n_bits) - 1);
  if (d < 1e-8) d = 1e-8;
  const double z = rint(-x_min / d);  // Python round(): half-to-even
  if (isnan(fmn) || isnan(fmx) || isnan(z)) {
    delta[row] = zp[row] = raw_zp[row] = NAN;
    return;
  }
  delta[row] = (float)d;
  zp[row] = (float)z;
  raw_zp[row] = (float)(-x_min);
}

struct Cand {
  float d[kCand], z[kCand];
};

// Candidate i of quant_layer.py:151-162 for a row with fp32 extrema (mx, mn).
__device__ __forceinline__ void candidate(float mx, float mn, int i, int n_bits, float& d,
                                          float& z, float& nmin) {
  const float s = (float)(1.0 - (double)i * 0.01);  // python float -> fp32 scalar
  const float nmax = __fmul_rn(mx, s);
  nmin = __fmul_rn(mn, s);
  d = __fsub_rn(nmax, nmin) / (float)((1 << n_bits) - 1);
  z = rintf(-nmin / d);
}

// |e|^2.4 with NaN kept NaN (torch.pow): a candidate whose error is NaN anywhere scores NaN
// and is never the strict minimum, as in the reference (quant_layer.py:157-158)
__device__ __forceinline__ float pow24(float a) {
  return a > 0.0f ? exp2f(2.4f * log2f(a)) : (a == 0.0f ? 0.0f : a);
}

__global__ __launch_bounds__(kBlock) void mse_stage(const float* __restrict__ x, int64_t inner,
                                                    int nslice, const float* __restrict__ pmin,
                                                    const float* __restrict__ pmax, int n_bits,
                                                    int sym, double* __restrict__ part) {
  __shared__ float xs[kSlice];
  __shared__ float cd[kCand], cz[kCand];
  const int64_t row = blockIdx.y;
  const int64_t s0 = (int64_t)blockIdx.x * kSlice, s1 = min(s0 + (int64_t)kSlice, inner);
  const int len = (int)(s1 - s0);
  const float* r = x + row * inner + s0;
  for (int k = threadIdx.x; k < len; k += blockDim.x) xs[k] = r[k];
  float mn, mx;
  row_minmax(pmin, pmax, row, nslice, mn, mx);
  if (sym) {
    const float a = fmaxf(fabsf(mn), mx);
    mn = mn < 0.0f ? -a : 0.0f;
    mx = a;
  }
  for (int i = threadIdx.x; i < kCand; i += blockDim.x) {
    float nmin;
    candidate(mx, mn, i, n_bits, cd[i], cz[i], nmin);
  }
  __syncthreads();
  const float hi = (float)((1 << n_bits) - 1);  // quantize() clamps to [0, n-1] (quant_layer.py:173)
  const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
  for (int c = w; c < kCand; c += kBlock / kWave) {
    const float d = cd[c], z = cz[c];
    double acc = 0.0;
    for (int k = lane; k < len; k += kWave) {
      const float xv = xs[k];
      const float q = clampf(__fadd_rn(rintf(xv / d), z), 0.0f, hi);
      const float xq = __fmul_rn(__fsub_rn(q, z), d);
      acc += (double)pow24(fabsf(__fsub_rn(xv, xq)));
    }
    acc = wave_sum(acc);
    if (lane == 0) part[((size_t)row * nslice + blockIdx.x) * kCand + c] = acc;
  }
}

__global__ void finalize_mse(const double* __restrict__ part, const float* __restrict__ pmin,
                             const float* __restrict__ pmax, int64_t rows, int64_t inner,
                             int nslice, int n_bits, int sym, float* __restrict__ delta,
                             float* __restrict__ zp, float* __restrict__ raw_zp,
                             double* __restrict__ scores) {
  // one workgroup per row: wave w sums the slice partials of candidates w, w+4, ...
  // (lanes over slices, fixed shuffle tree), then thread 0 picks the first strict minimum
  __shared__ double sc[kCand];
  const int64_t row = blockIdx.x;
  const int lane = threadIdx.x & (kWave - 1), wv = threadIdx.x / kWave;
  for (int c = wv; c < kCand; c += blockDim.x / kWave) {
    double sum = 0.0;
    for (int s = lane; s < nslice; s += kWave) sum += part[((size_t)row * nslice + s) * kCand + c];
    sum = wave_sum(sum);
    if (lane == 0) sc[c] = sum / (double)inner;
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  float mn, mx;
  row_minmax(pmin, pmax, row, nslice, mn, mx);
  if (sym) {
    const float a = fmaxf(fabsf(mn), mx);
    mn = mn < 0.0f ? -a : 0.0f;
    mx = a;
  }
  // no candidate with a score below 1e10 (a NaN row, an infinite extremum, a constant row:
  // every score NaN) leaves the reference's delta None (quant_layer.py:147-162), which it
  // cannot use: NaN here, raised by the host layer
  double best = 1e10;
  float bd = NAN, bz = NAN, br = NAN;
  for (int c = 0; c < kCand; ++c) {
    const double score = sc[c];
    if (scores) scores[(size_t)row * kCand + c] = score;
    if (score < best) {
      best = score;
      float d, z, nmin;
      candidate(mx, mn, c, n_bits, d, z, nmin);
      bd = d;
      bz = sym ? 0.0f : z;
      br = sym ? 0.0f : -nmin;
    }
  }
  delta[row] = bd;
  zp[row] = bz;
  raw_zp[row] = br;
}

// ------------------------------------------------------------------ K10
// One wave per column j (4 columns per workgroup).  The reference scans c = k/level for
// k = level..1 and keeps the LAST (smallest) c whose normalized codes fit.  Every op in
// v(c) = ((W/c)/d + zero)/x_range is monotone (IEEE rounding is), so as c shrinks the
// column max can only grow and the min only fall: the set of fitting c is upward closed,
// and a binary search over k returns exactly the scan's answer in log2(level) passes of
// the column instead of level passes.  Each pass: lanes sweep the Co rows, wave min/max.
__global__ __launch_bounds__(kBlock) void inpscale_search_kernel(
    const float* __restrict__ W, const float* __restrict__ delta, const float* __restrict__ raw_zp,
    int64_t Co, int64_t J, float x_range, int level, float min_lim, float max_lim,
    float* __restrict__ inp) {
  const int64_t j = (int64_t)blockIdx.x * (blockDim.x / kWave) + threadIdx.x / kWave;
  const int lane = threadIdx.x & (kWave - 1);
  if (j >= J) return;
  auto cand = [&](int k) { return (float)((double)k / (double)level); };
  auto fits = [&](int k) {
    const float c = cand(k);
    float mn = INFINITY, mx = -INFINITY;
    for (int64_t co = lane; co < Co; co += kWave) {
      const float d = delta[co];
      const float zero = rintf(raw_zp[co] / d);
      const float v = __fadd_rn((W[co * J + j] / c) / d, zero) / x_range;
      mn = fminf(mn, v);
      mx = fmaxf(mx, v);
    }
    mn = wave_min(mn);
    mx = wave_max(mx);
    return mn > min_lim && mx < max_lim;
  };
  float cur = 1.0f;
  if (fits(level)) {
    int lo = 1, hi = level;  // fits(hi) holds
    while (lo < hi) {
      const int mid = lo + (hi - lo) / 2;
      if (fits(mid)) hi = mid;
      else lo = mid + 1;
    }
    cur = cand(hi);
  }
  if (lane == 0) inp[j] = cur;
}

__global__ __launch_bounds__(kBlock) void inpscale_fwd_kernel(
    const float* __restrict__ W, const float* __restrict__ inp, const float* __restrict__ delta,
    const float* __restrict__ raw_zp, int64_t Co, int64_t J, float hi, float* __restrict__ out) {
  const int64_t n = Co * J;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += stride) {
    const int64_t co = e / J, j = e - co * J;
    const float d = delta[co], c = inp[j];
    const float z = rintf(raw_zp[co] / d);
    const float q = clampf(__fadd_rn(rintf((W[e] / c) / d), z), 0.0f, hi);
    out[e] = __fmul_rn(__fmul_rn(__fsub_rn(q, z), d), c);
  }
}

static int nslices(int64_t inner) { return (int)((inner + kSlice - 1) / kSlice); }

}  // namespace ssq

using namespace ssq;

extern "C" size_t ssq_scale_init_workspace_size(int64_t rows, int64_t inner, int method) {
  const size_t ns = (size_t)nslices(inner);
  size_t b = 2 * rows * ns * sizeof(float);
  b = (b + 255) & ~(size_t)255;
  if (method == 1) b += rows * ns * kCand * sizeof(double);
  return b;
}

extern "C" int ssq_scale_init(const float* x, int64_t rows, int64_t inner, int n_bits, int sym,
                              int method, int scale_flag, float* delta, float* zp, float* raw_zp,
                              double* scores, void* ws, size_t ws_bytes, ssq_stream_t stream) {
  SSQ_REQUIRE(x && delta && zp && raw_zp && rows >= 1 && inner >= 1, SSQ_E_ARG,
              "ssq_scale_init: bad args");
  SSQ_REQUIRE(n_bits >= 1 && n_bits <= 8 && (method == 0 || method == 1), SSQ_E_ARG,
              "ssq_scale_init: n_bits in [1,8], method 0|1");
  SSQ_REQUIRE(rows < 65536, SSQ_E_ARG, "ssq_scale_init: rows < 65536");
  SSQ_REQUIRE(ws && ws_bytes >= ssq_scale_init_workspace_size(rows, inner, method), SSQ_E_WS,
              "ssq_scale_init: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  const int ns = nslices(inner);
  float* pmin = (float*)ws;
  float* pmax = pmin + rows * ns;
  size_t off = (2 * rows * ns * sizeof(float) + 255) & ~(size_t)255;
  hipLaunchKernelGGL(minmax_stage, dim3(ns, (unsigned)rows), dim3(kBlock), 0, s, x, inner, ns,
                     pmin, pmax);
  const dim3 fin((unsigned)((rows + 63) / 64));
  if (method == 0) {
    hipLaunchKernelGGL(finalize_max, fin, dim3(64), 0, s, pmin, pmax, rows, ns, n_bits, sym,
                       scale_flag, delta, zp, raw_zp);
  } else {
    double* part = (double*)((char*)ws + off);
    hipLaunchKernelGGL(mse_stage, dim3(ns, (unsigned)rows), dim3(kBlock), 0, s, x, inner, ns, pmin,
                       pmax, n_bits, sym, part);
    hipLaunchKernelGGL(finalize_mse, dim3((unsigned)rows), dim3(kBlock), 0, s, part, pmin, pmax, rows, inner, ns,
                       n_bits, sym, delta, zp, raw_zp, scores);
  }
  return check_launch("ssq_scale_init");
}

extern "C" int ssq_inpscale_search(const float* W, const float* delta, const float* raw_zp,
                                   int64_t Co, int64_t J, int n_bits, int level, float threshold,
                                   float* inp, ssq_stream_t stream) {
  SSQ_REQUIRE(W && delta && raw_zp && inp && Co >= 1 && J >= 1 && level >= 1, SSQ_E_ARG,
              "ssq_inpscale_search: bad args");
  const int xr = (1 << n_bits) - 1;
  const double min_lim = 0.0 - 0.5 / xr * threshold, max_lim = 1.0 + 0.5 / xr * threshold;
  const int64_t cols_per_block = kBlock / kWave;
  hipLaunchKernelGGL(inpscale_search_kernel,
                     dim3((unsigned)((J + cols_per_block - 1) / cols_per_block)),
                     dim3(kBlock), 0, (hipStream_t)stream, W, delta, raw_zp, Co, J, (float)xr,
                     level, (float)min_lim, (float)max_lim, inp);
  return check_launch("ssq_inpscale_search");
}

extern "C" int ssq_inpscale_fwd(const float* W, const float* inp, const float* delta,
                                const float* raw_zp, int64_t Co, int64_t J, int n_bits,
                                float* out, ssq_stream_t stream) {
  SSQ_REQUIRE(W && inp && delta && raw_zp && out && Co >= 1 && J >= 1, SSQ_E_ARG,
              "ssq_inpscale_fwd: bad args");
  hipLaunchKernelGGL(inpscale_fwd_kernel, dim3(grid_for(Co * J, kBlock)), dim3(kBlock), 0,
                     (hipStream_t)stream, W, inp, delta, raw_zp, Co, J,
                     (float)((1 << n_bits) - 1), out);
  return check_launch("ssq_inpscale_fwd");
}
