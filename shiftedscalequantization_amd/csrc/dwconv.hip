// K18: depthwise convolution forward and input gradient (MobileNetV2's 3x3 / stride-2
// depthwise convs, config 4).
//
// A depthwise conv has one input and one output channel per group: every output pixel is
// an R*S-term dot product of a weight row with a window of ONE input plane.  That is
// bandwidth work (read a plane, write a plane), not a GEMM.  MIOpen runs it on its naive
// direct kernels under cudnn.deterministic (the reference's setting, common.py:77-85):
// 120 us forward and 510 us input gradient for MobileNetV2 features.2 at batch 32, a
// third of the whole reconstruction iteration (tools/anat_session.sh).  Here a
// workgroup owns one or more (n, c) planes: it stages them in LDS (zero-padded, so the
// product loop has no bounds tests) with 8 loads in flight per thread, and sums the R*S
// products of each output cell in (r, s) order with separate fp32 multiplies and adds.
// Deterministic; within fp32 rounding of any other order.
#include <algorithm>

#include "ssq_common.h"

namespace ssq {

// Plane geometry shared by the forward and input-gradient kernels.  A workgroup owns P
// consecutive (n, c) planes (P > 1 for small planes so that 256 threads have work): it
// stages them (and their P weight rows) in LDS, then walks the P*OUT output cells with a
// linear thread index split by magic-number division (no per-cell integer divide).
struct DwGeo {
  int C, H, W, OH, OW, R, S, st, pad;
  int P;               // planes per workgroup
  int nplanes;         // Nb * C
  int Hs, Ws;          // staged plane (fwd: x padded by pad; dx: dy with a margin of R-1 / S-1)
  int mh, mw;          // dx: margins
  int out_h, out_w;    // cells computed per plane (fwd: OH x OW; dx: H x W)
  FastDiv d_ws, d_stage, d_outw, d_outp;  // by Ws, by Hs*Ws, by out_w, by out_h*out_w
};

// MODE 0: y[n,c,oh,ow] = sum_{r,s} w[c,r,s] * x[n,c,oh*st+r-pad, ow*st+s-pad]
// MODE 1: dx[n,c,ih,iw] = sum_{r,s: st | ih+pad-r, st | iw+pad-s} w[c,r,s] * dy[n,c,(ih+pad-r)/st,
//                                                                           (iw+pad-s)/st]
// ST > 0: compile-time stride (ST = 1, 2: shifts and masks); ST = 0: runtime stride.
template <int MODE, int ST, int RSMAX>
__global__ __launch_bounds__(256) void dw_kernel(const float* __restrict__ in,
                                                 const float* __restrict__ w,
                                                 float* __restrict__ out, DwGeo g) {
  extern __shared__ float lds[];
  const int tid = threadIdx.x;
  const int RS = g.R * g.S;
  const int plane0 = blockIdx.x * g.P;
  const int P = min(g.P, g.nplanes - plane0);
  const int st = ST > 0 ? ST : g.st;
  float* ws = lds;                      // [P][RS]
  float* xs = lds + g.P * RSMAX;        // [P][Hs][Ws]
  const int in_h = MODE == 0 ? g.H : g.OH, in_w = MODE == 0 ? g.W : g.OW;
  const int off_h = MODE == 0 ? g.pad : g.mh, off_w = MODE == 0 ? g.pad : g.mw;
  for (int e = tid; e < P * RS; e += 256) {
    const int pl = e / RS;  // tiny loop: P*RS <= 64*25
    ws[pl * RSMAX + (e - pl * RS)] = w[((plane0 + pl) % g.C) * RS + (e - pl * RS)];
  }
  // stage: 8 loads in flight per thread, then the 8 LDS stores
  const int stage = g.Hs * g.Ws, total = P * stage;
  const float* src = in + (int64_t)plane0 * in_h * in_w;
  for (int e0 = tid; e0 < total; e0 += 256 * 8) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int e = e0 + 256 * u;
      const int pl = (int)fdiv((uint32_t)e, g.d_stage);
      const int rem = e - pl * stage;
      const int rr = (int)fdiv((uint32_t)rem, g.d_ws), cc = rem - rr * g.Ws;
      const int ih = rr - off_h, iw = cc - off_w;
      const bool ok = e < total && ih >= 0 && ih < in_h && iw >= 0 && iw < in_w;
      const float t = src[ok ? ((int64_t)pl * in_h + ih) * in_w + iw : 0];
      v[u] = ok ? t : 0.0f;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (e0 + 256 * u < total) xs[e0 + 256 * u] = v[u];
  }
  __syncthreads();
  const int outp = g.out_h * g.out_w;
  float* dst = out + (int64_t)plane0 * outp;
  for (int o = tid; o < P * outp; o += 256) {
    const int pl = (int)fdiv((uint32_t)o, g.d_outp);
    const int rem = o - pl * outp;
    const int a = (int)fdiv((uint32_t)rem, g.d_outw), b = rem - a * g.out_w;
    const float* wr = ws + pl * RSMAX;
    const float* xp = xs + pl * stage;
    float acc = 0.0f;
    if (MODE == 0) {
      const float* xr = xp + a * st * g.Ws + b * st;
#pragma unroll
      for (int j = 0; j < RSMAX; ++j) {
        if (j < RS) {
          const int r = j / g.S, q = j - r * g.S;
          acc = __fadd_rn(acc, __fmul_rn(wr[j], xr[r * g.Ws + q]));
        }
      }
    } else {
#pragma unroll
      for (int j = 0; j < RSMAX; ++j) {
        if (j < RS) {
          const int r = j / g.S, q = j - r * g.S;
          const int th = a + g.pad - r, tw = b + g.pad - q;  // >= -(R-1), -(S-1)
          bool ok;
          int qh, qw;
          if (ST == 1) {
            ok = true;
            qh = th;
            qw = tw;
          } else if (ST == 2) {
            ok = ((th | tw) & 1) == 0;
            qh = th >> 1;  // exact for even th, also negative
            qw = tw >> 1;
          } else {
            const int fh = (th + st * g.mh) / st, fw = (tw + st * g.mw) / st;  // non-negative
            ok = fh * st == th + st * g.mh && fw * st == tw + st * g.mw;
            qh = fh - g.mh;
            qw = fw - g.mw;
          }
          // margins of R-1 / S-1 zero rows/cols keep every index inside the stage
          const float t = xp[ok ? (qh + g.mh) * g.Ws + (qw + g.mw) : 0];
          acc = __fadd_rn(acc, __fmul_rn(wr[j], ok ? t : 0.0f));
        }
      }
    }
    dst[o] = acc;
  }
}

static void dw_geo(int64_t Nb, int64_t C, int64_t H, int64_t W, int64_t R, int64_t S,
                   int64_t st, int64_t pad, int64_t OH, int64_t OW, int mode, DwGeo& g) {
  g.C = (int)C; g.H = (int)H; g.W = (int)W; g.OH = (int)OH; g.OW = (int)OW;
  g.R = (int)R; g.S = (int)S; g.st = (int)st; g.pad = (int)pad;
  g.nplanes = (int)(Nb * C);
  if (mode == 0) {
    g.mh = g.mw = 0;
    g.Hs = (int)(H + 2 * pad);
    g.Ws = (int)(W + 2 * pad);
    g.out_h = (int)OH;
    g.out_w = (int)OW;
  } else {
    g.mh = (int)R - 1;
    g.mw = (int)S - 1;
    // dy rows the taps can reach: (H-1+pad)/st; keep a zero margin on both sides
    g.Hs = (int)std::max<int64_t>(OH, (H - 1 + pad) / st + 1) + 2 * g.mh;
    g.Ws = (int)std::max<int64_t>(OW, (W - 1 + pad) / st + 1) + 2 * g.mw;
    g.out_h = (int)H;
    g.out_w = (int)W;
  }
  const int stage = g.Hs * g.Ws;
  const int outp = g.out_h * g.out_w;
  // planes per workgroup: ~2 output cells per thread, LDS stage <= 32 KiB, <= 64 planes
  int P = std::max(1, std::min(512 / std::max(outp, 1), 8192 / std::max(stage, 1)));
  P = std::min(P, 64);
  g.P = P;
  g.d_ws = make_fastdiv((uint32_t)g.Ws);
  g.d_stage = make_fastdiv((uint32_t)stage);
  g.d_outw = make_fastdiv((uint32_t)g.out_w);
  g.d_outp = make_fastdiv((uint32_t)outp);
}

static int dw_check(int64_t Nb, int64_t C, int64_t H, int64_t W, int64_t R, int64_t S,
                    int64_t st, int64_t pad, int64_t* OH, int64_t* OW, const char* what) {
  SSQ_REQUIRE(Nb >= 1 && C >= 1 && H >= 1 && W >= 1 && R >= 1 && S >= 1 && R * S <= 25 &&
                  st >= 1 && pad >= 0,
              SSQ_E_ARG, "%s: bad geometry (R*S <= 25)", what);
  *OH = (H + 2 * pad - R) / st + 1;
  *OW = (W + 2 * pad - S) / st + 1;
  SSQ_REQUIRE(*OH >= 1 && *OW >= 1 && Nb * C < (1ll << 31) && Nb * C * H * W < (1ll << 31) &&
                  Nb * C * *OH * *OW < (1ll << 31),
              SSQ_E_ARG, "%s: sizes", what);
  SSQ_REQUIRE((H + 2 * pad) * (W + 2 * pad) * (int64_t)sizeof(float) <= 128 * 1024, SSQ_E_ARG,
              "%s: plane of %lldx%lld exceeds the 128 KiB LDS stage", what, (long long)H,
              (long long)W);
  return SSQ_OK;
}

// dynamic LDS of a plan: the P weight rows (RSMAX wide) + the P staged planes
static int64_t dw_lds_bytes(const DwGeo& g) {
  const int64_t rsmax = g.R * g.S <= 9 ? 9 : 25;
  return ((int64_t)g.P * rsmax + (int64_t)g.P * g.Hs * g.Ws) * (int64_t)sizeof(float);
}
constexpr int64_t kDwLdsMax = 128 * 1024;   // the opted-in dynamic LDS

template <typename K>
static void lds_optin(K kernel) {
  hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                      128 * 1024);
}


template <int MODE, int ST>
static void dw_launch(const DwGeo& g, const float* in, const float* w, float* out,
                      hipStream_t s) {
  const size_t lds = ((size_t)g.P * 25 + (size_t)g.P * g.Hs * g.Ws) * sizeof(float);
  const dim3 grid((unsigned)((g.nplanes + g.P - 1) / g.P));
  if (g.R * g.S <= 9) {
    const size_t l9 = ((size_t)g.P * 9 + (size_t)g.P * g.Hs * g.Ws) * sizeof(float);
    hipLaunchKernelGGL((dw_kernel<MODE, ST, 9>), grid, dim3(256), l9, s, in, w, out, g);
  } else {
    hipLaunchKernelGGL((dw_kernel<MODE, ST, 25>), grid, dim3(256), lds, s, in, w, out, g);
  }
}

template <int MODE>
static void dw_optin() {
  lds_optin(dw_kernel<MODE, 0, 9>);
  lds_optin(dw_kernel<MODE, 0, 25>);
  lds_optin(dw_kernel<MODE, 1, 9>);
  lds_optin(dw_kernel<MODE, 1, 25>);
  lds_optin(dw_kernel<MODE, 2, 9>);
  lds_optin(dw_kernel<MODE, 2, 25>);
}

}  // namespace ssq

using namespace ssq;

extern "C" int ssq_dwconv_fwd(const float* x, const float* w, float* y, int64_t Nb, int64_t C,
                              int64_t H, int64_t W, int64_t R, int64_t S, int64_t stride,
                              int64_t pad, ssq_stream_t stream) {
  SSQ_REQUIRE(x && w && y, SSQ_E_ARG, "ssq_dwconv_fwd: null pointer");
  int64_t OH, OW;
  int rc = dw_check(Nb, C, H, W, R, S, stride, pad, &OH, &OW, "ssq_dwconv_fwd");
  if (rc) return rc;
  static bool attr = false;
  if (!attr) {
    dw_optin<0>();
    attr = true;
  }
  DwGeo g;
  dw_geo(Nb, C, H, W, R, S, stride, pad, OH, OW, 0, g);
  SSQ_REQUIRE(dw_lds_bytes(g) <= kDwLdsMax, SSQ_E_ARG,
              "ssq_dwconv_fwd: LDS stage %lld B exceeds 128 KiB", (long long)dw_lds_bytes(g));
  hipStream_t s = (hipStream_t)stream;
  if (stride == 1) dw_launch<0, 1>(g, x, w, y, s);
  else if (stride == 2) dw_launch<0, 2>(g, x, w, y, s);
  else dw_launch<0, 0>(g, x, w, y, s);
  return check_launch("ssq_dwconv_fwd");
}

extern "C" int ssq_dwconv_bwd_data(const float* dy, const float* w, float* dx, int64_t Nb,
                                   int64_t C, int64_t H, int64_t W, int64_t R, int64_t S,
                                   int64_t stride, int64_t pad, ssq_stream_t stream) {
  SSQ_REQUIRE(dy && w && dx, SSQ_E_ARG, "ssq_dwconv_bwd_data: null pointer");
  int64_t OH, OW;
  int rc = dw_check(Nb, C, H, W, R, S, stride, pad, &OH, &OW, "ssq_dwconv_bwd_data");
  if (rc) return rc;
  static bool attr = false;
  if (!attr) {
    dw_optin<1>();
    attr = true;
  }
  DwGeo g;
  dw_geo(Nb, C, H, W, R, S, stride, pad, OH, OW, 1, g);
  SSQ_REQUIRE(dw_lds_bytes(g) <= kDwLdsMax, SSQ_E_ARG,
              "ssq_dwconv_bwd_data: LDS stage %lld B exceeds 128 KiB", (long long)dw_lds_bytes(g));
  hipStream_t s = (hipStream_t)stream;
  if (stride == 1) dw_launch<1, 1>(g, dy, w, dx, s);
  else if (stride == 2) dw_launch<1, 2>(g, dy, w, dx, s);
  else dw_launch<1, 0>(g, dy, w, dx, s);
  return check_launch("ssq_dwconv_bwd_data");
}

extern "C" int ssq_dwconv_supported(int64_t Nb, int64_t C, int64_t H, int64_t W, int64_t R,
                                    int64_t S, int64_t stride, int64_t pad) {
  int64_t OH, OW;
  if (dw_check(Nb, C, H, W, R, S, stride, pad, &OH, &OW, "ssq_dwconv_supported")) return 0;
  DwGeo gf, gb;
  dw_geo(Nb, C, H, W, R, S, stride, pad, OH, OW, 0, gf);
  dw_geo(Nb, C, H, W, R, S, stride, pad, OH, OW, 1, gb);
  return dw_lds_bytes(gf) <= kDwLdsMax && dw_lds_bytes(gb) <= kDwLdsMax;
}
