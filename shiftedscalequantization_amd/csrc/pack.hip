// K15/K16: packed low-bit weight export.
//
// The reference saves a quantized model as an fp32 state_dict plus pickled shift choices
// (main_cifar10.py:86, myScaledMethods.py:204-205).  Every hard weight quantizer of this
// path dequantizes as
//     W_hat[e] = ((q[e] - zp[co]) * d1[co | co,ci]) (* d2[j])          (fp32, in this order)
// with integer codes q in [qmin, qmax]:
//   UniformAffineQuantizer / ChannelQuant 'none'  fq1:            d1 = fp32(delta*scale)
//   ChannelQuant adaShift hard (shift_fwd_col):                   d1 = fp32(delta*1.0)
//   ChannelQuant learned_hard_sigmoid hard (cand_value):          d1[co,ci] = fp32(delta*s_sel)
//   ChannelQuant 'adaround', AdaRoundQuantizer (adaround_fwd):    d1 = fp32(delta_at*scale)
//   ChannelQuantMSE (inpscale_fwd):                               d1 = delta, d2 = inp_scale
// so storing q in bs = 2/4/8 bits per code plus the small d1/zp/d2 vectors reproduces
// W_hat bit for bit.  The encoder recovers q from W_hat itself (k = rint(W/d2/d1), exact
// for |k| < 2^20) and counts every element whose decode is not bit-identical to W_hat, so
// a quantizer that is not of this form is reported, never silently approximated.
//
// Layout: a little-endian bit stream, code e at bits [e*bs, (e+1)*bs) of the buffer,
// stored as u = q - qmin.  Four codes form one group of 4*bs bits (a u8 / u16 / u32), so
// one thread handles one float4 of W_hat and one group.  HBM bytes: decode reads bs/8 and
// writes 4 B per element; encode the reverse.
#include "ssq_common.h"

namespace ssq {

struct PackGeo {
  uint32_t n, CiK, Ci;
  FastDiv div_cik, div_k;
  int per_ci;
  float qmin, qmax;
};

template <int BS>
struct GroupT;
template <>
struct GroupT<2> { typedef uint8_t T; };
template <>
struct GroupT<4> { typedef uint16_t T; };
template <>
struct GroupT<8> { typedef uint32_t T; };

__device__ __forceinline__ void elem_params(uint32_t e, const PackGeo& g, const float* zp,
                                            const float* d1, const float* d2, float& z,
                                            float& a, float& b) {
  const uint32_t co = fdiv(e, g.div_cik);
  const uint32_t j = e - co * g.CiK;
  z = zp[co];
  a = g.per_ci ? d1[co * g.Ci + fdiv(j, g.div_k)] : d1[co];
  b = d2 ? d2[j] : 1.0f;
}

__device__ __forceinline__ float dequant(float q, float z, float a, float b, bool has_d2) {
  const float w = __fmul_rn(__fsub_rn(q, z), a);
  return has_d2 ? __fmul_rn(w, b) : w;
}

template <int BS>
__global__ __launch_bounds__(kBlock) void pack_encode_kernel(const float* __restrict__ W,
                                                             const float* __restrict__ zp,
                                                             const float* __restrict__ d1,
                                                             const float* __restrict__ d2,
                                                             PackGeo g, int vec,
                                                             typename GroupT<BS>::T* __restrict__ out,
                                                             uint32_t* __restrict__ mismatch) {
  typedef typename GroupT<BS>::T T;
  const uint32_t ngroups = (g.n + 3) / 4;
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t v = blockIdx.x * blockDim.x + threadIdx.x; v < ngroups; v += stride) {
    const uint32_t e0 = 4 * v;
    float w[4];
    if (vec && e0 + 3 < g.n) {
      const f32x4 x = __builtin_nontemporal_load((const f32x4*)W + v);
      w[0] = x.x; w[1] = x.y; w[2] = x.z; w[3] = x.w;
    } else {
      for (int i = 0; i < 4; ++i) w[i] = e0 + i < g.n ? W[e0 + i] : 0.0f;
    }
    uint32_t bits = 0, bad = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (e0 + i >= g.n) continue;
      float z, a, b;
      elem_params(e0 + i, g, zp, d1, d2, z, a, b);
      const float k = rintf(d2 ? (w[i] / b) / a : w[i] / a);
      const float q = __fadd_rn(k, z);
      const bool ok = q >= g.qmin && q <= g.qmax && fabsf(k) < 1048576.0f &&
                      __float_as_uint(dequant(q, z, a, b, d2 != nullptr)) == __float_as_uint(w[i]);
      bad += ok ? 0u : 1u;
      const uint32_t u = ok ? (uint32_t)(int)__fsub_rn(q, g.qmin) : 0u;
      bits |= (u & ((1u << BS) - 1u)) << (i * BS);
    }
    out[v] = (T)bits;
    if (bad) atomicAdd(mismatch, bad);
  }
}

template <int BS>
__global__ __launch_bounds__(kBlock) void pack_decode_kernel(const typename GroupT<BS>::T* __restrict__ in,
                                                             const float* __restrict__ zp,
                                                             const float* __restrict__ d1,
                                                             const float* __restrict__ d2,
                                                             PackGeo g, int vec,
                                                             float* __restrict__ W) {
  const uint32_t ngroups = (g.n + 3) / 4;
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t v = blockIdx.x * blockDim.x + threadIdx.x; v < ngroups; v += stride) {
    const uint32_t bits = (uint32_t)in[v];
    const uint32_t e0 = 4 * v;
    float o[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float z, a, b;
      elem_params(min(e0 + i, g.n - 1), g, zp, d1, d2, z, a, b);
      const float q = __fadd_rn((float)((bits >> (i * BS)) & ((1u << BS) - 1u)), g.qmin);
      o[i] = dequant(q, z, a, b, d2 != nullptr);
    }
    if (vec && e0 + 3 < g.n) {
      f32x4 r;
      r.x = o[0]; r.y = o[1]; r.z = o[2]; r.w = o[3];
      __builtin_nontemporal_store(r, (f32x4*)W + v);
    } else {
      for (int i = 0; i < 4; ++i)
        if (e0 + i < g.n) W[e0 + i] = o[i];
    }
  }
}

static int pack_geo(const char* what, int64_t Co, int64_t Ci, int64_t K, int per_ci, int qmin,
                    int qmax, PackGeo& g) {
  SSQ_REQUIRE(Co >= 1 && Ci >= 1 && K >= 1 && qmin < qmax, SSQ_E_ARG, "%s: bad geometry", what);
  const int64_t n = Co * Ci * K;
  SSQ_REQUIRE(n < (1ll << 31), SSQ_E_ARG, "%s: tensor exceeds 2^31 elements", what);
  g.n = (uint32_t)n;
  g.CiK = (uint32_t)(Ci * K);
  g.Ci = (uint32_t)Ci;
  g.div_cik = make_fastdiv(g.CiK);
  g.div_k = make_fastdiv((uint32_t)K);
  g.per_ci = per_ci;
  g.qmin = (float)qmin;
  g.qmax = (float)qmax;
  return SSQ_OK;
}

}  // namespace ssq

using namespace ssq;

extern "C" int ssq_pack_bits(int n_bits) {
  if (n_bits < 1 || n_bits > 8) return 0;
  return n_bits <= 2 ? 2 : (n_bits <= 4 ? 4 : 8);
}

extern "C" size_t ssq_pack_bytes(int64_t n, int n_bits) {
  const int bs = ssq_pack_bits(n_bits);
  return bs ? (size_t)((n + 3) / 4) * (size_t)(bs / 2) : 0;
}

extern "C" int ssq_pack_encode(const float* What, const float* zp, const float* d1, int d1_per_ci,
                               const float* d2, int64_t Co, int64_t Ci, int64_t K, int n_bits,
                               int qmin, int qmax, void* packed, uint32_t* mismatch,
                               ssq_stream_t stream) {
  SSQ_REQUIRE(What && zp && d1 && packed && mismatch, SSQ_E_ARG, "ssq_pack_encode: null pointer");
  const int bs = ssq_pack_bits(n_bits);
  SSQ_REQUIRE(bs && qmax - qmin < (1 << bs), SSQ_E_ARG,
              "ssq_pack_encode: code range [%d, %d] does not fit %d-bit codes", qmin, qmax,
              n_bits);
  PackGeo g;
  int rc = pack_geo("ssq_pack_encode", Co, Ci, K, d1_per_ci, qmin, qmax, g);
  if (rc) return rc;
  const int vec = ((uintptr_t)What & 15) == 0;
  const dim3 grid(grid_for((g.n + 3) / 4, kBlock, 4096));
  hipStream_t s = (hipStream_t)stream;
  if (bs == 2)
    hipLaunchKernelGGL(pack_encode_kernel<2>, grid, dim3(kBlock), 0, s, What, zp, d1, d2, g, vec,
                       (uint8_t*)packed, mismatch);
  else if (bs == 4)
    hipLaunchKernelGGL(pack_encode_kernel<4>, grid, dim3(kBlock), 0, s, What, zp, d1, d2, g, vec,
                       (uint16_t*)packed, mismatch);
  else
    hipLaunchKernelGGL(pack_encode_kernel<8>, grid, dim3(kBlock), 0, s, What, zp, d1, d2, g, vec,
                       (uint32_t*)packed, mismatch);
  return check_launch("ssq_pack_encode");
}

extern "C" int ssq_pack_decode(const void* packed, const float* zp, const float* d1,
                               int d1_per_ci, const float* d2, int64_t Co, int64_t Ci, int64_t K,
                               int n_bits, int qmin, float* What, ssq_stream_t stream) {
  SSQ_REQUIRE(What && zp && d1 && packed, SSQ_E_ARG, "ssq_pack_decode: null pointer");
  const int bs = ssq_pack_bits(n_bits);
  SSQ_REQUIRE(bs, SSQ_E_ARG, "ssq_pack_decode: n_bits %d not in [1, 8]", n_bits);
  PackGeo g;
  int rc = pack_geo("ssq_pack_decode", Co, Ci, K, d1_per_ci, qmin, qmin + (1 << bs) - 1, g);
  if (rc) return rc;
  const int vec = ((uintptr_t)What & 15) == 0;
  const dim3 grid(grid_for((g.n + 3) / 4, kBlock, 4096));
  hipStream_t s = (hipStream_t)stream;
  if (bs == 2)
    hipLaunchKernelGGL(pack_decode_kernel<2>, grid, dim3(kBlock), 0, s, (const uint8_t*)packed, zp,
                       d1, d2, g, vec, What);
  else if (bs == 4)
    hipLaunchKernelGGL(pack_decode_kernel<4>, grid, dim3(kBlock), 0, s, (const uint16_t*)packed,
                       zp, d1, d2, g, vec, What);
  else
    hipLaunchKernelGGL(pack_decode_kernel<8>, grid, dim3(kBlock), 0, s, (const uint32_t*)packed,
                       zp, d1, d2, g, vec, What);
  return check_launch("ssq_pack_decode");
}
