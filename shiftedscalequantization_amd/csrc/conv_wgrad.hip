// K17: deterministic convolution weight gradient on the fp32 matrix cores.
//
// The reconstruction loops differentiate every conv weight (W_hat feeds the adaShift /
// AdaRound backward).  The reference runs with cudnn.deterministic = True (common.py:
// 77-85); on MIOpen that setting rules out the atomic split-K weight-gradient solvers and
// falls back to per-sample im2col + GEMM (or naive kernels): 0.9 ms for a ResNet-18
// layer1 3x3 conv at batch 32, 4-5x the whole rest of the iteration.  This kernel computes
//   dW[g, co, (ci, r, s)] = sum_{n, oh, ow} dy[n, g*Cog + co, oh, ow]
//                           * x[n, g*Cig + ci, oh*st + r - pad, ow*st + s - pad]
// as an implicit GEMM (M = Cog, N = Cig*R*S, K = N*OH*OW) on v_mfma_f32_32x32x2_f32 (exact
// fp32 products, k-ordered fp32 accumulation), deterministically:
//   stage 1: workgroup (n-tile, g*m-tiles, split) owns a 64 x 128 output tile and a fixed
//            range of K chunks (one chunk = TH output rows of one sample); per chunk it
//            stages dy[64 co][TH*OW px] and the x rows the chunk touches in LDS, then each
//            wave runs 64 x 32 of the tile (two 32x32 accumulators sharing one gathered
//            x operand per lane, the expensive one);
//            the tile is written to its split's slot of the workspace;
//   stage 2: dW = the splits summed in split order.
// Same inputs -> same bits, run to run (no atomics).  Within tolerance of any other
// summation order (the MIOpen / CPU results), like every fp32 convolution gradient.
#include <algorithm>

#include "ssq_common.h"

namespace ssq {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kTM = 64;    // co per workgroup tile
constexpr int kTN = 128;   // (ci, r, s) columns per workgroup tile
constexpr int kMaxPx = 128;  // output pixels per chunk (even)
constexpr int kXSlots = 16;  // x values per thread per chunk (plan keeps the tile within)

struct WgradGeo {
  int Nb, C, H, W, Co, OH, OW, R, S, st, pad, G, Cig, Cog;
  int Ncol;         // Cig*R*S
  int TH;           // output rows per chunk
  int P;            // TH*OW (pixels per chunk, <= kMaxPx)
  int Pp;           // P rounded up to even
  int chunks_per_n; // ceil(OH / TH)
  int nchunks;      // Nb * chunks_per_n
  int cps;          // chunks per split
  int nsplit;
  int in_rows;      // (TH-1)*st + R  (x rows staged per chunk)
  int ci_span;      // channels staged per chunk (max over tiles)
  int m_tiles;      // ceil(Cog / kTM)
  FastDiv div_wp, div_rows;  // by W + 2*pad, by in_rows
};

__global__ __launch_bounds__(256, 2) void wgrad_stage1(const float* __restrict__ x,
                                                    const float* __restrict__ dy, WgradGeo g,
                                                    float* __restrict__ part) {
  extern __shared__ float lds[];
  const int lda = g.Pp + 1;                      // odd: A reads conflict-free
  const int Wp = g.W + 2 * g.pad;                // x rows staged with zero padding columns
  float* As = lds;                               // [kTM][lda]
  float* Xs = lds + kTM * lda;                   // [ci_span][in_rows][Wp]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nt = blockIdx.x;
  const int grp = blockIdx.y / g.m_tiles, mt = blockIdx.y - grp * g.m_tiles;
  const int split = blockIdx.z;
  const int co0 = mt * kTM;                      // within the group
  const int col0 = nt * kTN;
  const int RS = g.R * g.S;
  const int ci_lo = col0 / RS;                   // first channel the tile touches
  // wave w owns columns col0 + 32w .. +31 (one per lane & 31) and all 64 rows of the
  // tile (two 32-row accumulators sharing this lane's gathered x value)
  const int col = col0 + wave * 32 + (lane & 31);
  const bool cval = col < g.Ncol;
  int xbase;
  {
    const int c = cval ? col : 0;
    const int ci = c / RS, rs = c - ci * RS;
    const int r = rs / g.S;
    xbase = ((ci - ci_lo) * g.in_rows + r) * Wp + (rs - r * g.S);
  }
  // the K range of a chunk is split in two halves, one per lane half (the MFMA's k = 0 / 1)
  const int half = lane >> 5, arow = lane & 31;
  const int Ph = g.Pp >> 1;
  const int px0 = half * Ph;
  const int oh_start = px0 / g.OW, ow_start = px0 - oh_start * g.OW;
  const int row_adj = g.st * Wp - g.OW * g.st;   // offset change when ow wraps
  const int HW = g.H * g.W, OHW = g.OH * g.OW;
  const int xtot = g.ci_span * g.in_rows * Wp;
  const int zslot = xtot;                        // Xs[xtot] = 0: the B operand past a chunk
  if (tid == 0) Xs[zslot] = 0.0f;
  const FastDiv dWp = g.div_wp, dRows = g.div_rows;
  const int c_begin = split * g.cps, c_end = min(c_begin + g.cps, g.nchunks);

  // x tile element i of the chunk starting at input row ih0 (0 outside the image)
  auto x_elem = [&](const float* sx, int ih0, int i) {
    float v = 0.0f;
    if (i < xtot) {
      const int q = (int)fdiv((uint32_t)i, dWp), w = i - q * Wp;
      const int cl = (int)fdiv((uint32_t)q, dRows), rr = q - cl * g.in_rows;
      const int ci = ci_lo + cl, ih = ih0 + rr, iw = w - g.pad;
      if (ci < g.Cig && ih >= 0 && ih < g.H && iw >= 0 && iw < g.W)
        v = sx[(int64_t)ci * HW + (int64_t)ih * g.W + iw];
    }
    return v;
  };
  // ---- global -> register prefetch of one chunk (issued before the previous chunk's
  // MFMAs); x tiles beyond kXSlots values per thread load the rest synchronously
  float ra[2][16], rx[kXSlots];
  auto load_chunk = [&](int c) {
    const int n = c / g.chunks_per_n;
    const int oh0 = (c - n * g.chunks_per_n) * g.TH;
    const int P = min(g.TH, g.OH - oh0) * g.OW;
    const int ih0 = oh0 * g.st - g.pad;
    const float* sa = dy + ((int64_t)n * g.Co + (int64_t)grp * g.Cog + co0) * OHW +
                      (int64_t)oh0 * g.OW;
#pragma unroll
    for (int jr = 0; jr < 16; ++jr) {
      const int r = wave + 4 * jr;
      const bool rv = co0 + r < g.Cog;
#pragma unroll
      for (int jp = 0; jp < 2; ++jp) {
        const int p = lane + 64 * jp;
        ra[jp][jr] = (rv && p < P) ? sa[(int64_t)r * OHW + p] : 0.0f;
      }
    }
    const float* sx = x + ((int64_t)n * g.C + (int64_t)grp * g.Cig) * HW;
#pragma unroll
    for (int j = 0; j < kXSlots; ++j) rx[j] = x_elem(sx, ih0, tid + 256 * j);
  };
  auto store_chunk = [&](int c) {
#pragma unroll
    for (int jr = 0; jr < 16; ++jr)
#pragma unroll
      for (int jp = 0; jp < 2; ++jp) {
        const int p = lane + 64 * jp;
        if (p < g.Pp) As[(wave + 4 * jr) * lda + p] = ra[jp][jr];
      }
#pragma unroll
    for (int j = 0; j < kXSlots; ++j) {
      const int i = tid + 256 * j;
      if (i < xtot) Xs[i] = rx[j];
    }
    if (xtot > 256 * kXSlots) {
      const int n = c / g.chunks_per_n;
      const int ih0 = (c - n * g.chunks_per_n) * g.TH * g.st - g.pad;
      const float* sx = x + ((int64_t)n * g.C + (int64_t)grp * g.Cig) * HW;
      for (int i = tid + 256 * kXSlots; i < xtot; i += 256) Xs[i] = x_elem(sx, ih0, i);
    }
  };

  f32x16 acc0 = {0}, acc1 = {0};
  if (c_begin < c_end) load_chunk(c_begin);
  for (int c = c_begin; c < c_end; ++c) {
    const int n = c / g.chunks_per_n;
    const int oh0 = (c - n * g.chunks_per_n) * g.TH;
    const int P = min(g.TH, g.OH - oh0) * g.OW;
    __syncthreads();                  // the previous chunk's MFMAs are done with the LDS
    store_chunk(c);
    __syncthreads();
    if (c + 1 < c_end) load_chunk(c + 1);
    int ow = ow_start, px = px0;
    int off = xbase + oh_start * g.st * Wp + ow_start * g.st;
    // one step's operands; the next step's are read while this step's MFMAs run
    auto fetch = [&](float& a0, float& a1, float& b) {
      b = Xs[px < P ? off : zslot];           // past the chunk: A and B both 0
      a0 = As[arow * lda + px];
      a1 = As[(arow + 32) * lda + px];
      ++px;
      ++ow;
      off += g.st;
      const bool wrap = ow == g.OW;
      ow = wrap ? 0 : ow;
      off += wrap ? row_adj : 0;
    };
    float a0, a1, b;
    fetch(a0, a1, b);
    for (int t = 0; t < Ph; ++t) {
      // (the fetch after the last step reads A's pad column and the zero slot: unused)
      float na0, na1, nb;
      fetch(na0, na1, nb);
      acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b, acc1, 0, 0, 0);
      a0 = na0;
      a1 = na1;
      b = nb;
    }
  }
  // write this split's tile: C[row][col], row = (r&3) + 8*(r>>2) + 4*(lane>>5), col = lane&31
  if (!cval) return;
  float* dst = part + ((int64_t)split * g.G + grp) * (int64_t)g.Cog * g.Ncol + col;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const f32x16 acc = t == 0 ? acc0 : acc1;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = co0 + t * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      if (row < g.Cog) dst[(int64_t)row * g.Ncol] = acc[r];
    }
  }
}

// dW = the splits summed in a fixed order: wave w of a workgroup sums its quarter of the
// splits in split order (8 loads in flight per lane), then the four wave sums are added
// in wave order.  Same bits run to run; 4x the parallelism of one thread per element.
__global__ __launch_bounds__(256) void wgrad_stage2(const float* __restrict__ part, int nsplit,
                                                    int64_t n, float* __restrict__ dw) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int q = (nsplit + 3) >> 2;
  const int s0 = min(w * q, nsplit), s1 = min(s0 + q, nsplit);
  for (int64_t base = (int64_t)blockIdx.x * 64; base < n; base += (int64_t)gridDim.x * 64) {
    const int64_t i = base + lane;
    const int64_t ic = i < n ? i : n - 1;
    float a = 0.0f;
    int s = s0;
    for (; s + 8 <= s1; s += 8) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = part[(int64_t)(s + u) * n + ic];
#pragma unroll
      for (int u = 0; u < 8; ++u) a = __fadd_rn(a, v[u]);
    }
    for (; s < s1; ++s) a = __fadd_rn(a, part[(int64_t)s * n + ic]);
    red[w][lane] = a;
    __syncthreads();
    if (w == 0 && i < n)
      dw[i] = __fadd_rn(__fadd_rn(__fadd_rn(red[0][lane], red[1][lane]), red[2][lane]), red[3][lane]);
    __syncthreads();
  }
}

// Depthwise convs (one input and one output channel per group): dW[c, r, s] is a
// reduction of R*S products per output pixel over (n, oh, ow) -- no GEMM, a bandwidth-
// bound pass over x and dy (MIOpen's deterministic path for these runs at < 1 TFLOP/s,
// tools/wgrad_bench.py).  Workgroup (c, split) walks samples [n0, n0+spl) of channel c:
// the zero-padded x plane is staged in LDS (no bounds tests in the product loop), threads
// are laid over (output row, output column) once (no per-pixel division), each keeps R*S
// fp32 partials over its pixels, and the workgroup reduces them in a fixed order (wave
// shuffle tree, waves in order) into part[split][c][rs].
template <int RSMAX>
__global__ __launch_bounds__(256) void wgrad_dw_stage1(const float* __restrict__ x,
                                                       const float* __restrict__ dy, int C, int H,
                                                       int W, int OH, int OW, int R, int S,
                                                       int st, int pad, int spl,
                                                       FastDiv dWp, float* __restrict__ part) {
  extern __shared__ float xs[];  // [H + 2 pad][W + 2 pad]
  __shared__ float red[4][RSMAX];
  const int c = blockIdx.x, split = blockIdx.y;
  const int n0 = split * spl;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int RS = R * S;
  const int Hp = H + 2 * pad, Wp = W + 2 * pad;
  const int HpWp = Hp * Wp;
  // product layout: thread -> (output row o0 + k*op, output column ocw)
  const int ocols = min(OW, 256), orp = 256 / ocols;
  const int or0 = tid / ocols, ocw = tid - or0 * ocols;
  float acc[RSMAX];
#pragma unroll
  for (int j = 0; j < RSMAX; ++j) acc[j] = 0.0f;
  const int OHW = OH * OW, HW = H * W;
  for (int n = n0; n < n0 + spl; ++n) {
    const float* xp = x + ((int64_t)n * C + c) * HW;
    const float* dp = dy + ((int64_t)n * C + c) * OHW;
    __syncthreads();  // the previous sample's products are done with the plane
    // 8 loads in flight per thread, then the 8 LDS stores
    for (int e0 = tid; e0 < HpWp; e0 += 256 * 8) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int e = e0 + 256 * u;
        const int rr = (int)fdiv((uint32_t)e, dWp), cc = e - rr * Wp;
        const int ih = rr - pad, iw = cc - pad;
        const bool ok = e < HpWp && ih >= 0 && ih < H && iw >= 0 && iw < W;
        const float t = xp[ok ? ih * W + iw : 0];
        v[u] = ok ? t : 0.0f;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (e0 + 256 * u < HpWp) xs[e0 + 256 * u] = v[u];
    }
    __syncthreads();
    if (or0 < orp) {
      for (int oh = or0; oh < OH; oh += orp) {
        for (int ow = ocw; ow < OW; ow += ocols) {
          const float g = dp[oh * OW + ow];
          const float* xr = xs + oh * st * Wp + ow * st;
#pragma unroll
          for (int j = 0; j < RSMAX; ++j) {
            if (j < RS) {
              const int r = j / S, q = j - r * S;
              acc[j] = __fadd_rn(acc[j], __fmul_rn(g, xr[r * Wp + q]));
            }
          }
        }
      }
    }
  }
#pragma unroll
  for (int j = 0; j < RSMAX; ++j) {
    float v = acc[j];
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = __fadd_rn(v, __shfl_xor(v, o));
    if (lane == 0) red[w][j] = v;
  }
  __syncthreads();
  if (tid < RS)
    part[((int64_t)split * C + c) * RS + tid] =
        __fadd_rn(__fadd_rn(__fadd_rn(red[0][tid], red[1][tid]), red[2][tid]), red[3][tid]);
}

static bool is_depthwise(int64_t C, int64_t Co, int64_t G) { return G == C && G == Co && G > 1; }
static bool dw_lds_ok(int64_t H, int64_t W, int64_t pad) {
  return (H + 2 * pad) * (W + 2 * pad) * (int64_t)sizeof(float) <= 128 * 1024;
}

// depthwise plan: samples per split so that C * nsplit fills the chip (~1024 workgroups)
static int dw_splits(int64_t Nb, int64_t C, int* spl) {
  int64_t ns = std::max<int64_t>(1, std::min<int64_t>(Nb, (1024 + C - 1) / C));
  *spl = (int)((Nb + ns - 1) / ns);
  // every split must hold exactly spl samples: shrink to a divisor of Nb
  while (Nb % *spl) ++*spl;
  return (int)(Nb / *spl);
}

static int wgrad_plan(int64_t Nb, int64_t C, int64_t H, int64_t W, int64_t Co, int64_t R,
                      int64_t S, int64_t st, int64_t pad, int64_t G, WgradGeo& g,
                      size_t* lds_bytes) {
  SSQ_REQUIRE(Nb >= 1 && C >= 1 && H >= 1 && W >= 1 && Co >= 1 && R >= 1 && S >= 1 && st >= 1 &&
                  pad >= 0 && G >= 1 && C % G == 0 && Co % G == 0,
              SSQ_E_ARG, "ssq_conv_wgrad: bad geometry");
  const int64_t OH = (H + 2 * pad - R) / st + 1, OW = (W + 2 * pad - S) / st + 1;
  SSQ_REQUIRE(OH >= 1 && OW >= 1 && Nb * C * H * W < (1ll << 31) && Nb * Co * OH * OW < (1ll << 31),
              SSQ_E_ARG, "ssq_conv_wgrad: sizes");
  SSQ_REQUIRE(OW <= kMaxPx, SSQ_E_ARG, "ssq_conv_wgrad: output width %lld > %d",
              (long long)OW, kMaxPx);
  g.Nb = (int)Nb; g.C = (int)C; g.H = (int)H; g.W = (int)W; g.Co = (int)Co;
  g.OH = (int)OH; g.OW = (int)OW; g.R = (int)R; g.S = (int)S; g.st = (int)st; g.pad = (int)pad;
  g.G = (int)G; g.Cig = (int)(C / G); g.Cog = (int)(Co / G);
  g.Ncol = g.Cig * g.R * g.S;
  // channels a 128-column tile can touch: floor((kTN-1)/RS) + 2
  const int RS = g.R * g.S;
  g.ci_span = std::min(g.Cig, (kTN - 1) / RS + 2);
  // output rows per chunk: up to kMaxPx pixels, shrunk until the tile fits 64 KiB of LDS
  // (two workgroups per CU)
  g.TH = (int)std::max<int64_t>(1, std::min<int64_t>(OH, kMaxPx / OW));
  auto lds_for = [&](int th) {
    const int pp = (th * g.OW + 1) & ~1;
    return sizeof(float) * ((size_t)kTM * (pp + 1) +
                            (size_t)g.ci_span * ((th - 1) * g.st + g.R) * (g.W + 2 * g.pad) + 1);
  };
  auto xslots = [&](int th) {
    return ((size_t)g.ci_span * ((th - 1) * g.st + g.R) * (g.W + 2 * g.pad) + 255) / 256;
  };
  while (g.TH > 1 && (lds_for(g.TH) > 64 * 1024 || xslots(g.TH) > (size_t)kXSlots)) --g.TH;
  g.P = g.TH * g.OW;
  g.Pp = (g.P + 1) & ~1;
  g.chunks_per_n = (g.OH + g.TH - 1) / g.TH;
  g.nchunks = g.Nb * g.chunks_per_n;
  g.in_rows = (g.TH - 1) * g.st + g.R;
  g.div_wp = make_fastdiv((uint32_t)(g.W + 2 * g.pad));
  g.div_rows = make_fastdiv((uint32_t)g.in_rows);
  g.m_tiles = (g.Cog + kTM - 1) / kTM;
  const int n_tiles = (g.Ncol + kTN - 1) / kTN;
  const int64_t tiles = (int64_t)n_tiles * g.m_tiles * g.G;
  // enough workgroups to fill 256 CUs twice, at least 2 chunks each
  int nsplit = (int)std::max<int64_t>(1, std::min<int64_t>(g.nchunks / 2, (512 + tiles - 1) / tiles));
  g.cps = (g.nchunks + nsplit - 1) / nsplit;
  g.nsplit = (g.nchunks + g.cps - 1) / g.cps;
  *lds_bytes = lds_for(g.TH);
  SSQ_REQUIRE(*lds_bytes <= 160 * 1024, SSQ_E_ARG, "ssq_conv_wgrad: LDS tile %zu B too large",
              *lds_bytes);
  return SSQ_OK;
}

}  // namespace ssq

using namespace ssq;

extern "C" size_t ssq_conv_wgrad_workspace_size(int64_t Nb, int64_t C, int64_t H, int64_t W,
                                                int64_t Co, int64_t R, int64_t S, int64_t stride,
                                                int64_t pad, int64_t groups) {
  if (is_depthwise(C, Co, groups) && R * S <= 25 && Nb >= 1 && dw_lds_ok(H, W, pad)) {
    int spl;
    const int ns = dw_splits(Nb, C, &spl);
    return (size_t)ns * (size_t)C * (size_t)(R * S) * sizeof(float);
  }
  WgradGeo g;
  size_t lds;
  if (wgrad_plan(Nb, C, H, W, Co, R, S, stride, pad, groups, g, &lds)) return 0;
  return (size_t)g.nsplit * (size_t)Co * (size_t)g.Ncol * sizeof(float);
}

extern "C" int ssq_conv_wgrad(const float* x, const float* dy, int64_t Nb, int64_t C, int64_t H,
                              int64_t W, int64_t Co, int64_t R, int64_t S, int64_t stride,
                              int64_t pad, int64_t groups, float* dw, void* ws, size_t ws_bytes,
                              ssq_stream_t stream) {
  SSQ_REQUIRE(x && dy && dw, SSQ_E_ARG, "ssq_conv_wgrad: null pointer");
  hipStream_t s = (hipStream_t)stream;
  if (is_depthwise(C, Co, groups) && R * S <= 25 && dw_lds_ok(H, W, pad)) {
    SSQ_REQUIRE(Nb >= 1 && H >= 1 && W >= 1 && stride >= 1 && pad >= 0, SSQ_E_ARG,
                "ssq_conv_wgrad: bad geometry");
    const int64_t OH = (H + 2 * pad - R) / stride + 1, OW = (W + 2 * pad - S) / stride + 1;
    SSQ_REQUIRE(OH >= 1 && OW >= 1 && Nb * C * H * W < (1ll << 31) && Nb * C * OH * OW < (1ll << 31),
                SSQ_E_ARG, "ssq_conv_wgrad: sizes");
    int spl;
    const int ns = dw_splits(Nb, C, &spl);
    const size_t need = (size_t)ns * (size_t)C * (size_t)(R * S) * sizeof(float);
    SSQ_REQUIRE(ws && ws_bytes >= need, SSQ_E_WS, "ssq_conv_wgrad: workspace too small");
    const dim3 grid((unsigned)C, (unsigned)ns);
    const size_t lds = (size_t)(H + 2 * pad) * (W + 2 * pad) * sizeof(float);
    static bool dw_attr = false;
    if (!dw_attr) {  // dynamic LDS beyond 64 KiB must be opted into
      hipFuncSetAttribute((const void*)wgrad_dw_stage1<9>,
                          hipFuncAttributeMaxDynamicSharedMemorySize, 128 * 1024);
      hipFuncSetAttribute((const void*)wgrad_dw_stage1<25>,
                          hipFuncAttributeMaxDynamicSharedMemorySize, 128 * 1024);
      dw_attr = true;
    }
    if (R * S <= 9)
      hipLaunchKernelGGL(wgrad_dw_stage1<9>, grid, dim3(256), lds, s, x, dy, (int)C, (int)H, (int)W,
                         (int)OH, (int)OW, (int)R, (int)S, (int)stride, (int)pad, spl,
                         make_fastdiv((uint32_t)(W + 2 * pad)), (float*)ws);
    else
      hipLaunchKernelGGL(wgrad_dw_stage1<25>, grid, dim3(256), lds, s, x, dy, (int)C, (int)H, (int)W,
                         (int)OH, (int)OW, (int)R, (int)S, (int)stride, (int)pad, spl,
                         make_fastdiv((uint32_t)(W + 2 * pad)), (float*)ws);
    const int64_t n = C * R * S;
    hipLaunchKernelGGL(wgrad_stage2, dim3((unsigned)std::min<int64_t>((n + 63) / 64, 4096)),
                       dim3(256), 0, s, (const float*)ws, ns, n, dw);
    return check_launch("ssq_conv_wgrad");
  }
  WgradGeo g;
  size_t lds;
  int rc = wgrad_plan(Nb, C, H, W, Co, R, S, stride, pad, groups, g, &lds);
  if (rc) return rc;
  const size_t need = (size_t)g.nsplit * (size_t)Co * (size_t)g.Ncol * sizeof(float);
  SSQ_REQUIRE(ws && ws_bytes >= need, SSQ_E_WS, "ssq_conv_wgrad: workspace too small");
  static bool lds_attr = false;
  if (!lds_attr) {  // dynamic LDS beyond 64 KiB must be opted into
    hipFuncSetAttribute((const void*)wgrad_stage1, hipFuncAttributeMaxDynamicSharedMemorySize,
                        160 * 1024);
    lds_attr = true;
  }
  const dim3 grid((g.Ncol + kTN - 1) / kTN, g.m_tiles * g.G, g.nsplit);
  hipLaunchKernelGGL(wgrad_stage1, grid, dim3(256), lds, s, x, dy, g, (float*)ws);
  const int64_t n = (int64_t)Co * g.Ncol;
  hipLaunchKernelGGL(wgrad_stage2, dim3((unsigned)std::min<int64_t>((n + 63) / 64, 4096)),
                     dim3(256), 0, s, (const float*)ws, g.nsplit, n, dw);
  return check_launch("ssq_conv_wgrad");
}
