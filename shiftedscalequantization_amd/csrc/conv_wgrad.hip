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
//   stage 1: workgroup (n-tile, g*m-tiles, split) owns a TM x TN output tile and a fixed
//            range of K chunks; the tile is written to its split's slot of the workspace;
//   stage 2: dW = the splits summed in a fixed order.
// Same inputs -> same bits, run to run (no atomics).  Within tolerance of any other
// summation order (the MIOpen / CPU results), like every fp32 convolution gradient.
// Depthwise convs take a separate bandwidth-bound reduction (wgrad_dw_stage1).
#include <stdlib.h>

#include <algorithm>
#include <type_traits>

#include "ssq_common.h"

namespace ssq {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kUnr = 2;  // k-steps per operand group (4 LDS reads + 4 MFMAs each)

struct WgradGeo {
  int Nb, C, H, W, Co, OH, OW, R, S, st, pad, G, Cig, Cog;
  int Ncol;          // Cig*R*S
  int WM;            // waves along M (TM = 64*WM, TN = 256/WM)
  int Pq;            // output pixels per chunk (64 or 128; a sample's last chunk may be short)
  int lda;           // A row pitch in LDS: Pq + 1 (odd: conflict-free A reads)
  int chunks_per_n;  // ceil(OH*OW / Pq)
  int nchunks;       // Nb * chunks_per_n
  int cps;           // chunks per split
  int nsplit;
  int in_rows;       // x rows staged per chunk: (output rows a chunk can span - 1)*st + R
  int ci_span;       // channels staged per chunk (max over tiles)
  int xtile;         // ci_span * in_rows * (W + 2 pad)
  int m_tiles, n_tiles;
};

// Stage 1.  Workgroup (n-tile, g*m-tiles, split) owns a TM x TN tile of dW (4 waves as
// WM x (4/WM), each wave 64 x 64 = 2 x 2 v_mfma_f32_32x32x2_f32 accumulators) and the
// chunks [split*cps, ...) of K = (n, pixel): a chunk is Pq consecutive output pixels of
// one sample (row-crossing), so dy[co][chunk] is one contiguous row segment per co.
// Staging is LDS-DMA (global_load_lds, 4 B per lane, no registers): per chunk, each dy
// row segment -> A[co][0..P) and each x row the chunk touches -> X[ci][row][pad..pad+W)
// (padding columns stay zero; rows outside the image / channel range are zeroed with
// ds_write).  Two LDS buffers: chunk c+1's DMA is issued before chunk c's MFMAs and
// retired (vmcnt(0) + barrier) before they are read.  A k-step gives each lane two A
// values (rows lane&31, +32) and two gathered B values (columns lane&31, +32) for four
// MFMAs; the lane halves walk disjoint halves of the chunk (the MFMA's k = 0 / 1), so a
// lane's pixel advances by one per step and its x offset incrementally.  Operand groups of
// kUnr steps are read one group ahead of the MFMAs that use them.
template <int WM>
__global__ __launch_bounds__(256, 1) void wgrad_stage1(const float* __restrict__ x,
                                                    const float* __restrict__ dy, WgradGeo g,
                                                    float* __restrict__ part) {
  constexpr int WN = 4 / WM, TM = 64 * WM, TN = 64 * WN;
  extern __shared__ float lds[];
  const int Pq = g.Pq, lda = g.lda;
  const int Wp = g.W + 2 * g.pad;
  const int xbuf = g.xtile + 1;                    // + zero slot
  float* Abuf = lds;                               // [2][TM][lda]
  float* Xbuf = lds + 2 * TM * lda;                // [2][xtile + 1]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave - wm * WN;
  const int grp = blockIdx.y / g.m_tiles, mt = blockIdx.y - grp * g.m_tiles;
  const int split = blockIdx.z;
  const int co0 = mt * TM;                         // within the group
  const int col0 = blockIdx.x * TN;
  const int RS = g.R * g.S;
  const int ci_lo = col0 / RS;
  const int wrow = co0 + wm * 64, wcol = col0 + wn * 64;
  int xb[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    // a column past Ncol gathers from the tile's first column (in range, result unused)
    const int col = wcol + 32 * j + (lane & 31);
    const int c = col < g.Ncol ? col : ci_lo * RS;
    const int ci = c / RS, rs = c - ci * RS;
    const int r = rs / g.S;
    xb[j] = ((ci - ci_lo) * g.in_rows + r) * Wp + (rs - r * g.S);
  }
  const int half = lane >> 5;
  const int arow = (wm * 64 + (lane & 31)) * lda;
  const int OHW = g.OH * g.OW, HW = g.H * g.W;
  const int row_adj = g.st * Wp - g.OW * g.st;     // x offset change when ow wraps
  const int c_begin = split * g.cps, c_end = min(c_begin + g.cps, g.nchunks);
  const int nrows_x = g.ci_span * g.in_rows;

  // both buffers zeroed once: A rows past Cog, X padding columns and the zero slot are
  // never written by the DMA (a short chunk's A tail and out-of-image X rows are zeroed
  // per chunk below)
  for (int i = tid; i < 2 * TM * lda + 2 * xbuf; i += 256) lds[i] = 0.0f;
  __syncthreads();

  // chunk c -> (sample, first pixel, pixel count, first output row)
  auto chunk_geo = [&](int c, int& n, int& p0, int& P, int& oh_first) {
    n = c / g.chunks_per_n;
    p0 = (c - n * g.chunks_per_n) * Pq;
    P = min(Pq, OHW - p0);
    oh_first = p0 / g.OW;
  };
  auto stage = [&](int c, int b) {
    int n, p0, P, oh_first;
    chunk_geo(c, n, p0, P, oh_first);
    float* A = Abuf + b * TM * lda;
    float* X = Xbuf + b * xbuf;
    // dy: row r (co0 + r < Cog) -> A[r][0..P); a short chunk's tail columns -> 0
    const float* sa = dy + ((int64_t)n * g.Co + (int64_t)grp * g.Cog + co0) * OHW + p0;
    const int rows = min(TM, g.Cog - co0);
    for (int r = wave; r < rows; r += 4) {
      for (int k0 = 0; k0 < Pq; k0 += 64) {
        const int k = k0 + lane;
        if (k < P)
          __builtin_amdgcn_global_load_lds((const void*)(sa + (int64_t)r * OHW + k),
                                           (void*)(A + r * lda + k0), 4, 0, 0);
        else if (k < Pq)
          A[r * lda + k] = 0.0f;
      }
    }
    // x: staged row q = (cl, rr) -> channel ci_lo + cl, input row ih0 + rr
    const int ih0 = oh_first * g.st - g.pad;
    const float* sx = x + ((int64_t)n * g.C + (int64_t)grp * g.Cig) * HW;
    for (int q = wave; q < nrows_x; q += 4) {
      const int cl = q / g.in_rows, rr = q - cl * g.in_rows;
      const int ci = ci_lo + cl, ih = ih0 + rr;
      float* drow = X + q * Wp + g.pad;
      const bool ok = ci < g.Cig && ih >= 0 && ih < g.H;
      for (int k0 = 0; k0 < g.W; k0 += 64) {
        const int k = k0 + lane;
        if (k < g.W) {
          if (ok)
            __builtin_amdgcn_global_load_lds(
                (const void*)(sx + (int64_t)ci * HW + (int64_t)ih * g.W + k),
                (void*)(drow + k0), 4, 0, 0);
          else
            drow[k] = 0.0f;
        }
      }
    }
  };

  f32x16 acc00 = {0}, acc01 = {0}, acc10 = {0}, acc11 = {0};
  if (c_begin < c_end) stage(c_begin, 0);
  for (int c = c_begin; c < c_end; ++c) {
    const int b = (c - c_begin) & 1;
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __syncthreads();                  // chunk c staged; chunk c-1's reads of buffer b^1 done
    if (c + 1 < c_end) stage(c + 1, b ^ 1);
    int n, p0, P, oh_first;
    chunk_geo(c, n, p0, P, oh_first);
    const float* As = Abuf + b * TM * lda;
    const float* Xs = Xbuf + b * xbuf;
    const int zslot = g.xtile;        // Xs[zslot] = 0: B past the chunk's pixels
    // k-steps of this chunk: its P pixels in two lane halves, rounded up to kUnr
    const int Ph = ((P + 1) / 2 + kUnr - 1) / kUnr * kUnr;
    int px = half * Ph;
    int ow, off;
    {
      const int pix = p0 + px;
      const int oh = pix / g.OW;
      ow = pix - oh * g.OW;
      off = (oh - oh_first) * g.st * Wp + ow * g.st;
    }
    float A0[kUnr], A1[kUnr], B0[kUnr], B1[kUnr];
    auto fetch = [&](int u) {
      const bool in = px < P;
      B0[u] = Xs[in ? xb[0] + off : zslot];
      B1[u] = Xs[in ? xb[1] + off : zslot];
      A0[u] = As[arow + px];
      A1[u] = As[arow + 32 * lda + px];
      ++px;
      ++ow;
      off += g.st;
      const bool wrap = ow == g.OW;
      ow = wrap ? 0 : ow;
      off += wrap ? row_adj : 0;
    };
#pragma unroll
    for (int u = 0; u < kUnr; ++u) fetch(u);
    for (int t = 0; t < Ph; t += kUnr) {
      float a0[kUnr], a1[kUnr], b0[kUnr], b1[kUnr];
#pragma unroll
      for (int u = 0; u < kUnr; ++u) {
        a0[u] = A0[u];
        a1[u] = A1[u];
        b0[u] = B0[u];
        b1[u] = B1[u];
      }
      // next group's operands (none after the last group)
      if (t + kUnr < Ph) {
#pragma unroll
        for (int u = 0; u < kUnr; ++u) fetch(u);
      }
#pragma unroll
      for (int u = 0; u < kUnr; ++u) {
        acc00 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[u], b0[u], acc00, 0, 0, 0);
        acc01 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[u], b1[u], acc01, 0, 0, 0);
        acc10 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[u], b0[u], acc10, 0, 0, 0);
        acc11 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[u], b1[u], acc11, 0, 0, 0);
      }
    }
  }
  // this split's tile: C[row][col], row = (r&3) + 8*(r>>2) + 4*(lane>>5), col = lane&31
  float* dst = part + ((int64_t)split * g.G + grp) * (int64_t)g.Cog * g.Ncol;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const f32x16 acc = t == 0 ? acc00 : t == 1 ? acc01 : t == 2 ? acc10 : acc11;
    const int col = wcol + 32 * (t & 1) + (lane & 31);
    if (col >= g.Ncol) continue;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = wrow + 32 * (t >> 1) + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      if (row < g.Cog) dst[(int64_t)row * g.Ncol + col] = acc[r];
    }
  }
}

// ------------------------------------------------------------------ 1x1 convolutions
// A 1x1 conv's weight gradient is a plain GEMM, dW[co, ci] = sum_(n, p) dy[n, co, p] *
// x[n, ci, src(p)], src(p) = (p / OW) * st * W + (p % OW) * st: no window, so instead of the
// R x S input-row tile both operands are staged the same way -- per chunk of Pq1 output
// pixels of one sample, A[co][k] = dy rows (contiguous) and B[ci][k] = x at src(p) (a
// strided gather for stride 2), LDS-DMA'd 4 B per lane into two buffers.  Waves tile the
// workgroup's TM x TN block as 64 x 64 (2 x 2 v_mfma_f32_32x32x2_f32 accumulators, exact
// fp32); lane half h walks pixels h*Pq1/2 + t of the chunk (the MFMA's k = h), so both
// operands are read with the same conflict-free pitch.  Splits over chunks, summed in a
// fixed order by wgrad_stage2: deterministic.  (The R x S kernel's x tile needs
// ci_span * in_rows * W floats; at 56x56 stride 2 that overflows the LDS.)
constexpr int kPq1 = 64;
constexpr int kLd1 = kPq1 + 1;     // odd pitch: row r, column c -> bank (r + c) mod 32-ish

struct W1Geo {
  int Nb, C, HW, W, Co, OW, OHW, st, G, Cig, Cog;
  int WM, m_tiles, n_tiles, chunks_per_n, nchunks, cps, nsplit;
  FastDiv dOW;
};

template <int WM>
__global__ __launch_bounds__(256) void wgrad_1x1_stage1(const float* __restrict__ x,
                                                        const float* __restrict__ dy, W1Geo g,
                                                        float* __restrict__ part) {
  constexpr int WN = 4 / WM, TM = 64 * WM, TN = 64 * WN;
  __shared__ float lds[2 * (TM + TN) * kLd1];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave - wm * WN;
  const int grp = blockIdx.y / g.m_tiles, mt = blockIdx.y - grp * g.m_tiles;
  const int co0 = mt * TM, ci0 = blockIdx.x * TN;
  const int rows_a = min(TM, g.Cog - co0), rows_b = min(TN, g.Cig - ci0);
  const int c_begin = blockIdx.z * g.cps, c_end = min(c_begin + g.cps, g.nchunks);
  // buffer b: A = lds + b*(TM+TN)*kLd1 [TM][kLd1], B right after it [TN][kLd1]
  auto Abuf = [&](int b) { return lds + b * (TM + TN) * kLd1; };
  auto Bbuf = [&](int b) { return lds + b * (TM + TN) * kLd1 + TM * kLd1; };
  // rows past the channel ranges stay zero (their products are discarded anyway)
  for (int i = tid; i < 2 * (TM + TN) * kLd1; i += 256) lds[i] = 0.0f;
  __syncthreads();

  auto stage = [&](int c, int b) {
    const int n = c / g.chunks_per_n;
    const int p0 = (c - n * g.chunks_per_n) * kPq1;
    const int P = min(kPq1, g.OHW - p0);
    const int k = lane;
    const float* sa = dy + ((int64_t)n * g.Co + (int64_t)grp * g.Cog + co0) * g.OHW + p0;
    for (int r = wave; r < rows_a; r += 4) {
      if (k < P)
        __builtin_amdgcn_global_load_lds((const void*)(sa + (int64_t)r * g.OHW + k),
                                         (void*)(Abuf(b) + r * kLd1), 4, 0, 0);
      else
        Abuf(b)[r * kLd1 + k] = 0.0f;
    }
    const int p = p0 + k;
    const int oh = (int)fdiv((uint32_t)p, g.dOW), ow = p - oh * g.OW;
    const int src = oh * g.st * g.W + ow * g.st;
    const float* sb = x + ((int64_t)n * g.C + (int64_t)grp * g.Cig + ci0) * g.HW + src;
    for (int r = wave; r < rows_b; r += 4) {
      if (k < P)
        __builtin_amdgcn_global_load_lds((const void*)(sb + (int64_t)r * g.HW),
                                         (void*)(Bbuf(b) + r * kLd1), 4, 0, 0);
      else
        Bbuf(b)[r * kLd1 + k] = 0.0f;
    }
  };

  f32x16 acc00 = {0}, acc01 = {0}, acc10 = {0}, acc11 = {0};
  const int ar = (wm * 64 + (lane & 31)) * kLd1, br = (wn * 64 + (lane & 31)) * kLd1;
  const int kh = (lane >> 5) * (kPq1 / 2);
  if (c_begin < c_end) stage(c_begin, 0);
  for (int c = c_begin; c < c_end; ++c) {
    const int b = (c - c_begin) & 1;
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __syncthreads();                  // chunk c staged; chunk c-1's reads of buffer b^1 done
    if (c + 1 < c_end) stage(c + 1, b ^ 1);
    const float* A = Abuf(b);
    const float* B = Bbuf(b);
#pragma unroll 4
    for (int t = 0; t < kPq1 / 2; ++t) {
      const float a0 = A[ar + kh + t], a1 = A[ar + 32 * kLd1 + kh + t];
      const float b0 = B[br + kh + t], b1 = B[br + 32 * kLd1 + kh + t];
      acc00 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc00, 0, 0, 0);
      acc01 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc01, 0, 0, 0);
      acc10 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc10, 0, 0, 0);
      acc11 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc11, 0, 0, 0);
    }
  }
  // C[row][col], row = (r&3) + 8*(r>>2) + 4*(lane>>5), col = lane&31 (as wgrad_stage1)
  float* dst = part + ((int64_t)blockIdx.z * g.G + grp) * (int64_t)g.Cog * g.Cig;
  const int wrow = co0 + wm * 64, wcol = ci0 + wn * 64;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const f32x16 acc = t == 0 ? acc00 : t == 1 ? acc01 : t == 2 ? acc10 : acc11;
    const int col = wcol + 32 * (t & 1) + (lane & 31);
    if (col >= g.Cig) continue;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = wrow + 32 * (t >> 1) + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      if (row < g.Cog) dst[(int64_t)row * g.Cig + col] = acc[r];
    }
  }
}

static int wgrad_1x1_plan(int64_t Nb, int64_t C, int64_t H, int64_t W, int64_t Co, int64_t st,
                          int64_t G, W1Geo& g) {
  SSQ_REQUIRE(Nb >= 1 && C >= 1 && H >= 1 && W >= 1 && Co >= 1 && st >= 1 && G >= 1 &&
                  C % G == 0 && Co % G == 0,
              SSQ_E_ARG, "ssq_conv_wgrad: bad geometry");
  const int64_t OH = (H - 1) / st + 1, OW = (W - 1) / st + 1;
  SSQ_REQUIRE(Nb * C * H * W < (1ll << 31) && Nb * Co * OH * OW < (1ll << 31), SSQ_E_ARG,
              "ssq_conv_wgrad: sizes");
  g.Nb = (int)Nb; g.C = (int)C; g.HW = (int)(H * W); g.W = (int)W; g.Co = (int)Co;
  g.OW = (int)OW; g.OHW = (int)(OH * OW); g.st = (int)st; g.G = (int)G;
  g.Cig = (int)(C / G); g.Cog = (int)(Co / G);
  g.dOW = make_fastdiv((uint32_t)OW);
  // 128 x 128 workgroup tile: its two (TM + TN) x kLd1 buffers (133 KB) fit the LDS,
  // the 64 x 256 forms' do not
  g.WM = 2;
  const int TM = 64 * g.WM, TN = 256 / g.WM;
  g.m_tiles = (g.Cog + TM - 1) / TM;
  g.n_tiles = (g.Cig + TN - 1) / TN;
  g.chunks_per_n = (g.OHW + kPq1 - 1) / kPq1;
  g.nchunks = g.Nb * g.chunks_per_n;
  const int64_t tiles = (int64_t)g.m_tiles * g.n_tiles * g.G;
  // ~2 workgroups per CU over the grid, at least 4 chunks each
  int nsplit = (int)std::max<int64_t>(1, std::min<int64_t>(g.nchunks / 4, (512 + tiles - 1) / tiles));
  g.cps = (g.nchunks + nsplit - 1) / nsplit;
  g.nsplit = (g.nchunks + g.cps - 1) / g.cps;
  return SSQ_OK;
}

// ------------------------------------------------------------------ im2col-DMA form
// Any R x S / stride / padding, as one implicit GEMM whose K = (n, output pixel) runs
// across samples: a chunk is kPqI consecutive k.  Per chunk each lane owns one k (its
// sample, output row/column computed once) and both operands are gathered by LDS-DMA with
// per-lane global addresses straight into GEMM layout -- A[co][k] = dy[n, co, p] and
// B[col][k] = x[n, ci, oh*st + r - pad, ow*st + s - pad] for col = (ci, r, s); taps that
// fall in the padding (and k past the end) read a zero page, so no LDS row is written by
// anything but the DMA.  Rows are padded to a pitch of kPqI + 2 floats: every lane's
// ds_read_b64 of two consecutive k (two MFMA k-steps) is bank-conflict-free.  Two 66 KB
// buffers per workgroup (a 32-pixel chunk with two workgroups per CU measured 1.5-2x
// slower: the per-lane gather DMA issue, not the MFMA, set the pace).  Waves tile the workgroup block as
// 64 x 64 (2 x 2 v_mfma_f32_32x32x2_f32, exact fp32); splits over chunks, summed in a
// fixed order by wgrad_stage2: deterministic.
constexpr int kPqI = 64;
constexpr int kLdI = kPqI + 2;
__device__ float g_wgrad_zero_page[64];   // zero-initialised, never written

struct I2cGeo {
  int C, H, W, Co, OW, OHW, S, RS, st, pad, G, Cig, Cog, Ncol;
  int64_t K;
  int m_tiles, n_tiles, cps, nsplit;
  int64_t nchunks;
  FastDiv dOHW, dOW, dRS, dS;
};

template <int WM>
__global__ __launch_bounds__(256) void wgrad_i2c_stage1(const float* __restrict__ x,
                                                           const float* __restrict__ dy,
                                                           I2cGeo g, float* __restrict__ part) {
  constexpr int WN = 4 / WM, TM = 64 * WM, TN = 64 * WN, ROWS = TM + TN;
  __shared__ float lds[2 * ROWS * kLdI];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave - wm * WN;
  const int grp = blockIdx.y / g.m_tiles, mt = blockIdx.y - grp * g.m_tiles;
  const int co0 = mt * TM, col0 = blockIdx.x * TN;
  const int64_t c_begin = (int64_t)blockIdx.z * g.cps;
  const int64_t c_end = min(c_begin + g.cps, g.nchunks);
  const float* zero = g_wgrad_zero_page;
  const float* xg = x + (int64_t)grp * g.Cig * g.H * g.W;
  const float* dyg = dy + (int64_t)grp * g.Cog * g.OHW;
  const int64_t xs_n = (int64_t)g.C * g.H * g.W, dys_n = (int64_t)g.Co * g.OHW;

  auto stage = [&](int64_t c, int b) {
    if (lane >= kPqI) return;
    const int64_t k = c * kPqI + lane;
    const bool kin = k < g.K;
    const uint32_t kk = kin ? (uint32_t)k : 0u;
    const int n = (int)fdiv(kk, g.dOHW), p = (int)kk - n * g.OHW;
    const int oh = (int)fdiv((uint32_t)p, g.dOW), ow = p - oh * g.OW;
    const int ih0 = oh * g.st - g.pad, iw0 = ow * g.st - g.pad;
    const float* arow = dyg + n * dys_n + p;
    const float* xrow = xg + n * xs_n;
    float* dst = lds + (size_t)b * ROWS * kLdI;
    for (int rr = wave; rr < ROWS; rr += 4) {
      const float* src;
      if (rr < TM) {
        const int co = co0 + rr;
        src = (kin && co < g.Cog) ? arow + (int64_t)co * g.OHW : zero;
      } else {
        const int col = col0 + rr - TM;
        const int ci = (int)fdiv((uint32_t)col, g.dRS), rs = col - ci * g.RS;
        const int r = (int)fdiv((uint32_t)rs, g.dS), sc = rs - r * g.S;
        const int ih = ih0 + r, iw = iw0 + sc;
        const bool ok = kin && col < g.Ncol && ih >= 0 && ih < g.H && iw >= 0 && iw < g.W;
        src = ok ? xrow + ((int64_t)ci * g.H + ih) * g.W + iw : zero;
      }
      __builtin_amdgcn_global_load_lds((const void*)src, (void*)(dst + rr * kLdI), 4, 0, 0);
    }
  };

  f32x16 acc00 = {0}, acc01 = {0}, acc10 = {0}, acc11 = {0};
  const int h = lane >> 5;
  const int ar = (wm * 64 + (lane & 31)) * kLdI + h * (kPqI / 2);
  const int br = (TM + wn * 64 + (lane & 31)) * kLdI + h * (kPqI / 2);
  if (c_begin < c_end) stage(c_begin, 0);
  for (int64_t c = c_begin; c < c_end; ++c) {
    const int b = (int)((c - c_begin) & 1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();                  // chunk c staged; chunk c-1's reads of buffer b^1 done
    if (c + 1 < c_end) stage(c + 1, b ^ 1);
    const float* L = lds + (size_t)b * ROWS * kLdI;
#pragma unroll
    for (int u = 0; u < kPqI / 4; ++u) {
      typedef float f32x2 __attribute__((ext_vector_type(2)));
      const f32x2 a0 = *(const f32x2*)(L + ar + 2 * u);
      const f32x2 a1 = *(const f32x2*)(L + ar + 32 * kLdI + 2 * u);
      const f32x2 b0 = *(const f32x2*)(L + br + 2 * u);
      const f32x2 b1 = *(const f32x2*)(L + br + 32 * kLdI + 2 * u);
      acc00 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0.x, b0.x, acc00, 0, 0, 0);
      acc01 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0.x, b1.x, acc01, 0, 0, 0);
      acc10 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1.x, b0.x, acc10, 0, 0, 0);
      acc11 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1.x, b1.x, acc11, 0, 0, 0);
      acc00 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0.y, b0.y, acc00, 0, 0, 0);
      acc01 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0.y, b1.y, acc01, 0, 0, 0);
      acc10 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1.y, b0.y, acc10, 0, 0, 0);
      acc11 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1.y, b1.y, acc11, 0, 0, 0);
    }
  }
  float* dst = part + ((int64_t)blockIdx.z * g.G + grp) * (int64_t)g.Cog * g.Ncol;
  const int wrow = co0 + wm * 64, wcol = col0 + wn * 64;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const f32x16 acc = t == 0 ? acc00 : t == 1 ? acc01 : t == 2 ? acc10 : acc11;
    const int col = wcol + 32 * (t & 1) + (lane & 31);
    if (col >= g.Ncol) continue;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = wrow + 32 * (t >> 1) + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      if (row < g.Cog) dst[(int64_t)row * g.Ncol + col] = acc[r];
    }
  }
}

static int wgrad_i2c_plan(int64_t Nb, int64_t C, int64_t H, int64_t W, int64_t Co, int64_t R,
                          int64_t S, int64_t st, int64_t pad, int64_t G, I2cGeo& g) {
  SSQ_REQUIRE(Nb >= 1 && C >= 1 && H >= 1 && W >= 1 && Co >= 1 && R >= 1 && S >= 1 && st >= 1 &&
                  pad >= 0 && G >= 1 && C % G == 0 && Co % G == 0,
              SSQ_E_ARG, "ssq_conv_wgrad: bad geometry");
  const int64_t OH = (H + 2 * pad - R) / st + 1, OW = (W + 2 * pad - S) / st + 1;
  SSQ_REQUIRE(OH >= 1 && OW >= 1 && Nb * C * H * W < (1ll << 31) &&
                  Nb * Co * OH * OW < (1ll << 31),
              SSQ_E_ARG, "ssq_conv_wgrad: sizes");
  g.C = (int)C; g.H = (int)H; g.W = (int)W; g.Co = (int)Co; g.OW = (int)OW;
  g.OHW = (int)(OH * OW); g.S = (int)S; g.RS = (int)(R * S); g.st = (int)st; g.pad = (int)pad;
  g.G = (int)G; g.Cig = (int)(C / G); g.Cog = (int)(Co / G);
  g.Ncol = g.Cig * g.RS;
  g.K = Nb * OH * OW;
  g.dOHW = make_fastdiv((uint32_t)g.OHW);
  g.dOW = make_fastdiv((uint32_t)OW);
  g.dRS = make_fastdiv((uint32_t)g.RS);
  g.dS = make_fastdiv((uint32_t)S);
  g.nchunks = (g.K + kPqI - 1) / kPqI;
  return SSQ_OK;
}

// workgroup tile (64 WM x 256 / WM) wasting the fewest MFMA slots on padding, then the
// split count: ~4 workgroups per CU over the grid, partials bounded to ~16 MB
static void wgrad_i2c_tiles(I2cGeo& g, int* wm_out) {
  int64_t best = INT64_MAX;
  int wmb = 2;
  for (int wm : {2}) {
    const int64_t TM = 64 * wm, TN = 256 / wm;
    const int64_t cost = ((g.Cog + TM - 1) / TM) * ((g.Ncol + TN - 1) / TN) * TM * TN;
    if (cost < best) {
      best = cost;
      wmb = wm;
    }
  }
  *wm_out = wmb;
  const int TM = 64 * wmb, TN = 256 / wmb;
  g.m_tiles = (g.Cog + TM - 1) / TM;
  g.n_tiles = (g.Ncol + TN - 1) / TN;
  const int64_t tiles = (int64_t)g.m_tiles * g.n_tiles * g.G;
  const int64_t by_grid = (1024 + tiles - 1) / tiles;
  const int64_t by_mem = std::max<int64_t>(1, (4ll << 20) / ((int64_t)g.Co * g.Ncol));
  int64_t ns = std::min<int64_t>(by_grid, by_mem);
  ns = std::max<int64_t>(1, std::min<int64_t>(ns, g.nchunks / 4));
  g.cps = (int)((g.nchunks + ns - 1) / ns);
  g.nsplit = (int)((g.nchunks + g.cps - 1) / g.cps);
}

// dW = the splits summed in a fixed order: wave w of a workgroup sums its quarter of the
// splits in split order (8 loads in flight per lane), then the four wave sums are added
// in wave order.  Same bits run to run; 4x the parallelism of one thread per element.
__global__ __launch_bounds__(256) void wgrad_stage2(const float* __restrict__ part, int nsplit,
                                                    int64_t n, float* __restrict__ dw,
                                                    int64_t perm_inner = 0, int perm_rs = 0) {
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
    if (w == 0 && i < n) {
      // perm_rs > 0: part is [split][tap][co*ci] (band form), dW is [co*ci][tap]
      int64_t o = i;
      if (perm_rs > 0) {
        const int64_t t = i / perm_inner;
        o = (i - t * perm_inner) * perm_rs + t;
      }
      dw[o] = __fadd_rn(__fadd_rn(__fadd_rn(red[0][lane], red[1][lane]), red[2][lane]), red[3][lane]);
    }
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
constexpr int kPf = 8;  // dy loads in flight per thread in the depthwise product loops

template <int RSMAX>
__global__ __launch_bounds__(256) void wgrad_dw_stage1(const float* __restrict__ x,
                                                       const float* __restrict__ dy, int C, int H,
                                                       int W, int OH, int OW, int R, int S,
                                                       int st, int pad, int spl, int bh,
                                                       int nbands, FastDiv dWp,
                                                       float* __restrict__ part) {
  extern __shared__ float xs[];  // the band's padded input rows [(bh - 1) st + R][W + 2 pad]
  __shared__ float red[4][RSMAX];
  const int c = blockIdx.x, split = blockIdx.y / nbands, band = blockIdx.y - split * nbands;
  const int n0 = split * spl;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int RS = R * S;
  const int Wp = W + 2 * pad;
  const int oh_lo = band * bh, oh_hi = min(OH, oh_lo + bh);
  const int prow0 = oh_lo * st;  // first padded input row of the band
  const int HpWp = ((oh_hi - 1) * st + R - prow0) * Wp;  // elements staged per sample
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
    __syncthreads();  // the previous sample's products are done with the rows
    // 8 loads in flight per thread, then the 8 LDS stores
    for (int e0 = tid; e0 < HpWp; e0 += 256 * 8) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int e = e0 + 256 * u;
        const int rr = (int)fdiv((uint32_t)e, dWp), cc = e - rr * Wp;
        const int ih = prow0 + rr - pad, iw = cc - pad;
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
      // the dy values of kPf rows are loaded together: one load latency per kPf products
      for (int ow = ocw; ow < OW; ow += ocols) {
        for (int oh0 = oh_lo + or0; oh0 < oh_hi; oh0 += kPf * orp) {
          float g[kPf];
#pragma unroll
          for (int k = 0; k < kPf; ++k) {
            const int oh = oh0 + k * orp;
            g[k] = 0.0f;
            if (oh < oh_hi) g[k] = dp[oh * OW + ow];
          }
#pragma unroll 1
          for (int k = 0; k < kPf; ++k) {  // rolled (g shifts down): no hoisted LDS reads
            const int oh = oh0 + k * orp;
            if (oh >= oh_hi) break;
            const float* xr = xs + (oh * st - prow0) * Wp + ow * st;
#pragma unroll
            for (int j = 0; j < RSMAX; ++j) {
              if (j < RS) {
                const int r = j / S, q = j - r * S;
                acc[j] = __fadd_rn(acc[j], __fmul_rn(g[0], xr[r * Wp + q]));
              }
            }
#pragma unroll
            for (int t = 0; t + 1 < kPf; ++t) g[t] = g[t + 1];
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
    part[((int64_t)blockIdx.y * C + c) * RS + tid] =
        __fadd_rn(__fadd_rn(__fadd_rn(red[0][tid], red[1][tid]), red[2][tid]), red[3][tid]);
}

// Depthwise weight gradient on small planes (<= 4 KiB padded: 28x28 and below), where a
// sample's plane is too few products (49 on 7x7) to hide a load round trip per sample:
// workgroup (c, split) stages nb samples' zero-padded x planes per pass (16 loads in flight
// per thread, one barrier pair per pass) and lays its threads over (sample, pixel); dy is
// read straight from global memory, one independent load per product row.  Partials and
// their fixed-order reduction as wgrad_dw_stage1.
template <int RSMAX>
__global__ __launch_bounds__(256) void wgrad_dw_small(const float* __restrict__ x,
                                                      const float* __restrict__ dy, int C, int H,
                                                      int W, int OH, int OW, int R, int S, int st,
                                                      int pad, int spl, int nb, FastDiv dWp,
                                                      FastDiv dP, FastDiv dOHW, FastDiv dOW,
                                                      float* __restrict__ part) {
  extern __shared__ float xs[];  // [nb][H + 2 pad][W + 2 pad]
  __shared__ float red[4][RSMAX];
  const int c = blockIdx.x, split = blockIdx.y;
  const int n0 = split * spl;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int RS = R * S;
  const int Wp = W + 2 * pad, HpWp = (H + 2 * pad) * Wp;
  const int OHW = OH * OW, HW = H * W;
  constexpr int U = 8;
  float acc[RSMAX];
#pragma unroll
  for (int j = 0; j < RSMAX; ++j) acc[j] = 0.0f;
  for (int n = n0; n < n0 + spl; n += nb) {
    const int cnt = min(nb, n0 + spl - n);
    const float* xb = x + ((int64_t)n * C + c) * HW;
    const float* db = dy + ((int64_t)n * C + c) * OHW;
    const int tot = cnt * HpWp, totp = cnt * OHW;
    __syncthreads();  // the previous pass's products are done with the planes
    for (int e0 = tid; e0 < tot; e0 += 256 * U) {
      float v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int e = e0 + 256 * u;
        const int j = (int)fdiv((uint32_t)e, dP), rem = e - j * HpWp;
        const int rr = (int)fdiv((uint32_t)rem, dWp), cc = rem - rr * Wp;
        const int ih = rr - pad, iw = cc - pad;
        v[u] = 0.0f;  // padding and slots past the pass issue no load
        if (e < tot && ih >= 0 && ih < H && iw >= 0 && iw < W) v[u] = xb[(int64_t)j * C * HW + ih * W + iw];
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (e0 + 256 * u < tot) xs[e0 + 256 * u] = v[u];
    }
    __syncthreads();
    for (int p0 = tid; p0 < totp; p0 += 256 * kPf) {
      float g[kPf];
#pragma unroll
      for (int k = 0; k < kPf; ++k) {  // the dy values of kPf pixels in one load round
        const int p = p0 + 256 * k;
        const int j = (int)fdiv((uint32_t)p, dOHW);
        g[k] = 0.0f;
        if (p < totp) g[k] = db[(int64_t)j * C * OHW + (p - j * OHW)];
      }
#pragma unroll 1
      for (int k = 0; k < kPf; ++k) {  // rolled (g shifts down): no hoisted LDS reads
        const int p = p0 + 256 * k;
        if (p >= totp) break;
        const int j = (int)fdiv((uint32_t)p, dOHW), q = p - j * OHW;
        const int oh = (int)fdiv((uint32_t)q, dOW), ow = q - oh * OW;
        const float* xr = xs + j * HpWp + oh * st * Wp + ow * st;
#pragma unroll
        for (int kk = 0; kk < RSMAX; ++kk) {
          if (kk < RS) {
            const int r = kk / S, q2 = kk - r * S;
            acc[kk] = __fadd_rn(acc[kk], __fmul_rn(g[0], xr[r * Wp + q2]));
          }
        }
#pragma unroll
        for (int t = 0; t + 1 < kPf; ++t) g[t] = g[t + 1];
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
// samples staged per pass by wgrad_dw_small (0: the plane is over 4 KiB, wgrad_dw_stage1)
static int dw_stage(int64_t H, int64_t W, int64_t pad, int spl) {
  const int64_t b = (H + 2 * pad) * (W + 2 * pad) * (int64_t)sizeof(float);
  if (b > 4096) return 0;
  return (int)std::max<int64_t>(1, std::min<int64_t>(spl, 32 * 1024 / b));
}
// output rows per band of wgrad_dw_stage1: planes over 8 KiB are cut into row bands of
// <= 8 KiB of staged input each (more, smaller workgroups: a 112x112 plane is 8 bands)
static int dw_band_rows(int64_t H, int64_t W, int64_t R, int64_t st, int64_t pad, int64_t OH) {
  const int64_t Wp = W + 2 * pad, row = Wp * (int64_t)sizeof(float);
  if ((H + 2 * pad) * row <= 8192) return (int)OH;
  const int64_t rows = std::max<int64_t>(R, 8192 / row);
  return (int)std::min<int64_t>(OH, (rows - R) / st + 1);
}
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

static size_t wgrad_lds(int wm, int pq, int64_t xtile) {
  return sizeof(float) * (2 * (size_t)(64 * wm) * (pq + 1) + 2 * (size_t)(xtile + 1));
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
  g.Nb = (int)Nb; g.C = (int)C; g.H = (int)H; g.W = (int)W; g.Co = (int)Co;
  g.OH = (int)OH; g.OW = (int)OW; g.R = (int)R; g.S = (int)S; g.st = (int)st; g.pad = (int)pad;
  g.G = (int)G; g.Cig = (int)(C / G); g.Cog = (int)(Co / G);
  g.Ncol = g.Cig * g.R * g.S;
  const int RS = g.R * g.S;
  const int64_t Wp = W + 2 * pad;
  // Candidate layouts WM = 1, 2, 4 (TM = 64 WM, TN = 256 / WM) x Pq = 128, 64, in MFMA
  // slots (64 cycles): every tile runs 2 MFMAs per pixel per wave, plus per chunk a fixed
  // ~40 and one slot per LDS-DMA instruction a wave issues (A rows + x rows, / 4 waves).
  // A/B knob: SSQ_K17_MAXLDS caps the LDS tile (bytes) -- 80 KiB lets two workgroups share
  // a CU (8 waves: twice the latency hiding of one)
  static const int64_t max_lds = [] {
    const char* v = getenv("SSQ_K17_MAXLDS");
    return (int64_t)(v && *v ? atoll(v) : 160 * 1024);
  }();
  double best = 1e300;
  for (int wm : {1, 2, 4}) {
    for (int pq : {128, 64}) {
      const int TM = 64 * wm, TN = 256 / wm;
      const int64_t span = std::min<int64_t>(g.Cig, (TN - 1) / RS + 2);
      const int64_t orows = (pq - 1 + OW - 1) / OW + 1;     // output rows a chunk can span
      const int64_t in_rows = (orows - 1) * st + R;
      const int64_t xtile = span * in_rows * Wp;
      if ((int64_t)wgrad_lds(wm, pq, xtile) > max_lds) continue;
      const int64_t cpn = (OH * OW + pq - 1) / pq;
      const int64_t tiles = ((g.Cog + TM - 1) / TM) * ((g.Ncol + TN - 1) / TN);
      const double dma = (double)(std::min<int64_t>(TM, g.Cog) * ((pq + 63) / 64) +
                                  span * in_rows * ((W + 63) / 64)) / 4.0;
      const double cost = (double)tiles * Nb * (2.0 * OH * OW + cpn * (40.0 + dma));
      if (cost < best) {
        best = cost;
        g.WM = wm;
        g.Pq = pq;
        g.ci_span = (int)span;
        g.in_rows = (int)in_rows;
        g.xtile = (int)xtile;
      }
    }
  }
  SSQ_REQUIRE(best < 1e300, SSQ_E_ARG, "ssq_conv_wgrad: input rows too wide for the LDS tile");
  const int TM = 64 * g.WM, TN = 256 / g.WM;
  g.lda = g.Pq + 1;
  g.chunks_per_n = (int)((OH * OW + g.Pq - 1) / g.Pq);
  g.nchunks = g.Nb * g.chunks_per_n;
  g.m_tiles = (g.Cog + TM - 1) / TM;
  g.n_tiles = (g.Ncol + TN - 1) / TN;
  const int64_t tiles = (int64_t)g.n_tiles * g.m_tiles * g.G;
  // about two workgroups per CU over the grid, at least 2 chunks each
  int nsplit = (int)std::max<int64_t>(1, std::min<int64_t>(g.nchunks / 2, (512 + tiles - 1) / tiles));
  g.cps = (g.nchunks + nsplit - 1) / nsplit;
  g.nsplit = (g.nchunks + g.cps - 1) / g.cps;
  *lds_bytes = wgrad_lds(g.WM, g.Pq, g.xtile);
  return SSQ_OK;
}

// ------------------------------------------------------------------ band form (3x3, pad 1)
// Ungrouped 3x3 / pad 1 convs at stride 1 or 2 with Cin, Cout multiples of 32 (every
// ResNet-18 3x3 conv).  The GEMM columns are regrouped as (tap, ci): a wave owns 32 co x
// 32 ci x all 9 taps (9 v_mfma_f32_32x32x2_f32 accumulators), so one dy fragment feeds 9
// MFMAs and the 9 taps of an input channel are 3 row windows of the same staged x rows.
// K = (n, output pixel) is walked in bands of RB whole output rows of one sample: per band
// the workgroup stages
//   A[co][q]          = dy[n, co, oh0 + q / OW, q % OW]              (q < RB * OW)
//   X[ci][ir][4 + iw] = x[n, ci, oh0*st - 1 + ir, iw]                (ir < (RB-1)*st + 3)
// by LDS-DMA into a double buffer, every LDS piece of which is DMA-written -- from dy / x
// or, for padding columns, out-of-image rows and pitch pads, from a zero page:
//   * 16-byte pieces (global_load_lds_dwordx4) when rows are 16-B aligned (W, OW, the
//     band's dy span multiples of 4 floats): the per-lane sources are band-independent,
//     computed once per kernel (no division in the staging);
//   * 4-byte pieces otherwise (14x14 and 7x7 planes), sources by magic-number division.
// A lane walks V consecutive pixels of its lane half per step (V = 4, 2 or 1 by OW): A by
// one ds_read of V floats, each tap row's window of (V-1)*st + 3 floats, 9*V MFMAs per
// step, the next step's operands read during this step's MFMAs (two register sets used
// alternately).  A band whose pixel count does not split into the two lane halves is
// padded with pixels whose A is zero (their x reads are clamped to the last real pixel).  Pitches are odd multiples of 4 floats
// (conflict-free 16-B reads).  Partials go to part[split][tap][co][ci] (coalesced) and
// wgrad_stage2 sums the splits in a fixed order into dW[co][ci][tap]: deterministic.
constexpr int kBandMaxNI = 20;     // 16-B DMA instructions per wave per band (80 KB buffers)
__device__ float g_band_zero_page[4 * 64];   // zero-initialised, never written

struct BandGeo {
  int C, H, W, Co, OW, OHW, Cig, Cog;
  int RB, Q, Qp, PA, IR, PXrow, PXci;
  int TMc, CBc;          // workgroup tile: co rows, input channels
  int bufsz;             // floats per LDS buffer (a multiple of 1024)
  int d16;               // 16-byte DMA with precomputed sources (else 4-byte pieces)
  int ni_w;              // DMA instructions per wave per band
  int bands_per_n, nchunks, cps, nsplit, m_tiles, n_tiles, remap;
  FastDiv dPA, dPXci, dPXrow;
};

template <int N>
using IntC = std::integral_constant<int, N>;

// NWV = 4: one wave per SIMD, each wave all 9 taps of its 32 co x 32 ci tile.  NWV = 8: two
// waves per SIMD -- waves w and w + 4 own the same tile, w taps 0-4 (80 AGPRs), w + 4 taps
// 5-8 (64): both walk every pixel of the band, each reading only its two tap rows, so while
// one waits on LDS, the band barrier or its staging, the other keeps the SIMD's MFMA pipe
// busy.  Every tap's accumulator sums the same pixels in the same order either way: the
// two forms give the same bits.
template <int WMX, int ST, int V, int NWV>
__global__ __launch_bounds__(64 * NWV, 1) void wgrad_band_stage1(const float* __restrict__ x,
                                                                 const float* __restrict__ dy,
                                                                 BandGeo g, float* __restrict__ part) {
  static_assert(NWV == 4 || NWV == 8, "4 or 8 waves");
  constexpr int WNX = 4 / WMX;
  constexpr int kSlots = kBandMaxNI * 4 / NWV;   // 16-B pieces per wave per band, at most
  extern __shared__ float lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wt = wave & 3, role = wave >> 2;
  const int wm = wt / WNX, wn = wt - wm * WNX;
  // XCD-aware order (remap): the tiles of one split run on one XCD and share its L2
  int wg = blockIdx.x;
  const int tiles = g.m_tiles * g.n_tiles;
  if (g.remap) {
    const int per = (int)gridDim.x >> 3;
    wg = (wg & 7) * per + (wg >> 3);
  }
  const int split = wg / tiles, tile = wg - split * tiles;
  const int mt = tile / g.n_tiles, nt = tile - mt * g.n_tiles;
  const int co0 = mt * g.TMc, ci0 = nt * g.CBc;
  const int c_begin = split * g.cps, c_end = min(c_begin + g.cps, g.nchunks);
  const int abytes = g.TMc * g.PA;
  // this wave's DMA pieces: piece j = wave + NWV*i of the buffer (256 floats per 16-B
  // piece, 64 per 4-B piece)
  const int n16 = g.d16 ? min(kSlots, (g.bufsz / 256 - wave + NWV - 1) / NWV) : 0;
  const int n4 = g.d16 ? 0 : (g.bufsz / 64 - wave + NWV - 1) / NWV;

  // 16-B form: per-lane DMA sources, band-independent: kind 0 zero page, 1 dy, 2 x row ir
  int soff[kSlots], meta[kSlots];
#pragma unroll
  for (int i = 0; i < kSlots; ++i) {
    soff[i] = 0;
    meta[i] = 0;
    if (i < n16) {
      const int o = (wave + NWV * i) * 256 + lane * 4;
      if (o < abytes) {
        const int row = (int)fdiv((uint32_t)o, g.dPA), col = o - row * g.PA;
        if (col < g.Q && co0 + row < g.Cog) {
          soff[i] = (co0 + row) * g.OHW + col;   // + n*Co*OHW + oh0*OW per band
          meta[i] = 1;
        }
      } else {
        const int o2 = o - abytes;
        const int cl = (int)fdiv((uint32_t)o2, g.dPXci), rem = o2 - cl * g.PXci;
        const int ir = (int)fdiv((uint32_t)rem, g.dPXrow), iw = rem - ir * g.PXrow - 4;
        if (cl < g.CBc && ci0 + cl < g.Cig && ir < g.IR && iw >= 0 && iw < g.W) {
          soff[i] = ((ci0 + cl) * g.H + ir) * g.W + iw;   // + n*C*H*W + ih0*W per band
          meta[i] = 2 | (ir << 2);
        }
      }
    }
  }
  // band c's sources: its sample's dy rows from oh0 and x rows from ih0 = oh0*st - 1
  struct Band {
    const float* ab;
    const float* xb;
    int ih0;
  };
  auto band_of = [&](int c) {
    const int n = c / g.bands_per_n;
    const int oh0 = (c - n * g.bands_per_n) * g.RB;
    const int ih0 = oh0 * ST - 1;
    return Band{dy + (int64_t)n * g.Co * g.OHW + oh0 * g.OW,
                x + (int64_t)n * g.C * g.H * g.W + (int64_t)ih0 * g.W, ih0};
  };
  // 16-B form: the whole band in one go; branch-free source selection: dy row piece,
  // x row piece, or the zero page
  auto stage16 = [&](const Band& bd, int b) {
    const float* zero = g_band_zero_page + lane * 4;
    float* dst = lds + b * g.bufsz + wave * 256;
#pragma unroll
    for (int i = 0; i < kSlots; ++i) {
      if (i < n16) {
        // selects, not branches: bitwise conditions, 64-bit addresses picked by value
        const int kind = meta[i] & 3;
        const unsigned ih = (unsigned)(bd.ih0 + (meta[i] >> 2));
        const bool ok = (kind == 1) | ((kind == 2) & (ih < (unsigned)g.H));
        const uint64_t pa = (uint64_t)(bd.ab + soff[i]), px = (uint64_t)(bd.xb + soff[i]);
        const uint64_t p = ok ? (kind == 1 ? pa : px) : (uint64_t)zero;
        __builtin_amdgcn_global_load_lds((const void*)p, (void*)(dst + i * NWV * 256), 16, 0, 0);
      }
    }
  };
  // 4-B form: pieces [i0, i1) of this wave; piece j = wave + NWV*i covers floats
  // [64j, 64j + 64), all in the A region or all in the X region (the A region is a
  // multiple of 64 floats)
  const int HW = g.H * g.W;
  auto stage4 = [&](const Band& bd, int b, int i0, int i1) {
    const float* zero = g_band_zero_page + lane;
    float* dst = lds + b * g.bufsz + wave * 64;
    for (int i = i0; i < i1; ++i) {
      const int o = (wave + NWV * i) * 64 + lane;
      const float* src = zero;
      if ((wave + NWV * i) * 64 < abytes) {
        const int row = (int)fdiv((uint32_t)o, g.dPA), col = o - row * g.PA;
        if (col < g.Q && co0 + row < g.Cog) src = bd.ab + (co0 + row) * g.OHW + col;
      } else {
        const int o2 = o - abytes;
        const int cl = (int)fdiv((uint32_t)o2, g.dPXci), rem = o2 - cl * g.PXci;
        const int ir = (int)fdiv((uint32_t)rem, g.dPXrow), iw = rem - ir * g.PXrow - 4;
        const unsigned ih = (unsigned)(bd.ih0 + ir);
        if (cl < g.CBc && ci0 + cl < g.Cig && ir < g.IR && iw >= 0 && iw < g.W &&
            ih < (unsigned)g.H)
          src = bd.xb + (ci0 + cl) * HW + ir * g.W + iw;
      }
      __builtin_amdgcn_global_load_lds((const void*)src, (void*)(dst + i * NWV * 64), 4, 0, 0);
    }
  };

  typedef float f32x4v __attribute__((ext_vector_type(4)));
  typedef float f32x2v __attribute__((ext_vector_type(2)));
  const int h = lane >> 5, l32 = lane & 31;
  const int arow = (wm * 32 + l32) * g.PA;
  const int xrow = abytes + (wn * 32 + l32) * g.PXci;
  const int q0 = h * (g.Qp >> 1);
  const int ngroups = g.Qp / (2 * V);
  // the last real pixel: x reads of padding pixels (A = 0) are clamped to it
  const int last_row = (g.Q - 1) / g.OW, last_col = (g.Q - 1) - last_row * g.OW;
  constexpr int NW = (V - 1) * ST + 3;   // window floats per tap row: V pixels x 3 taps
  // 4-B form: the next band's pieces are spread over the first half of this band's
  // steps, issued between the MFMAs (their address math runs in the MFMA shadow)
  const int per_step = (n4 + max(1, ngroups / 2) - 1) / max(1, ngroups / 2);
  if (c_begin < c_end) {
    const Band bd = band_of(c_begin);
    if (g.d16) stage16(bd, 0);
    else stage4(bd, 0, 0, n4);
  }

  // the band loop and the partial store for taps [T0, T1)
  auto body = [&](auto t0c, auto t1c) {
    constexpr int T0 = decltype(t0c)::value, T1 = decltype(t1c)::value, NT = T1 - T0;
    constexpr int R0 = T0 / 3, NR = (T1 - 1) / 3 - R0 + 1;   // tap rows read
    f32x16 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = f32x16{0};
    // one step's operands: A (V pixels) and the tap-row windows, read one step ahead
    auto fetch = [&](const float* L, int q, int orow, int ow, float (&a)[V],
                     float (&w)[NR][NW]) {
      if constexpr (V == 4) {
        const f32x4v av = *(const f32x4v*)(L + arow + q);
        a[0] = av.x; a[1] = av.y; a[2] = av.z; a[3] = av.w;
      } else if constexpr (V == 2) {
        const f32x2v av = *(const f32x2v*)(L + arow + q);
        a[0] = av.x; a[1] = av.y;
      } else {
        a[0] = L[arow + q];
      }
      int xr_row = orow, xr_col = ow;
      if (q >= g.Q) {
        xr_row = last_row;
        xr_col = last_col - (V - 1);
      }
      const float* xr0 = L + xrow + (xr_row * ST + R0) * g.PXrow + xr_col * ST + 3;
#pragma unroll
      for (int r = 0; r < NR; ++r) {
        const float* xr = xr0 + r * g.PXrow;
        if constexpr (V == 4) {
          w[r][0] = xr[0];
          const f32x4v t1 = *(const f32x4v*)(xr + 1);
          w[r][1] = t1.x; w[r][2] = t1.y; w[r][3] = t1.z; w[r][4] = t1.w;
          if constexpr (ST == 1) {
            w[r][5] = xr[5];
          } else {
            const f32x4v t2 = *(const f32x4v*)(xr + 5);
            w[r][5] = t2.x; w[r][6] = t2.y; w[r][7] = t2.z; w[r][8] = t2.w;
          }
        } else {
#pragma unroll
          for (int j = 0; j < NW; ++j) w[r][j] = xr[j];
        }
      }
    };
    auto mfmas = [&](const float (&a)[V], const float (&w)[NR][NW]) {
#pragma unroll
      for (int r = 0; r < NR; ++r)
#pragma unroll
        for (int v = 0; v < V; ++v)
#pragma unroll
          for (int s = 0; s < 3; ++s) {
            const int tap = (R0 + r) * 3 + s;
            if (tap >= T0 && tap < T1)
              acc[tap - T0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[v], w[r][v * ST + s],
                                                                   acc[tap - T0], 0, 0, 0);
          }
    };
    // Each half step: the other set's LDS reads interleaved one per MFMA at the front of
    // the step's NT*V MFMAs (scheduler directive), so they land long before that set's
    // MFMAs wait for them
    auto interleave = [&]() {
      constexpr int NM = NT * V, ND = NM < 12 ? NM : 12;
#pragma unroll
      for (int k = 0; k < ND; ++k) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // 1 MFMA
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);   // 1 DS read
      }
      __builtin_amdgcn_sched_group_barrier(0x008, NM - ND, 0);
    };
    for (int c = c_begin; c < c_end; ++c) {
      const int b = (c - c_begin) & 1;
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();             // band c staged; band c-1's reads of buffer b^1 done
      const bool more = c + 1 < c_end;
      const Band nb = band_of(more ? c + 1 : c);
      if (more && g.d16) stage16(nb, b ^ 1);
      const float* L = lds + b * g.bufsz;
      int q = q0, orow = q0 / g.OW, ow = q0 - orow * g.OW;
      auto advance = [&]() {
        q += V;
        ow += V;
        if (ow == g.OW) {
          ow = 0;
          ++orow;
        }
      };
      auto stage_slice = [&](int gi) {
        if (more && !g.d16) {
          const int i0 = gi * per_step;
          if (i0 < n4) stage4(nb, b ^ 1, i0, min(i0 + per_step, n4));
        }
      };
      // two operand sets used alternately, each read one step ahead of its MFMAs.  The
      // pair loop fetches unconditionally (its last fetch, one step past the band, reads
      // in-buffer pitch pads / the clamped last pixel and is never used): with no
      // conditional definitions the sets keep their registers, so the MFMAs wait only for
      // their own set's reads, not for the set just issued (a conditional fetch made the
      // compiler copy the new set into place behind an lgkmcnt(0) every step)
      float a0[V], w0[NR][NW], a1[V], w1[NR][NW];
      fetch(L, q, orow, ow, a0, w0);
      const int npairs = ngroups >> 1;
      for (int gp = 0; gp < npairs; ++gp) {
        stage_slice(2 * gp);
        advance();
        fetch(L, q, orow, ow, a1, w1);
        mfmas(a0, w0);
        interleave();
        stage_slice(2 * gp + 1);
        advance();
        fetch(L, q, orow, ow, a0, w0);
        mfmas(a1, w1);
        interleave();
      }
      if (ngroups & 1) {
        stage_slice(ngroups - 1);
        mfmas(a0, w0);
      }
    }
    // part[split][tap][co][ci]: C[row][col], row = (i&3) + 8*(i>>2) + 4*h, col = lane&31
    const int co_w = co0 + wm * 32, ci = ci0 + wn * 32 + l32;
    if (ci < g.Cig) {
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        float* dst = part + ((int64_t)split * 9 + T0 + t) * g.Cog * g.Cig;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int co = co_w + (i & 3) + 8 * (i >> 2) + 4 * h;
          if (co < g.Cog) dst[(int64_t)co * g.Cig + ci] = acc[t][i];
        }
      }
    }
  };
  if constexpr (NWV == 4) {
    body(IntC<0>{}, IntC<9>{});
  } else {
    if (role == 0) body(IntC<0>{}, IntC<5>{});
    else body(IntC<5>{}, IntC<9>{});
  }
}

// The band kernel's waves per workgroup: 8 (two per SIMD, the default), or 4 (one per
// SIMD) under ssq_conv_wgrad_set_form(4) or the A/B knob SSQ_BAND_WAVES=4
static int g_wgrad_form = 0;
static int band_waves() {
  static const int w = [] {
    const char* e = getenv("SSQ_BAND_WAVES");
    return e && *e && atoi(e) == 4 ? 4 : 8;
  }();
  return g_wgrad_form == 4 ? 4 : w;
}

// band plan: 0 if the shape is not a band shape or no tile fits two buffers in the LDS
static int band_plan(int64_t Nb, int64_t C, int64_t H, int64_t W, int64_t Co, int64_t R,
                     int64_t S, int64_t st, int64_t pad, int64_t G, BandGeo& g, int* wmx,
                     int* vpx) {
  if (G != 1 || R != 3 || S != 3 || pad != 1 || (st != 1 && st != 2)) return 0;
  const int64_t OH = (H + 2 - 3) / st + 1, OW = (W + 2 - 3) / st + 1;
  if (OH < 1 || OW < 1 || Co % 32 || C % 32) return 0;
  if (Nb * C * H * W >= (1ll << 31) || Nb * Co * OH * OW >= (1ll << 31)) return 0;
  g.C = (int)C; g.H = (int)H; g.W = (int)W; g.Co = (int)Co; g.OW = (int)OW;
  g.OHW = (int)(OH * OW); g.Cig = (int)C; g.Cog = (int)Co;
  const int V = OW % 4 == 0 ? 4 : (OW % 2 == 0 ? 2 : 1);
  auto odd4 = [](int v) { v = (v + 3) / 4 * 4; return (v / 4) % 2 ? v : v + 4; };
  const int64_t budget = 160 * 1024 / 2 / 4;   // floats per buffer
  bool found = false;
  double best = 1e300;
  // every (tile, band height) whose double buffer fits; the cheapest per output pixel by
  // a per-wave cycle model: 9 MFMAs (64 cycles) per padded pixel pair, ~1500 cycles of
  // wait + barrier per band, 16-B DMA issue ~40 cycles per instruction (before the MFMAs),
  // 4-B DMA ~10 (interleaved with them)
  for (int wm : {2, 4}) {
    const int TMc = 32 * wm, CBc = 32 * (4 / wm);
    if (wm == 4 && Co < 128) continue;
    for (int rb = (int)std::min<int64_t>(OH, 8); rb >= 1; --rb) {
      if (OH % rb) continue;
      const int Q = rb * (int)OW, Qp = (Q + 2 * V - 1) / (2 * V) * (2 * V);
      const int IR = (rb - 1) * (int)st + 3;
      // 16-B pieces need 16-B aligned x rows and dy spans
      const bool d16 = W % 4 == 0 && g.OHW % 4 == 0 && Q % 4 == 0 && Qp == Q;
      // LDS columns read: up to (OW - 1)*st + 3 + 2 (+ the 16-B form's whole row)
      const int need = (int)((OW - 1) * st) + 6;
      const int PXrow = d16 ? (int)W + 8 : (std::max<int>(need, (int)W + 4) + 3) / 4 * 4;
      const int PA = odd4(Qp + 1), PXci = odd4(IR * PXrow);
      const int64_t buf = ((int64_t)TMc * PA + (int64_t)CBc * PXci + 1023) / 1024 * 1024;
      if (buf > budget) continue;
      const int ni = d16 ? (int)(buf / 1024) : (int)(buf / 256);
      if (d16 && ni > kBandMaxNI) continue;
      const double cost = (288.0 * Qp + 1500.0 + (d16 ? 40.0 : 10.0) * ni) / Q;
      if (cost >= best) continue;
      best = cost;
      g.RB = rb; g.Q = Q; g.Qp = Qp; g.PA = PA; g.IR = IR; g.PXrow = PXrow; g.PXci = PXci;
      g.TMc = TMc; g.CBc = CBc; g.bufsz = (int)buf; g.d16 = d16 ? 1 : 0; g.ni_w = ni;
      *wmx = wm;
      *vpx = V;
      found = true;
    }
  }
  if (!found) return 0;
  g.dPA = make_fastdiv((uint32_t)g.PA);
  g.dPXci = make_fastdiv((uint32_t)g.PXci);
  g.dPXrow = make_fastdiv((uint32_t)g.PXrow);
  g.m_tiles = (g.Cog + g.TMc - 1) / g.TMc;
  g.n_tiles = (g.Cig + g.CBc - 1) / g.CBc;
  g.bands_per_n = (int)(OH / g.RB);
  g.nchunks = (int)Nb * g.bands_per_n;
  const int tiles = g.m_tiles * g.n_tiles;
  // one workgroup per CU (the two buffers take most of the LDS): ~256 workgroups
  int ns = std::max(1, std::min(g.nchunks, (256 + tiles - 1) / tiles));
  g.cps = (g.nchunks + ns - 1) / ns;
  g.nsplit = (g.nchunks + g.cps - 1) / g.cps;
  g.remap = ((int64_t)g.nsplit * tiles) % 8 == 0;
  return 1;
}

// Non-depthwise form: 0 auto, 1 the R x S input-row-tile kernel (1x1 on its GEMM), 2 the
// im2col-DMA kernel for every shape, 3 the band kernel where it applies, 4 the same at 4
// waves per workgroup (A/B knob: ssq_conv_wgrad_set_form; g_wgrad_form is above).  Auto
// takes the band kernel for the shapes band_plan accepts, then the im2col-DMA kernel for
// ungrouped R x S > 1 convs with >= 128 output channels (its 128 x 128 tile is half idle
// below that): ResNet-18 3x3 stride-2 convs 2-2.3x faster than the row-tile kernel, 3x3
// stride-1 1.1-1.4x (profiles/r2_wgrad_forms.log).
static bool use_band(int64_t Nb, int64_t C, int64_t H, int64_t W, int64_t Co, int64_t R,
                     int64_t S, int64_t st, int64_t pad, int64_t G, BandGeo& g, int* wmx,
                     int* vpx) {
  if (g_wgrad_form != 0 && g_wgrad_form != 3 && g_wgrad_form != 4) return false;
  return band_plan(Nb, C, H, W, Co, R, S, st, pad, G, g, wmx, vpx) != 0;
}
static bool use_i2c(int64_t R, int64_t S, int64_t Co, int64_t G) {
  if (g_wgrad_form != 0) return g_wgrad_form == 2;
  return R * S > 1 && G == 1 && Co >= 128;
}

}  // namespace ssq

using namespace ssq;

extern "C" int ssq_conv_wgrad_set_form(int form) {
  const int old = g_wgrad_form;
  if (form >= 0 && form <= 4) g_wgrad_form = form;
  return old;
}

extern "C" int ssq_conv_wgrad_kind(int64_t Nb, int64_t C, int64_t H, int64_t W, int64_t Co,
                                   int64_t R, int64_t S, int64_t stride, int64_t pad,
                                   int64_t groups) {
  if (is_depthwise(C, Co, groups) && R * S <= 25 && Nb >= 1 && dw_lds_ok(H, W, pad)) return 5;
  BandGeo gb;
  int wmx, vpx;
  if (use_band(Nb, C, H, W, Co, R, S, stride, pad, groups, gb, &wmx, &vpx)) return gb.d16 ? 3 : 6;
  if (use_i2c(R, S, Co, groups)) {
    I2cGeo gi;
    return wgrad_i2c_plan(Nb, C, H, W, Co, R, S, stride, pad, groups, gi) ? 0 : 2;
  }
  if (R == 1 && S == 1 && pad == 0) {
    W1Geo g1;
    return wgrad_1x1_plan(Nb, C, H, W, Co, stride, groups, g1) ? 0 : 4;
  }
  WgradGeo g;
  size_t lds;
  return wgrad_plan(Nb, C, H, W, Co, R, S, stride, pad, groups, g, &lds) ? 0 : 1;
}

extern "C" size_t ssq_conv_wgrad_workspace_size(int64_t Nb, int64_t C, int64_t H, int64_t W,
                                                int64_t Co, int64_t R, int64_t S, int64_t stride,
                                                int64_t pad, int64_t groups) {
  if (is_depthwise(C, Co, groups) && R * S <= 25 && Nb >= 1 && dw_lds_ok(H, W, pad)) {
    int spl;
    const int ns = dw_splits(Nb, C, &spl);
    const int64_t OH = (H + 2 * pad - R) / stride + 1;
    int64_t nbands = 1;
    if (dw_stage(H, W, pad, spl) == 0 && OH >= 1) {
      const int bh = dw_band_rows(H, W, R, stride, pad, OH);
      nbands = (OH + bh - 1) / bh;
    }
    return (size_t)ns * (size_t)nbands * (size_t)C * (size_t)(R * S) * sizeof(float);
  }
  {
    BandGeo gb;
    int wmx, vpx;
    if (use_band(Nb, C, H, W, Co, R, S, stride, pad, groups, gb, &wmx, &vpx))
      return (size_t)gb.nsplit * 9 * (size_t)Co * (size_t)C * sizeof(float);
  }
  if (use_i2c(R, S, Co, groups)) {
    I2cGeo gi;
    int wm;
    if (wgrad_i2c_plan(Nb, C, H, W, Co, R, S, stride, pad, groups, gi)) return 0;
    wgrad_i2c_tiles(gi, &wm);
    return (size_t)gi.nsplit * (size_t)Co * (size_t)gi.Ncol * sizeof(float);
  }
  if (R == 1 && S == 1 && pad == 0) {
    W1Geo g1;
    if (wgrad_1x1_plan(Nb, C, H, W, Co, stride, groups, g1)) return 0;
    return (size_t)g1.nsplit * (size_t)Co * (size_t)g1.Cig * sizeof(float);
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
    const int64_t plane = (H + 2 * pad) * (W + 2 * pad);
    const int nb = dw_stage(H, W, pad, spl);
    if (nb > 0) {
      const size_t lds = (size_t)nb * plane * sizeof(float);  // <= 32 KiB
      const FastDiv dWp = make_fastdiv((uint32_t)(W + 2 * pad)), dP = make_fastdiv((uint32_t)plane),
                    dOHW = make_fastdiv((uint32_t)(OH * OW)), dOW = make_fastdiv((uint32_t)OW);
      if (R * S <= 9)
        hipLaunchKernelGGL(wgrad_dw_small<9>, grid, dim3(256), lds, s, x, dy, (int)C, (int)H,
                           (int)W, (int)OH, (int)OW, (int)R, (int)S, (int)stride, (int)pad, spl,
                           nb, dWp, dP, dOHW, dOW, (float*)ws);
      else
        hipLaunchKernelGGL(wgrad_dw_small<25>, grid, dim3(256), lds, s, x, dy, (int)C, (int)H,
                           (int)W, (int)OH, (int)OW, (int)R, (int)S, (int)stride, (int)pad, spl,
                           nb, dWp, dP, dOHW, dOW, (float*)ws);
      const int64_t n = C * R * S;
      hipLaunchKernelGGL(wgrad_stage2, dim3((unsigned)std::min<int64_t>((n + 63) / 64, 4096)),
                         dim3(256), 0, s, (const float*)ws, ns, n, dw);
      return check_launch("ssq_conv_wgrad");
    }
    const int bh = dw_band_rows(H, W, R, stride, pad, OH);
    const int nbands = (int)((OH + bh - 1) / bh);
    SSQ_REQUIRE(ws_bytes >= need * (size_t)nbands, SSQ_E_WS, "ssq_conv_wgrad: workspace too small");
    const dim3 gridb((unsigned)C, (unsigned)(ns * nbands));
    const size_t lds = (size_t)(((int64_t)bh - 1) * stride + R) * (W + 2 * pad) * sizeof(float);
    static bool dw_attr = false;
    if (!dw_attr) {  // dynamic LDS beyond 64 KiB must be opted into
      hipFuncSetAttribute((const void*)wgrad_dw_stage1<9>,
                          hipFuncAttributeMaxDynamicSharedMemorySize, 128 * 1024);
      hipFuncSetAttribute((const void*)wgrad_dw_stage1<25>,
                          hipFuncAttributeMaxDynamicSharedMemorySize, 128 * 1024);
      dw_attr = true;
    }
    if (R * S <= 9)
      hipLaunchKernelGGL(wgrad_dw_stage1<9>, gridb, dim3(256), lds, s, x, dy, (int)C, (int)H, (int)W,
                         (int)OH, (int)OW, (int)R, (int)S, (int)stride, (int)pad, spl, bh, nbands,
                         make_fastdiv((uint32_t)(W + 2 * pad)), (float*)ws);
    else
      hipLaunchKernelGGL(wgrad_dw_stage1<25>, gridb, dim3(256), lds, s, x, dy, (int)C, (int)H, (int)W,
                         (int)OH, (int)OW, (int)R, (int)S, (int)stride, (int)pad, spl, bh, nbands,
                         make_fastdiv((uint32_t)(W + 2 * pad)), (float*)ws);
    const int64_t n = C * R * S;
    hipLaunchKernelGGL(wgrad_stage2, dim3((unsigned)std::min<int64_t>((n + 63) / 64, 4096)),
                       dim3(256), 0, s, (const float*)ws, ns * nbands, n, dw);
    return check_launch("ssq_conv_wgrad");
  }
  {
    BandGeo gb;
    int wmx, vpx;
    if (use_band(Nb, C, H, W, Co, R, S, stride, pad, groups, gb, &wmx, &vpx)) {
      const size_t needb = (size_t)gb.nsplit * 9 * (size_t)Co * (size_t)C * sizeof(float);
      SSQ_REQUIRE(ws && ws_bytes >= needb, SSQ_E_WS, "ssq_conv_wgrad: workspace too small");
      typedef void (*BandK)(const float*, const float*, BandGeo, float*);
      // [8 waves][wm == 4][stride == 2][V = 4, 2, 1]
#define SSQ_BK(NWV)                                                                          \
  {{{wgrad_band_stage1<2, 1, 4, NWV>, wgrad_band_stage1<2, 1, 2, NWV>,                        \
     wgrad_band_stage1<2, 1, 1, NWV>},                                                        \
    {wgrad_band_stage1<2, 2, 4, NWV>, wgrad_band_stage1<2, 2, 2, NWV>,                        \
     wgrad_band_stage1<2, 2, 1, NWV>}},                                                       \
   {{wgrad_band_stage1<4, 1, 4, NWV>, wgrad_band_stage1<4, 1, 2, NWV>,                        \
     wgrad_band_stage1<4, 1, 1, NWV>},                                                        \
    {wgrad_band_stage1<4, 2, 4, NWV>, wgrad_band_stage1<4, 2, 2, NWV>,                        \
     wgrad_band_stage1<4, 2, 1, NWV>}}}
      static const BandK kernels[2][2][2][3] = {SSQ_BK(4), SSQ_BK(8)};
#undef SSQ_BK
      static bool band_attr = false;
      if (!band_attr) {  // two 80 KB buffers: the whole LDS
        for (auto& a0 : kernels)
          for (auto& a : a0)
            for (auto& b : a)
              for (BandK k : b)
                hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    160 * 1024);
        band_attr = true;
      }
      const int w8 = band_waves() == 8;
      const BandK kb = kernels[w8][wmx == 4][stride == 2][vpx == 4 ? 0 : (vpx == 2 ? 1 : 2)];
      const dim3 gridb((unsigned)(gb.nsplit * gb.m_tiles * gb.n_tiles));
      const size_t ldsb = 2 * (size_t)gb.bufsz * sizeof(float);
      hipLaunchKernelGGL(kb, gridb, dim3(w8 ? 512 : 256), ldsb, s, x, dy, gb, (float*)ws);
      const int64_t inner = Co * C, nb = 9 * inner;
      hipLaunchKernelGGL(wgrad_stage2, dim3((unsigned)std::min<int64_t>((nb + 63) / 64, 4096)),
                         dim3(256), 0, s, (const float*)ws, gb.nsplit, nb, dw, inner, 9);
      return check_launch("ssq_conv_wgrad");
    }
  }
  if (use_i2c(R, S, Co, groups)) {
    I2cGeo gi;
    int wm;
    const int rci = wgrad_i2c_plan(Nb, C, H, W, Co, R, S, stride, pad, groups, gi);
    if (rci) return rci;
    wgrad_i2c_tiles(gi, &wm);
    const size_t needi = (size_t)gi.nsplit * (size_t)Co * (size_t)gi.Ncol * sizeof(float);
    SSQ_REQUIRE(ws && ws_bytes >= needi, SSQ_E_WS, "ssq_conv_wgrad: workspace too small");
    const dim3 gridi(gi.n_tiles, gi.m_tiles * gi.G, gi.nsplit);
    (void)wm;
    hipLaunchKernelGGL(wgrad_i2c_stage1<2>, gridi, dim3(256), 0, s, x, dy, gi, (float*)ws);
    const int64_t ni = (int64_t)Co * gi.Ncol;
    hipLaunchKernelGGL(wgrad_stage2, dim3((unsigned)std::min<int64_t>((ni + 63) / 64, 4096)),
                       dim3(256), 0, s, (const float*)ws, gi.nsplit, ni, dw);
    return check_launch("ssq_conv_wgrad");
  }
  if (R == 1 && S == 1 && pad == 0) {
    W1Geo g1;
    const int rc1 = wgrad_1x1_plan(Nb, C, H, W, Co, stride, groups, g1);
    if (rc1) return rc1;
    const size_t need1 = (size_t)g1.nsplit * (size_t)Co * (size_t)g1.Cig * sizeof(float);
    SSQ_REQUIRE(ws && ws_bytes >= need1, SSQ_E_WS, "ssq_conv_wgrad: workspace too small");
    const dim3 grid1(g1.n_tiles, g1.m_tiles * g1.G, g1.nsplit);
    hipLaunchKernelGGL(wgrad_1x1_stage1<2>, grid1, dim3(256), 0, s, x, dy, g1, (float*)ws);
    const int64_t n1 = (int64_t)Co * g1.Cig;
    hipLaunchKernelGGL(wgrad_stage2, dim3((unsigned)std::min<int64_t>((n1 + 63) / 64, 4096)),
                       dim3(256), 0, s, (const float*)ws, g1.nsplit, n1, dw);
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
    hipFuncSetAttribute((const void*)wgrad_stage1<1>, hipFuncAttributeMaxDynamicSharedMemorySize,
                        160 * 1024);
    hipFuncSetAttribute((const void*)wgrad_stage1<2>, hipFuncAttributeMaxDynamicSharedMemorySize,
                        160 * 1024);
    hipFuncSetAttribute((const void*)wgrad_stage1<4>, hipFuncAttributeMaxDynamicSharedMemorySize,
                        160 * 1024);
    lds_attr = true;
  }
  const dim3 grid(g.n_tiles, g.m_tiles * g.G, g.nsplit);
  if (g.WM == 1)
    hipLaunchKernelGGL(wgrad_stage1<1>, grid, dim3(256), lds, s, x, dy, g, (float*)ws);
  else if (g.WM == 2)
    hipLaunchKernelGGL(wgrad_stage1<2>, grid, dim3(256), lds, s, x, dy, g, (float*)ws);
  else
    hipLaunchKernelGGL(wgrad_stage1<4>, grid, dim3(256), lds, s, x, dy, g, (float*)ws);
  const int64_t n = (int64_t)Co * g.Ncol;
  hipLaunchKernelGGL(wgrad_stage2, dim3((unsigned)std::min<int64_t>((n + 63) / 64, 4096)),
                     dim3(256), 0, s, (const float*)ws, g.nsplit, n, dw);
  return check_launch("ssq_conv_wgrad");
}

// ------------------------------------------------------------------ GEMM operands
// The conv weight gradient as ONE library GEMM, for the small output planes where it beats
// the band kernel (ResNet-18 layer3/4: 14x14 and 7x7 planes, K = N*OH*OW of 1.5-6 K):
//   dW[Co, C*R*S] = dy2[Co, N*P] @ col[N*P, C*R*S],  P = OH*OW,
//   dy2[co][n*P + p] = dy[n][co][p],
//   col[n*P + p][(ci*R + r)*S + s] = x[n][ci][oh*st + r - pad][ow*st + s - pad] (0 outside).
// One launch writes both operands (workgroups [0, nb1) col in 64 x 64 tiles transposed
// through LDS -- x read along the output pixels, col written along its rows, 16-B stores
// when a row is a multiple of 4 columns -- the rest dy2); the x / dy reads hit L2.  The GEMM
// (torch.matmul: hipBLASLt, fp32, one deterministic kernel per shape) is the caller's.
__global__ __launch_bounds__(kBlock) void wgrad_gemm_operands(
    const float* __restrict__ x, const float* __restrict__ dy, uint32_t C, uint32_t H,
    uint32_t W, uint32_t Co, uint32_t R, uint32_t S, uint32_t st, int pad, uint32_t OW,
    uint32_t NP, FastDiv dRS, FastDiv dS, FastDiv dP, FastDiv dOW, uint32_t CRS,
    uint32_t P, uint32_t nb1, uint32_t tiles_k, uint32_t vec4, float* __restrict__ col,
    float* __restrict__ dy2) {
  if (blockIdx.x < nb1) {
    // 64 rows x 64 columns per workgroup through LDS: the x reads run along the rows (output
    // pixels: consecutive addresses for stride 1), the col writes along the columns (16-B
    // stores when vec4)
    __shared__ float tile[64][65];
    const uint32_t tk = blockIdx.x % tiles_k, tp = blockIdx.x / tiles_k;
    const uint32_t row0 = tp * 64, k0 = tk * 64, RS = R * S;
    // thread -> one row (output pixel) and columns kb, kb + 4, ..: the 16 loads in flight
    const uint32_t pp = threadIdx.x & 63, kb = threadIdx.x >> 6, row = row0 + pp;
    const bool rok = row < NP;
    const uint32_t n = rok ? fdiv(row, dP) : 0u, p = row - n * P;
    const uint32_t oh = fdiv(p, dOW), ow = p - oh * OW;
    const int ih0 = (int)(oh * st) - pad, iw0 = (int)(ow * st) - pad;
    const float* xn = x + (size_t)n * C * H * W;
    float v[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const uint32_t k = k0 + kb + 4 * j;
      const uint32_t ci = fdiv(k, dRS), rs = k - ci * RS;
      const uint32_t r = fdiv(rs, dS), sc = rs - r * S;
      const int ih = ih0 + (int)r, iw = iw0 + (int)sc;
      v[j] = 0.0f;
      if (rok && k < CRS && ih >= 0 && ih < (int)H && iw >= 0 && iw < (int)W)
        v[j] = xn[((size_t)ci * H + ih) * W + iw];
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) tile[kb + 4 * j][pp] = v[j];
    __syncthreads();
    if (vec4) {
      for (uint32_t i = threadIdx.x; i < 64 * 16; i += kBlock) {
        const uint32_t pp = i >> 4, kq = (i & 15) << 2;
        const uint32_t row = row0 + pp, k = k0 + kq;
        if (row < NP && k < CRS)  // CRS % 4 == 0: the 4 columns are all in range
          *reinterpret_cast<float4*>(col + (size_t)row * CRS + k) =
              make_float4(tile[kq][pp], tile[kq + 1][pp], tile[kq + 2][pp], tile[kq + 3][pp]);
      }
    } else {
      for (uint32_t i = threadIdx.x; i < 64 * 64; i += kBlock) {
        const uint32_t pp = i >> 6, kk = i & 63;
        const uint32_t row = row0 + pp, k = k0 + kk;
        if (row < NP && k < CRS) col[(size_t)row * CRS + k] = tile[kk][pp];
      }
    }
    return;
  }
  const uint32_t nb2 = gridDim.x - nb1;
  const uint32_t n2 = Co * NP;
  for (uint32_t e = (blockIdx.x - nb1) * kBlock + threadIdx.x; e < n2; e += nb2 * kBlock) {
    const uint32_t co = e / NP, q = e - co * NP;
    const uint32_t n = fdiv(q, dP), p = q - n * P;
    dy2[e] = dy[((size_t)n * Co + co) * P + p];
  }
}

// The im2col matrix of a conv whose input is the previous conv's K13 epilogue output, the
// epilogue applied on the fly (ResNet BasicBlock conv1 -> conv2 on the small planes, where
// conv2's forward and weight gradient are GEMMs over this matrix): x = epilogue(y),
//   t = y + bias[c]; t = t * gamma[c] + phi[c]; t = act(t); t = fq(t)   (each step optional)
// -- the very fp32 ops of bias_act_kernel (recon.hip), so col is bit for bit the im2col of
// the materialised epilogue output, which is never written.  Padding stays 0 (the conv pads
// the epilogue's output).
template <int ACT>
__device__ __forceinline__ float epi_in(float v, uint32_t c, const float* __restrict__ bias,
                                        const float* __restrict__ gamma,
                                        const float* __restrict__ phi, bool quant,
                                        const QParams& qp) {
  float t = bias ? __fadd_rn(v, bias[c]) : v;
  if (gamma) t = __fadd_rn(__fmul_rn(t, gamma[c]), phi[c]);
  t = act_fwd<ACT>(t);
  if (quant) {
    float q;
    t = fq1(t, qp, &q);
  }
  return t;
}

template <int ACT>
__global__ __launch_bounds__(kBlock) void gemm_col_epi(
    const float* __restrict__ y, const float* __restrict__ bias, const float* __restrict__ gamma,
    const float* __restrict__ phi, const float* __restrict__ qdelta,
    const float* __restrict__ qzp, float qlo, float qhi, uint32_t C, uint32_t H, uint32_t W,
    uint32_t R, uint32_t S, uint32_t st, int pad, uint32_t OW, uint32_t NP, FastDiv dCRS,
    FastDiv dRS, FastDiv dS, FastDiv dP, FastDiv dOW, uint32_t CRS, uint32_t P,
    float* __restrict__ col) {
  const bool quant = qdelta != nullptr;
  QParams qp{1.0f, 0.0f, qlo, qhi};
  if (quant) {
    qp.d = qdelta[0];
    qp.z = qzp[0];
  }
  const uint32_t n1 = NP * CRS;
  for (uint32_t e = blockIdx.x * kBlock + threadIdx.x; e < n1; e += gridDim.x * kBlock) {
    const uint32_t row = fdiv(e, dCRS), k = e - row * CRS;
    const uint32_t n = fdiv(row, dP), p = row - n * P;
    const uint32_t oh = fdiv(p, dOW), ow = p - oh * OW;
    const uint32_t ci = fdiv(k, dRS), rs = k - ci * R * S;
    const uint32_t r = fdiv(rs, dS), s = rs - r * S;
    const int ih = (int)(oh * st + r) - pad, iw = (int)(ow * st + s) - pad;
    float v = 0.0f;
    if (ih >= 0 && ih < (int)H && iw >= 0 && iw < (int)W)
      v = epi_in<ACT>(y[(((size_t)n * C + ci) * H + ih) * W + iw], ci, bias, gamma, phi, quant,
                      qp);
    col[e] = v;
  }
}

extern "C" int ssq_gemm_col_epilogue(const float* y, const float* bias, const float* gamma,
                                     const float* phi, int relu, const float* delta,
                                     const float* zp, int qmin, int qmax, int64_t Nb, int64_t C,
                                     int64_t H, int64_t W, int64_t R, int64_t S, int64_t stride,
                                     int64_t pad, float* col, ssq_stream_t stream) {
  SSQ_REQUIRE(y && col, SSQ_E_ARG, "ssq_gemm_col_epilogue: null pointer");
  SSQ_REQUIRE(!gamma == !phi, SSQ_E_ARG, "ssq_gemm_col_epilogue: gamma and phi go together");
  SSQ_REQUIRE(!delta || (zp && qmin < qmax), SSQ_E_ARG, "ssq_gemm_col_epilogue: act quantizer");
  SSQ_REQUIRE(relu >= 0 && relu <= 2, SSQ_E_ARG, "ssq_gemm_col_epilogue: activation code %d", relu);
  SSQ_REQUIRE(Nb >= 1 && C >= 1 && H >= 1 && W >= 1 && R >= 1 && S >= 1 && stride >= 1 &&
                  pad >= 0, SSQ_E_ARG, "ssq_gemm_col_epilogue: bad geometry");
  const int64_t OH = (H + 2 * pad - R) / stride + 1, OW = (W + 2 * pad - S) / stride + 1;
  SSQ_REQUIRE(OH >= 1 && OW >= 1, SSQ_E_ARG, "ssq_gemm_col_epilogue: empty output plane");
  const int64_t P = OH * OW, NP = Nb * P, CRS = C * R * S;
  SSQ_REQUIRE(NP * CRS < (1ll << 31) && Nb * C * H * W < (1ll << 31), SSQ_E_ARG,
              "ssq_gemm_col_epilogue: operands exceed 2^31 elements");
  const uint32_t nb = (uint32_t)std::min<int64_t>((NP * CRS + kBlock - 1) / kBlock, 8192);
#define SSQ_GCE(A)                                                                          \
  hipLaunchKernelGGL(gemm_col_epi<A>, dim3(nb), dim3(kBlock), 0, (hipStream_t)stream, y, bias, \
                     gamma, phi, delta, zp, (float)qmin, (float)qmax, (uint32_t)C, (uint32_t)H, \
                     (uint32_t)W, (uint32_t)R, (uint32_t)S, (uint32_t)stride, (int)pad,         \
                     (uint32_t)OW, (uint32_t)NP, make_fastdiv((uint32_t)CRS),                   \
                     make_fastdiv((uint32_t)(R * S)), make_fastdiv((uint32_t)S),                \
                     make_fastdiv((uint32_t)P), make_fastdiv((uint32_t)OW), (uint32_t)CRS,      \
                     (uint32_t)P, col)
  if (relu == 2) SSQ_GCE(2); else if (relu == 1) SSQ_GCE(1); else SSQ_GCE(0);
#undef SSQ_GCE
  return check_launch("ssq_gemm_col_epilogue");
}

extern "C" int ssq_wgrad_gemm_operands(const float* x, const float* dy, int64_t Nb, int64_t C,
                                       int64_t H, int64_t W, int64_t Co, int64_t R, int64_t S,
                                       int64_t stride, int64_t pad, float* col, float* dy2,
                                       ssq_stream_t stream) {
  SSQ_REQUIRE((x && col) || (dy && dy2), SSQ_E_ARG, "ssq_wgrad_gemm_operands: null pointer");
  if (!(x && col)) col = nullptr;
  if (!(dy && dy2)) dy2 = nullptr;
  SSQ_REQUIRE(Nb >= 1 && C >= 1 && H >= 1 && W >= 1 && Co >= 1 && R >= 1 && S >= 1 &&
                  stride >= 1 && pad >= 0, SSQ_E_ARG, "ssq_wgrad_gemm_operands: bad geometry");
  const int64_t OH = (H + 2 * pad - R) / stride + 1, OW = (W + 2 * pad - S) / stride + 1;
  SSQ_REQUIRE(OH >= 1 && OW >= 1, SSQ_E_ARG, "ssq_wgrad_gemm_operands: empty output plane");
  const int64_t P = OH * OW, NP = Nb * P, CRS = C * R * S;
  SSQ_REQUIRE(NP * CRS < (1ll << 31) && Co * NP < (1ll << 31) && Nb * C * H * W < (1ll << 31),
              SSQ_E_ARG, "ssq_wgrad_gemm_operands: operands exceed 2^31 elements");
  // col in 64 x 64 tiles (float4 stores when the rows are whole 16-B pieces)
  const bool vec4 = col && CRS % 4 == 0 && ((uintptr_t)col & 15) == 0;
  const int64_t tiles_k = (CRS + 63) / 64, tiles = ((NP + 63) / 64) * tiles_k;
  SSQ_REQUIRE(tiles < (1ll << 31), SSQ_E_ARG, "ssq_wgrad_gemm_operands: too many tiles");
  const uint32_t nb1 = col ? (uint32_t)tiles : 0u;
  const uint32_t nb2 = dy2 ? (uint32_t)std::min<int64_t>((Co * NP + kBlock - 1) / kBlock, 2048) : 0u;
  hipLaunchKernelGGL(wgrad_gemm_operands, dim3(nb1 + nb2), dim3(kBlock), 0, (hipStream_t)stream,
                     x, dy, (uint32_t)C, (uint32_t)H, (uint32_t)W, (uint32_t)Co, (uint32_t)R,
                     (uint32_t)S, (uint32_t)stride, (int)pad, (uint32_t)OW, (uint32_t)NP,
                     make_fastdiv((uint32_t)(R * S)), make_fastdiv((uint32_t)S),
                     make_fastdiv((uint32_t)P), make_fastdiv((uint32_t)OW), (uint32_t)CRS,
                     (uint32_t)P, nb1, (uint32_t)tiles_k, (uint32_t)vec4, col, dy2);
  return check_launch("ssq_wgrad_gemm_operands");
}
