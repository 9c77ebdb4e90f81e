// K5p / K6p: the prepared adaShift path, multi-segment.
//
// In the fused loop (layer_recon_fused_shiftedScale.py:59-66) W, delta, the shift
// candidates and beta are frozen: only alpha learns.  The reference therefore computes its
// floors x_q ONCE (channelQuant.py:284-286) and each iteration only re-mixes them.  The
// prepared path does the same: ssq_adashift_prepare evaluates, once, every floor
// F_i = floor(W / (delta*s_i)) with the very fp32 ops the recomputing kernels use, packed as
// int8 bytes into one 32-bit word per weight (S <= 4), and the rounding term
// h(beta) (or [beta >= 0]) as fp32.  The per-iteration kernels then stream
// fpack + hterm (+ gWhat) with no divide and no exp per element -- 12 B/elem forward
// (fpack, hterm in; What out) and 12 B/elem backward (gWhat, fpack, hterm in), the §8(d)
// algorithmic bytes -- and produce bit-identical What / identical gradients.  The alpha
// backward is one launch for weights with Co*K <= 1280 (bwd_tiling_prep: one workgroup
// per input channel, which it finalises) and two fixed-order launches otherwise
// (chunk partials, then one wave per input channel).  Both kernels are latency-bound at
// ResNet-18 sizes, so the loads a thread needs are issued before their first use.
//
// Every kernel takes a table of up to kMaxPrepSeg weights ("segments"), so the adaShift
// forward of ALL the convs of a block is one launch and their alpha backward one: the
// weights of a block depend only on alpha, which is fixed for the iteration
// (quant/_engine.py stash_block_weights).
#include <stdlib.h>

#include "adashift_common.h"
#include "fin_tasks.h"
#include "prep_ride.h"

namespace ssq {

constexpr int kMaxPrepS = 4;
constexpr int kRBP = 8;            // rows per load batch
constexpr int kMaxPrepSeg = 8;     // weights per launch (a block has <= 4 convs)

__global__ __launch_bounds__(kBlock) void adashift_prepare_kernel(
    const float* __restrict__ W, const float* __restrict__ beta, const float* __restrict__ delta,
    Shifts sh, Geo g, uint32_t n, int hard_r, uint32_t* __restrict__ fpack,
    float* __restrict__ hterm, int* __restrict__ overflow) {
  const uint32_t stride = gridDim.x * blockDim.x;
  int bad = 0;
  for (uint32_t e = blockIdx.x * blockDim.x + threadIdx.x; e < n; e += stride) {
    const uint32_t co = e / g.CiK;
    const float w = W[e], d = delta[co];
    uint32_t word = 0;
    for (int i = 0; i < sh.n; ++i) {
      const float F = floorf(w / __fmul_rn(d, sh.s[i]));   // = soft_floor's candidate
      bad |= !(F >= -128.0f && F <= 127.0f);
      const int fi = F >= -128.0f && F <= 127.0f ? (int)F : 0;
      word |= ((uint32_t)(fi & 0xff)) << (8 * i);
    }
    fpack[e] = word;
    const float b = beta[e];
    hterm[e] = hard_r ? (b >= 0.0f ? 1.0f : 0.0f) : rect_sigmoid(b);
  }
  if (bad) atomicOr(overflow, 1);
}

__device__ __forceinline__ float unpack_floor(uint32_t word, int i) {
  return (float)(int8_t)(uint8_t)(word >> (8 * i));
}


// Column tiling (as col_tiling: whole input channels per workgroup, ncb*K <= 256 columns,
// 256 threads) with row chunks of >= 8 rows so each thread keeps 2-3 x 8 loads in flight and
// the partials stay small (nchunk x Ci x S doubles); ~1536 workgroups at most per weight.
// A/B tuning (tools/adashift_bench.py --blocks): SSQ_PREP_WGS = target workgroups per
// weight, SSQ_PREP_ROWS = minimum rows per chunk; read once.
static uint32_t prep_env(const char* name, uint32_t dflt) {
  const char* v = getenv(name);
  return v && *v ? (uint32_t)atoi(v) : dflt;
}
static ColTiling col_tiling_prep(const Geo& g) {
  static const uint32_t kWgs = prep_env("SSQ_PREP_WGS", 1536);
  static const uint32_t kRows = prep_env("SSQ_PREP_ROWS", kRBP);
  ColTiling t;
  t.ncb = g.K >= (uint32_t)kBlock ? 1u : (uint32_t)kBlock / g.K;
  if (t.ncb > g.Ci) t.ncb = g.Ci;
  t.ncolblk = (g.Ci + t.ncb - 1) / t.ncb;
  t.threads = kBlock;
  uint32_t want = kWgs / t.ncolblk;
  const uint32_t by_rows = (g.Co + kRows - 1) / kRows;
  if (want > by_rows) want = by_rows;
  if (want > kMaxChunks) want = kMaxChunks;
  if (want < 1) want = 1;
  t.R = (g.Co + want - 1) / want;
  t.nchunk = (g.Co + t.R - 1) / t.R;
  t.whole = 0;
  t.form = 0;
  return t;
}

// Alpha-backward tiling.  Weights with Co*K <= 2304 (ResNet-18 layer1 - layer3 3x3 convs)
// and 1x1 weights with Co <= 256 take one workgroup per input channel (alpha_bwd_channel,
// channels in XCD-aware order): its 256 threads take the channel's Co*K (row, tap) elements
// -- thread t: elements t, t + 256, ..., kChanPer per batch, every load of a batch issued
// before any math, the next batch while the current one is summed -- and reduce them in the
// workgroup (fixed shuffle tree per wave, then the
// 4 waves in order): one launch, no partials, and as many workgroups as input channels.
// Larger weights keep the thread-column tiling of the forward (chunks of rows) and a stage-2
// launch that sums the chunk partials.  The tiling depends only on the weight's own shape, so
// a multi-segment launch gives each weight its single-launch bits.
//
// Measured and not kept (tools/alpha_cold.py; profiles/r3_alpha_variants.txt,
// profiles/r4_k6p_forms.txt): a wave-column form (one wave-width of columns over all rows,
// Co <= 64: 10 workgroups for a layer1 conv, bound by those few CUs' loads) -- 10.4 us on
// layer1 against 8.3 us here; one-launch forms that hand the chunk partials to the last
// arriving workgroup of a column block (write-through partials, a device-scope ticket) --
// 6-13 us slower than the stage-2 launch they save; and this form with 9 elements per thread
// (up to Co*K = 2304, layer3 3x3) -- equal on layer3 (16.0 vs 15.8 us) but its registers
// (97 VGPRs) cost the other forms' occupancy.
constexpr uint32_t kChanPer = 5;                      // elements per thread per batch
constexpr uint32_t kChanElems = kChanPer * kBlock;    // 1280: one batch
constexpr uint32_t kChanBatches = 4;                  // batches in the per-channel form

// XCD-aware channel order of the per-channel form: workgroups b and b + 8 share an XCD (and
// its L2), and neighbouring input channels share cache lines (K = 9: a row's 36 B of channel
// ci sit next to ci + 1's; K = 1: 32 channels per 128-B line), so the workgroups one XCD
// runs take a contiguous run of channels: local workgroup j -> the (j / 8)-th channel of
// run j % 8.  A bijection on [0, n) for any n; per-channel sums are unchanged.
__device__ __forceinline__ uint32_t xcd_channel(uint32_t j, uint32_t n) {
  const uint32_t q = n >> 3, rem = n & 7, r = j & 7;
  return r * q + min(r, rem) + (j >> 3);
}

static ColTiling bwd_tiling_prep(const Geo& g) {
  // SSQ_K6P_FORM (A/B): 3 = the per-channel form where it fits, else thread-column (default);
  // 0 = thread-column stage 1 + stage 2 everywhere
  static const uint32_t kForm = prep_env("SSQ_K6P_FORM", 3);
  // rows per channel: a thread's elements sit one row (Ci*K floats) apart, so a 1x1 weight
  // with many rows is read as Co scattered words per workgroup (r4, cold whole-block launches:
  // layer4.0 with its 512-row downsample here 20.1 -> 26.3 us, layer3.0 with its 256-row one
  // 9.2 -> 11.8 us; layer2.0's 128-row one in a single launch 13.0 -> 9.8 us, stage 2
  // included) -- before the XCD-aware channel order (xcd_channel), which puts the 32
  // channels sharing a 1x1 row's cache line on one XCD; SSQ_K6P_CHAN_CO for A/B
  static const uint32_t kMaxCo = prep_env("SSQ_K6P_CHAN_CO", 256);
  // elements per input channel the per-channel form takes: up to kChanBatches batches of
  // kChanPer per thread, each batch's loads issued while the previous one is summed
  // (SSQ_K6P_CHAN_ELEMS, A/B).  r4: one batch (1280); r5: 2304 = ResNet-18 layer3's 3x3
  // convs in two batches, so layer3 blocks take one launch.  Cold whole-block launches
  // (profiles/r5_k6p_xcd_ab.txt), XCD order on: layer3.0 15.4 us in one launch vs 9.4 + 6.3
  // in two; layer4 (Co*K = 4608, four batches) 29-34 us vs 20.4-24.1 + 6.2, so layer4 keeps
  // two.  In the loop (bench.py recon, r5y): layer3.0 / 3.1 alpha backward 13.4 / 13.1 us vs
  // 14.5 / 14.7, it/s 1996-1999 / 2024-2031 vs 1990-1991 / 2014-2023.
  static const uint32_t kMaxElems = prep_env("SSQ_K6P_CHAN_ELEMS", 2304);
  if (kForm != 3 || g.Co * g.K > kMaxElems || g.Co * g.K > kChanBatches * kChanElems ||
      (g.Co > kMaxCo && g.K == 1))
    return col_tiling_prep(g);
  ColTiling t;
  t.form = 3;
  t.threads = kBlock;
  t.ncb = 1;
  t.ncolblk = g.Ci;
  t.R = g.Co;
  t.nchunk = 1;
  // SSQ_K6P_XCD (A/B): 1 = XCD-aware channel order (whole = 2), 0 = channel = workgroup
  static const uint32_t kXcd = prep_env("SSQ_K6P_XCD", 1);
  t.whole = kXcd ? 2 : 1;
  return t;
}

struct PrepSeg {
  const uint32_t* fpack;
  const float* hterm;
  const float* alpha;
  const float* delta;
  const float* zp;
  const float* gWhat;
  float* What;
  double* part;
  float* galpha;
  float* reg_vals;
  Geo g;
  ColTiling tl;
  uint32_t blk0;     // first workgroup of this segment (forward / stage 1)
  uint32_t wave0;    // first wave of this segment (stage 2: one wave per input channel)
  uint32_t stage2;   // its chunks are reduced by the stage-2 launch
  FastDiv divK;      // per-channel form: (row, tap) of a flat element index
  float lo, hi;
  float* alpha_w;    // fused optimizer step (ssq_adam_arm): alpha, its Adam m / v (or null)
  float* am;
  float* av;
};
struct PrepTable {
  PrepSeg s[kMaxPrepSeg];
  int nseg;
  AdamConst ac;
};
static_assert(kMaxPrepSeg <= kMaxAdamSegs, "adam_attach covers one launch's segments");
static_assert(sizeof(PrepTable) + sizeof(FinTable) + 64 <= 4096, "kernel arguments over 4 KiB");

// the segment of workgroup (or wave) `id` (uniform: the table is read with scalar loads
// from the kernel arguments, as ssq_adam's)
template <bool BY_WAVE>
__device__ __forceinline__ int find_seg(const PrepTable& tab, uint32_t id) {
  int si = 0;
  while (si + 1 < tab.nseg && id >= (BY_WAVE ? tab.s[si + 1].wave0 : tab.s[si + 1].blk0)) ++si;
  return si;
}

// Forward: thread t of the workgroup owns column j = ci0*K + t of the chunk's rows.  Every
// load is in flight before any math: the alpha row first (loads retire in order, so its
// wait leaves the rows in flight), then the first row batch; each later batch is fetched
// before the current one is stored.
template <int NS, int HARD_T>
__device__ __forceinline__ void shift_fwd_body(const PrepTable& tab, uint32_t bid) {
  const PrepSeg& sg = tab.s[find_seg<false>(tab, bid)];
  const Geo& g = sg.g;
  const uint32_t local = bid - sg.blk0;
  const uint32_t bx = local % sg.tl.ncolblk, by = local / sg.tl.ncolblk;
  const uint32_t ci0 = bx * sg.tl.ncb;
  const uint32_t nci = min(sg.tl.ncb, g.Ci - ci0);
  const uint32_t t = threadIdx.x;
  if (t >= nci * g.K) return;
  const uint32_t ci = ci0 + t / g.K, j = ci0 * g.K + t;
  const uint32_t co0 = by * sg.tl.R, co1 = min(co0 + sg.tl.R, g.Co);
  const uint32_t* __restrict__ fpack = sg.fpack;
  const float* __restrict__ hterm = sg.hterm;
  const float* __restrict__ delta = sg.delta;
  const float* __restrict__ zp = sg.zp;
  float* __restrict__ What = sg.What;
  const float lo = sg.lo, hi = sg.hi;
  float a[kMaxS];
  load_row(sg.alpha, ci, NS, a);
  uint32_t fw[kRBP];
  float h[kRBP], d[kRBP], z[kRBP];
  auto fetch = [&](uint32_t c) {
#pragma unroll
    for (int r = 0; r < kRBP; ++r) {
      fw[r] = 0u;
      h[r] = d[r] = z[r] = 0.0f;
      if (c + r < co1) {
        const uint32_t e = (c + r) * g.CiK + j;
        fw[r] = fpack[e];
        h[r] = hterm[e];
        d[r] = delta[c + r];
        z[r] = zp[c + r];
      }
    }
  };
  fetch(co0);
  float p[kMaxS];
  soft_targets<kMaxS>(a, NS, nullptr, p);
  const int sel = argmax_first(p, NS);
  for (uint32_t co = co0; co < co1; co += kRBP) {
    float o[kRBP];
#pragma unroll
    for (int r = 0; r < kRBP; ++r) {
      float xf;
      if (HARD_T) {
        xf = unpack_floor(fw[r], sel);
      } else {
        xf = __fmul_rn(unpack_floor(fw[r], 0), p[0]);
#pragma unroll
        for (int i = 1; i < NS; ++i) xf = __fadd_rn(xf, __fmul_rn(unpack_floor(fw[r], i), p[i]));
      }
      const float q = clampf(__fadd_rn(__fadd_rn(xf, h[r]), z[r]), lo, hi);
      o[r] = __fmul_rn(__fsub_rn(q, z[r]), __fmul_rn(d[r], 1.0f));
    }
    if (co + kRBP < co1) fetch(co + kRBP);
#pragma unroll
    for (int r = 0; r < kRBP; ++r)
      if (co + r < co1) What[(co + r) * g.CiK + j] = o[r];
  }
}

template <int NS, int HARD_T>
__global__ __launch_bounds__(kBlock) void shift_fwd_prep(PrepTable tab) {
  shift_fwd_body<NS, HARD_T>(tab, blockIdx.x);
}

// The iteration start (prep_ride.h): workgroups [0, ngw) gather the batch rows, the rest
// run the queued prepared forward.
// nfwd > 0: the forward's nfwd workgroups come first (dispatched first, so their short,
// latency-bound bodies run beside the gather's stream instead of after it); 0: after.
template <bool VEC, int NS, int HARD_T>
__global__ __launch_bounds__(kBlock) void gather_shift_fwd(GatherArgs ga, uint32_t ngw,
                                                           PrepTable tab, uint32_t nfwd) {
  if (nfwd) {
    if (blockIdx.x < nfwd) {
      shift_fwd_body<NS, HARD_T>(tab, blockIdx.x);
      return;
    }
    const uint32_t b = blockIdx.x - nfwd;
    gather2_body<VEC>(ga, b % ga.gx, b / ga.gx);
    return;
  }
  if (blockIdx.x < ngw) {
    gather2_body<VEC>(ga, blockIdx.x % ga.gx, blockIdx.x / ga.gx);
    return;
  }
  shift_fwd_body<NS, HARD_T>(tab, blockIdx.x - ngw);
}

template <bool VEC>
__global__ __launch_bounds__(kBlock) void gather2_kernel(GatherArgs ga) {
  gather2_body<VEC>(ga, blockIdx.x, blockIdx.y);
}

// d/dalpha of one weight element: the unclamped rounding u = sum_i F_i p_i + h + zp passes
// the clamp's gradient (inclusive bounds) and contributes g_int * F_i to shift i's sum.
template <int NS>
__device__ __forceinline__ void alpha_accumulate(uint32_t fw, float h, float d, float z, float gy,
                                                 const float* p, float lo, float hi,
                                                 double* acc) {
  float F[NS];
#pragma unroll
  for (int i = 0; i < NS; ++i) F[i] = unpack_floor(fw, i);
  float xf = __fmul_rn(F[0], p[0]);
#pragma unroll
  for (int i = 1; i < NS; ++i) xf = __fadd_rn(xf, __fmul_rn(F[i], p[i]));
  const float u = __fadd_rn(__fadd_rn(xf, h), z);
  const float gi = (u >= lo && u <= hi) ? __fmul_rn(gy, __fmul_rn(d, 1.0f)) : 0.0f;
#pragma unroll
  for (int i = 0; i < NS; ++i) acc[i] += (double)gi * (double)F[i];
}

// Input channel ci of the segment in one workgroup (bwd_tiling_prep form 3).
template <int NS>
__device__ __forceinline__ void alpha_bwd_channel(const PrepSeg& sg, const AdamConst& ac,
                                                  uint32_t ci, double* red, float reg_lambda,
                                                  float reg_b, const float* __restrict__ reg_dev) {
  const Geo& g = sg.g;
  const uint32_t n = g.Co * g.K, t = threadIdx.x;
  const uint32_t lane = t & (kWave - 1), w = t / kWave;
  float a[kMaxS];
  load_row(sg.alpha, ci, NS, a);
  float pp[kMaxS], pm[kMaxS], pv[kMaxS];
  const bool fin = t == 0;
  if (fin && sg.am) {                 // the armed Adam state, loaded with everything else
#pragma unroll
    for (int i = 0; i < NS; ++i) {
      pp[i] = sg.alpha_w[(size_t)ci * NS + i];
      pm[i] = sg.am[(size_t)ci * NS + i];
      pv[i] = sg.av[(size_t)ci * NS + i];
    }
  }
  if (reg_dev) {
    reg_lambda = reg_dev[0];
    reg_b = reg_dev[1];
  }
  uint32_t fw[kChanPer];
  float h[kChanPer], gy[kChanPer], d[kChanPer], z[kChanPer];
  // batch b: elements t + (b * kChanPer + e) * kBlock
  auto fetch = [&](uint32_t b) {
#pragma unroll
    for (uint32_t e = 0; e < kChanPer; ++e) {
      const uint32_t f = t + (b * kChanPer + e) * kBlock;
      fw[e] = 0u;
      h[e] = gy[e] = d[e] = z[e] = 0.0f;
      if (f < n) {
        const uint32_t co = fdiv(f, sg.divK);
        const uint32_t idx = co * g.CiK + ci * g.K + (f - co * g.K);
        fw[e] = sg.fpack[idx];
        h[e] = sg.hterm[idx];
        gy[e] = sg.gWhat[idx];
        d[e] = sg.delta[co];
        z[e] = sg.zp[co];
      }
    }
  };
  fetch(0);
  float p[kMaxS];
  soft_targets<kMaxS>(a, NS, nullptr, p);
  double acc[NS];
#pragma unroll
  for (int i = 0; i < NS; ++i) acc[i] = 0.0;
  const uint32_t nb = (n + kChanElems - 1) / kChanElems;   // uniform per workgroup
  for (uint32_t b = 0; b < nb; ++b) {
    uint32_t fw1[kChanPer];
    float h1[kChanPer], gy1[kChanPer], d1[kChanPer], z1[kChanPer];
#pragma unroll
    for (uint32_t e = 0; e < kChanPer; ++e) {
      fw1[e] = fw[e];
      h1[e] = h[e];
      gy1[e] = gy[e];
      d1[e] = d[e];
      z1[e] = z[e];
    }
    if (b + 1 < nb) fetch(b + 1);
#pragma unroll
    for (uint32_t e = 0; e < kChanPer; ++e)
      if (t + (b * kChanPer + e) * kBlock < n)
        alpha_accumulate<NS>(fw1[e], h1[e], d1[e], z1[e], gy1[e], p, sg.lo, sg.hi, acc);
  }
#pragma unroll
  for (int i = 0; i < NS; ++i) acc[i] = wave_sum(acc[i]);
  if (lane == 0) {
#pragma unroll
    for (int i = 0; i < NS; ++i) red[w * NS + i] = acc[i];
  }
  __syncthreads();
  if (!fin) return;
  double tot[kMaxS];
#pragma unroll
  for (int i = 0; i < NS; ++i) {
    double s = red[i];
#pragma unroll
    for (int k = 1; k < kBlock / kWave; ++k) s += red[k * NS + i];
    tot[i] = s;
  }
  float sm[kMaxS], ga[kMaxS];
  soft_targets<kMaxS>(a, NS, sm, p);
  float reg = 0.0f;
  if (reg_lambda != 0.0f) {
    double racc = 0.0;
#pragma unroll
    for (int i = 0; i < NS; ++i) {
      double rv, rg;
      reg_term(p[i], reg_lambda, reg_b, 0, rv, rg);
      racc += rv;
      tot[i] += rg;
    }
    reg = (float)((double)reg_lambda * racc);
  }
  softmax_clamp_bwd(sm, NS, tot, ga);
#pragma unroll
  for (int i = 0; i < NS; ++i) sg.galpha[(size_t)ci * NS + i] = ga[i];
  if (sg.reg_vals) sg.reg_vals[ci] = reg;
  if (sg.am) {
    const AdamRef r{sg.alpha_w, sg.am, sg.av};
#pragma unroll
    for (int i = 0; i < NS; ++i)
      adam_apply_loaded(ac, r, (uint32_t)(ci * NS + i), ga[i], pp[i], pm[i], pv[i]);
  }
}

// Backward, one launch for every segment: per-channel segments finish here; the
// thread-column stage 1 of the others writes sums of g_int * F_i per (chunk, ci) into
// part[(ci*nchunk + chunk)*S + i] (input-channel-major: stage 2 reads one coalesced run).
template <int NS>
__global__ __launch_bounds__(kBlock) void alpha_bwd_prep(PrepTable tab, float reg_lambda,
                                                          float reg_b,
                                                          const float* __restrict__ reg_dev,
                                                          FinTable fin, uint32_t nmain) {
  // queued finalize tasks (fin_tasks.h) ride on this launch: its first workgroups
  (void)nmain;
  if (blockIdx.x < fin.nwg) {
    run_fin(fin, blockIdx.x);
    return;
  }
  const uint32_t bid = blockIdx.x - fin.nwg;
  __shared__ double red[kBlock * NS];
  const PrepSeg& sg = tab.s[find_seg<false>(tab, bid)];
  const Geo& g = sg.g;
  const uint32_t local = bid - sg.blk0;
  if (sg.tl.form == 3) {             // uniform per workgroup
    const uint32_t ci = sg.tl.whole == 2 ? xcd_channel(local, g.Ci) : local;
    alpha_bwd_channel<NS>(sg, tab.ac, ci, red, reg_lambda, reg_b, reg_dev);
    return;
  }
  const uint32_t bx = local % sg.tl.ncolblk, by = local / sg.tl.ncolblk;
  const uint32_t ci0 = bx * sg.tl.ncb;
  const uint32_t nci = min(sg.tl.ncb, g.Ci - ci0);
  const uint32_t t = threadIdx.x;
  double acc[NS];
#pragma unroll
  for (int i = 0; i < NS; ++i) acc[i] = 0.0;
  if (t < nci * g.K) {
    const uint32_t ci = ci0 + t / g.K, j = ci0 * g.K + t;
    const uint32_t* __restrict__ fpack = sg.fpack;
    const float* __restrict__ hterm = sg.hterm;
    const float* __restrict__ gWhat = sg.gWhat;
    const float* __restrict__ delta = sg.delta;
    const float* __restrict__ zp = sg.zp;
    const uint32_t co0 = by * sg.tl.R, co1 = min(co0 + sg.tl.R, g.Co);
    // the alpha row first, then the first row batch, both before the softmax (loads retire
    // in order: the alpha wait leaves the rows in flight); each later batch is fetched
    // before the current one is accumulated.  Rows are added in order, as before.
    float a[kMaxS], p[kMaxS];
    load_row(sg.alpha, ci, NS, a);
    uint32_t fw[kRBP];
    float h[kRBP], d[kRBP], z[kRBP], gy[kRBP];
    auto fetch = [&](uint32_t c) {
#pragma unroll
      for (int r = 0; r < kRBP; ++r) {
        fw[r] = 0u;
        h[r] = d[r] = z[r] = gy[r] = 0.0f;
        if (c + r < co1) {
          const uint32_t e = (c + r) * g.CiK + j;
          fw[r] = fpack[e];
          h[r] = hterm[e];
          gy[r] = gWhat[e];
          d[r] = delta[c + r];
          z[r] = zp[c + r];
        }
      }
    };
    fetch(co0);
    soft_targets<kMaxS>(a, NS, nullptr, p);
    for (uint32_t co = co0; co < co1; co += kRBP) {
      uint32_t fw1[kRBP];
      float h1[kRBP], d1[kRBP], z1[kRBP], gy1[kRBP];
#pragma unroll
      for (int r = 0; r < kRBP; ++r) {
        fw1[r] = fw[r];
        h1[r] = h[r];
        d1[r] = d[r];
        z1[r] = z[r];
        gy1[r] = gy[r];
      }
      if (co + kRBP < co1) fetch(co + kRBP);
#pragma unroll
      for (int r = 0; r < kRBP; ++r)
        if (co + r < co1)
          alpha_accumulate<NS>(fw1[r], h1[r], d1[r], z1[r], gy1[r], p, sg.lo, sg.hi, acc);
    }
  }
#pragma unroll
  for (int i = 0; i < NS; ++i) red[t * NS + i] = acc[i];
  __syncthreads();
  if (t < nci) {
#pragma unroll
    for (int i = 0; i < NS; ++i) {
      double sum = 0.0;
      for (uint32_t k = 0; k < g.K; ++k) sum += red[(t * g.K + k) * NS + i];
      sg.part[((size_t)(ci0 + t) * sg.tl.nchunk + by) * NS + i] = sum;
    }
  }
}

// Stage 2 (thread-column segments): one wave per (segment, input channel).  Every load the wave needs (alpha row, the device (lambda, b)
// pair, lane c's chunks c, c+64, ... -- one coalesced run per round) is issued before any
// math; lanes i < S evaluate shift i's regulariser term meanwhile; a fixed shuffle tree adds
// the lanes and lane 0 applies the softmax/clamp backward (same values, same order as
// alpha_chain).  Deterministic, no atomics.
constexpr uint32_t kMaxPrepChunkRounds = kMaxChunks / kWave;

template <int NS>
__global__ __launch_bounds__(kBlock) void alpha_bwd_prep_stage2(PrepTable tab, float reg_lambda,
                                                                 float reg_b,
                                                                 const float* __restrict__ reg_dev) {
  const uint32_t wave = blockIdx.x * (kBlock / kWave) + threadIdx.x / kWave;
  const uint32_t lane = threadIdx.x & (kWave - 1);
  const PrepSeg& sg = tab.s[find_seg<true>(tab, __builtin_amdgcn_readfirstlane(wave))];
  const uint32_t ci = wave - sg.wave0;
  if (!sg.stage2 || ci >= sg.g.Ci) return;
  const uint32_t nchunk = sg.tl.nchunk;
  float a[kMaxS];
  load_row(sg.alpha, ci, NS, a);
  float ap[kMaxS], am[kMaxS], av[kMaxS];   // the armed Adam state, loaded with the partials
  if (sg.am && lane == 0) {
#pragma unroll
    for (int i = 0; i < NS; ++i) {
      ap[i] = sg.alpha_w[(size_t)ci * NS + i];
      am[i] = sg.am[(size_t)ci * NS + i];
      av[i] = sg.av[(size_t)ci * NS + i];
    }
  }
  if (reg_dev) {
    reg_lambda = reg_dev[0];
    reg_b = reg_dev[1];
  }
  const double* pp = sg.part + (size_t)ci * nchunk * NS;
  double v[kMaxPrepChunkRounds][NS];
#pragma unroll
  for (uint32_t r = 0; r < kMaxPrepChunkRounds; ++r) {
    const uint32_t c = lane + r * kWave;
#pragma unroll
    for (int i = 0; i < NS; ++i) v[r][i] = c < nchunk ? pp[(size_t)c * NS + i] : 0.0;
  }
  float sm[kMaxS], p[kMaxS];
  soft_targets<kMaxS>(a, NS, sm, p);
  double rv = 0.0, rg = 0.0;
  if (reg_lambda != 0.0f && lane < (uint32_t)NS) {
    float pl = p[0];
#pragma unroll
    for (int i = 1; i < NS; ++i)
      if ((uint32_t)i == lane) pl = p[i];
    reg_term(pl, reg_lambda, reg_b, 0, rv, rg);
  }
  double tot[kMaxS];
#pragma unroll
  for (int i = 0; i < NS; ++i) {
    tot[i] = v[0][i];
#pragma unroll
    for (uint32_t r = 1; r < kMaxPrepChunkRounds; ++r) tot[i] += v[r][i];
    tot[i] = wave_sum(tot[i]);
  }
  double rvs[kMaxS], rgs[kMaxS];
#pragma unroll
  for (int i = 0; i < NS; ++i) {
    rvs[i] = __shfl(rv, i, kWave);
    rgs[i] = __shfl(rg, i, kWave);
  }
  if (lane != 0) return;
  float ga[kMaxS], reg = 0.0f;
  if (reg_lambda != 0.0f) {
    double acc = 0.0;
#pragma unroll
    for (int i = 0; i < NS; ++i) {
      acc += rvs[i];
      tot[i] += rgs[i];
    }
    reg = (float)((double)reg_lambda * acc);
  }
  softmax_clamp_bwd(sm, NS, tot, ga);
#pragma unroll
  for (int i = 0; i < NS; ++i) sg.galpha[(size_t)ci * NS + i] = ga[i];
  if (sg.reg_vals) sg.reg_vals[ci] = reg;
  if (sg.am) {                        // the fused optimizer step
    const AdamRef r{sg.alpha_w, sg.am, sg.av};
#pragma unroll
    for (int i = 0; i < NS; ++i)
      adam_apply_loaded(tab.ac, r, (uint32_t)(ci * NS + i), ga[i], ap[i], am[i], av[i]);
  }
}

// ------------------------------------------------------------------ host side
struct SegArgs {
  int nseg;
  const uint32_t* const* fpack;
  const float* const* hterm;
  const float* const* alpha;
  const float* const* delta;
  const float* const* zp;
  const int64_t* Co;
  const int64_t* Ci;
  const int64_t* K;
  const int* qmin;
  const int* qmax;
};

static int make_seg(const SegArgs& a, int i, PrepSeg& sg, const char* what) {
  SSQ_REQUIRE(a.fpack[i] && a.hterm[i] && a.alpha[i] && a.delta[i] && a.zp[i], SSQ_E_ARG,
              "%s: null pointer in segment %d", what, i);
  const int rc = make_geo(a.Co[i], a.Ci[i], a.K[i], 0, sg.g);
  if (rc) return rc;
  SSQ_REQUIRE(sg.g.K <= (uint32_t)kBlock, SSQ_E_ARG, "%s: kernel window K > %d", what, kBlock);
  SSQ_REQUIRE(a.qmin[i] < a.qmax[i], SSQ_E_ARG, "%s: qmin >= qmax", what);
  sg.fpack = a.fpack[i];
  sg.hterm = a.hterm[i];
  sg.alpha = a.alpha[i];
  sg.delta = a.delta[i];
  sg.zp = a.zp[i];
  sg.gWhat = nullptr;
  sg.What = nullptr;
  sg.part = nullptr;
  sg.galpha = nullptr;
  sg.reg_vals = nullptr;
  sg.alpha_w = sg.am = sg.av = nullptr;
  sg.divK = make_fastdiv(sg.g.K);
  sg.tl = col_tiling_prep(sg.g);
  sg.lo = (float)a.qmin[i];
  sg.hi = (float)a.qmax[i];
  return SSQ_OK;
}

static size_t part_bytes(const PrepSeg& sg, int S) {
  const size_t b = (size_t)sg.tl.nchunk * sg.g.Ci * S * sizeof(double);
  return (b + 255) / 256 * 256;
}

// ------------------------------------------------------------------ deferred forward
struct PendingFwd {
  bool on;
  hipStream_t s;
  PrepTable tab;
  uint32_t blk;
  int S, hard;
};
static bool g_fwd_defer = false;
static PendingFwd g_fwd_pend{};

static int launch_fwd(hipStream_t s, const PrepTable& tab, uint32_t blk, int S, int hard) {
#define SSQ_FWDP(NS)                                                                         \
  do {                                                                                       \
    if (hard)                                                                                \
      hipLaunchKernelGGL((shift_fwd_prep<NS, 1>), dim3(blk), dim3(kBlock), 0, s, tab);       \
    else                                                                                     \
      hipLaunchKernelGGL((shift_fwd_prep<NS, 0>), dim3(blk), dim3(kBlock), 0, s, tab);       \
  } while (0)
  switch (S) {
    case 1: SSQ_FWDP(1); break;
    case 2: SSQ_FWDP(2); break;
    case 3: SSQ_FWDP(3); break;
    default: SSQ_FWDP(4); break;
  }
#undef SSQ_FWDP
  return check_launch("ssq_adashift_fwd_prepared_multi");
}

static int flush_fwd(hipStream_t s) {
  if (!g_fwd_pend.on || g_fwd_pend.s != s) return SSQ_OK;
  g_fwd_pend.on = false;
  return launch_fwd(s, g_fwd_pend.tab, g_fwd_pend.blk, g_fwd_pend.S, g_fwd_pend.hard);
}

int launch_gather(hipStream_t s, const GatherArgs& a, bool vec) {
  if (!(g_fwd_defer && g_fwd_pend.on && g_fwd_pend.s == s)) {
    const dim3 grid(a.gx, a.nrows);
    if (vec)
      hipLaunchKernelGGL(gather2_kernel<true>, grid, dim3(kBlock), 0, s, a);
    else
      hipLaunchKernelGGL(gather2_kernel<false>, grid, dim3(kBlock), 0, s, a);
    return SSQ_OK;
  }
  const PendingFwd f = g_fwd_pend;
  g_fwd_pend.on = false;
  const uint32_t ngw = a.gx * a.nrows;
  const dim3 grid(ngw + f.blk);
  // The forward's workgroups first in the grid when they are a short tail beside the gather
  // (at most half its workgroups: ResNet-18 layer1 - layer3); after it when the forward is
  // the launch's bulk (layer4: 56 MB of weights against a 13 MB batch), so the What the
  // next conv reads are the launch's last writes.  bench.py's recon loops (r5k5, ABAB):
  // forward first, traced start launch 0.4-1.2 us shorter on every block and layer3 it/s
  // +0.7 %, but layer4.0 / 4.1 -0.6 / -1.6 %.  SSQ_K5P_FIRST=0: always after (A/B).
  static const bool kFirst = prep_env("SSQ_K5P_FIRST", 1) != 0;
  const uint32_t nfwd = kFirst && 2 * f.blk <= ngw ? f.blk : 0;
#define SSQ_GF(V, NS)                                                                        \
  do {                                                                                       \
    if (f.hard)                                                                              \
      hipLaunchKernelGGL((gather_shift_fwd<V, NS, 1>), grid, dim3(kBlock), 0, s, a, ngw, f.tab, nfwd); \
    else                                                                                     \
      hipLaunchKernelGGL((gather_shift_fwd<V, NS, 0>), grid, dim3(kBlock), 0, s, a, ngw, f.tab, nfwd); \
  } while (0)
#define SSQ_GFS(V)                    \
  switch (f.S) {                      \
    case 1: SSQ_GF(V, 1); break;      \
    case 2: SSQ_GF(V, 2); break;      \
    case 3: SSQ_GF(V, 3); break;      \
    default: SSQ_GF(V, 4); break;     \
  }
  if (vec) {
    SSQ_GFS(true)
  } else {
    SSQ_GFS(false)
  }
#undef SSQ_GFS
#undef SSQ_GF
  return SSQ_OK;
}

}  // namespace ssq

using namespace ssq;

extern "C" int ssq_adashift_prepare(const float* W, const float* beta, const float* delta,
                                    const float* shifts, int S, int64_t Co, int64_t Ci, int64_t K,
                                    int hard_round, uint32_t* fpack, float* hterm, int* overflow,
                                    ssq_stream_t stream) {
  SSQ_GEO(Co, Ci, K, 0, g);
  SSQ_SHIFTS(shifts, S, sh);
  SSQ_REQUIRE(S <= kMaxPrepS, SSQ_E_ARG, "ssq_adashift_prepare: S <= %d", kMaxPrepS);
  SSQ_REQUIRE(W && beta && delta && fpack && hterm && overflow, SSQ_E_ARG,
              "ssq_adashift_prepare: null");
  const uint32_t n = g.Co * g.CiK;
  hipLaunchKernelGGL(adashift_prepare_kernel, dim3(grid_for(n, kBlock)), dim3(kBlock), 0,
                     (hipStream_t)stream, W, beta, delta, sh, g, n, hard_round, fpack, hterm,
                     overflow);
  return check_launch("ssq_adashift_prepare");
}

extern "C" int ssq_adashift_fwd_prepared_multi(int nseg, const uint32_t* const* fpack,
                                               const float* const* hterm,
                                               const float* const* alpha,
                                               const float* const* delta, const float* const* zp,
                                               const int64_t* Co, const int64_t* Ci,
                                               const int64_t* K, const int* qmin, const int* qmax,
                                               int S, int hard_targets, float* const* What,
                                               ssq_stream_t stream) {
  const char* what = "ssq_adashift_fwd_prepared_multi";
  SSQ_REQUIRE(nseg >= 1 && fpack && hterm && alpha && delta && zp && Co && Ci && K && qmin &&
                  qmax && What, SSQ_E_ARG, "%s: bad arrays", what);
  SSQ_REQUIRE(S >= 1 && S <= kMaxPrepS, SSQ_E_ARG, "%s: 1 <= S <= %d", what, kMaxPrepS);
  const SegArgs a{nseg, fpack, hterm, alpha, delta, zp, Co, Ci, K, qmin, qmax};
  hipStream_t s = (hipStream_t)stream;
  for (int base = 0; base < nseg; base += kMaxPrepSeg) {
    PrepTable tab;
    tab.nseg = nseg - base < kMaxPrepSeg ? nseg - base : kMaxPrepSeg;
    uint32_t blk = 0;
    for (int k = 0; k < tab.nseg; ++k) {
      PrepSeg& sg = tab.s[k];
      const int rc = make_seg(a, base + k, sg, what);
      if (rc) return rc;
      SSQ_REQUIRE(What[base + k], SSQ_E_ARG, "%s: null What", what);
      sg.What = What[base + k];
      sg.blk0 = blk;
      sg.wave0 = 0;
      sg.stage2 = 0;
      blk += sg.tl.ncolblk * sg.tl.nchunk;
    }
    // deferred: this table rides on the stream's next gather (prep_ride.h); a table still
    // queued from an earlier call is launched first
    int rc = g_fwd_pend.on ? flush_fwd(g_fwd_pend.s) : SSQ_OK;
    if (rc) return rc;
    if (g_fwd_defer && nseg <= kMaxPrepSeg) {
      g_fwd_pend.on = true;
      g_fwd_pend.s = s;
      g_fwd_pend.tab = tab;
      g_fwd_pend.blk = blk;
      g_fwd_pend.S = S;
      g_fwd_pend.hard = hard_targets;
      return SSQ_OK;
    }
    rc = launch_fwd(s, tab, blk, S, hard_targets);
    if (rc) return rc;
  }
  return SSQ_OK;
}

extern "C" int ssq_set_deferred_prep_fwd(int on) {
  const int prev = g_fwd_defer ? 1 : 0;
  g_fwd_defer = on != 0;
  // switching off: a forward still queued (on whichever stream) launches now, on its stream
  if (!g_fwd_defer && g_fwd_pend.on) (void)flush_fwd(g_fwd_pend.s);
  return prev;
}

extern "C" int ssq_flush_prep_fwd(ssq_stream_t stream) { return flush_fwd((hipStream_t)stream); }

extern "C" size_t ssq_adashift_bwd_prepared_multi_workspace_size(int nseg, const int64_t* Co,
                                                                 const int64_t* Ci,
                                                                 const int64_t* K, int S) {
  if (nseg < 1 || !Co || !Ci || !K || S < 1 || S > kMaxPrepS) return 0;
  size_t total = 0;
  for (int i = 0; i < nseg; ++i) {
    PrepSeg sg;
    if (make_geo(Co[i], Ci[i], K[i], 0, sg.g) != SSQ_OK) return 0;
    sg.tl = bwd_tiling_prep(sg.g);
    total += part_bytes(sg, S);
  }
  return total;
}

extern "C" int ssq_adashift_bwd_prepared_multi(
    int nseg, const float* const* gWhat, const uint32_t* const* fpack, const float* const* hterm,
    const float* const* alpha, const float* const* delta, const float* const* zp,
    const int64_t* Co, const int64_t* Ci, const int64_t* K, const int* qmin, const int* qmax,
    int S, float reg_lambda, float reg_b, const float* reg_dev, float* const* galpha,
    float* const* reg_vals, void* ws, size_t ws_bytes, ssq_stream_t stream) {
  const char* what = "ssq_adashift_bwd_prepared_multi";
  SSQ_REQUIRE(nseg >= 1 && gWhat && fpack && hterm && alpha && delta && zp && Co && Ci && K &&
                  qmin && qmax && galpha, SSQ_E_ARG, "%s: bad arrays", what);
  SSQ_REQUIRE(S >= 1 && S <= kMaxPrepS, SSQ_E_ARG, "%s: 1 <= S <= %d", what, kMaxPrepS);
  SSQ_REQUIRE(ws && ws_bytes >= ssq_adashift_bwd_prepared_multi_workspace_size(nseg, Co, Ci, K, S),
              SSQ_E_WS, "%s: workspace too small", what);
  const SegArgs a{nseg, fpack, hterm, alpha, delta, zp, Co, Ci, K, qmin, qmax};
  hipStream_t s = (hipStream_t)stream;
  char* wsp = (char*)ws;
  for (int base = 0; base < nseg; base += kMaxPrepSeg) {
    PrepTable tab;
    tab.nseg = nseg - base < kMaxPrepSeg ? nseg - base : kMaxPrepSeg;
    uint32_t blk = 0, waves = 0;
    for (int k = 0; k < tab.nseg; ++k) {
      PrepSeg& sg = tab.s[k];
      const int i = base + k;
      const int rc = make_seg(a, i, sg, what);
      if (rc) return rc;
      SSQ_REQUIRE(gWhat[i] && galpha[i], SSQ_E_ARG, "%s: null gWhat/galpha", what);
      sg.tl = bwd_tiling_prep(sg.g);
      sg.gWhat = gWhat[i];
      sg.galpha = galpha[i];
      sg.reg_vals = reg_vals ? reg_vals[i] : nullptr;
      sg.part = (double*)wsp;
      wsp += part_bytes(sg, S);
      sg.blk0 = blk;
      blk += sg.tl.ncolblk * sg.tl.nchunk;
      sg.stage2 = sg.tl.form == 0;
      sg.wave0 = waves;
      if (sg.stage2) waves += sg.g.Ci;
    }
    const unsigned blocks2 = (waves + kBlock / kWave - 1) / (kBlock / kWave);
    const size_t shm = 0;
    // queued finalize tasks of this stream ride on the first launch (their inputs live in
    // their producers' own workspace slots, not in this one)
    FinTable fin{};
    if (base == 0) fin = fin_take(s);
    tab.ac = AdamConst{};
    if (base == 0 && nseg <= kMaxPrepSeg) {
      // the loop's armed optimizer step, when this launch can take all of it (fin_tasks.h)
      int64_t len[kMaxPrepSeg];
      AdamRef refs[kMaxPrepSeg];
      for (int k = 0; k < tab.nseg; ++k) len[k] = Ci[k] * S;
      if (adam_attach(s, tab.nseg, alpha, len, refs, fin, &tab.ac))
        for (int k = 0; k < tab.nseg; ++k) {
          tab.s[k].alpha_w = refs[k].p;
          tab.s[k].am = refs[k].m;
          tab.s[k].av = refs[k].v;
        }
    }
#define SSQ_BWDP(NS)                                                                          \
  do {                                                                                        \
    hipLaunchKernelGGL((alpha_bwd_prep<NS>), dim3(blk + fin.nwg), dim3(kBlock), shm, s, tab,  \
                       reg_lambda, reg_b, reg_dev, fin, blk);                                 \
    if (blocks2)                                                                              \
      hipLaunchKernelGGL((alpha_bwd_prep_stage2<NS>), dim3(blocks2), dim3(kBlock), 0, s, tab, \
                         reg_lambda, reg_b, reg_dev);                                         \
  } while (0)
    switch (S) {
      case 1: SSQ_BWDP(1); break;
      case 2: SSQ_BWDP(2); break;
      case 3: SSQ_BWDP(3); break;
      default: SSQ_BWDP(4); break;
    }
#undef SSQ_BWDP
    const int rc = check_launch(what);
    if (rc) return rc;
  }
  return SSQ_OK;
}

// single-weight forms (nseg = 1)
extern "C" int ssq_adashift_fwd_prepared(const uint32_t* fpack, const float* hterm,
                                         const float* alpha, const float* delta, const float* zp,
                                         int S, int64_t Co, int64_t Ci, int64_t K, int hard_targets,
                                         int qmin, int qmax, float* What, ssq_stream_t stream) {
  return ssq_adashift_fwd_prepared_multi(1, &fpack, &hterm, &alpha, &delta, &zp, &Co, &Ci, &K,
                                         &qmin, &qmax, S, hard_targets, &What, stream);
}

extern "C" size_t ssq_adashift_bwd_prepared_workspace_size(int64_t Co, int64_t Ci, int64_t K,
                                                           int S) {
  return ssq_adashift_bwd_prepared_multi_workspace_size(1, &Co, &Ci, &K, S);
}

extern "C" int ssq_adashift_bwd_prepared(const float* gWhat, const uint32_t* fpack,
                                         const float* hterm, const float* alpha,
                                         const float* delta, const float* zp, int S, int64_t Co,
                                         int64_t Ci, int64_t K, int qmin, int qmax,
                                         float reg_lambda, float reg_b, const float* reg_dev,
                                         float* galpha, float* reg_vals, void* ws,
                                         size_t ws_bytes, ssq_stream_t stream) {
  return ssq_adashift_bwd_prepared_multi(1, &gWhat, &fpack, &hterm, &alpha, &delta, &zp, &Co, &Ci,
                                         &K, &qmin, &qmax, S, reg_lambda, reg_b, reg_dev, &galpha,
                                         reg_vals ? &reg_vals : nullptr, ws, ws_bytes, stream);
}
