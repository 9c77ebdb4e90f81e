// Deferred finalize tasks of the reconstruction iteration.
//
// Two per-iteration reductions end in a small finalize launch of their own: the lp_loss
// value (K11: 1024 workgroup partials -> 1 float) and the K13 epilogue backward's
// per-channel gamma^z / phi^z sums (+ the act quantizer's delta / zp sums).  Each such
// launch is a few microseconds of launch and load latency for a few KB of data.  With
// deferral on (ssq_set_deferred_finalize, turned on by the fused recon loop's body) the
// producing entry point does not launch its finalize: it queues it as a task on its
// stream, and the next "host" launch on that stream (epilogue_bwd_rows, the prepared alpha
// backward's first kernel) runs the queued tasks in extra workgroups at the front of its
// grid (dispatched first: they run beside the launch's own work).  The task code is kept
// lean in registers: it is inlined into those kernels, whose occupancy it sets (a 16-deep
// act-sum batch once took them from 8 to 3 waves per SIMD).
// Same device code, same summation order: bit-identical results, fewer launches.
//
// Rules that keep it correct whatever runs in between:
//   * a task's inputs live in a workspace slot only its producer writes (the Python side
//     gives lp_loss its own slot and alternates the epilogue backward between two), and
//     every producer entry first hands pending tasks to its own launch, so at most one
//     task per producer is pending;
//   * ssq_adam (which reads gamma^z / phi^z / delta gradients) attaches its update to the
//     pending tasks when it can (each parameter's step where its gradient is finalised, or
//     as a kind-3 task when that gradient is already final) and launches them as ONE
//     kernel -- no Adam launch of its own; otherwise it, the lp_loss entry points and
//     ssq_flush_finalize launch whatever is still pending as one standalone kernel first;
//     ssq_set_deferred_finalize(0) only flips the flag (it has no stream), so the caller
//     flushes before turning deferral off -- the recon loop flushes at the end of its body
//     (kernels.deferred_finalize).
#pragma once

#include "ssq_common.h"

namespace ssq {

constexpr int kLossBlocks = 1024;   // lp_loss workgroup partials
constexpr uint32_t kFinBatch = 16;  // loads in flight per thread in the row-walking finalizes
constexpr int kEpiParts = 9;        // doubles per (n, c) row of the epilogue backward
                                    // (slot 6: the fused tail's row loss; 7 / 8: its
                                    // residual epilogue's gamma / phi sums)

// The recon loop's optimizer step applied where each gradient is finalised (ssq_adam_arm):
// ssq_adam's update, torch.optim.Adam's single-tensor step, op for op.
struct AdamConst {
  float w1, b2, w2, eps;     // 1 - beta1, beta2, 1 - beta2, eps
  const float* hyper;        // device (-lr/bc1, sqrt(bc2)) of this step
};
struct AdamRef {
  float* p;                  // the parameter (nullptr: no fused step)
  float* m;
  float* v;
};
// the update of one entry: (p, m, v) -> the new values, in place
__device__ __forceinline__ void adam_update(const AdamConst& c, float g, float& p, float& m,
                                            float& v) {
  const float nss = c.hyper[0], bc2s = c.hyper[1];
  m = __fadd_rn(m, __fmul_rn(c.w1, __fsub_rn(g, m)));
  v = __fadd_rn(__fmul_rn(v, c.b2), __fmul_rn(__fmul_rn(c.w2, g), g));
  const float denom = __fadd_rn(__fdiv_rn(__fsqrt_rn(v), bc2s), c.eps);
  p = __fadd_rn(p, __fdiv_rn(__fmul_rn(nss, m), denom));
}
// the update of one entry from its loaded (p, m, v)
__device__ __forceinline__ void adam_apply_loaded(const AdamConst& c, const AdamRef& r, uint32_t e,
                                                  float g, float p, float m, float v) {
  adam_update(c, g, p, m, v);
  r.p[e] = p;
  r.m[e] = m;
  r.v[e] = v;
}
__device__ __forceinline__ void adam_apply(const AdamConst& c, const AdamRef& r, uint32_t e,
                                           float g) {
  adam_apply_loaded(c, r, e, g, r.p[e], r.m[e], r.v[e]);
}

struct FinTask {
  int kind;                  // 0: lp_loss value, 1: epilogue backward sums,
                             // 2: loss value from the epilogue rows (fused tail),
                             // 3: the fused Adam step of one final gradient (o[0], a elems)
  uint32_t nwg;              // workgroups the task takes
  const double* part;
  uint32_t a, b, c;          // loss: nblk; epilogue: N, C, nb; rows loss: rows; adam: n
  uint32_t s0;               // epilogue: the row records' gamma / phi slot pair (0, or 7)
  double m;                  // loss: M
  float* o[4];               // loss: o[0]; epilogue: ggamma, gphi, gdelta, gzp; adam: grad
  AdamRef ad[3];             // epilogue: the gamma / phi / delta steps fused in; adam: ad[0]
};
constexpr int kMaxFin = 12;
constexpr int kMaxAdamSegs = 8;      // alpha segments of one prepared alpha-backward launch
struct FinTable {
  FinTask t[kMaxFin];
  int n;
  uint32_t nwg;
  AdamConst ac;
};

// lp_loss value: the workgroup partials summed in index order (every load issued first)
__device__ __forceinline__ void fin_loss(const double* __restrict__ part, int nblk, double m,
                                         float* __restrict__ out) {
  __shared__ double red[16];
  double v[kLossBlocks / kBlock];
#pragma unroll
  for (int k = 0; k < kLossBlocks / kBlock; ++k) {
    const int i = threadIdx.x + k * kBlock;
    v[k] = i < nblk ? part[i] : 0.0;
  }
  double a = 0.0;
#pragma unroll
  for (int k = 0; k < kLossBlocks / kBlock; ++k) a += v[k];
  a = block_sum(a, red);
  if (threadIdx.x == 0) out[0] = (float)(a / m);
}

// epilogue backward: workgroups [0, nb) the per-channel gamma / phi gradients, kEpiChan
// channels per workgroup, the samples n split over its 4 waves (wave w sums n = w, w + 4,
// ... in order, then the 4 wave sums are added in wave order: every load of a channel in
// flight at once); workgroups [nb, nb + nd) (when launched) the act quantizer's delta / zp
// gradients: workgroup nb + j sums the j-th of nd contiguous row ranges in a fixed order,
// and the last to arrive adds the nd partials in range order (deterministic, as
// fq_bwd_finalize; one range below kDeltaRows rows -- a single workgroup walking 16K
// strided row records was 12 us of load latency on ResNet-18 layer4)
constexpr uint32_t kEpiChan = kBlock / 4;
constexpr uint32_t kDeltaRows = 1024;   // rows per delta workgroup (one batch of loads)
constexpr uint32_t kMaxDeltaWg = 16;
__host__ __device__ inline uint32_t delta_wgs(uint32_t rows) {
  const uint32_t d = (rows + kDeltaRows - 1) / kDeltaRows;
  return d < 1 ? 1 : (d > kMaxDeltaWg ? kMaxDeltaWg : d);
}
// the delta partials: after the row records and the fused tail's loss partials
// (ssq_epilogue_bwd_workspace_size)
__host__ __device__ inline size_t delta_part_offset(size_t rows) {
  return rows * kEpiParts + (rows + 3) / 4;
}
// the delta reduction's last-arriver counter: one word after its partials, in the calling
// epilogue backward's own workspace -- so two calls (other streams, other workspaces) never
// share a counter.  The launch that writes the rows' records stores zero there (it runs
// before any finalize of those records, in stream order), the last arriver resets it.
__host__ __device__ inline size_t delta_ticket_offset(size_t rows) {
  return delta_part_offset(rows) + 4 * kMaxDeltaWg;
}
__device__ __forceinline__ void fin_epi(uint32_t bid, const double* __restrict__ part, uint32_t N,
                                        uint32_t C, uint32_t nb, uint32_t nd, uint32_t s0,
                                        float* __restrict__ ggamma,
                                        float* __restrict__ gphi, float* __restrict__ gdelta,
                                        float* __restrict__ gzp, const AdamConst& ac,
                                        const AdamRef* ad) {
  __shared__ double red[16];
  if (bid < nb) {
    __shared__ double wsum[4][kEpiChan][2];
    const uint32_t cl = threadIdx.x % kEpiChan, w = threadIdx.x / kEpiChan;
    const uint32_t c = bid * kEpiChan + cl;
    // the fused Adam steps' state, loaded with the partials (one memory round trip, not two)
    float st[2][3] = {{0.0f, 0.0f, 0.0f}, {0.0f, 0.0f, 0.0f}};
    if (w == 0 && c < C) {
#pragma unroll
      for (int j = 0; j < 2; ++j)
        if (ad[j].p) {
          st[j][0] = ad[j].p[c];
          st[j][1] = ad[j].m[c];
          st[j][2] = ad[j].v[c];
        }
    }
    double sg = 0, sp = 0;
    if (c < C) {
#pragma unroll 8
      for (uint32_t n = w; n < N; n += 4) {
        sg += part[((int64_t)n * C + c) * kEpiParts + s0];
        sp += part[((int64_t)n * C + c) * kEpiParts + s0 + 1];
      }
    }
    wsum[w][cl][0] = sg;
    wsum[w][cl][1] = sp;
    __syncthreads();
    if (w == 0 && c < C) {
      sg = wsum[0][cl][0] + wsum[1][cl][0] + wsum[2][cl][0] + wsum[3][cl][0];
      sp = wsum[0][cl][1] + wsum[1][cl][1] + wsum[2][cl][1] + wsum[3][cl][1];
      if (ggamma) ggamma[c] = (float)sg;
      if (gphi) gphi[c] = (float)sp;
      if (ad[0].p) adam_apply_loaded(ac, ad[0], c, (float)sg, st[0][0], st[0][1], st[0][2]);
      if (ad[1].p) adam_apply_loaded(ac, ad[1], c, (float)sp, st[1][0], st[1][1], st[1][2]);
    }
    return;
  }
  float sd[3] = {0.0f, 0.0f, 0.0f};    // the delta step's state, loaded with the sums
  if (ad[2].p && threadIdx.x == 0) {
    sd[0] = ad[2].p[0];
    sd[1] = ad[2].m[0];
    sd[2] = ad[2].v[0];
  }
  const uint32_t rows = N * C, j = bid - nb;
  const uint32_t per = (rows + nd - 1) / nd, lo = j * per, hi = min(rows, lo + per);
  double a[4] = {0, 0, 0, 0};
  constexpr uint32_t kB = kFinBatch / 4;   // 4 sums per row: keep the registers of the
                                            // host kernels this rides on (occupancy) low
  for (uint32_t r0 = lo + threadIdx.x; r0 < hi; r0 += kB * kBlock) {
    double v[kB][4];
#pragma unroll
    for (uint32_t b = 0; b < kB; ++b) {
      const uint32_t r = r0 + b * kBlock;
#pragma unroll
      for (int k = 0; k < 4; ++k) v[b][k] = r < hi ? part[(int64_t)r * kEpiParts + 2 + k] : 0.0;
    }
#pragma unroll
    for (uint32_t b = 0; b < kB; ++b)
      if (r0 + b * kBlock < hi)
#pragma unroll
        for (int k = 0; k < 4; ++k) a[k] += v[b][k];
  }
  for (int k = 0; k < 4; ++k) a[k] = block_sum(a[k], red);
  if (nd > 1) {
    double* dp = const_cast<double*>(part) + delta_part_offset(rows);
    if (threadIdx.x == 0)
      for (int k = 0; k < 4; ++k) st_sc1(dp + 4 * j + k, a[k]);
    __shared__ int last;
    __shared__ double dps[4 * kMaxDeltaWg];
    unsigned* ticket = (unsigned*)(const_cast<double*>(part) + delta_ticket_offset(rows));
    if (!arrive_last(ticket, nd, &last)) return;
    if (threadIdx.x < 4 * nd) dps[threadIdx.x] = ld_sc1(dp + threadIdx.x);
    __syncthreads();
    if (threadIdx.x == 0)
      for (int k = 0; k < 4; ++k) {
        double t = 0.0;
        for (uint32_t i = 0; i < nd; ++i) t += dps[4 * i + k];
        a[k] = t;
      }
  }
  if (threadIdx.x == 0) {
    const float gd = (float)(a[0] - a[1]);
    if (gdelta) gdelta[0] = gd;
    if (gzp) gzp[0] = (float)(a[2] - a[3]);
    if (ad[2].p) adam_apply_loaded(ac, ad[2], 0, gd, sd[0], sd[1], sd[2]);
  }
}

// fused tail (ssq_epilogue_loss_bwd): the launch's per-workgroup loss partials (contiguous,
// after the rows' records) summed in order, one workgroup: thread t adds partials t, t + 256,
// ... in order, kFinBatch loads in flight at a time, then the fixed block tree
__device__ __forceinline__ void fin_loss_rows(const double* __restrict__ part, uint32_t rows,
                                              double m, float* __restrict__ out) {
  __shared__ double red[16];
  double a = 0.0;
  for (uint32_t r0 = threadIdx.x; r0 < rows; r0 += kFinBatch * kBlock) {
    double v[kFinBatch];
#pragma unroll
    for (uint32_t k = 0; k < kFinBatch; ++k) {
      const uint32_t r = r0 + k * kBlock;
      v[k] = r < rows ? part[r] : 0.0;
    }
#pragma unroll
    for (uint32_t k = 0; k < kFinBatch; ++k)
      if (r0 + k * kBlock < rows) a += v[k];
  }
  a = block_sum(a, red);
  if (threadIdx.x == 0) out[0] = (float)(a / m);
}

// the fused Adam step of one final gradient (small tensors: gamma^z / phi^z), one workgroup
__device__ __forceinline__ void fin_adam(const AdamConst& ac, const AdamRef& r,
                                         const float* __restrict__ g, uint32_t n) {
  for (uint32_t e = threadIdx.x; e < n; e += kBlock) adam_apply(ac, r, e, g[e]);
}

// Workgroup k of the table's tasks (k < ft.nwg).
__device__ __forceinline__ void run_fin(const FinTable& ft, uint32_t k) {
  for (int i = 0; i < ft.n; ++i) {
    const FinTask& t = ft.t[i];
    if (k < t.nwg) {
      if (t.kind == 0)
        fin_loss(t.part, (int)t.a, t.m, t.o[0]);
      else if (t.kind == 1)
        fin_epi(k, t.part, t.a, t.b, t.c, t.nwg - t.c, t.s0, t.o[0], t.o[1], t.o[2], t.o[3],
                ft.ac, t.ad);
      else if (t.kind == 2)
        fin_loss_rows(t.part, t.a, t.m, t.o[0]);
      else
        fin_adam(ft.ac, t.ad[0], t.o[0], t.a);
      return;
    }
    k -= t.nwg;
  }
}

// host side (recon.hip)
// The armed optimizer step (ssq_adam_arm) of stream s, attached to the alpha-backward launch
// about to run (nseg segments of parameters alpha[i], len[i] elements; ft = the finalize
// tasks riding on it): true when every armed parameter's update can run inside that launch
// -- alpha in its finaliser (refs[i]), gamma^z / phi^z in their riding finalize task or as
// extra kind-3 tasks appended to ft (gradients finished by earlier launches) -- and then
// the attachments are made and *ac filled; false (nothing attached) otherwise.
bool adam_attach(hipStream_t s, int nseg, const float* const* alpha, const int64_t* len,
                 AdamRef* refs, FinTable& ft, AdamConst* ac);
bool fin_defer_on();
int fin_push(hipStream_t s, const FinTask& t);   // queue (flushes first when full)
FinTable fin_take(hipStream_t s);                // remove and return the stream's pending tasks
int fin_flush(hipStream_t s);                    // launch the pending tasks standalone

}  // namespace ssq
