// The fused loop's iteration start in one launch: the batch gather (K14, recon.hip) and the
// prepared adaShift forward of every conv of the block (K5p, adashift_prep.hip).  Both only
// read state fixed for the iteration (the staged indices; alpha), so with the prepared
// forward deferred (ssq_set_deferred_prep_fwd) it queues its table on its stream and the
// next ssq_gather_rows2 on that stream runs it in extra workgroups of the gather launch:
// one launch less per iteration, same code, bit-identical results.
#pragma once

#include <type_traits>

#include "ssq_common.h"

namespace ssq {

struct GatherArgs {
  const float* s0;
  float* d0;
  int64_t row0;
  const float* s1;
  float* d1;
  int64_t row1;
  const int64_t* idx;
  uint32_t gx;      // workgroups per batch row
  uint32_t nrows;   // batch rows
  // staged form (ssq_gather_rows2_staged): idx is one slot of a device ring of iterations'
  // words; its first stage_n words are also copied to stage_dst (the loop's static slot,
  // read by the iteration's later launches), by the workgroup of (bx, r) = (0, 0)
  int64_t* stage_dst;
  uint32_t stage_n;
};

// dst[k] = src[k] for k = k0, k0 + stride, ... < n: kGatherU loads in flight per lane
// before their stores (src and dst never overlap)
constexpr int kGatherU = 4;
template <typename T>
__device__ __forceinline__ void copy_strided(const T* __restrict__ src, T* __restrict__ dst,
                                             int64_t k0, int64_t n, int64_t stride) {
  for (int64_t k = k0; k < n; k += kGatherU * stride) {
    T v[kGatherU];
#pragma unroll
    for (int u = 0; u < kGatherU; ++u)
      if (k + u * stride < n) v[u] = src[k + u * stride];
#pragma unroll
    for (int u = 0; u < kGatherU; ++u)
      if (k + u * stride < n) dst[k + u * stride] = v[u];
  }
}

// dst_k[r, :] = src_k[idx[r], :] for batch row r, workgroup bx of the row's gx; 16-B
// vectors when rows allow it.  Its source row index is one scalar load; the workgroups of
// a row stride over the concatenated row of both sources: no per-element division.
template <bool VEC>
__device__ __forceinline__ void gather2_body(const GatherArgs& a, uint32_t bx, uint32_t r) {
  typedef typename std::conditional<VEC, f32x4, float>::type T;
  const int64_t w = VEC ? 4 : 1;
  const int64_t r0 = a.row0 / w, r1 = a.s1 ? a.row1 / w : 0;
  if (a.stage_dst && bx == 0 && r == 0)
    for (uint32_t k = threadIdx.x; k < a.stage_n; k += blockDim.x) a.stage_dst[k] = a.idx[k];
  const int64_t src = a.idx[r];
  const T* a0 = (const T*)a.s0 + src * r0;
  T* b0 = (T*)a.d0 + (int64_t)r * r0;
  const int64_t stride = (int64_t)a.gx * blockDim.x;
  const int64_t k0 = (int64_t)bx * blockDim.x + threadIdx.x;
  copy_strided(a0, b0, k0, r0, stride);
  if (a.s1) {
    const T* a1 = (const T*)a.s1 + src * r1;
    T* b1 = (T*)a.d1 + (int64_t)r * r1;
    copy_strided(a1, b1, k0, r1, stride);
  }
}

// Launch the gather; when a prepared forward is queued on stream s, in the same launch.
int launch_gather(hipStream_t s, const GatherArgs& a, bool vec);

}  // namespace ssq
