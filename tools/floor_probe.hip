// The ~5 us "launch floor" of a small kernel that follows a large one: how much
// of it is the predecessor's dirty data (an L2 write-back the next launch waits for) and how
// much a fixed cost per dependent boundary?  MI355X_MICROARCH.md prices a dependent boundary
// at 1.45-1.9 us plus dirty bytes / ~6 TB/s.
//
// Per round: a producer writes D MB (D = 0, 4, 16, 64) with one store policy -- plain,
// non-temporal (nt) or write-through (sc1: agent-scope relaxed atomic stores, vector
// global_store ... sc1) -- over a freshly read source, then an EMPTY kernel (1 workgroup)
// follows on the same stream.  The durations come from rocprofv3 --kernel-trace (empty
// kernel's begin-end) and, independently, from HIP events around the (producer, empty) pair
// vs the producer alone, which catches a cost that lands between the kernels instead of
// inside the second one's timestamps.  Also: two empty kernels back to back (no producer),
// and a graph-captured (producer, empty) pair.
//   hipcc -O3 --offload-arch=gfx950 tools/floor_probe.hip -o tools/floor_probe
//   rocprofv3 --kernel-trace --stats -d OUT -- tools/floor_probe     (or run alone: events)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));  \
      return 1;                                                                  \
    }                                                                            \
  } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) unsigned long long gu64;

__global__ void k_empty(float* out) {
  if (threadIdx.x == 1000000) out[0] = 0.0f;
}

// write n float4 with the chosen policy (0 plain, 1 nt, 2 sc1 write-through); the values
// come from a source pass so the stores are real data, not a memset
template <int POL>
__global__ __launch_bounds__(256) void k_write(const f4* __restrict__ a, f4* __restrict__ b,
                                               size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x) {
    const f4 v = a[i];
    if (POL == 0) {
      b[i] = v;
    } else if (POL == 1) {
      __builtin_nontemporal_store(v, &b[i]);
    } else {
      gu64* p = (gu64*)&b[i];
      unsigned long long lo, hi;
      __builtin_memcpy(&lo, &v, 8);
      __builtin_memcpy(&hi, ((const char*)&v) + 8, 8);
      __hip_atomic_store(p, lo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(p + 1, hi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// evict: read 512 MB (no writes) so every round starts with clean caches
__global__ __launch_bounds__(256) void k_evict(const f4* __restrict__ a, float* out, size_t n) {
  float s = 0.0f;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x)
    s += a[i].x;
  if (s == 12345.0f) out[0] = s;
}

typedef void (*WK)(const f4*, f4*, size_t);

static float med(std::vector<float> v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

int main() {
  const size_t big = (size_t)512 << 20;
  f4 *ev, *src, *dst;
  float* out;
  CK(hipMalloc(&ev, big));
  CK(hipMalloc(&src, (size_t)64 << 20));
  CK(hipMalloc(&dst, (size_t)64 << 20));
  CK(hipMalloc(&out, 4096));
  CK(hipMemset(ev, 0, big));
  CK(hipMemset(src, 0, (size_t)64 << 20));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipEvent_t e0, e1, e2;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventCreate(&e2));
  const WK ks[3] = {k_write<0>, k_write<1>, k_write<2>};
  const char* pol[3] = {"plain", "nt", "sc1"};
  const int mbs[4] = {0, 4, 16, 64};
  const int reps = 30;
  printf("{\"probe\": \"floor_probe\", \"reps\": %d, \"rows\": [\n", reps);
  bool first = true;
  for (int p = 0; p < 3; ++p) {
    for (int mb : mbs) {
      const size_t n = ((size_t)mb << 20) / sizeof(f4);
      const unsigned grid = mb == 0 ? 1u : 1024u;
      std::vector<float> pair, alone;
      for (int r = 0; r < reps; ++r) {
        // producer alone, then producer + empty, each after an eviction pass
        hipLaunchKernelGGL(k_evict, dim3(2048), dim3(256), 0, s, ev, out, big / sizeof(f4));
        CK(hipEventRecord(e0, s));
        hipLaunchKernelGGL(ks[p], dim3(grid), dim3(256), 0, s, src, dst, n);
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        alone.push_back(ms * 1e3f);
        hipLaunchKernelGGL(k_evict, dim3(2048), dim3(256), 0, s, ev, out, big / sizeof(f4));
        CK(hipEventRecord(e0, s));
        hipLaunchKernelGGL(ks[p], dim3(grid), dim3(256), 0, s, src, dst, n);
        hipLaunchKernelGGL(k_empty, dim3(1), dim3(256), 0, s, out);
        CK(hipEventRecord(e2, s));
        CK(hipEventSynchronize(e2));
        CK(hipEventElapsedTime(&ms, e0, e2));
        pair.push_back(ms * 1e3f);
      }
      printf("%s  {\"policy\": \"%s\", \"dirty_mb\": %d, \"producer_us\": %.2f, "
             "\"producer_plus_empty_us\": %.2f, \"empty_adds_us\": %.2f}",
             first ? "" : ",\n", pol[p], mb, med(alone), med(pair), med(pair) - med(alone));
      first = false;
    }
  }
  // empty after empty (no producer), and the pair from a captured graph
  {
    std::vector<float> two;
    for (int r = 0; r < reps; ++r) {
      hipLaunchKernelGGL(k_evict, dim3(2048), dim3(256), 0, s, ev, out, big / sizeof(f4));
      CK(hipEventRecord(e0, s));
      hipLaunchKernelGGL(k_empty, dim3(1), dim3(256), 0, s, out);
      hipLaunchKernelGGL(k_empty, dim3(1), dim3(256), 0, s, out);
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      two.push_back(ms * 1e3f);
    }
    printf(",\n  {\"policy\": \"none\", \"what\": \"empty+empty\", \"us\": %.2f}", med(two));
  }
  for (int p = 0; p < 3; ++p) {
    const size_t n = ((size_t)16 << 20) / sizeof(f4);
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    hipLaunchKernelGGL(ks[p], dim3(1024), dim3(256), 0, s, src, dst, n);
    hipLaunchKernelGGL(k_empty, dim3(1), dim3(256), 0, s, out);
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    hipGraph_t g1;
    hipGraphExec_t ge1;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    hipLaunchKernelGGL(ks[p], dim3(1024), dim3(256), 0, s, src, dst, n);
    CK(hipStreamEndCapture(s, &g1));
    CK(hipGraphInstantiate(&ge1, g1, nullptr, nullptr, 0));
    std::vector<float> pair, alone;
    for (int r = 0; r < reps; ++r) {
      float ms;
      hipLaunchKernelGGL(k_evict, dim3(2048), dim3(256), 0, s, ev, out, big / sizeof(f4));
      CK(hipEventRecord(e0, s));
      CK(hipGraphLaunch(ge1, s));
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms, e0, e1));
      alone.push_back(ms * 1e3f);
      hipLaunchKernelGGL(k_evict, dim3(2048), dim3(256), 0, s, ev, out, big / sizeof(f4));
      CK(hipEventRecord(e0, s));
      CK(hipGraphLaunch(ge, s));
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms, e0, e1));
      pair.push_back(ms * 1e3f);
    }
    printf(",\n  {\"policy\": \"%s\", \"dirty_mb\": 16, \"graph\": true, \"producer_us\": %.2f, "
           "\"producer_plus_empty_us\": %.2f, \"empty_adds_us\": %.2f}",
           pol[p], med(alone), med(pair), med(pair) - med(alone));
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
    CK(hipGraphExecDestroy(ge1));
    CK(hipGraphDestroy(g1));
  }
  printf("\n]}\n");
  CK(hipStreamSynchronize(s));
  return 0;
}
