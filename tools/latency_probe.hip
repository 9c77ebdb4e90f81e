// Kernel-duration floor on this box: how long does a launch take whose work is a chain of
// 0, 1, 2 or 3 dependent global-memory round trips on data that a large streaming pass has
// just evicted from L2 / MALL (as in the recon loop, where every small kernel follows an
// activation-sized pass)?  Read the durations from rocprofv3 --kernel-trace --stats:
//   hipcc -O3 --offload-arch=gfx950 tools/latency_probe.hip -o /tmp/latency_probe
//   rocprofv3 --kernel-trace --stats -d OUT -- /tmp/latency_probe
#include <hip/hip_runtime.h>

#include <cstdio>

#define CK(x)                                                             \
  do {                                                                    \
    hipError_t e_ = (x);                                                  \
    if (e_ != hipSuccess) {                                               \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                           \
    }                                                                     \
  } while (0)

__global__ void k_empty(float* out) {
  if (threadIdx.x == 1000000) out[0] = 0.0f;
}

// every lane: one load, one store
__global__ void k_chain1(const float* __restrict__ a, float* __restrict__ out) {
  const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
  out[i] = a[i] + 1.0f;
}

// load an index, then load through it (two dependent round trips), store
__global__ void k_chain2(const int* __restrict__ idx, const float* __restrict__ a,
                         float* __restrict__ out) {
  const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
  out[i] = a[idx[i]] + 1.0f;
}

__global__ void k_chain3(const int* __restrict__ idx, const float* __restrict__ a,
                         float* __restrict__ out) {
  const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
  const int j = idx[idx[i]];
  out[i] = a[j] + 1.0f;
}

// 16 independent loads per lane at a 1 KB stride, all in flight, then one store
__global__ void k_wide16(const float* __restrict__ a, float* __restrict__ out) {
  const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
  float v[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) v[r] = a[i + r * 65536u];
  float s = 0.0f;
#pragma unroll
  for (int r = 0; r < 16; ++r) s += v[r];
  out[i] = s;
}

__global__ void k_flush(const float4* __restrict__ a, float4* __restrict__ b, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x)
    b[i] = a[i];
}

typedef float f4 __attribute__((ext_vector_type(4)));
__global__ void k_flush_nt(const float4* __restrict__ a4, float4* __restrict__ b4, size_t n) {
  const f4* a = (const f4*)a4;
  f4* b = (f4*)b4;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x)
    __builtin_nontemporal_store(a[i], &b[i]);
}

__global__ void k_flush_rd(const float4* __restrict__ a, float* __restrict__ out, size_t n) {
  float s = 0.0f;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x)
    s += a[i].x;
  if (s == 12345.0f) out[0] = s;
}

// which part of the previous kernel's work does the next (empty) launch pay for?
// after: a 512 MB copy with plain stores / with non-temporal stores / a 512 MB read-only
// pass / a plain-store copy of 8 MB, 64 MB
static int after_probe(float4* fa, float4* fb, float* out) {
  const size_t n4 = ((size_t)512 << 20) / sizeof(float4);
  for (int r = 0; r < 50; ++r) {
    hipLaunchKernelGGL(k_flush, dim3(2048), dim3(256), 0, 0, fa, fb, n4);
    hipLaunchKernelGGL(k_empty, dim3(1), dim3(256), 0, 0, out);
    hipLaunchKernelGGL(k_flush_nt, dim3(2048), dim3(256), 0, 0, fa, fb, n4);
    hipLaunchKernelGGL(k_empty, dim3(1), dim3(256), 0, 0, out);
    hipLaunchKernelGGL(k_flush_rd, dim3(2048), dim3(256), 0, 0, fa, out, n4);
    hipLaunchKernelGGL(k_empty, dim3(1), dim3(256), 0, 0, out);
    hipLaunchKernelGGL(k_flush, dim3(2048), dim3(256), 0, 0, fa, fb, n4 / 64);
    hipLaunchKernelGGL(k_empty, dim3(1), dim3(256), 0, 0, out);
    hipLaunchKernelGGL(k_flush, dim3(2048), dim3(256), 0, 0, fa, fb, n4 / 8);
    hipLaunchKernelGGL(k_empty, dim3(1), dim3(256), 0, 0, out);
  }
  CK(hipDeviceSynchronize());
  printf("after-probe done\n");
  return 0;
}

int main() {
  const size_t big = (size_t)512 << 20;   // 512 MB each way: well past L2 + MALL
  float4 *fa, *fb;
  float *a, *out;
  int* idx;
  CK(hipMalloc(&fa, big));
  CK(hipMalloc(&fb, big));
  CK(hipMalloc(&a, 64u << 20));
  CK(hipMalloc(&out, 64u << 20));
  CK(hipMalloc(&idx, 64u << 20));
  CK(hipMemset(fa, 0, big));
  CK(hipMemset(a, 0, 64u << 20));
  CK(hipMemset(idx, 0, 64u << 20));
  const size_t n4 = big / sizeof(float4);
  const int reps = 50;
  for (int grid : {1, 16, 256, 1024}) {
    for (int r = 0; r < reps; ++r) {
      hipLaunchKernelGGL(k_flush, dim3(2048), dim3(256), 0, 0, fa, fb, n4);
      hipLaunchKernelGGL(k_empty, dim3(grid), dim3(256), 0, 0, out);
      hipLaunchKernelGGL(k_flush, dim3(2048), dim3(256), 0, 0, fa, fb, n4);
      hipLaunchKernelGGL(k_chain1, dim3(grid), dim3(256), 0, 0, a, out);
      hipLaunchKernelGGL(k_flush, dim3(2048), dim3(256), 0, 0, fa, fb, n4);
      hipLaunchKernelGGL(k_chain2, dim3(grid), dim3(256), 0, 0, idx, a, out);
      hipLaunchKernelGGL(k_flush, dim3(2048), dim3(256), 0, 0, fa, fb, n4);
      hipLaunchKernelGGL(k_chain3, dim3(grid), dim3(256), 0, 0, idx, a, out);
      hipLaunchKernelGGL(k_flush, dim3(2048), dim3(256), 0, 0, fa, fb, n4);
      if (grid <= 256) hipLaunchKernelGGL(k_wide16, dim3(grid), dim3(256), 0, 0, a, out);
    }
    CK(hipDeviceSynchronize());
    // hot: back to back, no flush
    for (int r = 0; r < reps; ++r) {
      hipLaunchKernelGGL(k_chain1, dim3(grid), dim3(256), 0, 0, a, out);
      hipLaunchKernelGGL(k_chain2, dim3(grid), dim3(256), 0, 0, idx, a, out);
    }
    CK(hipDeviceSynchronize());
    printf("grid %d done\n", grid);
  }
  return after_probe(fa, fb, out);
}
