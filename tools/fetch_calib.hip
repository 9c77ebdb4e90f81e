// FETCH_SIZE calibration by access width on gfx950: the guide's x2 correction is measured
// for 16-B-per-lane streaming reads; this reads one 256 MB buffer with 4-, 8- and 16-byte
// coalesced loads per lane (each kernel once, each reading every byte once) so that one
// rocprofv3 --pmc FETCH_SIZE pass gives FETCH_SIZE / bytes per width.
//   hipcc -O3 --offload-arch=gfx950 tools/fetch_calib.hip -o tools/fetch_calib
//   rocprofv3 --pmc FETCH_SIZE --output-format csv -d OUT -o f -- tools/fetch_calib
#include <hip/hip_runtime.h>

#include <cstdio>

template <typename T>
__global__ void read_w(const T* __restrict__ a, float* __restrict__ out, size_t n) {
  float s = 0.0f;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x) {
    const T v = a[i];
    s += *(const float*)&v;
  }
  if (s == 12345.0f) out[0] = s;   // never true for the zero-filled buffer: no store
}

int main() {
  const size_t bytes = (size_t)256 << 20;
  void* a;
  float* out;
  if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
  if (hipMemset(a, 0, bytes) != hipSuccess) return 1;
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(read_w<float>, dim3(4096), dim3(256), 0, 0, (const float*)a, out,
                       bytes / 4);
    hipLaunchKernelGGL(read_w<float2>, dim3(4096), dim3(256), 0, 0, (const float2*)a, out,
                       bytes / 8);
    hipLaunchKernelGGL(read_w<float4>, dim3(4096), dim3(256), 0, 0, (const float4*)a, out,
                       bytes / 16);
  }
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  printf("read %zu bytes per launch\n", bytes);
  return 0;
}
