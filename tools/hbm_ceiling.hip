// HBM ceiling probe for the K1 streaming kernel (standalone, no torch):
// read-only, write-only and copy rates over an 822 MB fp32 tensor (the K1 workload size)
// for register loads (plain / nt), LDS-DMA loads (global_load_lds_dwordx4, plain / nt) and
// plain / nt stores, at 1-4 workgroups per CU.  Answers: what does the HBM give a pure
// read, a pure write and a read+write stream on this box, i.e. where K1's 8 B/elem sits.
//   hipcc -O3 --offload-arch=gfx950 tools/hbm_ceiling.hip -o /tmp/hbm_ceiling && /tmp/hbm_ceiling
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e = (x);                                                       \
    if (e != hipSuccess) {                                                    \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);         \
      return 1;                                                               \
    }                                                                         \
  } while (0)

template <bool NT>
__device__ __forceinline__ f32x4 ld(const f32x4* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}
template <bool NT>
__device__ __forceinline__ void st(f32x4 v, f32x4* p) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

// grid-stride, U float4 loads per thread in flight
template <int U, bool NT>
__global__ __launch_bounds__(256) void rd_reg(const f32x4* __restrict__ s, float* __restrict__ sink,
                                              long n4) {
  const long stride = (long)gridDim.x * blockDim.x;
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  f32x4 acc = {0, 0, 0, 0};
  for (; i + (U - 1) * stride < n4; i += U * stride) {
    f32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = ld<NT>(&s[i + u * stride]);
#pragma unroll
    for (int u = 0; u < U; ++u) acc += v[u];
  }
  if (acc.x + acc.y + acc.z + acc.w == 12345.678f) sink[0] = 1.0f;
}

// LDS-DMA: each wave streams 1 KiB pieces into its own LDS ring (U slots), no consumer
template <int U, int AUX>
__global__ __launch_bounds__(256) void rd_glds(const f32x4* __restrict__ s, float* __restrict__ sink,
                                               long n4) {
  __shared__ f32x4 ring[4][U][64];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const long stride = (long)gridDim.x * blockDim.x;
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + (U - 1) * stride < n4; i += U * stride) {
#pragma unroll
    for (int u = 0; u < U; ++u)
      __builtin_amdgcn_global_load_lds((const void*)&s[i + u * stride], (void*)&ring[wave][u][0],
                                       16, 0, AUX);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (ring[wave][0][lane].x == 12345.678f) sink[0] = 1.0f;
}

template <int U, bool NT>
__global__ __launch_bounds__(256) void wr(f32x4* __restrict__ d, long n4) {
  const long stride = (long)gridDim.x * blockDim.x;
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const f32x4 v = {1.0f, 2.0f, 3.0f, (float)threadIdx.x};
  for (; i + (U - 1) * stride < n4; i += U * stride) {
#pragma unroll
    for (int u = 0; u < U; ++u) st<NT>(v, &d[i + u * stride]);
  }
}

// stores with an explicit cache-policy suffix (gfx950 sc0 / sc1 / nt bits)
#define ST_ASM(NAME, POL)                                                                  \
  __device__ __forceinline__ void NAME(f32x4 v, f32x4* p) {                                \
    asm volatile("global_store_dwordx4 %0, %1, off " POL ::"v"(p), "v"(v) : "memory");     \
  }
ST_ASM(st_sc0, "sc0")
ST_ASM(st_sc1, "sc1")
ST_ASM(st_sc01, "sc0 sc1")
ST_ASM(st_sc01nt, "sc0 sc1 nt")
ST_ASM(st_sc1nt, "sc1 nt")
ST_ASM(st_sc0nt, "sc0 nt")

template <int U, int POL, int BS>
__global__ __launch_bounds__(1024) void wr_pol(f32x4* __restrict__ d, long n4) {
  const long stride = (long)gridDim.x * BS;
  long i = (long)blockIdx.x * BS + threadIdx.x;
  const f32x4 v = {1.0f, 2.0f, 3.0f, (float)threadIdx.x};
  for (; i + (U - 1) * stride < n4; i += U * stride) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      f32x4* q = &d[i + u * stride];
      if constexpr (POL == 0) *q = v;
      else if constexpr (POL == 1) __builtin_nontemporal_store(v, q);
      else if constexpr (POL == 2) st_sc0(v, q);
      else if constexpr (POL == 3) st_sc1(v, q);
      else if constexpr (POL == 4) st_sc01(v, q);
      else if constexpr (POL == 5) st_sc01nt(v, q);
      else if constexpr (POL == 6) st_sc1nt(v, q);
      else st_sc0nt(v, q);
    }
  }
}

template <int U, int POL, int BS>
__global__ __launch_bounds__(1024) void cp_pol(const f32x4* __restrict__ s, f32x4* __restrict__ d,
                                               long n4) {
  const long stride = (long)gridDim.x * BS;
  long i = (long)blockIdx.x * BS + threadIdx.x;
  for (; i + (U - 1) * stride < n4; i += U * stride) {
    f32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(&s[i + u * stride]);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int u = 0; u < U; ++u) {
      f32x4* q = &d[i + u * stride];
      if constexpr (POL == 0) *q = v[u];
      else if constexpr (POL == 1) __builtin_nontemporal_store(v[u], q);
      else if constexpr (POL == 2) st_sc0(v[u], q);
      else if constexpr (POL == 3) st_sc1(v[u], q);
      else if constexpr (POL == 4) st_sc01(v[u], q);
      else if constexpr (POL == 5) st_sc01nt(v[u], q);
      else if constexpr (POL == 6) st_sc1nt(v[u], q);
      else st_sc0nt(v[u], q);
    }
  }
}

template <int U, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void cp(const f32x4* __restrict__ s, f32x4* __restrict__ d,
                                          long n4) {
  const long stride = (long)gridDim.x * blockDim.x;
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + (U - 1) * stride < n4; i += U * stride) {
    f32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = ld<NTL>(&s[i + u * stride]);
#pragma unroll
    for (int u = 0; u < U; ++u) st<NTS>(v[u], &d[i + u * stride]);
  }
}

// workgroup-contiguous chunks: WG b owns [b*chunk, (b+1)*chunk)
template <int U, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void cp_chunk(const f32x4* __restrict__ s, f32x4* __restrict__ d,
                                                long n4, long chunk) {
  long i = (long)blockIdx.x * chunk + threadIdx.x;
  const long end = std::min((long)(blockIdx.x + 1) * chunk, n4);
  for (; i + (U - 1) * 256 < end; i += U * 256) {
    f32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = ld<NTL>(&s[i + u * 256]);
#pragma unroll
    for (int u = 0; u < U; ++u) st<NTS>(v[u], &d[i + u * 256]);
  }
}

// LDS-DMA read (nt) + ds_read + store: the staging form of a copy
template <int U, int AUX, bool NTS>
__global__ __launch_bounds__(256) void cp_glds(const f32x4* __restrict__ s, f32x4* __restrict__ d,
                                               long n4) {
  __shared__ f32x4 ring[4][U][64];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const long stride = (long)gridDim.x * blockDim.x;
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + (U - 1) * stride < n4; i += U * stride) {
#pragma unroll
    for (int u = 0; u < U; ++u)
      __builtin_amdgcn_global_load_lds((const void*)&s[i + u * stride], (void*)&ring[wave][u][0],
                                       16, 0, AUX);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int u = 0; u < U; ++u) st<NTS>(ring[wave][u][lane], &d[i + u * stride]);
  }
}

struct Res {
  const char* name;
  int wgs;
  double gbs;
};

int main() {
  const long n = 1024L * 64 * 56 * 56;  // 205,520,896 floats = 822 MB (K1 workload)
  const long n4 = n / 4;
  const int NBUF = 3;                   // rotate buffers so nothing is L2/MALL-warm
  f32x4 *src[NBUF], *dst[NBUF];
  for (int b = 0; b < NBUF; ++b) {
    CK(hipMalloc(&src[b], n * 4));
    CK(hipMalloc(&dst[b], n * 4));
    CK(hipMemset(src[b], 0, n * 4));
    CK(hipMemset(dst[b], 0, n * 4));
  }
  float* sink;
  CK(hipMalloc(&sink, 4));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<Res> out;
  auto timeit = [&](const char* name, int wgs, double bytes_per_elem, auto launch) {
    for (int w = 0; w < 3; ++w) launch(w % NBUF);
    std::vector<float> ms;
    for (int r = 0; r < 5; ++r) {
      hipEventRecord(e0);
      for (int k = 0; k < 12; ++k) launch(k % NBUF);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float t;
      hipEventElapsedTime(&t, e0, e1);
      ms.push_back(t / 12);
    }
    std::sort(ms.begin(), ms.end());
    const double gbs = bytes_per_elem * n / (ms[2] * 1e-3) / 1e9;
    out.push_back({name, wgs, gbs});
    printf("%-28s wgs=%5d  %7.1f GB/s  (%.1f%% of 8 TB/s)  %.1f us\n", name, wgs, gbs,
           gbs / 80.0, ms[2] * 1e3);
    fflush(stdout);
  };
  const char* pol_names[8] = {"plain", "nt", "sc0", "sc1", "sc0 sc1", "sc0 sc1 nt", "sc1 nt", "sc0 nt"};
  char nm[64];
#define WR_POL(P)                                                                        \
  for (int wgs : {128, 256}) {                                                           \
    snprintf(nm, sizeof nm, "write %s u8", pol_names[P]);                                \
    timeit(nm, wgs, 4, [&](int b) { wr_pol<8, P, 256><<<wgs, 256>>>(dst[b], n4); });     \
    snprintf(nm, sizeof nm, "copy ntl/%s u8", pol_names[P]);                             \
    timeit(nm, wgs, 8, [&](int b) { cp_pol<8, P, 256><<<wgs, 256>>>(src[b], dst[b], n4); }); \
  }
  WR_POL(0) WR_POL(1) WR_POL(2) WR_POL(3) WR_POL(4) WR_POL(5) WR_POL(6) WR_POL(7)
  for (int wgs : {64, 128, 192, 256}) {
    timeit("read reg nt u8", wgs, 4, [&](int b) { rd_reg<8, true><<<wgs, 256>>>(src[b], sink, n4); });
    timeit("write nt u8 b256", wgs, 4, [&](int b) { wr_pol<8, 1, 256><<<wgs, 256>>>(dst[b], n4); });
    timeit("write nt u16 b256", wgs, 4, [&](int b) { wr_pol<16, 1, 256><<<wgs, 256>>>(dst[b], n4); });
    timeit("write nt u4 b512", wgs, 4, [&](int b) { wr_pol<4, 1, 512><<<wgs, 512>>>(dst[b], n4); });
    timeit("write nt u8 b512", wgs, 4, [&](int b) { wr_pol<8, 1, 512><<<wgs, 512>>>(dst[b], n4); });
    timeit("write nt u4 b1024", wgs, 4, [&](int b) { wr_pol<4, 1, 1024><<<wgs, 1024>>>(dst[b], n4); });
    timeit("copy reg nt/nt u4", wgs, 8, [&](int b) { cp<4, true, true><<<wgs, 256>>>(src[b], dst[b], n4); });
    timeit("copy reg nt/nt u8", wgs, 8, [&](int b) { cp<8, true, true><<<wgs, 256>>>(src[b], dst[b], n4); });
    timeit("copy nt/nt u4 b512", wgs, 8, [&](int b) { cp_pol<4, 1, 512><<<wgs, 512>>>(src[b], dst[b], n4); });
    timeit("copy nt/nt u8 b512", wgs, 8, [&](int b) { cp_pol<8, 1, 512><<<wgs, 512>>>(src[b], dst[b], n4); });
  }
  CK(hipDeviceSynchronize());
  std::sort(out.begin(), out.end(), [](const Res& a, const Res& b) { return a.gbs > b.gbs; });
  printf("best: %s wgs=%d %.1f GB/s\n", out[0].name, out[0].wgs, out[0].gbs);
  return 0;
}
