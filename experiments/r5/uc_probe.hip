// Per-CU copy throughput from / to uncached (hipDeviceMallocUncached) vs ordinary device memory,
// with W workgroups of 768 threads (one per CU): the in-kernel exchange of a gated pass
// (csrc/hip/gate.hpp) copies with a fraction of the CUs while the others march.
//   hipcc --offload-arch=gfx950 -O3 -o uc_probe experiments/r5/uc_probe.hip && ./uc_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

// mode 0: 8-byte lanes (float2), 1: 16-byte lanes (float4), 2: 8-byte lanes with system-coherent
// (sc0 sc1) loads; B cells in flight per thread
template <int MODE, int B>
__global__ __launch_bounds__(768) void k_copy(const float2* __restrict__ src, float2* __restrict__ dst,
                                              size_t n) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if constexpr (MODE == 1) {
    const float4* s4 = (const float4*)src;
    float4* d4 = (float4*)dst;
    const size_t n4 = n / 2;
    for (size_t i0 = t; i0 < n4; i0 += B * stride) {
      float4 c[B];
#pragma unroll
      for (int j = 0; j < B; ++j)
        if (i0 + j * stride < n4) c[j] = s4[i0 + j * stride];
#pragma unroll
      for (int j = 0; j < B; ++j)
        if (i0 + j * stride < n4) d4[i0 + j * stride] = c[j];
    }
  } else {
    for (size_t i0 = t; i0 < n; i0 += B * stride) {
      float2 c[B];
#pragma unroll
      for (int j = 0; j < B; ++j)
        if (i0 + j * stride < n) {
          if constexpr (MODE == 2) {
            const unsigned long long w = __hip_atomic_load((const unsigned long long*)(src + i0 + j * stride),
                                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            c[j] = *(const float2*)&w;
          } else {
            c[j] = src[i0 + j * stride];
          }
        }
#pragma unroll
      for (int j = 0; j < B; ++j)
        if (i0 + j * stride < n) dst[i0 + j * stride] = c[j];
    }
  }
}

template <int MODE, int B>
static float run(const float2* s, float2* d, size_t n, int wgs) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  k_copy<MODE, B><<<wgs, 768>>>(s, d, n);
  (void)hipEventRecord(e0);
  for (int r = 0; r < 10; ++r) k_copy<MODE, B><<<wgs, 768>>>(s, d, n);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  return ms / 10;
}

int main() {
  const size_t n = (size_t)1 << 19;  // 512 Ki cells = 4 MiB (a z-slab exchange's order)
  float2 *uc0, *uc1, *cc0, *cc1;
  CK(hipExtMallocWithFlags((void**)&uc0, n * 8, hipDeviceMallocUncached));
  CK(hipExtMallocWithFlags((void**)&uc1, n * 8, hipDeviceMallocUncached));
  CK(hipMalloc((void**)&cc0, n * 8));
  CK(hipMalloc((void**)&cc1, n * 8));
  CK(hipMemset(uc0, 0, n * 8));
  CK(hipMemset(cc0, 0, n * 8));
  printf("{\"bytes\": %zu}\n", n * 8);
  for (int wgs : {32, 64, 128, 256}) {
    struct R { const char* name; float ms; };
    std::vector<R> rs = {
        {"cached->cached 8B", run<0, 16>(cc0, cc1, n, wgs)},
        {"cached->UC 8B", run<0, 16>(cc0, uc1, n, wgs)},
        {"UC->cached 8B", run<0, 16>(uc0, cc1, n, wgs)},
        {"cached->UC 16B", run<1, 8>(cc0, uc1, n, wgs)},
        {"UC->cached 16B", run<1, 8>(uc0, cc1, n, wgs)},
        {"UC->cached 8B B4", run<0, 4>(uc0, cc1, n, wgs)},
        {"sys-load cached->cached 8B", run<2, 16>(cc0, cc1, n, wgs)},
    };
    for (auto& r : rs)
      printf("{\"wgs\": %d, \"copy\": \"%s\", \"us\": %.2f, \"GBps\": %.1f, \"GBps_per_wg\": %.2f}\n",
             wgs, r.name, r.ms * 1e3, n * 8 / (r.ms * 1e6), n * 8 / (r.ms * 1e6) / wgs);
  }
  return 0;
}
