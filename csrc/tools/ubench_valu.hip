// SPDX-License-Identifier: MIT
// VALU issue-rate micro-benchmark for the instructions the fused kernel's Philox noise uses
// (gfx950).  Each lane runs 8 independent dependency chains of one operation; the kernel time
// over the whole chip gives the per-SIMD issue cost of that operation relative to v_fma_f32.
//
//   hipcc -O3 --offload-arch=gfx950 csrc/tools/ubench_valu.hip -o build/bin/ubench_valu
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHECK(x)                                                             \
  do {                                                                       \
    hipError_t e = (x);                                                      \
    if (e != hipSuccess) {                                                   \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                 \
      return 1;                                                              \
    }                                                                        \
  } while (0)

constexpr int kIters = 4096;
constexpr int kChains = 8;

enum Op { kFma = 0, kPkFma, kMadU64, kMulHi, kMulLo, kMulU24, kBitop3, kCvt };

template <int OP>
__global__ __launch_bounds__(256) void k_ubench(uint32_t* out, uint32_t seed) {
  uint32_t a[kChains];
  float f[kChains];
#pragma unroll
  for (int c = 0; c < kChains; ++c) {
    a[c] = seed + threadIdx.x * 7919u + c * 104729u;
    f[c] = (float)a[c] * 1e-9f;
  }
  const uint32_t M = 0xD2511F53u ^ seed;
  const float fm = 0.999f + (float)seed * 1e-12f;
  // every operation is one inline-asm instruction on its own chain, so the compiler neither
  // vectorises nor fuses them; 8 chains hide the dependency latency
#pragma unroll 4
  for (int i = 0; i < kIters; ++i) {
#pragma unroll
    for (int c = 0; c < kChains; ++c) {
      if constexpr (OP == kFma) {
        asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(f[c]) : "s"(fm));
      } else if constexpr (OP == kPkFma) {
        typedef float f2 __attribute__((ext_vector_type(2)));
        f2 v = {f[c], f[c] + 1.f};
        asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(v) : "v"(v));
        f[c] = v.x;
      } else if constexpr (OP == kMadU64) {
        uint64_t p;
        asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, 0" : "=v"(p) : "v"(a[c]), "s"(M) : "vcc");
        a[c] = (uint32_t)p;
      } else if constexpr (OP == kMulHi) {
        asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a[c]) : "s"(M));
      } else if constexpr (OP == kMulLo) {
        asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[c]) : "s"(M));
      } else if constexpr (OP == kMulU24) {
        asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a[c]) : "s"(M));
      } else if constexpr (OP == kBitop3) {
        asm volatile("v_bitop3_b32 %0, %0, %1, %1 bitop3:0x96" : "+v"(a[c]) : "s"(M));
      } else {
        asm volatile("v_cvt_f32_u32 %0, %0" : "+v"(a[c]));
      }
    }
  }
  uint32_t acc = 0;
#pragma unroll
  for (int c = 0; c < kChains; ++c) acc ^= a[c] ^ __float_as_uint(f[c]);
  if (acc == 0x12345678u) out[0] = acc;
}

template <int OP>
int run(const char* name, uint32_t* d, int nblocks) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  k_ubench<OP><<<nblocks, 256>>>(d, 1);
  CHECK(hipGetLastError());
  CHECK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int r = 0; r < 5; ++r) {
    CHECK(hipEventRecord(e0));
    k_ubench<OP><<<nblocks, 256>>>(d, 1);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best) best = ms;
  }
  const double ops = (double)nblocks * 256 / 64 * kIters * kChains;  // wave-instructions
  int cus = 256;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  // cycles per wave-instruction per SIMD at the nominal 2.4 GHz
  const double cyc = best * 1e-3 * 2.4e9 * cus * 4 / ops;
  printf("%-14s %9.3f ms  %6.2f SIMD-cycles per wave64 instruction (incl. loop overhead)\n", name,
         best, cyc);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return 0;
}

int main() {
  uint32_t* d = nullptr;
  CHECK(hipMalloc(&d, 64));
  int cus = 256;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const int nb = cus * 8;  // 8 workgroups of 4 waves per CU = 8 waves per SIMD
  int rc = 0;
  rc |= run<kFma>("v_fma_f32", d, nb);
  rc |= run<kPkFma>("v_pk_fma_f32", d, nb);
  rc |= run<kMadU64>("v_mad_u64_u32", d, nb);
  rc |= run<kMulHi>("v_mul_hi_u32", d, nb);
  rc |= run<kMulLo>("v_mul_lo_u32", d, nb);
  rc |= run<kMulU24>("v_mul_u32_u24", d, nb);
  rc |= run<kBitop3>("v_bitop3_b32", d, nb);
  rc |= run<kCvt>("v_cvt_f32_u32", d, nb);
  (void)hipFree(d);
  return rc;
}
