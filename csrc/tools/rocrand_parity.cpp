// Prints rocRAND Philox4x32-10 outputs for (seed, subsequence, offset) triples read from stdin,
// using rocRAND's own engine (rocrand_philox4x32_10.h) on the host.  tests/test_noise.py
// compares them with the framework's counter-mode evaluation (csrc/include/gs/common.h).
#include <rocrand/rocrand_philox4x32_10.h>

#include <cstdio>

int main() {
  unsigned long long seed, sub, off;
  while (std::scanf("%llu %llu %llu", &seed, &sub, &off) == 3) {
    rocrand_device::philox4x32_10_engine e(seed, sub, off);
    std::printf("%u\n", e.next());
  }
  return 0;
}
