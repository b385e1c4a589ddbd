// Host write-path probe for the BP4 output step (the reference's L=64 example writes two 1 MB
// fields per output step and is bound by that write): time per step of the two payloads written
// by one thread in sequence (the writer's current path) against 2 and 4 threads writing disjoint
// ranges with pwrite, into a fresh file in the current directory.
//   g++ -O2 -pthread -o write_probe csrc/tools/write_probe.cpp && ./write_probe [MB per field]
#include <fcntl.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

static double now_us() {
  return std::chrono::duration<double, std::micro>(
             std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  const size_t field = (size_t)(argc > 1 ? atof(argv[1]) : 1.0) * (1 << 20);
  const int steps = 100;
  std::vector<char> a(field, 1), b(field, 2);
  for (int threads : {1, 2, 4, 1, 2, 4}) {
    const char* path = "write_probe.bin";
    const int fd = open(path, O_WRONLY | O_CREAT | O_TRUNC, 0644);
    if (fd < 0) { perror("open"); return 1; }
    std::vector<double> t(steps);
    for (int s = 0; s < steps; ++s) {
      const off_t base = (off_t)s * 2 * field;
      const double t0 = now_us();
      if (threads == 1) {
        if (pwrite(fd, a.data(), field, base) != (ssize_t)field ||
            pwrite(fd, b.data(), field, base + field) != (ssize_t)field) { perror("pwrite"); return 1; }
      } else {
        std::vector<std::thread> th;
        const size_t part = 2 * field / threads;
        for (int k = 0; k < threads; ++k)
          th.emplace_back([&, k] {
            const size_t off = k * part;
            const char* src = off < field ? a.data() + off : b.data() + (off - field);
            if (pwrite(fd, src, part, base + off) != (ssize_t)part) perror("pwrite");
          });
        for (auto& x : th) x.join();
      }
      t[s] = now_us() - t0;
    }
    close(fd);
    unlink(path);
    std::sort(t.begin(), t.end());
    printf("threads %d: median %.1f us per step of 2 x %.2f MB (%.2f GB/s), p10 %.1f p90 %.1f\n", threads,
           t[steps / 2], field / 1048576.0, 2.0 * field / t[steps / 2] / 1e3, t[steps / 10], t[9 * steps / 10]);
  }
  return 0;
}
