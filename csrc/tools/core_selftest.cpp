// SPDX-License-Identifier: MIT
// Native self-test of the runtime (scheduler, halo plans, CPU backend, BP4 writer), built for
// the host sanitizers:  make asan && build/asan/core_selftest
//                                         make tsan && build/tsan/core_selftest
//
// N ranks are emulated by N threads of ONE process, each owning an Engine over the CPU
// backend.  The transport callback is an in-process exchange: every rank publishes its packed
// send buffer, a barrier, each rank copies the messages addressed to it straight out of its
// peers' send buffers (matched by direction: my receive d <-> the peer's send 26-d), a second
// barrier.  The decomposed run must equal a one-rank run bit for bit -- the same invariant the
// gloo multi-process tests check, here under ASan/UBSan/TSan.  It also writes and closes a
// small BP4 file from every rank.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "gs/capi.h"

extern "C" {
void* bp4_open(const char* path, const char* io_name, int32_t rank, int32_t nranks,
               int32_t column_major);
int bp4_define_attribute(void* h, const char* name, int32_t type, const void* data, int64_t n);
int bp4_define_variable(void* h, const char* name, int32_t type, int32_t ndims,
                        const uint64_t* shape, const uint64_t* start, const uint64_t* count);
int bp4_begin_step(void* h);
int bp4_put(void* h, int32_t var, const void* data);
int bp4_end_step(void* h);
int64_t bp4_step_metadata(void* h, char** out);
int bp4_write_metadata(void* h, int32_t nblobs, const char* const* blobs, const int64_t* sizes);
int bp4_close(void* h);
const char* bp4_last_error(void);
int64_t bp4_async_submit(void* h, int (*wait_fn)(void*), void* wait_arg, int32_t var_step,
                         int32_t step, int32_t var_u, const void* u, int32_t var_v, const void* v,
                         const void* part, int32_t nmm);
int bp4_async_result(void* h, int64_t ticket, const char** out, int64_t* n);
}

namespace {

class Barrier {
 public:
  explicit Barrier(int n) : n_(n) {}
  void wait() {
    std::unique_lock<std::mutex> lk(m_);
    const long gen = gen_;
    if (++count_ == n_) {
      count_ = 0;
      ++gen_;
      cv_.notify_all();
    } else {
      cv_.wait(lk, [&] { return gen_ != gen; });
    }
  }

 private:
  std::mutex m_;
  std::condition_variable cv_;
  int n_, count_ = 0;
  long gen_ = 0;
};

struct Case {
  int L, dims[3], fuse, steps, periodic;
};

struct Rank;

struct World {
  int n;
  Barrier bar;
  std::vector<Rank*> ranks;
  explicit World(int n_) : n(n_), bar(n_), ranks(n_, nullptr) {}
};

struct Msg {
  int dir, peer;
  int64_t offset, cells;
};

struct Rank {
  World* w;
  int rank;
  int nx, ny, nz, ox, oy, oz;
  gs::Geom g;
  std::vector<double> b0, b1, send, recv;
  gs_engine* e = nullptr;
  std::vector<Msg> smsg, rmsg;
};

int split(int L, int parts, int c, int* off) {
  const int base = L / parts, rem = L % parts;
  *off = c * base + (c < rem ? c : rem);
  return base + (c < rem ? 1 : 0);
}

int rank_of(int cx, int cy, int cz, const int* d, bool periodic) {
  int c[3] = {cx, cy, cz};
  for (int a = 0; a < 3; ++a) {
    if (periodic) c[a] = ((c[a] % d[a]) + d[a]) % d[a];
    else if (c[a] < 0 || c[a] >= d[a]) return -1;
  }
  return (c[0] * d[1] + c[1]) * d[2] + c[2];
}

// transport callback: in-process exchange between the thread-ranks
int exchange_cb(void* user) {
  Rank* r = (Rank*)user;
  World* w = r->w;
  w->bar.wait();  // every rank has packed its send buffer
  for (const Msg& m : r->rmsg) {
    if (m.peer == r->rank) continue;  // self copies are done by the engine
    const Rank* p = w->ranks[m.peer];
    bool found = false;
    for (const Msg& s : p->smsg)
      if (s.peer == r->rank && s.dir == 26 - m.dir) {
        if (s.cells != m.cells) {
          fprintf(stderr, "message size mismatch %lld vs %lld\n", (long long)s.cells,
                  (long long)m.cells);
          return 1;
        }
        memcpy(&r->recv[2 * m.offset], &p->send[2 * s.offset], sizeof(double) * 2 * m.cells);
        found = true;
      }
    if (!found) {
      fprintf(stderr, "rank %d: no matching send for dir %d from %d\n", r->rank, m.dir, m.peer);
      return 1;
    }
  }
  w->bar.wait();  // nobody repacks while others still read
  return 0;
}

bool check(int rc, const char* what) {
  if (rc != 0) fprintf(stderr, "%s failed: %s\n", what, gs_last_error());
  return rc == 0;
}

// Runs one case; fills `out` with the global u field (z, y, x).
bool run_case(const Case& c, int nranks, const int* dims, int fuse, std::vector<double>& out,
              const std::string& bp_dir) {
  World w(nranks);
  std::vector<Rank> R(nranks);
  bool ok = true;
  std::mutex okm;
  for (int r = 0; r < nranks; ++r) {
    Rank& k = R[r];
    k.w = &w;
    k.rank = r;
    w.ranks[r] = &k;
    const int cz = r % dims[2], cy = (r / dims[2]) % dims[1], cx = r / (dims[1] * dims[2]);
    k.nx = split(c.L, dims[0], cx, &k.ox);
    k.ny = split(c.L, dims[1], cy, &k.oy);
    k.nz = split(c.L, dims[2], cz, &k.oz);
    gs_make_geom(&k.g, k.nx, k.ny, k.nz, fuse, k.ox, k.oy, k.oz, c.L, c.L, c.L, c.periodic);
    int32_t nbr[27];
    for (int d = 0; d < 27; ++d) {
      const int dx = d / 9 - 1, dy = (d / 3) % 3 - 1, dz = d % 3 - 1;
      nbr[d] = d == 13 ? -1 : rank_of(cx + dx, cy + dy, cz + dz, dims, c.periodic != 0);
    }
    const int64_t n = gs_geom_total_elems(&k.g);
    k.b0.assign(2 * n, 0.0);
    k.b1.assign(2 * n, 0.0);
    int64_t sc = 0, rc = 0;
    gs_plan_sizes(&k.g, nbr, fuse > 1 ? 1 : 0, &sc, &rc);
    k.send.assign(2 * (sc > 0 ? sc : 1), 0.0);
    k.recv.assign(2 * (rc > 0 ? rc : 1), 0.0);
    gs::Params p{};
    p.F = 0.02; p.k = 0.048; p.dt = 1.0; p.Du = 0.2; p.Dv = 0.1; p.noise = 0.1; p.seed = 4242;
    k.e = gs_create(1 /* fp64 */, &k.g, &p, nbr, r, fuse, 1, k.b0.data(), k.b1.data(), k.send.data(),
                    k.recv.data(), nullptr);
    if (!k.e) {
      fprintf(stderr, "gs_create: %s\n", gs_last_error());
      return false;
    }
    int64_t si, ri;
    int32_t ns, nr;
    gs_plan_info(k.e, &si, &ri, &ns, &nr);
    int64_t m4[4];
    for (int i = 0; i < ns; ++i) {
      gs_plan_msg(k.e, 0, i, m4);
      k.smsg.push_back({(int)m4[0], (int)m4[1], m4[2], m4[3]});
    }
    for (int i = 0; i < nr; ++i) {
      gs_plan_msg(k.e, 1, i, m4);
      k.rmsg.push_back({(int)m4[0], (int)m4[1], m4[2], m4[3]});
    }
    ok = ok && check(gs_set_transport(k.e, exchange_cb, &k), "set_transport");
  }
  out.assign((size_t)c.L * c.L * c.L, 0.0);
  std::vector<std::thread> th;
  for (int r = 0; r < nranks; ++r)
    th.emplace_back([&, r] {
      Rank& k = R[r];
      bool good = check(gs_init_fields(k.e), "init") && check(gs_advance(k.e, c.steps), "advance");
      std::vector<double> u((size_t)k.nx * k.ny * k.nz), v(u.size());
      good = good && check(gs_extract(k.e, u.data(), v.data()), "extract");
      for (int z = 0; z < k.nz; ++z)
        for (int y = 0; y < k.ny; ++y)
          for (int x = 0; x < k.nx; ++x)
            out[((size_t)(k.oz + z) * c.L + (k.oy + y)) * c.L + (k.ox + x)] =
                u[((size_t)z * k.ny + y) * k.nx + x];
      if (!bp_dir.empty()) {  // every rank writes its block of U
        void* h = bp4_open(bp_dir.c_str(), "SimulationOutput", r, nranks, 0);
        good = good && h;
        if (h) {
          const double F = 0.02;
          bp4_define_attribute(h, "F", 6, &F, 1);
          const uint64_t shape[3] = {(uint64_t)c.L, (uint64_t)c.L, (uint64_t)c.L};
          const uint64_t start[3] = {(uint64_t)k.oz, (uint64_t)k.oy, (uint64_t)k.ox};
          const uint64_t count[3] = {(uint64_t)k.nz, (uint64_t)k.ny, (uint64_t)k.nx};
          const int var = bp4_define_variable(h, "U", 6, 3, shape, start, count);
          good = good && var >= 0 && bp4_begin_step(h) == 0 && bp4_put(h, var, u.data()) == 0 &&
                 bp4_end_step(h) == 0;
          char* blob = nullptr;
          const int64_t nb = bp4_step_metadata(h, &blob);
          // rank 0 would gather every rank's blob; each thread-rank writes its own here
          if (r == 0 && nb > 0) {
            const char* blobs[1] = {blob};
            const int64_t sizes[1] = {nb};
            good = good && bp4_write_metadata(h, 1, blobs, sizes) == 0;
          }
          good = good && bp4_close(h) == 0;
          if (!good) fprintf(stderr, "bp4: %s\n", bp4_last_error());
        }
      }
      gs_destroy(k.e);
      std::lock_guard<std::mutex> lk(okm);
      ok = ok && good;
    });
  for (auto& t : th) t.join();
  return ok;
}

// The asynchronous output path's host threads (io/output.py + bp4_async_*): one writer's
// native thread writes queued steps (after a stand-in "device copy" wait) while the caller takes
// each finished step's blob and appends the metadata -- the pattern of the driver's output
// queue, two steps in flight.  Checked for races by `make tsan`, for leaks by `make asan`.
int fake_copy_wait(void* arg) {
  std::this_thread::sleep_for(std::chrono::microseconds(50 + (int)(intptr_t)arg % 3 * 40));
  return 0;
}

bool run_async_writer(const std::string& dir) {
  const int nx = 9, ny = 7, nz = 5, steps = 12;
  void* h = bp4_open(dir.c_str(), "SimulationOutput", 0, 1, 0);
  if (!h) return false;
  const uint64_t shape[3] = {nz, ny, nx}, start[3] = {0, 0, 0};
  const int vs = bp4_define_variable(h, "step", 2, 0, nullptr, nullptr, nullptr);
  const int vu = bp4_define_variable(h, "U", 5, 3, shape, start, shape);
  const int vv = bp4_define_variable(h, "V", 5, 3, shape, start, shape);
  std::vector<std::vector<float>> u(steps, std::vector<float>(nx * ny * nz)), v = u;
  std::vector<std::vector<float>> part(steps, std::vector<float>(8));
  for (int s = 0; s < steps; ++s) {
    for (size_t i = 0; i < u[s].size(); ++i) {
      u[s][i] = (float)(s + i % 11);
      v[s][i] = (float)(s - (int)(i % 5));
    }
    // two chunks' (u min, u max, v min, v max)
    const size_t half = u[s].size() / 2;
    auto mm = [&](const std::vector<float>& a, size_t b, size_t e, float* o) {
      o[0] = *std::min_element(a.begin() + b, a.begin() + e);
      o[1] = *std::max_element(a.begin() + b, a.begin() + e);
    };
    mm(u[s], 0, half, &part[s][0]);
    mm(v[s], 0, half, &part[s][2]);
    mm(u[s], half, u[s].size(), &part[s][4]);
    mm(v[s], half, v[s].size(), &part[s][6]);
  }
  bool good = vs >= 0 && vu >= 0 && vv >= 0;
  std::vector<int64_t> tickets;
  size_t done = 0;
  auto commit = [&]() {
    const char* blob = nullptr;
    int64_t n = 0;
    good = good && bp4_async_result(h, tickets[done++], &blob, &n) == 0 && n > 0;
    if (good) {
      const char* blobs[1] = {blob};
      const int64_t sizes[1] = {n};
      good = bp4_write_metadata(h, 1, blobs, sizes) == 0;  // md.0 / md.idx, beside the data thread
    }
  };
  for (int s = 0; s < steps && good; ++s) {
    while (tickets.size() - done >= 2) commit();
    const int64_t t = bp4_async_submit(h, fake_copy_wait, (void*)(intptr_t)s, vs, 10 * s, vu,
                                       u[s].data(), vv, v[s].data(), part[s].data(), 2);
    good = good && t >= 0;
    tickets.push_back(t);
  }
  while (good && done < tickets.size()) commit();
  good = bp4_close(h) == 0 && good;
  if (!good) fprintf(stderr, "bp4 async: %s\n", bp4_last_error());
  return good;
}

}  // namespace

int main(int argc, char** argv) {
  const std::string tmp = argc > 1 ? argv[1] : "/tmp";
  const Case cases[] = {
      {14, {2, 2, 2}, 2, 7, 0}, {13, {1, 2, 2}, 3, 5, 0}, {16, {1, 1, 4}, 3, 7, 0},
      {12, {2, 1, 1}, 1, 6, 1}, {16, {2, 2, 2}, 3, 6, 1}, {15, {3, 1, 1}, 2, 5, 0},
  };
  int fails = 0;
  for (const Case& c : cases) {
    std::vector<double> one, many;
    const int d1[3] = {1, 1, 1};
    const int n = c.dims[0] * c.dims[1] * c.dims[2];
    const bool ok1 = run_case(c, 1, d1, 1, one, "");
    const bool okn = run_case(c, n, c.dims, c.fuse, many, tmp + "/gs_selftest_" + std::to_string(n) + ".bp");
    size_t bad = 0;
    for (size_t i = 0; i < one.size(); ++i)
      if (memcmp(&one[i], &many[i], sizeof(double)) != 0) ++bad;
    const bool pass = ok1 && okn && bad == 0;
    printf("L=%d dims=%dx%dx%d fuse=%d periodic=%d: %s (%zu mismatches)\n", c.L, c.dims[0],
           c.dims[1], c.dims[2], c.fuse, c.periodic, pass ? "ok" : "FAIL", bad);
    fails += pass ? 0 : 1;
  }
  const bool aw = run_async_writer(tmp + "/gs_selftest_async.bp");
  printf("bp4 asynchronous writer thread, 12 steps, 2 in flight: %s\n", aw ? "ok" : "FAIL");
  fails += aw ? 0 : 1;
  printf(fails ? "SELFTEST FAILED\n" : "SELFTEST OK\n");
  return fails ? 1 : 0;
}
