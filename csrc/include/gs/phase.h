// SPDX-License-Identifier: MIT
// Per-phase timing of the scheduler's passes ("hipEvent-based per-phase timers:
// halo pack, comm, interior, boundary").  The reference times only the whole run
// (gray-scott.jl:12, `@time julia_main()`); its phases are exchange! -> calculate! -> swap
// (src/simulation/public.jl:58-68).
//
// The engine brackets every phase of a pass with two timestamps taken *in stream order on the
// stream the phase runs on* (Backend::prof_mark: a hipEvent on the GPU, the host clock on the
// synchronous CPU backend), so overlapped work on the compute and communication streams is
// timed without synchronising anything.  Profiling is switched on for an explicit window only
// (Engine::prof_start / prof_stop); outside it the marks cost one predictable branch.
//
// PhaseLog keeps the records; summarize() turns the timestamps into per-pass phase times:
//   * phase_us[p]     median over the window's passes of the time phase p took in a pass
//                     (the sum of its intervals in that pass; passes without it are skipped)
//   * per_pass[p]     mean number of intervals of phase p per pass
//   * exchange_us     median per pass of the halo exchange's span: first begin of pack /
//                     transport / unpack to the last end of them (includes waiting for peers)
//   * pass_us         the window's wall time (first to last timestamp) / passes
#pragma once

#include <stdint.h>

#include <algorithm>
#include <vector>

namespace gs {

enum Phase : int32_t {
  kPhPack = 0,     // halo gather into the send buffer (IPC: stores straight into the peers)
  kPhTransport,    // RCCL group / IPC signal + wait / host callback / in-place RCCL planes
  kPhUnpack,       // halo scatter into the ghost cells
  kPhInner,        // overlapped pass: the inner box (runs while the halos fly)
  kPhShell,        // overlapped pass: the face slabs after the halos landed
  kPhFused,        // non-overlapped pass: the whole-interior temporally blocked kernel
  kPhStep,         // single-step kernels (fuse = 1, or no fused kernel for this depth)
  kPhBc,           // outer-boundary ghost refresh (ensure_bc)
  kNumPhases
};

inline const char* phase_name(int p) {
  static const char* n[kNumPhases] = {"pack", "transport", "unpack", "inner",
                                      "shell", "fused", "step", "bc"};
  return p >= 0 && p < kNumPhases ? n[p] : "?";
}

// layout of the summary array (doubles) returned by Engine::prof_stop / gs_prof_stop
constexpr int kProfHead = 5;  // passes, steps, window_us, pass_us, exchange_us
constexpr int kProfLen = kProfHead + 2 * kNumPhases;

struct PhaseRec {
  int32_t phase;  // Phase, or -1 for the window's start / end stamps
  int32_t begin;  // 1 begin, 0 end
  int32_t pass;   // pass index within the window
};

struct PhaseLog {
  std::vector<PhaseRec> recs;
  size_t cap = 0;
  bool on = false;
  bool overflow = false;
  int32_t pass = -1;   // index of the pass being issued (-1: before the first)
  int32_t npass = 0;   // passes started in the window
  int64_t steps = 0;   // steps they advance

  void start(size_t max_records) {
    recs.clear();
    recs.reserve(max_records);
    cap = max_records;
    on = true;
    overflow = false;
    pass = -1;
    npass = 0;
    steps = 0;
  }
  void begin_pass(int k) {
    if (!on) return;
    pass = npass++;
    steps += k;
  }
  // slot of the next record, or -1 (off / full: the record is dropped, `overflow` is set)
  int next(int32_t phase, bool begin) {
    if (!on) return -1;
    if (recs.size() >= cap) {
      overflow = true;
      return -1;
    }
    recs.push_back(PhaseRec{phase, begin ? 1 : 0, pass});
    return (int)recs.size() - 1;
  }
};

inline double median_of(std::vector<double> v) {
  if (v.empty()) return 0.0;
  std::sort(v.begin(), v.end());
  const size_t n = v.size();
  return n & 1 ? v[n / 2] : 0.5 * (v[n / 2 - 1] + v[n / 2]);
}

// t_us[i]: timestamp of record i (any common origin).  out: kProfLen doubles (layout above:
// head, then {median us, intervals per pass} for every phase).  Returns the number of passes.
inline int summarize(const PhaseLog& log, const double* t_us, double* out) {
  for (int i = 0; i < kProfLen; ++i) out[i] = 0.0;
  const size_t n = log.recs.size();
  const int np = log.npass;
  out[1] = (double)log.steps;
  if (n == 0 || np <= 0) return 0;
  double tmin = t_us[0], tmax = t_us[0];
  for (size_t i = 0; i < n; ++i) {
    tmin = std::min(tmin, t_us[i]);
    tmax = std::max(tmax, t_us[i]);
  }
  // per pass x phase: summed time and interval count; per pass: exchange span
  std::vector<double> sum((size_t)np * kNumPhases, 0.0), cnt((size_t)np * kNumPhases, 0.0);
  std::vector<double> xlo((size_t)np, 1e300), xhi((size_t)np, -1e300);
  double open[kNumPhases];
  int open_pass[kNumPhases];
  for (int p = 0; p < kNumPhases; ++p) open[p] = -1.0, open_pass[p] = -1;
  for (size_t i = 0; i < n; ++i) {
    const PhaseRec& r = log.recs[i];
    if (r.phase < 0 || r.phase >= kNumPhases || r.pass < 0 || r.pass >= np) continue;
    const int p = r.phase;
    if (r.begin) {
      open[p] = t_us[i];
      open_pass[p] = r.pass;
      continue;
    }
    if (open_pass[p] < 0) continue;  // an end without its begin (overflowed log)
    const size_t k = (size_t)open_pass[p] * kNumPhases + p;
    sum[k] += std::max(0.0, t_us[i] - open[p]);
    cnt[k] += 1.0;
    if (p <= kPhUnpack) {
      xlo[open_pass[p]] = std::min(xlo[open_pass[p]], open[p]);
      xhi[open_pass[p]] = std::max(xhi[open_pass[p]], t_us[i]);
    }
    open_pass[p] = -1;
  }
  out[0] = np;
  out[2] = tmax - tmin;
  out[3] = (tmax - tmin) / np;
  std::vector<double> v;
  for (int q = 0; q < np; ++q)
    if (xhi[q] >= xlo[q]) v.push_back(xhi[q] - xlo[q]);
  out[4] = median_of(v);
  for (int p = 0; p < kNumPhases; ++p) {
    v.clear();
    double c = 0.0;
    for (int q = 0; q < np; ++q) {
      const size_t k = (size_t)q * kNumPhases + p;
      c += cnt[k];
      if (cnt[k] > 0) v.push_back(sum[k]);
    }
    out[kProfHead + 2 * p] = median_of(v);
    out[kProfHead + 2 * p + 1] = c / np;
  }
  return np;
}

}  // namespace gs
