// SPDX-License-Identifier: MIT
// Backend-independent time-stepping scheduler (the native runtime around the kernels).
//
// Reference call stack being replaced: public.jl:45 iterate! ->
// exchange! (communication.jl:138-199, host-staged blocking Sendrecv) -> calculate! ->
// swap (public.jl:67-68).  Here one "pass" fuses up to H steps per halo exchange:
//   pack -> transport (RCCL / callback / self-copy) -> unpack -> k steps -> swap.
// The outer-boundary ghost values of each buffer are kept at the parity the reference's
// init + swap pattern implies by `ensure_bc`, so the stencil kernels never
// need per-cell boundary predicates on level-0 data.
#pragma once

#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <algorithm>
#include <chrono>
#include <stdexcept>
#include <string>
#include <vector>

#include "gs/common.h"
#include "gs/debug.h"
#include "gs/phase.h"
#include "gs/trace.h"

namespace gs {

enum DType : int32_t { kF32 = 0, kF64 = 1 };

// Seconds a blocked communication step (RCCL set-up, a halo exchange, a device wait) may take
// before it becomes an error: GS_COMM_TIMEOUT, read at every call so a caller that changes it
// for one engine (the data-path tuner's candidates) is obeyed.  Default 900.
inline double comm_timeout_s() {
  const char* e = getenv("GS_COMM_TIMEOUT");
  const double v = e ? atof(e) : 900.0;
  return v > 0.0 ? v : 900.0;
}

// Transport callback: exchange the packed send buffer into the receive buffer.
// Returns 0 on success.
typedef int (*TransportFn)(void* user);

class Backend {
 public:
  virtual ~Backend() {}
  // fill box of buffer b with a constant (u,v) pair
  virtual void fill_box(int b, const Box& box, double u, double v) = 0;
  // several boxes of buffer b with one (u,v) pair (the outer ghost faces: one launch on GPU)
  virtual void fill_boxes(int b, const Box* boxes, int n, double u, double v) {
    for (int i = 0; i < n; ++i) fill_box(b, boxes[i], u, v);
  }
  // one explicit Euler step over `region`, reading buffer src at time t, writing dst
  virtual void step(int src, int dst, const Box& region, int64_t t) = 0;
  // temporally blocked kernel: n steps over the interior, src at time t -> dst at t+n.
  // Returns false if unsupported for this n (the scheduler then falls back to step()).
  virtual bool fused(int src, int dst, int n, int64_t t) { (void)src; (void)dst; (void)n; (void)t; return false; }
  // optional one-time preparation (autotuning) of the fused kernel for depth n; must not
  // change the state held in buffer src
  virtual void prepare_fused(int src, int dst, int n, int64_t t) { (void)src; (void)dst; (void)n; (void)t; }
  // milliseconds of one whole-interior fused pass of depth n as timed by prepare_fused (0 if
  // not timed: tuning disabled or a configuration pinned)
  virtual double fused_ms(int n) const { (void)n; return 0.0; }
  // fused() restricted to the output z-runs [zlo0, +zlen0) and [zlo1, +zlen1) (zlen1 may be 0).
  // Supported exactly when fused_supported(n); reads level-0 planes zlo-n .. zend+n-1 only.
  virtual bool fused_supported(int n) const { (void)n; return false; }
  // leave_room: launch fewer workgroups than the device holds so concurrently running
  // communication kernels (RCCL) find free slots instead of waiting for this kernel to end.
  // mask (bit0 -x, bit1 +x, bit2 -y, bit3 +y): outputs within n of those faces are not
  // written -- the inner part of an overlapped pass, whose tiles may read in-flight halos.
  virtual bool fused_runs(int src, int dst, int n, int64_t t, int zlo0, int zlen0, int zlo1,
                          int zlen1, bool leave_room = false, int mask = 0) {
    (void)src; (void)dst; (void)n; (void)t; (void)zlo0; (void)zlen0; (void)zlo1; (void)zlen1;
    (void)leave_room; (void)mask;
    return false;
  }
  // the shell of an overlapped n-step pass: the n cells next to every face flagged in `sides`
  // (bit0 -x, bit1 +x, bit2 -y, bit3 +y, bit4 -z, bit5 +z), src at time t -> dst.  Supported
  // exactly when fused_supported(n).  variant >= 0 forces one implementation (tests).
  virtual bool shell(int src, int dst, int n, int64_t t, int sides, int variant = -1) {
    (void)src; (void)dst; (void)n; (void)t; (void)sides; (void)variant;
    return false;
  }
  // Gated pass (device transport with in-kernel exchange, csrc/hip/gate.hpp): one launch per
  // pass that packs, signals, waits and unpacks inside the fused kernel.  gated_supported: this
  // backend can run depth-n passes that way now (IPC transport set up, a landing route for
  // every message); prepare_gated: tune it (every rank the same passes); fused_gated: one pass
  // src -> dst including the halo exchange of src.
  virtual bool gated_supported(int n) const { (void)n; return false; }
  virtual void prepare_gated(int src, int dst, int n, int64_t t) { (void)src; (void)dst; (void)n; (void)t; }
  // first / last: the pass opens / closes a run of gated passes (carried exchanges stay inside
  // a run)
  virtual bool fused_gated(int src, int dst, int n, int64_t t, bool first, bool last) {
    (void)src; (void)dst; (void)n; (void)t; (void)first; (void)last;
    return false;
  }
  // in-place transport of a zplanes plan straight from / into field buffer b (no pack)
  virtual bool native_exchange_inplace(int b, const HaloPlan& p) { (void)b; (void)p; return false; }
  // asynchronous communication stream.  comm_fork: the comm stream waits for the compute
  // work issued so far; comm_join: the compute stream waits for the comm work issued so far;
  // comm_select(true) routes pack / unpack / self_copy / native_exchange* / host_sync to the
  // comm stream, comm_select(false) back to the compute stream.
  virtual bool has_comm_stream() const { return false; }
  virtual void comm_fork() {}
  virtual void comm_join() {}
  virtual void comm_select(bool on) { (void)on; }
  // event slots (0..3) for finer cross-stream ordering: mark records slot `which` on the comm
  // (on_comm) or compute stream at this point; wait_mark makes that stream wait for the slot's
  // last record
  virtual void mark(int which, bool on_comm) { (void)which; (void)on_comm; }
  virtual void wait_mark(int which, bool on_comm) { (void)which; (void)on_comm; }
  // whether native_exchange_inplace would carry this plan (device transport, no self copies)
  virtual bool can_exchange_inplace(const HaloPlan& p) const { (void)p; return false; }
  // whether native_exchange has a device transport (RCCL) configured
  virtual bool has_native_transport() const { return false; }
  virtual void pack(int b, const HaloPlan& p) = 0;
  virtual void unpack(int b, const HaloPlan& p) = 0;
  // copy send-buffer cells [src_off, +n) to recv-buffer cells [dst_off, +n)
  virtual void self_copy(int64_t src_off, int64_t dst_off, int64_t n) = 0;
  // native transport (RCCL); returns false if not configured
  virtual bool native_exchange(const HaloPlan& p) { (void)p; return false; }
  // loopback: messages to this rank also go through the native transport (tests)
  virtual void set_loopback(bool on) { (void)on; }
  // forget the device transport (RCCL communicator, IPC mappings) after a failed trial
  virtual void drop_transport() {}
  virtual void host_sync() {}
  // wait for all queued device work; a backend with a device transport turns a hang or an
  // asynchronous transport error into an exception after `timeout_s` seconds (watchdog)
  virtual void wait_all(double timeout_s) { (void)timeout_s; host_sync(); }
  virtual void extract(int b, void* u, void* v) = 0;
  // extract plus each chunk's min / max of u and v (cap quadruples {umin, umax, vmin, vmax} of the
  // field's type at `part`); returns the number written, or -1 if the backend has no such path
  virtual int extract_minmax(int b, void* u, void* v, void* part, int cap) {
    (void)b; (void)u; (void)v; (void)part; (void)cap;
    return -1;
  }
  virtual void insert(int b, const void* u, const void* v) = 0;
  // random interior of buffer b, a function of the global cell only (gs::random_init_cell)
  virtual void randomize(int b, uint64_t seed, double lo, double hi) = 0;
  // seed cube into buffer b
  virtual void seed(int b) = 0;
  // sum / min / max of u and v over the interior: out[6]
  virtual void stats(int b, double* out) = 0;

  // Per-phase timing (gs/phase.h).  prof_reserve: room for n timestamps; prof_mark: take
  // timestamp `slot` in stream order on the stream the phase's work is issued to (phase -1: the
  // compute stream); prof_times: all n timestamps in microseconds from a common origin, once
  // the work has finished.  The default is the host clock, exact for a synchronous backend.
  virtual void prof_reserve(int n) { host_us_.assign((size_t)n, 0.0); }
  virtual void prof_mark(int slot, int phase) {
    (void)phase;
    if (slot >= 0 && (size_t)slot < host_us_.size())
      host_us_[(size_t)slot] = std::chrono::duration<double, std::micro>(
                                   std::chrono::steady_clock::now().time_since_epoch()).count();
  }
  virtual void prof_times(double* us, int n) {
    for (int i = 0; i < n; ++i) us[i] = (size_t)i < host_us_.size() ? host_us_[(size_t)i] : 0.0;
  }

 private:
  std::vector<double> host_us_;
};

// The cheapest partition of nsteps into passes of depth 2..kmax, given each depth's pass time
// cost[k] (all > 0, else an empty plan): an exact dynamic programme over the last kPlanTail
// steps, before them passes of the depth with the lowest time per step.  nsteps = 1 is a lone
// single step (depth 1).  (Engine::plan_passes; tests/test_planner.py.)
//   fill = 0: deepest passes first.  fill > 0 (non-periodic grids): one outer-ghost refresh
// (Engine::ensure_bc) costs `fill`, and one runs whenever two consecutive passes differ in depth
// parity -- the buffer read next is then read at the other time parity than when it was last
// filled; pp is the depth parity a first pass needs to avoid one (-1: no preference).  The plan
// is then the cheapest of the best all-even, all-odd and mixed partitions with those refreshes
// counted, its passes grouped by parity (pp's group first), deepest first within a group:
// 4,4,3,3,3,3 after an even pass, not 3,3,3,3,4,4.
constexpr int64_t kPlanTail = 240;
namespace plan_detail {
// the cheapest partition using the depths whose parity bit is in `allow` (bit0 even, bit1 odd);
// *total = 1e300 if there is none
inline std::vector<int> solve(const double* cost, int kmax, int64_t nsteps, int allow,
                              double* total) {
  std::vector<int> out;
  *total = 1e300;
  auto ok = [&](int k) { return ((allow >> (k & 1)) & 1) != 0; };
  int dbest = 0;
  for (int k = 2; k <= kmax; ++k)
    if (ok(k) && (dbest == 0 || cost[k] / k < cost[dbest] / dbest)) dbest = k;
  if (dbest == 0) return out;
  const int64_t head = nsteps > kPlanTail ? (nsteps - kPlanTail) / dbest : 0;
  const int tail = (int)(nsteps - head * dbest);
  std::vector<double> best((size_t)tail + 1, 1e300);
  std::vector<int> how((size_t)tail + 1, 0);
  best[0] = 0.0;
  for (int m = 2; m <= tail; ++m)
    for (int k = kmax; k >= 2; --k)  // ties: the deeper pass (fewer launches)
      if (ok(k) && k <= m && best[(size_t)(m - k)] < 1e300 &&
          best[(size_t)(m - k)] + cost[k] < best[(size_t)m] * (1.0 - 1e-12)) {
        best[(size_t)m] = best[(size_t)(m - k)] + cost[k];
        how[(size_t)m] = k;
      }
  if (tail == 1) {
    if (!(allow & 2)) return out;  // a lone single step is odd
  } else if (!(best[(size_t)tail] < 1e300)) {
    return out;
  }
  out.assign((size_t)head, dbest);
  for (int m = tail; m >= 2; m -= how[(size_t)m]) out.push_back(how[(size_t)m]);
  if (tail == 1) out.push_back(1);
  *total = (double)head * cost[dbest] + (tail == 1 ? 0.0 : best[(size_t)tail]);
  return out;
}
}  // namespace plan_detail

inline std::vector<int> plan_depths(const double* cost, int kmax, int64_t nsteps,
                                    double fill = 0.0, int pp = -1) {
  std::vector<int> out;
  if (nsteps < 1 || kmax < 2) return out;
  for (int k = 2; k <= kmax; ++k)
    if (!(cost[k] > 0.0)) return out;
  double tot = 0.0;
  if (!(fill > 0.0)) {
    out = plan_detail::solve(cost, kmax, nsteps, 3, &tot);
    std::sort(out.begin(), out.end(), [](int x, int y) { return x > y; });
    return out;
  }
  // the refreshes a plan made of these parities needs (grouped, pp's group first)
  auto refreshes = [&](const std::vector<int>& p) {
    bool ev = false, od = false;
    for (int k : p) (k & 1 ? od : ev) = true;
    if (ev && od) return 1;
    if (pp < 0 || p.empty()) return 0;
    return (od ? 1 : 0) != pp ? 1 : 0;
  };
  double best = 1e300;
  for (int allow : {3, 1, 2}) {  // ties: the plain optimum
    double t = 0.0;
    std::vector<int> p = plan_detail::solve(cost, kmax, nsteps, allow, &t);
    if (!(t < 1e300)) continue;
    t += fill * refreshes(p);
    if (t < best * (1.0 - 1e-12)) {
      best = t;
      out = p;
    }
  }
  const int first = pp >= 0 ? pp : (out.empty() ? 0 : (*std::max_element(out.begin(), out.end()) & 1));
  std::sort(out.begin(), out.end(), [first](int x, int y) {
    const int gx = (x & 1) != first, gy = (y & 1) != first;
    return gx != gy ? gx < gy : x > y;
  });
  return out;
}

struct EngineConfig {
  Geom g;
  Params p;
  int32_t nbr[27];
  int32_t rank;
  int32_t fuse;        // max steps per halo exchange (<= g.H)
  int32_t use_fused;   // allow the temporally-blocked kernel
};

class Engine {
 public:
  Engine(const EngineConfig& c, Backend* be) : cfg_(c), be_(be) {
    if (c.fuse < 1 || c.fuse > c.g.H) throw std::runtime_error("fuse must be in [1, H]");
    int nb = 0;
    for (int d = 0; d < 27; ++d) {
      if (d == 13 || c.nbr[d] < 0) continue;
      ++nb;
      if (c.nbr[d] != c.rank) has_remote_ = true;
    }
    has_nbr_ = nb > 0;
    plan_ = make_halo_plan(c.g, c.nbr, c.g.H > 1 || c.fuse > 1);
    bc_parity_[0] = bc_parity_[1] = -1;
  }
  ~Engine() { delete be_; }

  const HaloPlan& plan() const { return plan_; }
  Backend* backend() { return be_; }
  int cur() const { return cur_; }
  int64_t step() const { return t_; }
  void set_step(int64_t t) { t_ = t; bc_parity_[0] = bc_parity_[1] = -1; }
  void set_transport(TransportFn fn, void* user) { tfn_ = fn; tuser_ = user; }
  // back to "no transport" (the fallback chain tries the next one from a clean state)
  void drop_transport() {
    tfn_ = nullptr;
    tuser_ = nullptr;
    be_->drop_transport();
  }
  // comm/compute overlap: -1 auto (on with a device transport and a comm stream),
  // 0 off, 1 on where possible
  void set_overlap(int mode) { overlap_ = mode; }
  // Loopback (tests): periodic wraps onto this rank travel through the device transport
  // (RCCL send/recv to self) instead of self copies, so a single GPU exercises the whole
  // multi-rank data path: packed and in-place messages, the comm stream and the overlap.
  void set_loopback(bool on) {
    loopback_ = on;
    be_->set_loopback(on);
    has_remote_ = false;
    for (int d = 0; d < 27; ++d)
      if (d != 13 && cfg_.nbr[d] >= 0 && (on || cfg_.nbr[d] != cfg_.rank)) has_remote_ = true;
  }
  // whether a pass of k steps runs with the halo exchange overlapped with the inner update:
  // the inner box (cells >= k from every face with a neighbour) while the halos fly, then the
  // k-deep face slabs ("auto" only with a device transport: a host callback serialises anyway)
  bool overlapped(int k) const {
    const Geom& g = cfg_.g;
    return (overlap_ == 1 || (overlap_ == -1 && tfn_ == nullptr)) && cfg_.use_fused && k > 1 &&
           has_remote_ && be_->has_comm_stream() && be_->fused_supported(k) &&
           g.nz >= 2 * k + 1 && g.nx >= 2 * k + 1 && g.ny >= 2 * k + 1;
  }
  double comm_calls() const { return (double)ncomm_; }

  // Per-phase timing window (gs/phase.h): from prof_start on, every phase of every
  // pass is bracketed by two timestamps in stream order (at most max_records in all);
  // prof_stop waits for the device (watchdog: timeout_s) and writes the summary, kProfLen
  // doubles.  Returns 1 if records were dropped (window too long for max_records), else 0.
  void prof_start(int max_records) {
    plog_.start((size_t)(max_records < 4 ? 4 : max_records));
    be_->prof_reserve((int)plog_.cap);
    pm(-1, true);  // the window's start, on the compute stream
  }
  int prof_stop(double* out, double timeout_s) {
    if (!plog_.on) throw std::runtime_error("prof_stop without prof_start");
    pm(-1, false);  // every pass ends joined to the compute stream
    plog_.on = false;
    be_->wait_all(timeout_s);
    std::vector<double> t(plog_.recs.size(), 0.0);
    if (!t.empty()) be_->prof_times(t.data(), (int)t.size());
    summarize(plog_, t.data(), out);
    return plog_.overflow ? 1 : 0;
  }

  // Reference init (Simulation_CPU.jl:14-65): u = 1 everywhere (ghosts included), v = 0,
  // u_temp = v_temp = 0, then the 13^3 seed cube.
  void init_fields() {
    const Geom& g = cfg_.g;
    Box all{-g.H, -g.H, -g.H, g.nx + 2 * g.H, g.ny + 2 * g.H, g.nz + 2 * g.H};
    be_->fill_box(0, all, 1.0, 0.0);
    be_->fill_box(1, all, 0.0, 0.0);
    be_->seed(0);
    cur_ = 0;
    t_ = 0;
    bc_parity_[0] = 0;  // u ghosts = 1 -> even time
    bc_parity_[1] = 1;  // u_temp ghosts = 0 -> odd time
  }

  // Random-init the current state's interior (u, v ~ U[lo, hi), decomposition-invariant).
  void randomize(uint64_t seed, double lo, double hi) { be_->randomize(cur_, seed, lo, hi); }

  // Tune every fused depth this engine can use, without changing the state.
  void prepare() {
    if (!cfg_.use_fused) return;
    for (int n = 2; n <= cfg_.fuse; ++n) {
      be_->prepare_fused(cur_, 1 - cur_, n, t_);
      if (gated(n)) {
        // the gated pass's table and expected exchange time (every rank the same passes)
        be_->prepare_gated(cur_, 1 - cur_, n, t_);
        continue;
      }
      // tune the overlapped passes' post-exchange launches now too (their first call times
      // the candidates), so no tuning lands inside a timed region; all on the compute stream
      if (overlapped(n)) {
        const Split sp = overlap_split(n);
        inner_run(cur_, 1 - cur_, n, t_, sp);
        shell_run(cur_, 1 - cur_, n, t_, sp);
      }
    }
    // Without a halo exchange to amortise, the depth is a pure kernel-cost choice: use the one
    // with the lowest tuned time per step (small grids: T=2 tiles waste less on the 2T halo,
    // large ones: T=3 saves HBM traffic; profiles/r2_fuse_small.txt, r3_small_grid.txt).
    if (auto_depth_ && !has_remote_ && cfg_.fuse >= 3) {
      double best = 0.0;
      for (int n = 2; n <= cfg_.fuse; ++n) {
        const double ms = be_->fused_ms(n);
        if (ms <= 0.0) {
          best = 0.0;
          break;
        }
        if (best == 0.0 || ms / n < best) {
          best = ms / n;
          depth_ = n;
        }
      }
      // nothing timed (GS_AUTOTUNE=0 or a pinned configuration): the plane-size rule measured
      // with the default tile -- T=2 below 160^2 x-y planes (L=64: 54k vs 42k MLUPS at T=3,
      // profiles/r2_fuse_small.txt), else the full depth up to T=3 (the untuned T=4 tile is the
      // unfolded one, 10 % under T=3 at L=512: profiles/r6_t4.txt)
      if (best == 0.0) depth_ = (cfg_.g.nx < 160 || cfg_.g.ny < 160) ? 2 : (cfg_.fuse > 3 ? 3 : 0);
    }
    // the planner's price of a parity switch: one outer-ghost refresh of the other buffer
    // (timed on the device's clock; its contents are reset just below)
    fill_ms_ = 0.0;
    if (!cfg_.g.periodic && !has_remote_ && planner_ && !plog_.on) {
      constexpr int kReps = 4;
      be_->prof_reserve(2);
      be_->prof_mark(0, -1);
      for (int r = 0; r < kReps; ++r) {
        bc_parity_[1 - cur_] = -1;
        ensure_bc(1 - cur_, t_ + r);
      }
      be_->prof_mark(1, -1);
      be_->host_sync();
      double us[2] = {0.0, 0.0};
      be_->prof_times(us, 2);
      fill_ms_ = us[1] > us[0] ? (us[1] - us[0]) * 1e-3 / kReps : 0.0;
    }
    // the timing runs scribbled over the other buffer: restore the reference's zeroed
    // u_temp/v_temp (ghosts included) so the ghost-parity bookkeeping stays exact
    const Geom& g = cfg_.g;
    Box all{-g.H, -g.H, -g.H, g.nx + 2 * g.H, g.ny + 2 * g.H, g.nz + 2 * g.H};
    be_->fill_box(1 - cur_, all, 0.0, 0.0);
    bc_parity_[1 - cur_] = 1;  // u ghosts = 0 <-> odd time
  }

  void exchange() {
    exchange_start();
    exchange_finish();
  }

  // Stage 1 of a halo exchange: everything that can be issued without blocking the host
  // (pack, periodic self copies, RCCL send/recv -- in place for a zplanes plan).
  void exchange_start() {
    TraceRange tr("gs.exchange_start");
    xpending_ = kNone;
    if (!has_nbr_) return;
    if (plan_.zplanes && has_remote_ && be_->can_exchange_inplace(plan_)) {
      pm(kPhTransport, true);
      const bool done = be_->native_exchange_inplace(cur_, plan_);
      pm(kPhTransport, false);
      if (done) {
        ++ncomm_;
        return;  // nothing to unpack
      }
    }
    pm(kPhPack, true);
    be_->pack(cur_, plan_);
    // self messages (periodic wrap onto the same rank)
    bool remote = false;
    for (int i = 0; i < plan_.nrecv; ++i) {
      const HaloMsg& r = plan_.recv[i];
      if (r.peer == cfg_.rank && !loopback_) {
        const int sd = 26 - r.dir;  // my send towards -d lands in my ghost d
        for (int j = 0; j < plan_.nsend; ++j)
          if (plan_.send[j].dir == sd && plan_.send[j].peer == cfg_.rank)
            be_->self_copy(plan_.send[j].offset, r.offset, box_cells(r.box));
      } else {
        remote = true;
      }
    }
    pm(kPhPack, false);
    xpending_ = kUnpack;
    if (remote) {
      ++ncomm_;
      const bool native = be_->has_native_transport();
      if (native) pm(kPhTransport, true);
      if (!be_->native_exchange(plan_)) {
        if (!tfn_) throw std::runtime_error("halo exchange needs a transport (RCCL or callback)");
        xpending_ = kCallback;
      }
      if (native) pm(kPhTransport, false);
    }
  }

  // Stage 2: host-side transports (callback) and the unpack.
  void exchange_finish(bool on_comm = false) {
    TraceRange tr("gs.exchange_finish");
    if (xpending_ == kCallback) {
      be_->host_sync();
      pm(kPhTransport, true);
      if (tfn_(tuser_) != 0) throw std::runtime_error("transport callback failed");
      pm(kPhTransport, false);
      // the callback's device copies were issued on the compute stream
      if (on_comm) be_->comm_fork();
    }
    if (xpending_ != kNone) {
      pm(kPhUnpack, true);
      be_->unpack(cur_, plan_);
      pm(kPhUnpack, false);
    }
    xpending_ = kNone;
  }

  // Fill the outer (global-boundary) ghost shells of buffer b with the boundary value of
  // time t.  Faces cover the full ghost-extended range so edges/corners are covered too.
  void ensure_bc(int b, int64_t t) {
    TraceRange tr("gs.ensure_bc");
    const Geom& g = cfg_.g;
    if (g.periodic) return;
    const int par = (int)(t & 1);
    if (bc_parity_[b] == par) return;
    const double u = bc_u(t);
    const int H = g.H;
    Box faces[6];
    int nf = 0;
    for (int a = 0; a < 3; ++a)
      for (int s = -1; s <= 1; s += 2) {
        int dd[3] = {0, 0, 0};
        dd[a] = s;
        if (cfg_.nbr[dir_index(dd[0], dd[1], dd[2])] >= 0) continue;
        // whole padded rows along x (the row padding is never read for a stored cell): every
        // write is a run of aligned 64-byte segments -- an x face of 3-cell pieces per row cost
        // ~30 us at 512^3, partial-line writes
        Box bx{-g.xo, -H, -H, g.px, g.ny + 2 * H, g.nz + 2 * H};
        if (a == 0) {
          bx.x0 = s < 0 ? -g.xo : g.nx;
          bx.nx = s < 0 ? g.xo : g.px - g.xo - g.nx;
        } else {
          int32_t* o = a == 1 ? &bx.y0 : &bx.z0;
          int32_t* c = a == 1 ? &bx.ny : &bx.nz;
          const int n = a == 1 ? g.ny : g.nz;
          *o = s < 0 ? -H : n;
          *c = H;
        }
        faces[nf++] = bx;
      }
    if (nf) {
      pm(kPhBc, true);
      be_->fill_boxes(b, faces, nf, u, 0.0);
      pm(kPhBc, false);
    }
    bc_parity_[b] = par;
  }

  // whether full-depth passes run gated: the exchange inside the pass's fused launch
  // (gate.hpp; the IPC transport).  Taken before the stream-overlapped modes; the debug knob
  // gated = 0 (tests, A/B) or overlap off disable it.
  bool gated(int k) const {
    return gate_ && overlap_ != 0 && cfg_.use_fused && k > 1 && k < 32 &&
           ((gate_depths_ >> k) & 1) && has_remote_ && tfn_ == nullptr && be_->gated_supported(k);
  }

  // gated passes off for this engine (the ranks of a job agree: either every rank's passes
  // carry the exchange in-kernel or none does -- models/grayscott.py)
  void set_gated(bool on) { gate_ = on && debug_knobs().gated != 0; }
  // gated passes of depth k only (off: that depth's passes -- prepare()'s tuning of it, a
  // remainder pass -- take the stream-overlapped or plain path).  The ranks agree per depth:
  // gated_supported(k) depends on per-rank state (gate_fits, the per-depth occupancy, shared
  // landing slots), and a rank that tunes or runs a gated depth its peers do not waits for
  // exchanges that never come (models/grayscott.py _agree_gated_depths).
  void set_gated_depth(int k, bool on) {
    if (k < 0 || k >= 32) return;
    if (on) gate_depths_ |= (1u << k);
    else gate_depths_ &= ~(1u << k);
  }

  // whether full-depth passes run as a chain on two streams (advance_chained): any device
  // transport (RCCL in place or packed, IPC peer writes) -- a host callback serialises anyway
  bool chained(int k) const {
    return chain_ && overlapped(k) && tfn_ == nullptr &&
           (be_->can_exchange_inplace(plan_) || be_->has_native_transport());
  }

  // steps per pass: the fuse depth, or the measured cheaper one (prepare, single rank, when
  // the depth was left to the engine: set_auto_depth)
  int depth() const { return depth_ > 0 ? depth_ : cfg_.fuse; }
  void set_auto_depth(bool on) {
    auto_depth_ = on;
    if (!on) depth_ = 0;
  }

  // Pass-depth plan of one advance() on a single rank (no halo exchange to amortise): the
  // partition of nsteps into passes of depth 2..fuse with the lowest summed tuned pass time
  // (Backend::fused_ms, timed by prepare() on the live state), deepest passes first.  The greedy
  // min(nsteps, depth) schedule ends a 20-step window at depth 3 with a depth-2 pass for the
  // last two steps, which moves as many HBM bytes as a full pass; here every depth's measured
  // cost decides (20 = 6 x 3 + 2, 4 x 3 + 2 x 4 or 5 x 4).  Exact dynamic programme over the last
  // kPlanTail steps; before that, passes of the depth with the lowest time per step.  Empty when
  // the depths are not all timed (tuning off, a pinned configuration): the greedy schedule then.
  std::vector<int> plan_passes(int64_t nsteps) const {
    if (!planner_ || !auto_depth_ || has_remote_ || !cfg_.use_fused || cfg_.fuse < 3 || nsteps < 2)
      return {};
    double cost[8] = {0.0};
    const int kmax = cfg_.fuse < 7 ? cfg_.fuse : 7;
    for (int k = 2; k <= kmax; ++k) cost[k] = be_->fused_ms(k);
    // a first pass of depth parity pp reads the other buffer next at the time parity its outer
    // ghosts already hold (ensure_bc); unknown ghosts need a refresh whatever the plan
    const int by = bc_parity_[1 - cur_];
    const int pp = by >= 0 ? by ^ (int)(t_ & 1) : -1;
    std::vector<int> plan = plan_depths(cost, kmax, nsteps,
                                         cfg_.g.periodic || !debug_knobs().plan_fill ? 0.0 : fill_ms_, pp);
    if (debug_knobs().plan_order == 1) std::reverse(plan.begin(), plan.end());
    return plan;
  }
  // planner off (tests, A/B): the greedy min(nsteps, depth) schedule
  void set_plan(bool on) { planner_ = on; }
  // milliseconds of one outer-ghost refresh as timed by prepare() (0: periodic or not timed)
  double fill_ms() const { return fill_ms_; }

  void advance(int64_t nsteps) {
    const std::vector<int> plan = plan_passes(nsteps);
    if (!plan.empty()) {
      for (int k : plan) advance_depth(k, k);
    } else {
      advance_depth(nsteps, depth());
    }
    // the state at t_ is whole, outer ghosts included: the refresh its last pass made
    // necessary belongs to this call, not to the next one (a no-op if the parity holds)
    if (nsteps > 0) ensure_bc(cur_, t_);
  }

 private:
  void advance_depth(int64_t nsteps, const int kmax) {
    while (nsteps > 0) {
      const int k = (int)(nsteps < kmax ? nsteps : kmax);
      const int oth = 1 - cur_;
      if (nsteps >= (int64_t)k && gated(k)) {  // (its passes are counted inside)
        const int64_t npass = nsteps / k;
        advance_gated(k, npass);
        nsteps -= npass * k;
        continue;
      }
      if (nsteps >= 2 * (int64_t)k && chained(k)) {  // (its passes are counted inside)
        const int64_t npass = nsteps / k;
        advance_chained(k, npass);
        nsteps -= npass * k;
        continue;
      }
      plog_.begin_pass(k);
      if (overlapped(k)) {
        // One overlapped pass: the inner part (overlap_split) needs no halo, so it runs on
        // the compute stream while the exchange is in flight on the comm stream; the end
        // slabs (and, packed plans, the ring tiles) follow once the halos have landed.
        ensure_bc(cur_, t_);  // before the fork: the exchanged planes carry these ghosts
        be_->comm_fork();
        // the inner launch waits for a mark the comm stream records just before the exchange,
        // so RCCL's kernel reaches the GPU first (see advance_chained)
        be_->mark(3, true);
        be_->comm_select(true);
        exchange_start();
        be_->comm_select(false);
        be_->wait_mark(3, false);
        const Split sp = overlap_split(k);
        {
          TraceRange tr("gs.fused_inner");
          inner_run(cur_, oth, k, t_, sp);
        }
        be_->comm_select(true);
        exchange_finish(true);
        be_->comm_select(false);
        be_->comm_join();  // the compute stream sees the landed halos
        {
          TraceRange tr("gs.fused_shell");
          shell_run(cur_, oth, k, t_, sp);
        }
        cur_ = oth;
        t_ += k;
        nsteps -= k;
        continue;
      }
      exchange();
      if (k > 1 && cfg_.use_fused) {
        ensure_bc(cur_, t_);
        TraceRange tr("gs.fused");
        pm(kPhFused, true);
        const bool done = be_->fused(cur_, oth, k, t_);
        pm(kPhFused, false);
        if (done) {
          cur_ = oth;
          t_ += k;
          nsteps -= k;
          continue;
        }
      }
      for (int s = 0; s < k; ++s) {
        ensure_bc(cur_, t_);
        const Box r = pass_region(cfg_.g, cfg_.nbr, k, s);
        TraceRange tr("gs.step");
        pm(kPhStep, true);
        be_->step(cur_, 1 - cur_, r, t_);
        pm(kPhStep, false);
        cur_ = 1 - cur_;
        ++t_;
      }
      nsteps -= k;
    }
  }

 private:
  // Gated passes: one fused launch per pass carries the halo exchange (gate.hpp).  Both buffers'
  // outer ghosts are set up front (their time parities stay fixed while k does), so a pass is
  // exactly one launch on the compute stream: no pack / unpack kernels, no comm stream, no
  // cross-stream event.
  void advance_gated(int k, int64_t npass) {
    ensure_bc(cur_, t_);
    ensure_bc(1 - cur_, t_ + k);
    for (int64_t p = 0; p < npass; ++p) {
      const int oth = 1 - cur_;
      plog_.begin_pass(k);
      TraceRange tr("gs.fused_gated");
      pm(kPhFused, true);
      if (!be_->fused_gated(cur_, oth, k, t_, p == 0, p + 1 == npass))
        throw std::runtime_error("gated pass: the backend refused the launch");
      pm(kPhFused, false);
      ++ncomm_;
      cur_ = oth;
      t_ += k;
    }
  }

  // Chained overlapped passes over a device transport (RCCL).  The critical chain -- halo
  // exchange of pass p, then its post-exchange launches (z end slabs, ring tiles), then the
  // exchange of pass p+1 -- stays on the comm stream with no cross-stream hop; the inner part
  // runs on the compute stream.  Ordering (S = source, D = destination buffer of pass p):
  //   comm:    exchange(S_p) -> [wait inner_{p-1}] -> shell S_p -> D_p -> mark 2
  //   compute: [wait mark 2 = shell_{p-1}] -> inner S_p -> D_p -> mark p&1
  // The shell reads S_p within k of the faces with neighbours: the halos (same stream), its
  // own previous output (same stream) and inner_{p-1}'s cells (waited); it overwrites cells
  // inner_{p-1} read.  The inner part reads S_p = shell_{p-1} + inner_{p-1} and overwrites
  // cells that shell_{p-1} read (waited).  The exchange writes only ghost cells and sends
  // (packs) cells within k of the faces -- all written by the previous shell, since inner
  // outputs are at least k away from every face with a neighbour.  Both buffers' outer ghosts
  // are set before the chain (their time parities stay fixed through it), so no fill runs
  // inside.
  //   The inner launch waits for mark 2 through a cross-stream hop while the RCCL kernel
  // follows the shell on its own stream, so RCCL's kernel reaches the GPU first.  That order
  // matters: RCCL's kernel (64 workgroups of 256 threads at 132 VGPRs on the loopback) does not
  // fit beside a fused-kernel workgroup, and started after the inner launch it waits for that
  // launch to end (93 us instead of 19).  Running the shell after inner_p instead (on either
  // stream) measured 146 us per pass vs 136 us for this schedule (512 x 512 x 64, k = 3, RCCL
  // loopback; profiles/r2_overlap_schedules.txt).
  void advance_chained(int k, int64_t npass) {
    const Split sp = overlap_split(k);
    ensure_bc(cur_, t_);
    ensure_bc(1 - cur_, t_ + k);
    be_->comm_fork();
    for (int64_t p = 0; p < npass; ++p) {
      const int oth = 1 - cur_;
      plog_.begin_pass(k);
      be_->comm_select(true);
      exchange_start();      // in-place RCCL group, or pack + RCCL group, on the comm stream
      exchange_finish(true);  // (packed plans) unpack
      be_->comm_select(false);
      if (p > 0) be_->wait_mark(2, false);
      {
        TraceRange tr("gs.fused_inner");
        inner_run(cur_, oth, k, t_, sp);
      }
      be_->mark((int)(p & 1), false);
      if (p > 0) be_->wait_mark((int)((p - 1) & 1), true);
      {
        TraceRange tr("gs.fused_shell");
        be_->comm_select(true);
        shell_run(cur_, oth, k, t_, sp);
        be_->comm_select(false);
      }
      be_->mark(2, true);
      cur_ = oth;
      t_ += k;
    }
    be_->comm_join();
  }

  // Cell-granular split of an overlapped k-step pass.  The inner box -- planes [z0, z1), and
  // along x / y every cell at least k from a face flagged in `sides` -- is clear of every face
  // with a neighbour; a face without one (global boundary) needs no halo, so its cells join
  // the inner part.  The shell is the k-deep slab at each flagged face (bit0 -x, bit1 +x,
  // bit2 -y, bit3 +y, bit4 -z, bit5 +z).
  struct Split {
    int z0, z1, sides;
  };
  Split overlap_split(int k) const {
    const int nz = cfg_.g.nz;
    const int32_t* nb = cfg_.nbr;
    Split sp;
    sp.z0 = nb[dir_index(0, 0, -1)] >= 0 ? k : 0;
    sp.z1 = nb[dir_index(0, 0, 1)] >= 0 ? nz - k : nz;
    sp.sides = (nb[dir_index(-1, 0, 0)] >= 0 ? 1 : 0) | (nb[dir_index(1, 0, 0)] >= 0 ? 2 : 0) |
               (nb[dir_index(0, -1, 0)] >= 0 ? 4 : 0) | (nb[dir_index(0, 1, 0)] >= 0 ? 8 : 0) |
               (sp.z0 > 0 ? 16 : 0) | (sp.z1 < nz ? 32 : 0);
    return sp;
  }
  // the inner box: all x-y tiles over planes [z0, z1), outputs clipped by the x / y mask,
  // leaving workgroup slots free for the communication kernels that run beside it
  void inner_run(int src, int dst, int k, int64_t t, const Split& sp) {
    if (sp.z1 <= sp.z0) return;
    pm(kPhInner, true);
    be_->fused_runs(src, dst, k, t, sp.z0, sp.z1 - sp.z0, 0, 0, true, sp.sides & 15);
    pm(kPhInner, false);
  }
  // the shell: the k-deep face slabs, after the halos have landed
  void shell_run(int src, int dst, int k, int64_t t, const Split& sp) {
    if (!sp.sides) return;
    pm(kPhShell, true);
    if (!be_->shell(src, dst, k, t, sp.sides))
      throw std::runtime_error("overlapped pass: the backend has no shell kernel for this depth");
    pm(kPhShell, false);
  }

  // a phase timestamp (profiling window only)
  void pm(int phase, bool begin) {
    if (!plog_.on) return;
    const int slot = plog_.next(phase, begin);
    if (slot >= 0) be_->prof_mark(slot, phase);
  }

  EngineConfig cfg_;
  Backend* be_;
  HaloPlan plan_;
  bool has_nbr_ = false;
  bool has_remote_ = false;
  int overlap_ = -1;
  int depth_ = 0;  // measured steps per pass (0: cfg_.fuse)
  bool auto_depth_ = false;
  bool loopback_ = false;
  // debug knob overlap_chain = 0 (tests): overlapped passes one by one (gs/debug.h)
  bool chain_ = debug_knobs().overlap_chain != 0;
  // debug knob gated = 0 (tests, A/B): no gated passes (gs/debug.h)
  bool gate_ = debug_knobs().gated != 0;
  uint32_t gate_depths_ = 0xffffffffu;  // set_gated_depth
  bool planner_ = true;  // plan_passes (set_plan)
  double fill_ms_ = 0.0;  // prepare(): one ensure_bc refresh (the planner's parity-switch cost)
  enum { kNone, kUnpack, kCallback };
  int xpending_ = kNone;
  int cur_ = 0;
  int64_t t_ = 0;
  int bc_parity_[2];
  TransportFn tfn_ = nullptr;
  void* tuser_ = nullptr;
  int64_t ncomm_ = 0;
  PhaseLog plog_;
};

}  // namespace gs
