// SPDX-License-Identifier: MIT
// gfx950 (MI355X, CDNA4) backend: hand-written HIP kernels + RCCL halo transport.
//
// Reference kernels replaced: K2/K3/K4 calculate_kernel! (ext/CUDAExt.jl:
// 135-161, ext/AMDGPUExt.jl:179-210, Simulation_KA.jl:177-203), K6-K9 populate!/fills,
// K10 device RNG, K12/K13 MPI face datatypes + Sendrecv!, K14 get_fields.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "gs/capi_impl.h"
#include "kernels.hpp"

// The fused kernel and the shell kernels are instantiated in their own translation units
// (csrc/hip/inst/*.hip), compiled in parallel.
namespace gsk {
extern template bool launch_fused<float>(const Vec2<float>::type*, Vec2<float>::type*, const Geom&,
                                         const gs::Params&, int, int64_t, hipStream_t, int, int,
                                         int, int, int, int, int, int, bool, const GateLaunch*);
extern template bool launch_fused<double>(const Vec2<double>::type*, Vec2<double>::type*,
                                          const Geom&, const gs::Params&, int, int64_t,
                                          hipStream_t, int, int, int, int, int, int, int, int, bool,
                                          const GateLaunch*);
extern template int fused_gated_occupancy<float>(int, int, bool);
extern template int fused_gated_occupancy<double>(int, int, bool);
extern template bool launch_shell<float>(const void*, void*, const Geom&, const gs::Params&, int,
                                         int64_t, int, int, hipStream_t);
extern template bool launch_shell<double>(const void*, void*, const Geom&, const gs::Params&, int,
                                          int64_t, int, int, hipStream_t);
}  // namespace gsk

#define HIP_CHECK(expr)                                                                   \
  do {                                                                                    \
    hipError_t _e = (expr);                                                               \
    if (_e != hipSuccess)                                                                 \
      throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(_e) + " at " + \
                               __FILE__ + ":" + std::to_string(__LINE__) + " (" #expr ")"); \
  } while (0)

#define NCCL_CHECK(expr)                                                                  \
  do {                                                                                    \
    ncclResult_t _r = (expr);                                                             \
    if (_r != ncclSuccess && _r != ncclInProgress)                                        \
      throw std::runtime_error(std::string("RCCL error: ") + ncclGetErrorString(_r) +      \
                               " (" #expr ")");                                           \
  } while (0)

namespace {

// an IPC export: the landing-buffer and flag handles, then the device's PCI bus id
constexpr int kIpcPciBytes = 32;
constexpr int kIpcHandleBytes = 2 * (int)sizeof(hipIpcMemHandle_t) + kIpcPciBytes;
constexpr int kIpcTabStride = 2 + 3 * gs::kMaxMsgs;

using gs::Box;
using gs::Geom;

// One RCCL communicator per process, reused by every engine over the same (nranks, rank):
// data-path tuning builds a dozen engines in sequence, and each communicator set-up costs
// seconds at 8 ranks.  Every rank makes the same sequence of engines, so all reuse together.
struct SharedComm {
  ncclComm_t comm = nullptr;
  int nranks = -1, rank = -1;
};
SharedComm& shared_comm() {
  static SharedComm c;
  return c;
}

// set once a configuration is chosen explicitly through gs_fused_select / gs_fused_sched
bool& fused_pinned() {
  static bool v = false;
  return v;
}

template <typename T>
class HipBackend final : public gs::Backend {
 public:
  using V2 = typename gsk::Vec2<T>::type;

  // the launch being tuned: z-runs, store mask and the workgroup slots it leaves free
  // (whole interior: zlen0 < 0)
  struct Part {
    int zlo0, zlen0, zlo1, zlen1, mask, reserve;
    bool operator==(const Part& o) const {
      return zlo0 == o.zlo0 && zlen0 == o.zlen0 && zlo1 == o.zlo1 && zlen1 == o.zlen1 &&
             mask == o.mask && reserve == o.reserve;
    }
  };
  // tuned shapes of the overlapped passes' post-exchange parts (one entry per launch shape)
  struct PartChoice {
    int n;
    Part pt;
    int cfg, sched;
  };
  // the shell variant chosen per (depth, sides) (see shell())
  struct ShellChoice {
    int n, sides, variant;
    float ms[2];
  };

  HipBackend(const Geom& g, const gs::Params& p, void* b0, void* b1, void* send, void* recv,
             hipStream_t stream)
      : g_(g), p_(p), stream_(stream) {
    buf_[0] = (V2*)b0;
    buf_[1] = (V2*)b1;
    send_ = (V2*)send;
    recv_ = (V2*)recv;
    if (!b0 || !b1) throw std::runtime_error("null field buffer");
    HIP_CHECK(hipGetDevice(&dev_));
    HIP_CHECK(hipMalloc(&ws_, sizeof(double) * 6 * kStatBlocks));
    HIP_CHECK(hipEventCreateWithFlags(&ev_, hipEventDisableTiming));
    // cross-stream ordering events (a device-scope release measured the same,
    // profiles/r2_xstream_event.txt, so the default flags stay)
    HIP_CHECK(hipEventCreateWithFlags(&ev_fork_, hipEventDisableTiming));
    HIP_CHECK(hipEventCreateWithFlags(&ev_join_, hipEventDisableTiming));
    for (hipEvent_t& e : marks_) HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    // halo traffic on its own high-priority stream so it overlaps the inner-plane kernel
    int lo = 0, hi = 0;
    HIP_CHECK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    HIP_CHECK(hipStreamCreateWithPriority(&comm_stream_, hipStreamNonBlocking, hi));
    xs_ = stream_;
  }
  ~HipBackend() override {
    ipc_release();
    gate_release();
    if (comm_ && comm_ != shared_comm().comm) ncclCommDestroy(comm_);
    if (ws_) (void)hipFree(ws_);
    if (ev_) (void)hipEventDestroy(ev_);
    if (ev_fork_) (void)hipEventDestroy(ev_fork_);
    if (ev_join_) (void)hipEventDestroy(ev_join_);
    for (hipEvent_t e : marks_)
      if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : prof_ev_) (void)hipEventDestroy(e);
    if (comm_stream_) (void)hipStreamDestroy(comm_stream_);
  }

  void fill_box(int b, const Box& bx, double u, double v) override {
    if (gs::box_cells(bx) == 0) return;
    gsk::launch_fill<T>(buf_[b], g_, bx, (T)u, (T)v, stream_);
    HIP_CHECK(hipGetLastError());
  }

  void fill_boxes(int b, const Box* boxes, int n, double u, double v) override {
    if (n > 6) {
      gs::Backend::fill_boxes(b, boxes, n, u, v);
      return;
    }
    gsk::launch_fill_boxes<T>(buf_[b], g_, boxes, n, (T)u, (T)v, stream_);
    HIP_CHECK(hipGetLastError());
  }

  void seed(int b) override {
    gsk::launch_seed<T>(buf_[b], g_, stream_);
    HIP_CHECK(hipGetLastError());
  }

  void step(int src, int dst, const Box& R, int64_t t) override {
    if (gs::box_cells(R) == 0) return;
    gsk::launch_step1<T>(buf_[src], buf_[dst], g_, p_, R, t, stream_);
    HIP_CHECK(hipGetLastError());
  }

  bool fused(int src, int dst, int n, int64_t t) override {
    if (n < 2 || n > kMaxDepth) return false;
    if (!tuned_[n]) autotune(src, dst, n, t);
    // an explicit gs_fused_select / gs_fused_sched overrides the tuned choice at any time
    const bool pin = fused_pinned();
    const bool ok = gsk::launch_fused<T>(buf_[src], buf_[dst], g_, p_, n, t, stream_,
                                         pin ? -1 : cfg_[n], pin ? -1 : sched_[n], 0, -1, 0, 0,
                                         0, 0, /*allow_block=*/true);
    if (ok) HIP_CHECK(hipGetLastError());
    return ok;
  }

  bool fused_supported(int n) const override { return gsk::fused_supported(g_, n); }

  bool fused_runs(int src, int dst, int n, int64_t t, int zlo0, int zlen0, int zlo1,
                  int zlen1, bool leave_room, int mask) override {
    if (!gsk::fused_supported(g_, n)) return false;
    if (!tuned_[n]) autotune(src, dst, n, t);
    const bool pin = fused_pinned();
    // launched on the selected stream (comm_select).  Every part of an overlapped pass -- the
    // inner box (slots left free), the z end slabs (short, latency-bound) -- gets its own tuned
    // tile shape / schedule; the whole interior keeps the choice made for it.
    int c = cfg_[n], sc = sched_[n];
    const int reserve = leave_room ? kOverlapReserve : 0;
    const bool whole = zlo0 == 0 && zlen0 == g_.nz && zlen1 <= 0 && mask == 0 && reserve == 0;
    if (!whole && !pin) {
      const PartChoice& pc =
          part_choice(src, dst, n, t, Part{zlo0, zlen0, zlo1, zlen1, mask, reserve});
      c = pc.cfg;
      sc = pc.sched;
    }
    const bool ok = gsk::launch_fused<T>(buf_[src], buf_[dst], g_, p_, n, t, xs_,
                                         pin ? -1 : c, pin ? -1 : sc, zlo0, zlen0,
                                         zlo1, zlen1, reserve, mask);
    if (!ok) throw std::runtime_error("fused_runs: invalid z-runs or mask");
    HIP_CHECK(hipGetLastError());
    return true;
  }

  // tuned {cfg, sched} of a z-run launch (first use times the candidates)
  const PartChoice& part_choice(int src, int dst, int n, int64_t t, const Part& pt) {
    for (const PartChoice& q : parts_)
      if (q.n == n && q.pt == pt) return q;
    parts_.push_back(PartChoice{n, pt, cfg_[n], sched_[n]});
    PartChoice& pc = parts_.back();
    float ms = 0.f;
    if (!autotune_part(src, dst, n, t, pt, &pc.cfg, &pc.sched, &ms)) {
      pc.cfg = cfg_[n];
      pc.sched = sched_[n];
    }
    return pc;
  }

  // The shell of an overlapped pass (engine.h shell_run): the n-deep slabs at the faces in
  // `sides`.  Two ways, timed against each other at first use per (n, sides) and the faster
  // kept: (0) one k_slab launch for every face; (1) the z slabs as one two-run k_fused launch
  // (its own tuned tile) and the x / y slabs as a k_slab launch after it.  (Round 4 also tried
  // the two launches of (1) side by side, the z slabs on a forked side stream: 49.6 us vs 38.3
  // sequential and 26.2 for (0), one-sided 256^3 at k=3, profiles/r4_shell.txt -- removed.)
  bool shell(int src, int dst, int n, int64_t t, int sides, int variant) override {
    if (!gsk::fused_supported(g_, n) || !sides) return sides == 0;
    if (!tuned_[n]) autotune(src, dst, n, t);
    if (variant >= 0) {
      shell_variant(src, dst, n, t, sides, variant & 1);
      return true;
    }
    ShellChoice* sc = nullptr;
    for (ShellChoice& q : shells_)
      if (q.n == n && q.sides == sides) sc = &q;
    if (!sc) {
      shells_.push_back(ShellChoice{n, sides, 0, {0.f, 0.f}});
      sc = &shells_.back();
      if (sides & 48) {
        // warm both (the first k_fused z-run launch tunes its own shape), then best of 3
        hipStream_t keep = xs_;
        xs_ = stream_;
        hipEvent_t e0, e1;
        HIP_CHECK(hipEventCreate(&e0));
        HIP_CHECK(hipEventCreate(&e1));
        float best[2] = {1e30f, 1e30f};
        for (int r = 0; r < 4; ++r)
          for (int v = 0; v < 2; ++v) {
            HIP_CHECK(hipEventRecord(e0, stream_));
            shell_variant(src, dst, n, t, sides, v);
            HIP_CHECK(hipEventRecord(e1, stream_));
            HIP_CHECK(hipEventSynchronize(e1));
            float ms = 0.f;
            HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
            if (r > 0 && ms < best[v]) best[v] = ms;
          }
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
        xs_ = keep;
        sc->variant = best[1] < best[0] ? 1 : 0;
        sc->ms[0] = best[0];
        sc->ms[1] = best[1];
      }
    }
    shell_variant(src, dst, n, t, sides, sc->variant);
    return true;
  }

  void shell_variant(int src, int dst, int n, int64_t t, int sides, int variant) {
    int slab_sides = sides;
    if (variant == 1 && (sides & 48)) {
      const int la = (sides & 16) ? n : 0, lb = (sides & 32) ? n : 0;
      if (la > 0) fused_runs(src, dst, n, t, 0, la, g_.nz - lb, lb, false, 0);
      else fused_runs(src, dst, n, t, g_.nz - lb, lb, 0, 0, false, 0);
      slab_sides = sides & 15;
    }
    if (slab_sides) {
      if (!gsk::launch_shell<T>(buf_[src], buf_[dst], g_, p_, n, t, slab_sides, num_cus(), xs_))
        throw std::runtime_error("shell: unsupported sub-domain (needs >= 2n cells per axis)");
      HIP_CHECK(hipGetLastError());
    }
  }

  int num_cus() const {
    static int cus = 0;
    if (!cus && (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev_) !=
                     hipSuccess || cus < 1))
      cus = 256;
    return cus;
  }

  // Per-phase timing (gs/phase.h): one timing event per timestamp, recorded on the stream the
  // phase is issued to -- halo and overlapped-pass phases follow comm_select, the rest (the
  // whole-interior kernel, single steps, boundary fills, the window's stamps) run on the
  // compute stream.  Events are created once and reused by later windows.
  void prof_reserve(int n) override {
    while ((int)prof_ev_.size() < n) {
      hipEvent_t e;
      HIP_CHECK(hipEventCreate(&e));
      prof_ev_.push_back(e);
    }
    prof_n_ = n;
  }
  void prof_mark(int slot, int phase) override {
    if (slot < 0 || slot >= prof_n_) return;
    const bool selectable = phase >= gs::kPhPack && phase <= gs::kPhShell;
    HIP_CHECK(hipEventRecord(prof_ev_[slot], selectable ? xs_ : stream_));
  }
  void prof_times(double* us, int n) override {
    for (int i = 0; i < n; ++i) {
      float ms = 0.f;
      if (i > 0 && i < prof_n_) HIP_CHECK(hipEventElapsedTime(&ms, prof_ev_[0], prof_ev_[i]));
      us[i] = 1e3 * (double)ms;
    }
  }

  bool has_comm_stream() const override { return comm_stream_ != nullptr; }
  hipStream_t main_stream() const { return stream_; }
  void comm_fork() override {
    HIP_CHECK(hipEventRecord(ev_fork_, stream_));
    HIP_CHECK(hipStreamWaitEvent(comm_stream_, ev_fork_, 0));
  }
  void comm_join() override {
    HIP_CHECK(hipEventRecord(ev_join_, comm_stream_));
    HIP_CHECK(hipStreamWaitEvent(stream_, ev_join_, 0));
  }
  void comm_select(bool on) override { xs_ = on ? comm_stream_ : stream_; }
  void mark(int which, bool on_comm) override {
    HIP_CHECK(hipEventRecord(marks_[which & 3], on_comm ? comm_stream_ : stream_));
  }
  void wait_mark(int which, bool on_comm) override {
    HIP_CHECK(hipStreamWaitEvent(on_comm ? comm_stream_ : stream_, marks_[which & 3], 0));
  }
  bool has_native_transport() const override { return comm_ != nullptr || ipc_; }
  bool can_exchange_inplace(const gs::HaloPlan& p) const override {
    if (!comm_ || ipc_ || !p.zplanes || inplace_off_) return false;
    if (!loopback_)
      for (int i = 0; i < p.nrecv; ++i)
        if (p.recv[i].peer == rank_) return false;
    return true;
  }

  // zplanes plan: every message is a contiguous run of storage planes of buffer b, so RCCL
  // sends and receives them in place.  Same message order as the packed path (sends ascend
  // in direction, receives descend), which keeps two messages to one peer matched.
  bool native_exchange_inplace(int b, const gs::HaloPlan& p) override {
    if (!comm_ || ipc_ || !p.zplanes || inplace_off_) return false;
    if (!loopback_)
      for (int i = 0; i < p.nrecv; ++i)
        if (p.recv[i].peer == rank_) return false;
    NCCL_CHECK(ncclGroupStart());
    for (int i = 0; i < p.nsend; ++i) {
      const gs::HaloMsg& m = p.send[i];
      NCCL_CHECK(ncclSend(buf_[b] + gs::box_start(g_, m.box),
                          (size_t)gs::box_cells(m.box) * sizeof(V2), ncclUint8, m.peer, comm_, xs_));
    }
    for (int i = 0; i < p.nrecv; ++i) {
      const gs::HaloMsg& m = p.recv[i];
      NCCL_CHECK(ncclRecv(buf_[b] + gs::box_start(g_, m.box),
                          (size_t)gs::box_cells(m.box) * sizeof(V2), ncclUint8, m.peer, comm_, xs_));
    }
    group_end();
    return true;
  }

  void prepare_fused(int src, int dst, int n, int64_t t) override {
    if (n >= 2 && n <= kMaxDepth && !tuned_[n]) autotune(src, dst, n, t);
  }

  // On-device autotuning of the fused kernel's tile shape and work schedule.  The kernel only
  // reads `src` and writes `dst`, so every candidate can be timed on the live buffers without
  // changing the simulation state, and all candidates produce bit-identical results.
  // Disabled by GS_AUTOTUNE=0 or by an explicit GS_FUSED_CFG / GS_FUSED_SCHED.
  static bool autotune_enabled() {
    const char* e = getenv("GS_AUTOTUNE");
    return !((e && atoi(e) == 0) || getenv("GS_FUSED_CFG") || getenv("GS_FUSED_SCHED") ||
             fused_pinned());
  }
  // best {cfg, sched} for one launch shape; false if tuning is disabled / unsupported
  // fixed_cfg >= 0 keeps the tile shape and tunes the schedule only (a ring launch must use
  // the tile grid of the inner launch it complements)
  // Process-wide cache of tuning results per launch shape: data-path tuning (and the golden
  // checks) build many engines over the same sub-domain shape; each would re-time the same
  // candidates.  The key holds everything a launch's cost depends on: the local and global
  // extents (edge tiles, the Philox counter width), the launch part and the workgroup slots
  // left free beside it.
  struct TuneKey {
    int tsize, nx, ny, nz, H, periodic, noise, n, fixed, q32, reserve;
    int64_t Lx, Ly, Lz;
    Part pt;
    bool operator==(const TuneKey& o) const {
      return tsize == o.tsize && nx == o.nx && ny == o.ny && nz == o.nz && H == o.H &&
             periodic == o.periodic && noise == o.noise && n == o.n && fixed == o.fixed &&
             q32 == o.q32 && reserve == o.reserve && Lx == o.Lx && Ly == o.Ly && Lz == o.Lz &&
             pt == o.pt;
    }
  };
  struct TuneVal {
    int cfg, sched;
    float ms;
  };
  static std::vector<std::pair<TuneKey, TuneVal>>& tune_cache() {
    static std::vector<std::pair<TuneKey, TuneVal>> c;
    return c;
  }
  bool autotune_part(int src, int dst, int n, int64_t t, const Part& pt, int* cfg, int* sched,
                     float* ms_best, int fixed_cfg = -1) {
    if (!autotune_enabled()) return false;
    const TuneKey key{(int)sizeof(T), g_.nx, g_.ny, g_.nz, g_.H, g_.periodic,
                      p_.noise != 0.0 ? 1 : 0, n, fixed_cfg, gsk::philox_q32(g_) ? 1 : 0,
                      pt.reserve, g_.Lx, g_.Ly, g_.Lz, pt};
    for (const auto& kv : tune_cache())
      if (kv.first == key) {
        *cfg = kv.second.cfg;
        *sched = kv.second.sched;
        *ms_best = kv.second.ms;
        return true;
      }
    if (!autotune_run(src, dst, n, t, pt, cfg, sched, ms_best, fixed_cfg)) return false;
    tune_cache().push_back({key, TuneVal{*cfg, *sched, *ms_best}});
    return true;
  }
  bool autotune_run(int src, int dst, int n, int64_t t, const Part& pt, int* cfg, int* sched,
                    float* ms_best, int fixed_cfg) {
    struct Cand { int cfg, sched; };
    std::vector<Cand> cands;
    // tile variants are instantiated for the production path only (fused.hpp run_fused_cfg)
    const bool variants = !g_.periodic && p_.noise != 0.0 && gsk::philox_q32(g_);
    std::vector<int> cfgs;
    bool blk_ok = false;  // the block kernel is a candidate (whole-interior launch it supports)
    if (fixed_cfg >= 0) {
      cfgs = {fixed_cfg};
    } else if (!variants) {
      cfgs = {0};
    } else {
      int nt = 0;
      const gsk::FusedCfgEntry* tab = gsk::fused_cfg_table(&nt);
      const int dflt = sizeof(T) == 4 ? gsk::fused_cfg_lookup("4x12:2s") : gsk::fused_cfg_lookup("4x8:1s");
      // the small-grid block kernel (k_block) serves whole-interior launches it supports only
      gsk::FusedArgs fa{};
      fa.g = g_;
      fa.q32 = gsk::philox_q32(g_) ? 1 : 0;
      fa.zlen[0] = pt.zlen0 < 0 ? g_.nz : pt.zlen0;
      fa.zlo[0] = pt.zlo0;
      fa.zlen[1] = pt.zlen1;
      fa.mx1 = g_.nx;
      fa.my1 = g_.ny;
      fa.reserve = pt.reserve;
      fa.allow_block = 1;
      blk_ok = pt.mask == 0 && gsk::block_supported(fa);
      for (int i = 0; i < nt; ++i)
        if ((sizeof(T) == 4 ? tab[i].f32 : tab[i].f64) && i != dflt && !strstr(tab[i].name, "-abl") &&
            (blk_ok || !gsk::fused_cfg_is_block(i)) &&
            gsk::block_cfg_fits(i, n, (int)sizeof(V2)) && gsk::fused_cfg_applies(i, g_, n) &&
            gsk::lr_cfg_fits(i, n) &&
            // T = 4 runs the LDS-ring shapes only (0 is its default 4x12:1sl, so 29 repeats it)
            (n < 4 || i == 0 || (gsk::fused_cfg_is_lr(i) && i != 29)))
          cfgs.push_back(i);
    }
    const int nsched = pt.zlen1 > 0 ? 1 : 3;  // two z-runs always use schedule 0
    for (int c : cfgs)  // (k_block has no work schedule)
      for (int sc = 0; sc < (gsk::fused_cfg_is_block(c) ? 1 : nsched); ++sc) cands.push_back({c, sc});
    auto launch = [&](const Cand& c) {
      return gsk::launch_fused<T>(buf_[src], buf_[dst], g_, p_, n, t, stream_, c.cfg, c.sched,
                                  pt.zlo0, pt.zlen0, pt.zlo1, pt.zlen1, pt.reserve, pt.mask,
                                  blk_ok);
    };
    // interleaved rounds (box-to-box and launch-to-launch jitter is several %): first launch
    // of each candidate is a warm-up, then the best of kRounds timed launches decides
    constexpr int kRounds = 3;
    std::vector<float> tbest(cands.size(), 1e30f);
    for (size_t i = 0; i < cands.size(); ++i)
      if (!launch(cands[i])) return false;
    hipEvent_t e0, e1;
    HIP_CHECK(hipEventCreate(&e0));
    HIP_CHECK(hipEventCreate(&e1));
    for (int r = 0; r < kRounds; ++r)
      for (size_t i = 0; i < cands.size(); ++i) {
        HIP_CHECK(hipEventRecord(e0, stream_));
        launch(cands[i]);
        HIP_CHECK(hipEventRecord(e1, stream_));
        HIP_CHECK(hipEventSynchronize(e1));
        HIP_CHECK(hipGetLastError());
        float ms = 0.f;
        HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
        if (ms < tbest[i]) tbest[i] = ms;
      }
    float best = 1e30f;
    for (size_t i = 0; i < cands.size(); ++i)
      if (tbest[i] < best) {
        best = tbest[i];
        *cfg = cands[i].cfg;
        *sched = cands[i].sched;
      }
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    *ms_best = best;
    return true;
  }

  void autotune(int src, int dst, int n, int64_t t) {
    tuned_[n] = true;
    const Part whole{0, -1, 0, 0, 0, 0};
    float ms = 0.f;
    if (autotune_part(src, dst, n, t, whole, &cfg_[n], &sched_[n], &ms)) tuned_ms_[n] = ms;
  }

  double fused_ms(int n) const override { return n >= 2 && n <= kMaxDepth ? tuned_ms_[n] : 0.0; }

  void fused_choice(int n, int* cfg, int* sched, float* ms) const {
    *cfg = cfg_[n];
    *sched = sched_[n];
    *ms = tuned_ms_[n];
  }

  void pack(int b, const gs::HaloPlan& p) override {
    if (p.nsend == 0) return;
    if (ipc_) {
      ipc_pack(b, p);
      return;
    }
    gsk::launch_pack<T, true>(buf_[b], send_, g_, p.send, p.nsend, xs_);
    HIP_CHECK(hipGetLastError());
  }
  void unpack(int b, const gs::HaloPlan& p) override {
    if (p.nrecv == 0) return;
    if (ipc_) {
      ipc_unpack(b, p);
      return;
    }
    gsk::launch_pack<T, false>(buf_[b], recv_, g_, p.recv, p.nrecv, xs_);
    HIP_CHECK(hipGetLastError());
  }

  // ---------------------------------------------------------------------------------------
  // IPC peer-write transport (transport = "ipc").  Each rank exports a landing buffer (two
  // slots of its plan's receive layout) and a flag array, both uncached device memory, through
  // hipIpcGetMemHandle, plus its device's PCI bus id; every rank maps its neighbours'
  // (hipIpcOpenMemHandle) after checking that its device can reach theirs
  // (hipDeviceCanAccessPeer).  Exchange n:
  //   pack:   one launch that stores every message straight into the receiving peer's
  //           landing slot n&1 (over xGMI); each wave waits for its stores to be acknowledged
  //           before it retires (the landing buffer is uncached: no L2 line holds them)
  //   unpack: one single-wave launch: ready_P[me] = n for each send peer P (system-scope
  //           release), then wait for ready[P] >= n for each receive peer P (system-scope
  //           acquire) -> unpack from my slot n&1
  // Slot reuse needs no flag of its own because the neighbour relation is symmetric (send
  // peers = receive peers, always so for a Cartesian grid; checked in ipc_connect): P's
  // ready(n-1) follows P's unpack of exchange n-2 in P's stream order, and this rank waits for
  // ready(n-1) (its unpack n-1) before its pack n, so P's slot n&1 is free by then.
  // All of it is stream-ordered device work on the halo stream (no host handshake), so the
  // scheduler's free-running passes and the comm/compute overlap work unchanged: the flags
  // are monotonic sequence numbers, which a consumer can wait on ahead of time, unlike
  // events.  Uncached memory keeps the landing data and the flags coherent between the GPUs
  // (no stale L2 lines on either side).  Messages to this rank itself (periodic wrap) go
  // through the local send / receive buffers and self copies, unless loopback is on, in
  // which case they take the landing-buffer path too (single-GPU test of the protocol).
  // A wait that times out sets a host-mapped word (the watchdog, wait_all, raises) and a
  // device word that makes every later unpack write NaN ghosts instead of stale landing data.
  void ipc_export(const gs::HaloPlan& p, int nranks, int rank, char* out) {
    ipc_release();
    rank_ = rank;
    ipc_nranks_ = nranks;
    landing_cells_ = std::max<int64_t>(p.recv_cells, 1);
    HIP_CHECK(hipExtMallocWithFlags((void**)&landing_, 2 * landing_cells_ * sizeof(V2),
                                    hipDeviceMallocUncached));
    // flags_[0, nranks): sequence flags; [nranks, 2 nranks): publication stamps (gate.hpp:
    // emulated carried exchanges)
    HIP_CHECK(hipExtMallocWithFlags((void**)&flags_, 2 * (size_t)nranks * sizeof(uint64_t),
                                    hipDeviceMallocUncached));
    HIP_CHECK(hipMemset(flags_, 0, 2 * (size_t)nranks * sizeof(uint64_t)));
    HIP_CHECK(hipMalloc((void**)&ipc_dflag_, sizeof(int)));
    HIP_CHECK(hipMemset(ipc_dflag_, 0, sizeof(int)));
    HIP_CHECK(hipDeviceSynchronize());
    HIP_CHECK(hipHostMalloc((void**)&ipc_err_, sizeof(int), hipHostMallocMapped));
    *ipc_err_ = 0;
    HIP_CHECK(hipHostGetDevicePointer((void**)&ipc_err_dev_, ipc_err_, 0));
    hipIpcMemHandle_t h[2];
    HIP_CHECK(hipIpcGetMemHandle(&h[0], landing_));
    HIP_CHECK(hipIpcGetMemHandle(&h[1], flags_));
    memset(out, 0, kIpcHandleBytes);
    memcpy(out, h, sizeof(h));
    HIP_CHECK(hipDeviceGetPCIBusId(out + sizeof(h), kIpcPciBytes - 1, dev_));
    int khz = 0;
    HIP_CHECK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev_));
    const double to = gs::comm_timeout_s();
    ipc_ticks_ = (uint64_t)(std::max(1.0, to) * (double)std::max(khz, 1) * 1000.0);
    const double emu = gs::debug_knobs().ipc_emulate_us;  // modelling only (gs/debug.h)
    ipc_emulate_ticks_ = (uint64_t)(std::max(0.0, emu) * (double)std::max(khz, 1) / 1000.0);
    xn_ = 0;
  }

  // handles: nranks x kIpcHandleBytes (every rank's ipc_export output); tabs: per rank
  // kIpcTabStride int64 = {nrecv, recv_cells, nrecv x (peer, offset, cells)} of its plan
  void ipc_connect(const gs::HaloPlan& p, const char* handles, const int64_t* tabs) {
    if (!landing_) throw std::runtime_error("ipc_connect before ipc_export");
    auto peer_index = [&](int r) -> int {
      for (size_t i = 0; i < peers_.size(); ++i)
        if (peers_[i].rank == r) return (int)i;
      if (r < 0 || r >= ipc_nranks_) throw std::runtime_error("ipc: peer rank out of range");
      PeerMap pm{r, nullptr, nullptr, std::max<int64_t>(tabs[(int64_t)r * kIpcTabStride + 1], 1),
                 false, dev_, 1};
      if (r == rank_) {
        pm.landing = landing_;
        pm.flags = flags_;
      } else {
        const char* hr = handles + (size_t)r * kIpcHandleBytes;
        char pci[kIpcPciBytes];
        memcpy(pci, hr + 2 * sizeof(hipIpcMemHandle_t), kIpcPciBytes);
        pci[kIpcPciBytes - 1] = 0;
        // the peer's device as this process numbers it (all of the node's GPUs are visible
        // to every rank); -1: not visible here, then the mapping itself is the check
        int pdev = -1;
        if (pci[0] && hipDeviceGetByPCIBusId(&pdev, pci) != hipSuccess) pdev = -1;
        pm.device = pdev;
        pm.p2p = pdev == dev_ ? 1 : -1;
        if (pdev >= 0 && pdev != dev_) {
          int can = 0;
          HIP_CHECK(hipDeviceCanAccessPeer(&can, dev_, pdev));
          if (!can)
            throw std::runtime_error("ipc: device " + std::to_string(dev_) +
                                     " cannot access peer device " + std::to_string(pdev) +
                                     " (rank " + std::to_string(r) + ", " + pci + ")");
          pm.p2p = 1;
        }
        hipIpcMemHandle_t h[2];
        memcpy(h, hr, sizeof(h));
        HIP_CHECK(hipIpcOpenMemHandle((void**)&pm.landing, h[0], hipIpcMemLazyEnablePeerAccess));
        HIP_CHECK(hipIpcOpenMemHandle((void**)&pm.flags, h[1], hipIpcMemLazyEnablePeerAccess));
        pm.opened = true;
      }
      peers_.push_back(pm);
      return (int)peers_.size() - 1;
    };
    send_peers_.clear();
    recv_peers_.clear();
    for (int i = 0; i < p.nsend; ++i) {
      const gs::HaloMsg& m = p.send[i];
      send_peer_[i] = -1;
      if (m.peer == rank_ && !loopback_) continue;  // self copy through send_ / recv_
      const int idx = peer_index(m.peer);
      send_peer_[i] = idx;
      if (std::find(send_peers_.begin(), send_peers_.end(), idx) == send_peers_.end())
        send_peers_.push_back(idx);
      if (m.peer == rank_ && gs::debug_knobs().ipc_pair_same_dir) {
        // modelling only (debug knob): a loopback message lands in the ghost box of its OWN
        // direction -- one-sided neighbour sets on one rank (timing; the values are no wrap)
        int64_t off = -1;
        for (int j = 0; j < p.nrecv; ++j)
          if (p.recv[j].peer == rank_ && p.recv[j].dir == m.dir &&
              gs::box_cells(p.recv[j].box) == gs::box_cells(m.box))
            off = p.recv[j].offset;
        if (off < 0) throw std::runtime_error("ipc: no same-direction receive (ipc_pair_same_dir)");
        send_off_[i] = off;
        continue;
      }
      // the k-th send to P matches the k-th receive at P from this rank (make_halo_plan)
      int k = 0;
      for (int j = 0; j < i; ++j) k += p.send[j].peer == m.peer ? 1 : 0;
      const int64_t* t = tabs + (int64_t)m.peer * kIpcTabStride;
      int64_t off = -1;
      for (int j = 0, seen = 0; j < (int)t[0]; ++j) {
        const int64_t* e = t + 2 + 3 * j;
        if (e[0] != rank_) continue;
        if (seen++ == k) {
          if (e[2] != gs::box_cells(m.box))
            throw std::runtime_error("ipc: message sizes of a send / receive pair differ");
          off = e[1];
          break;
        }
      }
      if (off < 0) throw std::runtime_error("ipc: peer has no matching receive");
      send_off_[i] = off;
    }
    for (int i = 0; i < p.nrecv; ++i) {
      const gs::HaloMsg& m = p.recv[i];
      recv_peer_[i] = -1;
      if (m.peer == rank_ && !loopback_) continue;
      const int idx = peer_index(m.peer);
      recv_peer_[i] = idx;
      if (std::find(recv_peers_.begin(), recv_peers_.end(), idx) == recv_peers_.end())
        recv_peers_.push_back(idx);
    }
    std::vector<int> a = send_peers_, b = recv_peers_;
    std::sort(a.begin(), a.end());
    std::sort(b.begin(), b.end());
    if (a != b)
      throw std::runtime_error("ipc: the transport needs symmetric neighbours (send peers = "
                               "receive peers), as every Cartesian decomposition has");
    ipc_ = true;
    // the gated pass (gate.hpp) packs every message straight into a landing slot: it needs a
    // landing-buffer route for each (no local self copies: a periodic wrap onto this rank
    // without loopback goes through the stream path)
    gplan_ = p;
    gate_plan_ok_ = p.nsend > 0 && p.nrecv > 0;
    for (int i = 0; i < p.nsend; ++i) gate_plan_ok_ = gate_plan_ok_ && send_peer_[i] >= 0;
    for (int i = 0; i < p.nrecv; ++i) gate_plan_ok_ = gate_plan_ok_ && recv_peer_[i] >= 0;
    // peer processes on this same GPU (tests): their gated launches compete for its slots
    gate_sharers_ = 0;
    for (const PeerMap& pm : peers_) gate_sharers_ += (pm.rank != rank_ && pm.device == dev_) ? 1 : 0;
    for (int& f : gate_fit_) f = -1;
    gate_release();
  }

  void ipc_pack(int b, const gs::HaloPlan& p) {
    ++xn_;
    const int64_t slot = (int64_t)(xn_ & 1);
    V2* ptrs[gs::kMaxMsgs];
    bool remote = false;
    uint32_t sysmask = 0;
    for (int i = 0; i < p.nsend; ++i) {
      const int idx = send_peer_[i];
      ptrs[i] = idx < 0 ? send_ + p.send[i].offset
                        : peers_[idx].landing + slot * peers_[idx].slot_cells + send_off_[i];
      remote = remote || idx >= 0;
      // a peer on another GPU (or an unidentified one): system-coherent stores over xGMI
      if (idx >= 0 && (peers_[idx].device != dev_ || gs::debug_knobs().ipc_system_stores))
        sysmask |= 1u << i;
    }
    // every wave with stores to a peer waits for them to be acknowledged before it retires
    gsk::launch_pack_ptrs<T, true>(buf_[b], ptrs, g_, p.send, p.nsend, xs_,
                                   remote && ipc_fence_, nullptr, sysmask);
    HIP_CHECK(hipGetLastError());
  }

  // The transport step of an IPC exchange (native_exchange): the engine issues it on the stream
  // of the same exchange's pack, after it, so the 'ready' signal (this rank's stores into the
  // peers have completed) is published here, fused with the wait for the peers' signals.
  void ipc_signal_wait() {
    if (!send_peers_.empty() || !recv_peers_.empty()) {
      gsk::IpcFlags s{}, w{};
      for (int idx : send_peers_) {
        s.f[s.n] = peers_[idx].flags + rank_;
        s.want[s.n++] = xn_;
      }
      for (int idx : recv_peers_) {
        w.f[w.n] = flags_ + peers_[idx].rank;
        w.want[w.n++] = xn_;
      }
      gsk::k_ipc_signal_wait<<<1, 64, 0, xs_>>>(s, w, ipc_ticks_, ipc_err_dev_, ipc_dflag_,
                                                ipc_emulate_ticks_);
      HIP_CHECK(hipGetLastError());
    }
  }

  // after ipc_signal_wait on the same stream: the peers' messages have landed in slot xn_ & 1
  void ipc_unpack(int b, const gs::HaloPlan& p) {
    const int64_t slot = (int64_t)(xn_ & 1);
    V2* ptrs[gs::kMaxMsgs];
    for (int i = 0; i < p.nrecv; ++i)
      ptrs[i] = (recv_peer_[i] < 0 ? recv_ : landing_ + slot * landing_cells_) + p.recv[i].offset;
    // 4 cells per lane: 16 (more loads in flight from the uncached landing buffer) measured
    // no better, overlapped or not (profiles/r3_unpack_items.txt)
    gsk::launch_pack_ptrs<T, false>(buf_[b], ptrs, g_, p.recv, p.nrecv, xs_, false, ipc_dflag_);
    HIP_CHECK(hipGetLastError());
  }

  // {rank, device (-1: not visible here), peer access (1 yes, -1 unknown)} per mapped peer
  int ipc_peers(int32_t* out, int cap) const {
    int n = 0;
    for (const PeerMap& pm : peers_)
      if (pm.rank != rank_ && n < cap) {
        out[3 * n] = pm.rank;
        out[3 * n + 1] = pm.device;
        out[3 * n + 2] = pm.p2p;
        ++n;
      }
    return n;
  }

  void ipc_release() {
    gate_release();
    gate_plan_ok_ = false;
    if (landing_ || !peers_.empty()) {
      (void)hipDeviceSynchronize();
      for (PeerMap& pm : peers_)
        if (pm.opened) {
          (void)hipIpcCloseMemHandle(pm.landing);
          (void)hipIpcCloseMemHandle(pm.flags);
        }
    }
    peers_.clear();
    if (landing_) (void)hipFree(landing_);
    if (flags_) (void)hipFree(flags_);
    if (ipc_dflag_) (void)hipFree(ipc_dflag_);
    if (ipc_err_) (void)hipHostFree(ipc_err_);
    landing_ = nullptr;
    flags_ = nullptr;
    ipc_dflag_ = nullptr;
    ipc_err_ = ipc_err_dev_ = nullptr;
    ipc_ = false;
  }

  // ---------------------------------------------------------------------------------------
  // Gated pass (gate.hpp, engine.h advance_gated): one k_fused launch per pass carries the IPC
  // halo exchange.  The host builds the unit table (one unit per workgroup, start-gated units
  // sized shorter by the expected exchange time) for the tile shape the full pass was tuned to,
  // and tunes that expected time on the device (gate_tune).
  bool gated_supported(int n) const override {
    // the gated entry exists for the production variants only (FCfg::GATE_OK): non-periodic,
    // noisy, 32-bit Philox counter
    return ipc_ && gate_plan_ok_ && gsk::fused_supported(g_, n) && n >= 2 && n <= 3 &&
           g_.nz >= 2 * n + 1 && !g_.periodic && p_.noise != 0.0 && gsk::philox_q32(g_) &&
           !gs::debug_knobs().philox_generic &&
           // peers sharing this GPU: only when asked (debug knob gated = 2) -- every rank's
           // waiting units must be resident at once, across processes (gate_table)
           (gate_sharers_ == 0 || gs::debug_knobs().gated >= 2) && gate_fits(n);
  }

  // whether a depth-n table fits the device's resident slots at all (its longest chunks: one
  // unit per tile column, or per column end): more units than slots could leave a packer
  // queued behind workgroups that wait for it -- e.g. a very flat sub-domain with more tile
  // columns than workgroup slots keeps the stream-overlapped passes (cached per depth)
  bool gate_fits(int n) const {
    if (gate_fit_[n] < 0) {
      try {
        int npk = 0, slots = 0;
        const size_t units = gate_table(n, 0, false, &npk, &slots, true).size();
        gate_fit_[n] = units <= (size_t)slots ? 1 : 0;
      } catch (const std::exception&) {
        gate_fit_[n] = 0;  // no gated entry / occupancy for this shape: the stream path
      }
    }
    return gate_fit_[n] == 1;
  }

  void gate_release() {
    if (d_gate_) (void)hipFree(d_gate_);
    if (d_counter_) (void)hipFree(d_counter_);
    if (d_stamps_) (void)hipFree(d_stamps_);
    d_stamps_ = nullptr;
    for (auto*& u : d_units_)
      if (u) { (void)hipFree(u); u = nullptr; }
    d_gate_ = nullptr;
    d_counter_ = nullptr;
    cnt_host_[0] = cnt_host_[1] = 0;
    for (int i = 0; i < 4; ++i) {
      gate_tuned_[i] = pairs_[i] = carry_[i] = false;
      nunits_[i] = npk_[i] = nprod_[i] = nwu_[i] = 0;
      gate_xp_[i] = gate_u_[i] = -1;
    }
  }

  // the transport half of the launch arguments (device copy, built once per IPC connection)
  void gate_setup() {
    if (d_gate_) return;
    gsk::GateArgs G{};
    const gs::HaloPlan& p = gplan_;
    G.nsend = p.nsend;
    for (int i = 0; i < p.nsend; ++i) {
      const PeerMap& pm = peers_[send_peer_[i]];
      G.sbox[i] = p.send[i].box;
      for (int sl = 0; sl < 2; ++sl) G.sdst[sl][i] = pm.landing + sl * pm.slot_cells + send_off_[i];
      if (pm.device != dev_ || gs::debug_knobs().ipc_system_stores) G.sysmask |= 1u << i;
    }
    G.nrecv = p.nrecv;
    for (int i = 0; i < p.nrecv; ++i) {
      G.rbox[i] = p.recv[i].box;
      for (int sl = 0; sl < 2; ++sl) G.rsrc[sl][i] = landing_ + sl * landing_cells_ + p.recv[i].offset;
    }
    for (int idx : recv_peers_) {
      G.wstamp[G.nwait] = flags_ + ipc_nranks_ + peers_[idx].rank;
      G.wflag[G.nwait++] = flags_ + peers_[idx].rank;
    }
    for (int idx : send_peers_) {
      G.sstamp[G.nsig] = peers_[idx].flags + ipc_nranks_ + rank_;
      G.sflag[G.nsig++] = peers_[idx].flags + rank_;
    }
    HIP_CHECK(hipMalloc((void**)&d_counter_, 2 * sizeof(uint32_t)));
    HIP_CHECK(hipMemset(d_counter_, 0, 2 * sizeof(uint32_t)));
    cnt_host_[0] = cnt_host_[1] = 0;
    G.counter = d_counter_;
    G.ticks = ipc_ticks_;
    G.min_ticks = ipc_emulate_ticks_;
    G.err = ipc_err_dev_;
    G.dflag = ipc_dflag_;
    if (gs::debug_knobs().gate_stamps) {
      HIP_CHECK(hipMalloc((void**)&d_stamps_, 11 * sizeof(unsigned long long)));
      HIP_CHECK(hipMemset(d_stamps_, 0, 11 * sizeof(unsigned long long)));
      G.stamps = d_stamps_;
    }
    HIP_CHECK(hipMalloc((void**)&d_gate_, sizeof(gsk::GateArgs)));
    HIP_CHECK(hipMemcpy(d_gate_, &G, sizeof(G), hipMemcpyHostToDevice));
  }

  // Unit table of a depth-n gated pass for the tile shape the full pass runs, with start-gated
  // chunks shorter by xp planes (the expected exchange time in plane-times): the smallest plane
  // budget per workgroup whose chunks fit the resident slots.  Sorted by (z0, tile): each XCD
  // group of workgroups gets a contiguous range (sched 3), i.e. neighbouring tiles at one depth.
  // pairs (U >= 0): the two-entries-per-workgroup table, xp the expected exchange and U the
  // cone unpack in plane-times (gs::gate_plan_pairs; empty when none fits the slots)
  std::vector<gsk::GateUnit> gate_table(int n, int xp, bool allpk, int* npk,
                                        int* slots_out = nullptr, bool longest = false,
                                        int U = -1) const {
    const int cfg = gsk::gated_shape_cfg(sizeof(T) == 8, g_, n);
    const char* name = gsk::fused_shape_name(cfg, sizeof(T) == 8, true);
    const gsk::TileGrid tg = gsk::fused_tile_grid(name, g_, n);
    // every unit resident at once (the device's occupancy of the gated entry): a start-gated
    // unit that waits for the peers holds its slot, so a packer left unscheduled behind waiting
    // units would stall every rank until the wall-clock bound
    const int per_cu = gsk::fused_gated_occupancy<T>(cfg, n, U >= 0);
    if (per_cu < 1) throw std::runtime_error("gated pass: no gated entry for this shape");
    // (peer processes on this GPU, debug knob gated = 2: this rank's share of the slots)
    const int slots = std::max(8, num_cus() * per_cu / (gate_sharers_ + 1));
    if (slots_out) *slots_out = slots;
    if (U >= 0) return gs::gate_plan_pairs(tg, g_, gplan_, n, xp, U, allpk, slots, npk);
    return gs::gate_plan(tg, g_, gplan_, n, xp, allpk, slots, longest, npk);
  }

  void gate_upload(int n, const std::vector<gsk::GateUnit>& u, int npk, bool pairs) {
    pairs_[n] = pairs;
    const size_t bytes = std::max<size_t>(u.size(), 1) * sizeof(gsk::GateUnit);
    if (!d_units_[n] || cap_units_[n] < u.size()) {
      if (d_units_[n]) (void)hipFree(d_units_[n]);
      HIP_CHECK(hipMalloc((void**)&d_units_[n], std::max<size_t>(bytes, 4096 * sizeof(gsk::GateUnit))));
      cap_units_[n] = std::max<size_t>(u.size(), 4096);
    }
    HIP_CHECK(hipStreamSynchronize(stream_));  // no launch still reads the previous table
    HIP_CHECK(hipMemcpy(d_units_[n], u.data(), bytes, hipMemcpyHostToDevice));
    nunits_[n] = (int)u.size();
    npk_[n] = npk;
    nprod_[n] = nwu_[n] = 0;
    for (const gsk::GateUnit& x : u) {
      nprod_[n] += x.prod != 0;
      nwu_[n] += x.wait != 0;
    }
  }

  // one gated pass src -> dst on the compute stream (exchange number ++xn_).  pre bit 0: its
  // exchange was carried by the previous launch (packed by its producers); bit 1: this launch's
  // producers carry the next one (gate.hpp gate_carry)
  void gate_launch(int src, int dst, int n, int64_t t, int pre = 0) {
    gsk::GateLaunch gl{};
    gl.units = d_units_[n];
    gl.nunits = nunits_[n];
    gl.gate = d_gate_;
    gl.n = ++xn_;
    if (!(pre & 1)) cnt_host_[gl.n & 1] += (uint32_t)npk_[n];
    gl.cnt = cnt_host_[gl.n & 1];
    if (pre & 2) {
      // arrivals of exchange n + 1: every producer after its carry, every start-gated unit
      // after its unpack (the peers' slot reuse waits for both)
      cnt_host_[(gl.n + 1) & 1] += (uint32_t)(nprod_[n] + nwu_[n]);
      gl.cnt2 = cnt_host_[(gl.n + 1) & 1];
    }
    gl.pre = pre;
    gl.npk = npk_[n];
    gl.pairs = pairs_[n] ? 1 : 0;
    if (d_stamps_) {  // debug knob gate_stamps: this launch's stamps only
      const unsigned long long init[8] = {~0ull, 0ull, ~0ull, 0ull, 0ull, 0ull, 0ull, 0ull};
      HIP_CHECK(hipMemcpyAsync(d_stamps_, init, sizeof(init), hipMemcpyHostToDevice, stream_));
    }
    if (!gsk::launch_fused<T>(buf_[src], buf_[dst], g_, p_, n, t, stream_,
                              gsk::gated_shape_cfg(sizeof(T) == 8, g_, n), 3, 0, g_.nz, 0, 0, 0,
                              0, false, &gl))
      throw std::runtime_error("gated pass: launch rejected");
    HIP_CHECK(hipGetLastError());
  }

  // Expected exchange time per pass (xp, plane-times) tuned on the device: each candidate
  // table is timed over a few passes, the fastest kept.  Every rank times the same candidates
  // in the same order (each pass is an exchange all ranks take part in); ranks may keep
  // different tables -- the protocol only needs every rank to pack and signal once per pass.
  void gate_tune(int src, int dst, int n, int64_t t) {
    if (!tuned_[n]) autotune(src, dst, n, t);
    gate_setup();
    // candidates: one-unit tables (expected exchange xp, packers), pairs tables (an ungated
    // chunk before each start-gated one: exchange X, unpack U) and carried one-unit tables (the
    // previous pass's producers pack: xp then covers the cone unpack and the carry); every rank
    // times the same list
    struct Cand { int xp, U; bool all, carry; };
    std::vector<Cand> cands;
    // debug knob gate_mode (tests, A/B): 1 one-unit only, 2 pairs only, 3 carried only
    const int mode = gs::debug_knobs().gate_mode;
    if (mode == 0 || mode == 3)
      for (int xp : {0, 2, 4, 6, 8, 12, 16, 24}) cands.push_back({xp, -1, false, true});
    for (int all = 0; all < 2; ++all) {
      if (mode == 0 || mode == 1)
        for (int xp : {0, 4, 8, 16, 24, 32}) cands.push_back({xp, -1, all != 0, false});
      if (mode == 0 || mode == 2)
        for (int X : {8, 16, 24, 32})
          for (int U : {4, 8}) cands.push_back({X, U, all != 0, false});
    }
    float best = 1e30f;
    Cand bc = cands[0];
    hipEvent_t e0, e1;
    HIP_CHECK(hipEventCreate(&e0));
    HIP_CHECK(hipEventCreate(&e1));
    for (const Cand& c : cands) {
      int npk = 0;
      std::vector<gsk::GateUnit> u = gate_table(n, c.xp, c.all, &npk, nullptr, false, c.U);
      const bool pairs = c.U >= 0 && !u.empty();
      // no pairs table fits this rank: it still makes the candidate's launches (with a one-unit
      // table), so every rank takes part in the same number of exchanges
      if (u.empty()) u = gate_table(n, 0, c.all, &npk);
      gate_upload(n, u, npk, pairs);
      // carried: a run of passes -- the first packs at its start, the timed ones find their
      // exchange carried, the last carries none.  A producer must be start-gated (it has then
      // seen the peers publish, i.e. finish with the slot it fills: gate.hpp gate_carry) --
      // true for the symmetric neighbour sets of a Cartesian grid; a table where it is not
      // runs the same launches uncarried and is not kept
      bool carry_ok = c.carry && !pairs;
      for (const gsk::GateUnit& x : u) carry_ok = carry_ok && (!x.prod || x.wait);
      const int pin = carry_ok ? 1 : 0, pout = carry_ok ? 2 : 0;
      gate_launch(src, dst, n, t, pout);  // warm-up
      HIP_CHECK(hipEventRecord(e0, stream_));
      for (int r = 0; r < 3; ++r) gate_launch(src, dst, n, t, pin | pout);
      HIP_CHECK(hipEventRecord(e1, stream_));
      if (c.carry) gate_launch(src, dst, n, t, pin);
      wait_all(gs::comm_timeout_s());
      float ms = 0.f;
      HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
      if (ms < best && (c.U < 0 || pairs) && (!c.carry || carry_ok)) { best = ms; bc = c; }
    }
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    int npk = 0;
    const std::vector<gsk::GateUnit> u = gate_table(n, bc.xp, bc.all, &npk, nullptr, false, bc.U);
    gate_upload(n, u, npk, bc.U >= 0);
    gate_xp_[n] = bc.xp;
    gate_u_[n] = bc.U;
    gate_allpk_[n] = bc.all;
    bool carry = bc.carry && bc.U < 0;
    for (const gsk::GateUnit& x : u) carry = carry && (!x.prod || x.wait);
    carry_[n] = carry;
    gate_ms_[n] = best / 3.f;
    gate_tuned_[n] = true;
  }

  void prepare_gated(int src, int dst, int n, int64_t t) override {
    if (gated_supported(n) && !gate_tuned_[n]) gate_tune(src, dst, n, t);
  }

  // first / last: the pass opens / closes the engine's run of gated passes (a carried exchange
  // never crosses a run: between runs the fields may change)
  bool fused_gated(int src, int dst, int n, int64_t t, bool first, bool last) override {
    if (!gated_supported(n)) return false;
    if (!gate_tuned_[n]) gate_tune(src, dst, n, t);
    const int pre = carry_[n] ? ((first ? 0 : 1) | (last ? 0 : 2)) : 0;
    gate_launch(src, dst, n, t, pre);
    return true;
  }

  // debug knob gate_stamps: the last gated launch's exchange, µs after its first packer or
  // waiting unit started -- {last arrival (packing done; -1: a carried exchange), first wait
  // done, last wait done, last unpack done, the longest and the mean unpack of one unit}, then
  // over every launch since set-up the longest and the mean carry of one producer (-1: none)
  void gate_stamps(double* out8) {
    for (int i = 0; i < 8; ++i) out8[i] = -1.0;
    if (!d_stamps_) return;
    HIP_CHECK(hipStreamSynchronize(stream_));
    unsigned long long h[11];
    HIP_CHECK(hipMemcpy(h, d_stamps_, sizeof(h), hipMemcpyDeviceToHost));
    int khz = 0;
    HIP_CHECK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev_));
    const double us = 1000.0 / (double)std::max(khz, 1);
    if (h[10]) {
      out8[6] = (double)h[8] * us;
      out8[7] = (double)h[9] * us / (double)h[10];
    }
    if (h[0] == ~0ull) return;
    for (int i = 0; i < 4; ++i)
      if (h[i + 1] >= h[0]) out8[i] = (double)(h[i + 1] - h[0]) * us;
    out8[4] = (double)h[5] * us;                                  // longest unit unpack
    out8[5] = h[7] ? (double)h[6] * us / (double)h[7] : 0.0;      // mean unit unpack
  }


  // {tuned xp (plane-times), table entries, packers, ms per pass, pairs U (-1: one-unit
  // table)} of depth n (xp -1: not tuned)
  void gate_info(int n, double* out6) const {
    out6[0] = gate_xp_[n];
    out6[1] = nunits_[n];
    out6[2] = npk_[n];
    out6[3] = gate_ms_[n];
    out6[4] = gate_u_[n];
    out6[5] = carry_[n] ? nprod_[n] : -1;  // carried exchanges: the producers
  }

  // Forget the device transport after a failed trial (the "auto" fallback chain): abort the
  // RCCL communicator -- it may be half broken -- and unmap the IPC peers, so the next
  // transport in the chain is the only one this engine uses.
  void drop_transport() override {
    // no device sync first: an RCCL kernel waiting for a peer that failed would never end;
    // ncclCommAbort is what releases it
    if (comm_) abort_comm();
    ipc_release();
  }
  bool ipc_active() const { return ipc_; }
  void self_copy(int64_t so, int64_t d, int64_t n) override {
    HIP_CHECK(hipMemcpyAsync(recv_ + d, send_ + so, sizeof(V2) * n, hipMemcpyDeviceToDevice, xs_));
  }

  bool native_exchange(const gs::HaloPlan& p) override {
    if (ipc_) {
      // the IPC pack already stored every message at its peer: signal and wait
      ipc_signal_wait();
      return true;
    }
    if (!comm_) return false;
    NCCL_CHECK(ncclGroupStart());
    for (int i = 0; i < p.nsend; ++i) {
      const gs::HaloMsg& m = p.send[i];
      if (m.peer == rank_ && !loopback_) continue;
      NCCL_CHECK(ncclSend(send_ + m.offset, (size_t)gs::box_cells(m.box) * sizeof(V2), ncclUint8,
                          m.peer, comm_, xs_));
    }
    for (int i = 0; i < p.nrecv; ++i) {
      const gs::HaloMsg& m = p.recv[i];
      if (m.peer == rank_ && !loopback_) continue;
      NCCL_CHECK(ncclRecv(recv_ + m.offset, (size_t)gs::box_cells(m.box) * sizeof(V2), ncclUint8,
                          m.peer, comm_, xs_));
    }
    group_end();
    return true;
  }

  void set_loopback(bool on) override { loopback_ = on; }

  void host_sync() override { HIP_CHECK(hipStreamSynchronize(xs_)); }

  // Watchdog wait: poll both streams and RCCL's asynchronous error state; a
  // transport error or no completion within timeout_s aborts the communicator and throws, so
  // one failed rank ends the job instead of hanging it.
  void wait_all(double timeout_s) override {
    if (!comm_ && !ipc_) {
      HIP_CHECK(hipStreamSynchronize(stream_));
      HIP_CHECK(hipStreamSynchronize(comm_stream_));
      return;
    }
    const auto t0 = std::chrono::steady_clock::now();
    int sleep_us = 20;
    // Timed regions end in this wait, so its detection latency adds to every measured window:
    // the first kSpinS seconds poll back to back (a yield between queries: ~1-2 us latency);
    // only a longer wait backs off to sleeps of up to 160 us (previously from the first poll,
    // which could report a 1 ms multi-rank window up to ~0.2 ms late).
    constexpr double kSpinS = 0.05;
    for (;;) {
      const hipError_t a = hipStreamQuery(stream_);
      const hipError_t b = hipStreamQuery(comm_stream_);
      // an IPC wait kernel that gave up (peer silent for GS_COMM_TIMEOUT) reports here
      if (ipc_err_ && __atomic_load_n(ipc_err_, __ATOMIC_ACQUIRE) != 0)
        throw std::runtime_error("IPC halo exchange: a peer did not signal within "
                                 "GS_COMM_TIMEOUT seconds (device wait timed out)");
      if (a == hipSuccess && b == hipSuccess) return;
      if (a != hipErrorNotReady) HIP_CHECK(a);
      if (b != hipErrorNotReady) HIP_CHECK(b);
      ncclResult_t async = ncclSuccess;
      if (comm_) NCCL_CHECK(ncclCommGetAsyncError(comm_, &async));
      if (async != ncclSuccess && async != ncclInProgress) {
        abort_comm();
        throw std::runtime_error(std::string("RCCL asynchronous error: ") + ncclGetErrorString(async));
      }
      const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      if (timeout_s > 0 && el > timeout_s) {
        if (comm_) abort_comm();
        throw std::runtime_error("halo exchange watchdog: device work not finished after " +
                                 std::to_string(timeout_s) + " s (GS_COMM_TIMEOUT)");
      }
      if (el < kSpinS) {
        std::this_thread::yield();
        continue;
      }
      std::this_thread::sleep_for(std::chrono::microseconds(sleep_us));
      if (sleep_us < 100) sleep_us *= 2;
    }
  }

  void extract(int b, void* u, void* v) override {
    gsk::launch_extract<T>(buf_[b], (T*)u, (T*)v, g_, stream_);
    HIP_CHECK(hipGetLastError());
  }
  int extract_minmax(int b, void* u, void* v, void* part, int cap) override {
    const int n = gsk::launch_extract_mm<T>(buf_[b], (T*)u, (T*)v, g_, (T*)part, cap, stream_);
    HIP_CHECK(hipGetLastError());
    return n;
  }
  // One output / checkpoint snapshot in a single call (models/grayscott.py snapshot_fields):
  // the compute stream waits for the previous D2H out of the device buffers (prev, may be
  // null), compacts the interior (with per-chunk min / max when part != null), and the I/O
  // stream copies it into the pinned host buffers, recording done.  Returns the min / max
  // quadruples copied (0: none).
  int snapshot(int b, void* du, void* dv, void* dpart, int cap, void* hu, void* hv, void* hpart,
               hipStream_t io, hipEvent_t prev, hipEvent_t ready, hipEvent_t done) {
    if (prev) HIP_CHECK(hipStreamWaitEvent(stream_, prev, 0));
    int n = 0;
    if (dpart) n = gsk::launch_extract_mm<T>(buf_[b], (T*)du, (T*)dv, g_, (T*)dpart, cap, stream_);
    if (!n) gsk::launch_extract<T>(buf_[b], (T*)du, (T*)dv, g_, stream_);
    HIP_CHECK(hipGetLastError());
    HIP_CHECK(hipEventRecord(ready, stream_));
    HIP_CHECK(hipStreamWaitEvent(io, ready, 0));
    const size_t bytes = (size_t)g_.nx * g_.ny * g_.nz * sizeof(T);
    HIP_CHECK(hipMemcpyAsync(hu, du, bytes, hipMemcpyDeviceToHost, io));
    HIP_CHECK(hipMemcpyAsync(hv, dv, bytes, hipMemcpyDeviceToHost, io));
    if (n) HIP_CHECK(hipMemcpyAsync(hpart, dpart, (size_t)4 * n * sizeof(T), hipMemcpyDeviceToHost, io));
    HIP_CHECK(hipEventRecord(done, io));
    return n;
  }

  void randomize(int b, uint64_t seed, double lo, double hi) override {
    gsk::launch_randomize<T>(buf_[b], g_, seed, lo, hi, stream_);
    HIP_CHECK(hipGetLastError());
  }
  void insert(int b, const void* u, const void* v) override {
    gsk::launch_insert<T>(buf_[b], (const T*)u, (const T*)v, g_, stream_);
    HIP_CHECK(hipGetLastError());
  }

  void stats(int b, double* out) override {
    gsk::launch_stats<T>(buf_[b], g_, (double*)ws_, kStatBlocks, stream_);
    HIP_CHECK(hipGetLastError());
    std::vector<double> h(6 * kStatBlocks);
    HIP_CHECK(hipMemcpyAsync(h.data(), ws_, sizeof(double) * h.size(), hipMemcpyDeviceToHost, stream_));
    HIP_CHECK(hipStreamSynchronize(stream_));
    double su = 0, sv = 0, mnu = 1e300, mxu = -1e300, mnv = 1e300, mxv = -1e300;
    for (int i = 0; i < kStatBlocks; ++i) {
      const double* q = &h[6 * i];
      su += q[0]; mnu = std::min(mnu, q[1]); mxu = std::max(mxu, q[2]);
      sv += q[3]; mnv = std::min(mnv, q[4]); mxv = std::max(mxv, q[5]);
    }
    out[0] = su; out[1] = mnu; out[2] = mxu; out[3] = sv; out[4] = mnv; out[5] = mxv;
  }

  // a failed communicator is aborted and never reused
  void abort_comm() {
    if (comm_ == shared_comm().comm) shared_comm() = SharedComm{};
    ncclCommAbort(comm_);
    comm_ = nullptr;
  }

  // what RCCL sees: communicator size, this rank in it, the device it drives
  void comm_info(int32_t* out3) const {
    out3[0] = out3[1] = out3[2] = -1;
    if (!comm_) return;
    int n = -1, r = -1, d = -1;
    NCCL_CHECK(ncclCommCount(comm_, &n));
    NCCL_CHECK(ncclCommUserRank(comm_, &r));
    NCCL_CHECK(ncclCommCuDevice(comm_, &d));
    out3[0] = n; out3[1] = r; out3[2] = d;
  }

  // The communicator is created non-blocking (config.blocking = 0) and its set-up is polled
  // under GS_COMM_TIMEOUT: a peer that never joins, or a bootstrap / topology stall on a fresh
  // node, becomes an error (the communicator aborted, the transport chain moves on) instead of
  // a process blocked inside ncclCommInitRank for the rest of the job.  Every later call on a
  // non-blocking communicator may also return ncclInProgress -- the first send / receive to a
  // peer sets up its connection asynchronously -- so each group end is completed the same way
  // (group_end) before anything else is enqueued behind it.
  void init_comm(const ncclUniqueId& id, int nranks, int rank) {
    SharedComm& sc = shared_comm();
    if (sc.comm && sc.nranks == nranks && sc.rank == rank) {
      rank_ = rank;
      comm_ = sc.comm;
      return;
    }
    rank_ = rank;
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;
    ncclComm_t c = nullptr;
    const ncclResult_t r = ncclCommInitRankConfig(&c, nranks, id, rank, &cfg);
    if (r != ncclSuccess && r != ncclInProgress) {
      if (c) ncclCommAbort(c);
      throw std::runtime_error(std::string("RCCL error: ") + ncclGetErrorString(r) +
                               " (ncclCommInitRankConfig)");
    }
    comm_ = c;
    complete(c, "communicator set-up (ncclCommInitRankConfig)");
    if (!sc.comm) sc = SharedComm{comm_, nranks, rank};  // kept for the process lifetime
  }

  // Wait for a non-blocking communicator's pending operation (set-up, a group's connection
  // set-up) under GS_COMM_TIMEOUT; on an error or timeout abort the communicator and throw.
  void complete(ncclComm_t c, const char* what) {
    const double to = gs::comm_timeout_s();
    const auto t0 = std::chrono::steady_clock::now();
    int sleep_us = 10;
    for (;;) {
      ncclResult_t st = ncclSuccess;
      const ncclResult_t q = ncclCommGetAsyncError(c, &st);
      if (q != ncclSuccess) st = q;
      if (st == ncclSuccess) return;
      if (st != ncclInProgress) {
        abort_comm();
        throw std::runtime_error(std::string("RCCL error: ") + ncclGetErrorString(st) + " in " +
                                 what);
      }
      const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      if (el > to) {
        abort_comm();
        throw std::runtime_error(std::string("RCCL ") + what + " did not complete within " +
                                 std::to_string(to) + " s (GS_COMM_TIMEOUT): a peer never joined "
                                 "or the node's topology set-up stalled");
      }
      std::this_thread::sleep_for(std::chrono::microseconds(sleep_us));
      if (sleep_us < 1000) sleep_us *= 2;
    }
  }

  // ncclGroupEnd on the non-blocking communicator: in steady state the group is enqueued before
  // it returns; the first exchange with a peer returns ncclInProgress while the connection is
  // made, and completes here, so the stream order of later work is unchanged
  void group_end() {
    const ncclResult_t r = ncclGroupEnd();
    if (r == ncclSuccess) return;
    if (r != ncclInProgress)
      throw std::runtime_error(std::string("RCCL error: ") + ncclGetErrorString(r) + " (ncclGroupEnd)");
    complete(comm_, "point-to-point connection set-up (ncclGroupEnd)");
  }

 private:
  static constexpr int kStatBlocks = 1024;
  // workgroup slots the inner part of an overlapped pass leaves free, so the communication
  // kernels (RCCL's, pack / unpack) start beside it (0-16 equal within noise, 64 slower:
  // profiles/r2_overlap_reserve.txt)
  // workgroup slots the overlapped inner launch leaves free for the comm chain: 16, 48 and 96
  // measured equal after the cell-granular split (profiles/r3_overlap_reserve.txt)
  static constexpr int kOverlapReserve = 16;
  Geom g_;
  gs::Params p_;
  hipStream_t stream_;
  V2* buf_[2];
  V2* send_;
  V2* recv_;
  void* ws_ = nullptr;
  hipEvent_t ev_ = nullptr;
  hipEvent_t ev_fork_ = nullptr, ev_join_ = nullptr;
  hipEvent_t marks_[4] = {nullptr, nullptr, nullptr, nullptr};
  std::vector<hipEvent_t> prof_ev_;  // per-phase timing events (prof_reserve)
  int prof_n_ = 0;
  hipStream_t comm_stream_ = nullptr;
  hipStream_t xs_ = nullptr;  // stream for halo traffic (compute or comm stream)
  bool inplace_off_ = getenv("GS_INPLACE_HALO") && atoi(getenv("GS_INPLACE_HALO")) == 0;
  int dev_ = 0;
  ncclComm_t comm_ = nullptr;
  int rank_ = 0;
  bool loopback_ = false;
  // IPC peer-write transport (ipc_export / ipc_connect)
  struct PeerMap {
    int rank;
    V2* landing;     // the peer's landing buffer (2 slots of slot_cells), mapped here
    uint64_t* flags;  // the peer's flag array, mapped here
    int64_t slot_cells;
    bool opened;     // opened through IPC (not this rank's own buffers)
    int device;      // the peer's device as numbered in this process (-1: not visible)
    int p2p;         // 1: this device can access the peer's (checked), -1: unknown
  };
  bool ipc_ = false;
  static constexpr bool ipc_fence_ = true;
  int ipc_nranks_ = 0;
  int* ipc_dflag_ = nullptr;  // device copy of the timeout word (unpacks write NaN once set)
  V2* landing_ = nullptr;
  uint64_t* flags_ = nullptr;
  int* ipc_err_ = nullptr;
  int* ipc_err_dev_ = nullptr;
  int64_t landing_cells_ = 0;
  uint64_t xn_ = 0;  // exchanges issued
  uint64_t ipc_ticks_ = 0;
  uint64_t ipc_emulate_ticks_ = 0;  // debug knob ipc_emulate_us: minimum exchange wait (modelling)
  std::vector<PeerMap> peers_;
  std::vector<int> send_peers_, recv_peers_;  // distinct peers (indices into peers_)
  int send_peer_[gs::kMaxMsgs], recv_peer_[gs::kMaxMsgs];
  int64_t send_off_[gs::kMaxMsgs];  // offset of send message i in its peer's landing slot
  // per fused depth (T = 4: fp32 whole-interior passes, the LDS-ring shapes)
  static constexpr int kMaxDepth = sizeof(T) == 4 ? 4 : 3;
  bool tuned_[5] = {false, false, false, false, false};
  int cfg_[5] = {-1, -1, -1, -1, -1};
  int sched_[5] = {-1, -1, -1, -1, -1};
  float tuned_ms_[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
  std::vector<ShellChoice> shells_;
  std::vector<PartChoice> parts_;
  // gated pass (gate_*)
  gs::HaloPlan gplan_{};
  bool gate_plan_ok_ = false;
  int gate_sharers_ = 0;  // peer ranks (other processes) on this GPU
  mutable int gate_fit_[4] = {-1, -1, -1, -1};  // gate_fits per depth (-1: not yet checked)
  bool gate_allpk_[4] = {false, false, false, false};  // tuned: every unit packs
  bool pairs_[4] = {false, false, false, false};       // the uploaded table is a pairs table
  int gate_u_[4] = {-1, -1, -1, -1};                   // tuned pairs U (-1: one-unit table)
  unsigned long long* d_stamps_ = nullptr;  // debug knob gate_stamps
  gsk::GateArgs* d_gate_ = nullptr;
  uint32_t* d_counter_ = nullptr;  // two words: exchange m counts on word m & 1
  uint32_t cnt_host_[2] = {0, 0};   // arrivals issued so far per word (its value after them)
  gsk::GateUnit* d_units_[4] = {nullptr, nullptr, nullptr, nullptr};
  size_t cap_units_[4] = {0, 0, 0, 0};
  int nunits_[4] = {0, 0, 0, 0};
  int npk_[4] = {0, 0, 0, 0};
  int gate_xp_[4] = {-1, -1, -1, -1};
  int nprod_[4] = {0, 0, 0, 0};  // the table's producers (carried exchanges)
  int nwu_[4] = {0, 0, 0, 0};    // the table's start-gated units
  bool carry_[4] = {false, false, false, false};  // tuned: runs of passes carry their exchanges
  float gate_ms_[4] = {0.f, 0.f, 0.f, 0.f};
  bool gate_tuned_[4] = {false, false, false, false};
};

}  // namespace

gs::Backend* gs_make_backend(int32_t dtype, const gs::Geom& g, const gs::Params& p, void* b0,
                             void* b1, void* send, void* recv, void* stream) {
  if (dtype == gs::kF32) return new HipBackend<float>(g, p, b0, b1, send, recv, (hipStream_t)stream);
  if (dtype == gs::kF64) return new HipBackend<double>(g, p, b0, b1, send, recv, (hipStream_t)stream);
  throw std::runtime_error("unsupported dtype");
}

// The engine's backend as a HipBackend<T> for the dtype the caller names: a checked cast, so
// a CPU engine or a dtype mismatch is an error, not undefined behaviour.
template <typename T>
HipBackend<T>* hip_backend_of(gs_engine* e) {
  if (!e || !e->eng) throw std::runtime_error("null engine");
  HipBackend<T>* b = dynamic_cast<HipBackend<T>*>(e->eng->backend());
  if (!b)
    throw std::runtime_error(std::string("engine is not a HIP ") +
                             (sizeof(T) == 4 ? "fp32" : "fp64") + " engine");
  return b;
}

// f(backend) on the engine's HipBackend of `dtype`
template <class F>
void with_hip_backend(gs_engine* e, int32_t dtype, F&& f) {
  if (dtype == gs::kF32) f(hip_backend_of<float>(e));
  else if (dtype == gs::kF64) f(hip_backend_of<double>(e));
  else throw std::runtime_error("unsupported dtype");
}

extern "C" {

int gs_rccl_unique_id(char* out, int32_t cap) {
  try {
    if (cap < (int32_t)sizeof(ncclUniqueId)) throw std::runtime_error("buffer too small");
    ncclUniqueId id;
    NCCL_CHECK(ncclGetUniqueId(&id));
    memcpy(out, &id, sizeof(id));
    return (int)sizeof(id);
  } catch (const std::exception& ex) {
    g_gs_err = ex.what();
    return -1;
  }
}

// {communicator size, rank in it, HIP device} of the engine's RCCL communicator (-1: none)
int gs_rccl_info(gs_engine* e, int32_t dtype, int32_t* out3) {
  try {
    with_hip_backend(e, dtype, [&](auto* b) { b->comm_info(out3); });
    return 0;
  } catch (const std::exception& ex) {
    g_gs_err = ex.what();
    return -1;
  }
}

// Timing experiment (experiments/r6/graph_probe_engine.py): microseconds per step of `reps` x
// advance(nsteps) enqueued as usual (out2[0]) and of the same advance(nsteps) captured once into a
// hipGraph and replayed `reps` times (out2[1]).  The replays repeat the captured time step, so the
// state afterwards is NOT a valid simulation state: timing only.
int gs_graph_probe(gs_engine* e, int32_t dtype, int64_t nsteps, int32_t reps, double* out2) {
  try {
    hipStream_t st = nullptr;
    with_hip_backend(e, dtype, [&](auto* b) { st = b->main_stream(); });
    hipEvent_t a, z;
    HIP_CHECK(hipEventCreate(&a));
    HIP_CHECK(hipEventCreate(&z));
    e->eng->advance(nsteps);  // warm
    HIP_CHECK(hipStreamSynchronize(st));
    HIP_CHECK(hipEventRecord(a, st));
    for (int r = 0; r < reps; ++r) e->eng->advance(nsteps);
    HIP_CHECK(hipEventRecord(z, st));
    HIP_CHECK(hipEventSynchronize(z));
    float ms = 0.f;
    HIP_CHECK(hipEventElapsedTime(&ms, a, z));
    out2[0] = 1e3 * ms / ((double)reps * nsteps);
    hipGraph_t g = nullptr;
    hipGraphExec_t ge = nullptr;
    HIP_CHECK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
    e->eng->advance(nsteps);
    HIP_CHECK(hipStreamEndCapture(st, &g));
    HIP_CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    HIP_CHECK(hipGraphLaunch(ge, st));
    HIP_CHECK(hipStreamSynchronize(st));
    HIP_CHECK(hipEventRecord(a, st));
    for (int r = 0; r < reps; ++r) HIP_CHECK(hipGraphLaunch(ge, st));
    HIP_CHECK(hipEventRecord(z, st));
    HIP_CHECK(hipEventSynchronize(z));
    HIP_CHECK(hipEventElapsedTime(&ms, a, z));
    out2[1] = 1e3 * ms / ((double)reps * nsteps);
    (void)hipGraphExecDestroy(ge);
    (void)hipGraphDestroy(g);
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(z);
    return 0;
  } catch (const std::exception& ex) {
    g_gs_err = ex.what();
    return -1;
  }
}

// Abort the process-wide RCCL communicator (job-wide failure handling: a rank that is about to
// exit on an error aborts its communicator first, so peers blocked in a halo exchange see an
// error instead of waiting for a message that never comes).  Engines must not be used after.
int gs_rccl_abort(void) {
  SharedComm& sc = shared_comm();
  if (!sc.comm) return 0;
  const ncclResult_t r = ncclCommAbort(sc.comm);
  sc = SharedComm{};
  return r == ncclSuccess ? 0 : -1;
}

// IPC peer-write transport.  gs_ipc_export allocates and exports this engine's landing buffer
// and flags (out: kIpcHandleBytes, returned); every rank then passes all ranks' exports and
// receive tables (per rank kIpcTabStride int64: nrecv, recv_cells, nrecv x (peer, offset,
// cells)) to gs_ipc_connect.
int gs_ipc_handle_bytes(void) { return kIpcHandleBytes; }
int gs_ipc_tab_stride(void) { return kIpcTabStride; }
int gs_ipc_export(gs_engine* e, int32_t dtype, int32_t nranks, int32_t rank, char* out) {
  try {
    with_hip_backend(e, dtype, [&](auto* b) { b->ipc_export(e->eng->plan(), nranks, rank, out); });
    return kIpcHandleBytes;
  } catch (const std::exception& ex) {
    g_gs_err = ex.what();
    return -1;
  }
}
int gs_ipc_connect(gs_engine* e, int32_t dtype, const char* handles, const int64_t* tabs) {
  try {
    with_hip_backend(e, dtype, [&](auto* b) { b->ipc_connect(e->eng->plan(), handles, tabs); });
    return 0;
  } catch (const std::exception& ex) {
    g_gs_err = ex.what();
    return -1;
  }
}

// The IPC peers this engine mapped: out = cap x {rank, device (-1: not visible in this
// process), peer access (1: hipDeviceCanAccessPeer said yes, -1: not checkable)}; returns the
// count, or -1 on error.
int gs_ipc_peers(gs_engine* e, int32_t dtype, int32_t* out, int32_t cap) {
  try {
    int n = 0;
    with_hip_backend(e, dtype, [&](auto* b) { n = b->ipc_peers(out, cap); });
    return n;
  } catch (const std::exception& ex) {
    g_gs_err = ex.what();
    return -1;
  }
}

// Peer-access matrix of the devices this process sees: out[i * n + j] = 1 if device i can
// access device j's memory (hipDeviceCanAccessPeer; the diagonal is 1).  Returns n, or -1.
int gs_peer_access(int32_t* out, int32_t cap) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return -1;
  if (n * n > cap) return -1;
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) {
      int can = i == j ? 1 : 0;
      if (i != j && hipDeviceCanAccessPeer(&can, i, j) != hipSuccess) can = -1;
      out[i * n + j] = can;
    }
  return n;
}

// PCI bus id of the current HIP device ("0000:05:00.0"); returns its length or -1
int gs_device_pci(char* out, int32_t cap) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return -1;
  if (hipDeviceGetPCIBusId(out, cap, dev) != hipSuccess) return -1;
  return (int)strlen(out);
}

int gs_rccl_init(gs_engine* e, const char* uid, int32_t nranks, int32_t rank, int32_t dtype) {
  try {
    ncclUniqueId id;
    memcpy(&id, uid, sizeof(id));
    with_hip_backend(e, dtype, [&](auto* b) { b->init_comm(id, nranks, rank); });
    return 0;
  } catch (const std::exception& ex) {
    g_gs_err = ex.what();
    return -1;
  }
}

}  // extern "C"

extern "C" {

// Select the fused-kernel configuration for fp32 (tuning; "" = measured default).
// Returns -1 for an unknown name.
int gs_fused_select(const char* name) {
  const int k = gsk::fused_cfg_lookup(name);
  if (k < 0) return -1;
  gsk::fused_cfg_slot() = k;
  fused_pinned() = true;
  return 0;
}

}  // extern "C"

extern "C" {

// Select the fused-kernel work schedule (0: even split, 1: XCD-grouped lockstep z-chunks).
int gs_fused_sched(int32_t sched) {
  if (sched < 0 || sched > 2) return -1;
  gsk::fused_sched_slot() = sched;
  fused_pinned() = true;
  return 0;
}

// Back to the autotuned choice (engines created afterwards tune again; tests that pinned a
// configuration call this so later engines in the process are not affected).
int gs_fused_unpin(void) {
  gsk::fused_cfg_slot() = -1;
  (void)gsk::fused_cfg_env();
  gsk::fused_sched_slot() = -1;
  (void)gsk::fused_sched_slot();
  fused_pinned() = false;
  return 0;
}

}  // extern "C"

extern "C" {

// Fused-kernel choice made by the autotuner for depth n: out = {cfg, sched}, ms = timing.
int gs_fused_choice(gs_engine* e, int32_t n, int32_t dtype, int32_t* out2, float* ms) {
  if (n < 0 || n > 4) return -1;
  try {
    int c = -1, s = -1;
    float t = 0.f;
    with_hip_backend(e, dtype, [&](auto* b) { b->fused_choice(n, &c, &s, &t); });
    out2[0] = c;
    out2[1] = s;
    *ms = t;
    return 0;
  } catch (const std::exception& ex) {
    g_gs_err = ex.what();
    return -1;
  }
}

}  // extern "C"

// the gated pass of depth n: out4 = {tuned expected exchange (plane-times, -1: not tuned),
// units, packers, ms per pass measured while tuning}
extern "C" int gs_gate_info(gs_engine* e, int32_t n, int32_t dtype, double* out6) {
  if (n < 0 || n > 3) return -1;
  try {
    with_hip_backend(e, dtype, [&](auto* b) { b->gate_info(n, out6); });
    return 0;
  } catch (const std::exception& ex) {
    g_gs_err = ex.what();
    return -1;
  }
}

// Snapshot events (HipBackend::snapshot): plain timing-disabled HIP events owned by the caller.
extern "C" void* gs_event_create() {
  hipEvent_t ev = nullptr;
  if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) return nullptr;
  return (void*)ev;
}
extern "C" void gs_event_destroy(void* ev) {
  if (ev) (void)hipEventDestroy((hipEvent_t)ev);
}
// wait for an event (the caller's thread; ctypes releases the GIL): 0, or -1 on an error.
// Polled (hipEventQuery + short sleeps), not hipEventSynchronize: the writer thread waits here
// while the stepping thread enqueues its next launches, and a blocking event wait inside the
// runtime stalled those (the output step's snapshot call took ~85 us in the loop vs ~25 us
// alone, scripts/profile_output.py)
// (bounded: a device copy that never completes is an error after GS_COMM_TIMEOUT, like every
// other device wait of the runtime -- the output writer thread's wait_fn, csrc/io/bp4.cpp)
extern "C" int gs_event_sync(void* ev) {
  int sleep_us = 5;
  const auto t0 = std::chrono::steady_clock::now();
  const double tmo = gs::comm_timeout_s();
  for (;;) {
    const hipError_t r = hipEventQuery((hipEvent_t)ev);
    if (r == hipSuccess) return 0;
    if (r != hipErrorNotReady) {
      g_gs_err = std::string("event sync: ") + hipGetErrorString(r);
      return -1;
    }
    if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > tmo) {
      g_gs_err = "event sync: not complete after GS_COMM_TIMEOUT = " + std::to_string(tmo) + " s";
      return -1;
    }
    std::this_thread::sleep_for(std::chrono::microseconds(sleep_us));
    if (sleep_us < 50) sleep_us *= 2;
  }
}
extern "C" int gs_snapshot(gs_engine* e, int32_t dtype, void* du, void* dv, void* dpart, int32_t cap,
                           void* hu, void* hv, void* hpart, void* io, void* prev, void* ready,
                           void* done) {
  try {
    int n = 0;
    with_hip_backend(e, dtype, [&](auto* b) {
      n = b->snapshot(e->eng->cur(), du, dv, dpart, cap, hu, hv, hpart, (hipStream_t)io,
                      (hipEvent_t)prev, (hipEvent_t)ready, (hipEvent_t)done);
    });
    return n;
  } catch (const std::exception& ex) {
    g_gs_err = ex.what();
    return -1;
  }
}

extern "C" int gs_gate_stamps(gs_engine* e, int32_t dtype, double* out8) {
  try {
    with_hip_backend(e, dtype, [&](auto* b) { b->gate_stamps(out8); });
    return 0;
  } catch (const std::exception& ex) {
    g_gs_err = ex.what();
    return -1;
  }
}

extern "C" const char* gs_fused_cfg_name(int32_t index) {
  int n = 0;
  const gsk::FusedCfgEntry* t = gsk::fused_cfg_table(&n);
  return (index >= 0 && index < n) ? t[index].name : nullptr;
}

// index of a fused-kernel configuration name in this build (-1: unknown, e.g. an ablation
// variant in the production library)
extern "C" int gs_fused_cfg_lookup(const char* name) { return gsk::fused_cfg_lookup(name); }
#include "probe.hpp"
