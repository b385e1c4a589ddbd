// SPDX-License-Identifier: MIT
// Implementation of the C ABI in capi.h.  Included exactly once by each backend library,
// which must define:
//   gs::Backend* gs_make_backend(int32_t dtype, const gs::Geom& g, const gs::Params& p,
//                                void* b0, void* b1, void* send, void* recv, void* stream);
//   void gs_backend_post_create(gs::Engine* e);   // optional hook (may be empty)
#pragma once

#include <stdlib.h>

#include <exception>
#include <string>

#include "gs/capi.h"
#include "gs/engine.h"
#include "gs/gate_plan.h"

gs::Backend* gs_make_backend(int32_t dtype, const gs::Geom& g, const gs::Params& p, void* b0,
                             void* b1, void* send, void* recv, void* stream);

struct gs_engine {
  gs::Engine* eng;
};

static thread_local std::string g_gs_err;

#define GS_TRY(body)                          \
  try {                                       \
    body;                                     \
    return 0;                                 \
  } catch (const std::exception& ex) {        \
    g_gs_err = ex.what();                     \
    return -1;                                \
  }

extern "C" {

const char* gs_last_error(void) { return g_gs_err.c_str(); }

gs_engine* gs_create(int32_t dtype, const gs::Geom* g, const gs::Params* p, const int32_t* nbr27,
                     int32_t rank, int32_t fuse, int32_t use_fused, void* buf0, void* buf1,
                     void* sendbuf, void* recvbuf, void* stream) {
  try {
    gs::EngineConfig c{};
    c.g = *g;
    c.p = *p;
    for (int i = 0; i < 27; ++i) c.nbr[i] = nbr27[i];
    c.rank = rank;
    c.fuse = fuse;
    c.use_fused = use_fused;
    gs::Backend* be = gs_make_backend(dtype, *g, *p, buf0, buf1, sendbuf, recvbuf, stream);
    gs_engine* e = new gs_engine;
    e->eng = new gs::Engine(c, be);
    return e;
  } catch (const std::exception& ex) {
    g_gs_err = ex.what();
    return nullptr;
  }
}

void gs_destroy(gs_engine* e) {
  if (!e) return;
  delete e->eng;
  delete e;
}

int gs_init_fields(gs_engine* e) { GS_TRY(e->eng->init_fields()) }
int gs_prepare(gs_engine* e) { GS_TRY(e->eng->prepare()) }
int gs_set_overlap(gs_engine* e, int32_t mode) { GS_TRY(e->eng->set_overlap(mode)) }
int gs_set_loopback(gs_engine* e, int32_t on) { GS_TRY(e->eng->set_loopback(on != 0)) }
int gs_overlapped(gs_engine* e, int32_t k) { return e->eng->overlapped(k) ? 1 : 0; }
int gs_chained(gs_engine* e, int32_t k) { return e->eng->chained(k) ? 1 : 0; }
int gs_gated(gs_engine* e, int32_t k) { return e->eng->gated(k) ? 1 : 0; }

// The gated pass's unit table (gs/gate_plan.h) for a sub-domain and neighbour set, host only:
// tests check it on the CPU.  out: up to cap units of 6 int32 (tile, z0, z1, pk, wait, prod), so
// it must hold 6 * cap; returns the unit count (may exceed cap), -1 on bad arguments (including a
// tile with no output rows: (rows * waves - 2n) & ~3 <= 0).  grid_out (9 int32): the TileGrid.
// pairs: the two-units-per-workgroup table (xp = the expected exchange X, unpack = U).
int gs_gate_plan(const gs::Geom* g, const int32_t* nbr27, int32_t n, int32_t xp, int32_t allpk,
                 int32_t slots, int32_t longest, int32_t rows, int32_t waves, int32_t fold,
                 int32_t pairs, int32_t unpack, int32_t* out, int32_t cap, int32_t* npk,
                 int32_t* grid_out) {
  if (!g || !nbr27 || n < 1 || n > g->H || rows < 4 || waves < 1) return -1;
  if (((rows * waves - 2 * n) & ~3) <= 0) return -1;  // no output rows: tile_grid's ystep <= 0
  const gs::HaloPlan p = gs::make_halo_plan(*g, nbr27, true);
  const gs::TileGrid tg = gs::tile_grid(rows, waves, fold != 0, *g, n);
  int k = 0;
  const std::vector<gs::GateUnit> u =
      pairs ? gs::gate_plan_pairs(tg, *g, p, n, xp, unpack, allpk != 0, slots, &k)
            : gs::gate_plan(tg, *g, p, n, xp, allpk != 0, slots, longest != 0, &k);
  for (size_t i = 0; i < u.size() && (int64_t)i < cap; ++i) {
    out[6 * i] = u[i].tile;
    out[6 * i + 1] = u[i].z0;
    out[6 * i + 2] = u[i].z1;
    out[6 * i + 3] = u[i].pk;
    out[6 * i + 4] = u[i].wait;
    out[6 * i + 5] = u[i].prod;
  }
  if (npk) *npk = k;
  if (grid_out) {
    const int v[9] = {tg.xstep, tg.ystep, tg.ybase, tg.ntx, tg.nty, tg.ntxf, tg.nfold, tg.ntiles, tg.rt};
    for (int i = 0; i < 9; ++i) grid_out[i] = v[i];
  }
  return (int)u.size();
}
int gs_set_gated(gs_engine* e, int32_t on) {
  e->eng->set_gated(on != 0);
  return 0;
}
int gs_set_gated_depth(gs_engine* e, int32_t k, int32_t on) {
  e->eng->set_gated_depth(k, on != 0);
  return 0;
}
int gs_depth(gs_engine* e) { return e->eng->depth(); }
int gs_set_auto_depth(gs_engine* e, int32_t on) { GS_TRY(e->eng->set_auto_depth(on != 0)) }
int gs_set_plan(gs_engine* e, int32_t on) { GS_TRY(e->eng->set_plan(on != 0)) }
int gs_plan_depths(const double* cost, int32_t kmax, int64_t nsteps, int32_t* out, int32_t cap) {
  if (kmax < 2 || kmax > 7) return -1;
  const std::vector<int> p = gs::plan_depths(cost, kmax, nsteps);
  for (size_t i = 0; i < p.size() && (int32_t)i < cap; ++i) out[i] = p[i];
  return (int)p.size();
}
int gs_plan_depths_bc(const double* cost, int32_t kmax, int64_t nsteps, double fill, int32_t pp,
                      int32_t* out, int32_t cap) {
  if (kmax < 2 || kmax > 7) return -1;
  const std::vector<int> p = gs::plan_depths(cost, kmax, nsteps, fill, pp);
  for (size_t i = 0; i < p.size() && (int32_t)i < cap; ++i) out[i] = p[i];
  return (int)p.size();
}
double gs_fill_ms(gs_engine* e) { return e->eng->fill_ms(); }
int gs_plan_passes(gs_engine* e, int64_t nsteps, int32_t* out, int32_t cap) {
  try {
    const std::vector<int> p = e->eng->plan_passes(nsteps);
    for (size_t i = 0; i < p.size() && (int32_t)i < cap; ++i) out[i] = p[i];
    return (int)p.size();
  } catch (const std::exception& ex) {
    g_gs_err = ex.what();
    return -1;
  }
}
int gs_plan_zplanes(gs_engine* e) { return e->eng->plan().zplanes; }
// Timing primitives: one fused k-step update of the given z-runs (store mask: engine.h
// fused_runs) / of the shell slabs at `sides`, from the current buffer into the other one
// (interior cells only, so the next pass overwrites them; the state is unchanged).
int gs_fused_runs_raw(gs_engine* e, int32_t k, int32_t zlo0, int32_t zlen0, int32_t zlo1,
                      int32_t zlen1, int32_t mask, int32_t leave_room) {
  GS_TRY({
    gs::Engine& g = *e->eng;
    if (!g.backend()->fused_runs(g.cur(), 1 - g.cur(), k, g.step(), zlo0, zlen0, zlo1, zlen1,
                                 leave_room != 0, mask))
      throw std::runtime_error("fused runs unsupported for this k / backend");
  })
}
int gs_shell_raw(gs_engine* e, int32_t k, int32_t sides, int32_t variant) {
  GS_TRY({
    gs::Engine& g = *e->eng;
    if (!g.backend()->shell(g.cur(), 1 - g.cur(), k, g.step(), sides, variant))
      throw std::runtime_error("shell unsupported for this k / backend");
  })
}
int gs_advance(gs_engine* e, int64_t n) { GS_TRY(e->eng->advance(n)) }
int gs_exchange(gs_engine* e) { GS_TRY(e->eng->exchange()) }
int64_t gs_get_step(gs_engine* e) { return e->eng->step(); }
int gs_set_step(gs_engine* e, int64_t t) { GS_TRY(e->eng->set_step(t)) }
int gs_current_buffer(gs_engine* e) { return e->eng->cur(); }
// Waits for all queued work.  GS_COMM_TIMEOUT (seconds, default 900; read at every call) bounds
// the wait when a device transport is active: a hung or failed halo exchange becomes an error,
// not a hang.
int gs_sync(gs_engine* e) { GS_TRY(e->eng->backend()->wait_all(gs::comm_timeout_s())) }
int gs_extract(gs_engine* e, void* u, void* v) {
  GS_TRY(e->eng->backend()->extract(e->eng->cur(), u, v))
}
// extract + per-chunk min / max (Backend::extract_minmax): the number of quadruples written at
// `part` (<= cap), -2 when the backend has no such path, -1 on error
int gs_extract_minmax(gs_engine* e, void* u, void* v, void* part, int32_t cap) {
  try {
    const int n = e->eng->backend()->extract_minmax(e->eng->cur(), u, v, part, cap);
    return n < 0 ? -2 : n;
  } catch (const std::exception& ex) {
    g_gs_err = ex.what();
    return -1;
  }
}
int gs_insert(gs_engine* e, const void* u, const void* v) {
  GS_TRY(e->eng->backend()->insert(e->eng->cur(), u, v))
}
int gs_randomize(gs_engine* e, uint64_t seed, double lo, double hi) {
  GS_TRY(e->eng->randomize(seed, lo, hi))
}
int gs_stats(gs_engine* e, double* out6) { GS_TRY(e->eng->backend()->stats(e->eng->cur(), out6)) }
int gs_set_transport(gs_engine* e, int (*fn)(void*), void* user) {
  GS_TRY(e->eng->set_transport(fn, user))
}
int gs_drop_transport(gs_engine* e) { GS_TRY(e->eng->drop_transport()) }

// Per-phase timing window (gs/phase.h): gs_prof_start(e, max_records) ... steps ...
// gs_prof_stop(e, out) waits for the device and writes gs_prof_len() doubles (layout:
// gs/phase.h kProfHead, then {median us, intervals per pass} per phase in gs_phase_name order).
// gs_prof_stop returns 1 if the window had more records than max_records, 0, or -1 on error.
int gs_prof_len(void) { return gs::kProfLen; }
// test / modelling switches (gs/debug.h); 0, or -1 for an unknown name
int gs_debug_set(const char* name, double value) { return gs::debug_set(name, value); }
int gs_phase_count(void) { return gs::kNumPhases; }
const char* gs_phase_name(int32_t i) { return gs::phase_name(i); }
int gs_prof_start(gs_engine* e, int32_t max_records) { GS_TRY(e->eng->prof_start(max_records)) }
int gs_prof_stop(gs_engine* e, double* out) {
  try {
    return e->eng->prof_stop(out, gs::comm_timeout_s());
  } catch (const std::exception& ex) {
    g_gs_err = ex.what();
    return -1;
  }
}

int gs_plan_info(gs_engine* e, int64_t* sc, int64_t* rc, int32_t* ns, int32_t* nr) {
  const gs::HaloPlan& p = e->eng->plan();
  *sc = p.send_cells; *rc = p.recv_cells; *ns = p.nsend; *nr = p.nrecv;
  return 0;
}

int gs_plan_msg(gs_engine* e, int32_t which, int32_t i, int64_t* out4) {
  const gs::HaloPlan& p = e->eng->plan();
  const gs::HaloMsg* m = which == 0 ? p.send : p.recv;
  const int n = which == 0 ? p.nsend : p.nrecv;
  if (i < 0 || i >= n) return -1;
  out4[0] = m[i].dir; out4[1] = m[i].peer; out4[2] = m[i].offset; out4[3] = gs::box_cells(m[i].box);
  return 0;
}

int64_t gs_geom_total_elems(const gs::Geom* g) { return gs::total_elems(*g); }

void gs_make_geom(gs::Geom* out, int nx, int ny, int nz, int H, int64_t ox, int64_t oy,
                  int64_t oz, int64_t Lx, int64_t Ly, int64_t Lz, int periodic) {
  *out = gs::make_geom(nx, ny, nz, H, ox, oy, oz, Lx, Ly, Lz, periodic);
}

void gs_noise_block(int64_t gx, int64_t gy4, int64_t gz, int64_t Lx, int64_t Ly, uint64_t step,
                    uint64_t seed, uint32_t* out4) {
  gs::U4 r = gs::noise_block(gx, gy4, gz, Lx, Ly, step, seed);
  out4[0] = r.x; out4[1] = r.y; out4[2] = r.z; out4[3] = r.w;
}

int gs_plan_sizes(const gs::Geom* g, const int32_t* nbr27, int32_t diagonals, int64_t* sc,
                  int64_t* rc) {
  gs::HaloPlan p = gs::make_halo_plan(*g, nbr27, diagonals != 0);
  *sc = p.send_cells;
  *rc = p.recv_cells;
  return 0;
}

}  // extern "C"
