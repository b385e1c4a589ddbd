// SPDX-License-Identifier: MIT
// C ABI shared by libgs_core.so (CPU/OpenMP backend) and libgs_hip.so (gfx950 backend).
// Python binds both through ctypes (grayscott_amd/ops/native.py); the CLI tools link them.
#pragma once

#include <stdint.h>
#include "gs/common.h"

extern "C" {

typedef struct gs_engine gs_engine;

// Create an engine over caller-owned buffers.  buf0/buf1: the two (u,v) state buffers
// (gs::total_elems(g) pairs each).  sendbuf/recvbuf: packed halo buffers (plan sizes, may
// be NULL when the rank has no neighbour).  stream: hipStream_t for the HIP backend.
gs_engine* gs_create(int32_t dtype, const gs::Geom* g, const gs::Params* p, const int32_t* nbr27,
                     int32_t rank, int32_t fuse, int32_t use_fused, void* buf0, void* buf1,
                     void* sendbuf, void* recvbuf, void* stream);
void gs_destroy(gs_engine* e);
const char* gs_last_error(void);

int gs_init_fields(gs_engine* e);
int gs_prepare(gs_engine* e);  // autotune the fused kernel (state unchanged)
int gs_set_overlap(gs_engine* e, int32_t mode);  // -1 auto, 0 off, 1 on
int gs_set_loopback(gs_engine* e, int32_t on);  // self messages via the device transport
int gs_overlapped(gs_engine* e, int32_t k);      // 1 if a k-step pass overlaps its exchange
int gs_chained(gs_engine* e, int32_t k);         // 1 if runs of k-step passes are chained on two streams
int gs_set_gated(gs_engine* e, int32_t on);      // allow (1) / forbid (0) gated passes
int gs_set_gated_depth(gs_engine* e, int32_t k, int32_t on);  // the same for depth k only
int gs_gate_plan(const gs::Geom* g, const int32_t* nbr27, int32_t n, int32_t xp, int32_t allpk,
                 int32_t slots, int32_t longest, int32_t rows, int32_t waves, int32_t fold,
                 int32_t pairs, int32_t unpack, int32_t* out, int32_t cap, int32_t* npk,
                 int32_t* grid_out);  // gs/gate_plan.h
int gs_gated(gs_engine* e, int32_t k);           // 1 if k-step passes carry the exchange in-kernel (gate.hpp)
int gs_depth(gs_engine* e);                      // steps per pass (fuse, or the measured depth)
int gs_set_auto_depth(gs_engine* e, int32_t on);  // let prepare() pick the depth (single rank)
int gs_set_plan(gs_engine* e, int32_t on);        // pass-depth planner on (default) / off (greedy)
// the pass depths advance(nsteps) would run (engine.h plan_passes; 0: the greedy schedule); at
// most cap written, the plan's length returned
int gs_plan_passes(gs_engine* e, int64_t nsteps, int32_t* out, int32_t cap);
// gs::plan_depths for given pass times cost[0..kmax] (cost[k]: depth k; kmax <= 7)
int gs_plan_depths(const double* cost, int32_t kmax, int64_t nsteps, int32_t* out, int32_t cap);
// the same with the outer-ghost refresh priced: `fill` per depth-parity switch, pp the parity a
// first pass needs to avoid one (-1: none)
int gs_plan_depths_bc(const double* cost, int32_t kmax, int64_t nsteps, double fill, int32_t pp,
                      int32_t* out, int32_t cap);
double gs_fill_ms(gs_engine* e);                 // one refresh as timed by prepare (ms)
int gs_plan_zplanes(gs_engine* e);               // 1 if halos are whole contiguous z planes
int gs_fused_runs_raw(gs_engine* e, int32_t k, int32_t zlo0, int32_t zlen0, int32_t zlo1,
                      int32_t zlen1, int32_t mask, int32_t leave_room);  // timing (state unchanged)
// variant: -1 the tuned choice, 0 all faces through k_slab, 1 z faces through k_fused
int gs_shell_raw(gs_engine* e, int32_t k, int32_t sides, int32_t variant);
int gs_advance(gs_engine* e, int64_t nsteps);
int gs_exchange(gs_engine* e);
int64_t gs_get_step(gs_engine* e);
int gs_set_step(gs_engine* e, int64_t t);
int gs_current_buffer(gs_engine* e);
int gs_sync(gs_engine* e);
int gs_extract(gs_engine* e, void* u, void* v);
int gs_extract_minmax(gs_engine* e, void* u, void* v, void* part, int32_t cap);
int gs_insert(gs_engine* e, const void* u, const void* v);
int gs_stats(gs_engine* e, double* out6);
// random interior u, v ~ U[lo, hi) keyed on the global cell (any decomposition: same state)
int gs_randomize(gs_engine* e, uint64_t seed, double lo, double hi);
int gs_set_transport(gs_engine* e, int (*fn)(void*), void* user);
int gs_drop_transport(gs_engine* e);  // forget RCCL / IPC / callback transport (fallback)
// per-phase timing window (gs/phase.h): summary of gs_prof_len() doubles
int gs_prof_len(void);
int gs_debug_set(const char* name, double value);  // test switches (gs/debug.h)
int gs_phase_count(void);
const char* gs_phase_name(int32_t i);
int gs_prof_start(gs_engine* e, int32_t max_records);
int gs_prof_stop(gs_engine* e, double* out);  // 0 ok, 1 records dropped, -1 error
// halo plan introspection: counts and per-message (dir, peer, offset, cells)
int gs_plan_info(gs_engine* e, int64_t* send_cells, int64_t* recv_cells, int32_t* nsend, int32_t* nrecv);
int gs_plan_msg(gs_engine* e, int32_t which, int32_t i, int64_t* out4);

// helpers usable without an engine
int64_t gs_geom_total_elems(const gs::Geom* g);
void gs_make_geom(gs::Geom* out, int nx, int ny, int nz, int H, int64_t ox, int64_t oy, int64_t oz,
                  int64_t Lx, int64_t Ly, int64_t Lz, int periodic);
void gs_noise_block(int64_t gx, int64_t gy4, int64_t gz, int64_t Lx, int64_t Ly, uint64_t step,
                    uint64_t seed, uint32_t* out4);
int gs_plan_sizes(const gs::Geom* g, const int32_t* nbr27, int32_t diagonals, int64_t* send_cells,
                  int64_t* recv_cells);
}
