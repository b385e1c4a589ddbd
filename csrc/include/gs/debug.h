// SPDX-License-Identifier: MIT
// Test / modelling switches of the native libraries, set only through the C API
// (gs_debug_set, grayscott_amd.ops.native.debug_set) -- never from the environment, so a stray
// variable on a production node cannot change what the shipped kernels do.
//   overlap_chain   1 (default): full-depth overlapped passes run chained on two streams
//                   (engine.h advance_chained); 0: one overlapped pass at a time (tests of
//                   the unchained path).  Read when an engine is created.
//   philox_generic  0 (default); 1: the fused kernel always takes the 64-bit-counter Philox
//                   path (tests: it equals the 32-bit one bit for bit).
//   ipc_emulate_us  0 (default); > 0: every IPC exchange lasts at least this long (modelling a
//                   slower link on one GPU when timing the overlap).  Read by ipc_export.
//   ipc_system_stores 0 (default); 1: the IPC pack stores every peer-bound message with system
//                   coherence, as it always does for a peer on another GPU (tests of that path
//                   on one GPU).
//   gated           1 (default): full-depth passes over the IPC transport run gated (the exchange
//                   inside the pass's fused launch, csrc/hip/gate.hpp) when every peer runs on
//                   another GPU (or is this rank: loopback); 0: the stream-overlapped /
//                   sequential paths (tests, A/B); 2: also with peer processes on this GPU (tests:
//                   each rank's table then takes its share of the device's workgroup slots, so
//                   every rank's waiting units fit at once).  Read when an engine is created.
//   gate_stamps     0 (default); 1: gated passes record wall-clock stamps of their exchange (first
//                   packer start, last arrival, first / last wait done, last unpack done; read
//                   back by gs_gate_stamps -- scripts/bench_gated.py).  Read when the IPC
//                   transport connects.
//   ipc_pair_same_dir 0 (default); 1: modelling only -- a loopback IPC message lands in the ghost
//                   box of its own direction, so one rank can time a one-sided neighbour set
//                   (+x, +y, +z: a 2x2x2 rank); the values are no wrap.  Read at connect.
//   gate_mode       0 (default): the gated pass's tuner times carried, one-unit and pairs tables;
//                   1: one-unit tables packed at the start only; 2: pairs tables only; 3: carried
//                   one-unit tables only (tests of each kernel path).  Read at tuning.
//   plan_order      0 (default): a planned window runs its deepest passes first (engine.h
//                   plan_passes); 1: shallowest first (A/B of the power ramp inside a short
//                   window).  Read at every advance().
//   plan_fill       1 (default): the planner prices a depth-parity switch at one outer-ghost
//                   refresh (engine.h plan_depths, Engine::fill_ms); 0: refreshes not counted
//                   (A/B).  Read at every advance().
//   cpu_ftz         1 (default): the CPU solver flushes fp32 denormals in its step region
//                   (MXCSR FTZ + DAZ; ~100x faster where the reference example's v field
//                   passes through them); 0: IEEE denormals, the reference's and the GPU's
//                   fp32 behaviour bit for bit (exact-parity runs).  fp64 never flushes.
#pragma once

#include <string.h>

namespace gs {

struct DebugKnobs {
  int overlap_chain = 1;
  int philox_generic = 0;
  double ipc_emulate_us = 0.0;
  int ipc_system_stores = 0;
  int gate_stamps = 0;
  int ipc_pair_same_dir = 0;
  int gate_mode = 0;
  int cpu_ftz = 1;
  int gated = 1;
  int plan_order = 0;
  int plan_fill = 1;
};

inline DebugKnobs& debug_knobs() {
  static DebugKnobs k;
  return k;
}

// 0 on success, -1 for an unknown knob
inline int debug_set(const char* name, double value) {
  DebugKnobs& k = debug_knobs();
  if (!name) return -1;
  if (!strcmp(name, "overlap_chain")) k.overlap_chain = value != 0.0 ? 1 : 0;
  else if (!strcmp(name, "philox_generic")) k.philox_generic = value != 0.0 ? 1 : 0;
  else if (!strcmp(name, "ipc_emulate_us")) k.ipc_emulate_us = value > 0.0 ? value : 0.0;
  else if (!strcmp(name, "ipc_system_stores")) k.ipc_system_stores = value != 0.0 ? 1 : 0;
  else if (!strcmp(name, "gate_stamps")) k.gate_stamps = value != 0.0 ? 1 : 0;
  else if (!strcmp(name, "ipc_pair_same_dir")) k.ipc_pair_same_dir = value != 0.0 ? 1 : 0;
  else if (!strcmp(name, "gate_mode")) k.gate_mode = (int)value;
  else if (!strcmp(name, "cpu_ftz")) k.cpu_ftz = value != 0.0 ? 1 : 0;
  else if (!strcmp(name, "gated")) k.gated = value >= 2.0 ? 2 : (value != 0.0 ? 1 : 0);
  else if (!strcmp(name, "plan_order")) k.plan_order = value != 0.0 ? 1 : 0;
  else if (!strcmp(name, "plan_fill")) k.plan_fill = value != 0.0 ? 1 : 0;
  else return -1;
  return 0;
}

}  // namespace gs
