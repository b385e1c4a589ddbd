// SPDX-License-Identifier: MIT
// gfx950 kernels for the Gray-Scott engine (included by backend_hip.hip only).
#pragma once

#include <hip/hip_runtime.h>

#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <utility>

#include "gs/common.h"
#include "gs/debug.h"
#include "gs/gate_plan.h"

namespace gsk {

using gs::Box;
using gs::Geom;

template <typename T> struct Vec2;
template <> struct Vec2<float> { using type = float2; };
template <> struct Vec2<double> { using type = double2; };

__device__ __forceinline__ int64_t wrap(int64_t a, int64_t L) {
  return a < 0 ? a + L : (a >= L ? a - L : a);
}

// ------------------------------------------------------------------------------------------
// fills / seed
// ------------------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void k_fill(typename Vec2<T>::type* __restrict__ f, Geom g, Box b,
                                              T u, T v) {
  const int64_t n = gs::box_cells(b);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int x = (int)(i % b.nx);
    const int64_t r = i / b.nx;
    const int y = (int)(r % b.ny);
    const int z = (int)(r / b.ny);
    typename Vec2<T>::type c;
    c.x = u;
    c.y = v;
    f[gs::lin(g, b.x0 + x, b.y0 + y, b.z0 + z)] = c;
  }
}

template <typename T>
void launch_fill(typename Vec2<T>::type* f, const Geom& g, const Box& b, T u, T v, hipStream_t s) {
  const int64_t n = gs::box_cells(b);
  const int blocks = (int)std::min<int64_t>((n + 255) / 256, 8192);
  k_fill<T><<<blocks, 256, 0, s>>>(f, g, b, u, v);
}

// up to 6 boxes in one launch (blockIdx.y = box): the outer ghost faces of a buffer
struct FillBoxes {
  Box box[6];
};

template <typename T>
__global__ __launch_bounds__(256) void k_fill_boxes(typename Vec2<T>::type* __restrict__ f, Geom g,
                                                    FillBoxes bs, T u, T v) {
  const Box b = bs.box[blockIdx.y];
  const uint32_t n = (uint32_t)gs::box_cells(b);  // a ghost face of one sub-domain: < 2^31
  const uint32_t bnx = (uint32_t)b.nx, bny = (uint32_t)b.ny;
  typename Vec2<T>::type c;
  c.x = u;
  c.y = v;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const uint32_t r = i / bnx;
    const uint32_t z = r / bny;
    f[gs::lin(g, b.x0 + (int)(i - r * bnx), b.y0 + (int)(r - z * bny), b.z0 + (int)z)] = c;
  }
}

template <typename T>
void launch_fill_boxes(typename Vec2<T>::type* f, const Geom& g, const Box* boxes, int n, T u, T v,
                       hipStream_t s) {
  FillBoxes bs{};
  int64_t mx = 0;
  for (int i = 0; i < n; ++i) {
    bs.box[i] = boxes[i];
    mx = std::max<int64_t>(mx, gs::box_cells(boxes[i]));
  }
  if (n <= 0 || mx == 0) return;
  const int bx = (int)std::max<int64_t>(1, std::min<int64_t>((mx + 255) / 256, 2048));
  k_fill_boxes<T><<<dim3(bx, n, 1), 256, 0, s>>>(f, g, bs, u, v);
}

template <typename T>
void launch_seed(typename Vec2<T>::type* f, const Geom& g, hipStream_t s) {
  // global cube [L/2-6, L/2+6]^3 clipped to this rank
  const int64_t L[3] = {g.Lx, g.Ly, g.Lz};
  const int64_t o[3] = {g.ox, g.oy, g.oz};
  const int n[3] = {g.nx, g.ny, g.nz};
  int lo[3], cnt[3];
  for (int a = 0; a < 3; ++a) {
    const int64_t mn = L[a] / 2 - 6, mx = L[a] / 2 + 6;
    const int64_t l = std::max<int64_t>(mn, o[a]) - o[a];
    const int64_t h = std::min<int64_t>(mx + 1, o[a] + n[a]) - o[a];
    lo[a] = (int)l;
    cnt[a] = h > l ? (int)(h - l) : 0;
  }
  Box b{lo[0], lo[1], lo[2], cnt[0], cnt[1], cnt[2]};
  if (gs::box_cells(b) == 0) return;
  launch_fill<T>(f, g, b, (T)0.25, (T)0.33, s);
}

#include "stencil.hpp"
#include "slab.hpp"

// ------------------------------------------------------------------------------------------
// halo pack / unpack: all messages in one launch (blockIdx.y = message)
// ------------------------------------------------------------------------------------------
struct PackArgs {
  Box box[gs::kMaxMsgs];
  // each message's packed cells: a local send / receive buffer, or (IPC transport) the
  // landing buffer of the peer that receives it, mapped into this process
  void* ptr[gs::kMaxMsgs];
  // first workgroup of each message (prefix sum of its share), n messages, kPackItems cells
  // per thread: the grid is sized by the messages' cells, not (largest message) x (count)
  int32_t b0[gs::kMaxMsgs + 1];
  int32_t n;
  // PACK into peer memory (IPC): every wave waits for its stores to the peer's landing buffer
  // to be acknowledged before it ends (s_waitcnt 0), so they are complete before the ready flag
  // can be published.  Not a system-scope fence: the landing buffer is uncached, so no L2
  // line holds them, while __threadfence_system() writes back every XCD's dirty L2 lines --
  // the fused kernel's output -- once per wave (+80 us per exchange on the loopback,
  // profiles/r3_ipc_fence.txt)
  int32_t fence;
  // PACK into peer memory (IPC): bit m set -> message m's stores carry system coherence
  // (relaxed system-scope atomic stores, global_store ... sc0 sc1: written through to the
  // memory of the receiving GPU, not held in any cache on the way).  Set for every message to
  // a peer on another device (or one whose device this process cannot identify); stores to a
  // landing buffer on this device stay plain (uncached memory, same agent).
  uint32_t sysmask;
  // unpack from a landing buffer (IPC): a nonzero device word (a timed-out wait) makes the
  // unpack write NaN ghosts instead of the stale landing data
  const int* err;
};

constexpr int kPackItems = 4;

// Gather (PACK) or scatter every halo message of a plan in one launch.  Workgroup -> message by
// the prefix table (a uniform scan over <= 26 entries), then kPackItems cells per thread, 256
// consecutive cells per pass so a row's cells go to neighbouring lanes.  Sizing the grid by
// the total cell count matters: one workgroup row per message at the largest message's size
// launched ~20k mostly empty workgroups for a 256^3 rank and took ~10 us per pack / unpack.
// one workgroup's kPackItems x 256 cells: workgroup `blk` of the prefix table
// a cell stored with system coherence, as 8-byte relaxed system-scope atomic stores (vector
// stores with the sc0 sc1 bits: no cache on the way holds them)
template <typename V>
__device__ __forceinline__ void store_system(V* p, const V& c) {
  static_assert(sizeof(V) % 8 == 0, "8-byte words");
  const uint64_t* w = reinterpret_cast<const uint64_t*>(&c);
  uint64_t* d = reinterpret_cast<uint64_t*>(p);
#pragma unroll
  for (int i = 0; i < (int)(sizeof(V) / 8); ++i)
    __hip_atomic_store(d + i, w[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

template <typename T, bool PACK, int ITEMS = kPackItems>
__device__ __forceinline__ void pack_block(typename Vec2<T>::type* __restrict__ f, const Geom& g,
                                           const PackArgs& a, int blk, bool poison) {
  int m = 0;
  while (m + 1 < a.n && blk >= a.b0[m + 1]) ++m;
  const Box b = a.box[m];
  typename Vec2<T>::type* __restrict__ p = (typename Vec2<T>::type*)a.ptr[m];
  // a message box holds < 2^31 cells (halo slabs of one sub-domain): 32-bit index math
  // (the 64-bit divisions dominated this kernel)
  const uint32_t n = (uint32_t)gs::box_cells(b);
  const uint32_t bnx = (uint32_t)b.nx, bny = (uint32_t)b.ny;
  const uint32_t base = (uint32_t)(blk - a.b0[m]) * (256u * ITEMS) + threadIdx.x;
  // all loads first (ITEMS in flight per lane), then the stores
  const bool sys = PACK && ((a.sysmask >> m) & 1u);  // uniform: one message per workgroup
  typename Vec2<T>::type c[ITEMS];
  int64_t jj[ITEMS];
#pragma unroll
  for (int k = 0; k < ITEMS; ++k) {
    const uint32_t i = base + 256u * k;
    const uint32_t r = i / bnx;
    const int x = (int)(i - r * bnx);
    const uint32_t z = r / bny;
    const int y = (int)(r - z * bny);
    jj[k] = gs::lin(g, b.x0 + x, b.y0 + y, b.z0 + (int)z);
    if (i < n) c[k] = PACK ? f[jj[k]] : p[i];
    if (!PACK && poison) c[k].x = c[k].y = __builtin_nan("");
  }
#pragma unroll
  for (int k = 0; k < ITEMS; ++k) {
    const uint32_t i = base + 256u * k;
    if (i < n) {
      if (PACK && sys) store_system(p + i, c[k]);
      else if (PACK) p[i] = c[k];
      else f[jj[k]] = c[k];
    }
  }
}

template <typename T, bool PACK, int ITEMS = kPackItems>
__global__ __launch_bounds__(256) void k_pack(typename Vec2<T>::type* __restrict__ f,
                                              Geom g, PackArgs a) {
  // a timed-out IPC wait: poison the ghosts (wave-uniform load of a device word)
  const bool poison = !PACK && a.err && __hip_atomic_load(a.err, __ATOMIC_RELAXED,
                                                          __HIP_MEMORY_SCOPE_AGENT) != 0;
  pack_block<T, PACK, ITEMS>(f, g, a, (int)blockIdx.x, poison);
  if (PACK && a.fence) __builtin_amdgcn_s_waitcnt(0);
}

// msgs[i]'s packed cells live at ptrs[i] (any mix of local and peer-mapped buffers)
template <typename T, bool PACK, int ITEMS = kPackItems>
void launch_pack_ptrs(typename Vec2<T>::type* f, typename Vec2<T>::type* const* ptrs,
                      const Geom& g, const gs::HaloMsg* msgs, int n, hipStream_t st,
                      bool fence = false, const int* err = nullptr, uint32_t sysmask = 0) {
  PackArgs a;
  a.n = n;
  a.fence = fence ? 1 : 0;
  a.sysmask = sysmask;
  a.err = err;
  int32_t nb = 0;
  for (int i = 0; i < n; ++i) {
    a.box[i] = msgs[i].box;
    a.ptr[i] = ptrs[i];
    a.b0[i] = nb;
    const int64_t c = gs::box_cells(msgs[i].box);
    nb += (int32_t)std::max<int64_t>(1, (c + 256 * ITEMS - 1) / (256 * ITEMS));
  }
  a.b0[n] = nb;
  if (nb == 0) return;
  k_pack<T, PACK, ITEMS><<<dim3(nb, 1, 1), 256, 0, st>>>(f, g, a);
}

// msgs[i]'s packed cells at buf + msgs[i].offset (the plan's send / receive buffer layout)
template <typename T, bool PACK>
void launch_pack(typename Vec2<T>::type* f, typename Vec2<T>::type* buf, const Geom& g,
                 const gs::HaloMsg* msgs, int n, hipStream_t st) {
  typename Vec2<T>::type* ptrs[gs::kMaxMsgs];
  for (int i = 0; i < n; ++i) ptrs[i] = buf + msgs[i].offset;
  launch_pack_ptrs<T, PACK>(f, ptrs, g, msgs, n, st);
}

// ------------------------------------------------------------------------------------------
// IPC peer-write transport: sequence flags in uncached (fine-grained) memory shared between the
// ranks of a node.  The signal-wait kernel publishes one sequence number per peer flag with
// system-scope release stores (vector stores; every wave of the pack kernel before it on the
// stream waited for its uncached peer stores to be acknowledged, k_pack `fence`), then polls up to
// kMaxMsgs flags until each reaches its target (system-scope acquire loads, one lane per flag)
// or until `ticks` of the 100 MHz wall clock have passed -- then it reports through a
// host-mapped word (the watchdog) and a device word (the following unpack writes NaN) and
// exits, so a dead peer never leaves a wave spinning.
// ------------------------------------------------------------------------------------------
struct IpcFlags {
  uint64_t* f[gs::kMaxMsgs];
  uint64_t want[gs::kMaxMsgs];
  int32_t n;
};

// lane i < a.n polls flag i until it reaches its target or `ticks` have passed since t0
__device__ __forceinline__ void ipc_poll(const IpcFlags& a, uint64_t t0, uint64_t ticks, int* err,
                                         int* dflag) {
  const int i = threadIdx.x;
  if (i >= a.n) return;
  while (__hip_atomic_load(a.f[i], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < a.want[i]) {
    if (wall_clock64() - t0 > ticks) {
      __hip_atomic_store(dflag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return;
    }
    __builtin_amdgcn_s_sleep(2);
  }
}

// signal, then wait, in one launch (the pack -> signal -> wait -> unpack chain of one exchange
// has one launch fewer); signalling first keeps two ranks waiting on each other deadlock-free
//   min_ticks > 0 (debug switch ipc_emulate_us, gs/debug.h; modelling only): the launch also lasts at least that long,
//   so a one-GPU loopback run can stand in for a slower inter-GPU link when timing overlap
[[maybe_unused]] static __global__ __launch_bounds__(64) void k_ipc_signal_wait(
    IpcFlags s, IpcFlags w, uint64_t ticks, int* err, int* dflag, uint64_t min_ticks) {
  const int i = threadIdx.x;
  const uint64_t t0 = wall_clock64();
  if (i < s.n) __hip_atomic_store(s.f[i], s.want[i], __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  if (min_ticks && i == 0)
    while (wall_clock64() - t0 < min_ticks) __builtin_amdgcn_s_sleep(1);
  ipc_poll(w, t0, ticks, err, dflag);
}

// ------------------------------------------------------------------------------------------
// ghost-stripped interior <-> contiguous (z,y,x) arrays (get_fields, Simulation_CPU.jl:125)
// ------------------------------------------------------------------------------------------
template <typename T, bool EXTRACT>
__global__ __launch_bounds__(256) void k_interior(typename Vec2<T>::type* __restrict__ f,
                                                  T* __restrict__ u, T* __restrict__ v, Geom g) {
  const int x = blockIdx.x * 256 + threadIdx.x;
  const int y = blockIdx.y;
  const int z = blockIdx.z;
  if (x >= g.nx) return;
  const int64_t j = gs::lin(g, x, y, z);
  const int64_t o = ((int64_t)z * g.ny + y) * g.nx + x;
  if (EXTRACT) {
    const typename Vec2<T>::type c = f[j];
    if (u) u[o] = c.x;
    if (v) v[o] = c.y;
  } else {
    typename Vec2<T>::type c;
    c.x = u[o];
    c.y = v[o];
    f[j] = c;
  }
}

// decomposition-invariant random interior (gs::random_init_cell), one thread per cell
template <typename T>
__global__ __launch_bounds__(256) void k_randomize(typename Vec2<T>::type* __restrict__ f, Geom g,
                                                   uint64_t seed, double lo, double hi) {
  const int x = blockIdx.x * 256 + threadIdx.x;
  const int y = blockIdx.y;
  const int z = blockIdx.z;
  if (x >= g.nx) return;
  double u, v;
  gs::random_init_cell(g.ox + x, g.oy + y, g.oz + z, g.Lx, g.Ly, seed, lo, hi, &u, &v);
  typename Vec2<T>::type c;
  c.x = (T)u;
  c.y = (T)v;
  f[gs::lin(g, x, y, z)] = c;
}

template <typename T>
void launch_randomize(typename Vec2<T>::type* f, const Geom& g, uint64_t seed, double lo,
                      double hi, hipStream_t st) {
  dim3 grid((g.nx + 255) / 256, g.ny, g.nz);
  k_randomize<T><<<grid, 256, 0, st>>>(f, g, seed, lo, hi);
}

template <typename T>
void launch_extract(const typename Vec2<T>::type* f, T* u, T* v, const Geom& g, hipStream_t st) {
  dim3 grid((g.nx + 255) / 256, g.ny, g.nz);
  k_interior<T, true><<<grid, 256, 0, st>>>(const_cast<typename Vec2<T>::type*>(f), u, v, g);
}
// Output snapshot with the BP4 block characteristics (SURVEY K14 + the writer's min / max): the
// ghost-free copy of u and v AND each workgroup's min / max of both, so the host writer does not
// scan the arrays again (a single-thread pass over 2 x 1 MB took ~75 us per field of the
// reference example's output step, profiles/r5_output.txt).  Grid (ceil(nx / 256), G): workgroup
// (bx, by) takes x columns bx*256 .. +255 of rows by, by + G, ... (row = y + ny * z); partials:
// 4 values (u min, u max, v min, v max) per workgroup, reduced on the host (fmin / fmax: exact,
// order-independent; a NaN is skipped).
constexpr int kMinMaxRows = 1024;

template <typename T>
__global__ __launch_bounds__(256) void k_extract_mm(const typename Vec2<T>::type* __restrict__ f,
                                                    T* __restrict__ u, T* __restrict__ v, Geom g,
                                                    T* __restrict__ part) {
  const int x = blockIdx.x * 256 + threadIdx.x;
  const int rows = g.ny * g.nz;
  const T inf = (T)INFINITY;
  T a = inf, b = -inf, c = inf, d = -inf;
  if (x < g.nx) {
    for (int r = blockIdx.y; r < rows; r += gridDim.y) {
      const int z = r / g.ny, y = r - z * g.ny;
      const typename Vec2<T>::type e = f[gs::lin(g, x, y, z)];
      const int64_t o = (int64_t)r * g.nx + x;
      u[o] = e.x;
      v[o] = e.y;
      a = fmin(a, e.x); b = fmax(b, e.x);
      c = fmin(c, e.y); d = fmax(d, e.y);
    }
  }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) {
    a = fmin(a, __shfl_xor(a, m)); b = fmax(b, __shfl_xor(b, m));
    c = fmin(c, __shfl_xor(c, m)); d = fmax(d, __shfl_xor(d, m));
  }
  __shared__ T w[4][4];
  const int wave = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { w[wave][0] = a; w[wave][1] = b; w[wave][2] = c; w[wave][3] = d; }
  __syncthreads();
  if (threadIdx.x < 4) {
    const int k = threadIdx.x;
    T r = w[0][k];
    for (int i = 1; i < 4; ++i) r = (k & 1) ? fmax(r, w[i][k]) : fmin(r, w[i][k]);
    part[4 * ((int64_t)blockIdx.y * gridDim.x + blockIdx.x) + k] = r;
  }
}

// returns the number of partial quadruples written (at most `cap`)
template <typename T>
int launch_extract_mm(const typename Vec2<T>::type* f, T* u, T* v, const Geom& g, T* part,
                      int cap, hipStream_t st) {
  const int gx = (g.nx + 255) / 256;
  const int rows = g.ny * g.nz;
  int gy = std::min(rows, kMinMaxRows);
  gy = std::max(1, std::min(gy, cap / std::max(1, gx)));
  if (gx * gy > cap || rows < 1) return -1;
  k_extract_mm<T><<<dim3(gx, gy), 256, 0, st>>>(f, u, v, g, part);
  return gx * gy;
}

template <typename T>
void launch_insert(typename Vec2<T>::type* f, const T* u, const T* v, const Geom& g, hipStream_t st) {
  dim3 grid((g.nx + 255) / 256, g.ny, g.nz);
  k_interior<T, false><<<grid, 256, 0, st>>>(f, const_cast<T*>(u), const_cast<T*>(v), g);
}

// ------------------------------------------------------------------------------------------
// diagnostics: per-block partial sum/min/max of u and v (off the hot path)
// ------------------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void k_stats(const typename Vec2<T>::type* __restrict__ f, Geom g,
                                               double* __restrict__ out) {
  __shared__ double sh[6][256];
  double su = 0, sv = 0, mnu = 1e300, mxu = -1e300, mnv = 1e300, mxv = -1e300;
  const int64_t n = (int64_t)g.nx * g.ny * g.nz;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int x = (int)(i % g.nx);
    const int64_t r = i / g.nx;
    const typename Vec2<T>::type c = f[gs::lin(g, x, (int)(r % g.ny), (int)(r / g.ny))];
    const double u = c.x, v = c.y;
    su += u; sv += v;
    mnu = fmin(mnu, u); mxu = fmax(mxu, u);
    mnv = fmin(mnv, v); mxv = fmax(mxv, v);
  }
  const int t = threadIdx.x;
  sh[0][t] = su; sh[1][t] = mnu; sh[2][t] = mxu; sh[3][t] = sv; sh[4][t] = mnv; sh[5][t] = mxv;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (t < w) {
      sh[0][t] += sh[0][t + w];
      sh[3][t] += sh[3][t + w];
      sh[1][t] = fmin(sh[1][t], sh[1][t + w]);
      sh[4][t] = fmin(sh[4][t], sh[4][t + w]);
      sh[2][t] = fmax(sh[2][t], sh[2][t + w]);
      sh[5][t] = fmax(sh[5][t], sh[5][t + w]);
    }
    __syncthreads();
  }
  if (t < 6) out[6 * blockIdx.x + t] = sh[t][0];
}

template <typename T>
void launch_stats(const typename Vec2<T>::type* f, const Geom& g, double* ws, int blocks, hipStream_t st) {
  k_stats<T><<<blocks, 256, 0, st>>>(f, g, ws);
}

#include "gate.hpp"

}  // namespace gsk
