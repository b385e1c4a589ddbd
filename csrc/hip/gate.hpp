// SPDX-License-Identifier: MIT
// Gated pass: the halo exchange carried inside the k_fused launch of the pass (IPC transport).
// Included inside namespace gsk at the end of kernels.hpp (it uses store_system and the IPC
// wall clock of the pack / wait kernels above).
//
// The reference exchanges every halo with blocking host Sendrecv! calls and only then computes
// (src/simulation/public.jl:58-64, communication.jl:138-199).  The stream-overlapped pass
// (engine.h: inner launch + k_slab shell) hides the exchange but recomputes the k-deep face
// slabs in a second, latency-bound launch: ~1.4x the full pass on a 2x2x2 rank
// (profiles/r4_shell.txt).  Here a pass is one launch and every output is computed once:
//   * the host splits each tile column into z-chunks, one unit per workgroup (GateUnit);
//     a unit whose level-0 cone reads a ghost cell that a neighbour fills is START-GATED, every
//     other unit marches at once;
//   * start-gated units (or, as tuned, every unit) are the packers: each copies its share of
//     every outgoing message straight into the receiving peer's landing buffer (IPC-mapped;
//     system-coherent stores across devices), waits for its stores to be acknowledged and bumps
//     a device counter; the packer whose add completes the pass's count publishes this
//     exchange's sequence number in every send peer's flag array (gate_pack);
//   * then each start-gated unit polls its own flags until every receive peer has published
//     (a wall-clock bound turns a dead peer into an error, not a hang), copies the ghost cells
//     of its own cone out of its landing slot (cones of neighbouring tiles overlap: a few cells
//     are copied twice, with equal values), drops its L1 and marches (gate_unpack);
//   * the host sizes the chunks so that every workgroup finishes together: gated chunks are
//     shorter by the expected exchange time (tuned on the device, backend_hip.hip gate_tune;
//     the planner is gs/gate_plan.h).  Pairs tables give a workgroup an ungated chunk first and
//     run the wait and unpack between its two marches (k_fused_gated<..., PAIRS>);
//   * carried exchanges (gate_carry): inside a run of passes the producers pack the NEXT
//     exchange from their own outputs at the end of their march, so a pass only unpacks.
// No fence wider than the workgroup runs inside the launch (gfx950: a system release is
// buffer_wbl2, an agent acquire buffer_inv sc1 -- the XCD's whole L2 under the marching
// workgroups): the landing slots and flags are uncached, so nothing the protocol reads can be
// stale in a cache, and every store is acknowledged (s_waitcnt) before the arrival it precedes.
// The same monotonic flags and two landing slots as the stream transport (backend_hip.hip
// ipc_*): exchange n uses slot n & 1; a rank starts packing n only after its previous launch,
// whose gated units waited for every peer's n - 1, so the peers have consumed slot n & 1 (their
// launch n - 2 read it).  Results are bit-identical to the full pass: the arithmetic is k_fused's,
// and chunking never changes a value.
#pragma once

struct GateArgs {
  // outgoing messages: boxes (local interior cells), destination in the receiving peer's landing
  // slot 0 / 1 (mapped into this process), bit m of sysmask: system-coherent stores
  Box sbox[gs::kMaxMsgs];
  void* sdst[2][gs::kMaxMsgs];
  int32_t nsend;
  uint32_t sysmask;
  // incoming messages: ghost boxes (local), their data in this rank's landing slot 0 / 1
  Box rbox[gs::kMaxMsgs];
  const void* rsrc[2][gs::kMaxMsgs];
  int32_t nrecv;
  // sequence flags: this rank's (one per receive peer) and the peers' (one per send peer)
  uint64_t* wflag[gs::kMaxMsgs];
  uint64_t* sflag[gs::kMaxMsgs];
  int32_t nwait, nsig;
  // arrivals of exchange m on word m & 1, monotonic over the engine's gated passes (a launch
  // may count two exchanges: its own start-packed one and the next, carried, one)
  uint32_t* counter;
  // debug knob ipc_emulate_us, carried exchanges: the publisher's wall clock when it published
  // (this rank's word per receive peer / the peers' words per send peer)
  uint64_t* wstamp[gs::kMaxMsgs];
  uint64_t* sstamp[gs::kMaxMsgs];
  uint64_t ticks;      // wall-clock ticks a wait may take (GS_COMM_TIMEOUT)
  uint64_t min_ticks;  // debug knob ipc_emulate_us: the exchange lasts at least this long
  int* err;            // host-mapped: a wait timed out (the watchdog raises)
  int* dflag;          // device copy: later copies write NaN instead of stale landing data
  // debug knob gate_stamps: wall-clock stamps of the launch's exchange (null: none) --
  // [0] min start (packer or waiting unit), [1] max packer arrival, [2] min / [3] max wait
  // done, [4] max unpack done, [5] max / [6] sum of a unit's unpack duration (wait done ->
  // unpack done), [7] units; over all launches since set-up: [8] max / [9] sum of a producer's
  // carry (march done -> arrival), [10] producers
  unsigned long long* stamps;
};

// One message (pack) or the part of one inside a unit's cone (unpack), flattened: the pieces
// of all messages form one index space [0, total), so a thread's cells of EVERY message are in
// flight before its first store.  (On gfx9 the vector memory counter covers loads and stores and
// retires in order: a loop of load -> store per message waits one uncached store / load round
// trip per message -- 26 messages cost 45 us of packing and 25 us of unpacking that way.)
struct GatePiece {
  void* ptr;          // pack: the message's destination; unpack: its data in the landing slot
  int x0, y0, z0;     // first cell (local coordinates)
  int nx, ny;         // extent in x / y (z: until the next piece's start)
  uint32_t start;     // first flat index
  int sx0, sy0, sz0;  // unpack: origin of the message box in the landing slot
  int snx, sny;       //         and its x / y extent
  int sys;            // pack: system-coherent stores (a peer on another GPU)
  float inx, iny;     // 1 / nx, 1 / ny (gate_div)
};

template <typename T>
constexpr int gate_batch() { return sizeof(T) == 4 ? 16 : 8; }  // cells per thread per batch

// q = k / d for k < 2^24 from a float reciprocal (exact after one correction step): the
// flat-index decodes below run per cell, integer division is ~40 instructions
__device__ __forceinline__ uint32_t gate_div(uint32_t k, uint32_t d, float inv) {
  uint32_t q = (uint32_t)((float)k * inv);
  const int32_t r = (int32_t)(k - q * d);
  if (r < 0) --q;
  else if (r >= (int32_t)d) ++q;
  return q;
}

// one arrival (thread 0) at exchange m's counter; the arrival that completes the count publishes
// m in every send peer's flag array.  carried: stamp the publication first (emulated exchange)
__device__ __forceinline__ void gate_arrive(const GateArgs& G, uint64_t m, uint32_t target,
                                            bool carried) {
  const uint32_t old = __hip_atomic_fetch_add(G.counter + (m & 1), 1u, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
  if (old + 1u != target) return;
  if (carried && G.min_ticks) {
    const uint64_t now = wall_clock64();
    for (int i = 0; i < G.nsig; ++i)
      __hip_atomic_store(G.sstamp[i], now, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the stamp lands before the flag
  }
  for (int i = 0; i < G.nsig; ++i)
    __hip_atomic_store(G.sflag[i], m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// 1. pack + arrive: this packer's share of every outgoing message, then its arrival at the
// pass's counter (the last arrival publishes the exchange)
template <typename T>
__device__ __forceinline__ void gate_pack(const FusedArgs& a, int pk) {
  using V2 = typename Vec2<T>::type;
  constexpr int B = gate_batch<T>();
  const GateArgs& G = *a.gate;
  const Geom& g = a.g;
  const int slot = (int)(a.gate_n & 1);
  const uint32_t nt = blockDim.x, tid = threadIdx.x;
  const uint64_t t0 = wall_clock64();
  V2* f = (V2*)a.field;
  __shared__ GatePiece gp[gs::kMaxMsgs];
  __shared__ uint32_t gcells[gs::kMaxMsgs];
  __shared__ uint32_t gtotal;
  __shared__ int gnp;
  // the piece table: one thread per message (their loads of the arguments in parallel), then
  // thread 0 numbers the cells (and drops empty pieces) in LDS
  auto number = [&](int nmsg) {
    __syncthreads();
    if (tid == 0) {
      uint32_t acc = 0;
      int np = 0;
      for (int m = 0; m < nmsg; ++m) {
        if (!gcells[m]) continue;
        if (np != m) gp[np] = gp[m];
        gp[np++].start = acc;
        acc += gcells[m];
      }
      gtotal = acc;
      gnp = np;
    }
    __syncthreads();
  };
  // 1. this packer's share of the outgoing messages: flat cells pk * nt + tid, strided by all
  // packers' threads
  if (tid < (uint32_t)G.nsend) {
    const Box b = G.sbox[tid];
    gp[tid] = GatePiece{G.sdst[slot][tid], b.x0, b.y0, b.z0, b.nx, b.ny, 0u, 0, 0, 0, 0, 0,
                        (int)((G.sysmask >> tid) & 1u), 1.0f / (float)b.nx, 1.0f / (float)b.ny};
    gcells[tid] = (uint32_t)gs::box_cells(b);
  }
  number(G.nsend);
  {
    const uint32_t total = gtotal, stride = (uint32_t)a.gate_npk * nt;
    const int np = gnp;
    const bool small = total < (1u << 24);  // every piece-local index exact in a float
    for (uint32_t i0 = (uint32_t)pk * nt + tid; i0 < total; i0 += B * stride) {
      V2 c[B];
      V2* dst[B];
      int sys[B];
      int m = 0;
#pragma unroll
      for (int j = 0; j < B; ++j) {
        const uint32_t i = i0 + (uint32_t)j * stride;
        dst[j] = nullptr;
        if (i < total) {
          while (m + 1 < np && gp[m + 1].start <= i) ++m;  // i grows with j
          const GatePiece& q = gp[m];
          const uint32_t k = i - q.start;
          const uint32_t r = small ? gate_div(k, (uint32_t)q.nx, q.inx) : k / (uint32_t)q.nx;
          const uint32_t z = small ? gate_div(r, (uint32_t)q.ny, q.iny) : r / (uint32_t)q.ny;
          const int x = (int)(k - r * (uint32_t)q.nx), y = (int)(r - z * (uint32_t)q.ny);
          c[j] = f[gs::lin(g, q.x0 + x, q.y0 + y, q.z0 + (int)z)];
          dst[j] = (V2*)q.ptr + k;
          sys[j] = q.sys;
        }
      }
#pragma unroll
      for (int j = 0; j < B; ++j) {
        if (!dst[j]) continue;
        if (sys[j]) store_system(dst[j], c[j]);
        else *dst[j] = c[j];
      }
    }
  }
  // every wave's stores acknowledged (uncached or system-coherent: no cache holds them), then
  // one arrival per packer; the last one publishes the exchange.  No release fence: on gfx950 a
  // system-scope release writes back the XCD's whole L2 (buffer_wbl2), here full of the marching
  // workgroups' output lines -- and nothing it would write back is part of a message: every
  // packer's landing stores are already acknowledged when its arrival is counted, and the flag
  // store issues after the count (the same ordering as the stream path's pack / signal kernels)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    if (G.stamps) {
      atomicMin(G.stamps + 0, (unsigned long long)t0);
      atomicMax(G.stamps + 1, (unsigned long long)wall_clock64());
    }
    gate_arrive(G, a.gate_n, a.gate_cnt, false);
  }
}

// 2. + 3. wait for the peers' flags and copy the ghost cells of the level-0 cone
// [X0, X0 + xw) x [Y0, Y0 + yext) x [za, zb) out of the landing slot
template <typename T, int BATCH = gate_batch<T>()>
__device__ __forceinline__ void gate_unpack(const FusedArgs& a, int X0, int xw, int Y0, int yext,
                                         int za, int zb, uint64_t t0) {
  using V2 = typename Vec2<T>::type;
  constexpr int B = BATCH;  // (a pairs table's second entry unpacks with the march state live)
  const GateArgs& G = *a.gate;
  const Geom& g = a.g;
  const int slot = (int)(a.gate_n & 1);
  const uint32_t nt = blockDim.x, tid = threadIdx.x;
  V2* f = (V2*)a.field;
  __shared__ GatePiece gp[gs::kMaxMsgs];
  __shared__ uint32_t gcells[gs::kMaxMsgs];
  __shared__ uint32_t gtotal;
  __shared__ int gnp;
  // the piece table: one thread per message (their loads of the arguments in parallel), then
  // thread 0 numbers the cells (and drops empty pieces) in LDS
  auto number = [&](int nmsg) {
    __syncthreads();
    if (tid == 0) {
      uint32_t acc = 0;
      int np = 0;
      for (int m = 0; m < nmsg; ++m) {
        if (!gcells[m]) continue;
        if (np != m) gp[np] = gp[m];
        gp[np++].start = acc;
        acc += gcells[m];
      }
      gtotal = acc;
      gnp = np;
    }
    __syncthreads();
  };
  // the unpack's piece table -- the cone [X0, X0 + xw) x [Y0, Y0 + yext) x [za, zb)'s part of
  // every received message, one flat index space again -- built while the exchange is in
  // flight, so after the flags only the copies remain
  if (tid < (uint32_t)G.nrecv) {
    const Box b = G.rbox[tid];
    const int x0 = max(b.x0, X0), x1 = min(b.x0 + b.nx, X0 + xw);
    const int y0 = max(b.y0, Y0), y1 = min(b.y0 + b.ny, Y0 + yext);
    const int z0 = max(b.z0, za), z1 = min(b.z0 + b.nz, zb);
    const bool any = x0 < x1 && y0 < y1 && z0 < z1;
    gp[tid] = GatePiece{const_cast<void*>(G.rsrc[slot][tid]), x0, y0, z0, x1 - x0, y1 - y0, 0u,
                        b.x0, b.y0, b.z0, b.nx, b.ny, 0, any ? 1.0f / (float)(x1 - x0) : 0.f,
                        any ? 1.0f / (float)(y1 - y0) : 0.f};
    gcells[tid] = any ? (uint32_t)((x1 - x0) * (y1 - y0) * (z1 - z0)) : 0u;
  }
  number(G.nrecv);
  // 2. every receive peer's messages of this exchange have landed (bounded wait).  Relaxed
  // system-scope polls (the flags are uncached: every load reads memory).  No acquire fence (on
  // gfx950 an agent-scope acquire invalidates the XCD's L2, which the marching workgroups
  // stream through): the landing slot is uncached too, so no cache can hold a stale copy of
  // the messages, and the copies below issue only after the polls return.
  const bool carried = (a.gate_pre & 1) != 0;
  if (tid < (uint32_t)G.nwait) {
    uint64_t* w = G.wflag[tid];
    bool ok = true;
    while (__hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < a.gate_n) {
      if (wall_clock64() - t0 > G.ticks) {
        __hip_atomic_store(G.dflag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(G.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        ok = false;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    // emulated exchange, carried: it lands min_ticks after its publication (a later stamp --
    // the peer's next exchange already published -- only lengthens the wait)
    if (ok && carried && G.min_ticks) {
      const uint64_t st = __hip_atomic_load(G.wstamp[tid], __ATOMIC_RELAXED,
                                            __HIP_MEMORY_SCOPE_SYSTEM);
      while ((int64_t)(wall_clock64() - st) < (int64_t)G.min_ticks) __builtin_amdgcn_s_sleep(1);
    }
  }
  // emulated exchange, packed at the start: it lands min_ticks after the unit's start
  if (G.min_ticks && !carried && tid == 0)
    while (wall_clock64() - t0 < G.min_ticks) __builtin_amdgcn_s_sleep(1);
  unsigned long long wdone = 0;
  if (G.stamps && tid == 0) {
    atomicMin(G.stamps + 0, (unsigned long long)t0);
    wdone = (unsigned long long)wall_clock64();
    atomicMin(G.stamps + 2, wdone);
    atomicMax(G.stamps + 3, wdone);
  }
  __syncthreads();
  // 3. the ghost cells of this unit's level-0 cone (piece table built before the wait, above)
  const bool poison = __hip_atomic_load(G.dflag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
  {
    const uint32_t total = gtotal;
    const int np = gnp;
    const bool small = total < (1u << 24);
    for (uint32_t i0 = tid; i0 < total; i0 += B * nt) {
      V2 c[B];
      int64_t o[B];
      int p = 0;
#pragma unroll
      for (int j = 0; j < B; ++j) {
        const uint32_t i = i0 + (uint32_t)j * nt;
        o[j] = -1;
        if (i < total) {
          while (p + 1 < np && gp[p + 1].start <= i) ++p;
          const GatePiece& q = gp[p];
          const uint32_t k = i - q.start;
          const uint32_t r = small ? gate_div(k, (uint32_t)q.nx, q.inx) : k / (uint32_t)q.nx;
          const uint32_t zz = small ? gate_div(r, (uint32_t)q.ny, q.iny) : r / (uint32_t)q.ny;
          const int x = q.x0 + (int)(k - r * (uint32_t)q.nx);
          const int y = q.y0 + (int)(r - zz * (uint32_t)q.ny);
          const int z = q.z0 + (int)zz;
          c[j] = ((const V2*)q.ptr)[((int64_t)(z - q.sz0) * q.sny + (y - q.sy0)) * q.snx +
                                   (x - q.sx0)];
          o[j] = gs::lin(g, x, y, z);
        }
      }
#pragma unroll
      for (int j = 0; j < B; ++j) {
        if (o[j] < 0) continue;
        V2 v = c[j];
        if (poison) v.x = v.y = __builtin_nan("");
        f[o[j]] = v;
      }
    }
  }
  // the march's loads (other waves' cells too) come after every wave's ghost stores; and this
  // CU's L1 forgets the lines the packing loaded: an interior cache line next to a face also
  // holds ghost cells, stale ones from before the copies above (buffer_inv sc0: L1 only)
  asm volatile("s_waitcnt vmcnt(0)\n\tbuffer_inv sc0" ::: "memory");
  __syncthreads();
  if (G.stamps && tid == 0) {
    const unsigned long long u = (unsigned long long)wall_clock64();
    atomicMax(G.stamps + 4, u);
    atomicMax(G.stamps + 5, u - wdone);
    atomicAdd(G.stamps + 6, u - wdone);
    atomicAdd(G.stamps + 7, 1ull);
  }
  // a pass that carries the next exchange: this unit is done with landing slot gate_n & 1, so
  // the peers may fill it again (exchange gate_n + 2) once the next exchange is published
  if ((a.gate_pre & 2) && tid == 0) gate_arrive(G, a.gate_n + 1, a.gate_cnt2, true);
}

// 4. carried exchange (a.gate_pre & 2): at the end of its march, a producer unit copies its own
// outputs [ox0, ox1) x [oy0, oy1) x [z0, z1) that lie in an outgoing message -- the next
// exchange's data, final now -- into the peers' landing slot (gate_n + 1) & 1 and arrives; the
// producers' output boxes cover every message once (gs/gate_plan.h gate_mark_producers).  The
// next pass then finds its exchange published at its start: no pack, no wait for the peers'
// packers, only the cone unpack.  Slot reuse: a producer is a start-gated unit (symmetric
// neighbours), so it has seen the peers publish gate_n, which they do only after every unit
// of theirs that read slot gate_n + 1 & 1 (exchange gate_n - 1) arrived (gate_unpack above).
template <typename T>
__device__ __forceinline__ void gate_carry(const FusedArgs& a, const void* dv, int ox0, int ox1,
                                           int oy0, int oy1, int z0, int z1) {
  using V2 = typename Vec2<T>::type;
  constexpr int B = gate_batch<T>();
  const GateArgs& G = *a.gate;
  const Geom& g = a.g;
  const V2* d = (const V2*)dv;
  const uint64_t m = a.gate_n + 1;
  const uint64_t tc0 = wall_clock64();
  const int slot = (int)(m & 1);
  const uint32_t nt = blockDim.x, tid = threadIdx.x;
  __shared__ GatePiece gp[gs::kMaxMsgs];
  __shared__ uint32_t gcells[gs::kMaxMsgs];
  __shared__ uint32_t gtotal;
  __shared__ int gnp;
  // this workgroup's output stores acknowledged (then in its XCD's L2) before they are read
  // back; the CU's L1 forgets what it held
  asm volatile("s_waitcnt vmcnt(0)\n\tbuffer_inv sc0" ::: "memory");
  if (tid < (uint32_t)G.nsend) {
    const Box b = G.sbox[tid];
    const int x0 = max(b.x0, ox0), x1 = min(b.x0 + b.nx, ox1);
    const int y0 = max(b.y0, oy0), y1 = min(b.y0 + b.ny, oy1);
    const int zz0 = max(b.z0, z0), zz1 = min(b.z0 + b.nz, z1);
    const bool any = x0 < x1 && y0 < y1 && zz0 < zz1;
    gp[tid] = GatePiece{G.sdst[slot][tid], x0, y0, zz0, x1 - x0, y1 - y0, 0u, b.x0, b.y0, b.z0,
                        b.nx, b.ny, (int)((G.sysmask >> tid) & 1u),
                        any ? 1.0f / (float)(x1 - x0) : 0.f, any ? 1.0f / (float)(y1 - y0) : 0.f};
    gcells[tid] = any ? (uint32_t)((x1 - x0) * (y1 - y0) * (zz1 - zz0)) : 0u;
  }
  __syncthreads();
  if (tid == 0) {
    uint32_t acc = 0;
    int np = 0;
    for (int i = 0; i < G.nsend; ++i) {
      if (!gcells[i]) continue;
      if (np != i) gp[np] = gp[i];
      gp[np++].start = acc;
      acc += gcells[i];
    }
    gtotal = acc;
    gnp = np;
  }
  __syncthreads();
  const uint32_t total = gtotal;
  const int np = gnp;
  const bool small = total < (1u << 24);
  // (a piece index and a 32-bit offset per cell, not a pointer: this runs after the march, in
  // the same register allocation)
  for (uint32_t i0 = tid; i0 < total; i0 += B * nt) {
    V2 c[B];
    int32_t off[B], pc[B];
    int p = 0;
#pragma unroll
    for (int j = 0; j < B; ++j) {
      const uint32_t i = i0 + (uint32_t)j * nt;
      pc[j] = -1;
      if (i < total) {
        while (p + 1 < np && gp[p + 1].start <= i) ++p;
        const GatePiece& q = gp[p];
        const uint32_t k = i - q.start;
        const uint32_t r = small ? gate_div(k, (uint32_t)q.nx, q.inx) : k / (uint32_t)q.nx;
        const uint32_t zz = small ? gate_div(r, (uint32_t)q.ny, q.iny) : r / (uint32_t)q.ny;
        const int x = q.x0 + (int)(k - r * (uint32_t)q.nx);
        const int y = q.y0 + (int)(r - zz * (uint32_t)q.ny);
        const int z = q.z0 + (int)zz;
        c[j] = d[gs::lin(g, x, y, z)];
        off[j] = ((z - q.sz0) * q.sny + (y - q.sy0)) * q.snx + (x - q.sx0);
        pc[j] = p;
      }
    }
#pragma unroll
    for (int j = 0; j < B; ++j) {
      if (pc[j] < 0) continue;
      const GatePiece& q = gp[pc[j]];
      V2* dst = (V2*)q.ptr + off[j];
      if (q.sys) store_system(dst, c[j]);
      else *dst = c[j];
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every landing store acknowledged
  __syncthreads();
  if (tid == 0) {
    if (G.stamps) {
      const unsigned long long dt = (unsigned long long)(wall_clock64() - tc0);
      atomicMax(G.stamps + 8, dt);
      atomicAdd(G.stamps + 9, dt);
      atomicAdd(G.stamps + 10, 1ull);
    }
    gate_arrive(G, m, a.gate_cnt2, true);
  }
}

// a start-gated unit in the one-unit table: pack (a packer), then wait and unpack (gated)
template <typename T>
__device__ __forceinline__ void gate_start(const FusedArgs& a, int pk, bool wait, int X0, int xw,
                                        int Y0, int yext, int za, int zb) {
  const uint64_t t0 = wall_clock64();  // the exchange's start (timeout, emulated duration)
  if (pk >= 0) gate_pack<T>(a, pk);
  if (wait) gate_unpack<T, gate_batch<T>()>(a, X0, xw, Y0, yext, za, zb, t0);
}
