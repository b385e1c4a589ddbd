// SPDX-License-Identifier: MIT
// The unit table of a gated pass (csrc/hip/gate.hpp): host-only planning shared by the HIP
// backend (HipBackend::gate_table) and the CPU library's test entry (gs_gate_plan), so the
// planner is checked on the CPU against an independent cone computation
// (tests/test_gate_plan.py).
//
// A fused-kernel launch enumerates tiles in x / y (k_fused's tile grid: 64-lane x tiles of
// xstep = 64 - 2n outputs, ROWS x WAVES-row y tiles of ystep outputs, the last x strip optionally
// folded into half-wave tiles, two y-tiles per wave); each tile column is marched along z.  A
// gated pass cuts every column into z-chunks, one unit per workgroup:
//   * a unit whose level-0 read box -- its tile window x [z0 - n, z1 + n) -- meets a ghost box
//     a neighbour fills (a receive box of the halo plan) is START-GATED;
//   * a column whose window meets an x / y ghost box at interior planes (a "strip") is gated over
//     its whole length; otherwise only its end chunks that read z ghosts are, at least n planes
//     long so the middle chunks read no ghost;
//   * chunks are cut at a common plane budget tau per workgroup (gated chunks shorter by the
//     expected exchange time xp, in plane-times) -- the smallest tau whose units fit the resident
//     slots, or the longest chunks (tau = tmax: one unit per column / column end) if none does.
#pragma once

#include <algorithm>
#include <cstdint>
#include <vector>

#include "common.h"

namespace gs {

struct TileGrid {
  int xstep, ystep, ybase, ntx, nty, ntxf, nfold, ntiles, rt;
};

// the tile grid of a ROWS x WAVES configuration at depth n (FusedLaunch::run + fold_strip)
inline TileGrid tile_grid(int rows, int waves, bool fold, const Geom& g, int n) {
  TileGrid t{};
  auto mod4 = [](int64_t v) { return (int)(((v % 4) + 4) % 4); };
  t.rt = rows * waves;
  t.xstep = 64 - 2 * n;
  t.ystep = (t.rt - 2 * n) & ~3;
  t.ybase = -mod4(g.oy - n);
  t.ntx = (g.nx + t.xstep - 1) / t.xstep;
  t.nty = (g.ny - t.ybase + t.ystep - 1) / t.ystep;
  t.ntxf = t.ntx;
  t.nfold = 0;
  t.ntiles = t.ntx * t.nty;
  const int rem = g.nx - (t.ntx - 1) * t.xstep;
  if (fold && t.ntx >= 2 && rem <= 32 - 2 * n) {
    t.ntxf = t.ntx - 1;
    t.nfold = (t.nty + 1) / 2;
    t.ntiles = t.ntxf * t.nty + t.nfold;
  }
  return t;
}

// level-0 read window of tile `tile` in x / y: [X0, X0 + xw) x [Y0, Y0 + yext)
inline void tile_window(const TileGrid& t, int tile, int n, int* X0, int* xw, int* Y0, int* yext) {
  int tx, ty;
  if (t.nfold && tile >= t.ntxf * t.nty) {
    const int f = tile - t.ntxf * t.nty;
    tx = t.ntxf;
    ty = 2 * f;
    *xw = 32;
    *yext = t.rt + t.ystep;
  } else {
    tx = tile % t.ntxf;
    ty = tile / t.ntxf;
    *xw = 64;
    *yext = t.rt;
  }
  *X0 = tx * t.xstep - n;
  *Y0 = t.ybase + ty * t.ystep - n;
}

// output window of tile `tile` in x / y: [ox0, ox1) x [oy0, oy1), the cells its launch stores
// (fused.hpp fused_body: xstep columns -- a folded tile 32 - 2n -- and ystep rows -- a folded
// tile two y-tiles --, clipped to the sub-domain); the tiles' windows partition the interior
inline void tile_output(const TileGrid& t, const Geom& g, int tile, int n, int* ox0, int* ox1,
                        int* oy0, int* oy1) {
  int X0, xw, Y0, ye;
  tile_window(t, tile, n, &X0, &xw, &Y0, &ye);
  const bool folded = xw == 32;
  *ox0 = std::max(X0 + n, 0);
  *ox1 = std::min(X0 + n + (folded ? 32 - 2 * n : t.xstep), g.nx);
  *oy0 = std::max(Y0 + n, 0);
  *oy1 = std::min(Y0 + n + (folded ? 2 : 1) * t.ystep, g.ny);
}

struct GateUnit {
  int32_t tile;    // tile index (the launch's enumeration)
  int32_t z0, z1;  // output planes [z0, z1)
  int32_t pk;      // >= 0: a packer, its index; -1: none (every start-gated unit packs)
  int32_t wait;    // 1: start-gated (waits for the peers, copies its cone's ghosts)
  int32_t prod;    // 1: its outputs meet a send box (a carried exchange: it packs them at its end)
};

// The cells a unit carries into the next exchange's messages: its output box, open past the
// sub-domain's faces (a message also holds ghost / padding cells there -- z slabs send whole
// storage planes -- which the units at that face carry; set up front, unchanged by a pass).  The
// boxes of all units still partition space, so every message cell is carried exactly once.
constexpr int kCarryFar = 1 << 28;
inline Box carry_window(const TileGrid& tg, const Geom& g, const GateUnit& x, int n) {
  int ox0, ox1, oy0, oy1;
  tile_output(tg, g, x.tile, n, &ox0, &ox1, &oy0, &oy1);
  if (ox0 <= 0) ox0 = -kCarryFar;
  if (ox1 >= g.nx) ox1 = kCarryFar;
  if (oy0 <= 0) oy0 = -kCarryFar;
  if (oy1 >= g.ny) oy1 = kCarryFar;
  const int z0 = x.z0 <= 0 ? -kCarryFar : x.z0, z1 = x.z1 >= g.nz ? kCarryFar : x.z1;
  return Box{ox0, oy0, z0, ox1 - ox0, oy1 - oy0, z1 - z0};
}

// prod of every unit: its carry window meets an outgoing message
inline void gate_mark_producers(const TileGrid& tg, const Geom& g, const HaloPlan& p, int n,
                                std::vector<GateUnit>* u) {
  for (GateUnit& x : *u) {
    x.prod = 0;
    if (x.tile < 0) continue;
    const Box w = carry_window(tg, g, x, n);
    for (int i = 0; i < p.nsend && !x.prod; ++i) {
      const Box& b = p.send[i].box;
      if (b.x0 < w.x0 + w.nx && w.x0 < b.x0 + b.nx && b.y0 < w.y0 + w.ny &&
          w.y0 < b.y0 + b.ny && b.z0 < w.z0 + w.nz && w.z0 < b.z0 + b.nz)
        x.prod = 1;
    }
  }
}

// Which ghost reads each tile column has: strip (an x / y ghost box at interior planes: gated
// over its whole length), lo / hi (the z ghosts below / above, read by its end chunks)
struct GateCol { bool strip, lo, hi; };
inline std::vector<GateCol> gate_columns(const TileGrid& tg, const Geom& g, const HaloPlan& p,
                                         int n) {
  const int nz = g.nz;
  auto dep = [&](int X0, int xw, int Y0, int ye, int z0, int z1) {
    for (int i = 0; i < p.nrecv; ++i) {
      const Box& b = p.recv[i].box;
      if (b.x0 < X0 + xw && X0 < b.x0 + b.nx && b.y0 < Y0 + ye && Y0 < b.y0 + b.ny &&
          b.z0 < z1 + n && z0 - n < b.z0 + b.nz)
        return true;
    }
    return false;
  };
  std::vector<GateCol> cols((size_t)tg.ntiles);
  for (int t = 0; t < tg.ntiles; ++t) {
    int X0, xw, Y0, ye;
    tile_window(tg, t, n, &X0, &xw, &Y0, &ye);
    cols[t].strip = dep(X0, xw, Y0, ye, n, nz - n);
    cols[t].lo = dep(X0, xw, Y0, ye, 0, 1);
    cols[t].hi = dep(X0, xw, Y0, ye, nz - 1, nz);
  }
  return cols;
}

// The unit table (see above).  fill: a unit's pipeline fill + ramp in plane-times (the launch
// model: 5n).  Sorted by (z0, tile), so each XCD group of workgroups (sched 3) gets a contiguous
// range: neighbouring tiles at one depth.  allpk: every unit packs (else the start-gated ones).
inline std::vector<GateUnit> gate_plan(const TileGrid& tg, const Geom& g, const HaloPlan& p,
                                       int n, int xp, bool allpk, int slots, bool longest,
                                       int* npk) {
  const int nz = g.nz;
  const std::vector<GateCol> cols = gate_columns(tg, g, p, n);
  const int F = 5 * n;
  auto build = [&](int tau, std::vector<GateUnit>* out) -> int {
    const int lg = std::max(1, tau - F - xp), li = std::max(1, tau - F);
    int cnt = 0;
    auto sect = [&](int t, int a, int b, int len, bool gated) {
      if (b <= a) return;
      const int k = (b - a + len - 1) / len;
      for (int i = 0; i < k; ++i) {
        const int z0 = a + (int)((int64_t)(b - a) * i / k);
        const int z1 = a + (int)((int64_t)(b - a) * (i + 1) / k);
        if (out) out->push_back(GateUnit{t, z0, z1, gated ? 0 : -1, gated ? 1 : 0, 0});
        ++cnt;
      }
    };
    for (int t = 0; t < tg.ntiles; ++t) {
      const GateCol& c = cols[t];
      const int P = c.lo ? std::max(n, std::min(lg, nz)) : 0;
      const int S = c.hi ? std::max(n, std::min(lg, nz)) : 0;
      if (c.strip || P + S >= nz) {
        sect(t, 0, nz, lg, true);
      } else {
        sect(t, 0, P, lg, true);
        sect(t, P, nz - S, li, false);
        sect(t, nz - S, nz, lg, true);
      }
    }
    return cnt;
  };
  const int tmax = F + xp + nz + 1;
  int tau = longest ? tmax : F + 1;
  while (tau < tmax && build(tau, nullptr) > slots) ++tau;
  std::vector<GateUnit> u;
  build(tau, &u);
  std::stable_sort(u.begin(), u.end(), [](const GateUnit& a, const GateUnit& b) {
    return a.z0 != b.z0 ? a.z0 < b.z0 : a.tile < b.tile;
  });
  int k = 0;
  for (auto& x : u)
    if (x.wait || allpk) x.pk = k++;
  *npk = k;
  gate_mark_producers(tg, g, p, n, &u);
  return u;
}

// PAIRS variant: every workgroup runs up to two units in turn -- first an ungated chunk (entry
// 2w), then a start-gated one (entry 2w + 1), whose wait for the peers' flags and cone unpack
// happen between the two marches, so the first chunk covers the exchange instead of an idle
// wait.  Entries with tile = -1 are empty.  Model, in plane-times: a unit costs its planes plus
// fill = 3n - 1 (the skewed pipeline's fill and drain); a pair costs max(fill + a, X) + U + fill
// + g for an ungated chunk of a planes and a gated chunk of g planes (X: the exchange, U: the
// cone unpack, both expected values the device tunes); the table takes the smallest makespan M
// that fits `slots` workgroups.  pk of entry 2w: the workgroup's packer index (-1: none): the
// workgroups with a gated unit pack, or every one (allpk).
inline std::vector<GateUnit> gate_plan_pairs(const TileGrid& tg, const Geom& g, const HaloPlan& p,
                                             int n, int X, int U, bool allpk, int slots,
                                             int* npk) {
  const int nz = g.nz;
  const std::vector<GateCol> cols = gate_columns(tg, g, p, n);
  const int Fu = 3 * n - 1;
  struct Piece { int t, z0, z1; };
  // the gated chunks (at most lg planes) and the ungated ranges for a gated chunk length lg
  auto split = [&](int lg, std::vector<Piece>* gated, std::vector<Piece>* free_) {
    for (int t = 0; t < tg.ntiles; ++t) {
      const GateCol& c = cols[t];
      const int P = c.lo ? std::max(n, std::min(lg, nz)) : 0;
      const int S = c.hi ? std::max(n, std::min(lg, nz)) : 0;
      auto cut = [&](int a, int b) {
        if (b <= a) return;
        const int k = (b - a + lg - 1) / lg;
        for (int i = 0; i < k; ++i)
          gated->push_back(Piece{t, a + (int)((int64_t)(b - a) * i / k),
                                 a + (int)((int64_t)(b - a) * (i + 1) / k)});
      };
      if (c.strip || P + S >= nz) {
        cut(0, nz);
      } else {
        cut(0, P);
        if (nz - S > P) free_->push_back(Piece{t, P, nz - S});
        cut(nz - S, nz);
      }
    }
  };
  // the smallest makespan M (and its gated chunk length) whose pieces fit the slots
  int bestM = -1, bestLg = nz;
  for (int lg = std::max(1, n); lg <= nz; lg = lg < 8 ? lg + 1 : lg + lg / 8) {
    std::vector<Piece> gated, free_;
    split(lg, &gated, &free_);
    if ((int)gated.size() > slots) continue;
    int64_t wu = 0;
    for (const Piece& f : free_) wu += f.z1 - f.z0;
    // M: every gated chunk's pair ends by M; the ungated planes fit the pairs' first slots and
    // the single workgroups
    int lo = 1, hi = 4 * (nz + X + U + 2 * Fu) + 8;
    auto fits = [&](int M) {
      int64_t cap = 0;
      for (const Piece& q : gated) {
        const int tail = U + Fu + (q.z1 - q.z0);
        if (std::max(X, 0) + tail > M) return false;  // not even without a first chunk
        cap += std::max(0, M - tail - Fu);             // planes of a first chunk before it
      }
      cap += (int64_t)(slots - (int)gated.size()) * std::max(0, M - Fu);
      return cap >= wu;
    };
    if (!fits(hi)) continue;
    while (lo < hi) {
      const int mid = (lo + hi) / 2;
      if (fits(mid)) hi = mid; else lo = mid + 1;
    }
    if (bestM < 0 || lo < bestM) { bestM = lo; bestLg = lg; }
  }
  std::vector<GateUnit> u;
  *npk = 0;
  if (bestM < 0) return u;  // no pairs table fits
  std::vector<Piece> gated, free_;
  split(bestLg, &gated, &free_);
  std::stable_sort(gated.begin(), gated.end(), [](const Piece& a, const Piece& b) {
    return a.z0 != b.z0 ? a.z0 < b.z0 : a.t < b.t;
  });
  const GateUnit none{-1, 0, 0, -1, 0, 0};
  // cut the ungated ranges into the pairs' first chunks, then into single units; a chunk never
  // crosses a column, so a range's short remainder can waste a pair's room: raise M until the
  // workgroups fit
  for (int M = bestM; M <= bestM + nz + 1; ++M) {
    u.clear();
    size_t fi = 0;
    int fz = free_.empty() ? 0 : free_[0].z0;
    auto take = [&](int len, Piece* out) -> bool {
      while (fi < free_.size() && fz >= free_[fi].z1)
        if (++fi < free_.size()) fz = free_[fi].z0;
      if (fi >= free_.size() || len <= 0) return false;
      const int z1 = std::min(free_[fi].z1, fz + len);
      *out = Piece{free_[fi].t, fz, z1};
      fz = z1;
      return true;
    };
    for (const Piece& q : gated) {
      Piece a{};
      const bool first = take(M - (U + Fu + (q.z1 - q.z0)) - Fu, &a);
      u.push_back(first ? GateUnit{a.t, a.z0, a.z1, -1, 0, 0} : none);
      u.push_back(GateUnit{q.t, q.z0, q.z1, -1, 1, 0});
    }
    for (;;) {
      Piece a{};
      if (!take(M - Fu, &a)) break;
      u.push_back(GateUnit{a.t, a.z0, a.z1, -1, 0, 0});
      u.push_back(none);
    }
    if ((int)(u.size() / 2) <= slots) break;
  }
  if ((int)(u.size() / 2) > slots) {
    u.clear();
    return u;
  }
  int k = 0;
  for (size_t w = 0; w < u.size(); w += 2)
    if (allpk || u[w + 1].wait) u[w].pk = k++;
  *npk = k;
  return u;
}

}  // namespace gs
