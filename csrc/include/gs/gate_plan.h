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

struct GateUnit {
  int32_t tile;    // tile index (the launch's enumeration)
  int32_t z0, z1;  // output planes [z0, z1)
  int32_t pk;      // >= 0: a packer, its index; -1: none (every start-gated unit packs)
  int32_t wait;    // 1: start-gated (waits for the peers, copies its cone's ghosts)
};

// The unit table (see above).  fill: a unit's pipeline fill + ramp in plane-times (the launch
// model: 5n).  Sorted by (z0, tile), so each XCD group of workgroups (sched 3) gets a contiguous
// range: neighbouring tiles at one depth.  allpk: every unit packs (else the start-gated ones).
inline std::vector<GateUnit> gate_plan(const TileGrid& tg, const Geom& g, const HaloPlan& p,
                                       int n, int xp, bool allpk, int slots, bool longest,
                                       int* npk) {
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
  struct Col { bool strip, lo, hi; };
  std::vector<Col> cols((size_t)tg.ntiles);
  for (int t = 0; t < tg.ntiles; ++t) {
    int X0, xw, Y0, ye;
    tile_window(tg, t, n, &X0, &xw, &Y0, &ye);
    cols[t].strip = dep(X0, xw, Y0, ye, n, nz - n);
    cols[t].lo = dep(X0, xw, Y0, ye, 0, 1);
    cols[t].hi = dep(X0, xw, Y0, ye, nz - 1, nz);
  }
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
        if (out) out->push_back(GateUnit{t, z0, z1, gated ? 0 : -1, gated ? 1 : 0});
        ++cnt;
      }
    };
    for (int t = 0; t < tg.ntiles; ++t) {
      const Col& c = cols[t];
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
  return u;
}

}  // namespace gs
