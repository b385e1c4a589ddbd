// SPDX-License-Identifier: MIT
// Shared host/device definitions for the MI355X Gray-Scott engine.
//
// Behavioural spec (reference /root/reference):
//   lap(x)   = (x[i-1]+x[i+1]+x[j-1]+x[j+1]+x[k-1]+x[k+1] - 6 x) / 6      Common.jl:13-18
//   du       = Du lap(u) - u v^2 + F (1-u) + noise * U(-1,1)               Simulation_CPU.jl:96-109
//   dv       = Dv lap(v) + u v^2 - (F+k) v
//   u' = u + dt du ; v' = v + dv dt
//
// Storage: one interleaved (u,v) pair per cell ("uv" layout), x fastest, then y, then z,
// with a ghost shell of width H on every side.  The interior x=0 column is padded to a
// 64-byte boundary so that wide vector loads stay aligned on gfx950.
#pragma once

#include <stdint.h>
#include <stddef.h>
#include <math.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define GS_HD __host__ __device__ __forceinline__
#else
#define GS_HD inline
#endif

namespace gs {

// ------------------------------------------------------------------------------------------
// Geometry of one rank's sub-domain.
// ------------------------------------------------------------------------------------------
struct Geom {
  int32_t nx, ny, nz;        // interior extent
  int32_t H;                 // ghost width (>= steps fused per halo exchange)
  int32_t xo;                // element offset of interior x = 0 inside a padded row
  int32_t px;                // padded row pitch (elements)
  int32_t py;                // rows per plane   (= ny + 2H)
  int32_t pz;                // planes           (= nz + 2H)
  int64_t ox, oy, oz;        // global offset of interior (0,0,0)
  int64_t Lx, Ly, Lz;        // global extent
  int32_t periodic;          // 1: periodic global boundary, 0: reference (Dirichlet-ish, §0.3)
  int32_t _pad;
};

GS_HD int64_t plane_elems(const Geom& g) { return (int64_t)g.px * g.py; }
GS_HD int64_t total_elems(const Geom& g) { return plane_elems(g) * g.pz; }
// linear element index of local cell (x,y,z); x,y,z in [-H, n+H)
GS_HD int64_t lin(const Geom& g, int x, int y, int z) {
  return ((int64_t)(z + g.H) * g.py + (y + g.H)) * g.px + (x + g.xo);
}

inline Geom make_geom(int nx, int ny, int nz, int H, int64_t ox, int64_t oy, int64_t oz,
                      int64_t Lx, int64_t Ly, int64_t Lz, int periodic) {
  Geom g{};
  g.nx = nx; g.ny = ny; g.nz = nz; g.H = H;
  // 8 elements = 64 B (fp32 pairs) / 128 B (fp64 pairs)
  g.xo = ((H + 7) / 8) * 8;
  g.px = ((g.xo + nx + H + 7) / 8) * 8;
  g.py = ny + 2 * H;
  g.pz = nz + 2 * H;
  g.ox = ox; g.oy = oy; g.oz = oz;
  g.Lx = Lx; g.Ly = Ly; g.Lz = Lz;
  g.periodic = periodic;
  return g;
}

// ------------------------------------------------------------------------------------------
// Model parameters (Settings, Structs.jl:4-28).
// ------------------------------------------------------------------------------------------
struct Params {
  double F, k, dt, Du, Dv, noise;
  uint64_t seed;
};

// A box in local coordinates: [x0,x0+nx) x [y0,y0+ny) x [z0,z0+nz)
struct Box {
  int32_t x0, y0, z0;
  int32_t nx, ny, nz;
};

GS_HD int64_t box_cells(const Box& b) { return (int64_t)b.nx * b.ny * b.nz; }

// ------------------------------------------------------------------------------------------
// Noise: rocRAND Philox4x32-10 stream (rocrand_philox4x32_10.h), evaluated counter-mode.
//   cell (gx,gy,gz), step n  ->  engine(seed, subsequence = n, offset = 4*q + (gy & 3))
//   with q = gx + Lx*((gy >> 2) + Ly4*gz),  Ly4 = ceil(Ly / 4).
// One Philox block therefore feeds four consecutive y-rows of one (x,z) column: the gfx950
// kernels give each thread a strip of rows, so a block is consumed by the thread that made
// it.  The stream depends only on global coordinates and the step, so results are
// decomposition- and restart-invariant.
// ------------------------------------------------------------------------------------------
struct U4 { uint32_t x, y, z, w; };

GS_HD void philox_round(uint32_t& c0, uint32_t& c1, uint32_t& c2, uint32_t& c3,
                        uint32_t k0, uint32_t k1) {
  const uint64_t m0 = (uint64_t)0xD2511F53u * c0;
  const uint64_t m1 = (uint64_t)0xCD9E8D57u * c2;
  const uint32_t hi0 = (uint32_t)(m0 >> 32), lo0 = (uint32_t)m0;
  const uint32_t hi1 = (uint32_t)(m1 >> 32), lo1 = (uint32_t)m1;
  const uint32_t n0 = hi1 ^ c1 ^ k0;
  const uint32_t n2 = hi0 ^ c3 ^ k1;
  c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
}

GS_HD U4 philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint64_t seed) {
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
  for (int r = 0; r < 10; ++r) {
    philox_round(c0, c1, c2, c3, k0, k1);
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return U4{c0, c1, c2, c3};
}

GS_HD U4 noise_block(int64_t gx, int64_t gy4, int64_t gz, int64_t Lx, int64_t Ly,
                     uint64_t step, uint64_t seed) {
  const uint64_t Ly4 = ((uint64_t)Ly + 3) >> 2;
  const uint64_t q = (uint64_t)gx + (uint64_t)Lx * ((uint64_t)gy4 + Ly4 * (uint64_t)gz);
  return philox4x32_10((uint32_t)q, (uint32_t)(q >> 32), (uint32_t)step,
                       (uint32_t)(step >> 32), seed);
}

// Random initial state (benchmarks: "random-init u/v", BASELINE.json), keyed on the global
// cell id only, so every decomposition starts from the same global state:
//   (w0, w1) = Philox4x32-10(counter = {q, q >> 32, ~0, ~0}, key = seed),
//   q = gx + Lx * (gy + Ly * gz);  u = lo + (hi - lo) * (w0 >> 8) 2^-24, v likewise with w1.
// Step ~0 (2^64 - 1) is never a noise step.  The 24-bit fractions are exact in fp32 and fp64;
// u = (hi - lo) * frac + lo is evaluated unfused (a rounded product, then a rounded sum) on
// every backend, exactly as the numpy oracle does (ops/reference.py random_fields), so any
// [lo, hi) gives the same bits everywhere.
GS_HD void random_init_cell(int64_t gx, int64_t gy, int64_t gz, int64_t Lx, int64_t Ly,
                            uint64_t seed, double lo, double hi, double* u, double* v) {
#if defined(__clang__)
#pragma clang fp contract(off)
#endif
  const uint64_t q = (uint64_t)gx + (uint64_t)Lx * ((uint64_t)gy + (uint64_t)Ly * (uint64_t)gz);
  const U4 r = philox4x32_10((uint32_t)q, (uint32_t)(q >> 32), 0xFFFFFFFFu, 0xFFFFFFFFu, seed);
  const double s = 5.9604644775390625e-08;  // 2^-24
  const double w = hi - lo;
  *u = w * ((double)(r.x >> 8) * s) + lo;
  *v = w * ((double)(r.y >> 8) * s) + lo;
}

GS_HD uint32_t u4_get(const U4& r, int i) {
  return i == 0 ? r.x : (i == 1 ? r.y : (i == 2 ? r.z : r.w));
}

// signed 32-bit word -> uniform on [-1, 1) (exactly representable in fp32 and fp64)
template <typename T>
GS_HD T uniform_pm1(uint32_t w) {
  return (T)(int32_t)w * (T)4.656612873077392578125e-10;  // 2^-31
}

// ------------------------------------------------------------------------------------------
// Boundary value for the reference's non-periodic topology: buffers are
// never written on the outer ghost shell; u ghosts start at 1 in u and 0 in u_temp, so the
// state at time t sees u_ghost = 1 for even t and 0 for odd t.  v ghosts are always 0.
// ------------------------------------------------------------------------------------------
GS_HD double bc_u(int64_t t) { return (t & 1) ? 0.0 : 1.0; }

// ------------------------------------------------------------------------------------------
// The per-cell update, shared by every backend.  `r` is the uniform draw in [-1,1).
// ------------------------------------------------------------------------------------------
template <typename T>
struct Coef {
  T Du6, Dv6, Du, Dv, F, Fk, dt, noise;
};

template <typename T>
GS_HD Coef<T> make_coef(const Params& p) {
  Coef<T> c;
  c.Du = (T)p.Du; c.Dv = (T)p.Dv;
  c.Du6 = (T)(p.Du / 6.0); c.Dv6 = (T)(p.Dv / 6.0);
  c.F = (T)p.F; c.Fk = (T)(p.F + p.k); c.dt = (T)p.dt; c.noise = (T)p.noise;
  return c;
}

template <typename T>
GS_HD void gs_update(const Coef<T>& c, T u, T v, T su, T sv, T r, T& uo, T& vo) {
  // su/sv: sum of the six face neighbours.  Du*lap = Du/6*sum - Du*u
  const T uvv = u * v * v;
  const T du = c.Du6 * su - c.Du * u - uvv + c.F * ((T)1 - u) + c.noise * r;
  const T dv = c.Dv6 * sv - c.Dv * v + uvv - c.Fk * v;
  uo = u + du * c.dt;
  vo = v + dv * c.dt;
}

// ------------------------------------------------------------------------------------------
// Halo plan: 26-direction exchange of H-deep slabs (faces, edges, corners).
// Direction index d = (dx+1)*9 + (dy+1)*3 + (dz+1); d = 13 is the rank itself.
// send_box[d] : interior cells adjacent to side d       (what the neighbour at d needs)
// recv_box[d] : ghost cells on side d                   (filled by the neighbour at d)
// For the 7-point stencil with one fused step only the 6 faces are needed.
// ------------------------------------------------------------------------------------------
constexpr int kMaxMsgs = 26;

struct HaloMsg {
  int32_t dir;        // 0..26
  int32_t peer;       // rank
  Box box;            // region in local coordinates
  int64_t offset;     // element offset inside the packed buffer (in cells, not bytes)
};

struct HaloPlan {
  int32_t nsend, nrecv;
  // 1: the only neighbours are along z and every message is a run of whole storage planes
  // (x/y ghosts and row padding included), i.e. one contiguous range of the field buffer that
  // a transport can send / receive in place, without pack / unpack kernels
  int32_t zplanes;
  HaloMsg send[kMaxMsgs];
  HaloMsg recv[kMaxMsgs];
  int64_t send_cells, recv_cells;
};

GS_HD int dir_index(int dx, int dy, int dz) { return (dx + 1) * 9 + (dy + 1) * 3 + (dz + 1); }

inline void dir_of(int d, int& dx, int& dy, int& dz) {
  dx = d / 9 - 1; dy = (d / 3) % 3 - 1; dz = d % 3 - 1;
}

inline Box side_box(const Geom& g, int dx, int dy, int dz, bool ghost) {
  // along one axis: side -1 -> [0,H) interior / [-H,0) ghost; +1 -> [n-H,n) / [n,n+H); 0 -> [0,n)
  auto axis = [&](int s, int n, int32_t& o, int32_t& c) {
    if (s == 0) { o = 0; c = n; }
    else if (s < 0) { o = ghost ? -g.H : 0; c = g.H; }
    else { o = ghost ? n : n - g.H; c = g.H; }
  };
  Box b;
  axis(dx, g.nx, b.x0, b.nx);
  axis(dy, g.ny, b.y0, b.ny);
  axis(dz, g.nz, b.z0, b.nz);
  return b;
}

// nbr[27]: peer rank for each direction or -1.  Messages to the same peer are ordered so
// that the k-th send from A to B matches the k-th receive at B from A: sends ascend in d,
// receives descend in d (the matching send for recv d is the peer's send -d = 26-d).
inline bool z_only_neighbours(const int32_t* nbr) {
  for (int d = 0; d < 27; ++d) {
    int dx, dy, dz; dir_of(d, dx, dy, dz);
    if ((dx != 0 || dy != 0) && nbr[d] >= 0) return false;
  }
  return true;
}

// Storage-plane form of a z message box: the full padded plane extent in x and y.
inline Box full_planes(const Geom& g, Box b) {
  b.x0 = -g.xo; b.nx = g.px;
  b.y0 = -g.H; b.ny = g.py;
  return b;
}

inline HaloPlan make_halo_plan(const Geom& g, const int32_t* nbr, bool diagonals) {
  HaloPlan p{};
  p.zplanes = z_only_neighbours(nbr) ? 1 : 0;
  int64_t off = 0;
  for (int d = 0; d < 27; ++d) {
    if (d == 13 || nbr[d] < 0) continue;
    int dx, dy, dz; dir_of(d, dx, dy, dz);
    if (!diagonals && (dx != 0) + (dy != 0) + (dz != 0) != 1) continue;
    HaloMsg m; m.dir = d; m.peer = nbr[d]; m.box = side_box(g, dx, dy, dz, false); m.offset = off;
    if (p.zplanes) m.box = full_planes(g, m.box);
    off += box_cells(m.box);
    p.send[p.nsend++] = m;
  }
  p.send_cells = off;
  off = 0;
  for (int d = 26; d >= 0; --d) {
    if (d == 13 || nbr[d] < 0) continue;
    int dx, dy, dz; dir_of(d, dx, dy, dz);
    if (!diagonals && (dx != 0) + (dy != 0) + (dz != 0) != 1) continue;
    HaloMsg m; m.dir = d; m.peer = nbr[d]; m.box = side_box(g, dx, dy, dz, true); m.offset = off;
    if (p.zplanes) m.box = full_planes(g, m.box);
    off += box_cells(m.box);
    p.recv[p.nrecv++] = m;
  }
  p.recv_cells = off;
  return p;
}

// Element offset of a message box's first cell in the field buffer (contiguous for zplanes).
inline int64_t box_start(const Geom& g, const Box& b) { return lin(g, b.x0, b.y0, b.z0); }

// Region updated by fused step s (0-based) of an n-step pass: the interior grown by
// (n-1-s) cells on every side that has a neighbour (ghost data valid there), never on a
// global boundary side.
inline Box pass_region(const Geom& g, const int32_t* nbr, int n, int s) {
  const int e = n - 1 - s;
  int lo[3], hi[3];
  const int sz[3] = {g.nx, g.ny, g.nz};
  for (int a = 0; a < 3; ++a) {
    int dm[3] = {0, 0, 0}, dp[3] = {0, 0, 0};
    dm[a] = -1; dp[a] = 1;
    lo[a] = nbr[dir_index(dm[0], dm[1], dm[2])] >= 0 ? -e : 0;
    hi[a] = sz[a] + (nbr[dir_index(dp[0], dp[1], dp[2])] >= 0 ? e : 0);
  }
  return Box{lo[0], lo[1], lo[2], hi[0] - lo[0], hi[1] - lo[1], hi[2] - lo[2]};
}

}  // namespace gs
