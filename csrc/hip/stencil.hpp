// SPDX-License-Identifier: MIT
// gfx950 stencil kernels (included inside namespace gsk by kernels.hpp).
//
// Hot op of the reference: calculate! (Simulation_CPU.jl:77-113; GPU variants
// ext/CUDAExt.jl:135-161, ext/AMDGPUExt.jl:179-210, Simulation_KA.jl:177-203), whose GPU
// thread mapping (thread = (k, j), serial i-loop) is uncoalesced and unpipelined (D9).
//
// CDNA4 design:
//  * lanes run along x (the contiguous axis) -> 512 B (fp32) / 1 KiB (fp64) per wave load
//  * x-neighbours come from the adjacent lanes through DPP wave shifts (`v_add_f32_dpp
//    wave_shl:1/wave_shr:1`), not from memory
//  * each thread owns a strip of ROWS y-rows, so y-neighbours are its own registers; only a
//    wave's first/last row crosses waves, through a few hundred bytes of LDS
//  * z is marched; per level the thread keeps the centre and a running partial sum of the
//    previous plane (4 registers per cell instead of a 3-plane ring)
//  * k_fused chains T time levels in registers (temporal blocking): HBM is read once and
//    written once per T steps.  T=2 halves the compulsory traffic of the 16 B/cell step.
//  * one Philox4x32-10 block serves the four y-rows of a quad (rocRAND stream, common.h)
#pragma once

// ------------------------------------------------------------------------------------------
// DPP lane shifts.  shr: lane i receives lane i-1; shl: lane i receives lane i+1.
// Lanes without a source receive 0 (they only ever feed tile-halo cells); bound_ctrl gives
// that 0 without materialising an old-value register (one v_mov per shift otherwise).
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ float lane_from_left(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x138, 0xf, 0xf, true));
}
__device__ __forceinline__ float lane_from_right(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x130, 0xf, 0xf, true));
}
__device__ __forceinline__ double lane_from_left(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)b, 0x138, 0xf, 0xf, true);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), 0x138, 0xf, 0xf, true);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ double lane_from_right(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)b, 0x130, 0xf, 0xf, true);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), 0x130, 0xf, 0xf, true);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

// positive modulo 4 of a possibly negative 64-bit value
__host__ __device__ __forceinline__ int mod4(int64_t v) { return (int)(((v % 4) + 4) % 4); }

// ------------------------------------------------------------------------------------------
// k_step1: one step over an arbitrary box (extended regions, shells, remainders).
// Block = 64 lanes (x) x 4 y-quads; each thread owns one globally aligned y-quad (4 rows).
// Planes are prefetched one iteration ahead.
// ------------------------------------------------------------------------------------------
struct StepArgs {
  Geom g;
  Box r;
  int32_t zchunk;
  int32_t ybase;  // local y of quad 0 (aligned so that oy + ybase is a multiple of 4)
  int64_t t;
};

template <typename T, bool NOISE>
__global__ __launch_bounds__(256) void k_step1(const typename Vec2<T>::type* __restrict__ s,
                                               typename Vec2<T>::type* __restrict__ d,
                                               StepArgs a, gs::Coef<T> c, uint64_t seed) {
  using V2 = typename Vec2<T>::type;
  const Geom& g = a.g;
  const int lane = threadIdx.x;
  const int x = a.r.x0 + blockIdx.x * 64 + lane;
  const int yq = a.ybase + 4 * (blockIdx.y * 4 + threadIdx.y);  // first row of this quad
  const int z0 = a.r.z0 + blockIdx.z * a.zchunk;
  const int z1 = min(z0 + a.zchunk, a.r.z0 + a.r.nz);
  const int rx1 = a.r.x0 + a.r.nx, ry1 = a.r.y0 + a.r.ny;
  if (yq + 3 < a.r.y0 || yq >= ry1 || z0 >= z1) return;  // whole wave leaves together
  const int H = g.H;
  const int xc = clampi(x, -H, g.nx + H - 1);
  const int64_t PZ = gs::plane_elems(g);
  const V2* __restrict__ sc = s + xc + g.xo;
  // row offsets (y clamped into the allocation) for rows -1..4 of the quad
  int ro[6];
#pragma unroll
  for (int j = 0; j < 6; ++j) ro[j] = (clampi(yq + j - 1, -H, g.ny + H - 1) + H) * g.px;
  auto plane = [&](int z) -> int64_t { return (int64_t)(clampi(z, -H, g.nz + H - 1) + H) * PZ; };
  V2 pm[4], p0[4], pp[4], hm, hp;
  {
    const int64_t zm = plane(z0 - 1), z_0 = plane(z0), zp = plane(z0 + 1);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      pm[j] = sc[zm + ro[j + 1]];
      p0[j] = sc[z_0 + ro[j + 1]];
      pp[j] = sc[zp + ro[j + 1]];
    }
    hm = sc[z_0 + ro[0]];
    hp = sc[z_0 + ro[5]];
  }
  const int64_t gx = wrap(g.ox + x, g.Lx);
  const bool xok = x < rx1;
  bool rok[4];
  int64_t gyr[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    rok[j] = (yq + j >= a.r.y0) && (yq + j < ry1);
    gyr[j] = wrap(g.oy + yq + j, g.Ly);
  }
  for (int z = z0; z < z1; ++z) {
    // prefetch the next iteration's planes
    V2 nn[4], nhm, nhp;
    {
      const int64_t z2 = plane(z + 2), z1p = plane(z + 1);
#pragma unroll
      for (int j = 0; j < 4; ++j) nn[j] = sc[z2 + ro[j + 1]];
      nhm = sc[z1p + ro[0]];
      nhp = sc[z1p + ro[5]];
    }
    const int64_t gz = wrap(g.oz + z, g.Lz);
    gs::U4 blk{0, 0, 0, 0};
    V2 o[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const V2 ym = j == 0 ? hm : p0[j - 1];
      const V2 yp = j == 3 ? hp : p0[j + 1];
      T xmu = lane_from_left(p0[j].x), xpu = lane_from_right(p0[j].x);
      T xmv = lane_from_left(p0[j].y), xpv = lane_from_right(p0[j].y);
      if (lane == 0 || lane == 63) {
        const int64_t row = plane(z) + ro[j + 1];
        const int xn = clampi(x + (lane == 0 ? -1 : 1), -H, g.nx + H - 1);
        const V2 e = s[row + xn + g.xo];
        if (lane == 0) { xmu = e.x; xmv = e.y; } else { xpu = e.x; xpv = e.y; }
      }
      const T su = (xmu + xpu) + (ym.x + yp.x) + (pm[j].x + pp[j].x);
      const T sv = (xmv + xpv) + (ym.y + yp.y) + (pm[j].y + pp[j].y);
      T r = (T)0;
      if (NOISE) {
        if (j == 0 || (gyr[j] & 3) == 0)
          blk = gs::noise_block(gx, gyr[j] >> 2, gz, g.Lx, g.Ly, (uint64_t)a.t, seed);
        r = gs::uniform_pm1<T>(gs::u4_get(blk, (int)(gyr[j] & 3)));
      }
      gs::gs_update<T>(c, p0[j].x, p0[j].y, su, sv, r, o[j].x, o[j].y);
    }
    const int64_t zo = (int64_t)(z + H) * PZ;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (xok && rok[j]) d[zo + ro[j + 1] + x + g.xo] = o[j];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      pm[j] = p0[j];
      p0[j] = pp[j];
      pp[j] = nn[j];
    }
    hm = nhm;
    hp = nhp;
  }
}

template <typename T>
void launch_step1(const typename Vec2<T>::type* s, typename Vec2<T>::type* d, const Geom& g,
                  const gs::Params& p, const Box& r, int64_t t, hipStream_t st) {
  StepArgs a;
  a.g = g;
  a.r = r;
  a.t = t;
  a.ybase = r.y0 - mod4(g.oy + r.y0);
  const int nq = (r.y0 + r.ny - a.ybase + 3) / 4;
  const int bx = (r.nx + 63) / 64, by = (nq + 3) / 4;
  const int64_t xy = (int64_t)bx * by;
  int nzc = (int)std::max<int64_t>(1, (2048 + xy - 1) / xy);
  int zc = (r.nz + nzc - 1) / nzc;
  zc = std::max(zc, std::min(r.nz, 8));
  nzc = (r.nz + zc - 1) / zc;
  a.zchunk = zc;
  dim3 grid(bx, by, nzc), block(64, 4, 1);
  const gs::Coef<T> c = gs::make_coef<T>(p);
  if (p.noise != 0.0) k_step1<T, true><<<grid, block, 0, st>>>(s, d, a, c, p.seed);
  else k_step1<T, false><<<grid, block, 0, st>>>(s, d, a, c, p.seed);
}

// ------------------------------------------------------------------------------------------
// k_fused: T time levels per HBM pass over the interior (temporal blocking).
//
// Work unit = one (tile, z-plane) pair; the units are split evenly over a persistent grid
// of `occupancy x CUs` workgroups, each walking one or two contiguous z-segments.
// Tile = 64 columns (one lane each) x WAVES*ROWS rows of level-0 data (ghosts included);
// it yields (64-2T) x ystep interior outputs.  A segment [z0,z1) streams level-0 planes
// z0-T .. z1+T-1; level l produces plane p-l at iteration p; level T is stored.
// Intermediate levels that fall outside the global domain (non-periodic) are reset to the
// boundary value of their time level, exactly what the single-step path sees in its ghosts.
// ------------------------------------------------------------------------------------------
#include "fused.hpp"
