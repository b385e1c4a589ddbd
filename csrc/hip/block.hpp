// SPDX-License-Identifier: MIT
// k_block: the fused T-step pass for SMALL grids, every time level of a block held in LDS.
// Included inside namespace gsk by kernels.hpp, after fused.hpp (it shares fused.hpp's cell
// update order, Philox stream and DPP sums, so its results are bit-identical to k_fused's and it
// is simply one more candidate of the fused kernel's autotuner: fused_cfg_table "blk*").
//
// Why a second kernel: k_fused marches each tile along z through a 3T-1 iteration pipeline fill.
// On the reference's example grid (L = 64, examples/settings-files.toml) a workgroup's chunk is
// 1-2 planes, so a pass is that fill chain's latency (~1.3 us per iteration, profiles/
// r3_small_grid.txt: 9.5 us per T=2 pass, 55k MLUPS) while the chip's VALU work is ~0.6 us.
// Here a workgroup owns an output block of whole x rows x BY rows x BZ planes, loads the block's
// level-0 dependency cone (BY+2T rows x BZ+2T planes, every load in flight at once: one memory
// latency, with the Philox words of all its items drawn meanwhile) into LDS, computes the T
// levels from LDS into LDS (ping-pong buffers, one barrier per level; each wave takes whole 4-row
// noise quads, so one Philox draw serves 4 cells as in k_fused), and writes the last level
// straight to HBM.  The intermediate levels are recomputed on the block's halo (the dependency
// cone), which costs 2.5-3.7x the useful cell updates -- cheap at this size, where the chip is
// otherwise idle (L=64: 55k -> 81k MLUPS in round 3, profiles/r3_block.txt; 99k with round 4's
// scalar-unit work cut, below).
//
// Scope: x rows fit one wave (nx <= 64) and both x faces are the global (non-periodic)
// boundary, so no x halo is computed: a level's x ghost is the boundary value of its time level
// (engine.h ensure_bc for level 0 -- so only Backend::fused(), always called after it, launches
// k_block: FusedArgs.allow_block -- the k_fused reset rule for the others) and enters the
// x-neighbour sum of lane 0 / lane 63 as an exact correction (below).  y / z faces may have
// neighbours (their halos are H >= T deep, as for k_fused).
//
// The update computed is the reference's calculate! (Simulation_CPU.jl:92-112), T steps per pass.
#pragma once

struct BlockArgs {
  Geom g;
  int64_t t;
  int32_t yb;   // local y of block row 0 (<= 0; (oy + yb) % 4 == 0: whole noise quads)
  int32_t nby;  // blocks along y (grid = nby x ceil(nz / BZ))
  int32_t gr;   // nx == 64: no lane holds the +x ghost; lane 63 adds it explicitly
};

template <typename T_, int TL_, int BY_, int BZ_, int NW_, bool NOISE_, bool KV_ = true,
          bool LH_ = false>
struct BCfg {
  using T = T_;
  using V2 = typename PairT<T>::type;
  static constexpr int TL = TL_, BY = BY_, BZ = BZ_, NW = NW_;
  static constexpr bool NOISE = NOISE_;
  // Philox round keys 4-10 held in VGPRs (filled once) instead of rebuilt on the SALU per draw:
  // L=64 T=3 83.5k vs 80.3k MLUPS, T=2 77.6k vs 72.3k (in-process A/B, profiles/r3_block.txt)
  static constexpr bool KV = KV_;
  // the last level's items are half quads (2 rows): it has only BY/4 x BZ quads, so whole-quad
  // items leave most waves idle there; the halves' Philox draws happen in the load shadow
  static constexpr bool LH = LH_;
  // LDS rows: local y0-5 .. y0+BY+4 (intermediate levels compute the quads [y0-4, y0+BY+4) and
  // read one row beyond); LDS planes z0-T .. z0+BZ+T-1
  static constexpr int R0 = 5;
  static constexpr int NR = BY + 10;
  static constexpr int NP = BZ + 2 * TL;
  static constexpr int LDS_BYTES = (2 * NP * NR + 1) * 64 * (int)sizeof(V2);  // + the load sink
  // whether the two level buffers fit the CU's LDS (run_block falls back to k_fused if not)
  static constexpr bool FITS = LDS_BYTES <= 160 * 1024;  // (= fused.hpp block_cfg_fits)
  static_assert(BY % 4 == 0, "blocks hold whole noise quads");
  // level l+1's work items (noise quad, plane): intermediate levels one quad of halo on each
  // side in y and TL-1-l planes in z; each wave takes items wave, wave + NW, ...
  static constexpr int nq(int l) { return BY / 4 + (l + 1 < TL ? 2 : 0); }
  static constexpr int npl(int l) { return BZ + 2 * (TL - 1 - l); }
  static constexpr int S(int l) { return (LH && l + 1 == TL) ? 2 : 1; }  // items per quad
  static constexpr int items(int l) { return nq(l) * S(l) * npl(l); }
  static constexpr int per_wave(int l) { return (items(l) + NW - 1) / NW; }
  static constexpr int JMAX = per_wave(0);
};

// f(std::integral_constant<int, 0>), ..., f(std::integral_constant<int, N-1>): per-level code
// with the level as a compile-time constant (array extents and trip counts depend on it)
template <class F, int... I>
__device__ __forceinline__ void for_levels_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void for_levels(F&& f) {
  for_levels_impl(f, std::make_integer_sequence<int, N>{});
}

// ------------------------------------------------------------------------------------------
// The kernel is written for the scalar unit: it is shared by the CU's waves, so with 16 waves per
// CU the per-wave SALU count, not the VALU count, sets the pass time.  Round 3's version issued
// per wave ~540 SALU before the first barrier (a division per load, storage-bounds checks and a
// descriptor per load, the Philox rounds 1-3 key schedule per draw) and ~140 per level item
// (64-bit row / plane bounds, exec-masked boundary resets, 64-bit store addresses), ~1050 in all
// against ~610 VALU; L=64 ran at 81k MLUPS.  This one issues ~630 SALU (L=64: 99k MLUPS,
// profiles/r4_block_sl.txt):
//   * one buffer descriptor over each whole state buffer (< 1 GiB: block_supported): a row or plane
//     outside the storage is an offset outside the buffer (loads read 0, stores are dropped), and
//     a load's plane / row come from a per-wave split of the wave index plus one carry;
//   * the step-uniform words of each level's Philox rounds 1-3 (philox_uniform) once per level;
//   * boundary resets as bit selects (a per-lane x mask, a uniform row condition; no exec
//     branches), 32-bit coordinates, stores through the descriptor behind a uniform row branch.
// Bit-identical to k_fused: same sum order, Philox words and resets.
// ------------------------------------------------------------------------------------------

// m ? b : a, bit by bit (one v_bfi_b32)
__device__ __forceinline__ float fsel(uint32_t m, float a, float b) {
  return __uint_as_float((__float_as_uint(a) & ~m) | (__float_as_uint(b) & m));
}

template <class C>
__global__ __launch_bounds__(64 * C::NW, 1) void k_block(const typename C::V2* __restrict__ s,
                                                          typename C::V2* __restrict__ d,
                                                          BlockArgs a, FoldCoef<typename C::T> f,
                                                          uint64_t seed) {
  using T = typename C::T;
  using V2 = typename C::V2;
  static_assert(sizeof(T) == 4 && C::KV, "k_block: fp32, Philox round keys in VGPRs");
  constexpr int TL = C::TL, BY = C::BY, BZ = C::BZ, NW = C::NW, NR = C::NR, NP = C::NP;
  __shared__ V2 buf[2][NP][NR][64];  // [level parity][plane][row][lane]
  const Geom& g = a.g;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int by = blockIdx.x, bz = blockIdx.y;  // a 2D grid: no division by nby per wave
  const int y0 = a.yb + by * BY, z0 = bz * BZ;

  V2 kc;
  {
    const T k0 = f.kc.x, k1 = f.kc.y;
    asm volatile("v_mov_b32 %0, %1" : "=v"(kc.x) : "s"(k0));
    asm volatile("v_mov_b32 %0, %1" : "=v"(kc.y) : "s"(k1));
  }
  const T ar31 = f.ar * (T)4.656612873077392578125e-10;
  const uint32_t Ly4 = (uint32_t)((g.Ly + 3) >> 2);
  uint32_t kv[14];
#pragma unroll
  for (int r = 3; r < 10; ++r) {
    const uint32_t k0 = (uint32_t)seed + (uint32_t)r * kPhW0;
    const uint32_t k1 = (uint32_t)(seed >> 32) + (uint32_t)r * kPhW1;
    asm volatile("v_mov_b32 %0, %1" : "=v"(kv[2 * (r - 3)]) : "s"(k0));
    asm volatile("v_mov_b32 %0, %1" : "=v"(kv[2 * (r - 3) + 1]) : "s"(k1));
  }
  constexpr int SZ = (int)sizeof(V2);
  const int pitchb = g.px * SZ;
  const int pzb = g.px * g.py * SZ;
  const int total = pzb * g.pz;  // < 1 GiB (block_supported)
  const __amdgpu_buffer_rsrc_t rs = plane_rsrc((const char*)s, total);
  const __amdgpu_buffer_rsrc_t rd = plane_rsrc((const char*)d, total);
  // lane byte offsets (loads: the row's cells and its +x ghosts; stores: the interior); an
  // offset of 0x80000000 plus any row offset below 1 GiB lies outside the buffer
  const int lane_ld = lane < g.nx + g.H ? (lane + g.xo) * SZ : (int)0x80000000;
  const int lane_st = lane < g.nx ? (lane + g.xo) * SZ : (int)0x80000000;
  const uint32_t xmask = (g.ox + lane >= g.Lx) ? 0xFFFFFFFFu : 0u;  // outside the global x range

  // level 0: the outputs' dependency cone, rows y0-T .. y0+BY+T-1 of planes z0-T .. z0+BZ+T-1;
  // load i = wave + j NW is row i % NL of plane i / NL, from the wave's own split and a carry
  constexpr int NL = BY + 2 * TL;
  constexpr int NLD = NP * NL;
  constexpr int JL = (NLD + NW - 1) / NW;
  const int wpz = wave / NL, wr = wave - wpz * NL;
  // byte offset of cone row 0 of cone plane 0 (may be negative: rows above the storage)
  const int base = ((z0 - TL + g.H) * g.py + (y0 - TL + g.H)) * pitchb;
  gs::U4 W[TL][C::JMAX];  // noise words per (level, item of this wave)
  // LDS target of a load past the cone (never read): the writes stay unconditional, so the
  // compiler keeps every load ahead of the noise draws instead of sinking each one into its own
  // branch with a full wait (seven memory latencies in a row)
  __shared__ V2 sink[64];
  {
    V2 lv[JL];
    int lds[JL];
#pragma unroll
    for (int j = 0; j < JL; ++j) {
      int r = wr + (j * NW) % NL, pz = wpz + (j * NW) / NL;
      if (r >= NL) {  // uniform
        r -= NL;
        ++pz;
      }
      // (a load past the cone -- the last j of some waves -- re-reads the cone's last plane and
      // is not written to LDS: no select on the address)
      lds[j] = pz < NP ? pz * NR + (C::R0 - TL) + r : -1;  // (-1: the sink)
      const int roff = base + min(pz, NP - 1) * pzb + r * pitchb;
      lv[j] = bload(rs, lane_ld + roff, (V2*)nullptr);
    }
    // a compiler memory barrier: the loads may not sink below it towards their first use -- they
    // must all be in flight while the noise words are drawn
    asm volatile("" ::: "memory");
    // the noise words of every item this wave will compute, at every level, while the loads
    // are in flight (they depend on the cell and the step only)
    if constexpr (C::NOISE) {
      for_levels<TL>([&](auto LC) {
        constexpr int l = decltype(LC)::value;
        const PhiloxU pu = philox_uniform((uint64_t)(a.t + l), seed);
#pragma unroll
        for (int j = 0; j < C::per_wave(l); ++j) {
          const int it = wave + j * NW;
          if (it < C::items(l)) {
            constexpr int S = C::S(l);
            const int zi = it / (C::nq(l) * S), rem = it - zi * (C::nq(l) * S);
            const int qi = rem / S, h = rem - qi * S;
            const int qy = y0 - (l + 1 < TL ? 4 : 0) + 4 * qi;
            const int z = z0 - (TL - 1 - l) + zi;
            const uint32_t gy4 = (uint32_t)((g.oy + qy) >> 2);
            const uint32_t qu = (uint32_t)g.Lx * (gy4 + Ly4 * (uint32_t)(g.oz + z));
            const gs::U4 q = philox_lane(qu + (uint32_t)(g.ox + lane), pu, kv);
            W[l][j] = (S == 1 || h == 0) ? q : gs::U4{q.z, q.w, q.z, q.w};  // a half's words first
          }
        }
      });
    }
    V2(*b0)[64] = &buf[0][0][0];
#pragma unroll
    for (int j = 0; j < JL; ++j) {
      V2* dst = lds[j] >= 0 ? &b0[lds[j]][lane] : &sink[lane];
      *dst = lv[j];
    }
  }
  // rows the quads read beyond the cone (level 0: R0-5 .. R0-T-1 and R0+BY+T .. NR-1; the
  // level-1 buffer's first and last rows are never computed): defined zeros
  constexpr int NZR = C::R0 - TL;  // zero rows per side of level 0
  for (int i = wave; i < NP * (2 * NZR + 2); i += NW) {
    const int pz = i / (2 * NZR + 2), j = i - pz * (2 * NZR + 2);
    if (j < 2 * NZR) buf[0][pz][j < NZR ? j : NR - 2 * NZR + j][lane] = V2{(T)0, (T)0};
    else buf[1][pz][j == 2 * NZR ? 0 : NR - 1][lane] = V2{(T)0, (T)0};
  }
  __syncthreads();

  for_levels<TL>([&](auto LC) {
    constexpr int l = decltype(LC)::value;
    const V2(*in)[NR][64] = buf[l & 1];
    V2(*out)[NR][64] = buf[(l + 1) & 1];
    constexpr bool last = l + 1 == TL;
    constexpr int mq = last ? 0 : 1;  // intermediate levels: one quad of halo each side
    constexpr int nq = C::nq(l);
    constexpr int dz = TL - 1 - l;    // planes of halo this level still needs
    // x ghosts of level l: as in k_block (lane 0's left neighbour added after the DPP sum, lane
    // 63's right one into yz before it; other lanes add +0)
    const T bin = (T)gs::bc_u(a.t + l);
    const V2 gl = lane == 0 ? V2{bin, (T)0} : V2{(T)0, (T)0};
    const V2 gr = (a.gr && lane == 63) ? V2{bin, (T)0} : V2{(T)0, (T)0};
    const T bout = (T)gs::bc_u(a.t + l + 1);
#pragma unroll
    for (int j = 0; j < C::per_wave(l); ++j) {
      const int it = wave + j * NW;
      if (it >= C::items(l)) break;  // wave-uniform
      constexpr int S = C::S(l), HR = 4 / S;  // rows per item
      const int zi = it / (nq * S), rem = it - zi * (nq * S);
      const int qi = rem / S, h = rem - qi * S;
      const int qy = y0 - 4 * mq + 4 * qi + HR * h;  // local y of the item's first row
      const int z = z0 - dz + zi;
      const int pz = z - (z0 - TL);
      const int ry = qy - y0 + C::R0;
      V2 row[6], pm[4], pp[4];
#pragma unroll
      for (int k = 0; k < HR + 2; ++k) row[k] = lds_load2(&in[pz][ry - 1 + k][lane]);
#pragma unroll
      for (int k = 0; k < HR; ++k) {
        pm[k] = lds_load2(&in[pz - 1][ry + k][lane]);
        pp[k] = lds_load2(&in[pz + 1][ry + k][lane]);
      }
      const gs::U4 blk = C::NOISE ? W[l][j] : gs::U4{0, 0, 0, 0};
      const int gz = (int)g.oz + z;
      const bool zout = (unsigned)gz >= (unsigned)g.Lz;  // (negative: huge)
      // the last level's stores: this item's plane and rows inside the interior (uniform)
      const int zoff = (z + g.H) * pzb;
#pragma unroll
      for (int k = 0; k < HR; ++k) {
        const V2 c = row[k + 1];
        V2 yz = (row[k] + row[k + 2]) + pm[k];
        if (a.gr) yz = yz + gr;
        V2 A{lane_pair_sum_add<false>(c.x, yz.x), lane_pair_sum_add<false>(c.y, yz.y)};
        A = A + gl;
        const V2 sum = A + pp[k];
        const V2 tt = c * c.yy;
        const V2 uvv = tt.xx * c.yy;
        V2 P = __builtin_elementwise_fma(f.kd, uvv, kc);
        P = __builtin_elementwise_fma(f.ks, sum, P);
        P = __builtin_elementwise_fma(f.kcc, c, P);
        if constexpr (C::NOISE) {
          const uint32_t w = k == 0 ? blk.x : (k == 1 ? blk.y : (k == 2 ? blk.z : blk.w));
          P.x = fma(ar31, (T)(int32_t)w, P.x);
        }
        const int y = qy + k;
        if constexpr (!last) {
          const bool rout = zout || (unsigned)((int)g.oy + y) >= (unsigned)g.Ly;  // uniform
          const uint32_t m = xmask | (rout ? 0xFFFFFFFFu : 0u);
          P.x = fsel(m, P.x, bout);
          P.y = fsel(m, P.y, (T)0);
          out[pz][ry + k][lane] = P;
        } else {
          if (y >= 0 && y < g.ny && z < g.nz)  // uniform
            bstore(rd, lane_st + zoff + (y + g.H) * pitchb, P);
        }
      }
    }
    if constexpr (!last) __syncthreads();
  });
}

template <class C>
bool run_block(const void* s, void* d, const FusedArgs& a0, const gs::Params& p, hipStream_t st) {
  if constexpr (!C::FITS) {
    return false;
  } else {
  const Geom& g = a0.g;
  BlockArgs a{};
  a.g = g;
  a.t = a0.t;
  a.yb = -mod4(g.oy);
  a.nby = (g.ny - a.yb + C::BY - 1) / C::BY;
  a.gr = g.nx == 64 ? 1 : 0;
  const int nbz = (g.nz + C::BZ - 1) / C::BZ;
  const FoldCoef<typename C::T> f = make_fold<typename C::T>(p);
  k_block<C><<<dim3((unsigned)a.nby, (unsigned)nbz, 1), 64 * C::NW, 0, st>>>(
      (const typename C::V2*)s, (typename C::V2*)d, a, f, p.seed);
  return true;
  }
}

// whether k_block can run this launch: one Backend::fused() allows (its x ghosts are the
// boundary values ensure_bc wrote), the whole interior (no z-runs / store mask / reserve),
// whole non-periodic x rows of at most 64 cells, a 32-bit Philox counter, state buffers below
// 1 GiB (k_block addresses a whole buffer through one descriptor)
inline bool block_supported(const FusedArgs& a) {
  const Geom& g = a.g;
  if (gs::total_elems(g) * 16 >= (int64_t)1 << 30) return false;
  return a.allow_block && !g.periodic && g.nx <= 64 && g.ox == 0 && g.nx == g.Lx && a.q32 && a.zlo[0] == 0 &&
         a.zlen[0] == g.nz && a.zlen[1] == 0 && a.mx0 == 0 && a.mx1 == g.nx && a.my0 == 0 &&
         a.my1 == g.ny && a.reserve == 0;
}
