// SPDX-License-Identifier: MIT
// k_fused: T time levels per HBM pass over the interior (temporal blocking) for gfx950.
// Included inside namespace gsk by kernels.hpp, after stencil.hpp.
//
// Work unit = one (tile, z-plane) pair; the units are split evenly over a persistent grid
// of `occupancy x CUs` workgroups, each walking one or two contiguous z-segments.
// Tile = 64 columns (one lane each) x WAVES*ROWS rows of level-0 data (ghosts included);
// it yields (64-2T) x ystep interior outputs.  A segment [z0,z1) streams level-0 planes
// z0-T .. z1+T-1; at iteration p level l produces plane p-l; level T is stored.
//
// Register plan (no rotation copies): level-0 planes live in a 3-deep ring LD[3] (plane p,
// p-1 and the prefetch of p+1); level-l outputs in a 2-deep ring OUT[l][2]; per consumer
// level a running partial sum A (xy-neighbours of plane q-1 plus plane q-2).  The loop is
// unrolled by the ring period (6) so every ring index is a compile-time constant.
// Memory goes through buffer descriptors built per plane: 32-bit lane offsets, no address
// VGPRs, out-of-range loads return 0 and masked stores use an out-of-range offset.
// Intermediate levels outside the global domain (non-periodic) are reset to the boundary
// value of their time level -- what the single-step path reads from its ghost shell.
#pragma once

struct FusedArgs {
  Geom g;
  int32_t ntx, nty;
  int32_t xstep, ystep;
  int32_t ybase;
  int32_t bcfix;
  int64_t units;
  int32_t sched;   // 0: units split evenly; 1: XCD-grouped z-chunks walked in lockstep
  int32_t nchunk;  // sched 1: z-chunks per tile
  int32_t ntiles;  // tiles enumerated (ntx * nty, or the inner / ring subset)
  // tile subset (comm/compute overlap of packed halos): 0 all tiles, 1 the inner rectangle
  // [itx0, itx1) x [ity0, ity1) (no input cell within reach of a fresh halo), 2 its ring
  int32_t tmode;
  int32_t sides;  // bit0/1/2/3: neighbour at -x/+x/-y/+y (whose halo is in flight)
  int32_t itx0, itx1, ity0, ity1;
  int32_t grpM;    // sched 1: workgroups per XCD group (grid = 8 * grpM)
  int32_t cfg;     // tile/prefetch configuration index (fused_cfg_names)
  int64_t t;
  int64_t buf_bytes;  // bytes of one state buffer (descriptor range)
  int32_t reserve;    // workgroup slots to leave free (comm kernels running alongside)
  // output z-runs [zlo[r], zlo[r] + zlen[r]) (zlen[1] may be 0); a tile's units enumerate the
  // planes of run 0 then run 1 (nzv = zlen[0] + zlen[1] units per tile)
  int32_t zlo[2], zlen[2];
  int32_t nzv;
};

// Folded update coefficients: u' = au*u + asu*su + ac - dt*uvv + ar*r ; v' = bv*v + bsv*sv + dt*uvv
template <typename T>
struct FoldCoef {
  T au, asu, ac, ar, dt, bv, bsv;
};

template <typename T>
inline FoldCoef<T> make_fold(const gs::Params& p) {
  FoldCoef<T> f;
  f.au = (T)(1.0 - p.dt * (p.Du + p.F));
  f.asu = (T)(p.dt * p.Du / 6.0);
  f.ac = (T)(p.dt * p.F);
  f.ar = (T)(p.dt * p.noise);
  f.dt = (T)p.dt;
  f.bv = (T)(1.0 - p.dt * (p.Dv + p.F + p.k));
  f.bsv = (T)(p.dt * p.Dv / 6.0);
  return f;
}

typedef unsigned int gs_u2 __attribute__((ext_vector_type(2)));
typedef unsigned int gs_u4 __attribute__((ext_vector_type(4)));

// Descriptor for the plane starting `off_bytes` into a buffer of `total_bytes`.  The range is
// empty when the plane is disabled (total_bytes == 0) or starts outside the buffer, so every
// access through it is dropped (loads return 0) -- never a wild address.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t plane_rsrc(const void* base, int64_t off_bytes,
                                                             int64_t total_bytes) {
  const int64_t rem = total_bytes - off_bytes;
  const bool inside = total_bytes > 0 && off_bytes >= 0 && rem > 0;
  const int nrec = inside ? (int)(rem > 0x7ffffff0LL ? 0x7ffffff0LL : rem) : 0;
  return __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)base + off_bytes), 0, nrec,
                                           0x00020000);
}

// Descriptor for storage plane `plane` (0-based, ghosts included) of a buffer of `nplanes`
// planes of `pzb` bytes, covering that plane only.  All the checks are 32-bit and wave-uniform
// (SALU); the 64-bit form above needs VALU compares.  Accesses past the plane's end -- tile
// rows beyond the ghost layer -- read 0 instead of the next plane's data: neither ever reaches
// a stored output (an output depends on rows within T <= H of it).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t plane_rsrc_p(const void* base, int plane,
                                                               int nplanes, int64_t pzb, bool on) {
  const bool inside = on && (unsigned)plane < (unsigned)nplanes;
  const int nrec = inside ? (int)(pzb > 0x7ffffff0LL ? 0x7ffffff0LL : pzb) : 0;
  return __builtin_amdgcn_make_buffer_rsrc(
      (void*)((const char*)base + (int64_t)(inside ? plane : 0) * pzb), 0, nrec, 0x00020000);
}

__device__ __forceinline__ float2 bload(__amdgpu_buffer_rsrc_t r, int voff, int soff, float2*) {
  const gs_u2 v = __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, 0);
  return make_float2(__uint_as_float(v.x), __uint_as_float(v.y));
}
__device__ __forceinline__ double2 bload(__amdgpu_buffer_rsrc_t r, int voff, int soff, double2*) {
  const gs_u4 v = __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0);
  return make_double2(__longlong_as_double(((long long)v.y << 32) | v.x),
                      __longlong_as_double(((long long)v.w << 32) | v.z));
}
__device__ __forceinline__ void bstore(__amdgpu_buffer_rsrc_t r, int voff, int soff, float2 c) {
  gs_u2 v;
  v.x = __float_as_uint(c.x);
  v.y = __float_as_uint(c.y);
  __builtin_amdgcn_raw_buffer_store_b64(v, r, voff, soff, 0);
}
__device__ __forceinline__ void bstore(__amdgpu_buffer_rsrc_t r, int voff, int soff, double2 c) {
  const unsigned long long a = (unsigned long long)__double_as_longlong(c.x);
  const unsigned long long b = (unsigned long long)__double_as_longlong(c.y);
  gs_u4 v;
  v.x = (unsigned)a; v.y = (unsigned)(a >> 32); v.z = (unsigned)b; v.w = (unsigned)(b >> 32);
  __builtin_amdgcn_raw_buffer_store_b128(v, r, voff, soff, 0);
}

// a ^ b ^ c in one gfx950 instruction (the compiler does not form v_bitop3 from xor chains)
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t r;
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "s"(c));
  return r;
}

// Device form of gs::noise_block (same stream, bit for bit).
//  * The 10-round key schedule is rebuilt from an opaque copy of the seed at every call:
//    otherwise the compiler hoists the 20 loop-invariant key words out of the plane loop, runs
//    out of SGPRs and spills them to VGPR lanes (one v_readlane per use in the hot loop).
//    Rebuilt, they are 20 SALU adds.
//  * Rounds 1-2 still see wave-uniform counter words (step, and its products), which the
//    compiler folds on the SALU; from round 3 on every word varies per lane and each output
//    word's two xors become one v_bitop3.
template <bool kOpaqueStep = true>
__device__ __forceinline__ gs::U4 noise_block_dev(int64_t gx, int64_t gy4, int64_t gz, int64_t Lx,
                                                  int64_t Ly, uint64_t step, uint64_t seed) {
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
  asm volatile("" : "+s"(k0), "+s"(k1));
  const uint64_t Ly4 = ((uint64_t)Ly + 3) >> 2;
  const uint64_t q = (uint64_t)gx + (uint64_t)Lx * ((uint64_t)gy4 + Ly4 * (uint64_t)gz);
  uint32_t c0 = (uint32_t)q, c1 = (uint32_t)(q >> 32), c2 = (uint32_t)step,
           c3 = (uint32_t)(step >> 32);
  // the step words are wave-uniform and loop-invariant per time level: without this the
  // compiler hoists their round-1/2 products out of the plane loop and spills them to VGPR
  // lanes (a v_readlane per use); recomputed they are a few SALU ops
  if constexpr (kOpaqueStep) asm volatile("" : "+s"(c2), "+s"(c3));
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    if (r < 2) {
      gs::philox_round(c0, c1, c2, c3, k0, k1);
    } else {
      const uint64_t m0 = (uint64_t)0xD2511F53u * c0;
      const uint64_t m1 = (uint64_t)0xCD9E8D57u * c2;
      const uint32_t n0 = xor3((uint32_t)(m1 >> 32), c1, k0);
      const uint32_t n2 = xor3((uint32_t)(m0 >> 32), c3, k1);
      c0 = n0; c1 = (uint32_t)m1; c2 = n2; c3 = (uint32_t)m0;
    }
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return gs::U4{c0, c1, c2, c3};
}

// Compile-time configuration of one fused-kernel instantiation.
//   ROWS x WAVES : rows per wave x waves per workgroup (tile height = ROWS*WAVES)
//   PF           : level-0 prefetch distance in planes (register ring of PF+2 planes)
//   SKEW         : level l consumes level l-1's output of the previous iteration, so all
//                  levels share ONE workgroup barrier per plane (output ring of 3)
constexpr int gs_gcd(int a, int b) { return b == 0 ? a : gs_gcd(b, a % b); }
constexpr int gs_lcm(int a, int b) { return a / gs_gcd(a, b) * b; }

template <typename T_, int TL_, int ROWS_, int WAVES_, int PF_, bool PERIODIC_, bool NOISE_,
          int MINW_ = 1, bool SKEW_ = false, int ABL_ = 0>
struct FCfg {
  static constexpr int MINW = MINW_;  // __launch_bounds__ min waves per SIMD
  using T = T_;
  using V2 = typename Vec2<T>::type;
  static constexpr int TL = TL_, ROWS = ROWS_, WAVES = WAVES_, PF = PF_;
  static constexpr bool PERIODIC = PERIODIC_, NOISE = NOISE_, SKEW = SKEW_;
  // the noise coefficient dt*noise*2^-31 in a VGPR (saves the uniform's v_mul; an SGPR
  // copy spilled, profiles/r1_ab_noise_fold.txt); ABL bit 6 restores the separate scale
  static constexpr bool FOLD31 = !(ABL_ & 64);
  // fp32 T=3: x-neighbour pair sum as one DPP move + one DPP add (lane_pair_sum): -36 VALU
  // and -16 VGPRs per unrolled period, +1.8 % at L=512 (profiles/r1_ab_xsum_dpp.txt); neutral
  // at T=2, which keeps the compiler's form.  ABL bit 7 restores it at T=3.
  static constexpr bool XSUM_DPP = sizeof(T_) == 4 && TL_ == 3 && !(ABL_ & 128);
  // ablation (timing experiments only, results are WRONG): bit0 = no workgroup barriers,
  // bit1 = every level-0 load reads plane 0 (L2-resident); bit2 (results exact) = hoistable
  // Philox key schedule (the pre-noise_block_dev code generation); bit3 (results exact) =
  // hoistable step words in the Philox counter (before the opaque-step change); bit4 (exact) =
  // float2 LDS reads split by the compiler into two ds_read_b32 (before lds_load2); bit5
  // (exact) = 64-bit buffer-range descriptors (before plane_rsrc_p); bit6 (exact) = separate
  // 2^-31 noise scale (before FOLD31); bit7 (exact) = compiler-formed x-neighbour sums at T=3
  // (before XSUM_DPP)
  static constexpr int ABL = ABL_;
  static constexpr int R = PF + 2;                    // level-0 ring slots
  static constexpr int NS = SKEW ? 3 : 2;             // level-l output ring / xch buffers
  static constexpr int PERIOD = gs_lcm(R, NS);
  static constexpr int NO = TL > 1 ? TL - 1 : 1;
};

template <class C>
struct FusedState {
  using V2 = typename C::V2;
  typename C::T ar31;  // dt * noise * 2^-31 held in a VGPR (C::FOLD31)
  V2 LD[C::R][C::ROWS];
  V2 OUT[C::NO][C::NS][C::ROWS];
  V2 A[C::TL][C::ROWS];
};

// Per-segment constants (wave-uniform values and the lane's offsets).
struct FusedSeg {
  int p, pend, ldend, z0;
  int lane, wave;
  int voff, svoff, pitchb;
  int srow0, srow1;
  int64_t gx, gxu, gy0;
  bool edge;
};

template <class C>
__device__ __forceinline__ int64_t gwrap(int64_t v, int64_t L) {
  if constexpr (C::PERIODIC) return wrap(v, L);
  else return v;
}

// left + right x-neighbours in two instructions: one DPP move and one DPP add (the compiler
// pairs the u and v halves into v_pk_add_f32 instead and keeps both moves).  Same rounding
// as lane_from_left(v) + lane_from_right(v).  The leading s_nop covers the VALU-write ->
// DPP-read hazard the compiler cannot see through inline asm.
__device__ __forceinline__ float lane_pair_sum(float v) {
  float t, r;
  asm volatile(
      "s_nop 1\n\t"
      "v_mov_b32_dpp %1, %2 wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
      "v_add_f32_dpp %0, %2, %1 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1"
      : "=v"(r), "=&v"(t)
      : "v"(v));
  return r;
}

// One (u, v) pair from LDS as a single 8-byte ds_read_b64 (the compiler otherwise splits a
// float2 into two ds_read_b32 at an 8-byte lane stride: 2-way bank conflicts).
__device__ __forceinline__ float2 lds_load2(const float2* p) {
  const uint64_t b = *reinterpret_cast<const uint64_t*>(__builtin_assume_aligned(p, 8));
  return make_float2(__uint_as_float((uint32_t)b), __uint_as_float((uint32_t)(b >> 32)));
}
__device__ __forceinline__ double2 lds_load2(const double2* p) { return *p; }

// One pipeline iteration p (i = p - pstart).  IR = i % R, IS = i % NS.
// Non-skewed: level l+1 is computed from level l of the SAME iteration (one barrier per level).
// Skewed: level l+1 consumes level l's output of the PREVIOUS iteration, so every level's
// input rows are published before a single barrier; level l produces plane p - (2l + 1).
template <class C, typename T, int IR, int IS>
__device__ __forceinline__ void fused_iter(FusedState<C>& S,
                                           typename C::V2 (*xch)[C::NS][C::WAVES][2][64],
                                           const FusedArgs& a, const FoldCoef<T>& f,
                                           uint64_t seed, const typename C::V2* src,
                                           typename C::V2* dst, const FusedSeg& sg) {
  using V2 = typename C::V2;
  constexpr int ROWS = C::ROWS, WAVES = C::WAVES, TL = C::TL, NS = C::NS;
  const Geom& g = a.g;
  const int p = sg.p;
  const int64_t PZB = gs::plane_elems(g) * (int64_t)sizeof(V2);
  // prefetch level-0 plane p+PF into the ring slot of plane p-2.  Issued unconditionally
  // (an empty descriptor past the segment) so every iteration has the same VMEM count and
  // the compiler's s_waitcnt vmcnt(N) can leave the prefetch in flight.
  {
    const bool pf_ok = p + C::PF < sg.ldend;
    const __amdgpu_buffer_rsrc_t r =
        (C::ABL & 32) ? plane_rsrc(src, (C::ABL & 2) ? 0 : (int64_t)(p + C::PF + g.H) * PZB,
                                   pf_ok ? a.buf_bytes : 0)
                      : plane_rsrc_p(src, (C::ABL & 2) ? 0 : p + C::PF + g.H, g.pz, PZB, pf_ok);
#pragma unroll
    for (int j = 0; j < ROWS; ++j)
      S.LD[(IR + C::PF) % C::R][j] = bload(r, sg.voff + j * sg.pitchb, 0, (V2*)nullptr);
  }
  if constexpr (C::SKEW) {
#pragma unroll
    for (int l = 0; l < TL; ++l) {
      const V2* in = l == 0 ? S.LD[IR] : S.OUT[l == 0 ? 0 : l - 1][(IS + NS - 1) % NS];
      xch[l][IS][sg.wave][0][sg.lane] = in[0];
      xch[l][IS][sg.wave][1][sg.lane] = in[ROWS - 1];
    }
    if constexpr (!(C::ABL & 1)) __syncthreads();
  }
#pragma unroll
  for (int l = 0; l < TL; ++l) {
    // input plane of consumer l and the centre plane one before it
    constexpr int kIn = C::SKEW ? (IS + NS - 1) % NS : IS;
    constexpr int kC = C::SKEW ? (IS + NS - 2) % NS : (IS + NS - 1) % NS;
    V2* in = l == 0 ? S.LD[IR] : S.OUT[l == 0 ? 0 : l - 1][kIn];
    V2* Cc = l == 0 ? S.LD[(IR + C::R - 1) % C::R] : S.OUT[l == 0 ? 0 : l - 1][kC];
    if constexpr (!C::SKEW) {
      xch[l][IS][sg.wave][0][sg.lane] = in[0];
      xch[l][IS][sg.wave][1][sg.lane] = in[ROWS - 1];
      if constexpr (!(C::ABL & 1)) __syncthreads();
    }
    V2 up, dn;
    if constexpr (C::ABL & 16) {  // ablation: the compiler's split float2 LDS reads
      up = sg.wave > 0 ? xch[l][IS][sg.wave - 1][1][sg.lane] : in[0];
      dn = sg.wave < WAVES - 1 ? xch[l][IS][sg.wave + 1][0][sg.lane] : in[ROWS - 1];
    } else {
      up = sg.wave > 0 ? lds_load2(&xch[l][IS][sg.wave - 1][1][sg.lane]) : in[0];
      dn = sg.wave < WAVES - 1 ? lds_load2(&xch[l][IS][sg.wave + 1][0][sg.lane]) : in[ROWS - 1];
    }
    const int q = C::SKEW ? p - (2 * l + 1) : p - l - 1;  // plane produced by level l+1
    const int64_t gz = gwrap<C>(g.oz + q, g.Lz);
    const uint64_t tstep = (uint64_t)(a.t + l);
    V2 res[ROWS];
#pragma unroll
    for (int m = 0; m < ROWS / 4; ++m) {
      gs::U4 blk{0, 0, 0, 0};
      if constexpr (C::NOISE) {
        const int64_t gyq = gwrap<C>(sg.gy0 + 4 * m, g.Ly);
        if constexpr (C::ABL & 4) blk = gs::noise_block(sg.gx, gyq >> 2, gz, g.Lx, g.Ly, tstep, seed);
        else blk = noise_block_dev<!(C::ABL & 8)>(sg.gx, gyq >> 2, gz, g.Lx, g.Ly, tstep, seed);
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int j = 4 * m + k;
        const V2 ym = j == 0 ? up : in[j - 1];
        const V2 yp = j == ROWS - 1 ? dn : in[j + 1];
        T xyu, xyv;
        if constexpr (C::XSUM_DPP) {
          xyu = lane_pair_sum(in[j].x) + (ym.x + yp.x);
          xyv = lane_pair_sum(in[j].y) + (ym.y + yp.y);
        } else {
          xyu = (lane_from_left(in[j].x) + lane_from_right(in[j].x)) + (ym.x + yp.x);
          xyv = (lane_from_left(in[j].y) + lane_from_right(in[j].y)) + (ym.y + yp.y);
        }
        const T su = S.A[l][j].x + in[j].x;
        const T sv = S.A[l][j].y + in[j].y;
        const T cu = Cc[j].x, cv = Cc[j].y;
        const T uvv = cu * cv * cv;
        T ru = f.ac;
        if constexpr (C::NOISE) {
          // (folding the 2^-31 of uniform_pm1 into ar saves a v_mul but costs an SGPR; the
          // extra spill reloads made it 2 % slower: profiles/r1_ab_noise_fold.txt)
          const uint32_t w = k == 0 ? blk.x : (k == 1 ? blk.y : (k == 2 ? blk.z : blk.w));
          if constexpr (C::FOLD31) ru = fma(S.ar31, (T)(int32_t)w, ru);
          else ru = fma(f.ar, gs::uniform_pm1<T>(w), ru);
        }
        res[j].x = fma(f.au, cu, fma(f.asu, su, fma(-f.dt, uvv, ru)));
        res[j].y = fma(f.bv, cv, fma(f.bsv, sv, f.dt * uvv));
        S.A[l][j].x = xyu + cu;
        S.A[l][j].y = xyv + cv;
      }
    }
    if (l + 1 < TL) {
      if (sg.edge) {
        const T bu = (T)gs::bc_u(a.t + l + 1);
        const bool zout = (g.oz + q < 0) || (g.oz + q >= g.Lz);
        const bool xout = sg.gxu < 0 || sg.gxu >= g.Lx;
#pragma unroll
        for (int j = 0; j < ROWS; ++j) {
          const int64_t gyj = sg.gy0 + j;
          if (zout || xout || gyj < 0 || gyj >= g.Ly) {
            res[j].x = bu;
            res[j].y = (T)0;
          }
        }
      }
#pragma unroll
      for (int j = 0; j < ROWS; ++j) S.OUT[l][IS][j] = res[j];
    } else {
      {  // unconditional stores: planes before the segment go to an empty descriptor
        const bool st_ok = q >= sg.z0;
        const __amdgpu_buffer_rsrc_t w =
            (C::ABL & 32) ? plane_rsrc(dst, (int64_t)(q + g.H) * PZB, st_ok ? a.buf_bytes : 0)
                          : plane_rsrc_p(dst, q + g.H, g.pz, PZB, st_ok);
#pragma unroll
        for (int j = 0; j < ROWS; ++j) {
          const int off = (j >= sg.srow0 && j < sg.srow1) ? sg.svoff + j * sg.pitchb : (int)0x80000000;
          bstore(w, off, 0, res[j]);
        }
      }
    }
  }
}

// Unrolled walk over one ring period; returns false when the segment is done.
template <class C, typename T, int I>
__device__ __forceinline__ bool fused_period(FusedState<C>& S,
                                             typename C::V2 (*xch)[C::NS][C::WAVES][2][64],
                                             const FusedArgs& a, const FoldCoef<T>& f,
                                             uint64_t seed, const typename C::V2* src,
                                             typename C::V2* dst, FusedSeg& sg) {
  if constexpr (I == C::PERIOD) {
    return true;
  } else {
    fused_iter<C, T, I % C::R, I % C::NS>(S, xch, a, f, seed, src, dst, sg);
    if (++sg.p >= sg.pend) return false;
    return fused_period<C, T, I + 1>(S, xch, a, f, seed, src, dst, sg);
  }
}

// Enumerated tile index -> (tx, ty) of the full ntx x nty tile grid for the tile subset.
__device__ __forceinline__ void map_tile(const FusedArgs& a, int t, int& tx, int& ty) {
  if (a.tmode == 0) {
    tx = t % a.ntx;
    ty = t / a.ntx;
  } else if (a.tmode == 1) {
    const int w = a.itx1 - a.itx0;
    tx = a.itx0 + t % w;
    ty = a.ity0 + t / w;
  } else {
    // ring: full rows below ity0, the left / right parts of rows [ity0, ity1), full rows above
    const int n0 = a.ity0 * a.ntx;
    if (t < n0) {
      tx = t % a.ntx;
      ty = t / a.ntx;
      return;
    }
    t -= n0;
    const int mid = a.ntx - (a.itx1 - a.itx0), h = a.ity1 - a.ity0;
    if (t < h * mid) {
      ty = a.ity0 + t / mid;
      const int r = t % mid;
      tx = r < a.itx0 ? r : a.itx1 + (r - a.itx0);
      return;
    }
    t -= h * mid;
    tx = t % a.ntx;
    ty = a.ity1 + t / a.ntx;
  }
}

template <class C, typename T>
__global__ __launch_bounds__(64 * C::WAVES, C::MINW) void k_fused(const typename C::V2* __restrict__ s,
                                                         typename C::V2* __restrict__ d,
                                                         FusedArgs a, FoldCoef<T> f,
                                                         uint64_t seed) {
  using V2 = typename C::V2;
  constexpr int ROWS = C::ROWS, WAVES = C::WAVES, TL = C::TL;
  static_assert(ROWS % 4 == 0, "rows per wave must hold whole noise quads");
  __shared__ V2 xch[TL][C::NS][WAVES][2][64];  // [level][ring][wave][first/last row][lane]
  const Geom& g = a.g;
  FusedSeg sg;
  sg.lane = threadIdx.x & 63;
  sg.wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  sg.pitchb = g.px * (int)sizeof(V2);
  const int nzv = a.nzv;
  // Work list of this workgroup: logical units lu = chunk * ntiles + tile, lu0, lu0 + lstep, ...
  // (sched 0: one "unit", the even share [u, uend) of all tile-planes).
  // Workgroups b, b+8, b+16, ... share an XCD (round-robin dispatch; speed only, never
  // correctness): sched 1/2 give each XCD a contiguous range of units, i.e. spatially adjacent
  // tiles at the same z-chunk, so neighbours' shared halo lines are read while still resident
  // in that XCD's L2.  sched 1: one unit per workgroup; sched 2: the XCD's workgroups sweep
  // its range in lockstep rounds.
  const int b = blockIdx.x;
  const int nunits = a.ntiles * a.nchunk;
  int lu0 = 0, lu1 = 1, lstep = 1;
  if (a.sched == 1) {
    lu0 = (b % 8) * a.grpM + b / 8;
    lu1 = lu0 + 1;
    if (lu0 >= nunits) return;  // whole workgroup, before any barrier
  } else if (a.sched == 2) {
    const int per = (nunits + 7) / 8;
    lu0 = (b % 8) * per + b / 8;
    lu1 = min((b % 8 + 1) * per, nunits);
    lstep = gridDim.x / 8;
    if (lu0 >= lu1) return;
  }
  FusedState<C> S;
  if constexpr (C::FOLD31) {
    // exact: power-of-two scaling (gs::uniform_pm1 = int * 2^-31); a VGPR copy keeps the
    // coefficient out of the (full) SGPR budget
    const T c = f.ar * (T)4.656612873077392578125e-10;
    if constexpr (sizeof(T) == 4) asm volatile("v_mov_b32 %0, %1" : "=v"(S.ar31) : "s"(c));
    else asm volatile("v_mov_b64 %0, %1" : "=v"(S.ar31) : "s"(c));
  }

  for (int lu = lu0; lu < lu1; lu += lstep) {
    int64_t u, uend;
    if (a.sched == 0) {
      const int64_t U = a.units;
      u = (int64_t)blockIdx.x * U / gridDim.x;
      uend = (int64_t)(blockIdx.x + 1) * U / gridDim.x;
    } else {
      const int chunk = lu / a.ntiles, tile = lu % a.ntiles;
      u = (int64_t)tile * nzv + (int64_t)chunk * nzv / a.nchunk;
      uend = (int64_t)tile * nzv + (int64_t)(chunk + 1) * nzv / a.nchunk;
    }
    while (u < uend) {
      const int tile = (int)(u / nzv);
      const int zv = (int)(u % nzv);
      // a segment never crosses from one z-run into the other
      const int run = zv < a.zlen[0] ? 0 : 1;
      const int rv0 = run ? a.zlen[0] : 0;
      const int rv1 = run ? nzv : a.zlen[0];
      const int zv1 = (int)std::min<int64_t>(rv1, zv + (uend - u));
      const int z0 = a.zlo[run] + (zv - rv0);
      const int z1 = z0 + (zv1 - zv);
      u += zv1 - zv;
      int tx, ty;
      map_tile(a, tile, tx, ty);
      const int X0 = tx * a.xstep - TL;
      const int Y0 = a.ybase + ty * a.ystep - TL;
      const int x = X0 + sg.lane;
      const int ylo = Y0 + sg.wave * ROWS;
      // lane byte offset inside a plane (row ylo); negative values are out of range
      sg.voff = ((ylo + g.H) * g.px + x + g.xo) * (int)sizeof(V2);
      sg.gxu = g.ox + x;
      sg.gx = gwrap<C>(sg.gxu, g.Lx);
      sg.gy0 = g.oy + ylo;
      const int ox1 = min(X0 + TL + a.xstep, g.nx);
      const int oy0 = max(Y0 + TL, 0), oy1 = min(Y0 + TL + a.ystep, g.ny);
      const bool xin = x >= max(X0 + TL, 0) && x < ox1;
      sg.svoff = xin ? sg.voff : (int)0x80000000;  // masked lanes store out of range
      sg.srow0 = max(oy0 - ylo, 0);
      sg.srow1 = min(oy1 - ylo, ROWS);
      sg.edge = a.bcfix &&
          (g.ox + X0 < 0 || g.ox + X0 + 64 > g.Lx || g.oy + Y0 < 0 ||
           g.oy + Y0 + WAVES * ROWS > g.Ly || g.oz + z0 - TL < 0 || g.oz + z1 + TL > g.Lz);
      sg.z0 = z0;
  #pragma unroll
      for (int l = 0; l < TL; ++l)
  #pragma unroll
        for (int j = 0; j < ROWS; ++j) S.A[l][j].x = S.A[l][j].y = (T)0;
      sg.p = z0 - TL;
      sg.ldend = z1 + TL;
      sg.pend = C::SKEW ? z1 + 2 * TL - 1 : z1 + TL;
      const int64_t PZB = gs::plane_elems(g) * (int64_t)sizeof(V2);
  #pragma unroll
      for (int k = 0; k < C::PF; ++k) {
        {
          const __amdgpu_buffer_rsrc_t r = plane_rsrc_p(s, sg.p + k + g.H, g.pz, PZB,
                                                        sg.p + k < sg.ldend);
  #pragma unroll
          for (int j = 0; j < ROWS; ++j) S.LD[k][j] = bload(r, sg.voff + j * sg.pitchb, 0, (V2*)nullptr);
        }
      }
      while (fused_period<C, T, 0>(S, xch, a, f, seed, s, d, sg)) {
      }
    }
  }  // work list
}

// ------------------------------------------------------------------------------------------
inline int& fused_sched_slot();

template <class C, typename T>
struct FusedLaunch {
  static int occupancy() {
    static int occ = -1;
    if (occ < 0) {
      int o = 0;
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, k_fused<C, T>, 64 * C::WAVES, 0) !=
              hipSuccess || o < 1)
        o = 1;
      occ = o;
    }
    return occ;
  }
  static void run(const typename C::V2* s, typename C::V2* d, const FusedArgs& a0,
                  const gs::Params& p, hipStream_t st) {
    FusedArgs a = a0;
    a.xstep = 64 - 2 * C::TL;
    a.ystep = (C::WAVES * C::ROWS - 2 * C::TL) & ~3;
    a.ybase = -mod4(a.g.oy - C::TL);  // (oy + ybase - TL) % 4 == 0
    a.ntx = (a.g.nx + a.xstep - 1) / a.xstep;
    a.nty = (a.g.ny - a.ybase + a.ystep - 1) / a.ystep;
    a.ntiles = a.ntx * a.nty;
    if (a.tmode != 0) {
      // inner rectangle: tiles whose level-0 input box [X0, X0 + 64) x [Y0, Y0 + rows) stays
      // inside the interior on every side whose halo is in flight
      const int rows = C::WAVES * C::ROWS;
      int x0 = 0, x1 = a.ntx, y0 = 0, y1 = a.nty;
      if (a.sides & 1) while (x0 < a.ntx && x0 * a.xstep - C::TL < 0) ++x0;
      if (a.sides & 2) while (x1 > x0 && (x1 - 1) * a.xstep - C::TL + 64 > a.g.nx) --x1;
      if (a.sides & 4) while (y0 < a.nty && a.ybase + y0 * a.ystep - C::TL < 0) ++y0;
      if (a.sides & 8)
        while (y1 > y0 && a.ybase + (y1 - 1) * a.ystep - C::TL + rows > a.g.ny) --y1;
      if (x1 <= x0 || y1 <= y0) x0 = x1 = y0 = y1 = 0;  // no inner tile: the ring is all
      a.itx0 = x0; a.itx1 = x1; a.ity0 = y0; a.ity1 = y1;
      const int inner = (x1 - x0) * (y1 - y0);
      a.ntiles = a.tmode == 1 ? inner : a.ntiles - inner;
      if (a.ntiles == 0) return;
    }
    a.units = (int64_t)a.ntiles * a.nzv;
    static int cus = 0;
    if (!cus) {
      int dev = 0;
      (void)hipGetDevice(&dev);
      if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) cus = 256;
    }
    const int64_t slots = std::max<int64_t>(1, (int64_t)occupancy() * cus - a.reserve);
    // enough planes per workgroup to amortise the 2T-plane pipeline fill, but at least one
    // workgroup per (tile, z-run) so short runs (comm/compute-overlap slabs) stay parallel
    const int nruns = a.zlen[1] > 0 ? 2 : 1;
    int64_t nwg = std::max<int64_t>(a.units / (4 * C::TL + 8),
                                    nruns > 1 ? (int64_t)a.ntiles * nruns : 1);
    nwg = std::max<int64_t>(1, std::min<int64_t>(slots, nwg));
    a.nchunk = 1;
    if (a.sched == 1) {
      // one unit per workgroup: never more units than resident slots (a second, partial
      // round of workgroups would double the time)
      int nch = (int)(slots / a.ntiles);
      nch = std::max(1, std::min(nch, a.nzv / (4 * C::TL + 4) > 0 ? a.nzv / (4 * C::TL + 4) : 1));
      a.nchunk = nch;
      const int64_t nunits = (int64_t)a.ntiles * nch;
      a.grpM = (int)((nunits + 7) / 8);
      nwg = 8LL * a.grpM;
    } else if (a.sched == 2) {
      // persistent grid (8 XCD groups of M workgroups); pick the chunk count minimising
      // rounds x (planes per chunk + 2T pipeline fill)
      const int64_t M = std::max<int64_t>(1, slots / 8);
      int best = 1;
      int64_t bcost = INT64_MAX;
      // chunks of >= 2 planes: small sub-domains (one round) trade pipeline fill for
      // parallelism -- L=64 at T=2: 10.4 -> 6.8 us/step; large ones are set by the rounds
      // (profiles/r1_tune_chunking.txt).  GS_FUSED_CHDIV overrides the divisor.
      static const int chdiv = getenv("GS_FUSED_CHDIV") ? atoi(getenv("GS_FUSED_CHDIV")) : 2;
      const int maxch = std::max(1, a.nzv / std::max(1, chdiv));
      for (int nch = 1; nch <= maxch; ++nch) {
        const int64_t per = ((int64_t)a.ntiles * nch + 7) / 8;
        const int64_t rounds = (per + M - 1) / M;
        const int64_t cost = rounds * ((a.nzv + nch - 1) / nch + 2 * C::TL);
        if (cost < bcost) { bcost = cost; best = nch; }
      }
      a.nchunk = best;
      a.grpM = (int)M;
      nwg = 8 * M;
    }
    const FoldCoef<T> f = make_fold<T>(p);
    k_fused<C, T><<<(unsigned)nwg, 64 * C::WAVES, 0, st>>>(s, d, a, f, p.seed);
  }
};

// Tuning hook: a non-default fp32 configuration "<rows>x<waves>:<prefetch>[s|w<n>]" chosen by
// GS_FUSED_CFG at load time or gs_fused_select() at run time (index 0 = measured default).
inline int& fused_sched_slot() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("GS_FUSED_SCHED");
    v = e ? atoi(e) : 0;
  }
  return v;
}

inline const char* const* fused_cfg_names(int* n) {
  static const char* names[] = {"",       "4x8:1",  "4x8:2",  "4x8:4",   "8x4:1",   "8x4:2",
                                "4x16:2", "8x8:2",  "4x8:3",  "8x4:2w3", "8x4:1w3", "4x8:2w4",
                                "8x4:3",  "4x6:2",  "4x12:2", "4x4:2",   "4x12:3",  "8x4:1s",
                                "8x4:4s", "4x8:1s", "4x8:4s", "abl1",   "abl2",    "abl3",
                                "4x8:1w4", "4x16:1", "4x16:2w4", "4x8:2w3", "abl4", "4x8:1abl4",
                                "4x12:2s", "4x12:1s", "4x6:2s", "4x12:1", "4x12:1s-abl1",
                                "4x12:1s-abl2", "4x12:1s-abl8", "4x12:2s-abl8", "4x12:1s-abl16",
                                "4x12:2s-abl16", "4x12:1s-abl32", "4x12:1s-abl64",
                                "4x12:2s-abl64", "4x12:1s-abl128", "4x12:2s-abl128", "(unused)",
                                "4x8:1s-abl64"};
  *n = (int)(sizeof(names) / sizeof(names[0]));
  return names;
}

inline int& fused_cfg_slot() {
  static int v = -1;
  return v;
}

inline int fused_cfg_lookup(const char* e) {
  int n = 0;
  const char* const* names = fused_cfg_names(&n);
  if (!e) return 0;
  for (int i = 1; i < n; ++i)
    if (!strcmp(e, names[i])) return i;
  return e[0] ? -1 : 0;
}

inline int fused_cfg_env() {
  int& v = fused_cfg_slot();
  if (v < 0) {
    const int k = fused_cfg_lookup(getenv("GS_FUSED_CFG"));
    v = k < 0 ? 0 : k;
  }
  return v;
}

template <typename T, int TL, bool PER, bool NZ>
void run_fused_cfg(const typename Vec2<T>::type* s, typename Vec2<T>::type* d, const FusedArgs& a,
                   const gs::Params& p, hipStream_t st) {
  if constexpr (sizeof(T) == 8 && !PER && NZ) {
    switch (a.cfg) {  // fp64: only shapes that fit the register file without spills
      case 1: FusedLaunch<FCfg<T, TL, 4, 8, 1, PER, NZ>, T>::run(s, d, a, p, st); return;
      case 13: FusedLaunch<FCfg<T, TL, 4, 6, 2, PER, NZ>, T>::run(s, d, a, p, st); return;
      case 15: FusedLaunch<FCfg<T, TL, 4, 4, 2, PER, NZ>, T>::run(s, d, a, p, st); return;
      case 19: FusedLaunch<FCfg<T, TL, 4, 8, 1, PER, NZ, 1, true>, T>::run(s, d, a, p, st); return;
      case 32: FusedLaunch<FCfg<T, TL, 4, 6, 2, PER, NZ, 1, true>, T>::run(s, d, a, p, st); return;
      case 33: FusedLaunch<FCfg<T, TL, 4, 12, 1, PER, NZ>, T>::run(s, d, a, p, st); return;
      case 46: FusedLaunch<FCfg<T, TL, 4, 8, 1, PER, NZ, 1, true, 64>, T>::run(s, d, a, p, st); return;
      default: break;
    }
  }
  if constexpr (sizeof(T) == 4 && !PER && NZ) {
    switch (a.cfg) {
      case 1: FusedLaunch<FCfg<T, TL, 4, 8, 1, PER, NZ>, T>::run(s, d, a, p, st); return;
      case 2: FusedLaunch<FCfg<T, TL, 4, 8, 2, PER, NZ>, T>::run(s, d, a, p, st); return;
      case 3: FusedLaunch<FCfg<T, TL, 4, 8, 4, PER, NZ>, T>::run(s, d, a, p, st); return;
      case 4: FusedLaunch<FCfg<T, TL, 8, 4, 1, PER, NZ>, T>::run(s, d, a, p, st); return;
      case 5: FusedLaunch<FCfg<T, TL, 8, 4, 2, PER, NZ>, T>::run(s, d, a, p, st); return;
      case 6: FusedLaunch<FCfg<T, TL, 4, 16, 2, PER, NZ>, T>::run(s, d, a, p, st); return;
      case 7: FusedLaunch<FCfg<T, TL, 8, 8, 2, PER, NZ>, T>::run(s, d, a, p, st); return;
      case 8: FusedLaunch<FCfg<T, TL, 4, 8, 3, PER, NZ>, T>::run(s, d, a, p, st); return;
      case 9: FusedLaunch<FCfg<T, TL, 8, 4, 2, PER, NZ, 3>, T>::run(s, d, a, p, st); return;
      case 10: FusedLaunch<FCfg<T, TL, 8, 4, 1, PER, NZ, 3>, T>::run(s, d, a, p, st); return;
      case 11: FusedLaunch<FCfg<T, TL, 4, 8, 2, PER, NZ, 4>, T>::run(s, d, a, p, st); return;
      case 12: FusedLaunch<FCfg<T, TL, 8, 4, 3, PER, NZ>, T>::run(s, d, a, p, st); return;
      case 13: FusedLaunch<FCfg<T, TL, 4, 6, 2, PER, NZ>, T>::run(s, d, a, p, st); return;
      case 14: FusedLaunch<FCfg<T, TL, 4, 12, 2, PER, NZ>, T>::run(s, d, a, p, st); return;
      case 15: FusedLaunch<FCfg<T, TL, 4, 4, 2, PER, NZ>, T>::run(s, d, a, p, st); return;
      case 16: FusedLaunch<FCfg<T, TL, 4, 12, 3, PER, NZ>, T>::run(s, d, a, p, st); return;
      case 17: FusedLaunch<FCfg<T, TL, 8, 4, 1, PER, NZ, 1, true>, T>::run(s, d, a, p, st); return;
      case 18: FusedLaunch<FCfg<T, TL, 8, 4, 4, PER, NZ, 1, true>, T>::run(s, d, a, p, st); return;
      case 19: FusedLaunch<FCfg<T, TL, 4, 8, 1, PER, NZ, 1, true>, T>::run(s, d, a, p, st); return;
      case 20: FusedLaunch<FCfg<T, TL, 4, 8, 4, PER, NZ, 1, true>, T>::run(s, d, a, p, st); return;
      case 21: FusedLaunch<FCfg<T, TL, 4, 12, 2, PER, NZ, 1, false, 1>, T>::run(s, d, a, p, st); return;
      case 22: FusedLaunch<FCfg<T, TL, 4, 12, 2, PER, NZ, 1, false, 2>, T>::run(s, d, a, p, st); return;
      case 23: FusedLaunch<FCfg<T, TL, 4, 12, 2, PER, NZ, 1, false, 3>, T>::run(s, d, a, p, st); return;
      case 24: FusedLaunch<FCfg<T, TL, 4, 8, 1, PER, NZ, 4>, T>::run(s, d, a, p, st); return;
      case 25: FusedLaunch<FCfg<T, TL, 4, 16, 1, PER, NZ>, T>::run(s, d, a, p, st); return;
      case 26: FusedLaunch<FCfg<T, TL, 4, 16, 2, PER, NZ, 4>, T>::run(s, d, a, p, st); return;
      case 27: FusedLaunch<FCfg<T, TL, 4, 8, 2, PER, NZ, 3>, T>::run(s, d, a, p, st); return;
      case 28: FusedLaunch<FCfg<T, TL, 4, 12, 2, PER, NZ, 1, false, 4>, T>::run(s, d, a, p, st); return;
      case 29: FusedLaunch<FCfg<T, TL, 4, 8, 1, PER, NZ, 1, false, 4>, T>::run(s, d, a, p, st); return;
      case 30: FusedLaunch<FCfg<T, TL, 4, 12, 2, PER, NZ, 1, true>, T>::run(s, d, a, p, st); return;
      case 31: FusedLaunch<FCfg<T, TL, 4, 12, 1, PER, NZ, 1, true>, T>::run(s, d, a, p, st); return;
      case 32: FusedLaunch<FCfg<T, TL, 4, 6, 2, PER, NZ, 1, true>, T>::run(s, d, a, p, st); return;
      case 33: FusedLaunch<FCfg<T, TL, 4, 12, 1, PER, NZ>, T>::run(s, d, a, p, st); return;
      case 34: FusedLaunch<FCfg<T, TL, 4, 12, 1, PER, NZ, 1, true, 1>, T>::run(s, d, a, p, st); return;
      case 35: FusedLaunch<FCfg<T, TL, 4, 12, 1, PER, NZ, 1, true, 2>, T>::run(s, d, a, p, st); return;
      case 36: FusedLaunch<FCfg<T, TL, 4, 12, 1, PER, NZ, 1, true, 8>, T>::run(s, d, a, p, st); return;
      case 37: FusedLaunch<FCfg<T, TL, 4, 12, 2, PER, NZ, 1, true, 8>, T>::run(s, d, a, p, st); return;
      case 38: FusedLaunch<FCfg<T, TL, 4, 12, 1, PER, NZ, 1, true, 16>, T>::run(s, d, a, p, st); return;
      case 39: FusedLaunch<FCfg<T, TL, 4, 12, 2, PER, NZ, 1, true, 16>, T>::run(s, d, a, p, st); return;
      case 40: FusedLaunch<FCfg<T, TL, 4, 12, 1, PER, NZ, 1, true, 32>, T>::run(s, d, a, p, st); return;
      case 41: FusedLaunch<FCfg<T, TL, 4, 12, 1, PER, NZ, 1, true, 64>, T>::run(s, d, a, p, st); return;
      case 42: FusedLaunch<FCfg<T, TL, 4, 12, 2, PER, NZ, 1, true, 64>, T>::run(s, d, a, p, st); return;
      case 43: FusedLaunch<FCfg<T, TL, 4, 12, 1, PER, NZ, 1, true, 128>, T>::run(s, d, a, p, st); return;
      case 44: FusedLaunch<FCfg<T, TL, 4, 12, 2, PER, NZ, 1, true, 128>, T>::run(s, d, a, p, st); return;
      default: break;
    }
  }
  // measured defaults (MI355X, in-process A/B, profiles/r1_tune_inproc.json): fp32 uses the
  // 4x12 tile with a 2-plane prefetch (best at T=2 for 256^3 and at T=3 for 512^3); fp64 4x8
  if constexpr (sizeof(T) == 4) {
    FusedLaunch<FCfg<T, TL, 4, 12, 2, PER, NZ>, T>::run(s, d, a, p, st);
  } else {
    FusedLaunch<FCfg<T, TL, 4, 8, 2, PER, NZ>, T>::run(s, d, a, p, st);
  }
}

template <typename T, int TL>
void run_fused_tl(const typename Vec2<T>::type* s, typename Vec2<T>::type* d, const FusedArgs& a,
                  const gs::Params& p, hipStream_t st) {
  const bool per = a.g.periodic != 0, nz = p.noise != 0.0;
  if (per) {
    if (nz) run_fused_cfg<T, TL, true, true>(s, d, a, p, st);
    else run_fused_cfg<T, TL, true, false>(s, d, a, p, st);
  } else {
    if (nz) run_fused_cfg<T, TL, false, true>(s, d, a, p, st);
    else run_fused_cfg<T, TL, false, false>(s, d, a, p, st);
  }
}

inline bool fused_supported(const Geom& g, int n) {
  if (n < 2 || n > 3 || g.H < n) return false;
  return !(g.periodic && (g.Ly % 4 != 0));  // noise quads would straddle the wrap
}

// cfg / sched < 0: the process-wide selection (GS_FUSED_CFG / GS_FUSED_SCHED or the
// gs_fused_select / gs_fused_sched APIs).
template <typename T>
bool launch_fused(const typename Vec2<T>::type* s, typename Vec2<T>::type* d, const Geom& g,
                  const gs::Params& p, int n, int64_t t, hipStream_t st, int cfg = -1,
                  int sched = -1, int zlo0 = 0, int zlen0 = -1, int zlo1 = 0, int zlen1 = 0,
                  int reserve = 0, int tmode = 0, int sides = 0) {
  if (!fused_supported(g, n)) return false;
  FusedArgs a{};
  if (zlen0 < 0) zlen0 = g.nz;
  if (zlen1 <= 0) zlen1 = 0;
  if (zlen0 <= 0 || zlo0 < 0 || zlo0 + zlen0 > g.nz || (zlen1 && (zlo1 < 0 || zlo1 + zlen1 > g.nz)))
    return false;
  a.zlo[0] = zlo0; a.zlen[0] = zlen0;
  a.zlo[1] = zlo1; a.zlen[1] = zlen1;
  a.nzv = zlen0 + zlen1;
  a.reserve = reserve > 0 ? reserve : 0;
  a.tmode = tmode;
  a.sides = sides;
  a.g = g;
  a.t = t;
  a.cfg = cfg >= 0 ? cfg : fused_cfg_env();
  a.sched = sched >= 0 ? sched : fused_sched_slot();
  if (zlen1) a.sched = 0;  // two short runs: one workgroup per (tile, run)
  a.bcfix = g.periodic ? 0 : 1;
  a.buf_bytes = gs::total_elems(g) * (int64_t)sizeof(typename Vec2<T>::type);
  if (n == 2) run_fused_tl<T, 2>(s, d, a, p, st);
  else run_fused_tl<T, 3>(s, d, a, p, st);
  return true;
}
