// SPDX-License-Identifier: MIT
// k_slab: the boundary shell of an overlapped pass (cell-granular comm/compute overlap).
// Included inside namespace gsk by kernels.hpp, after fused.hpp.
//
// An overlapped k-step pass (engine.h) splits the interior into
//   * the inner box: every output cell at least k from each face whose halo is in flight.  It
//     depends on interior cells only, so k_fused computes it over ALL tiles while the exchange
//     runs, with a store mask that clips its outputs to the box (FusedArgs::mx0..my1);
//   * the shell: the k-deep slabs at those faces, computed here once the halos have landed.
// The reference exchanges halos with blocking Sendrecv! and then computes
// (src/simulation/communication.jl:138-199, src/simulation/public.jl:58-64): no overlap.
//
// A face slab is thin (k cells deep), so it is NOT tiled like the bulk (64 x-lanes per tile
// would waste 61 of 64 lanes on an x face).  Instead, in the face's own frame:
//   A  the lane axis: 64 lanes along one in-plane axis (64 - 2k outputs, DPP neighbours)
//   N  the face normal: the 3k cells [n0 - k, n0 + 2k) the outputs' dependency cone needs,
//      held per lane in registers (level L on cells [L, 3k - L))
//   M  the march axis: one plane per iteration; level L of plane p - L is computed from level
//      L-1's planes p-L-1 .. p-L+1 (three-plane register rings: no LDS, no barriers)
// orientation 0: x face (A=y, N=x, M=z); 1: y face (A=x, N=y, M=z); 2: z face (A=x, N=z, M=y).
// The Philox block of a cell serves the four cells of its y-quad, and each orientation shares
// it along its own y: across a quad of lanes (0: quad_transpose), between a lane's cells (1),
// across four march steps (2: a per-cell block cache).
// A face slab is small, so the launch is latency-bound: the level-0 planes are prefetched
// three iterations ahead, every access goes through a per-unit buffer descriptor (uniform
// offsets on the SALU, no 64-bit address VALU), and a unit's march chunk balances the
// outputs' cone fill against SIMD occupancy (launch_slabs_tl).
// Every wave is an independent unit (face, lane tile, march chunk).
//
// Bit-exactness: the overlapped pass must equal the one-rank run (k_fused everywhere) bit for
// bit, so every cell here evaluates k_fused's exact expression tree (fused.hpp cell_update):
//   fp32  s = (X- + (X+ + ((Y- + Y+) + Z-))) + Z+ ;  fp64  s = ((X- + X+) + ((Y- + Y+) + Z-)) + Z+
//   P = fma(kd, (cu cv) cv, kc);  P = fma(ks, s, P);  P = fma(kcc, c, P);  u += ar31 * int32(w)
// with X/Y/Z the true spatial axes whichever lane or register they come from, the same
// Philox4x32-10 word, and the same reset of intermediate levels outside the global domain.
#pragma once

struct SlabFace {
  int32_t orient;           // 0 x face, 1 y face, 2 z face (see above)
  int32_t n0;               // first output cell along N: outputs [n0, n0 + k)
  int32_t a0, a1;           // outputs along A
  int32_t m0, m1;           // outputs along M
  int32_t ntile, nchunk;    // lane tiles x march chunks
  int32_t abase, astep;     // tile t: lanes at A = abase + t * astep + lane, owning the
                            // outputs [a0 + t * astep, + astep)
  int32_t chunk;            // output planes per chunk
  int32_t u0;               // first unit (wave) of this face
};

struct SlabArgs {
  Geom g;
  int64_t t;
  int32_t nface, nunits;
  SlabFace f[6];
};

template <int OR> struct SlabAxes;  // axis index (0 x, 1 y, 2 z) of A, N, M
template <> struct SlabAxes<0> { static constexpr int A = 1, N = 0, M = 2; };
template <> struct SlabAxes<1> { static constexpr int A = 0, N = 1, M = 2; };
template <> struct SlabAxes<2> { static constexpr int A = 0, N = 2, M = 1; };

template <bool PER>
__device__ __forceinline__ int64_t gwrap_t(int64_t v, int64_t L) {
  if constexpr (PER) return wrap(v, L);
  else return v;
}

// k_fused's neighbour sum: x pair, y pair, z-1, z+1 in its association (see the header)
template <typename T>
__device__ __forceinline__ typename PairT<T>::type slab_sum(
    typename PairT<T>::type xm, typename PairT<T>::type xp, typename PairT<T>::type ym,
    typename PairT<T>::type yp, typename PairT<T>::type zm, typename PairT<T>::type zp) {
  const typename PairT<T>::type yz = (ym + yp) + zm;
  if constexpr (sizeof(T) == 4) return (xm + (xp + yz)) + zp;
  else return ((xm + xp) + yz) + zp;
}

template <typename T, int TL_, bool PER_, bool NOISE_, bool Q32_, int OR_>
struct SCfg {
  using V2 = typename PairT<T>::type;
  static constexpr int TL = TL_, OR = OR_, NC = 3 * TL_;
  static constexpr int PF = 3;  // level-0 prefetch distance (planes)
  static constexpr bool PER = PER_, NOISE = NOISE_, Q32 = Q32_;
  using AX = SlabAxes<OR_>;
};

// per-unit constants
struct SlabUnit {
  __amdgpu_buffer_rsrc_t src, dst;  // descriptors based at (A = -H, N = nb, M = pstart)
  int voff, svoff;       // this lane's byte offset (its A coordinate); for its stores (out of
                         // range on lanes that own no output)
  int sNb, sMb;          // byte strides along N and M
  int pstart;            // first level-0 plane
  int64_t gA, gN0, gM0;  // global coordinate of this lane, of level-0 cell 0, of M = 0
  int mc0, mc1;          // output planes along M
  int qr;                // lane & 3 (orientation 0: the lane's place in its y-quad)
  uint32_t qm1, qm2;     // all-ones where bit 0 / bit 1 of qr is set (branch-free selects)
  bool edge, aout;
};

// m ? b : a bit by bit (one v_bfi_b32); a lane-varying ?: may compile to exec-mask branches
__device__ __forceinline__ uint32_t bsel(uint32_t m, uint32_t a, uint32_t b) {
  return (a & ~m) | (b & m);
}
// a[r] for the lane-varying index r = (m2 ? 2 : 0) + (m1 ? 1 : 0): three v_bfi_b32
__device__ __forceinline__ uint32_t sel4(uint32_t m1, uint32_t m2, uint32_t a0, uint32_t a1,
                                         uint32_t a2, uint32_t a3) {
  return bsel(m2, bsel(m1, a0, a1), bsel(m1, a2, a3));
}

// lane s of each quad receives v of lane (s - M) & 3 (DPP quad_perm rotation)
template <int M>
__device__ __forceinline__ uint32_t quad_rot(uint32_t v) {
  if constexpr (M == 0) return v;
  constexpr int ctrl = M == 1 ? 0x93 : (M == 2 ? 0x4E : 0x39);
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, ctrl, 0xf, 0xf, false);
}

// Orientation 0 (lanes along y, y-quads aligned with lane quads): the four lanes of a quad
// each draw the Philox block of a different cell c0 + r and exchange words, so that lane s
// ends with word s (its y & 3) of each of the four cells' blocks -- one draw per four cells
// instead of four.  W: this lane's block; returns X[c] = word (lane & 3) of cell c0 + c.
//   Y[m] = W[(r + m) & 3] (per-lane rotation); Z[m] = Y[m] of lane (s - m) & 3 (DPP);
//   X[c] = Z[(s - c) & 3].  24 selects + 3 DPP moves.
__device__ __forceinline__ void quad_transpose(uint32_t m1, uint32_t m2, const gs::U4& W,
                                               uint32_t (&X)[4]) {
  const uint32_t w[4] = {W.x, W.y, W.z, W.w};
  uint32_t Z[4];
  Z[0] = sel4(m1, m2, w[0], w[1], w[2], w[3]);
  Z[1] = quad_rot<1>(sel4(m1, m2, w[1], w[2], w[3], w[0]));
  Z[2] = quad_rot<2>(sel4(m1, m2, w[2], w[3], w[0], w[1]));
  Z[3] = quad_rot<3>(sel4(m1, m2, w[3], w[0], w[1], w[2]));
#pragma unroll
  for (int c = 0; c < 4; ++c)
    X[c] = sel4(m1, m2, Z[(4 - c) & 3], Z[(5 - c) & 3], Z[(6 - c) & 3], Z[(7 - c) & 3]);
}

// The Philox block of global cell (gx, gy, gz) at `step` (gs::noise_block's stream); the round
// keys of rounds 4-10 come from VGPRs filled once per unit (kv), not rebuilt per call
template <class C>
__device__ __forceinline__ gs::U4 slab_block(const Geom& g, int64_t gx, int64_t gy, int64_t gz,
                                             int64_t step, uint64_t seed, const uint32_t* kv) {
  if constexpr (C::Q32) {
    const uint32_t Ly4 = (uint32_t)((g.Ly + 3) >> 2);
    return philox_dev<true, true>((uint32_t)gx + (uint32_t)g.Lx * ((uint32_t)(gy >> 2) +
                                                                   Ly4 * (uint32_t)gz),
                                  0u, (uint64_t)step, seed, kv);
  } else {
    return gs::noise_block(gx, gy >> 2, gz, g.Lx, g.Ly, (uint64_t)step, seed);
  }
}

__device__ __forceinline__ uint32_t word_of(const gs::U4& b, int i) {
  return i == 0 ? b.x : (i == 1 ? b.y : (i == 2 ? b.z : b.w));
}

// registers of one unit
template <class C>
struct SlabRegs {
  using V2 = typename C::V2;
  V2 R[C::TL][3][C::NC];   // level L, ring slot (plane mod 3), cell j in [L, NC - L)
  V2 NX[C::PF][C::NC];     // level-0 planes in flight
  gs::U4 PC[C::OR == 2 && C::NOISE ? C::TL + 1 : 1][C::NC];  // orientation 2: block cache
  uint32_t kv[14];         // Philox round keys of rounds 4-10
};

// Level L (1..TL) of plane q from level L-1's ring slots IM (plane q-1), IC (q), IP (q+1).
// The unused entries of R are never touched, so they take no registers.  Level TL is stored.
template <class C, typename T, int L, int IM, int IC, int IP>
__device__ __forceinline__ void slab_level(SlabRegs<C>& S, const SlabArgs& a, const SlabUnit& u,
                                           int q, const FoldCoef<T>& f, T ar31, uint64_t seed) {
  using V2 = typename C::V2;
  using AX = typename C::AX;
  constexpr int TL = C::TL, NC = C::NC, OR = C::OR;
  const Geom& g = a.g;
  const int64_t gM = u.gM0 + q;
  const int64_t Lg[3] = {g.Lx, g.Ly, g.Lz};
  const bool mout = u.edge && (gM < 0 || gM >= Lg[AX::M]);
  const T bu = (T)gs::bc_u(a.t + L);
  const int64_t step = a.t + (L - 1);
  // noise words of this level's cells
  uint32_t wq[C::NOISE ? NC : 1];
  if constexpr (C::NOISE) {
    if constexpr (OR == 0) {
      // y along the lanes: one draw per four cells, exchanged across the lane quad
      const int64_t gy = gwrap_t<C::PER>(u.gA, g.Ly), gz = gwrap_t<C::PER>(gM, g.Lz);
#pragma unroll
      for (int j0 = L; j0 < NC - L; j0 += 4) {
        const int jr = min(j0 + u.qr, NC - L - 1);  // this lane's cell of the group
        const gs::U4 W = slab_block<C>(g, gwrap_t<C::PER>(u.gN0 + jr, g.Lx), gy, gz, step, seed, S.kv);
        uint32_t X[4];
        quad_transpose(u.qm1, u.qm2, W, X);
#pragma unroll
        for (int c = 0; c < 4; ++c)
          if (j0 + c < NC - L) wq[j0 + c] = X[c];
      }
    } else if constexpr (OR == 1) {
      // y along N: the cells of one y-quad share a block (wave-uniform refresh)
      const int64_t gx = gwrap_t<C::PER>(u.gA, g.Lx), gz = gwrap_t<C::PER>(gM, g.Lz);
      gs::U4 blk{0, 0, 0, 0};
#pragma unroll
      for (int j = L; j < NC - L; ++j) {
        const int64_t gy = gwrap_t<C::PER>(u.gN0 + j, g.Ly);
        if (j == L || (gy & 3) == 0) blk = slab_block<C>(g, gx, gy, gz, step, seed, S.kv);
        wq[j] = word_of(blk, (int)(gy & 3));
      }
    } else {
      // y along the march: a cell's block serves four consecutive planes; refreshed at the
      // level's first plane and at every y-quad start (wave-uniform)
      const int64_t gx = gwrap_t<C::PER>(u.gA, g.Lx), gy = gwrap_t<C::PER>(gM, g.Ly);
      const bool refresh = (gy & 3) == 0 || q == u.mc0 - (TL - L);
      const int wi = (int)(gy & 3);
#pragma unroll
      for (int j = L; j < NC - L; ++j) {
        if (refresh) S.PC[L][j] = slab_block<C>(g, gx, gy, gwrap_t<C::PER>(u.gN0 + j, g.Lz), step, seed, S.kv);
        wq[j] = word_of(S.PC[L][j], wi);
      }
    }
  }
#pragma unroll
  for (int j = L; j < NC - L; ++j) {
    const V2 c = S.R[L - 1][IC][j];
    const V2 nm = S.R[L - 1][IC][j - 1], np = S.R[L - 1][IC][j + 1];  // N neighbours
    const V2 mm = S.R[L - 1][IM][j], mp = S.R[L - 1][IP][j];          // M neighbours
    const V2 lm = V2{lane_from_left(c.x), lane_from_left(c.y)};      // A neighbours
    const V2 lp = V2{lane_from_right(c.x), lane_from_right(c.y)};
    V2 sum;
    if constexpr (OR == 0) sum = slab_sum<T>(nm, np, lm, lp, mm, mp);       // X=N Y=A Z=M
    else if constexpr (OR == 1) sum = slab_sum<T>(lm, lp, nm, np, mm, mp);  // X=A Y=N Z=M
    else sum = slab_sum<T>(lm, lp, mm, mp, nm, np);                         // X=A Y=M Z=N
    const V2 tt = c * c.yy;
    const V2 uvv = tt.xx * c.yy;
    V2 P = __builtin_elementwise_fma(f.kd, uvv, f.kc);
    P = __builtin_elementwise_fma(f.ks, sum, P);
    P = __builtin_elementwise_fma(f.kcc, c, P);
    if constexpr (C::NOISE) P.x = fma(ar31, (T)(int32_t)wq[j], P.x);
    if constexpr (L < TL) {
      // outside the global domain: the boundary value of this time level (a select; the
      // cell / plane tests are wave-uniform)
      const int64_t gN = u.gN0 + j;
      const bool out = mout || gN < 0 || gN >= Lg[AX::N];
      const bool rst = u.edge && (out || u.aout);
      S.R[L][IC][j] = rst ? V2{bu, (T)0} : P;
    } else {
      // outputs: cells [TL, 2TL) of planes [mc0, mc1); lanes outside the tile's outputs
      // store to an out-of-range offset (dropped)
      const int off = (q >= u.mc0 && q < u.mc1) ? u.svoff : (int)0x80000000;
      bstore(u.dst, off + (j * u.sNb + (q - u.pstart) * u.sMb), P);
    }
  }
}

// one march iteration p (ring index I = (p - pstart) mod 3): level 0 of plane p from the
// prefetch queue, the prefetch of plane p + PF, then levels 1..TL bottom-up
template <class C, typename T, int I, int L = 1>
__device__ __forceinline__ void slab_levels(SlabRegs<C>& S, const SlabArgs& a, const SlabUnit& u,
                                            int p, const FoldCoef<T>& f, T ar31, uint64_t seed) {
  if constexpr (L <= C::TL) {
    const int q = p - L;
    // level L is needed on planes [mc0 - (TL - L), mc1 + (TL - L)) (the outputs' cone)
    if (q >= u.mc0 - (C::TL - L) && q < u.mc1 + (C::TL - L))
      slab_level<C, T, L, (I - L + 5) % 3, (I - L + 6) % 3, (I - L + 7) % 3>(S, a, u, q, f,
                                                                               ar31, seed);
    slab_levels<C, T, I, L + 1>(S, a, u, p, f, ar31, seed);
  }
}

template <class C>
__device__ __forceinline__ void slab_load(SlabRegs<C>& S, const SlabUnit& u, int slot, int p,
                                          int pend) {
  // planes past the unit's range read through an empty offset (keeps the VMEM count fixed)
  const int sp = p < pend ? (p - u.pstart) * u.sMb : 0;
  const int vo = p < pend ? u.voff : (int)0x80000000;
#pragma unroll
  for (int j = 0; j < C::NC; ++j)
    S.NX[slot][j] = bload(u.src, vo + (j * u.sNb + sp), (typename C::V2*)nullptr);
}

template <class C, typename T, int I>
__device__ __forceinline__ bool slab_iter(SlabRegs<C>& S, const SlabArgs& a, const SlabUnit& u,
                                          int& p, int pend, const FoldCoef<T>& f, T ar31,
                                          uint64_t seed) {
  if (p >= pend) return false;
#pragma unroll
  for (int j = 0; j < C::NC; ++j) S.R[0][I][j] = S.NX[I][j];
  slab_load<C>(S, u, I, p + C::PF, pend);
  slab_levels<C, T, I>(S, a, u, p, f, ar31, seed);
  ++p;
  return true;
}

template <class C, typename T>
__device__ __forceinline__ void slab_unit(const typename C::V2* __restrict__ s,
                                          typename C::V2* __restrict__ d, const SlabArgs& a,
                                          const SlabFace& F, int unit, const FoldCoef<T>& f,
                                          T ar31, uint64_t seed) {
  using V2 = typename C::V2;
  using AX = typename C::AX;
  constexpr int TL = C::TL, NC = C::NC;
  static_assert(C::PF == 3, "the prefetch queue is indexed by the ring slot");
  const Geom& g = a.g;
  const int lane = threadIdx.x & 63;
  const int tile = unit / F.nchunk, chunk = unit % F.nchunk;
  SlabUnit u;
  u.mc0 = F.m0 + chunk * F.chunk;
  u.mc1 = min(u.mc0 + F.chunk, F.m1);
  if (u.mc0 >= u.mc1) return;
  const int ext[3] = {g.nx, g.ny, g.nz};
  const int64_t org[3] = {g.ox, g.oy, g.oz};
  const int64_t Lg[3] = {g.Lx, g.Ly, g.Lz};
  const int64_t str[3] = {1, g.px, (int64_t)g.px * g.py};
  // this lane's A coordinate; the tile owns outputs [o, o + astep) (within lanes [TL, 64-TL))
  const int A0 = F.abase + tile * F.astep;
  const int ca = A0 + lane;
  const int o = F.a0 + tile * F.astep;
  const bool store = ca >= o && ca < o + F.astep && ca < F.a1;
  u.qr = lane & 3;
  u.qm1 = (lane & 1) ? 0xFFFFFFFFu : 0u;
  u.qm2 = (lane & 2) ? 0xFFFFFFFFu : 0u;
  const int cac = clampi(ca, -g.H, ext[AX::A] + g.H - 1);  // loads stay inside the allocation
  const int nb = F.n0 - TL;  // N coordinate of level-0 cell 0
  u.pstart = u.mc0 - TL;
  // descriptors based at (A = -H, N = nb, M = pstart); lane / cell / plane offsets in bytes
  int64_t e0;
  {
    int c[3];
    c[AX::A] = -g.H;
    c[AX::N] = nb;
    c[AX::M] = u.pstart;
    e0 = gs::lin(g, c[0], c[1], c[2]);
  }
  const int64_t left = (gs::total_elems(g) - e0) * (int64_t)sizeof(V2);
  const int range = (int)(left < 0x7ffffff0LL ? left : 0x7ffffff0LL);
  u.src = plane_rsrc((const char*)(s + e0), range);
  u.dst = plane_rsrc((const char*)(d + e0), range);
  u.voff = (int)((int64_t)(cac + g.H) * str[AX::A] * (int64_t)sizeof(V2));
  u.svoff = store ? u.voff : (int)0x80000000;
  u.sNb = (int)(str[AX::N] * (int64_t)sizeof(V2));
  u.sMb = (int)(str[AX::M] * (int64_t)sizeof(V2));
  u.gA = org[AX::A] + ca;
  u.gN0 = org[AX::N] + nb;
  u.gM0 = org[AX::M];
  // whether any cell this unit computes lies outside the global domain (non-periodic)
  u.edge = !C::PER && (org[AX::A] + A0 < 0 || org[AX::A] + A0 + 64 > Lg[AX::A] ||
                       u.gN0 < 0 || u.gN0 + NC > Lg[AX::N] ||
                       u.gM0 + u.mc0 - TL < 0 || u.gM0 + u.mc1 + TL > Lg[AX::M]);
  u.aout = u.edge && (u.gA < 0 || u.gA >= Lg[AX::A]);
  SlabRegs<C> S;
  if constexpr (C::NOISE && C::Q32) {
#pragma unroll
    for (int r = 3; r < 10; ++r) {
      const uint32_t k0 = (uint32_t)seed + (uint32_t)r * kPhW0;
      const uint32_t k1 = (uint32_t)(seed >> 32) + (uint32_t)r * kPhW1;
      asm volatile("v_mov_b32 %0, %1" : "=v"(S.kv[2 * (r - 3)]) : "s"(k0));
      asm volatile("v_mov_b32 %0, %1" : "=v"(S.kv[2 * (r - 3) + 1]) : "s"(k1));
    }
  }
  int p = u.pstart;
  const int pend = u.mc1 + TL;
#pragma unroll
  for (int k = 0; k < C::PF; ++k) slab_load<C>(S, u, k, p + k, pend);
  while (slab_iter<C, T, 0>(S, a, u, p, pend, f, ar31, seed) &&
         slab_iter<C, T, 1>(S, a, u, p, pend, f, ar31, seed) &&
         slab_iter<C, T, 2>(S, a, u, p, pend, f, ar31, seed)) {
  }
}

// OM: the face orientations compiled in (bit o: orientation o).  A unit's registers are those of
// the heaviest orientation in the kernel, so a launch without z faces (the x / y slabs next to
// z slabs computed by k_fused, backend shell variant 1) uses the x / y-only instantiation.
template <typename T, int TL, bool PER, bool NOISE, bool Q32, int OM = 7>
__global__ __launch_bounds__(256) void k_slab(const typename PairT<T>::type* __restrict__ s,
                                              typename PairT<T>::type* __restrict__ d,
                                              SlabArgs a, FoldCoef<T> f, uint64_t seed) {
  const int w = (int)(blockIdx.x * 4 + (threadIdx.x >> 6));
  const int unit = __builtin_amdgcn_readfirstlane(w);
  if (unit >= a.nunits) return;  // whole wave (no barriers in this kernel)
  int fi = 0;
  while (fi + 1 < a.nface && unit >= a.f[fi + 1].u0) ++fi;
  const SlabFace& F = a.f[fi];
  const T ar31 = f.ar * (T)4.656612873077392578125e-10;  // exact: power-of-two scaling
  if constexpr ((OM & 1) != 0)
    if (F.orient == 0) slab_unit<SCfg<T, TL, PER, NOISE, Q32, 0>, T>(s, d, a, F, unit - F.u0, f, ar31, seed);
  if constexpr ((OM & 2) != 0)
    if (F.orient == 1) slab_unit<SCfg<T, TL, PER, NOISE, Q32, 1>, T>(s, d, a, F, unit - F.u0, f, ar31, seed);
  if constexpr ((OM & 4) != 0)
    if (F.orient == 2) slab_unit<SCfg<T, TL, PER, NOISE, Q32, 2>, T>(s, d, a, F, unit - F.u0, f, ar31, seed);
}

// Host side: the face slabs of one overlapped pass.  faces[i] = {orient, side (-1 / +1)};
// a face's outputs: the k cells next to it along N, the given ranges along A and M.
struct SlabSpec {
  int orient, n0, a0, a1, m0, m1;
};

template <typename T, int TL, bool PER, bool NZ, bool Q32, int OM = 7>
void launch_slab_kernel(const void* s, void* d, const SlabArgs& a, const gs::Params& p,
                        hipStream_t st) {
  using V2 = typename PairT<T>::type;
  k_slab<T, TL, PER, NZ, Q32, OM><<<(unsigned)((a.nunits + 3) / 4), 256, 0, st>>>(
      (const V2*)s, (V2*)d, a, make_fold<T>(p), p.seed);
}

// resident 4-wave workgroups per CU of one k_slab instantiation (its register footprint:
// fp32 T=3 ~210 VGPRs, two waves per SIMD; fp64 T=3 one)
template <typename T, int TL, bool PER, bool NZ, bool Q32, int OM = 7>
int slab_occupancy() {
  static int occ = -1;
  if (occ < 0) {
    int o = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, k_slab<T, TL, PER, NZ, Q32, OM>, 256, 0) !=
            hipSuccess || o < 1)
      o = 1;
    occ = o;
  }
  return occ;
}

template <typename T, int TL>
void launch_slabs_tl(const void* s, void* d, const Geom& g, const gs::Params& p, int64_t t,
                     const SlabSpec* spec, int nspec, int cus, hipStream_t st) {
  SlabArgs a{};
  a.g = g;
  a.t = t;
  const bool per = g.periodic != 0, nz = p.noise != 0.0, q32 = philox_q32(g);
  // the production combination without z faces: the x / y-only kernel (fewer registers)
  bool zf = false;
  for (int i = 0; i < nspec; ++i) zf = zf || spec[i].orient == 2;
  const bool xy = !per && nz && q32 && !zf;
  const int occ = xy ? slab_occupancy<T, TL, false, true, true, 3>()
                : !nz ? (per ? slab_occupancy<T, TL, true, false, true>()
                             : slab_occupancy<T, TL, false, false, true>())
                : q32 ? (per ? slab_occupancy<T, TL, true, true, true>()
                             : slab_occupancy<T, TL, false, true, true>())
                      : (per ? slab_occupancy<T, TL, true, true, false>()
                             : slab_occupancy<T, TL, false, true, false>());
  const int64_t slots = (int64_t)occ * 4 * cus;  // resident waves
  // March chunk c.  A wave's work is W(c) = sum_L (c + 2 (TL - L)) (3 TL - 2 L) cell updates
  // (its outputs' cone: the fill costs 2 (TL - L) extra planes per level); waves are VALU-bound,
  // so co-resident waves share their SIMD: the time is ~ ceil(waves / SIMDs) x W(c).  Short
  // chunks drown in fill work, long ones leave SIMDs idle (one-sided 256^3, T=3: c = 4).
  (void)slots;
  const int64_t simds = 4LL * cus;
  int chunk = 1;
  int64_t best = INT64_MAX;
  for (int c = 1; c <= 64; ++c) {
    int64_t waves = 0;
    for (int i = 0; i < nspec; ++i) {
      const int m = spec[i].m1 - spec[i].m0, an = spec[i].a1 - spec[i].a0;
      if (m <= 0 || an <= 0) continue;
      const int astep = spec[i].orient == 0 ? 52 : 64 - 2 * TL;
      waves += (int64_t)((an + astep - 1) / astep) * ((m + c - 1) / c);
    }
    int64_t w = 0;
    for (int L = 1; L <= TL; ++L) w += (int64_t)(c + 2 * (TL - L)) * (3 * TL - 2 * L);
    const int64_t cost = ((waves + simds - 1) / simds) * w;
    if (cost < best) { best = cost; chunk = c; }
  }
  int u0 = 0;
  for (int i = 0; i < nspec; ++i) {
    const int m = spec[i].m1 - spec[i].m0, an = spec[i].a1 - spec[i].a0;
    if (m <= 0 || an <= 0) continue;
    SlabFace& F = a.f[a.nface++];
    F.orient = spec[i].orient;
    F.n0 = spec[i].n0;
    F.a0 = spec[i].a0; F.a1 = spec[i].a1;
    F.m0 = spec[i].m0; F.m1 = spec[i].m1;
    if (F.orient == 0) {
      // lanes along y: tiles start on a global y-quad (the noise draw shares one block per
      // quad across lanes) and step by 52, so the owned outputs stay in lanes [TL, 64 - TL)
      F.abase = (F.a0 - TL) - mod4(g.oy + F.a0 - TL);
      F.astep = 52;
    } else {
      F.abase = F.a0 - TL;
      F.astep = 64 - 2 * TL;
    }
    F.ntile = (an + F.astep - 1) / F.astep;
    F.chunk = chunk;
    F.nchunk = (m + chunk - 1) / chunk;
    F.u0 = u0;
    u0 += F.ntile * F.nchunk;
  }
  a.nunits = u0;
  if (u0 == 0) return;
  if (xy) {
    launch_slab_kernel<T, TL, false, true, true, 3>(s, d, a, p, st);
  } else if (!nz) {
    if (per) launch_slab_kernel<T, TL, true, false, true>(s, d, a, p, st);
    else launch_slab_kernel<T, TL, false, false, true>(s, d, a, p, st);
  } else if (q32) {
    if (per) launch_slab_kernel<T, TL, true, true, true>(s, d, a, p, st);
    else launch_slab_kernel<T, TL, false, true, true>(s, d, a, p, st);
  } else {
    if (per) launch_slab_kernel<T, TL, true, true, false>(s, d, a, p, st);
    else launch_slab_kernel<T, TL, false, true, false>(s, d, a, p, st);
  }
}

// The shell of an overlapped n-step pass over src -> dst: for every face whose bit is set in
// `sides` (bit0 -x, bit1 +x, bit2 -y, bit3 +y, bit4 -z, bit5 +z), the n cells next to it.
// Ownership (no cell twice): z slabs take whole planes; x slabs take every y over the planes
// between the z slabs; y slabs the x range between the x slabs.
template <typename T>
bool launch_shell(const void* s, void* d, const Geom& g, const gs::Params& p, int n, int64_t t,
                  int sides, int cus, hipStream_t st) {
  if (n < 2 || n > 3 || g.H < n) return false;
  const int nx = g.nx, ny = g.ny, nz = g.nz;
  if (nx < 2 * n || ny < 2 * n || nz < 2 * n) return false;
  const int z0 = (sides & 16) ? n : 0, z1 = (sides & 32) ? nz - n : nz;
  const int x0 = (sides & 1) ? n : 0, x1 = (sides & 2) ? nx - n : nx;
  SlabSpec sp[6];
  int k = 0;
  // z faces: A = x (all), M = y (all), N = z
  if (sides & 16) sp[k++] = SlabSpec{2, 0, 0, nx, 0, ny};
  if (sides & 32) sp[k++] = SlabSpec{2, nz - n, 0, nx, 0, ny};
  // x faces: A = y (all), M = z between the z slabs
  if (sides & 1) sp[k++] = SlabSpec{0, 0, 0, ny, z0, z1};
  if (sides & 2) sp[k++] = SlabSpec{0, nx - n, 0, ny, z0, z1};
  // y faces: A = x between the x slabs, M = z between the z slabs
  if (sides & 4) sp[k++] = SlabSpec{1, 0, x0, x1, z0, z1};
  if (sides & 8) sp[k++] = SlabSpec{1, ny - n, x0, x1, z0, z1};
  if (!k) return true;
  if (n == 2) launch_slabs_tl<T, 2>(s, d, g, p, t, sp, k, cus, st);
  else launch_slabs_tl<T, 3>(s, d, g, p, t, sp, k, cus, st);
  return true;
}
