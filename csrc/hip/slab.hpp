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
  int32_t ntile, nchunk;    // lane tiles (64 - 2k outputs each) x march chunks
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
  static constexpr bool PER = PER_, NOISE = NOISE_, Q32 = Q32_;
  using AX = SlabAxes<OR_>;
};

// per-unit constants
struct SlabUnit {
  int64_t base;          // element index of (A = lane, N = first level-0 cell, M = 0)
  int64_t sN, sM;        // element strides along N and M
  int64_t gA, gN0, gM0;  // global coordinate of this lane, of level-0 cell 0, of M = 0
  int mc0, mc1;          // output planes along M
  bool edge, aout, store;
};

template <class C, typename T>
__device__ __forceinline__ uint32_t slab_word(const SlabUnit& u, const Geom& g, int j, int64_t gM,
                                              int64_t step, uint64_t seed, gs::U4& blk,
                                              bool refresh) {
  using AX = typename C::AX;
  int64_t gc[3];
  gc[AX::A] = u.gA;
  gc[AX::N] = u.gN0 + j;
  gc[AX::M] = gM;
  const int64_t gx = gwrap_t<C::PER>(gc[0], g.Lx), gy = gwrap_t<C::PER>(gc[1], g.Ly),
                gz = gwrap_t<C::PER>(gc[2], g.Lz);
  if (refresh) {
    if constexpr (C::Q32) {
      const uint32_t Ly4 = (uint32_t)((g.Ly + 3) >> 2);
      blk = philox_dev<true>((uint32_t)gx + (uint32_t)g.Lx * ((uint32_t)(gy >> 2) +
                                                               Ly4 * (uint32_t)gz),
                             0u, (uint64_t)step, seed);
    } else {
      blk = gs::noise_block(gx, gy >> 2, gz, g.Lx, g.Ly, (uint64_t)step, seed);
    }
  }
  const int wi = (int)(gy & 3);
  return wi == 0 ? blk.x : (wi == 1 ? blk.y : (wi == 2 ? blk.z : blk.w));
}

// Level L (1..TL) of plane q from level L-1's ring slots IM (plane q-1), IC (q), IP (q+1).
// R[L][slot][j]: level L, cells j in [L, NC - L) (the unused entries are never touched, so
// they take no registers).  Level TL is stored.
template <class C, typename T, int L, int IM, int IC, int IP>
__device__ __forceinline__ void slab_level(typename C::V2 (&R)[C::TL][3][C::NC],
                                           typename C::V2* __restrict__ d, const SlabArgs& a,
                                           const SlabUnit& u, int q, const FoldCoef<T>& f,
                                           T ar31, uint64_t seed) {
  using V2 = typename C::V2;
  using AX = typename C::AX;
  constexpr int TL = C::TL, NC = C::NC, OR = C::OR;
  const Geom& g = a.g;
  const int64_t gM = u.gM0 + q;
  const int64_t Lg[3] = {g.Lx, g.Ly, g.Lz};
  const bool mout = u.edge && (gM < 0 || gM >= Lg[AX::M]);
  const T bu = (T)gs::bc_u(a.t + L);
  const int64_t step = a.t + (L - 1);
  gs::U4 blk{0, 0, 0, 0};
#pragma unroll
  for (int j = L; j < NC - L; ++j) {
    const V2 c = R[L - 1][IC][j];
    const V2 nm = R[L - 1][IC][j - 1], np = R[L - 1][IC][j + 1];  // N neighbours
    const V2 mm = R[L - 1][IM][j], mp = R[L - 1][IP][j];          // M neighbours
    const V2 lm = V2{lane_from_left(c.x), lane_from_left(c.y)};    // A neighbours
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
    if constexpr (C::NOISE) {
      // orientation 1 runs y along N: the cells of one y-quad share a Philox block (the
      // refresh test is wave-uniform); elsewhere each cell draws its own block
      bool refresh = true;
      if constexpr (OR == 1) {
        const int64_t gy = gwrap_t<C::PER>(u.gN0 + j, g.Ly);
        refresh = j == L || (gy & 3) == 0;
      }
      const uint32_t w = slab_word<C, T>(u, g, j, gM, step, seed, blk, refresh);
      P.x = fma(ar31, (T)(int32_t)w, P.x);
    }
    if constexpr (L < TL) {
      if (u.edge) {
        const int64_t gN = u.gN0 + j;
        if (u.aout || mout || gN < 0 || gN >= Lg[AX::N]) P = V2{bu, (T)0};
      }
      R[L][IC][j] = P;
    } else {
      // outputs: cells [TL, 2TL) of planes [mc0, mc1), lanes of the tile's output range
      if (j >= TL && j < 2 * TL && q >= u.mc0 && q < u.mc1 && u.store)
        d[u.base + (int64_t)j * u.sN + (int64_t)q * u.sM] = P;
    }
  }
}

// one march iteration p (ring index I = (p - pstart) mod 3): level 0 of plane p from the
// prefetch, the prefetch of plane p + 1, then levels 1..TL bottom-up
template <class C, typename T, int I, int L = 1>
__device__ __forceinline__ void slab_levels(typename C::V2 (&R)[C::TL][3][C::NC],
                                            typename C::V2* __restrict__ d, const SlabArgs& a,
                                            const SlabUnit& u, int p, const FoldCoef<T>& f,
                                            T ar31, uint64_t seed) {
  if constexpr (L <= C::TL) {
    const int q = p - L;
    // level L is needed on planes [mc0 - (TL - L), mc1 + (TL - L)) (the outputs' cone)
    if (q >= u.mc0 - (C::TL - L) && q < u.mc1 + (C::TL - L))
      slab_level<C, T, L, (I - L + 5) % 3, (I - L + 6) % 3, (I - L + 7) % 3>(R, d, a, u, q, f,
                                                                               ar31, seed);
    slab_levels<C, T, I, L + 1>(R, d, a, u, p, f, ar31, seed);
  }
}

template <class C, typename T, int I>
__device__ __forceinline__ bool slab_iter(typename C::V2 (&R)[C::TL][3][C::NC],
                                          typename C::V2 (&NX)[C::NC],
                                          const typename C::V2* __restrict__ s,
                                          typename C::V2* __restrict__ d, const SlabArgs& a,
                                          const SlabUnit& u, int& p, int pend,
                                          const FoldCoef<T>& f, T ar31, uint64_t seed) {
  if (p >= pend) return false;
#pragma unroll
  for (int j = 0; j < C::NC; ++j) R[0][I][j] = NX[j];
  if (p + 1 < pend) {
#pragma unroll
    for (int j = 0; j < C::NC; ++j) NX[j] = s[u.base + (int64_t)j * u.sN + (int64_t)(p + 1) * u.sM];
  }
  slab_levels<C, T, I>(R, d, a, u, p, f, ar31, seed);
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
  // this lane's A coordinate; outputs: lanes [TL, 64 - TL) of the tile, clipped to [a0, a1)
  const int A0 = F.a0 - TL + tile * (64 - 2 * TL);
  const int ca = A0 + lane;
  u.store = lane >= TL && lane < 64 - TL && ca >= F.a0 && ca < F.a1;
  const int cac = clampi(ca, -g.H, ext[AX::A] + g.H - 1);  // loads stay inside the allocation
  const int nb = F.n0 - TL;  // N coordinate of level-0 cell 0
  {
    int c[3];
    c[AX::A] = cac;
    c[AX::N] = nb;
    c[AX::M] = 0;
    u.base = gs::lin(g, c[0], c[1], c[2]);
  }
  u.sN = str[AX::N];
  u.sM = str[AX::M];
  u.gA = org[AX::A] + ca;
  u.gN0 = org[AX::N] + nb;
  u.gM0 = org[AX::M];
  // whether any cell this unit computes lies outside the global domain (non-periodic)
  u.edge = !C::PER && (org[AX::A] + A0 < 0 || org[AX::A] + A0 + 64 > Lg[AX::A] ||
                       u.gN0 < 0 || u.gN0 + NC > Lg[AX::N] ||
                       u.gM0 + u.mc0 - TL < 0 || u.gM0 + u.mc1 + TL > Lg[AX::M]);
  u.aout = u.edge && (u.gA < 0 || u.gA >= Lg[AX::A]);
  // a wave-uniform copy of the noise coefficient in a VGPR (as k_fused)
  V2 R[TL][3][NC];
  V2 NX[NC];
  int p = u.mc0 - TL;
  const int pend = u.mc1 + TL;
#pragma unroll
  for (int j = 0; j < NC; ++j) NX[j] = s[u.base + (int64_t)j * u.sN + (int64_t)p * u.sM];
  while (slab_iter<C, T, 0>(R, NX, s, d, a, u, p, pend, f, ar31, seed) &&
         slab_iter<C, T, 1>(R, NX, s, d, a, u, p, pend, f, ar31, seed) &&
         slab_iter<C, T, 2>(R, NX, s, d, a, u, p, pend, f, ar31, seed)) {
  }
}

template <typename T, int TL, bool PER, bool NOISE, bool Q32>
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
  switch (F.orient) {
    case 0: slab_unit<SCfg<T, TL, PER, NOISE, Q32, 0>, T>(s, d, a, F, unit - F.u0, f, ar31, seed); break;
    case 1: slab_unit<SCfg<T, TL, PER, NOISE, Q32, 1>, T>(s, d, a, F, unit - F.u0, f, ar31, seed); break;
    default: slab_unit<SCfg<T, TL, PER, NOISE, Q32, 2>, T>(s, d, a, F, unit - F.u0, f, ar31, seed); break;
  }
}

// Host side: the face slabs of one overlapped pass.  faces[i] = {orient, side (-1 / +1)};
// a face's outputs: the k cells next to it along N, the given ranges along A and M.
struct SlabSpec {
  int orient, n0, a0, a1, m0, m1;
};

template <typename T, int TL, bool PER, bool NZ, bool Q32>
void launch_slab_kernel(const void* s, void* d, const SlabArgs& a, const gs::Params& p,
                        hipStream_t st) {
  using V2 = typename PairT<T>::type;
  k_slab<T, TL, PER, NZ, Q32><<<(unsigned)((a.nunits + 3) / 4), 256, 0, st>>>(
      (const V2*)s, (V2*)d, a, make_fold<T>(p), p.seed);
}

// resident 4-wave workgroups per CU of one k_slab instantiation (its register footprint:
// fp32 T=3 ~210 VGPRs, two waves per SIMD; fp64 T=3 one)
template <typename T, int TL, bool PER, bool NZ, bool Q32>
int slab_occupancy() {
  static int occ = -1;
  if (occ < 0) {
    int o = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, k_slab<T, TL, PER, NZ, Q32>, 256, 0) !=
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
  const int occ = !nz ? (per ? slab_occupancy<T, TL, true, false, true>()
                             : slab_occupancy<T, TL, false, false, true>())
                : q32 ? (per ? slab_occupancy<T, TL, true, true, true>()
                             : slab_occupancy<T, TL, false, true, true>())
                      : (per ? slab_occupancy<T, TL, true, true, false>()
                             : slab_occupancy<T, TL, false, true, false>());
  const int64_t slots = (int64_t)occ * 4 * cus;  // resident waves
  // march chunk: minimise rounds x (chunk + 2 TL pipeline fill) over the resident wave slots
  int chunk = 1;
  int64_t best = INT64_MAX;
  for (int c = 1; c <= 64; ++c) {
    int64_t waves = 0;
    for (int i = 0; i < nspec; ++i) {
      const int m = spec[i].m1 - spec[i].m0, an = spec[i].a1 - spec[i].a0;
      if (m <= 0 || an <= 0) continue;
      waves += (int64_t)((an + (64 - 2 * TL) - 1) / (64 - 2 * TL)) * ((m + c - 1) / c);
    }
    const int64_t rounds = (waves + slots - 1) / slots;
    const int64_t cost = rounds * (c + 2 * TL);
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
    F.ntile = (an + (64 - 2 * TL) - 1) / (64 - 2 * TL);
    F.chunk = chunk;
    F.nchunk = (m + chunk - 1) / chunk;
    F.u0 = u0;
    u0 += F.ntile * F.nchunk;
  }
  a.nunits = u0;
  if (u0 == 0) return;
  if (!nz) {
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
