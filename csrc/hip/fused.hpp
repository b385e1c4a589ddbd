// SPDX-License-Identifier: MIT
// k_fused: T time levels per HBM pass over the interior (temporal blocking) for gfx950.
// Included inside namespace gsk by kernels.hpp, after stencil.hpp.
//
// The update being computed is the reference's calculate! (Simulation_CPU.jl:92-112), T steps
// per pass: HBM is read once and written once per T steps.
//
// Work unit = one (tile, z-plane) pair; the units are split over a grid of workgroups, each
// walking one or more contiguous z-segments.  Tile = 64 columns (one lane each) x WAVES*ROWS
// rows of level-0 data (ghosts included); it yields (64-2T) x ystep interior outputs.  A segment
// [z0,z1) streams level-0 planes z0-T .. z1+T-1.
//
// Register plan (no rotation copies): level-0 planes live in a ring LD[PF+2] (plane p, p-1 and
// the prefetches); level-l outputs in a ring OUT[l][NS]; per consumer level a running partial
// sum A (xy-neighbours of plane q-1 plus plane q-2).  The loop is unrolled by the ring period
// so every ring index is a compile-time constant.  Memory goes through buffer descriptors of
// one storage plane each, walked by a running 64-bit plane pointer: 32-bit lane offsets, no
// address VGPRs, out-of-range loads return 0 and masked stores use an out-of-range offset.
// Intermediate levels outside the global domain (non-periodic) are reset to the boundary value
// of their time level -- what the single-step path reads from its ghost shell.
//
// Energy per cell update is what limits this kernel on random data (profiles/
// r2_power_probe.txt: the same dispatch runs at the full clock on smooth data and ~20 % slower
// on rough data, with identical cycle counts), so every VALU instruction counts:
//  * fp32 arithmetic on the interleaved (u, v) pairs is packed (v_pk_add/v_pk_mul/v_pk_fma_f32);
//  * the x-neighbour pair sum and the y/z partial sum are two DPP adds, with no hazard wait
//    states (checked on the built code object);
//  * the LDS row exchange wraps around (wave 0 reads the last wave's row: a tile-halo row whose
//    value never reaches an output), so the exchange has no branches or register copies;
//  * waves whose rows are all outside a level's dependency cone skip that level (the row slack
//    of the 4-row noise quads: at T=3 the last wave of a 48-row tile skips levels 2 and 3);
//  * Philox rounds 1-3 keep their wave-uniform words on the SALU when the global counter fits
//    32 bits (Q32: Lx * ceil(Ly/4) * Lz < 2^32, every grid up to L = 2580).
#pragma once

// Gated pass (IPC transport, gate.hpp): ONE k_fused launch per pass that also carries the halo
// exchange.  Every workgroup runs one unit from a host-built table; a start-gated unit (its
// level-0 cone reads ghost cells a neighbour fills) first packs its share of the outgoing
// messages straight into the peers' landing buffers, the last packer signals the peers, then it
// waits for the peers' signals and copies the ghost cells of its own cone out of its landing
// slot before marching.  Ungated units (cone clear of every face with a neighbour) march at once.
using GateUnit = gs::GateUnit;  // a gated pass's unit (gs/gate_plan.h)
struct GateArgs;  // gate.hpp

struct FusedArgs {
  Geom g;
  int32_t ntx, nty;
  int32_t xstep, ystep;
  int32_t ybase;
  int32_t bcfix;
  int64_t units;
  int32_t sched;   // 0: units split evenly; 1: XCD-grouped z-chunks; 2: persistent XCD rounds
  int32_t nchunk;  // sched 1/2: z-chunks per tile
  int32_t ntiles;  // tiles enumerated (ntx * nty)
  // output store mask [mx0, mx1) x [my0, my1) (local x / y; the whole interior by default).
  // The inner part of an overlapped pass clips its outputs to the cells at least T from every
  // x / y face whose halo is in flight: those depend on interior cells only, so the tiles may
  // read ghost cells that are being written meanwhile (the values never reach a stored cell);
  // the k-deep face slabs are computed by k_slab once the halos have landed (slab.hpp).
  int32_t mx0, mx1, my0, my1;
  int32_t grpM;    // sched 1/2: workgroups per XCD group (grid = 8 * grpM)
  int32_t cfg;     // tile/prefetch configuration index (fused_cfg_names)
  int64_t t;
  int32_t reserve;    // workgroup slots to leave free (comm kernels running alongside)
  int32_t q32;        // Philox counter fits 32 bits (host check)
  // output z-runs [zlo[r], zlo[r] + zlen[r]) (zlen[1] may be 0); a tile's units enumerate the
  // planes of run 0 then run 1 (nzv = zlen[0] + zlen[1] units per tile)
  int32_t zlo[2], zlen[2];
  int32_t nzv;
  // the small-grid block kernel may serve this launch (Backend::fused(), and the autotuner's
  // timing of it): its level-0 x ghosts are then the engine's ensure_bc values (block.hpp)
  int32_t allow_block;
  // folded x strip (FCfg::FOLD): tiles [0, ntxf * nty) are the full 64-column tiles; the last
  // strip's narrow tiles (<= 32 - 2T outputs wide) run two per wave as nfold = ceil(nty / 2)
  // units -- lanes 0-31 y-tile 2f, lanes 32-63 y-tile 2f + 1 (idle past the last one)
  int32_t ntxf, nfold;
  // gated pass (sched 3, gate.hpp): the unit table (one unit per workgroup), the transport state,
  // the source buffer as a writable pointer (the in-kernel unpack fills its ghosts), this pass's
  // exchange number and the packer-arrival count its last packer reaches
  const GateUnit* gunits;
  const GateArgs* gate;
  void* field;
  uint64_t gate_n;
  uint32_t gate_cnt;
  int32_t gate_npk;  // packers of this launch (its start-gated units)
  int32_t ngunits;
  int32_t gate_pairs;  // 1: two table entries per workgroup (gs::gate_plan_pairs)
  // carried exchanges (gate.hpp gate_carry): bit 0 -- this pass's exchange was packed by the
  // previous launch's producers (no packing here); bit 1 -- this pass's producers pack the next
  // exchange (gate_n + 1) at their end, whose arrivals reach gate_cnt2
  int32_t gate_pre;
  uint32_t gate_cnt2;
};

template <typename T>
__device__ __forceinline__ void gate_start(const FusedArgs& a, int pk, bool wait, int X0, int xw,
                                        int Y0, int yext, int za, int zb);
template <typename T>
__device__ __forceinline__ void gate_pack(const FusedArgs& a, int pk);
template <typename T, int BATCH>
__device__ __forceinline__ void gate_unpack(const FusedArgs& a, int X0, int xw, int Y0, int yext,
                                         int za, int zb, uint64_t t0);
template <typename T>
__device__ __forceinline__ void gate_carry(const FusedArgs& a, const void* dv, int ox0, int ox1,
                                           int oy0, int oy1, int z0, int z1);

template <typename T> struct PairT;
template <> struct PairT<float> { typedef float type __attribute__((ext_vector_type(2))); };
template <> struct PairT<double> { typedef double type __attribute__((ext_vector_type(2))); };

// Folded update coefficients:
//   u' = au*u + asu*su + ac - dt*uvv + ar*r ;  v' = bv*v + bsv*sv + dt*uvv
// held as (u, v) pairs for the packed fp32 form: P = kd*uvv + kc ; P += ks*s ; P += kc2*c.
template <typename T>
struct FoldCoef {
  using P2 = typename PairT<T>::type;
  P2 kd, kc, ks, kcc;  // (-dt, dt), (ac, 0), (asu, bsv), (au, bv)
  T ar;                // dt * noise
};

template <typename T>
inline FoldCoef<T> make_fold(const gs::Params& p) {
  FoldCoef<T> f;
  f.kd = typename PairT<T>::type{(T)(-p.dt), (T)p.dt};
  f.kc = typename PairT<T>::type{(T)(p.dt * p.F), (T)0};
  f.ks = typename PairT<T>::type{(T)(p.dt * p.Du / 6.0), (T)(p.dt * p.Dv / 6.0)};
  f.kcc = typename PairT<T>::type{(T)(1.0 - p.dt * (p.Du + p.F)),
                                  (T)(1.0 - p.dt * (p.Dv + p.F + p.k))};
  f.ar = (T)(p.dt * p.noise);
  return f;
}

typedef unsigned int gs_u2 __attribute__((ext_vector_type(2)));
typedef unsigned int gs_u4 __attribute__((ext_vector_type(4)));

// Descriptor for one storage plane starting at `base` (bytes `nbytes`; 0 = disabled: every
// access through it is dropped, loads return 0).  Accesses past the plane's end -- tile rows
// beyond the ghost layer -- read 0 instead of the next plane's data: neither ever reaches a
// stored output (an output depends on rows within T <= H of it).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t plane_rsrc(const char* base, int nbytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, nbytes, 0x00020000);
}

__device__ __forceinline__ PairT<float>::type bload(__amdgpu_buffer_rsrc_t r, int voff,
                                                    PairT<float>::type*) {
  const gs_u2 v = __builtin_amdgcn_raw_buffer_load_b64(r, voff, 0, 0);
  return PairT<float>::type{__uint_as_float(v.x), __uint_as_float(v.y)};
}
__device__ __forceinline__ PairT<double>::type bload(__amdgpu_buffer_rsrc_t r, int voff,
                                                     PairT<double>::type*) {
  const gs_u4 v = __builtin_amdgcn_raw_buffer_load_b128(r, voff, 0, 0);
  return PairT<double>::type{__longlong_as_double(((long long)v.y << 32) | v.x),
                             __longlong_as_double(((long long)v.w << 32) | v.z)};
}
// AUX: the store's cache policy (gfx950: 1 sc0, 2 nt, 16 sc1; sc1 = device scope, written
// through the XCD's L2)
template <int AUX = 0>
__device__ __forceinline__ void bstore(__amdgpu_buffer_rsrc_t r, int voff, PairT<float>::type c) {
  gs_u2 v;
  v.x = __float_as_uint(c.x);
  v.y = __float_as_uint(c.y);
  __builtin_amdgcn_raw_buffer_store_b64(v, r, voff, 0, AUX);
}
template <int AUX = 0>
__device__ __forceinline__ void bstore(__amdgpu_buffer_rsrc_t r, int voff, PairT<double>::type c) {
  const unsigned long long a = (unsigned long long)__double_as_longlong(c.x);
  const unsigned long long b = (unsigned long long)__double_as_longlong(c.y);
  gs_u4 v;
  v.x = (unsigned)a; v.y = (unsigned)(a >> 32); v.z = (unsigned)b; v.w = (unsigned)(b >> 32);
  __builtin_amdgcn_raw_buffer_store_b128(v, r, voff, 0, AUX);
}

// a ^ b ^ c in one gfx950 instruction (the compiler does not form v_bitop3 from xor chains)
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t r;
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "s"(c));
  return r;
}

__device__ __forceinline__ uint32_t xor3v(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t r;
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

constexpr uint32_t kPhM0 = 0xD2511F53u, kPhM1 = 0xCD9E8D57u;
constexpr uint32_t kPhW0 = 0x9E3779B9u, kPhW1 = 0xBB67AE85u;

// Device Philox4x32-10 of counter (c0, c1, step_lo, step_hi): gs::noise_block's stream, bit
// for bit.  The key schedule and the step words are rebuilt from opaque copies at every call:
// otherwise the compiler hoists their loop-invariant products out of the plane loop, runs out
// of SGPRs and spills them to VGPR lanes (a v_readlane per use).  Rebuilt, they are a few
// SALU ops.
//   Q32 (c1 = 0): round 1's second product and the round-2 first product see only
//   wave-uniform words, so rounds 1-3 cost 1 + 3 + 4 VALU instead of 4 + 4 + 4.
//   KV: the round keys of rounds 4-10 come from VGPRs (kv, filled once per kernel) instead of
//   being rebuilt on the SALU at every call.
template <bool Q32, bool KV = false>
__device__ __forceinline__ gs::U4 philox_dev(uint32_t c0, uint32_t c1, uint64_t step,
                                             uint64_t seed, const uint32_t* kv = nullptr) {
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
  uint32_t s0 = (uint32_t)step, s1 = (uint32_t)(step >> 32);
  asm volatile("" : "+s"(k0), "+s"(k1), "+s"(s0), "+s"(s1));
  uint32_t c2, c3;
  if constexpr (Q32) {
    // round 1: (c0 lane, 0, s0, s1)
    const uint64_t m0 = (uint64_t)kPhM0 * c0;  // lane
    const uint64_t m1 = (uint64_t)kPhM1 * s0;  // uniform
    const uint32_t u0 = (uint32_t)(m1 >> 32) ^ k0;            // uniform (c1 = 0)
    const uint32_t l2 = (uint32_t)(m0 >> 32) ^ (s1 ^ k1);     // lane
    const uint32_t u1 = (uint32_t)m1;                          // uniform
    const uint32_t l3 = (uint32_t)m0;                          // lane
    k0 += kPhW0; k1 += kPhW1;
    // round 2: (u0, u1, l2, l3)
    const uint64_t n0 = (uint64_t)kPhM0 * u0;  // uniform
    const uint64_t n1 = (uint64_t)kPhM1 * l2;  // lane
    c0 = (uint32_t)(n1 >> 32) ^ (u1 ^ k0);                      // lane
    c2 = l3 ^ ((uint32_t)(n0 >> 32) ^ k1);                      // lane
    c1 = (uint32_t)n1;                                           // lane
    const uint32_t u3 = (uint32_t)n0;                            // uniform
    k0 += kPhW0; k1 += kPhW1;
    // round 3: (c0, c1, c2 lane; u3 uniform)
    const uint64_t p0 = (uint64_t)kPhM0 * c0;
    const uint64_t p1 = (uint64_t)kPhM1 * c2;
    c0 = xor3((uint32_t)(p1 >> 32), c1, k0);
    c2 = (uint32_t)(p0 >> 32) ^ (u3 ^ k1);
    c1 = (uint32_t)p1;
    c3 = (uint32_t)p0;
    k0 += kPhW0; k1 += kPhW1;
  } else {
    c2 = s0;
    c3 = s1;
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      gs::philox_round(c0, c1, c2, c3, k0, k1);
      k0 += kPhW0;
      k1 += kPhW1;
    }
  }
#pragma unroll
  for (int r = 3; r < 10; ++r) {
    const uint64_t m0 = (uint64_t)kPhM0 * c0;
    const uint64_t m1 = (uint64_t)kPhM1 * c2;
    uint32_t n0, n2;
    if constexpr (KV) {
      n0 = xor3v((uint32_t)(m1 >> 32), c1, kv[2 * (r - 3)]);
      n2 = xor3v((uint32_t)(m0 >> 32), c3, kv[2 * (r - 3) + 1]);
    } else {
      n0 = xor3((uint32_t)(m1 >> 32), c1, k0);
      n2 = xor3((uint32_t)(m0 >> 32), c3, k1);
      k0 += kPhW0;
      k1 += kPhW1;
    }
    c0 = n0; c1 = (uint32_t)m1; c2 = n2; c3 = (uint32_t)m0;
  }
  return gs::U4{c0, c1, c2, c3};
}

// The step-uniform part of philox_dev<true>(c0, 0, step, seed): the words of rounds 1-3 that do
// not depend on the lane's counter word c0.
struct PhiloxU {
  uint32_t x1, x2, x3, k3, x4;
};

__device__ __forceinline__ PhiloxU philox_uniform(uint64_t step, uint64_t seed) {
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
  const uint32_t s0 = (uint32_t)step, s1 = (uint32_t)(step >> 32);
  PhiloxU u;
  const uint64_t m1 = (uint64_t)kPhM1 * s0;          // round 1 (counter word 1 = 0)
  const uint32_t u0 = (uint32_t)(m1 >> 32) ^ k0;
  const uint32_t u1 = (uint32_t)m1;
  u.x1 = s1 ^ k1;
  k0 += kPhW0; k1 += kPhW1;
  const uint64_t n0 = (uint64_t)kPhM0 * u0;          // round 2
  u.x2 = u1 ^ k0;
  u.x3 = (uint32_t)(n0 >> 32) ^ k1;
  k0 += kPhW0; k1 += kPhW1;
  u.k3 = k0;                                         // round 3
  u.x4 = (uint32_t)n0 ^ k1;
  return u;
}

// philox_dev<true, true>(c0, 0, step, seed, kv), given philox_uniform(step, seed)
__device__ __forceinline__ gs::U4 philox_lane(uint32_t c0, const PhiloxU& u, const uint32_t* kv) {
  const uint64_t m0 = (uint64_t)kPhM0 * c0;          // round 1
  const uint32_t l2 = (uint32_t)(m0 >> 32) ^ u.x1;
  const uint32_t l3 = (uint32_t)m0;
  const uint64_t n1 = (uint64_t)kPhM1 * l2;          // round 2
  uint32_t a0 = (uint32_t)(n1 >> 32) ^ u.x2;
  uint32_t a2 = l3 ^ u.x3;
  uint32_t a1 = (uint32_t)n1;
  const uint64_t p0 = (uint64_t)kPhM0 * a0;          // round 3
  const uint64_t p1 = (uint64_t)kPhM1 * a2;
  a0 = xor3((uint32_t)(p1 >> 32), a1, u.k3);
  a2 = (uint32_t)(p0 >> 32) ^ u.x4;
  a1 = (uint32_t)p1;
  uint32_t a3 = (uint32_t)p0;
#pragma unroll
  for (int r = 3; r < 10; ++r) {                     // rounds 4-10: round keys in VGPRs
    const uint64_t m = (uint64_t)kPhM0 * a0;
    const uint64_t n = (uint64_t)kPhM1 * a2;
    const uint32_t b0 = xor3v((uint32_t)(n >> 32), a1, kv[2 * (r - 3)]);
    const uint32_t b2 = xor3v((uint32_t)(m >> 32), a3, kv[2 * (r - 3) + 1]);
    a0 = b0; a1 = (uint32_t)n; a2 = b2; a3 = (uint32_t)m;
  }
  return gs::U4{a0, a1, a2, a3};
}

// philox_lane with the step-uniform words held in VGPRs (u: x1, x2, x3, k3, x4), for kernels
// that keep them live across the whole kernel (the SGPR budget has no room for them there)
__device__ __forceinline__ gs::U4 philox_lane_v(uint32_t c0, const uint32_t* u, const uint32_t* kv) {
  const uint64_t m0 = (uint64_t)kPhM0 * c0;          // round 1
  const uint32_t l2 = (uint32_t)(m0 >> 32) ^ u[0];
  const uint32_t l3 = (uint32_t)m0;
  const uint64_t n1 = (uint64_t)kPhM1 * l2;          // round 2
  uint32_t a0 = (uint32_t)(n1 >> 32) ^ u[1];
  uint32_t a2 = l3 ^ u[2];
  uint32_t a1 = (uint32_t)n1;
  const uint64_t p0 = (uint64_t)kPhM0 * a0;          // round 3
  const uint64_t p1 = (uint64_t)kPhM1 * a2;
  a0 = xor3v((uint32_t)(p1 >> 32), a1, u[3]);
  a2 = (uint32_t)(p0 >> 32) ^ u[4];
  a1 = (uint32_t)p1;
  uint32_t a3 = (uint32_t)p0;
#pragma unroll
  for (int r = 3; r < 10; ++r) {
    const uint64_t m = (uint64_t)kPhM0 * a0;
    const uint64_t n = (uint64_t)kPhM1 * a2;
    const uint32_t b0 = xor3v((uint32_t)(n >> 32), a1, kv[2 * (r - 3)]);
    const uint32_t b2 = xor3v((uint32_t)(m >> 32), a3, kv[2 * (r - 3) + 1]);
    a0 = b0; a1 = (uint32_t)n; a2 = b2; a3 = (uint32_t)m;
  }
  return gs::U4{a0, a1, a2, a3};
}

// Compile-time configuration of one fused-kernel instantiation.
//   ROWS x WAVES : rows per wave x waves per workgroup (tile height = ROWS*WAVES)
//   PF           : level-0 prefetch distance in planes (register ring of PF+2 planes)
//   SKEW         : level l consumes level l-1's output of the previous iteration, so all
//                  levels share ONE workgroup barrier per plane
//   Q32          : the Philox counter fits 32 bits (rounds 1-3 partly on the SALU)
//   ABL          : ablations for timing experiments, GS_ABLATION builds only (results are
//                  WRONG by design): bit0 no workgroup barriers, bit1 every level-0 load reads
//                  plane 0 (L2-resident); bit2 (exact) Philox round keys 4-10 in VGPRs; bit3
//                  (exact) the x-neighbour sums' leading s_nop restored; bit4 (exact) the
//                  pipeline fill computes every level (no FILL skip); bit5 (exact) Philox only
//                  on lanes inside the x cone; bit6 (exact) Philox keys rebuilt on the SALU
//                  (KV off); bit7 / bit8 (exact) step-uniform Philox words in VGPRs forced
//                  on / off (PU); bit9 (exact) Philox blocks drawn before the barrier; bits 11 /
//                  12 (exact) nt / sc1 output stores
constexpr int gs_gcd(int a, int b) { return b == 0 ? a : gs_gcd(b, a % b); }
constexpr int gs_lcm(int a, int b) { return a / gs_gcd(a, b) * b; }

template <typename T_, int TL_, int ROWS_, int WAVES_, int PF_, bool PERIODIC_, bool NOISE_,
          bool SKEW_ = false, bool Q32_ = true, int ABL_ = 0, bool FOLD_ = false, int OPT_ = 0>
struct FCfg {
  using T = T_;
  using V2 = typename PairT<T>::type;
  static constexpr int TL = TL_, ROWS = ROWS_, WAVES = WAVES_, PF = PF_;
  static constexpr bool PERIODIC = PERIODIC_, NOISE = NOISE_, SKEW = SKEW_, Q32 = Q32_;
  static constexpr int ABL = ABL_;
  // the last x strip folded into half-wave tiles (FusedArgs::ntxf ..): non-periodic, 32-bit
  // noise counter (its lane part absorbs the upper half's y offset)
  static constexpr bool FOLD = FOLD_;
  // fp64 x-neighbour pair sums through LDS instead of DPP: the DP ALU has no wave-shift DPP (only
  // row_newbcast), so a lane shift of a double is two 32-bit v_mov_b32_dpp -- eight VALU per
  // cell-level for the (u, v) pair's two neighbours.  With LX each wave stores its rows once per
  // level (ds_write_b128) and reads both neighbours back (2 x ds_read_b128): LDS instructions
  // instead of VALU, latency hidden by the plane pipeline (the sums feed the next plane's partial
  // sum).  Same association, (left + right) + s, and the padding lanes read 0 like bound_ctrl:
  // bit-identical.  Candidate "<shape>x" of the fp64 autotuner.
  static constexpr bool LX = (OPT_ & 1) != 0;
  static_assert(!LX || sizeof(T_) == 8, "LDS x-sums are for fp64 (fp32 fuses the DPP into the add)");
  // Neighbour-only synchronisation of the skewed pipeline's LDS row exchange (OPT bit 1) instead
  // of one workgroup barrier per plane: a wave reads only its up / down partner's rows, so after
  // publishing its own rows it bumps its LDS sequence word and waits until both partners' words
  // reach the same iteration.  The waves of a workgroup drift by up to an iteration per
  // neighbour instead of meeting at one s_barrier (whose wait lines up every wave's stalls).
  // RAW: a partner's rows of iteration i are written before its word reaches i (one wave's LDS
  // instructions execute in order); WAR: slot i % 2 is rewritten at i + 2, after the partner has
  // published i + 1, i.e. finished its reads of i.  The wrap-around partners (wave 0's up, the
  // last wave's down) exchange tile-halo rows that never reach an output, so they are not waited
  // for.  Bit-identical.
  static constexpr bool NSYNC = (OPT_ & 2) != 0;
  static_assert(!NSYNC || SKEW_, "neighbour sync replaces the skewed pipeline's single barrier");
  // LDS-resident level-0 ring (OPT bit 2): the level-0 planes stream into an LDS ring of PF + 2
  // planes by gfx950 LDS-DMA (buffer_load_dwordx4 ... lds, 16 B per lane: one wave instruction
  // = two 64-pair tile rows), issued PF planes ahead right after the plane's barrier, and the
  // level-0 update reads its rows, y-neighbours and centre plane back with ds_read_b64.  No
  // VGPR ring (the register-ring design holds (PF + 2) x ROWS pairs per lane), no level-0 row
  // exchange, and the prefetch depth costs LDS instead of registers -- what makes T = 4 fit
  // the 12-wave workgroup's 168-VGPR budget.  Bit-identical to the register ring.
  static constexpr bool LR = (OPT_ & 4) != 0;
  static_assert(!LR || (SKEW_ && ROWS_ == 4 && !NSYNC && !LX && (sizeof(T_) == 4 || !FOLD_)),
                "the LDS ring is built for the skewed 4-row pipeline (fp64: unfolded tiles)");
  // fp64 LDS ring (LRC): the centre plane comes from registers -- the previous iteration's
  // level-0 rows, which are exactly the next iteration's centre -- so the ring holds only the
  // current plane and the prefetch (PF + 1 slots of 16-B pairs: a 4x8 tile's ring + two levels'
  // row exchange then fit the 160 KiB, 64 + 64 KiB at PF = 1).  fp32 reads the centre back from
  // the ring instead (PF + 2 slots; its registers are the tighter budget).
  static constexpr bool LRC = LR && sizeof(T_) == 8;
  // DMA pieces per wave and plane (16 B per lane, 1 KiB per wave instruction): fp32 two rows per
  // piece, fp64 one
  static constexpr int ND = LR ? ROWS_ * 64 * (int)sizeof(typename PairT<T_>::type) / 1024 : 0;
  static_assert(!FOLD_ || (Q32_ && !PERIODIC_ && ROWS_ == 4),
                "folded strips need Q32, a non-periodic grid and 4-row waves");
  static constexpr int R = LRC ? PF + 1 : PF + 2;     // level-0 ring slots (VGPRs or LDS)
  static constexpr int XL = LR ? (TL > 1 ? TL - 1 : 1) : TL;  // levels with an xch row exchange
  // the row-exchange slot of consumer level l (LR: level 0 reads the LDS ring instead)
  static constexpr int xi(int l) { return LR ? l - 1 : l; }
  // level-l output ring / xch buffers: 2 slots.  Skewed: level l+1 reads level l's outputs of
  // the two previous iterations (input and centre), and the levels run top-down within an
  // iteration, so level l overwrites its p-2 output only after level l+1 has consumed it.
  static constexpr int NS = 2;
  static constexpr int PERIOD = gs_lcm(R, NS);
  static constexpr int NO = TL > 1 ? TL - 1 : 1;
  static constexpr int RT = ROWS * WAVES;                 // tile rows
  // waves per SIMD the register budget must allow (__launch_bounds__' second argument is
  // waves per EU on gfx9): fp32 4-row tiles of 8 or 16 waves need 4 (<= 128 VGPRs: two
  // 8-wave workgroups or one 16-wave workgroup per CU); 12- and 6-wave tiles fill 3 (one or
  // two workgroups per CU, <= 168 VGPRs); the 8-row and fp64 tiles keep the compiler's choice
  //   fp64 4-row tiles of 6 or 8 waves run one workgroup per CU at any count <= 256 (2)
  static constexpr int WPEU =
      (sizeof(T) == 4 && ROWS == 4) ? ((WAVES == 8 || WAVES == 16) ? 4 : 3)
      : (sizeof(T) == 8 && ROWS == 4 && (WAVES == 6 || WAVES == 8)) ? 2 : 1;
  // Philox round keys 4-10 in VGPRs (filled once per kernel) instead of rebuilt on the SALU at
  // every draw, where the register budget has room for the 14 keys: fp32 shapes of <= 168 VGPRs
  // (the 128-VGPR shapes would spill, the fp64 ones are near 256).  L=512 T=3, random init, the
  // driver's window: 4x12:2s 689k -> 719k, 4x12:1s 695-698k -> 703-705k MLUPS (profiles/
  // r4_fused_ab.txt).  ABL bit 6 turns it off (A/B), bit 2 forces it on.
  // (fp64: the LDS-ring shapes, whose freed ring registers pay for the keys and the step words;
  // the register-ring fp64 tiles sit at ~247 VGPRs)
  static constexpr bool KV =
      (ABL_ & 4) != 0 || ((sizeof(T) == 4 ? WPEU == 3 : LRC) && (ABL_ & 64) == 0);
  // The step-uniform Philox words of rounds 1-3 (philox_uniform) computed once per kernel and
  // held in VGPRs, 5 per level, instead of rebuilt on the SALU at every draw (the SALU is
  // shared by the CU's four SIMDs and was the co-bottleneck of the noise path).  Default on the
  // single-prefetch KV shapes (4x12:1s: 161 VGPRs at T=3, inside the 168 budget); the 2-deep
  // prefetch shapes would exceed it.  L=512 T=3 random init: 4x12:1s 726k -> 746k MLUPS
  // (profiles/r4_fused_ab.txt).  ABL bit 7 forces it on, bit 8 turns it off (both exact).
  static constexpr bool PU_ANY =
      NOISE_ && KV && Q32_ && ((ABL_ & 128) != 0 || ((PF_ == 1 || LR) && (ABL_ & 256) == 0));
  // ... and where they live: VGPRs, or (PUL: the LDS-ring shapes at T >= 4, whose OUT / A rings
  // take the registers) an LDS table of 8 words per level, read back per draw by one broadcast
  // ds_read_b128 + ds_read_b32 (every lane the same address: no bank conflict)
  static constexpr bool PUL = PU_ANY && LR && TL_ >= 4;
  static constexpr bool PU = PU_ANY && !PUL;
  // KVL: the round keys too (the folded T >= 4 LDS-ring shape: its per-lane row store offsets
  // leave no room for them), 16 words read back per draw by four broadcast ds_read_b128
  static constexpr bool KVL = false;
  // pipeline-fill level skip (fused_iter FILL periods): its second copy of the unrolled body
  // costs ~16 VGPRs, free only where the budget is 168 or 256 (WPEU 3 / 2); with 128 it spills
  // or halves the occupancy (4x8:1s: -10 % at L=512, profiles/r2_fill_skip.txt)
  // (not on the folded T >= 4 LDS-ring shape: the second body copy does not fit its registers)
  static constexpr bool FILLSKIP = (WPEU == 3 || WPEU == 2) && !(ABL_ & 16) && !(LR && FOLD_ && TL_ >= 4);
  // ABL bit 9 (exact): every level's Philox block of the iteration drawn before the workgroup
  // barrier (three independent chains interleaved, overlapping the barrier wait) instead of at
  // the top of each level's branch (4-row tiles, the PU form)
  // (bit 10: only the top level's block, the first computed in the skewed order; bits 9 + 10:
  // the top two levels')
  static constexpr int HOISTN =
      !(PU && ROWS_ == 4) ? 0
      : ((ABL_ & 1536) == 1536) ? (TL_ < 2 ? TL_ : 2)
      : (ABL_ & 512) ? TL_ : (ABL_ & 1024) ? 1 : 0;
  static constexpr bool HOIST = HOISTN > 0;
  // ABL bits 11 / 12 (exact): the output stores non-temporal (nt) / device-scope (sc1, written
  // through L2, so the kernel-end release has no dirty L2 lines to write back)
  static constexpr int STORE_AUX = ((ABL_ & 2048) ? 2 : 0) | ((ABL_ & 4096) ? 16 : 0);
  static constexpr bool hoisted(int l) { return HOISTN > 0 && l >= TL_ - HOISTN; }
  static constexpr int YSTEP = (RT - 2 * TL) & ~3;        // output rows per tile
  // the shapes with a gated-pass entry (k_fused_gated, gate.hpp): the production path's skewed
  // 1-prefetch tiles -- fp32 4x12 (folded or not), fp64 4x8 -- non-periodic, noisy, 32-bit counter
  static constexpr bool GATE_OK = !PERIODIC_ && NOISE_ && Q32_ && ABL_ == 0 && OPT_ == 0 &&
                                  ROWS_ == 4 && SKEW_ && PF_ == 1 &&
                                  ((sizeof(T_) == 4 && WAVES_ == 12) || (sizeof(T_) == 8 && WAVES_ == 8));
  // rows of output level L = l + 1 that some stored output depends on: [l + 1, hi(l)]
  static constexpr int need_hi(int l) { return 2 * TL + YSTEP - 2 - l; }
};

template <class C>
struct FusedState {
  using V2 = typename C::V2;
  typename C::T ar31;  // dt * noise * 2^-31 held in a VGPR (an SGPR copy spills)
  typename C::V2 kc;   // (dt F, 0) held in VGPRs (the first packed FMA's addend)
  uint32_t kv[(C::KV && !C::KVL) ? 14 : 1];  // Philox round keys of rounds 4-10 (C::KV)
  uint32_t pu[C::PU ? 5 * C::TL : 1];  // step-uniform Philox words per level (C::PU)
  V2 LD[C::LR ? 1 : C::R][C::ROWS];  // (FCfg::LR: unused, the ring lives in LDS)
  V2 C0[C::LRC ? C::ROWS : 1];       // FCfg::LRC: the centre plane's rows (last iteration's input)
  V2 OUT[C::NO][C::NS][C::ROWS];
  V2 A[C::TL][C::ROWS];
};

// Per-segment constants (wave-uniform values and the lane's offsets).
struct FusedSeg {
  int p, pend, ldend, z0;
  int lane, wave, wup, wdn;  // LDS exchange partners (wrap around)
  int skip;                  // bit l: this wave's rows are outside level l+1's cone
  int voff, svoff, pitchb;
  int srow0, srow1;
  int soff[4];               // FOLD: per-lane store offset of each row (out of range: masked)
  int srows;                 // FOLD + LR at T >= 4: bit j set = this lane stores row j (offsets
                             // then rebuilt per store: 4 VGPRs fewer)
  int pzb;                   // bytes per storage plane
  const char* ldp;           // source plane of the next prefetch (p + PF)
  char* stp;                 // destination plane of this iteration's last-level output
  int64_t gx, gxu, gy0;
  uint32_t gx32;             // Q32 noise counter: lane part
  int gdy;                   // folded tile: this lane's y offset from gy0 (0 or ystep)
  bool edge;
  void* xl;                  // FCfg::LX: this wave's LDS rows (ROWS x 66 pairs, pads 0 / 65 zero)
  int* seq;                  // FCfg::NSYNC: the workgroup's per-wave sequence words (LDS)
  int it;                    // FCfg::NSYNC: pipeline iterations run by this workgroup so far
  bool wait_up, wait_dn;     // FCfg::NSYNC: whether this wave waits for its up / down partner
  int dvoff;                 // FCfg::LR: this lane's source offset of the wave's first DMA piece
                             // (the second: + 2 rows)
  uint32_t rbase;            // FCfg::LR: LDS address of ring slot 0, this wave's first row
  bool lst;                  // FCfg::LR: this wave stores the last level (its VMEM count)
  const uint32_t* puw;       // FCfg::PUL: the step-uniform Philox words (LDS, 8 per level)
};

// gfx950 LDS-DMA of 16 bytes per lane: buffer rsrc r at byte offset voff -> LDS address
// lds + 16 * lane (one wave instruction moves 1 KiB).  Inline asm rather than the builtin: the
// compiler orders every later LDS access and barrier behind a builtin DMA with s_waitcnt
// vmcnt(0), which drains the prefetch each plane; FCfg::LR counts its DMAs itself (lr_wait).
// M0 is saved and restored around it (the compiler reserves it).
// soff: a wave-uniform byte offset added to voff (the scalar offset field).
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, int voff, int soff, uint32_t lds) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %1\n\t"
      "buffer_load_dwordx4 %2, %3, %4 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "s"(lds), "v"(voff), "s"(r), "s"(soff)
      : "memory");
}

// One vector-memory store to an empty descriptor (num_records 0: dropped) that the compiler can
// neither merge nor delete.  FCfg::LR's counted waits (lr_wait) assume ROWS stores per pipeline
// iteration on the storing waves; builtin stores of the same value to the same out-of-range offset
// were merged -- the segment prologue issued one of its four padding stores, so the first
// iteration's lr_wait let three of the wave's DMA pieces still be in flight when the level-0 rows
// were read (an intermittent fp64 mismatch at segment starts, profiles/r6_f64_lr.txt).
__device__ __forceinline__ void pad_store(__amdgpu_buffer_rsrc_t r) {
  asm volatile("buffer_store_dword %0, off, %1, 0" ::"v"(0u), "s"(r) : "memory");
}

template <int N>
__device__ __forceinline__ void vmcnt_wait() {
  static_assert(N >= 0 && N < 64, "vmcnt field");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// FCfg::LR: wait until this wave's DMA of the plane consumed next has landed.  Per pipeline
// iteration a wave issues ND DMA pieces (fp32 2, fp64 4) right after the barrier and then S
// stores (ROWS when it stores the last level, else 0; constant per wave: the fill periods store to
// an empty descriptor), so the DMA of plane p (issued PF iterations back) has S + (PF - 1)(ND + S)
// younger VMEM operations (the segment prologue pads its DMAs with S empty stores to keep the
// count).
template <class C>
__device__ __forceinline__ void lr_wait(const FusedSeg& sg) {
  constexpr int S = C::ROWS, PF = C::PF, ND = C::ND;
  if (sg.lst) vmcnt_wait<S + (PF - 1) * (ND + S)>();
  else vmcnt_wait<(PF - 1) * ND>();
}

template <class C>
__device__ __forceinline__ int64_t gwrap(int64_t v, int64_t L) {
  if constexpr (C::PERIODIC) return wrap(v, L);
  else return v;
}

// v[lane-1] + v[lane+1] + s in two DPP adds (the right neighbour is added to s first): the
// y/z partial sum folds into the x-neighbour instructions.  Lanes without a source read 0
// (bound_ctrl); they only feed tile-halo cells.
//   No hazard wait states: a DPP read of a VGPR needs 2 wait states after a VALU write of it,
//   and the DPP sources here are level-0 planes (written by buffer loads, not the VALU) or
//   level outputs written in an earlier pipeline iteration.  The compiler cannot see through
//   the asm, so the built code object is checked instead: scripts/check_dpp_hazards.py scans
//   every DPP instruction of libgs_hip.so (`make check-isa`, tests/test_isa_hazards.py).  The
//   ablation bit 8 restores the leading `s_nop 1` (2.8 % slower, profiles/r2_ab_dpp_nop.txt).
template <bool NOP>
__device__ __forceinline__ float lane_pair_sum_add(float v, float s) {
  float t, r;
  if constexpr (NOP) {
    asm volatile(
        "s_nop 1\n\t"
        "v_add_f32_dpp %1, %2, %3 wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "v_add_f32_dpp %0, %2, %1 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1"
        : "=v"(r), "=&v"(t)
        : "v"(v), "v"(s));
  } else {
    asm volatile(
        "v_add_f32_dpp %1, %2, %3 wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "v_add_f32_dpp %0, %2, %1 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1"
        : "=v"(r), "=&v"(t)
        : "v"(v), "v"(s));
  }
  return r;
}
template <bool NOP>
__device__ __forceinline__ double lane_pair_sum_add(double v, double s) {
  return lane_from_left(v) + lane_from_right(v) + s;  // compiler DPP moves (hazards handled)
}

// One (u, v) pair from LDS as a single 8-byte ds_read_b64.
__device__ __forceinline__ PairT<float>::type lds_load2(const PairT<float>::type* p) {
  const uint64_t b = *reinterpret_cast<const uint64_t*>(__builtin_assume_aligned(p, 8));
  return PairT<float>::type{__uint_as_float((uint32_t)b), __uint_as_float((uint32_t)(b >> 32))};
}
__device__ __forceinline__ PairT<double>::type lds_load2(const PairT<double>::type* p) {
  return *p;
}

// The cell update of one level: neighbour sums, reaction, noise, Euler step, and the running
// partial sum for the next plane.  xs: x-neighbour pair sums, ym/yp: y-neighbours, in: this
// plane, c: the centre (plane before), w: the Philox word.
template <class C>
__device__ __forceinline__ typename C::V2 cell_update(typename C::V2& A, typename C::V2 in,
                                                      typename C::V2 c, typename C::V2 ym,
                                                      typename C::V2 yp, const FoldCoef<typename C::T>& f,
                                                      typename C::T ar31, typename C::V2 kc,
                                                      uint32_t w, typename C::V2 xs = {}) {
  using T = typename C::T;
  using V2 = typename C::V2;
  const V2 s = A + in;
  const V2 yz = (ym + yp) + c;
  constexpr bool nop = (C::ABL & 8) != 0;
  if constexpr (C::LX) A = V2{xs.x + yz.x, xs.y + yz.y};  // xs = left + right (LDS, FCfg::LX)
  else A = V2{lane_pair_sum_add<nop>(in.x, yz.x), lane_pair_sum_add<nop>(in.y, yz.y)};
  if constexpr (sizeof(T) == 8) {
    // fp64 has no packed arithmetic: the vector form below would compute uvv twice (4 v_mul_f64)
    // and, with kc in VGPRs as the first FMA's accumulator, copy it first (v_mov_b64 + v_fmac).
    // The same expression tree, scalarised: uvv = (cu cv) cv once; v's first term is dt uvv
    // (kc.y = 0: fma(dt, uvv, 0) rounds like the product); three-operand FMAs.  Bit-identical.
    const T uvv = (c.x * c.y) * c.y;
    V2 P;
    P.x = __builtin_fma(f.kd.x, uvv, kc.x);
    P.y = f.kd.y * uvv;
    P.x = __builtin_fma(f.ks.x, s.x, P.x);
    P.y = __builtin_fma(f.ks.y, s.y, P.y);
    P.x = __builtin_fma(f.kcc.x, c.x, P.x);
    P.y = __builtin_fma(f.kcc.y, c.y, P.y);
    if constexpr (C::NOISE) P.x = __builtin_fma(ar31, (T)(int32_t)w, P.x);
    return P;
  }
  // uvv in both halves: (cu cv, cv cv) then (cu cv cv, cu cv cv)
  const V2 t = c * c.yy;
  const V2 uvv = t.xx * c.yy;
  V2 P = __builtin_elementwise_fma(f.kd, uvv, kc);
  P = __builtin_elementwise_fma(f.ks, s, P);
  P = __builtin_elementwise_fma(f.kcc, c, P);
  if constexpr (C::NOISE) P.x = fma(ar31, (T)(int32_t)w, P.x);
  return P;
}

// One pipeline iteration p (i = p - pstart).  IR = i % R, IS = i % NS.
// Non-skewed: level l+1 is computed from level l of the SAME iteration (one barrier per level).
// Skewed: level l+1 consumes level l's output of the PREVIOUS iteration, so every level's
// input rows are published before a single barrier; level l produces plane p - (2l + 1).
// FCfg::LR: issue the wave's DMA pieces of level-0 plane p + PF (rows 4w .. 4w + 3) into ring
// slot `slot`.  Unconditional (an empty descriptor past the segment): constant VMEM count.
template <class C>
__device__ __forceinline__ void lr_dma(FusedSeg& sg, int slot, bool ok) {
  const __amdgpu_buffer_rsrc_t r = plane_rsrc(sg.ldp, ok ? sg.pzb : 0);
  constexpr uint32_t kSlot = C::RT * 64 * sizeof(typename C::V2);
  // (every piece's offset goes through voffset: the range check of a raw buffer access does not
  // include soffset, and a first piece above the plane must not drag a valid later piece out of
  // range with it).  fp32: piece k = rows 2k, 2k + 1; fp64: piece k = row k.
  constexpr int kRows = C::ROWS / C::ND;
#pragma unroll
  for (int k = 0; k < C::ND; ++k)
    dma16(r, sg.dvoff + k * kRows * sg.pitchb, 0, sg.rbase + (uint32_t)slot * kSlot + 1024u * k);
  sg.ldp += sg.pzb;
}

template <class C, typename T, int IR, int IS, bool FILL>
__device__ __forceinline__ void fused_iter(FusedState<C>& S,
                                           typename C::V2 (*xch)[C::NS][C::WAVES][2][64],
                                           typename C::V2 (*ring)[C::RT][64],
                                           const FusedArgs& a, const FoldCoef<T>& f,
                                           uint64_t seed, FusedSeg& sg) {
  using V2 = typename C::V2;
  constexpr int ROWS = C::ROWS, TL = C::TL, NS = C::NS;
  const Geom& g = a.g;
  const int p = sg.p;
  // prefetch level-0 plane p+PF into the ring slot of plane p-2.  Issued unconditionally
  // (an empty descriptor past the segment) so every iteration has the same VMEM count and
  // the compiler's s_waitcnt vmcnt(N) can leave the prefetch in flight.  (FCfg::LR: after the
  // barrier below, into the LDS ring.)
  if constexpr (!C::LR) {
    const bool pf_ok = p + C::PF < sg.ldend;
    const __amdgpu_buffer_rsrc_t r =
        plane_rsrc((C::ABL & 2) ? sg.ldp - (int64_t)(p + C::PF + g.H) * sg.pzb : sg.ldp,
                   pf_ok ? sg.pzb : 0);
#pragma unroll
    for (int j = 0; j < ROWS; ++j)
      S.LD[(IR + C::PF) % C::R][j] = bload(r, sg.voff + j * sg.pitchb, (V2*)nullptr);
    sg.ldp += sg.pzb;
  }
  gs::U4 pre[TL];  // hoisted blocks (C::HOIST); unused otherwise
  if constexpr (C::HOIST) {
    const uint32_t Ly4 = (uint32_t)((g.Ly + 3) >> 2);
    const uint32_t gy4 = (uint32_t)(gwrap<C>(sg.gy0, g.Ly) >> 2);
#pragma unroll
    for (int l = TL - C::HOISTN; l < TL; ++l) {
      const int q = C::SKEW ? p - (2 * l + 1) : p - l - 1;
      const int64_t gz = gwrap<C>(g.oz + q, g.Lz);
      const uint32_t qu = (uint32_t)g.Lx * (gy4 + Ly4 * (uint32_t)gz);
      pre[l] = philox_lane_v(qu + sg.gx32, &S.pu[5 * l], S.kv);
    }
  }
  if constexpr (C::SKEW) {
#pragma unroll
    for (int l = C::LR ? 1 : 0; l < TL; ++l) {
      const V2* in = l == 0 ? S.LD[C::LR ? 0 : IR] : S.OUT[l == 0 ? 0 : l - 1][(IS + NS - 1) % NS];
      xch[C::xi(l)][IS][sg.wave][0][sg.lane] = in[0];
      xch[C::xi(l)][IS][sg.wave][1][sg.lane] = in[ROWS - 1];
    }
    if constexpr (C::LR) {
      // this wave's DMA of plane p has landed; after the barrier every wave's has, and every
      // wave is done with plane p - 2's slot, which the DMA of plane p + PF then overwrites
      lr_wait<C>(sg);
      __syncthreads();
      lr_dma<C>(sg, (IR + C::PF) % C::R, p + C::PF < sg.ldend);
    } else if constexpr (C::NSYNC) {
      // publish this iteration's rows, then wait for the partners' (see FCfg::NSYNC)
      const int it = ++sg.it;
      asm volatile("" ::: "memory");
      __hip_atomic_store(&sg.seq[sg.wave], it, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      // bounded: a scheduling bug must end in wrong numbers (caught by the bitwise tests), never
      // in a wave that spins forever
      for (int spins = 0; spins < (1 << 22); ++spins) {
        const int a = sg.wait_up ? __hip_atomic_load(&sg.seq[sg.wup], __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_WORKGROUP) : it;
        const int b = sg.wait_dn ? __hip_atomic_load(&sg.seq[sg.wdn], __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_WORKGROUP) : it;
        if (a >= it && b >= it) break;
        __builtin_amdgcn_s_sleep(0);
      }
      asm volatile("" ::: "memory");
    } else if constexpr (!(C::ABL & 1)) {
      __syncthreads();
    }
  }
#pragma unroll
  for (int li = 0; li < TL; ++li) {
    const int l = C::SKEW ? TL - 1 - li : li;  // skewed: top level first (see NS)
    // input plane of consumer l and the centre plane one before it
    constexpr int kIn = C::SKEW ? (IS + NS - 1) % NS : IS;
    constexpr int kC = C::SKEW ? (IS + NS - 2) % NS : (IS + NS - 1) % NS;
    V2* in = l == 0 ? S.LD[C::LR ? 0 : IR] : S.OUT[l == 0 ? 0 : l - 1][kIn];
    V2* Cc = l == 0 ? S.LD[C::LR ? 0 : (IR + C::R - 1) % C::R] : S.OUT[l == 0 ? 0 : l - 1][kC];
    if constexpr (!C::SKEW) {
      xch[l][IS][sg.wave][0][sg.lane] = in[0];
      xch[l][IS][sg.wave][1][sg.lane] = in[ROWS - 1];
      if constexpr (!(C::ABL & 1)) __syncthreads();
    }
    const int q = C::SKEW ? p - (2 * l + 1) : p - l - 1;  // plane produced by level l+1
    // level l+1 is needed on planes [z0 - (T-1) + l, z1 + (T-1) - l) only (the dependency
    // cone of the segment's outputs), and the plane just below that range builds the running
    // partial sum A the first needed plane consumes.  The pipeline fill and drain iterations
    // compute it outside that range too: the first periods of a segment (FILL) skip those
    // level computations (uniform branches; the last level's stores stay unconditional -- to
    // the empty descriptor -- so every iteration keeps the same VMEM count for the counted
    // vmcnt waits).  In p: skewed q >= lo - 1 <=> p - z0 >= 3l + 1 - T and q < hi <=>
    // pend - p > T - 1 - l; non-skewed p - z0 >= 2l + 1 - T (no drain).  The steady-state
    // periods carry no checks, so their registers and schedule are unchanged.
    bool need = true;
    if constexpr (FILL) {
      const int d = p - sg.z0, e = sg.pend - p;
      need = d >= (C::SKEW ? 3 * l + 1 - TL : 2 * l + 1 - TL) && (!C::SKEW || e > TL - 1 - l);
      // (LRC: level 0 runs from the first iteration on -- it hands its rows on as the next
      // iteration's centre; the one extra level-0 update per segment feeds no needed plane)
      if constexpr (C::LRC) need = need || l == 0;
      if (!need && l + 1 == TL && !((sg.skip >> l) & 1)) {
        const __amdgpu_buffer_rsrc_t w = plane_rsrc(sg.stp, 0);
#pragma unroll
        for (int j = 0; j < ROWS; ++j) {
          if constexpr (C::LR) pad_store(w);  // (counted by lr_wait: never merged)
          else bstore<C::STORE_AUX>(w, (int)0x80000000, in[j]);
        }
      }
    }
    if (need && !((sg.skip >> l) & 1)) {  // wave-uniform
      V2 up, dn;
      V2 r0[C::LR ? ROWS : 1], c0[C::LR ? ROWS : 1];
      if (C::LR && l == 0) {
        // level 0 from the LDS ring: this plane's rows and the rows next to them (the wrap-around
        // rows of waves 0 / last are tile-halo rows whose values never reach an output), and
        // the centre plane before it
        constexpr int RT = C::RT;
        const int r = sg.wave * ROWS;
        up = lds_load2(&ring[IR][(r + RT - 1) % RT][sg.lane]);
        dn = lds_load2(&ring[IR][(r + ROWS) % RT][sg.lane]);
#pragma unroll
        for (int j = 0; j < (C::LR ? ROWS : 1); ++j) {
          r0[j] = lds_load2(&ring[IR][r + j][sg.lane]);
          if constexpr (!C::LRC) c0[j] = lds_load2(&ring[(IR + C::R - 1) % C::R][r + j][sg.lane]);
        }
        in = r0;
        Cc = C::LRC ? S.C0 : c0;  // (LRC: the rows become the next centre after the update)
      } else {
        up = lds_load2(&xch[C::xi(l)][IS][sg.wup][1][sg.lane]);
        dn = lds_load2(&xch[C::xi(l)][IS][sg.wdn][0][sg.lane]);
      }
      V2* xl = (V2*)sg.xl;
      if constexpr (C::LX) {
        // this wave's input rows out to LDS and the x neighbours back (one wave: LDS executes
        // its instructions in order, so no barrier; the asm keeps the compiler's order)
#pragma unroll
        for (int j = 0; j < ROWS; ++j) xl[j * 66 + sg.lane + 1] = in[j];
        asm volatile("" ::: "memory");
      }
      const int64_t gz = gwrap<C>(g.oz + q, g.Lz);
      const uint64_t tstep = (uint64_t)(a.t + l);
      V2 res[ROWS];
#pragma unroll
      for (int m = 0; m < ROWS / 4; ++m) {
        gs::U4 blk{0, 0, 0, 0};
        // ABL bit 32 (exact): the Philox draw only on lanes inside the level's x dependency cone
        // [l+1, 63-l) (the other lanes' values never reach a stored output): an exec-masked
        // draw, so the inactive lanes do not switch -- energy per cell update in the
        // power-limited regime
        if constexpr (C::NOISE) {
          bool draw = true;
          if constexpr ((C::ABL & 32) != 0) draw = sg.lane >= l + 1 && sg.lane < 63 - l;
          if (draw) {
          if constexpr (C::Q32) {
            // counter q = gx + Lx * (gy4 + Ly4 * gz) < 2^32: uniform part + lane part (a
            // quad never straddles the periodic wrap: Ly % 4 == 0 there)
            const uint32_t Ly4 = (uint32_t)((g.Ly + 3) >> 2);
            const uint32_t gy4 = (uint32_t)(gwrap<C>(sg.gy0 + 4 * m, g.Ly) >> 2);
            const uint32_t qu = (uint32_t)g.Lx * (gy4 + Ly4 * (uint32_t)gz);
            if (C::hoisted(l)) blk = pre[l];
            else if constexpr (C::PU) blk = philox_lane_v(qu + sg.gx32, &S.pu[5 * l], S.kv);
            else if constexpr (C::PUL) {
              const gs_u4 w = *(const gs_u4*)__builtin_assume_aligned(sg.puw + 8 * l, 16);
              const uint32_t u[5] = {w.x, w.y, w.z, w.w, sg.puw[8 * l + 4]};
              if constexpr (C::KVL) {
                uint32_t kv[16];
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                  const gs_u4 k4 = *(const gs_u4*)__builtin_assume_aligned(sg.puw + 8 * TL + 4 * i, 16);
                  kv[4 * i] = k4.x; kv[4 * i + 1] = k4.y; kv[4 * i + 2] = k4.z; kv[4 * i + 3] = k4.w;
                }
                blk = philox_lane_v(qu + sg.gx32, u, kv);
              } else {
                blk = philox_lane_v(qu + sg.gx32, u, S.kv);
              }
            }
            else blk = philox_dev<true, C::KV>(qu + sg.gx32, 0u, tstep, seed, S.kv);
          } else {
            const int64_t gyq = gwrap<C>(sg.gy0 + 4 * m, g.Ly);
            const uint64_t Ly4 = ((uint64_t)g.Ly + 3) >> 2;
            const uint64_t qq = (uint64_t)sg.gx + (uint64_t)g.Lx * ((uint64_t)(gyq >> 2) +
                                                                   Ly4 * (uint64_t)gz);
            blk = philox_dev<false, C::KV>((uint32_t)qq, (uint32_t)(qq >> 32), tstep, seed, S.kv);
          }
          }
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int j = 4 * m + k;
          const V2 ym = j == 0 ? up : in[j - 1];
          const V2 yp = j == ROWS - 1 ? dn : in[j + 1];
          const uint32_t w = k == 0 ? blk.x : (k == 1 ? blk.y : (k == 2 ? blk.z : blk.w));
          V2 xs{};
          if constexpr (C::LX) {
            const V2 xa = xl[j * 66 + sg.lane], xb = xl[j * 66 + sg.lane + 2];
            xs = V2{xa.x + xb.x, xa.y + xb.y};
          }
          res[j] = cell_update<C>(S.A[l][j], in[j], Cc[j], ym, yp, f, S.ar31, S.kc, w, xs);
        }
      }
      if constexpr (C::LX) asm volatile("" ::: "memory");
      if constexpr (C::LRC) {
        if (l == 0) {
#pragma unroll
          for (int j = 0; j < ROWS; ++j) S.C0[j] = in[j];  // the next iteration's centre
        }
      }
      if (l + 1 < TL) {
        if (sg.edge) {
          const T bu = (T)gs::bc_u(a.t + l + 1);
          const bool zout = (g.oz + q < 0) || (g.oz + q >= g.Lz);
          const bool xout = sg.gxu < 0 || sg.gxu >= g.Lx;
#pragma unroll
          for (int j = 0; j < ROWS; ++j) {
            int gdy = C::FOLD ? sg.gdy : 0;
            if constexpr (C::FOLD && C::LR && TL >= 4) gdy = (sg.srows & 16) ? a.ystep : 0;
            const int64_t gyj = sg.gy0 + j + gdy;
            if (zout || xout || gyj < 0 || gyj >= g.Ly) res[j] = V2{bu, (T)0};
          }
        }
#pragma unroll
        for (int j = 0; j < ROWS; ++j) S.OUT[l][IS][j] = res[j];
      } else {
        // unconditional stores: planes before the segment go to an empty descriptor
        const __amdgpu_buffer_rsrc_t w = plane_rsrc(sg.stp, q >= sg.z0 ? sg.pzb : 0);
#pragma unroll
        for (int j = 0; j < ROWS; ++j) {
          int off;
          if constexpr (C::FOLD && C::LR && TL >= 4)
            off = ((sg.srows >> j) & 1) ? sg.svoff + j * sg.pitchb : (int)0x80000000;
          else if constexpr (C::FOLD) off = sg.soff[j];  // per lane (a folded pair's halves differ)
          else off = (j >= sg.srow0 && j < sg.srow1) ? sg.svoff + j * sg.pitchb : (int)0x80000000;
          bstore<C::STORE_AUX>(w, off, res[j]);
        }
      }
    }
  }
  sg.stp += sg.pzb;
}

// Unrolled walk over one ring period; returns false when the segment is done.
template <class C, typename T, int I, bool FILL>
__device__ __forceinline__ bool fused_period(FusedState<C>& S,
                                             typename C::V2 (*xch)[C::NS][C::WAVES][2][64],
                                             typename C::V2 (*ring)[C::RT][64],
                                             const FusedArgs& a, const FoldCoef<T>& f,
                                             uint64_t seed, FusedSeg& sg) {
  if constexpr (I == C::PERIOD) {
    return true;
  } else {
    fused_iter<C, T, I % C::R, I % C::NS, FILL>(S, xch, ring, a, f, seed, sg);
    if (++sg.p >= sg.pend) return false;
    return fused_period<C, T, I + 1, FILL>(S, xch, ring, a, f, seed, sg);
  }
}

// level-0 read window of tile `tile` in x / y (gs::tile_window on the device)
template <class C>
__device__ __forceinline__ void gate_cone(const FusedArgs& a, int tile, int* X0, int* xw, int* Y0,
                                          int* yext) {
  constexpr int TL = C::TL;
  *xw = 64;
  *yext = C::WAVES * C::ROWS;
  if (C::FOLD && tile >= a.ntxf * a.nty) {
    const int f2 = tile - a.ntxf * a.nty;
    *X0 = a.ntxf * a.xstep - TL;
    *Y0 = a.ybase + 2 * f2 * a.ystep - TL;
    *xw = 32;
    *yext += a.ystep;
  } else {
    const int ntxe = C::FOLD ? a.ntxf : a.ntx;
    *X0 = (tile % ntxe) * a.xstep - TL;
    *Y0 = a.ybase + (tile / ntxe) * a.ystep - TL;
  }
}

// The kernel body; GATED: the gated pass's entry (k_fused_gated, sched 3), whose prologue
// carries the halo exchange (gate.hpp).  The plain entry compiles without any of it.
template <class C, typename T, int GATED>
__device__ __forceinline__ void fused_body(const typename C::V2* __restrict__ s,
                                           typename C::V2* __restrict__ d, const FusedArgs& a,
                                           const FoldCoef<T>& f, uint64_t seed) {
  constexpr int ROWS = C::ROWS, WAVES = C::WAVES, TL = C::TL;
  static_assert(ROWS % 4 == 0, "rows per wave must hold whole noise quads");
  __shared__ typename C::V2 xch[C::XL][C::NS][WAVES][2][64];  // [level][ring][wave][row][lane]
  // FCfg::LR: the level-0 plane ring [slot][tile row][column]
  __shared__ typename C::V2 ring[C::LR ? C::R : 1][C::LR ? C::RT : 1][64];
  __shared__ typename C::V2 xrow[C::LX ? WAVES * ROWS * 66 : 1];  // FCfg::LX rows, 1-lane pads
  const Geom& g = a.g;
  FusedSeg sg;
  sg.lane = threadIdx.x & 63;
  sg.wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  sg.xl = nullptr;
  __shared__ int seqw[C::NSYNC ? WAVES : 1];
  sg.seq = seqw;
  sg.it = 0;
  sg.wait_up = sg.wave > 0;
  sg.wait_dn = sg.wave < WAVES - 1;
  if constexpr (C::NSYNC) {
    if (sg.lane == 0) seqw[sg.wave] = 0;
    __syncthreads();  // once: every word initialised before any wave polls
  }
  if constexpr (C::LX) {
    typename C::V2* w = xrow + sg.wave * ROWS * 66;
    if (sg.lane < ROWS) {  // the pads read by lanes 0 / 63: 0, as DPP's bound_ctrl gives
      w[sg.lane * 66] = typename C::V2{(T)0, (T)0};
      w[sg.lane * 66 + 65] = typename C::V2{(T)0, (T)0};
    }
    sg.xl = w;
  }
  sg.wup = sg.wave == 0 ? WAVES - 1 : sg.wave - 1;
  sg.wdn = sg.wave == WAVES - 1 ? 0 : sg.wave + 1;
  sg.skip = 0;
#pragma unroll
  for (int l = 0; l < TL; ++l)
    if (sg.wave * ROWS > C::need_hi(l) || sg.wave * ROWS + ROWS - 1 < l + 1) sg.skip |= 1 << l;
  sg.pitchb = g.px * (int)sizeof(typename C::V2);
  sg.pzb = (int)(gs::plane_elems(g) * (int64_t)sizeof(typename C::V2));
  sg.lst = !((sg.skip >> (TL - 1)) & 1);
  sg.rbase = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)&ring[0][C::LR ? sg.wave * ROWS : 0][0];
  sg.dvoff = 0;
  typename C::V2 (*const ringp)[C::RT][64] = (typename C::V2 (*)[C::RT][64])ring;
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
  uint64_t t_gate = 0;  // (pairs tables: the workgroup's start, for the exchange's time bounds)
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
  } else if (GATED) {
    // gated pass: one table unit per workgroup (pairs: two entries, an ungated chunk then a
    // start-gated one), each XCD group a contiguous range (the host orders the table by z, then
    // tile)
    const int w = (b % 8) * a.grpM + b / 8;
    if constexpr (GATED == 2) {
      if (2 * w >= a.ngunits) return;
      lu0 = 2 * w;
      lu1 = lu0 + 2;
      const GateUnit e0 = a.gunits[lu0];
      t_gate = wall_clock64();  // the exchange's start for this workgroup (emulation, timeout)
      if (e0.pk >= 0) gate_pack<T>(a, e0.pk);  // the wait comes before the second entry
    } else {
      lu0 = w;
      lu1 = lu0 + 1;
      if (lu0 >= a.ngunits) return;
      // a start-gated unit packs, signals, waits and fills its cone's ghost cells first -- here,
      // before the march state below is live, so the production loop's registers are untouched
      const GateUnit un = a.gunits[lu0];
      const int pk = (a.gate_pre & 1) ? -1 : un.pk;  // a carried exchange is packed already
      if (pk >= 0 || un.wait) {
        int X0, xw, Y0, yext;
        gate_cone<C>(a, un.tile, &X0, &xw, &Y0, &yext);
        gate_start<T>(a, pk, un.wait != 0, X0, xw, Y0, yext, un.z0 - TL, un.z1 + TL);
      }
    }
  }
  FusedState<C> S;
  // a wave that skips a level still publishes that level's (never used) rows: keep them defined
#pragma unroll
  for (int l = 0; l < C::NO; ++l)
#pragma unroll
    for (int i = 0; i < C::NS; ++i)
#pragma unroll
      for (int j = 0; j < ROWS; ++j) S.OUT[l][i][j] = typename C::V2{(T)0, (T)0};
  {
    const T k0 = f.kc.x, k1 = f.kc.y;
    if constexpr (sizeof(T) == 4) {
      asm volatile("v_mov_b32 %0, %1" : "=v"(S.kc.x) : "s"(k0));
      asm volatile("v_mov_b32 %0, %1" : "=v"(S.kc.y) : "s"(k1));
    } else {
      asm volatile("v_mov_b64 %0, %1" : "=v"(S.kc.x) : "s"(k0));
      asm volatile("v_mov_b64 %0, %1" : "=v"(S.kc.y) : "s"(k1));
    }
  }
  if constexpr (C::KV && !C::KVL) {
#pragma unroll
    for (int r = 3; r < 10; ++r) {
      const uint32_t k0 = (uint32_t)seed + (uint32_t)r * kPhW0;
      const uint32_t k1 = (uint32_t)(seed >> 32) + (uint32_t)r * kPhW1;
      asm volatile("v_mov_b32 %0, %1" : "=v"(S.kv[2 * (r - 3)]) : "s"(k0));
      asm volatile("v_mov_b32 %0, %1" : "=v"(S.kv[2 * (r - 3) + 1]) : "s"(k1));
    }
  }
  __shared__ __attribute__((aligned(16))) uint32_t puw[C::PUL ? 8 * TL + 16 : 4];
  sg.puw = puw;
  if constexpr (C::PUL) {
    // written by wave 0 before the first segment's barrier (FCfg::LR opens every segment with one)
    if (sg.wave == 0 && sg.lane == 0) {
#pragma unroll
      for (int l = 0; l < TL; ++l) {
        const PhiloxU u = philox_uniform((uint64_t)(a.t + l), seed);
        puw[8 * l + 0] = u.x1;
        puw[8 * l + 1] = u.x2;
        puw[8 * l + 2] = u.x3;
        puw[8 * l + 3] = u.k3;
        puw[8 * l + 4] = u.x4;
      }
      if constexpr (C::KVL) {
#pragma unroll
        for (int r = 3; r < 10; ++r) {
          puw[8 * TL + 2 * (r - 3)] = (uint32_t)seed + (uint32_t)r * kPhW0;
          puw[8 * TL + 2 * (r - 3) + 1] = (uint32_t)(seed >> 32) + (uint32_t)r * kPhW1;
        }
      }
    }
  }
  if constexpr (C::PU) {
#pragma unroll
    for (int l = 0; l < TL; ++l) {
      const PhiloxU u = philox_uniform((uint64_t)(a.t + l), seed);
      const uint32_t w[5] = {u.x1, u.x2, u.x3, u.k3, u.x4};
#pragma unroll
      for (int i = 0; i < 5; ++i) asm volatile("v_mov_b32 %0, %1" : "=v"(S.pu[5 * l + i]) : "s"(w[i]));
    }
  }
  if constexpr (C::NOISE) {
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
    } else if (GATED) {
      const GateUnit un = a.gunits[lu];
      if (un.tile < 0) continue;  // an empty entry of a pairs table (uniform per workgroup)
      if constexpr (GATED == 2) {
        if (un.wait) {
          // the second entry of a pair: the peers' flags and the cone's ghosts, after the first
          // entry's march (which covered the exchange)
          int X0, xw, Y0, yext;
          gate_cone<C>(a, un.tile, &X0, &xw, &Y0, &yext);
          gate_unpack<T, 4>(a, X0, xw, Y0, yext, un.z0 - TL, un.z1 + TL, t_gate);
        }
      }
      u = (int64_t)un.tile * nzv + (un.z0 - a.zlo[0]);
      uend = (int64_t)un.tile * nzv + (un.z1 - a.zlo[0]);
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
      int tx, ty, xw = 64, dy = 0;  // x width of the tile in lanes; this lane's y offset
      bool live = true;             // false: the idle upper half of an unpaired folded tile
      if (C::FOLD && tile >= a.ntxf * a.nty) {
        // folded strip unit: lanes 0-31 y-tile ty, lanes 32-63 y-tile ty + 1 (pairs only)
        const int f = tile - a.ntxf * a.nty;
        tx = a.ntxf;
        ty = 2 * f;
        xw = 32;
        if (sg.lane >= 32) {
          if (ty + 1 < a.nty) dy = a.ystep;
          else live = false;
        }
      } else {
        const int ntxe = C::FOLD ? a.ntxf : a.ntx;  // full tiles per row of tiles
        tx = tile % ntxe;
        ty = tile / ntxe;
      }
      const int X0 = tx * a.xstep - TL;
      const int Y0 = a.ybase + ty * a.ystep - TL;
      const int x = X0 + (C::FOLD ? (sg.lane & (xw - 1)) : sg.lane);
      const int ylo = Y0 + sg.wave * ROWS;
      // lane byte offset inside a plane (row ylo + dy); negative values are out of range
      sg.voff = ((ylo + dy + g.H) * g.px + x + g.xo) * (int)sizeof(typename C::V2);
      sg.gxu = g.ox + x;
      sg.gx = gwrap<C>(sg.gxu, g.Lx);
      sg.gy0 = g.oy + ylo;
      sg.gdy = dy;
      // Q32 counter gx + Lx * (gy/4 + Ly4 * gz): the upper half's dy (a multiple of 4) joins the
      // lane part
      sg.gx32 = (uint32_t)sg.gx + (uint32_t)g.Lx * (uint32_t)(dy >> 2);
      const int ox1 = min(X0 + TL + (xw == 64 ? a.xstep : 32 - 2 * TL), a.mx1);
      const int oy0 = max(Y0 + TL, a.my0), oy1 = min(Y0 + TL + a.ystep, a.my1);
      const bool xin = live && x >= max(X0 + TL, a.mx0) && x < ox1;
      sg.svoff = xin ? sg.voff : (int)0x80000000;  // masked lanes store out of range
      sg.srow0 = max(oy0 - ylo, 0);
      sg.srow1 = min(oy1 - ylo, ROWS);
      if constexpr (C::FOLD) {
        // the lane's own y-tile (Y0 + dy): its store rows, folded into per-row offsets once
        const int oy0l = max(Y0 + dy + TL, a.my0), oy1l = min(Y0 + dy + TL + a.ystep, a.my1);
        const int r0 = max(oy0l - ylo - dy, 0), r1 = min(oy1l - ylo - dy, ROWS);
#pragma unroll
        for (int j = 0; j < ROWS; ++j)
          sg.soff[j] = (xin && j >= r0 && j < r1) ? sg.voff + j * sg.pitchb : (int)0x80000000;
        sg.srows = 0;
#pragma unroll
        for (int j = 0; j < ROWS; ++j) sg.srows |= (xin && j >= r0 && j < r1) ? 1 << j : 0;
        if (dy) sg.srows |= 16;  // (bit 4: the upper half's y offset, for the edge resets)
      }
      const int yext = WAVES * ROWS + (xw == 32 ? a.ystep : 0);
      sg.edge = a.bcfix &&
          (g.ox + X0 < 0 || g.ox + X0 + xw > g.Lx || g.oy + Y0 < 0 ||
           g.oy + Y0 + yext > g.Ly || g.oz + z0 - TL < 0 || g.oz + z1 + TL > g.Lz);
      sg.z0 = z0;
#pragma unroll
      for (int l = 0; l < TL; ++l)
#pragma unroll
        for (int j = 0; j < ROWS; ++j) S.A[l][j] = typename C::V2{(T)0, (T)0};
      if constexpr (C::LRC) {
#pragma unroll
        for (int j = 0; j < ROWS; ++j) S.C0[j] = typename C::V2{(T)0, (T)0};
      }
      sg.p = z0 - TL;
      sg.ldend = z1 + TL;
      sg.pend = C::SKEW ? z1 + 2 * TL - 1 : z1 + TL;
      // running plane pointers: next prefetch (p + PF) and this iteration's last-level output
      const int qlast = C::SKEW ? sg.p - (2 * TL - 1) : sg.p - TL;
      sg.ldp = (const char*)s + (int64_t)(sg.p + C::PF + g.H) * sg.pzb;
      sg.stp = (char*)d + (int64_t)(qlast + g.H) * sg.pzb;
      if constexpr (C::LR) {
        // the wave's DMA pieces: fp32 lane i moves pairs 2(i & 31), +1 of tile row 4w + 2k + i / 32
        // (folded tiles: image columns >= 32 are the upper y-tile's columns 0..31)
        // (fp64: lane i moves pair i of row 4w + k)
        const int c = C::ND == 2 ? 2 * (sg.lane & 31) : sg.lane;
        const int cx = (C::FOLD && xw == 32) ? (c & 31) : c;
        const int cdy = (C::FOLD && c >= 32 && live && xw == 32) ? a.ystep : 0;
        const int crow = C::ND == 2 ? (sg.lane >> 5) : 0;
        sg.dvoff = ((Y0 + sg.wave * ROWS + crow + cdy + g.H) * g.px + X0 + cx + g.xo) *
                   (int)sizeof(typename C::V2);
        // every wave is past the previous segment's ring reads and its own DMAs have landed
        // (a DMA of the old segment's drain must not land after this segment's prologue)
        vmcnt_wait<0>();
        __syncthreads();
        // prologue: planes p .. p + PF - 1 into slots 0 .. PF - 1, each followed by the S empty
        // stores a pipeline iteration issues (lr_wait's count)
        const char* keep = sg.ldp;
        sg.ldp = (const char*)s + (int64_t)(sg.p + g.H) * sg.pzb;
#pragma unroll
        for (int k = 0; k < C::PF; ++k) {
          lr_dma<C>(sg, k, sg.p + k < sg.ldend);
          if (sg.lst) {
            const __amdgpu_buffer_rsrc_t w = plane_rsrc(sg.stp, 0);
#pragma unroll
            for (int j = 0; j < ROWS; ++j) pad_store(w);
          }
        }
        sg.ldp = keep;
      } else {
#pragma unroll
      for (int k = 0; k < C::PF; ++k) {
        const int pl = (C::ABL & 2) ? 0 : sg.p + k + g.H;
        const __amdgpu_buffer_rsrc_t r = plane_rsrc((const char*)s + (int64_t)pl * sg.pzb,
                                                    sg.p + k < sg.ldend ? sg.pzb : 0);
#pragma unroll
        for (int j = 0; j < ROWS; ++j)
          S.LD[k][j] = bload(r, sg.voff + j * sg.pitchb, (typename C::V2*)nullptr);
      }
      }
      // pipeline fill: the first periods skip level work outside the outputs' dependency
      // cone (fused_iter, FILL); every level is needed from iteration 3T-1 (skewed) / 2T on
      bool more = true;
      if constexpr (C::FILLSKIP) {
        constexpr int kFillIters = C::SKEW ? 3 * TL - 1 : 2 * TL;
        constexpr int kFillPeriods = (kFillIters + C::PERIOD - 1) / C::PERIOD;
#pragma unroll 1
        for (int np = 0; np < kFillPeriods && more; ++np)
          more = fused_period<C, T, 0, true>(S, xch, ringp, a, f, seed, sg);
      }
      while (more && fused_period<C, T, 0, false>(S, xch, ringp, a, f, seed, sg)) {
      }
    }
  }  // work list
  if constexpr (C::LR) vmcnt_wait<0>();  // the drain's DMAs land before the wave ends
  if constexpr (GATED == 3) {
    // a pass that carries the next exchange: a producer packs its own outputs that lie in an
    // outgoing message, now final (gate.hpp gate_carry)
    if (a.gate_pre & 2) {
      const GateUnit un = a.gunits[lu0];
      if (un.prod) {
        int X0, xw, Y0, yext;
        gate_cone<C>(a, un.tile, &X0, &xw, &Y0, &yext);
        // its output window, open past the sub-domain's faces: a message also holds ghost /
        // padding cells there (z slabs send whole storage planes), set up front and unchanged
        // by the pass, which the tiles at that face carry (gs::carry_window)
        constexpr int kFar = 1 << 28;
        int ox0 = max(X0 + TL, a.mx0);
        int ox1 = min(X0 + TL + (xw == 64 ? a.xstep : 32 - 2 * TL), a.mx1);
        int oy0 = max(Y0 + TL, a.my0);
        int oy1 = min(Y0 + TL + (xw == 32 ? 2 : 1) * a.ystep, a.my1);
        if (ox0 <= 0) ox0 = -kFar;
        if (ox1 >= g.nx) ox1 = kFar;
        if (oy0 <= 0) oy0 = -kFar;
        if (oy1 >= g.ny) oy1 = kFar;
        gate_carry<T>(a, d, ox0, ox1, oy0, oy1, un.z0 <= 0 ? -kFar : un.z0,
                      un.z1 >= g.nz ? kFar : un.z1);
      }
    }
  }
}

template <class C, typename T>
__global__ __launch_bounds__(64 * C::WAVES, C::WPEU) void k_fused(const typename C::V2* __restrict__ s,
                                                            typename C::V2* __restrict__ d,
                                                            FusedArgs a, FoldCoef<T> f,
                                                            uint64_t seed) {
  fused_body<C, T, 0>(s, d, a, f, seed);
}

// the gated pass's entries (gate.hpp): instantiated for the shapes FCfg::GATE_OK names only.
// MODE 0: one-unit tables; 1: pairs tables (the unpack between two marches raises the register
// pressure); 2: one-unit tables whose pass carries the next exchange (gate_carry after the
// march).  Each its own code object, so no mode pays for another's code.
template <class C, typename T, int MODE>
__global__ __launch_bounds__(64 * C::WAVES, C::WPEU) void k_fused_gated(
    const typename C::V2* __restrict__ s, typename C::V2* __restrict__ d, FusedArgs a,
    FoldCoef<T> f, uint64_t seed) {
  fused_body<C, T, MODE == 1 ? 2 : (MODE == 2 ? 3 : 1)>(s, d, a, f, seed);
}

// ------------------------------------------------------------------------------------------
inline int& fused_sched_slot();

// Folded last x strip (FCfg::FOLD): when the last x strip of tiles holds <= 32 - 2T outputs,
// its y-tiles run two per wave (lanes 0-31 tile 2f, lanes 32-63 tile 2f + 1) and the strip
// costs half its tiles.  L=256 T=3: 5 x 7 = 35 tiles -> 4 x 7 + 4 = 32 units (one more z-chunk
// per tile fits the 256 workgroup slots); L=128: 3 x 4 -> 2 x 4 + 2.
template <class C>
inline void fold_strip(FusedArgs& a) {
  const int rem = a.g.nx - (a.ntx - 1) * a.xstep;  // outputs of the last strip (1..xstep)
  if (a.ntx < 2 || rem > 32 - 2 * C::TL) return;
  a.ntxf = a.ntx - 1;
  a.nfold = (a.nty + 1) / 2;
  a.ntiles = a.ntxf * a.nty + a.nfold;
}

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
  // resident workgroups per CU of the gated entry (the host sizes a gated table to these slots)
  // (one-unit tables: the lower of the plain and the carrying entry -- a run of passes uses both)
  static int gated_occupancy(bool pairs) {
    int o = 0, o2 = 0, o3 = 0;
    if constexpr (C::GATE_OK) {
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, k_fused_gated<C, T, 0>,
                                                       64 * C::WAVES, 0) != hipSuccess)
        o = 0;
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&o2, k_fused_gated<C, T, 1>,
                                                       64 * C::WAVES, 0) != hipSuccess)
        o2 = 0;
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&o3, k_fused_gated<C, T, 2>,
                                                       64 * C::WAVES, 0) != hipSuccess)
        o3 = 0;
    }
    return pairs ? o2 : std::min(o, o3);
  }
  static void run(const void* s, void* d, const FusedArgs& a0, const gs::Params& p,
                  hipStream_t st) {
    FusedArgs a = a0;
    a.xstep = 64 - 2 * C::TL;
    a.ystep = C::YSTEP;
    a.ybase = -mod4(a.g.oy - C::TL);  // (oy + ybase - TL) % 4 == 0
    a.ntx = (a.g.nx + a.xstep - 1) / a.xstep;
    a.nty = (a.g.ny - a.ybase + a.ystep - 1) / a.ystep;
    a.ntiles = a.ntx * a.nty;
    a.ntxf = a.ntx;
    a.nfold = 0;
    if constexpr (C::FOLD) fold_strip<C>(a);
    a.units = (int64_t)a.ntiles * a.nzv;
    static int cus = 0;
    if (!cus) {
      int dev = 0;
      (void)hipGetDevice(&dev);
      if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) cus = 256;
    }
    if (a.sched == 3) {
      // gated pass: the table holds one unit per workgroup (sized by the host to the slots)
      if constexpr (C::GATE_OK) {
        a.nchunk = 1;
        a.grpM = ((a.gate_pairs ? a.ngunits / 2 : a.ngunits) + 7) / 8;
        const FoldCoef<T> f = make_fold<T>(p);
        if (a.gate_pairs)
          k_fused_gated<C, T, 1><<<(unsigned)(8 * a.grpM), 64 * C::WAVES, 0, st>>>(
              (const typename C::V2*)s, (typename C::V2*)d, a, f, p.seed);
        else if (a.gate_pre & 2)
          k_fused_gated<C, T, 2><<<(unsigned)(8 * a.grpM), 64 * C::WAVES, 0, st>>>(
              (const typename C::V2*)s, (typename C::V2*)d, a, f, p.seed);
        else
          k_fused_gated<C, T, 0><<<(unsigned)(8 * a.grpM), 64 * C::WAVES, 0, st>>>(
              (const typename C::V2*)s, (typename C::V2*)d, a, f, p.seed);
      }
      return;  // (gated_shape_cfg never names a shape without the gated entry)
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
      // the reserved slots cost a chunk per tile only when they must: if the whole device's
      // chunking already leaves >= 8 slots over, keep it (256^3 rank: 7 chunks x 35 tiles of 256
      // slots, 11 left -- a 16-slot reserve would drop to 6 chunks, +15 % per workgroup)
      if (a.reserve > 0) {
        const int64_t all = (int64_t)occupancy() * cus;
        const int n0 = (int)(all / a.ntiles);
        if (all - (int64_t)n0 * a.ntiles >= std::min(a.reserve, 8)) nch = n0;
      }
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
      // (profiles/r1_tune_chunking.txt)
      const int maxch = std::max(1, a.nzv / 2);
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
    k_fused<C, T><<<(unsigned)nwg, 64 * C::WAVES, 0, st>>>(
        (const typename C::V2*)s, (typename C::V2*)d, a, f, p.seed);
  }
};

#include "block.hpp"

// Work-schedule override: GS_FUSED_SCHED at load time or gs_fused_sched() at run time.
inline int& fused_sched_slot() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("GS_FUSED_SCHED");
    v = e ? atoi(e) : 0;
  }
  return v;
}

// Tile / prefetch configurations "<rows>x<waves>:<prefetch>[s]" (s = skewed single-barrier
// pipeline).  Index 0 is the default (fp32: 4x12:2s, fp64: 4x8:1s, the measured winners at
// L >= 256, profiles/r1_tune_*); the autotuner times the rest on the live problem.  An entry
// whose name carries "-abl" exists only in GS_ABLATION builds (timing experiments).
struct FusedCfgEntry {
  const char* name;
  bool f32, f64;  // instantiated for fp32 / fp64 (others fall back to the default)
};

inline const FusedCfgEntry* fused_cfg_table(int* n) {
  static const FusedCfgEntry t[] = {
      {"", true, true},          //  0 default
      {"4x8:1", true, true},     //  1
      {"4x8:2", true, false},    //  2
      {"4x8:1s", true, true},    //  3
      {"4x8:2s", true, false},   //  4
      {"4x8:4s", true, false},   //  5
      {"8x4:1", true, false},    //  6
      {"8x4:2", true, false},    //  7
      {"8x4:1s", true, false},   //  8
      {"8x4:4s", true, false},   //  9
      {"4x12:1", true, true},    // 10
      {"4x12:2", true, false},   // 11
      {"4x12:3", true, false},   // 12
      {"4x12:1s", true, false},  // 13
      {"4x12:2s", true, false},  // 14
      {"4x6:2s", true, true},    // 15
      {"4x6:2", false, true},    // 16
      {"4x4:2", false, true},    // 17
      {"4x16:1", true, false},   // 18
      {"4x16:1s", true, false},  // 19  64-row tile, 4 waves per SIMD (fits 128 VGPRs)
      // small grids (block.hpp): k_block, output blocks of whole x rows x BY rows x BZ planes,
      // NW waves; timed only on launches it supports (block_supported), else the default shape
      {"blk8x2w8", true, false},   // 20
      {"blk4x4w8", true, false},   // 21
      {"blk8x2w16", true, false},  // 22
      {"blk4x4w16", true, false},  // 23
      {"blk8x4w16", true, false},  // 24  (T=2 only: T=3 levels do not fit the LDS)
      {"blk8x2w16l", true, false}, // 25  last level in half-quad items
      {"blk4x4w16l", true, false}, // 26  last level in half-quad items
      {"4x12:1sf", true, false},   // 27  the last x strip folded into half-wave tiles (FCfg::FOLD)
      // the level-0 ring in LDS, filled by LDS-DMA (FCfg::LR); the only shapes with a T = 4 entry
      {"4x12:2sl", true, false},   // 28  2-plane prefetch
      {"4x12:1sl", true, false},   // 29  1-plane prefetch (T = 4 default: the ring + 3 levels' xch fit)
      {"4x12:1sfl", true, false},  // 30  folded last strip
      {"4x12:3sl", true, false},   // 31  3-plane prefetch (T = 2 only: LDS)
      {"4x12:2sfl", true, false},  // 32  2-plane prefetch, folded last strip
      // fp64 LDS ring (FCfg::LRC: PF + 1 slots, the centre plane from registers); the freed ring
      // registers hold the Philox round keys and step words (KV / PU)
      {"4x8:1sl", false, true},    // 33
#ifdef GS_ABLATION
      // measured and rejected in round 5 (exact; kept for reproduction in the ablation build):
      // fp64 LDS x-sums 4-6 % slower, neighbour-only sync 5-6 % slower (profiles/r5_f64_counters.txt,
      // r5_nsync_rejected.txt)
      {"4x8:1sx", false, true},    // 34  fp64: x-neighbour sums through LDS (FCfg::LX)
      {"4x6:2sx", false, true},    // 35  fp64: x-neighbour sums through LDS (FCfg::LX)
      {"4x8:1x", false, true},     // 36  fp64: x-neighbour sums through LDS, unskewed
      {"4x12:1sn", true, false},   // 37  neighbour-only LDS sync instead of the barrier (NSYNC)
      {"4x12:1sfn", true, false},  // 38  folded last strip + neighbour-only sync
      {"4x12:2sn", true, false},   // 39  2-plane prefetch + neighbour-only sync
      {"4x8:1sxn", false, true},   // 40  fp64: LDS x-sums + neighbour-only sync
      {"4x8:1sn", false, true},    // 41  fp64: neighbour-only sync
      {"4x12:2s-abl1", true, false},  // 42  no barriers
      {"4x12:2s-abl2", true, false},  // 43  L2-resident loads
      {"4x12:1s-abl4", true, false},  // 44  Philox keys in VGPRs (exact)
      {"4x12:2s-abl4", true, false},  // 45  Philox keys in VGPRs (exact)
      {"4x12:1s-abl8", true, false},  // 46  DPP sums with the s_nop (exact)
      {"4x12:1s-abl12", true, false}, // 47  abl4 + abl8 (exact)
      {"4x12:1s-abl16", true, false}, // 48  pipeline fill computes every level (exact)
      {"4x8:1s-abl16", true, true},   // 49  pipeline fill computes every level (exact)
      {"4x6:2s-abl16", true, true},   // 50  pipeline fill computes every level (exact)
      {"4x12:1s-abl32", true, false}, // 51  Philox only on lanes in the x cone (exact)
      {"4x12:2s-abl64", true, false}, // 52  Philox keys rebuilt on the SALU (exact)
      {"4x12:1s-abl64", true, false}, // 53  Philox keys rebuilt on the SALU (exact)
      {"4x12:1s-abl256", true, false}, // 54  step-uniform Philox words on the SALU (exact)
      {"4x12:1s-abl512", true, false}, // 55  Philox blocks of all levels before the barrier (exact)
      {"4x12:1s-abl1024", true, false}, // 56  the top level's Philox block before the barrier (exact)
      {"4x12:1s-abl1536", true, false}, // 57  the top two levels' Philox blocks before the barrier
      {"4x12:1s-abl2048", true, false}, // 58  non-temporal output stores (exact)
      {"4x12:1s-abl4096", true, false}, // 59  device-scope (write-through) output stores (exact)
      {"4x12:1s-abl6144", true, false}, // 60  both (exact)
      {"4x12:2s-abl128", true, false},  // 61  2-plane prefetch + step-uniform Philox words in VGPRs
      {"4x12:3s-abl128", true, false},  // 62  3-plane prefetch + step-uniform Philox words in VGPRs
#endif
  };
  *n = (int)(sizeof(t) / sizeof(t[0]));
  return t;
}

// whether a config is worth timing for a launch of k steps over g: the folded-strip tiles
// (FCfg::FOLD) equal their unfolded shapes unless the last x strip fits half a wave
inline bool fused_cfg_applies(int i, const Geom& g, int k) {
  int n = 0;
  const FusedCfgEntry* t = fused_cfg_table(&n);
  if (i < 0 || i >= n) return true;
  const char* colon = strchr(t[i].name, ':');
  if (!colon || !strchr(colon, 'f')) return true;  // (folded shapes: "<rows>x<waves>:<pf>sf...")
  const int xstep = 64 - 2 * k;
  const int ntx = (g.nx + xstep - 1) / xstep;
  return ntx >= 2 && g.nx - (ntx - 1) * xstep <= 32 - 2 * k;
}

inline bool fused_cfg_is_block(int i) {
  int n = 0;
  const FusedCfgEntry* t = fused_cfg_table(&n);
  return i > 0 && i < n && !strncmp(t[i].name, "blk", 3);
}

// whether block configuration i (table entries 20-26: output blocks of BY rows x BZ planes)
// holds its two level buffers in the CU's LDS at depth tl -- BCfg::FITS without instantiating
// it; a configuration that does not fit would run the default k_fused shape under its name
constexpr int kBlkBY[7] = {8, 4, 8, 4, 8, 8, 4}, kBlkBZ[7] = {2, 4, 2, 4, 4, 2, 4};
constexpr bool block_k_fits(int k, int tl, int pair_bytes) {
  return (2 * (kBlkBZ[k] + 2 * tl) * (kBlkBY[k] + 10) + 1) * 64 * pair_bytes <= 160 * 1024;
}
static_assert(block_k_fits(0, 3, 8) == BCfg<float, 3, 8, 2, 8, true>::FITS &&
                  block_k_fits(4, 3, 8) == BCfg<float, 3, 8, 4, 16, true>::FITS &&
                  block_k_fits(4, 2, 8) == BCfg<float, 2, 8, 4, 16, true>::FITS &&
                  block_k_fits(1, 3, 8) == BCfg<float, 3, 4, 4, 8, true>::FITS &&
                  !block_k_fits(4, 3, 8) && block_k_fits(4, 2, 8),
              "block_cfg_fits must match BCfg::FITS");
inline bool block_cfg_fits(int i, int tl, int pair_bytes) {
  if (!fused_cfg_is_block(i) || i < 20 || i > 26) return true;
  return block_k_fits(i - 20, tl, pair_bytes);
}

inline int& fused_cfg_slot() {
  static int v = -1;
  return v;
}

// index of configuration `e` ("" or null = default), -1 if unknown in this build
inline int fused_cfg_lookup(const char* e) {
  int n = 0;
  const FusedCfgEntry* t = fused_cfg_table(&n);
  if (!e || !e[0]) return 0;
  for (int i = 1; i < n; ++i)
    if (!strcmp(e, t[i].name)) return i;
  return -1;
}

inline int fused_cfg_env() {
  int& v = fused_cfg_slot();
  if (v < 0) {
    const int k = fused_cfg_lookup(getenv("GS_FUSED_CFG"));
    v = k < 0 ? 0 : k;
  }
  return v;
}

// whether an LDS-ring shape (FCfg::LR, 4-row waves) fits the CU's 160 KiB at depth tl with a
// pf-plane prefetch: the ring (fp32 pf + 2 planes, fp64 pf + 1: FCfg::LRC) plus the tl - 1 levels'
// row exchange (2 slots), with 1 KiB to spare for the small tables
constexpr bool lr_fits(int tl, int pf, int waves = 12, int pair_bytes = 8) {
  return ((pf + (pair_bytes == 16 ? 1 : 2)) * 4 * waves * 64 +
          (tl > 1 ? tl - 1 : 1) * 2 * waves * 2 * 64) * pair_bytes <= 159 * 1024;
}
// the LDS-ring table entries (28 .. 33) as (prefetch, folded); 33 is the fp64 4x8 shape
constexpr int kLrPF[6] = {2, 1, 1, 3, 2, 1};
constexpr bool kLrFold[6] = {false, false, true, false, true, false};
inline bool fused_cfg_is_lr(int i) { return i >= 28 && i <= 33; }
inline bool lr_cfg_fits(int i, int tl) {
  if (!fused_cfg_is_lr(i)) return true;
  return i == 33 ? lr_fits(tl, kLrPF[i - 28], 8, 16) : lr_fits(tl, kLrPF[i - 28]);
}

// one LDS-ring shape: its launch where it fits the LDS at this depth, else false
template <typename T, int TL, bool PER, bool NZ, bool Q32, int PF, bool FOLD>
bool run_lr(const void* s, void* d, const FusedArgs& a, const gs::Params& p, hipStream_t st) {
  if constexpr (sizeof(T) == 4 && lr_fits(TL, PF) && (!FOLD || (Q32 && !PER))) {
    FusedLaunch<FCfg<T, TL, 4, 12, PF, PER, NZ, true, Q32, 0, FOLD, 4>, T>::run(s, d, a, p, st);
    return true;
  } else {
    return false;
  }
}

template <typename T, int TL, bool PER, bool NZ, bool Q32>
void run_fused_cfg(const void* s, void* d, const FusedArgs& a, const gs::Params& p,
                   hipStream_t st) {
  // T = 4: the LDS-ring shapes only (the register ring does not fit 168 VGPRs at this depth);
  // default 4x12:1sl
  if constexpr (TL == 4) {
    if constexpr (sizeof(T) == 4 && !PER && NZ && Q32) {
      switch (a.cfg) {
        case 30: if (run_lr<T, TL, PER, NZ, Q32, 1, true>(s, d, a, p, st)) return; break;
        default: break;
      }
    }
    run_lr<T, TL, PER, NZ, Q32, 1, false>(s, d, a, p, st);
    return;
  } else {
  // tile variants: non-periodic runs with noise and a 32-bit counter (the tuned production
  // path); everything else runs the default shape
  if constexpr (sizeof(T) == 8 && !PER && NZ && Q32) {
    switch (a.cfg) {  // fp64: only shapes that fit the register file without spills
      case 1: FusedLaunch<FCfg<T, TL, 4, 8, 1, PER, NZ>, T>::run(s, d, a, p, st); return;
      case 10: FusedLaunch<FCfg<T, TL, 4, 12, 1, PER, NZ>, T>::run(s, d, a, p, st); return;
      case 15: FusedLaunch<FCfg<T, TL, 4, 6, 2, PER, NZ, true>, T>::run(s, d, a, p, st); return;
      case 16: FusedLaunch<FCfg<T, TL, 4, 6, 2, PER, NZ>, T>::run(s, d, a, p, st); return;
      case 17: FusedLaunch<FCfg<T, TL, 4, 4, 2, PER, NZ>, T>::run(s, d, a, p, st); return;
      case 33:
        if constexpr (lr_fits(TL, 1, 8, 16)) {
          FusedLaunch<FCfg<T, TL, 4, 8, 1, PER, NZ, true, Q32, 0, false, 4>, T>::run(s, d, a, p, st);
          return;
        }
        break;

#ifdef GS_ABLATION
      case 34: FusedLaunch<FCfg<T, TL, 4, 8, 1, PER, NZ, true, true, 0, false, 1>, T>::run(s, d, a, p, st); return;
      case 35: FusedLaunch<FCfg<T, TL, 4, 6, 2, PER, NZ, true, true, 0, false, 1>, T>::run(s, d, a, p, st); return;
      case 36: FusedLaunch<FCfg<T, TL, 4, 8, 1, PER, NZ, false, true, 0, false, 1>, T>::run(s, d, a, p, st); return;
      case 40: FusedLaunch<FCfg<T, TL, 4, 8, 1, PER, NZ, true, true, 0, false, 3>, T>::run(s, d, a, p, st); return;
      case 41: FusedLaunch<FCfg<T, TL, 4, 8, 1, PER, NZ, true, true, 0, false, 2>, T>::run(s, d, a, p, st); return;
      case 49: FusedLaunch<FCfg<T, TL, 4, 8, 1, PER, NZ, true, true, 16>, T>::run(s, d, a, p, st); return;
      case 50: FusedLaunch<FCfg<T, TL, 4, 6, 2, PER, NZ, true, true, 16>, T>::run(s, d, a, p, st); return;
#endif
      default: break;
    }
  }
  if constexpr (sizeof(T) == 4 && !PER && NZ && Q32) {
    switch (a.cfg) {
      case 1: FusedLaunch<FCfg<T, TL, 4, 8, 1, PER, NZ>, T>::run(s, d, a, p, st); return;
      case 2: FusedLaunch<FCfg<T, TL, 4, 8, 2, PER, NZ>, T>::run(s, d, a, p, st); return;
      case 3: FusedLaunch<FCfg<T, TL, 4, 8, 1, PER, NZ, true>, T>::run(s, d, a, p, st); return;
      case 4: FusedLaunch<FCfg<T, TL, 4, 8, 2, PER, NZ, true>, T>::run(s, d, a, p, st); return;
      case 5: FusedLaunch<FCfg<T, TL, 4, 8, 4, PER, NZ, true>, T>::run(s, d, a, p, st); return;
      case 6: FusedLaunch<FCfg<T, TL, 8, 4, 1, PER, NZ>, T>::run(s, d, a, p, st); return;
      case 7: FusedLaunch<FCfg<T, TL, 8, 4, 2, PER, NZ>, T>::run(s, d, a, p, st); return;
      case 8: FusedLaunch<FCfg<T, TL, 8, 4, 1, PER, NZ, true>, T>::run(s, d, a, p, st); return;
      case 9: FusedLaunch<FCfg<T, TL, 8, 4, 4, PER, NZ, true>, T>::run(s, d, a, p, st); return;
      case 10: FusedLaunch<FCfg<T, TL, 4, 12, 1, PER, NZ>, T>::run(s, d, a, p, st); return;
      case 11: FusedLaunch<FCfg<T, TL, 4, 12, 2, PER, NZ>, T>::run(s, d, a, p, st); return;
      case 12: FusedLaunch<FCfg<T, TL, 4, 12, 3, PER, NZ>, T>::run(s, d, a, p, st); return;
      case 13: FusedLaunch<FCfg<T, TL, 4, 12, 1, PER, NZ, true>, T>::run(s, d, a, p, st); return;
      case 15: FusedLaunch<FCfg<T, TL, 4, 6, 2, PER, NZ, true>, T>::run(s, d, a, p, st); return;
      case 18: FusedLaunch<FCfg<T, TL, 4, 16, 1, PER, NZ>, T>::run(s, d, a, p, st); return;
      case 19: FusedLaunch<FCfg<T, TL, 4, 16, 1, PER, NZ, true>, T>::run(s, d, a, p, st); return;
      case 20: if (block_supported(a) && run_block<BCfg<T, TL, 8, 2, 8, NZ>>(s, d, a, p, st)) return; break;
      case 21: if (block_supported(a) && run_block<BCfg<T, TL, 4, 4, 8, NZ>>(s, d, a, p, st)) return; break;
      case 22: if (block_supported(a) && run_block<BCfg<T, TL, 8, 2, 16, NZ>>(s, d, a, p, st)) return; break;
      case 23: if (block_supported(a) && run_block<BCfg<T, TL, 4, 4, 16, NZ>>(s, d, a, p, st)) return; break;
      case 24: if (block_supported(a) && run_block<BCfg<T, TL, 8, 4, 16, NZ>>(s, d, a, p, st)) return; break;
      case 25: if (block_supported(a) && run_block<BCfg<T, TL, 8, 2, 16, NZ, true, true>>(s, d, a, p, st)) return; break;
      case 26: if (block_supported(a) && run_block<BCfg<T, TL, 4, 4, 16, NZ, true, true>>(s, d, a, p, st)) return; break;
      case 27: FusedLaunch<FCfg<T, TL, 4, 12, 1, PER, NZ, true, true, 0, true>, T>::run(s, d, a, p, st); return;
      case 28: if (run_lr<T, TL, PER, NZ, Q32, 2, false>(s, d, a, p, st)) return; break;
      case 29: if (run_lr<T, TL, PER, NZ, Q32, 1, false>(s, d, a, p, st)) return; break;
      case 30: if (run_lr<T, TL, PER, NZ, Q32, 1, true>(s, d, a, p, st)) return; break;
      case 31: if (run_lr<T, TL, PER, NZ, Q32, 3, false>(s, d, a, p, st)) return; break;
      case 32: if (run_lr<T, TL, PER, NZ, Q32, 2, true>(s, d, a, p, st)) return; break;
#ifdef GS_ABLATION
      case 37: FusedLaunch<FCfg<T, TL, 4, 12, 1, PER, NZ, true, true, 0, false, 2>, T>::run(s, d, a, p, st); return;
      case 38: FusedLaunch<FCfg<T, TL, 4, 12, 1, PER, NZ, true, true, 0, true, 2>, T>::run(s, d, a, p, st); return;
      case 39: FusedLaunch<FCfg<T, TL, 4, 12, 2, PER, NZ, true, true, 0, false, 2>, T>::run(s, d, a, p, st); return;
      case 42: FusedLaunch<FCfg<T, TL, 4, 12, 2, PER, NZ, true, true, 1>, T>::run(s, d, a, p, st); return;
      case 43: FusedLaunch<FCfg<T, TL, 4, 12, 2, PER, NZ, true, true, 2>, T>::run(s, d, a, p, st); return;
      case 44: FusedLaunch<FCfg<T, TL, 4, 12, 1, PER, NZ, true, true, 4>, T>::run(s, d, a, p, st); return;
      case 45: FusedLaunch<FCfg<T, TL, 4, 12, 2, PER, NZ, true, true, 4>, T>::run(s, d, a, p, st); return;
      case 46: FusedLaunch<FCfg<T, TL, 4, 12, 1, PER, NZ, true, true, 8>, T>::run(s, d, a, p, st); return;
      case 47: FusedLaunch<FCfg<T, TL, 4, 12, 1, PER, NZ, true, true, 12>, T>::run(s, d, a, p, st); return;
      case 48: FusedLaunch<FCfg<T, TL, 4, 12, 1, PER, NZ, true, true, 16>, T>::run(s, d, a, p, st); return;
      case 49: FusedLaunch<FCfg<T, TL, 4, 8, 1, PER, NZ, true, true, 16>, T>::run(s, d, a, p, st); return;
      case 50: FusedLaunch<FCfg<T, TL, 4, 6, 2, PER, NZ, true, true, 16>, T>::run(s, d, a, p, st); return;
      case 51: FusedLaunch<FCfg<T, TL, 4, 12, 1, PER, NZ, true, true, 32>, T>::run(s, d, a, p, st); return;
      case 52: FusedLaunch<FCfg<T, TL, 4, 12, 2, PER, NZ, true, true, 64>, T>::run(s, d, a, p, st); return;
      case 53: FusedLaunch<FCfg<T, TL, 4, 12, 1, PER, NZ, true, true, 64>, T>::run(s, d, a, p, st); return;
      case 54: FusedLaunch<FCfg<T, TL, 4, 12, 1, PER, NZ, true, Q32, 256>, T>::run(s, d, a, p, st); return;
      case 55: FusedLaunch<FCfg<T, TL, 4, 12, 1, PER, NZ, true, Q32, 512>, T>::run(s, d, a, p, st); return;
      case 56: FusedLaunch<FCfg<T, TL, 4, 12, 1, PER, NZ, true, Q32, 1024>, T>::run(s, d, a, p, st); return;
      case 57: FusedLaunch<FCfg<T, TL, 4, 12, 1, PER, NZ, true, Q32, 1536>, T>::run(s, d, a, p, st); return;
      case 58: FusedLaunch<FCfg<T, TL, 4, 12, 1, PER, NZ, true, Q32, 2048>, T>::run(s, d, a, p, st); return;
      case 59: FusedLaunch<FCfg<T, TL, 4, 12, 1, PER, NZ, true, Q32, 4096>, T>::run(s, d, a, p, st); return;
      case 60: FusedLaunch<FCfg<T, TL, 4, 12, 1, PER, NZ, true, Q32, 6144>, T>::run(s, d, a, p, st); return;
      case 61: FusedLaunch<FCfg<T, TL, 4, 12, 2, PER, NZ, true, Q32, 128>, T>::run(s, d, a, p, st); return;
      case 62: FusedLaunch<FCfg<T, TL, 4, 12, 3, PER, NZ, true, Q32, 128>, T>::run(s, d, a, p, st); return;
#endif
      default: break;  // 0 and 14: the default shape below
    }
  }
  if constexpr (sizeof(T) == 4) {
    FusedLaunch<FCfg<T, TL, 4, 12, 2, PER, NZ, true, Q32>, T>::run(s, d, a, p, st);
  } else {
    FusedLaunch<FCfg<T, TL, 4, 8, 1, PER, NZ, true, Q32>, T>::run(s, d, a, p, st);
  }
  }
}

template <typename T, int TL>
void run_fused_tl(const void* s, void* d, const FusedArgs& a, const gs::Params& p,
                  hipStream_t st) {
  const bool per = a.g.periodic != 0, nz = p.noise != 0.0;
  if (!nz) {
    if (per) run_fused_cfg<T, TL, true, false, true>(s, d, a, p, st);
    else run_fused_cfg<T, TL, false, false, true>(s, d, a, p, st);
  } else if (a.q32) {
    if (per) run_fused_cfg<T, TL, true, true, true>(s, d, a, p, st);
    else run_fused_cfg<T, TL, false, true, true>(s, d, a, p, st);
  } else {
    if (per) run_fused_cfg<T, TL, true, true, false>(s, d, a, p, st);
    else run_fused_cfg<T, TL, false, true, false>(s, d, a, p, st);
  }
}

// resident workgroups per CU of the gated entry that gated_shape_cfg names for depth n (0: none)
template <typename T>
int fused_gated_occupancy(int cfg, int n, bool pairs) {
  auto one = [&](auto tl) -> int {
    constexpr int TL = decltype(tl)::value;
    if constexpr (sizeof(T) == 8) {
      return FusedLaunch<FCfg<T, TL, 4, 8, 1, false, true, true, true>, T>::gated_occupancy(pairs);
    } else {
      if (cfg == fused_cfg_lookup("4x12:1sf"))
        return FusedLaunch<FCfg<T, TL, 4, 12, 1, false, true, true, true, 0, true>, T>::gated_occupancy(pairs);
      return FusedLaunch<FCfg<T, TL, 4, 12, 1, false, true, true>, T>::gated_occupancy(pairs);
    }
  };
  if (n == 2) return one(std::integral_constant<int, 2>{});
  if (n == 3) return one(std::integral_constant<int, 3>{});
  return 0;
}

// depths 2..3 on every path; 4 (fp32 only: the LDS-ring shapes) where max_n allows it -- whole-
// interior launches; the overlapped pass's shell kernels (slab.hpp) stop at 3
inline bool fused_supported(const Geom& g, int n, int max_n = 3) {
  if (n < 2 || n > max_n || n > 4 || g.H < n) return false;
  return !(g.periodic && (g.Ly % 4 != 0));  // noise quads would straddle the wrap
}

// whether the Philox counter q = gx + Lx * (gy4 + Ly4 * gz) of every cell fits 32 bits
inline bool philox_q32(const Geom& g) {
  const uint64_t Ly4 = ((uint64_t)g.Ly + 3) >> 2;
  return (uint64_t)g.Lx * Ly4 * (uint64_t)g.Lz <= 0xFFFFFFFFull;
}

// cfg / sched < 0: the process-wide selection (GS_FUSED_CFG / GS_FUSED_SCHED or the
// gs_fused_select / gs_fused_sched APIs).
// a gated pass's launch (sched 3): the unit table and transport state (gate.hpp)
struct GateLaunch {
  const GateUnit* units;
  int32_t nunits;
  const GateArgs* gate;
  uint64_t n;
  uint32_t cnt;
  int32_t npk;
  int32_t pairs;  // the table holds two entries per workgroup
  int32_t pre;    // FusedArgs::gate_pre (carried exchanges)
  uint32_t cnt2;  // the carried exchange's arrival count (pre bit 1)
};

// The tile grid a configuration's launch enumerates (FusedLaunch::run + fold_strip), on the host:
// the gated pass's unit table names tiles by this enumeration (gs/gate_plan.h)
using TileGrid = gs::TileGrid;
using gs::tile_window;
// the configuration run_fused_cfg actually launches for table entry cfg (variants exist for the
// non-periodic, noisy, 32-bit-counter production path only; everything else runs the default)
inline const char* fused_shape_name(int cfg, bool f64, bool variants) {
  int nt = 0;
  const FusedCfgEntry* tab = fused_cfg_table(&nt);
  const char* dflt = f64 ? "4x8:1s" : "4x12:2s";
  if (!variants || cfg <= 0 || cfg >= nt || fused_cfg_is_block(cfg)) return dflt;
  if (!(f64 ? tab[cfg].f64 : tab[cfg].f32)) return dflt;
  return tab[cfg].name;
}
// the configuration a gated pass launches (FCfg::GATE_OK shapes only): fp32 the folded 4x12:1sf
// where the last x strip folds, else 4x12:1s; fp64 the default 4x8:1s
inline int gated_shape_cfg(bool f64, const Geom& g, int n) {
  if (f64) return 0;
  const int k = fused_cfg_lookup("4x12:1sf");
  return fused_cfg_applies(k, g, n) ? k : fused_cfg_lookup("4x12:1s");
}
inline TileGrid fused_tile_grid(const char* name, const Geom& g, int n) {
  const int rows = atoi(name);
  const char* xp = strchr(name, 'x');
  const int waves = xp ? atoi(xp + 1) : 12;
  const char* colon = strchr(name, ':');
  return gs::tile_grid(rows, waves, colon && strchr(colon, 'f'), g, n);
}

template <typename T>
bool launch_fused(const typename Vec2<T>::type* s, typename Vec2<T>::type* d, const Geom& g,
                  const gs::Params& p, int n, int64_t t, hipStream_t st, int cfg = -1,
                  int sched = -1, int zlo0 = 0, int zlen0 = -1, int zlo1 = 0, int zlen1 = 0,
                  int reserve = 0, int mask = 0, bool allow_block = false,
                  const GateLaunch* gate = nullptr) {
  if (!fused_supported(g, n, sizeof(T) == 4 ? 4 : 3)) return false;
  if (n == 4 && (zlo0 != 0 || (zlen0 >= 0 && zlen0 != g.nz) || zlen1 > 0 || mask || gate))
    return false;  // T = 4: whole-interior launches only
  FusedArgs a{};
  a.allow_block = allow_block ? 1 : 0;
  if (zlen0 < 0) zlen0 = g.nz;
  if (zlen1 <= 0) zlen1 = 0;
  if (zlen0 <= 0 || zlo0 < 0 || zlo0 + zlen0 > g.nz || (zlen1 && (zlo1 < 0 || zlo1 + zlen1 > g.nz)))
    return false;
  // one storage plane must fit a buffer descriptor's 32-bit range
  if (gs::plane_elems(g) * (int64_t)sizeof(typename Vec2<T>::type) > 0x7ffffff0LL) return false;
  a.zlo[0] = zlo0; a.zlen[0] = zlen0;
  a.zlo[1] = zlo1; a.zlen[1] = zlen1;
  a.nzv = zlen0 + zlen1;
  a.reserve = reserve > 0 ? reserve : 0;
  // mask bit0/1/2/3: leave the n cells next to the -x/+x/-y/+y face unwritten (overlap)
  a.mx0 = (mask & 1) ? n : 0;
  a.mx1 = (mask & 2) ? g.nx - n : g.nx;
  a.my0 = (mask & 4) ? n : 0;
  a.my1 = (mask & 8) ? g.ny - n : g.ny;
  if (a.mx1 <= a.mx0 || a.my1 <= a.my0) return false;
  a.g = g;
  a.t = t;
  // debug knob philox_generic (gs/debug.h) forces the 64-bit-counter Philox path (tests: both
  // paths agree bitwise)
  a.q32 = (philox_q32(g) && !gs::debug_knobs().philox_generic) ? 1 : 0;
  a.cfg = cfg >= 0 ? cfg : fused_cfg_env();
  a.sched = sched >= 0 ? sched : fused_sched_slot();
  if (zlen1) a.sched = 0;  // two short runs: one workgroup per (tile, run)
  if (gate) {
    if (zlo0 != 0 || zlen0 != g.nz || zlen1 || mask || !gate->units || gate->nunits < 1) return false;
    a.sched = 3;
    a.gunits = gate->units;
    a.ngunits = gate->nunits;
    a.gate = gate->gate;
    a.field = const_cast<typename Vec2<T>::type*>(s);
    a.gate_n = gate->n;
    a.gate_cnt = gate->cnt;
    a.gate_npk = gate->npk;
    a.gate_pairs = gate->pairs ? 1 : 0;
    a.gate_pre = gate->pre;
    a.gate_cnt2 = gate->cnt2;
    if (a.gate_pairs && (gate->nunits & 1)) return false;
    if (a.gate_pairs && gate->pre) return false;  // carried exchanges: one-unit tables only
    a.allow_block = 0;
  } else if (a.sched == 3) {
    a.sched = 2;  // the gated schedule needs its table
  }
  a.bcfix = g.periodic ? 0 : 1;
  if (n == 2) run_fused_tl<T, 2>(s, d, a, p, st);
  else if (n == 3) run_fused_tl<T, 3>(s, d, a, p, st);
  else if constexpr (sizeof(T) == 4) run_fused_tl<T, 4>(s, d, a, p, st);
  return true;
}
