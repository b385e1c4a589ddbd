// SPDX-License-Identifier: MIT
// CPU backend: OpenMP implementation of every backend op.  It is both the `backend = "CPU"`
// solver (reference: Simulation_CPU.jl:14-133, Threads.@threads over z) and the golden
// model the gfx950 kernels are tested against.  Same Philox noise stream as the GPU.
#include <emmintrin.h>
#if defined(__x86_64__)
#include <immintrin.h>
#endif
#include <omp.h>
#include <string.h>

#include <algorithm>
#include <stdexcept>

#include "gs/capi_impl.h"

namespace {

using gs::Box;
using gs::Geom;

// Philox4x32-10 blocks of counters (q_i, q_i >> 32, step, step >> 32), key `seed`, for a row of
// cells (the noise cache of CpuBackend::step).  The AVX2 form runs eight counters per vector:
// _mm256_mul_epu32 gives the 32x32 -> 64-bit products of the even 32-bit lanes, the odd lanes
// go through a 64-bit shift, and blends reassemble the products' low / high words.  Integer
// arithmetic only, so it equals gs::philox4x32_10 bit for bit (tests/test_noise.py checks);
// chosen at run time when the CPU has AVX2 (the library is built for baseline x86-64).
void noise_blocks_scalar(const uint64_t* q, int n, uint64_t step, uint64_t seed, gs::U4* out) {
  for (int i = 0; i < n; ++i)
    out[i] = gs::philox4x32_10((uint32_t)q[i], (uint32_t)(q[i] >> 32), (uint32_t)step,
                               (uint32_t)(step >> 32), seed);
}

#if defined(__x86_64__)
__attribute__((target("avx2"))) void noise_blocks_avx2(const uint64_t* q, int n, uint64_t step,
                                                       uint64_t seed, gs::U4* out) {
  const __m256i m0 = _mm256_set1_epi32((int)0xD2511F53u), m1 = _mm256_set1_epi32((int)0xCD9E8D57u);
  int i = 0;
  for (; i + 8 <= n; i += 8) {
    alignas(32) uint32_t lo[8], hi[8];
    for (int k = 0; k < 8; ++k) {
      lo[k] = (uint32_t)q[i + k];
      hi[k] = (uint32_t)(q[i + k] >> 32);
    }
    __m256i c0 = _mm256_load_si256((const __m256i*)lo), c1 = _mm256_load_si256((const __m256i*)hi);
    __m256i c2 = _mm256_set1_epi32((int)(uint32_t)step), c3 = _mm256_set1_epi32((int)(uint32_t)(step >> 32));
    uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
    for (int r = 0; r < 10; ++r) {
      const __m256i e0 = _mm256_mul_epu32(c0, m0), o0 = _mm256_mul_epu32(_mm256_srli_epi64(c0, 32), m0);
      const __m256i e1 = _mm256_mul_epu32(c2, m1), o1 = _mm256_mul_epu32(_mm256_srli_epi64(c2, 32), m1);
      const __m256i lo0 = _mm256_blend_epi32(e0, _mm256_slli_epi64(o0, 32), 0xAA);
      const __m256i hi0 = _mm256_blend_epi32(_mm256_srli_epi64(e0, 32), o0, 0xAA);
      const __m256i lo1 = _mm256_blend_epi32(e1, _mm256_slli_epi64(o1, 32), 0xAA);
      const __m256i hi1 = _mm256_blend_epi32(_mm256_srli_epi64(e1, 32), o1, 0xAA);
      const __m256i n0 = _mm256_xor_si256(_mm256_xor_si256(hi1, c1), _mm256_set1_epi32((int)k0));
      const __m256i n2 = _mm256_xor_si256(_mm256_xor_si256(hi0, c3), _mm256_set1_epi32((int)k1));
      c0 = n0;
      c1 = lo1;
      c2 = n2;
      c3 = lo0;
      k0 += 0x9E3779B9u;
      k1 += 0xBB67AE85u;
    }
    alignas(32) uint32_t w[4][8];
    _mm256_store_si256((__m256i*)w[0], c0);
    _mm256_store_si256((__m256i*)w[1], c1);
    _mm256_store_si256((__m256i*)w[2], c2);
    _mm256_store_si256((__m256i*)w[3], c3);
    for (int k = 0; k < 8; ++k) out[i + k] = gs::U4{w[0][k], w[1][k], w[2][k], w[3][k]};
  }
  noise_blocks_scalar(q + i, n - i, step, seed, out + i);
}
#endif

// 1: the AVX2 form, 0: scalar (gs_noise_blocks' `impl`, -1: the one the step uses)
bool cpu_has_avx2() {
#if defined(__x86_64__)
  static const bool yes = __builtin_cpu_supports("avx2");
  return yes;
#else
  return false;
#endif
}

void noise_blocks(const uint64_t* q, int n, uint64_t step, uint64_t seed, gs::U4* out, int impl = -1) {
#if defined(__x86_64__)
  if (impl == 1 || (impl < 0 && cpu_has_avx2())) {
    noise_blocks_avx2(q, n, step, seed, out);
    return;
  }
#endif
  (void)impl;
  noise_blocks_scalar(q, n, step, seed, out);
}

// One row of fp32 cell updates, two cells (u0 v0 u1 v1) per SSE2 vector.  The operations and
// their order are those of gs::gs_update on each cell -- plain IEEE adds and multiplies (no FMA:
// x86-64's baseline has none), so the result is bit-identical to the scalar loop below, which
// also handles the last odd cell and fp64.  i: float index of the row's first cell, n: cells,
// r: the cells' noise draws (or null).
inline void row_update_f32(const float* s, float* d, int64_t i, int n, int64_t sy, int64_t sz,
                           const gs::Coef<float>& c, const float* r) {
  const __m128 k6 = _mm_setr_ps(c.Du6, c.Dv6, c.Du6, c.Dv6);
  const __m128 kd = _mm_setr_ps(c.Du, c.Dv, c.Du, c.Dv);
  const __m128 sg = _mm_setr_ps(-1.f, 1.f, -1.f, 1.f);
  const __m128 kf = _mm_setr_ps(c.F, -c.Fk, c.F, -c.Fk);  // u: F * (1 - u), v: -(Fk * v)
  const __m128 kn = _mm_set1_ps(c.noise);
  const __m128 dt = _mm_set1_ps(c.dt);
  const __m128 one = _mm_set1_ps(1.f);
  const __m128 um = _mm_castsi128_ps(_mm_setr_epi32(-1, 0, -1, 0));  // u lanes
  int x = 0;
  for (; x + 2 <= n; x += 2, i += 4) {
    const __m128 cc = _mm_loadu_ps(s + i);
    const __m128 sum = _mm_add_ps(
        _mm_add_ps(_mm_add_ps(_mm_loadu_ps(s + i - 2), _mm_loadu_ps(s + i + 2)),
                   _mm_add_ps(_mm_loadu_ps(s + i - sy), _mm_loadu_ps(s + i + sy))),
        _mm_add_ps(_mm_loadu_ps(s + i - sz), _mm_loadu_ps(s + i + sz)));
    const __m128 uu = _mm_shuffle_ps(cc, cc, _MM_SHUFFLE(2, 2, 0, 0));
    const __m128 vv = _mm_shuffle_ps(cc, cc, _MM_SHUFFLE(3, 3, 1, 1));
    const __m128 uvv = _mm_mul_ps(_mm_mul_ps(uu, vv), vv);
    __m128 dd = _mm_sub_ps(_mm_mul_ps(k6, sum), _mm_mul_ps(kd, cc));
    dd = _mm_add_ps(dd, _mm_mul_ps(sg, uvv));
    const __m128 pf = _mm_or_ps(_mm_and_ps(um, _mm_sub_ps(one, cc)), _mm_andnot_ps(um, cc));
    dd = _mm_add_ps(dd, _mm_mul_ps(kf, pf));
    // the u lanes add noise * r (noise * 0 without a draw, as gs_update does); v lanes keep dd
    const __m128 rr = r ? _mm_setr_ps(r[x], 0.f, r[x + 1], 0.f) : _mm_setzero_ps();
    const __m128 dn = _mm_add_ps(dd, _mm_mul_ps(kn, rr));
    dd = _mm_or_ps(_mm_and_ps(um, dn), _mm_andnot_ps(um, dd));
    _mm_storeu_ps(d + i, _mm_add_ps(cc, _mm_mul_ps(dd, dt)));
  }
  for (; x < n; ++x, i += 2) {
    const float u = s[i], v = s[i + 1];
    const float su = (s[i - 2] + s[i + 2]) + (s[i - sy] + s[i + sy]) + (s[i - sz] + s[i + sz]);
    const float sv = (s[i - 1] + s[i + 3]) + (s[i - sy + 1] + s[i + sy + 1]) +
                     (s[i - sz + 1] + s[i + sz + 1]);
    float uo, vo;
    gs::gs_update<float>(c, u, v, su, sv, r ? r[x] : 0.f, uo, vo);
    d[i] = uo;
    d[i + 1] = vo;
  }
}

template <typename T>
class CpuBackend final : public gs::Backend {
 public:
  CpuBackend(const Geom& g, const gs::Params& p, void* b0, void* b1, void* send, void* recv)
      : g_(g), p_(p) {
    buf_[0] = (T*)b0;
    buf_[1] = (T*)b1;
    send_ = (T*)send;
    recv_ = (T*)recv;
    if (!b0 || !b1) throw std::runtime_error("null field buffer");
  }

  void fill_box(int b, const Box& bx, double u, double v) override {
    T* d = buf_[b];
    const T uu = (T)u, vv = (T)v;
#pragma omp parallel for collapse(2) schedule(static)
    for (int z = bx.z0; z < bx.z0 + bx.nz; ++z)
      for (int y = bx.y0; y < bx.y0 + bx.ny; ++y) {
        T* row = d + 2 * gs::lin(g_, 0, y, z);
        for (int x = bx.x0; x < bx.x0 + bx.nx; ++x) {
          row[2 * x] = uu;
          row[2 * x + 1] = vv;
        }
      }
  }

  void seed(int b) override {
    // global cube [L/2-6, L/2+6]^3 (0-based, inclusive), clipped to this rank.
    // The reference only defines it for a cubic domain; use each axis' own extent.
    T* d = buf_[b];
    int64_t lo[3], hi[3];
    const int64_t L[3] = {g_.Lx, g_.Ly, g_.Lz};
    const int64_t o[3] = {g_.ox, g_.oy, g_.oz};
    const int n[3] = {g_.nx, g_.ny, g_.nz};
    for (int a = 0; a < 3; ++a) {
      const int64_t mn = L[a] / 2 - 6, mx = L[a] / 2 + 6;
      lo[a] = std::max<int64_t>(mn, o[a]) - o[a];
      hi[a] = std::min<int64_t>(mx + 1, o[a] + n[a]) - o[a];
    }
    for (int64_t z = lo[2]; z < hi[2]; ++z)
      for (int64_t y = lo[1]; y < hi[1]; ++y)
        for (int64_t x = lo[0]; x < hi[0]; ++x) {
          T* c = d + 2 * gs::lin(g_, (int)x, (int)y, (int)z);
          c[0] = (T)0.25;
          c[1] = (T)0.33;
        }
  }

  void step(int src, int dst, const Box& R, int64_t t) override {
    const T* s = buf_[src];
    T* d = buf_[dst];
    const gs::Coef<T> c = gs::make_coef<T>(p_);
    const bool noise = p_.noise != 0.0;
    const int64_t sx = 2, sy = 2 * (int64_t)g_.px, sz = 2 * gs::plane_elems(g_);
    const Geom g = g_;
    const uint64_t seed = p_.seed;
#pragma omp parallel
    {
      // fp32: denormals flushed to zero in this solver's arithmetic (MXCSR FTZ + DAZ, restored
      // after the region: the calling thread's numpy keeps IEEE behaviour).  The reference
      // example's v field passes through denormals (~30k cells at step 60 of the L=64 run),
      // which x86 handles in microcode at ~100x the cost; the values involved are below
      // 1.2e-38.  A deliberate deviation (docs/PARITY.md): the reference and the GPU keep IEEE
      // denormals; debug knob cpu_ftz = 0 restores them here too.  fp64 never flushes.
      const unsigned csr = _mm_getcsr();
      if (sizeof(T) == 4 && gs::debug_knobs().cpu_ftz) _mm_setcsr(csr | 0x8040u);
      gs::U4* cache = new gs::U4[R.nx > 0 ? R.nx : 1];
      uint64_t* qrow = new uint64_t[R.nx > 0 ? R.nx : 1];
      float* rrow = new float[R.nx > 0 ? R.nx : 1];
#pragma omp for schedule(static)
      for (int z = R.z0; z < R.z0 + R.nz; ++z) {
        int64_t gz = g.oz + z;
        if (gz < 0) gz += g.Lz; else if (gz >= g.Lz) gz -= g.Lz;
        for (int y = R.y0; y < R.y0 + R.ny; ++y) {
          int64_t gy = g.oy + y;
          if (gy < 0) gy += g.Ly; else if (gy >= g.Ly) gy -= g.Ly;
          if (noise && (y == R.y0 || (gy & 3) == 0)) {
            // gs::noise_block's counters for the row, then the blocks eight at a time
            const uint64_t Ly4 = ((uint64_t)g.Ly + 3) >> 2;
            const uint64_t qy = (uint64_t)g.Lx * ((uint64_t)(gy >> 2) + Ly4 * (uint64_t)gz);
            for (int x = R.x0; x < R.x0 + R.nx; ++x) {
              int64_t gx = g.ox + x;
              if (gx < 0) gx += g.Lx; else if (gx >= g.Lx) gx -= g.Lx;
              qrow[x - R.x0] = (uint64_t)gx + qy;
            }
            noise_blocks(qrow, R.nx, (uint64_t)t, seed, cache);
          }
          const int64_t base = 2 * gs::lin(g, 0, y, z);
          if constexpr (sizeof(T) == 4) {
            if (noise)
              for (int x = 0; x < R.nx; ++x)
                rrow[x] = gs::uniform_pm1<float>(gs::u4_get(cache[x], (int)(gy & 3)));
            row_update_f32(s, d, base + 2 * (int64_t)R.x0, R.nx, sy, sz, c,
                           noise ? rrow : nullptr);
            continue;
          }
          for (int x = R.x0; x < R.x0 + R.nx; ++x) {
            const int64_t i = base + 2 * (int64_t)x;
            const T u = s[i], v = s[i + 1];
            const T su = (s[i - sx] + s[i + sx]) + (s[i - sy] + s[i + sy]) + (s[i - sz] + s[i + sz]);
            const T sv = (s[i - sx + 1] + s[i + sx + 1]) + (s[i - sy + 1] + s[i + sy + 1]) +
                         (s[i - sz + 1] + s[i + sz + 1]);
            T r = (T)0;
            if (noise) r = gs::uniform_pm1<T>(gs::u4_get(cache[x - R.x0], (int)(gy & 3)));
            T uo, vo;
            gs::gs_update<T>(c, u, v, su, sv, r, uo, vo);
            d[i] = uo;
            d[i + 1] = vo;
          }
        }
      }
      delete[] cache;
      delete[] qrow;
      delete[] rrow;
      _mm_setcsr(csr);
    }
  }

  template <bool PACK>
  void pack_impl(int b, const gs::HaloMsg* msgs, int n, T* pk) {
    T* f = buf_[b];
    for (int m = 0; m < n; ++m) {
      const Box& bx = msgs[m].box;
      T* out = pk + 2 * msgs[m].offset;
#pragma omp parallel for collapse(2) schedule(static)
      for (int z = 0; z < bx.nz; ++z)
        for (int y = 0; y < bx.ny; ++y) {
          T* row = f + 2 * gs::lin(g_, bx.x0, bx.y0 + y, bx.z0 + z);
          T* p = out + 2 * ((int64_t)z * bx.ny + y) * bx.nx;
          if (PACK) memcpy(p, row, sizeof(T) * 2 * bx.nx);
          else memcpy(row, p, sizeof(T) * 2 * bx.nx);
        }
    }
  }
  void pack(int b, const gs::HaloPlan& p) override { pack_impl<true>(b, p.send, p.nsend, send_); }
  void unpack(int b, const gs::HaloPlan& p) override { pack_impl<false>(b, p.recv, p.nrecv, recv_); }
  void self_copy(int64_t so, int64_t d, int64_t n) override {
    memcpy(recv_ + 2 * d, send_ + 2 * so, sizeof(T) * 2 * n);
  }

  void extract(int b, void* uo, void* vo) override {
    const T* f = buf_[b];
    T* u = (T*)uo;
    T* v = (T*)vo;
#pragma omp parallel for collapse(2) schedule(static)
    for (int z = 0; z < g_.nz; ++z)
      for (int y = 0; y < g_.ny; ++y) {
        const T* row = f + 2 * gs::lin(g_, 0, y, z);
        const int64_t o = ((int64_t)z * g_.ny + y) * g_.nx;
        for (int x = 0; x < g_.nx; ++x) {
          if (u) u[o + x] = row[2 * x];
          if (v) v[o + x] = row[2 * x + 1];
        }
      }
  }

  void randomize(int b, uint64_t seed, double lo, double hi) override {
    T* f = buf_[b];
    const Geom g = g_;
#pragma omp parallel for collapse(2) schedule(static)
    for (int z = 0; z < g.nz; ++z)
      for (int y = 0; y < g.ny; ++y) {
        T* row = f + 2 * gs::lin(g, 0, y, z);
        for (int x = 0; x < g.nx; ++x) {
          double u, v;
          gs::random_init_cell(g.ox + x, g.oy + y, g.oz + z, g.Lx, g.Ly, seed, lo, hi, &u, &v);
          row[2 * x] = (T)u;
          row[2 * x + 1] = (T)v;
        }
      }
  }

  void insert(int b, const void* ui, const void* vi) override {
    T* f = buf_[b];
    const T* u = (const T*)ui;
    const T* v = (const T*)vi;
#pragma omp parallel for collapse(2) schedule(static)
    for (int z = 0; z < g_.nz; ++z)
      for (int y = 0; y < g_.ny; ++y) {
        T* row = f + 2 * gs::lin(g_, 0, y, z);
        const int64_t o = ((int64_t)z * g_.ny + y) * g_.nx;
        for (int x = 0; x < g_.nx; ++x) {
          row[2 * x] = u[o + x];
          row[2 * x + 1] = v[o + x];
        }
      }
  }

  void stats(int b, double* out) override {
    const T* f = buf_[b];
    double su = 0, sv = 0, mnu = 1e300, mxu = -1e300, mnv = 1e300, mxv = -1e300;
#pragma omp parallel for collapse(2) reduction(+ : su, sv) reduction(min : mnu, mnv) \
    reduction(max : mxu, mxv) schedule(static)
    for (int z = 0; z < g_.nz; ++z)
      for (int y = 0; y < g_.ny; ++y) {
        const T* row = f + 2 * gs::lin(g_, 0, y, z);
        for (int x = 0; x < g_.nx; ++x) {
          const double u = row[2 * x], v = row[2 * x + 1];
          su += u; sv += v;
          mnu = std::min(mnu, u); mxu = std::max(mxu, u);
          mnv = std::min(mnv, v); mxv = std::max(mxv, v);
        }
      }
    out[0] = su; out[1] = mnu; out[2] = mxu; out[3] = sv; out[4] = mnv; out[5] = mxv;
  }

 private:
  Geom g_;
  gs::Params p_;
  T* buf_[2];
  T* send_;
  T* recv_;
};

}  // namespace

gs::Backend* gs_make_backend(int32_t dtype, const gs::Geom& g, const gs::Params& p, void* b0,
                             void* b1, void* send, void* recv, void* stream) {
  (void)stream;
  if (dtype == gs::kF32) return new CpuBackend<float>(g, p, b0, b1, send, recv);
  if (dtype == gs::kF64) return new CpuBackend<double>(g, p, b0, b1, send, recv);
  throw std::runtime_error("unsupported dtype");
}

// Philox blocks of counters q[0, n) (gs::noise_block's (q, step, seed) stream) into out (4 words
// each): impl 0 scalar, 1 AVX2 (-1 when the CPU lacks it), -1 the form the CPU step uses.
extern "C" int gs_noise_blocks(const uint64_t* q, int32_t n, uint64_t step, uint64_t seed,
                               uint32_t* out, int32_t impl) {
  if (impl == 1 && !cpu_has_avx2()) return -1;
  noise_blocks(q, n, step, seed, reinterpret_cast<gs::U4*>(out), impl);
  return 0;
}

// OpenMP threads of the CPU backend in this process: n > 0 sets them, any n returns the
// current maximum (bench.py's golden check gives each of N ranks on a node cores / N threads)
extern "C" int gs_cpu_threads(int32_t n) {
#ifdef _OPENMP
  if (n > 0) omp_set_num_threads(n);
  return omp_get_max_threads();
#else
  (void)n;
  return 1;  // (the ThreadSanitizer self-test build has no OpenMP)
#endif
}
