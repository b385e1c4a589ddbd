"""Independent pure-Python (numpy + PyTorch) golden model.

Used only as a test oracle: the native CPU backend and the gfx950 kernels are checked against
it.  It re-implements, without sharing code with ``csrc/``:
  * the Philox4x32-10 noise stream (rocrand_philox4x32_10.h semantics, counter mode,
    one block per 4 consecutive y-rows: q = gx + Lx*((gy>>2) + ceil(Ly/4)*gz), word gy&3)
  * the reference initial condition (Simulation_CPU.jl:14-65)
  * one explicit Euler step of the Gray-Scott system (Simulation_CPU.jl:77-113, Common.jl:13-18)
  * the reference boundary behaviour: outer u ghost = 1 at even t, 0 at odd t.
Arrays are C-ordered (z, y, x), i.e. the same memory order as the Julia (x, y, z) arrays.
"""
from __future__ import annotations

from typing import Optional, Sequence, Tuple

import numpy as np

M0 = np.uint64(0xD2511F53)
M1 = np.uint64(0xCD9E8D57)
W0 = 0x9E3779B9
W1 = 0xBB67AE85
MASK32 = np.uint64(0xFFFFFFFF)


def philox4x32_10(c0, c1, c2, c3, seed: int):
    """Vectorised Philox4x32-10 on uint32 counters; returns 4 uint32 arrays."""
    c0 = np.asarray(c0, dtype=np.uint64) & MASK32
    c1 = np.asarray(c1, dtype=np.uint64) & MASK32
    c2 = np.asarray(c2, dtype=np.uint64) & MASK32
    c3 = np.asarray(c3, dtype=np.uint64) & MASK32
    k0 = seed & 0xFFFFFFFF
    k1 = (seed >> 32) & 0xFFFFFFFF
    for _ in range(10):
        p0 = M0 * c0
        p1 = M1 * c2
        hi0, lo0 = p0 >> np.uint64(32), p0 & MASK32
        hi1, lo1 = p1 >> np.uint64(32), p1 & MASK32
        n0 = hi1 ^ c1 ^ np.uint64(k0)
        n2 = hi0 ^ c3 ^ np.uint64(k1)
        c0, c1, c2, c3 = n0, lo1, n2, lo0
        k0 = (k0 + W0) & 0xFFFFFFFF
        k1 = (k1 + W1) & 0xFFFFFFFF
    return (c0.astype(np.uint32), c1.astype(np.uint32), c2.astype(np.uint32), c3.astype(np.uint32))


def noise(L: Sequence[int], offsets: Sequence[int], sizes: Sequence[int], step: int,
          seed: int, dtype=np.float64) -> np.ndarray:
    """Uniform[-1,1) draws for the cells of a sub-domain at ``step`` -> (nz, ny, nx)."""
    Lx, Ly, _ = (int(v) for v in L)
    Ly4 = (Ly + 3) // 4
    nx, ny, nz = (int(v) for v in sizes)
    gx = np.arange(offsets[0], offsets[0] + nx, dtype=np.uint64)
    gy = np.arange(offsets[1], offsets[1] + ny, dtype=np.uint64)
    gz = np.arange(offsets[2], offsets[2] + nz, dtype=np.uint64)
    Z, Y, X = np.meshgrid(gz, gy, gx, indexing="ij")
    q = X + np.uint64(Lx) * ((Y >> np.uint64(2)) + np.uint64(Ly4) * Z)
    st = np.uint64(step)
    r = philox4x32_10(q & MASK32, q >> np.uint64(32), st & MASK32, st >> np.uint64(32), seed)
    sel = (Y & np.uint64(3)).astype(np.int64)
    words = np.choose(sel, r)
    dt = np.dtype(dtype).type
    return words.view(np.int32).astype(dt) * dt(2.0 ** -31)


def init_fields(L: Sequence[int], offsets=(0, 0, 0), sizes=None, dtype=np.float64):
    """Interior of u, v after the reference init (13^3 seed cube at L/2 +- 6)."""
    L = [int(v) for v in L]
    sizes = list(sizes) if sizes is not None else list(L)
    u = np.ones((sizes[2], sizes[1], sizes[0]), dtype=dtype)
    v = np.zeros_like(u)
    sl = []
    for a in (2, 1, 0):
        lo = max(L[a] // 2 - 6, offsets[a]) - offsets[a]
        hi = min(L[a] // 2 + 7, offsets[a] + sizes[a]) - offsets[a]
        sl.append(slice(max(lo, 0), max(hi, 0)))
    u[tuple(sl)] = 0.25
    v[tuple(sl)] = 0.33
    return u, v


def random_fields(L: Sequence[int], offsets=(0, 0, 0), sizes=None, seed: int = 0,
                  lo: float = 0.0, hi: float = 1.0, dtype=np.float64):
    """The benchmarks' random initial interior (gs::random_init_cell): a function of the
    global cell only.  (w0, w1) = Philox4x32-10({q, q >> 32, ~0, ~0}, seed) with
    q = gx + Lx * (gy + Ly * gz); u = lo + (hi - lo) * (w0 >> 8) * 2^-24, v from w1."""
    L = [int(v) for v in L]
    sizes = list(sizes) if sizes is not None else list(L)
    gx = np.arange(offsets[0], offsets[0] + sizes[0], dtype=np.uint64)
    gy = np.arange(offsets[1], offsets[1] + sizes[1], dtype=np.uint64)
    gz = np.arange(offsets[2], offsets[2] + sizes[2], dtype=np.uint64)
    Z, Y, X = np.meshgrid(gz, gy, gx, indexing="ij")
    q = X + np.uint64(L[0]) * (Y + np.uint64(L[1]) * Z)
    full = np.full(q.shape, 0xFFFFFFFF, dtype=np.uint64)
    w0, w1, _, _ = philox4x32_10(q & MASK32, q >> np.uint64(32), full, full, seed)
    s = 2.0 ** -24
    u = (hi - lo) * ((w0 >> np.uint32(8)).astype(np.float64) * s) + lo
    v = (hi - lo) * ((w1 >> np.uint32(8)).astype(np.float64) * s) + lo
    return u.astype(dtype), v.astype(dtype)


def bc_u(t: int) -> float:
    return 0.0 if (t & 1) else 1.0


def step(u: np.ndarray, v: np.ndarray, t: int, F: float, k: float, dt: float, Du: float,
         Dv: float, noise_amp: float, seed: int, periodic: bool = False, backend: str = "numpy"):
    """One global step (single rank, whole domain) of the reference update at time ``t``."""
    L = (u.shape[2], u.shape[1], u.shape[0])
    if backend == "torch":
        return _step_torch(u, v, t, F, k, dt, Du, Dv, noise_amp, seed, periodic, L)
    dtype = u.dtype.type
    if periodic:
        up = np.pad(u, 1, mode="wrap")
        vp = np.pad(v, 1, mode="wrap")
    else:
        up = np.pad(u, 1, mode="constant", constant_values=bc_u(t))
        vp = np.pad(v, 1, mode="constant", constant_values=0.0)

    def nsum(a):
        return (a[1:-1, 1:-1, :-2] + a[1:-1, 1:-1, 2:]) + (a[1:-1, :-2, 1:-1] + a[1:-1, 2:, 1:-1]) + \
            (a[:-2, 1:-1, 1:-1] + a[2:, 1:-1, 1:-1])

    su, sv = nsum(up), nsum(vp)
    r = noise(L, (0, 0, 0), L, t, seed, dtype=u.dtype) if noise_amp != 0 else 0.0
    uvv = u * v * v
    du = dtype(Du / 6.0) * su - dtype(Du) * u - uvv + dtype(F) * (dtype(1) - u) + dtype(noise_amp) * r
    dv = dtype(Dv / 6.0) * sv - dtype(Dv) * v + uvv - dtype(F + k) * v
    return (u + du * dtype(dt)).astype(u.dtype), (v + dv * dtype(dt)).astype(v.dtype)


def _step_torch(u, v, t, F, k, dt, Du, Dv, noise_amp, seed, periodic, L):
    """Same update with a torch conv3d Laplacian (the "plain PyTorch reference")."""
    import torch
    import torch.nn.functional as Fn

    tu = torch.as_tensor(u)
    tv = torch.as_tensor(v)
    dtype = tu.dtype
    kern = torch.zeros((1, 1, 3, 3, 3), dtype=dtype, device=tu.device)
    for (a, b, c) in ((0, 1, 1), (2, 1, 1), (1, 0, 1), (1, 2, 1), (1, 1, 0), (1, 1, 2)):
        kern[0, 0, a, b, c] = 1.0
    if periodic:
        pu = Fn.pad(tu[None, None], (1, 1, 1, 1, 1, 1), mode="circular")
        pv = Fn.pad(tv[None, None], (1, 1, 1, 1, 1, 1), mode="circular")
    else:
        pu = Fn.pad(tu[None, None], (1, 1, 1, 1, 1, 1), mode="constant", value=bc_u(t))
        pv = Fn.pad(tv[None, None], (1, 1, 1, 1, 1, 1), mode="constant", value=0.0)
    su = Fn.conv3d(pu, kern)[0, 0]
    sv = Fn.conv3d(pv, kern)[0, 0]
    if noise_amp != 0:
        r = torch.as_tensor(noise(L, (0, 0, 0), L, t, seed, dtype=np.float64)).to(dtype)
    else:
        r = torch.zeros_like(tu)
    uvv = tu * tv * tv
    du = (Du / 6.0) * su - Du * tu - uvv + F * (1 - tu) + noise_amp * r
    dv = (Dv / 6.0) * sv - Dv * tv + uvv - (F + k) * tv
    return (tu + du * dt).numpy(), (tv + dv * dt).numpy()


def run(L, nsteps: int, F=0.02, k=0.048, dt=1.0, Du=0.2, Dv=0.1, noise_amp=0.0, seed=0,
        periodic=False, dtype=np.float64, backend="numpy", init_seed=None):
    """``nsteps`` global steps from the reference init, or (``init_seed`` given) from the
    benchmarks' random init (random_fields)."""
    if isinstance(L, int):
        L = (L, L, L)
    if init_seed is None:
        u, v = init_fields(L, dtype=dtype)
    else:
        u, v = random_fields(L, seed=init_seed, dtype=dtype)
    for t in range(nsteps):
        u, v = step(u, v, t, F, k, dt, Du, Dv, noise_amp, seed, periodic, backend)
    return u, v


# ------------------------------------------------------------------------------------------
# The same oracle as whole-tensor PyTorch code that runs on any device (the GPU tests run it on
# the MI355X itself, so the production kernels can be checked at L = 256 / 512 in seconds).
# Philox is re-derived once more for int64 tensors -- torch has no unsigned 64-bit multiply, so
# each 32 x 32-bit product is split at 16 bits -- and shares no code with csrc/ or the numpy
# version above (a CPU test checks the two streams agree bit for bit).
# ------------------------------------------------------------------------------------------
_M32 = 0xFFFFFFFF


def _mulhilo32_t(a, m: int):
    """(hi, lo) 32-bit halves of a * m for int64 tensors a in [0, 2^32), m < 2^32."""
    a_hi, a_lo = a >> 16, a & 0xFFFF
    x = a_lo * m                     # < 2^48
    y = a_hi * m                     # < 2^48
    hi = (y + (x >> 16)) >> 16       # floor(a m / 2^32)
    lo = (((y & 0xFFFF) << 16) + x) & _M32
    return hi, lo


def philox4x32_10_torch(c0, c1, c2, c3, seed: int):
    """Philox4x32-10 on int64 tensors holding uint32 values; returns 4 such tensors."""
    k0, k1 = seed & _M32, (seed >> 32) & _M32
    for _ in range(10):
        hi0, lo0 = _mulhilo32_t(c0, 0xD2511F53)
        hi1, lo1 = _mulhilo32_t(c2, 0xCD9E8D57)
        c0, c1, c2, c3 = hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0
        k0 = (k0 + W0) & _M32
        k1 = (k1 + W1) & _M32
    return c0, c1, c2, c3


def _global_index(L, device, torch):
    Lx, Ly, Lz = (int(v) for v in L)
    gz = torch.arange(Lz, dtype=torch.int64, device=device)[:, None, None]
    gy = torch.arange(Ly, dtype=torch.int64, device=device)[None, :, None]
    gx = torch.arange(Lx, dtype=torch.int64, device=device)[None, None, :]
    return gx, gy, gz


def random_fields_torch(L, seed: int, lo: float = 0.0, hi: float = 1.0, dtype=None, device="cpu"):
    """random_fields on a torch device: (u, v) as (Lz, Ly, Lx) tensors."""
    import torch
    dtype = dtype or torch.float32
    Lx, Ly, _ = (int(v) for v in L)
    gx, gy, gz = _global_index(L, device, torch)
    q = gx + Lx * (gy + Ly * gz)
    full = torch.full_like(q, _M32)
    w0, w1, _, _ = philox4x32_10_torch(q & _M32, q >> 32, full, full, seed)
    s = 2.0 ** -24
    u = (hi - lo) * ((w0 >> 8).to(torch.float64) * s) + lo
    v = (hi - lo) * ((w1 >> 8).to(torch.float64) * s) + lo
    return u.to(dtype), v.to(dtype)


def noise_torch(L, step: int, seed: int, dtype=None, device="cpu"):
    """noise() for the whole domain on a torch device: Uniform[-1, 1) draws, (Lz, Ly, Lx)."""
    import torch
    dtype = dtype or torch.float32
    Lx, Ly, Lz = (int(v) for v in L)
    Ly4 = (Ly + 3) // 4
    gz = torch.arange(Lz, dtype=torch.int64, device=device)[:, None, None]
    g4 = torch.arange(Ly4, dtype=torch.int64, device=device)[None, :, None]
    gx = torch.arange(Lx, dtype=torch.int64, device=device)[None, None, :]
    q = gx + Lx * (g4 + Ly4 * gz)                                      # one block per y-quad
    w = philox4x32_10_torch(q & _M32, q >> 32, torch.full_like(q, step & _M32),
                            torch.full_like(q, (step >> 32) & _M32), seed)
    words = torch.stack(w, dim=2).reshape(Lz, Ly4 * 4, Lx)[:, :Ly]  # row gy: word gy & 3
    signed = torch.where(words >= 2 ** 31, words - 2 ** 32, words)
    return signed.to(dtype) * (2.0 ** -31)


def run_torch(L, nsteps: int, F=0.02, k=0.048, dt=1.0, Du=0.2, Dv=0.1, noise_amp=0.0, seed=0,
              dtype=None, device="cpu", init_seed=None, init_lo=0.0, init_hi=1.0, u0=None,
              v0=None, arith: str = "storage"):
    """``run`` as device-resident PyTorch (non-periodic reference boundary): from
    the reference init, the benchmarks' random init (``init_seed``) or given (u0, v0).

    ``arith``: "storage" -- every operation in ``dtype`` (default float32); "julia" -- the
    reference's own Float32 arithmetic (``_step_julia``): Float32 storage, but the Laplacian,
    ``F * (1.0 - u)``, the noise term and the Euler update in Float64 (the Float64 literals
    promote them), the neighbour sum, ``u * v^2`` and ``(F + k) * v`` in Float32, rounded to
    Float32 on store.  Returns (u, v) tensors on ``device``."""
    import torch
    import torch.nn.functional as Fn
    dtype = dtype or torch.float32
    if arith not in ("storage", "julia"):
        raise ValueError(f"arith must be storage | julia, not {arith!r}")
    if isinstance(L, int):
        L = (L, L, L)
    if u0 is not None:
        u, v = u0.to(device=device, dtype=dtype), v0.to(device=device, dtype=dtype)
    elif init_seed is not None:
        u, v = random_fields_torch(L, init_seed, init_lo, init_hi, dtype, device)
    else:
        a, b = init_fields(L, dtype=np.float64)
        u = torch.as_tensor(a).to(device=device, dtype=dtype)
        v = torch.as_tensor(b).to(device=device, dtype=dtype)

    def nsum(p):
        return ((p[1:-1, 1:-1, :-2] + p[1:-1, 1:-1, 2:]) + (p[1:-1, :-2, 1:-1] + p[1:-1, 2:, 1:-1])
                + (p[:-2, 1:-1, 1:-1] + p[2:, 1:-1, 1:-1]))

    if arith == "julia":
        for t in range(nsteps):
            u, v = _step_julia(u, v, t, F, k, dt, Du, Dv, noise_amp, seed, L)
        return u, v
    for t in range(nsteps):
        su = nsum(Fn.pad(u, (1, 1, 1, 1, 1, 1), mode="constant", value=bc_u(t)))
        sv = nsum(Fn.pad(v, (1, 1, 1, 1, 1, 1), mode="constant", value=0.0))
        uvv = u * v * v
        du = (Du / 6.0) * su - Du * u - uvv + F * (1.0 - u)
        if noise_amp != 0:
            du = du + noise_amp * noise_torch(L, t, seed, dtype, device)
        dv = (Dv / 6.0) * sv - Dv * v + uvv - (F + k) * v
        u, v = u + du * dt, v + dv * dt
    return u, v


def _step_julia(u, v, t, F, k, dt, Du, Dv, noise_amp, seed, L):
    """One step with the reference's mixed precision for T = Float32, evaluated in Julia's
    order (src/simulation/Simulation_CPU.jl:82-109, Common.jl:13-18):

      params       Du, Dv, F, K, noise, dt = convert(Float32, ...)              (:82-87)
      laplacian    l = x[i-1] + x[i+1] + x[j-1] + x[j+1] + x[k-1] + x[k+1]       Float32, left
                       - 6.0 * x[i,j,k]                                           to right, then
                   l / 6.0                                                        Float64
      du = Du * lap_u - u * v^2 + F * (1.0 - u) + noise * rand(Uniform(-1, 1))  Float64
                   (u * v^2 is Float32: v^2 = v * v, then u * that)
      dv = Dv * lap_v + u * v^2 - (F + K) * v                                    Float64
                   ((F + K) * v is Float32)
      u_temp = u + du * dt ; v_temp = v + dv * dt                                Float64, stored
                                                                                 as Float32
    The uniform draw is this framework's Philox stream (the reference's ``rand`` is not
    reproducible), exact in Float64.  ``u``, ``v``: float32 tensors; returns float32 tensors."""
    import torch
    import torch.nn.functional as Fn
    f32 = np.float32
    Du32, Dv32, F32, K32 = float(f32(Du)), float(f32(Dv)), float(f32(F)), float(f32(k))
    n32, dt32 = float(f32(noise_amp)), float(f32(dt))
    FK32 = float(f32(F32) + f32(K32))  # F + K in Float32

    def lap(x, bc):
        p = Fn.pad(x, (1, 1, 1, 1, 1, 1), mode="constant", value=bc)
        s = p[1:-1, 1:-1, :-2] + p[1:-1, 1:-1, 2:]      # Float32, Julia's left-to-right order
        s = s + p[1:-1, :-2, 1:-1]
        s = s + p[1:-1, 2:, 1:-1]
        s = s + p[:-2, 1:-1, 1:-1]
        s = s + p[2:, 1:-1, 1:-1]
        return (s.double() - 6.0 * x.double()) / 6.0     # promoted by the 6.0 literals

    lu, lv = lap(u, bc_u(t)), lap(v, 0.0)
    uvv = (u * (v * v)).double()                         # u * v^2 in Float32
    du = Du32 * lu - uvv + F32 * (1.0 - u.double())
    if noise_amp != 0:
        du = du + n32 * noise_torch(L, t, seed, torch.float64, u.device)
    dv = Dv32 * lv + uvv - (FK32 * v).double()           # (F + K) * v in Float32
    return (u.double() + du * dt32).float(), (v.double() + dv * dt32).float()
