"""Host model of the small-grid block kernel's indexing (csrc/hip/block.hpp, k_block).

The GPU test (tests/test_gpu_block.py) checks k_block bit for bit against k_fused on the device.
This CPU test re-traces the kernel's index arithmetic in numpy -- the level-0 load of the
dependency cone into the LDS buffers, the quad work items of every level, the LDS rows and planes
each item reads and writes, the boundary resets, the x-ghost corrections of lanes 0 / 63, the
final stores -- and checks that
  * every LDS and global index the kernel forms is in range (no access outside the arrays), and
  * the blocked T-level result equals T global steps computed with the same floating-point
    operation order (k_fused's: s = (xm + (xp + ((ym + yp) + zm))) + zp and the folded update),
bit for bit, on sub-domains with and without y / z neighbours.
fp32 fused multiply-adds are modelled as an exact product plus one fp64 rounding then fp32 (the
same on both sides of the comparison).
"""
import numpy as np
import pytest

from grayscott_amd.ops.reference import bc_u, noise as ref_noise, random_fields

F, K, DT, DU, DV, NOISE, SEED = 0.02, 0.048, 1.0, 0.2, 0.1, 0.1, 19
f32 = np.float32


def fma(a, b, c):
    return (np.float64(a) * np.float64(b) + np.float64(c)).astype(f32)


def fold():
    return dict(kd=(f32(-DT), f32(DT)), kc=(f32(DT * F), f32(0)),
                ks=(f32(DT * DU / 6.0), f32(DT * DV / 6.0)),
                kcc=(f32(1.0 - DT * (DU + F)), f32(1.0 - DT * (DV + F + K))),
                ar31=f32(f32(DT * NOISE) * f32(4.656612873077392578125e-10)))


def update(c, s, w, fc):
    """The folded cell update on (u, v) pairs: c, s = lists [u, v] of arrays, w = Philox word."""
    cu, cv = c
    t0 = (cu * cv).astype(f32)
    uvv = (t0 * cv).astype(f32)
    out = []
    for i in range(2):
        p = fma(fc["kd"][i], uvv, fc["kc"][i])
        p = fma(fc["ks"][i], s[i], p)
        p = fma(fc["kcc"][i], c[i], p)
        out.append(p)
    if w is not None:
        out[0] = fma(fc["ar31"], w.view(np.int32).astype(f32), out[0])
    return out


def global_step(u, v, t, L, fc):
    """One step of the whole L^3 domain in k_fused's operation order."""
    b = f32(bc_u(t))
    up = np.pad(u, 1, constant_values=b)
    vp = np.pad(v, 1, constant_values=f32(0))
    s = []
    for a in (up, vp):
        c = a[1:-1, 1:-1, 1:-1]
        xm, xp = a[1:-1, 1:-1, :-2], a[1:-1, 1:-1, 2:]
        ym, yp = a[1:-1, :-2, 1:-1], a[1:-1, 2:, 1:-1]
        zm, zp = a[:-2, 1:-1, 1:-1], a[2:, 1:-1, 1:-1]
        yz = ((ym + yp).astype(f32) + zm).astype(f32)
        A = (xm + (xp + yz).astype(f32)).astype(f32)
        s.append((A + zp).astype(f32))
    r = ref_noise((L, L, L), (0, 0, 0), (L, L, L), t, SEED, dtype=np.float64)
    w = np.round(r * 2.0 ** 31).astype(np.int64).astype(np.int32).view(np.uint32)
    return update([u, v], s, w, fc)


def philox_words(gy, gz, gx, L, tstep):
    """k_block's draw for the quad at global row gy (a multiple of 4) of plane gz, lanes gx:
    the 32-bit counter gx + Lx * (gy4 + Ly4 * gz) in wrapping uint32 arithmetic."""
    from grayscott_amd.ops.reference import philox4x32_10
    M = 0xFFFFFFFF
    Ly4 = (L + 3) // 4
    gy4 = (gy >> 2) & M
    qu = (L * ((gy4 + Ly4 * (gz & M)) & M)) & M
    q = (np.uint64(qu) + gx.astype(np.uint64)) & np.uint64(M)
    st = np.uint64(tstep)
    return philox4x32_10(q, np.zeros_like(q), st & np.uint64(M), st >> np.uint64(32), SEED)


def block_pass(ustore, vstore, geo, t, TL, BY, BZ, fc):
    """k_block over a sub-domain: storage arrays (pz, py, px) with H ghosts, x at offset xo."""
    nx, ny, nz, H, xo, oy, oz, L = (geo[k] for k in ("nx", "ny", "nz", "H", "xo", "oy", "oz",
                                                      "L"))
    R0, NR, NP = 5, BY + 10, BZ + 2 * TL
    lane = np.arange(64)
    yb = -((oy % 4 + 4) % 4)
    nby = (ny - yb + BY - 1) // BY
    nbz = (nz + BZ - 1) // BZ
    out_u = np.full((nz, ny, nx), np.nan, dtype=f32)
    out_v = np.full((nz, ny, nx), np.nan, dtype=f32)
    written = np.zeros((nz, ny, nx), dtype=np.int32)
    for bid in range(nby * nbz):
        by, bz = bid % nby, bid // nby
        y0, z0 = yb + by * BY, bz * BZ
        buf = np.full((2, 2, NP, NR, 64), np.nan, dtype=f32)  # [level parity][u/v]...
        NL = BY + 2 * TL
        for i in range(NP * NL):
            pz, ry = i // NL, R0 - TL + (i % NL)
            assert 0 <= pz < NP and 0 <= ry < NR
            z, y = z0 - TL + pz, y0 - R0 + ry
            val = np.zeros((2, 64), dtype=f32)
            if -H <= z < nz + H and -H <= y < ny + H:
                ok = lane < nx + H
                xs = lane[ok] + xo
                assert xs.max() < ustore.shape[2]
                val[0, ok] = ustore[z + H, y + H, xs]
                val[1, ok] = vstore[z + H, y + H, xs]
            buf[0, :, pz, ry] = val
        NZR = R0 - TL
        for i in range(NP * (2 * NZR + 2)):
            pz, j = i // (2 * NZR + 2), i % (2 * NZR + 2)
            if j < 2 * NZR:
                r = j if j < NZR else NR - 2 * NZR + j
                assert 0 <= r < NR
                buf[0, :, pz, r] = 0
            else:
                buf[1, :, pz, 0 if j == 2 * NZR else NR - 1] = 0
        for lv in range(TL):
            inb, outb = lv & 1, (lv + 1) & 1
            last = lv + 1 == TL
            mq = 0 if last else 1
            nq = BY // 4 + 2 * mq
            dz = TL - 1 - lv
            npl = BZ + 2 * dz
            b_in, b_out = f32(bc_u(t + lv)), f32(bc_u(t + lv + 1))
            gl = [np.where(lane == 0, b_in, f32(0)).astype(f32), np.zeros(64, f32)]
            gr = [np.where((lane == 63) & (nx == 64), b_in, f32(0)).astype(f32), np.zeros(64, f32)]
            for it in range(nq * npl):
                zi, qi = it // nq, it % nq
                qy = y0 - 4 * mq + 4 * qi
                z = z0 - dz + zi
                pz = z - (z0 - TL)
                ry = qy - y0 + R0
                assert 1 <= pz <= NP - 2 and 1 <= ry and ry + 4 < NR
                row = buf[inb, :, pz, ry - 1:ry + 5]
                pm = buf[inb, :, pz - 1, ry:ry + 4]
                pp = buf[inb, :, pz + 1, ry:ry + 4]
                gz = oz + z
                words = philox_words(oy + qy, gz, lane, L, t + lv)
                for k in range(4):
                    c = [row[0, k + 1], row[1, k + 1]]
                    s = []
                    for i in range(2):
                        yz = ((row[i, k] + row[i, k + 2]).astype(f32) + pm[i, k]).astype(f32)
                        yz = (yz + gr[i]).astype(f32)
                        xp = np.concatenate([c[i][1:], [f32(0)]]).astype(f32)
                        xm = np.concatenate([[f32(0)], c[i][:-1]]).astype(f32)
                        A = (xm + (xp + yz).astype(f32)).astype(f32)
                        A = (A + gl[i]).astype(f32)
                        s.append((A + pp[i, k]).astype(f32))
                    P = update(c, s, words[k], fc)
                    y = qy + k
                    if not last:
                        gy = oy + y
                        outside = (gz < 0) | (gz >= L) | (lane >= L) | (gy < 0) | (gy >= L)
                        P[0] = np.where(outside, b_out, P[0]).astype(f32)
                        P[1] = np.where(outside, f32(0), P[1]).astype(f32)
                        assert ry + k < NR
                        buf[outb, 0, pz, ry + k] = P[0]
                        buf[outb, 1, pz, ry + k] = P[1]
                    elif 0 <= y < ny and z < nz:
                        assert z >= 0
                        out_u[z, y, :nx] = P[0][:nx]
                        out_v[z, y, :nx] = P[1][:nx]
                        written[z, y, :] += 1
    assert (written == 1).all(), "every interior cell stored exactly once"
    return out_u, out_v


def storage(gu, gv, geo, t):
    """Sub-domain storage with H ghosts: neighbours' cells where the global grid has them, the
    boundary value of time t outside it (engine.h ensure_bc), x rows padded like gs::make_geom."""
    nx, ny, nz, H, oy, oz, L = (geo[k] for k in ("nx", "ny", "nz", "H", "oy", "oz", "L"))
    xo = ((H + 7) // 8) * 8
    px = ((xo + nx + H + 7) // 8) * 8
    gpu = np.pad(gu, H, constant_values=f32(bc_u(t)))
    gpv = np.pad(gv, H, constant_values=f32(0))
    us = np.full((nz + 2 * H, ny + 2 * H, px), 7.0, dtype=f32)  # row padding: arbitrary
    vs = np.full_like(us, 7.0)
    us[:, :, xo - H:xo + nx + H] = gpu[oz:oz + nz + 2 * H, oy:oy + ny + 2 * H, :]
    vs[:, :, xo - H:xo + nx + H] = gpv[oz:oz + nz + 2 * H, oy:oy + ny + 2 * H, :]
    geo = dict(geo, xo=xo)
    return us, vs, geo


@pytest.mark.parametrize("L,TL,BY,BZ,sub", [
    (16, 2, 8, 2, None), (16, 3, 4, 4, None), (14, 3, 8, 1, None), (18, 2, 4, 1, None),
    # sub-domains with y / z neighbours (oy not a multiple of 4: a partial first quad)
    (16, 3, 8, 2, (6, 10, 5, 7)), (16, 2, 4, 2, (3, 9, 8, 8)),
    # x rows filling the wave (nx = 64: lane 63 adds the +x ghost), at / away from the boundary
    (64, 3, 8, 2, (22, 8, 30, 4)), (64, 2, 4, 1, (0, 8, 60, 4)),
])
def test_block_model_matches_global_steps(L, TL, BY, BZ, sub):
    fc = fold()
    u0, v0 = random_fields((L, L, L), seed=3, dtype=np.float32)
    u0, v0 = u0.astype(f32), v0.astype(f32)
    t = 4
    gu, gv = u0, v0
    for s in range(TL):
        gu, gv = global_step(gu, gv, t + s, L, fc)
    oy, ny, oz, nz = sub if sub else (0, L, 0, L)
    geo = dict(nx=L, ny=ny, nz=nz, H=3, oy=oy, oz=oz, L=L)
    us, vs, geo = storage(u0, v0, geo, t)
    bu, bv = block_pass(us, vs, geo, t, TL, BY, BZ, fc)
    np.testing.assert_array_equal(bu, gu[oz:oz + nz, oy:oy + ny, :])
    np.testing.assert_array_equal(bv, gv[oz:oz + nz, oy:oy + ny, :])
