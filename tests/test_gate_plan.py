"""The gated pass's unit table (csrc/include/gs/gate_plan.h), checked on the CPU against an
independent computation of each unit's level-0 read box (the planner is shared by the HIP
backend, backend_hip.hip gate_table; the GPU side is tests/test_gpu_gated.py).

For every sub-domain / neighbour set: the units of each tile column partition its planes
[0, nz); a unit is start-gated exactly when its read box -- the tile's x / y window x
[z0 - n, z1 + n) -- meets a ghost region a neighbour fills (H cells deep on that side); the
units fit the slots when some plane budget allows it; the table is sorted by (z0, tile) and the
packers are numbered 0..npk-1 (the start-gated units, or every unit); a unit is a producer
(it packs its outputs into the next exchange's messages at its end in a carried exchange)
exactly when its output box meets a send region, and the producers' output boxes cover every
send region's cells once."""
import itertools

import pytest

from grayscott_amd.ops import native

H = 3


def _nbr(dirs):
    """nbr27 with rank 0 at the given (dx, dy, dz) directions, -1 elsewhere (index
    (dx + 1) * 9 + (dy + 1) * 3 + (dz + 1))."""
    out = [-1] * 27
    for dx, dy, dz in dirs:
        out[(dx + 1) * 9 + (dy + 1) * 3 + (dz + 1)] = 0
    return out


def _ghost_regions(nx, ny, nz, dirs):
    def rng(d, n):
        return (-H, 0) if d < 0 else ((n, n + H) if d > 0 else (0, n))
    return [(rng(dx, nx), rng(dy, ny), rng(dz, nz)) for dx, dy, dz in dirs]


def _window(grid, tile, n):
    """Independent copy of the kernel's tile window (fused.hpp fused_body / gate prologue)."""
    if grid["nfold"] and tile >= grid["ntxf"] * grid["nty"]:
        f = tile - grid["ntxf"] * grid["nty"]
        tx, ty, xw, ye = grid["ntxf"], 2 * f, 32, grid["rt"] + grid["ystep"]
    else:
        tx, ty, xw, ye = tile % grid["ntxf"], tile // grid["ntxf"], 64, grid["rt"]
    x0 = tx * grid["xstep"] - n
    y0 = grid["ybase"] + ty * grid["ystep"] - n
    return (x0, x0 + xw), (y0, y0 + ye)


def _meets(a, b):
    return a[0] < b[1] and b[0] < a[1]


def _send_regions(g, dirs):
    """The outgoing messages (gs::make_halo_plan): interior side boxes, H deep; z slabs (z
    neighbours only) send whole storage planes, ghost and padding columns / rows included."""
    nx, ny, nz = g.nx, g.ny, g.nz

    def rng(d, n):
        return (0, H) if d < 0 else ((n - H, n) if d > 0 else (0, n))
    zplanes = all(dx == 0 and dy == 0 for dx, dy, _ in dirs)
    out = []
    for dx, dy, dz in dirs:
        sx, sy = rng(dx, nx), rng(dy, ny)
        if zplanes:
            sx, sy = (-g.xo, g.px - g.xo), (-H, g.py - H)
        out.append((sx, sy, rng(dz, nz)))
    return out


FAR = 1 << 28


def _carry_window(grid, tile, n, g, z0, z1):
    """Independent copy of the cells a unit carries: the cells its tile's launch stores
    (fused.hpp fused_body: ox1 / oy1) x [z0, z1), open past the sub-domain's faces."""
    (x0, x1), (y0, y1) = _window(grid, tile, n)
    folded = x1 - x0 == 32
    ox = [max(x0 + n, 0), min(x0 + n + (32 - 2 * n if folded else grid["xstep"]), g.nx)]
    oy = [max(y0 + n, 0), min(y0 + n + (2 if folded else 1) * grid["ystep"], g.ny)]
    oz = [z0, z1]
    for w, size in ((ox, g.nx), (oy, g.ny), (oz, g.nz)):
        if w[0] <= 0:
            w[0] = -FAR
        if w[1] >= size:
            w[1] = FAR
    return ox, oy, oz


def _check_producers(units, grid, n, g, dirs):
    sends = _send_regions(g, dirs)
    covered = [0] * len(sends)
    for t, z0, z1, pk, wait, prod in units:
        if t < 0:
            continue
        ox, oy, oz = _carry_window(grid, t, n, g, z0, z1)
        meets = False
        for i, (sx, sy, sz) in enumerate(sends):
            cx = max(0, min(ox[1], sx[1]) - max(ox[0], sx[0]))
            cy = max(0, min(oy[1], sy[1]) - max(oy[0], sy[0]))
            cz = max(0, min(oz[1], sz[1]) - max(oz[0], sz[0]))
            covered[i] += cx * cy * cz
            meets = meets or cx * cy * cz > 0
        assert bool(prod) == meets, (t, z0, z1, prod)
        if prod:
            assert wait, (t, z0, z1)  # symmetric neighbours: a producer read the same peer's ghosts
    for (sx, sy, sz), c in zip(sends, covered):
        assert c == (sx[1] - sx[0]) * (sy[1] - sy[0]) * (sz[1] - sz[0])


ONE_SIDED = [d for d in itertools.product((0, 1), repeat=3) if d != (0, 0, 0)]
ALL26 = [d for d in itertools.product((-1, 0, 1), repeat=3) if d != (0, 0, 0)]
Z_ONLY = [(0, 0, -1), (0, 0, 1)]
X_SPLIT = [(1, 0, 0)]


@pytest.mark.parametrize("shape,dirs,n,fold,xp,allpk,slots", [
    ((64, 64, 64), Z_ONLY, 3, False, 0, False, 256),
    ((256, 256, 64), Z_ONLY, 3, False, 16, False, 256),
    ((128, 128, 128), ONE_SIDED, 3, True, 8, False, 256),
    ((256, 256, 256), ONE_SIDED, 3, True, 16, True, 256),
    ((96, 80, 72), ALL26, 2, False, 4, False, 128),
    ((40, 40, 40), ALL26, 3, False, 0, False, 256),
    ((32, 64, 64), X_SPLIT, 3, False, 24, True, 64),
    ((512, 512, 8), Z_ONLY, 3, False, 0, False, 64),  # more columns than slots
])
def test_gate_plan_matches_independent_cones(shape, dirs, n, fold, xp, allpk, slots):
    nx, ny, nz = shape
    g = native.make_geom(nx, ny, nz, H, 0, 0, 0, nx * 2, ny * 2, nz * 2, False)
    units, npk, grid = native.gate_plan(g, _nbr(dirs), n, xp=xp, allpk=allpk, slots=slots,
                                        fold=fold)
    ghosts = _ghost_regions(nx, ny, nz, dirs)
    # each column's units partition [0, nz)
    by_tile = {}
    for t, z0, z1, pk, wait, prod in units:
        assert 0 <= t < grid["ntiles"] and 0 <= z0 < z1 <= nz
        by_tile.setdefault(t, []).append((z0, z1))
    assert sorted(by_tile) == list(range(grid["ntiles"]))
    for t, iv in by_tile.items():
        iv.sort()
        assert iv[0][0] == 0 and iv[-1][1] == nz
        assert all(a[1] == b[0] for a, b in zip(iv, iv[1:])), (t, iv)
    # start-gated exactly when the read box meets a neighbour's ghost region
    for t, z0, z1, pk, wait, prod in units:
        xr, yr = _window(grid, t, n)
        zr = (z0 - n, z1 + n)
        need = any(_meets(xr, gx) and _meets(yr, gy) and _meets(zr, gz) for gx, gy, gz in ghosts)
        assert bool(wait) == need, (t, z0, z1, wait, need)
    # fits the slots whenever the longest chunks do
    longest, _, _ = native.gate_plan(g, _nbr(dirs), n, xp=xp, allpk=allpk, slots=slots,
                                     fold=fold, longest=True)
    if len(longest) <= slots:
        assert len(units) <= slots
    # order and packer numbering
    assert units == sorted(units, key=lambda u: (u[1], u[0]))
    pks = [u[3] for u in units if u[3] >= 0]
    assert sorted(pks) == list(range(npk))
    if allpk:
        assert npk == len(units)
    else:
        assert all((u[3] >= 0) == bool(u[4]) for u in units)
    _check_producers(units, grid, n, g, dirs)


def test_gate_plan_tile_grid_matches_the_kernel():
    """The planner's tile grid is the launch's (FusedLaunch::run + fold_strip): L=256, n=3,
    4x12 tiles (58 x 40 outputs), the folded last x strip -- 4 x 7 full tiles + 4 folded units
    = 32 tiles."""
    g = native.make_geom(256, 256, 256, H, 0, 0, 0, 256, 256, 256, False)
    _, _, grid = native.gate_plan(g, _nbr(Z_ONLY), 3, fold=True)
    assert (grid["xstep"], grid["ystep"], grid["ntx"], grid["nty"]) == (58, 40, 5, 7)
    assert (grid["ntxf"], grid["nfold"], grid["ntiles"]) == (4, 4, 32)
    _, _, grid = native.gate_plan(g, _nbr(Z_ONLY), 3, fold=False)
    assert grid["ntiles"] == 35


@pytest.mark.parametrize("shape,dirs,n,fold,X,U,allpk,slots", [
    ((256, 256, 256), ONE_SIDED, 3, True, 16, 6, False, 256),
    ((256, 256, 256), ONE_SIDED, 3, True, 32, 6, True, 256),
    ((256, 256, 256), ALL26, 3, True, 24, 8, False, 256),
    ((96, 80, 72), ALL26, 2, False, 8, 4, False, 128),
    ((512, 512, 64), Z_ONLY, 3, False, 40, 6, False, 256),
    ((64, 64, 64), Z_ONLY, 3, False, 0, 0, True, 256),
])
def test_gate_plan_pairs(shape, dirs, n, fold, X, U, allpk, slots):
    """The two-units-per-workgroup table: entry 2w is an ungated chunk (or empty), 2w + 1 a
    start-gated chunk (or empty); together the chunks partition every column; only the second
    entries read ghosts (checked against the independent cones); at most `slots` workgroups."""
    nx, ny, nz = shape
    g = native.make_geom(nx, ny, nz, H, 0, 0, 0, nx * 2, ny * 2, nz * 2, False)
    units, npk, grid = native.gate_plan(g, _nbr(dirs), n, xp=X, allpk=allpk, slots=slots,
                                        fold=fold, pairs=True, unpack=U)
    assert units and len(units) % 2 == 0 and len(units) // 2 <= slots
    ghosts = _ghost_regions(nx, ny, nz, dirs)
    by_tile = {}
    for i, (t, z0, z1, pk, wait, prod) in enumerate(units):
        if t < 0:
            continue
        assert 0 <= z0 < z1 <= nz
        by_tile.setdefault(t, []).append((z0, z1))
        xr, yr = _window(grid, t, n)
        need = any(_meets(xr, gx) and _meets(yr, gy) and _meets((z0 - n, z1 + n), gz)
                   for gx, gy, gz in ghosts)
        assert bool(wait) == need, (i, t, z0, z1, wait, need)
        assert bool(wait) == (i % 2 == 1)  # gated units are second, ungated first
    assert sorted(by_tile) == list(range(grid["ntiles"]))
    for t, iv in by_tile.items():
        iv.sort()
        assert iv[0][0] == 0 and iv[-1][1] == nz
        assert all(a[1] == b[0] for a, b in zip(iv, iv[1:])), (t, iv)
    pks = [units[w][3] for w in range(0, len(units), 2) if units[w][3] >= 0]
    assert sorted(pks) == list(range(npk))
    for w in range(0, len(units), 2):
        if units[w + 1][4]:
            assert units[w][3] >= 0  # a workgroup with a gated unit packs
        if allpk:
            assert units[w][3] >= 0
