"""Domain decomposition + halo exchange (CPU backend, gloo, multi-process).

Reference: init_domain (communication.jl:59-96), exchange! (:138-199) and the functional
`mpirun -n 4` runs (test/functional/functional-GrayScott.jl).  Because the Philox noise is
keyed on global cell coordinates, a decomposed run must reproduce the single-rank run
bit for bit.
"""
import numpy as np
import pytest

from grayscott_amd.parallel.decomp import (all_domains, coords_of, dims_create, init_domain,
                                           rank_of, split_extent)

from .mp_utils import run_ranks


# ------------------------------------------------------------------------------------------
# Dims_create / Cart topology (pure functions)
# ------------------------------------------------------------------------------------------
@pytest.mark.parametrize("n,expect", [(1, [1, 1, 1]), (2, [2, 1, 1]), (3, [3, 1, 1]),
                                      (4, [2, 2, 1]), (6, [3, 2, 1]), (8, [2, 2, 2]),
                                      (12, [3, 2, 2]), (16, [4, 2, 2]), (24, [4, 3, 2]),
                                      (27, [3, 3, 3]), (64, [4, 4, 4]), (7, [7, 1, 1])])
def test_dims_create(n, expect):
    assert dims_create(n) == expect


def test_dims_create_fixed_entries():
    assert dims_create(8, [0, 1, 0]) == [4, 1, 2]
    assert dims_create(6, [0, 0, 3]) == [2, 1, 3]
    with pytest.raises(ValueError):
        dims_create(6, [4, 0, 0])


def test_coords_roundtrip():
    dims = [3, 2, 2]
    for r in range(12):
        assert rank_of(coords_of(r, dims), dims) == r
    assert coords_of(1, dims) == (0, 0, 1)  # last dimension fastest (row-major)


@pytest.mark.parametrize("L,p", [(64, 2), (65, 2), (30, 4), (7, 3), (128, 8)])
def test_split_extent_covers(L, p):
    tot, prev_end = 0, 0
    for c in range(p):
        s, o = split_extent(L, p, c)
        assert o == prev_end
        prev_end = o + s
        tot += s
    assert tot == L
    sizes = [split_extent(L, p, c)[0] for c in range(p)]
    assert max(sizes) - min(sizes) <= 1
    assert sizes == sorted(sizes, reverse=True)  # low coords absorb the remainder


def test_neighbors_nonperiodic_and_periodic():
    d = init_domain(64, 8, 0)
    assert d.dims == [2, 2, 2] and d.coords == (0, 0, 0)
    assert d.proc_neighbors == {"west": -1, "east": 4, "down": -1, "up": 2, "south": -1, "north": 1}
    assert d.neighbor(1, 1, 1) == 7
    p = init_domain(64, 8, 0, periodic=True)
    assert p.proc_neighbors["west"] == 4 and p.proc_neighbors["down"] == 2
    one = init_domain(16, 1, 0, periodic=True)
    assert all(r == 0 for i, r in enumerate(one.nbr27) if i != 13)


def test_all_domains_tile_the_grid():
    L = 37
    seen = np.zeros((L, L, L), dtype=int)
    for dom in all_domains(L, 12):
        o, s = dom.proc_offsets, dom.proc_sizes
        seen[o[2]:o[2] + s[2], o[1]:o[1] + s[1], o[0]:o[0] + s[0]] += 1
    assert (seen == 1).all()


# ------------------------------------------------------------------------------------------
# multi-process runs (gloo)
# ------------------------------------------------------------------------------------------
def _cfg(L, steps, fuse=1, periodic=False, noise=0.1, prec="Float64"):
    return {"settings": dict(L=L, precision=prec, F=0.02, k=0.048, dt=1.0, Du=0.2, Dv=0.1,
                             noise=noise, backend="CPU", periodic=periodic, seed=99),
            "steps": steps, "fuse": fuse, "transport": "torch"}


@pytest.mark.parametrize("world,L,fuse,periodic", [
    (2, 16, 1, False),
    (4, 18, 1, False),
    (8, 16, 2, False),
    (4, 13, 2, False),   # non-divisible L, remainder distribution (D5)
    (2, 12, 1, True),    # periodic, dims 2 -> both x-neighbours are the same rank
    (8, 16, 3, True),
])
def test_decomposed_run_matches_single_rank(world, L, fuse, periodic):
    steps = 7
    u1, v1, _ = run_ranks(1, _cfg(L, steps, 1, periodic))
    un, vn, meta = run_ranks(world, _cfg(L, steps, fuse, periodic))
    assert all(m["step"] == steps for m in meta)
    assert meta[0]["transport"] == "torch"
    np.testing.assert_array_equal(un, u1)
    np.testing.assert_array_equal(vn, v1)


@pytest.mark.parametrize("world,L,fuse,periodic", [
    (2, 16, 2, False),
    (4, 21, 3, False),   # uneven slabs
    (3, 17, 1, False),
    (2, 12, 2, True),    # periodic: x/y wrap onto self, so the generic 26-direction plan
])
def test_z_slab_decomposition_matches_single_rank(world, L, fuse, periodic):
    """1 x 1 x N slabs: halos are whole storage planes (zplanes plan) -- same answer."""
    steps = 7
    u1, v1, _ = run_ranks(1, _cfg(L, steps, 1, periodic))
    cfg = _cfg(L, steps, fuse, periodic)
    cfg["settings"]["decomposition"] = "z"
    un, vn, meta = run_ranks(world, cfg)
    assert all(m["zplanes"] == (not periodic) for m in meta)
    np.testing.assert_array_equal(un, u1)
    np.testing.assert_array_equal(vn, v1)


def test_choose_dims():
    from grayscott_amd.parallel.decomp import choose_dims
    assert choose_dims(512, 8, "auto", "hip") == [1, 1, 8]
    assert choose_dims(512, 8, "auto", "cpu") == dims_create(8)
    assert choose_dims(64, 8, "auto", "hip") == dims_create(8)   # 8-plane slabs: balanced
    assert choose_dims(64, 4, "balanced", "hip") == dims_create(4)
    assert choose_dims(64, 4, "z", "cpu") == [1, 1, 4]
    assert choose_dims(64, 1, "z", "hip") == [1, 1, 1]
    with pytest.raises(ValueError):
        choose_dims(64, 4, "diagonal", "hip")


@pytest.mark.parametrize("world,L,fuse,periodic,decomp", [
    (1, 14, 2, False, "balanced"),
    (1, 12, 3, True, "balanced"),
    (4, 16, 2, False, "balanced"),
    (2, 16, 3, False, "z"),
    (8, 16, 2, True, "balanced"),
])
def test_halo_poisoning(world, L, fuse, periodic, decomp):
    """NaN in every ghost / padding cell before the run never reaches the interior."""
    steps = 6
    u1, v1, _ = run_ranks(1, _cfg(L, steps, 1, periodic))
    cfg = _cfg(L, steps, fuse, periodic)
    cfg["settings"]["decomposition"] = decomp
    cfg["poison"] = True
    un, vn, _ = run_ranks(world, cfg)
    assert np.isfinite(un).all() and np.isfinite(vn).all()
    np.testing.assert_array_equal(un, u1)
    np.testing.assert_array_equal(vn, v1)


@pytest.mark.parametrize("world,L", [(4, 20), (3, 17)])
def test_random_init_is_decomposition_invariant(world, L):
    """The benchmarks' random init is a function of the global cell (gs::random_init_cell):
    N ranks start from -- and, 6 steps later, end at -- the same global state as one rank."""
    from grayscott_amd.ops import reference as ref
    cfg1 = _cfg(L, 0, 1, False)
    cfg1["random_init"] = 99
    u0, v0, _ = run_ranks(world, cfg1)
    ru, rv = ref.random_fields((L, L, L), seed=99, dtype=np.float32)
    np.testing.assert_array_equal(u0, ru)
    np.testing.assert_array_equal(v0, rv)
    cfg1["steps"] = 6
    cfgn = _cfg(L, 6, 1, False)
    cfgn["random_init"] = 99
    u1, v1, _ = run_ranks(1, cfg1)
    un, vn, _ = run_ranks(world, cfgn)
    np.testing.assert_array_equal(un, u1)
    np.testing.assert_array_equal(vn, v1)


def test_default_fuse_policy():
    """Steps per pass when fuse_steps = 0 (models/grayscott.py default_fuse): one rank without
    neighbours gets 4 ghost layers in fp32 (3 in fp64: the T = 4 entry is the fp32 LDS-ring
    kernel) and lets the engine measure the depths and plan the passes; with neighbours the
    depth follows the plane size (T=3 from 160^2 x-y planes, fp32 and fp64 alike since round 3,
    profiles/r3_f64_depth.txt); the CPU backend steps one at a time."""
    from grayscott_amd.models.grayscott import default_fuse

    assert default_fuse("hip", init_domain(64, 1, 0)) == 4
    assert default_fuse("hip", init_domain(64, 1, 0), "float64") == 3
    assert default_fuse("hip", init_domain(2, 1, 0)) == 2  # capped by the sub-domain extent
    big = init_domain(512, 8, 0, dims=[2, 2, 2])
    small = init_domain(128, 8, 0, dims=[2, 2, 2])
    for dt in ("float32", "float64"):
        assert default_fuse("hip", big, dt) == 3
        assert default_fuse("hip", small, dt) == 2
    assert default_fuse("cpu", init_domain(64, 1, 0)) == 1
