"""Model-level tests on the CPU backend (reference test/unit/simulation/unit-Simulation.jl and
the behavioural spec of SURVEY.md §0)."""
import numpy as np
import pytest

from grayscott_amd.models.grayscott import GrayScott
from grayscott_amd.ops import reference as ref
from grayscott_amd.parallel.decomp import init_domain
from grayscott_amd.utils.config import Settings


def _sim(L=16, prec="Float64", noise=0.0, fuse=None, periodic=False, **kw):
    s = Settings(L=L, precision=prec, F=0.02, k=0.048, dt=1.0, Du=0.2, Dv=0.1, noise=noise,
                 periodic=periodic, **kw)
    sim = GrayScott(s, init_domain(L, 1, 0, periodic=periodic), fuse=fuse)
    sim.init_fields()
    return sim


def test_init_fields_default_settings_float32():
    # unit-Simulation.jl:11-17: default Settings (L=128, CPU/Plain), Float32
    s = Settings(precision="Float32")
    sim = GrayScott(s, init_domain(s.L, 1, 0))
    sim.init_fields()
    u, v = sim.get_fields()
    assert u.dtype == np.float32 and u.shape == (128, 128, 128)
    assert (u[58:71, 58:71, 58:71] == np.float32(0.25)).all()
    assert (v[58:71, 58:71, 58:71] == np.float32(0.33)).all()
    assert u[57, 64, 64] == 1.0 and v[71, 64, 64] == 0.0
    assert (u == 0.25).sum() == 13 ** 3


def test_iterate_tiny_grid():
    # unit-Simulation.jl:19-32: one iterate! on L=2 (the seed cube covers everything)
    sim = _sim(L=2)
    u0, v0 = sim.get_fields()
    assert (u0 == 0.25).all()
    sim.iterate(1)
    u, v = sim.get_fields()
    ru, rv = ref.run(2, 1)
    np.testing.assert_allclose(u, ru, rtol=0, atol=1e-15)
    np.testing.assert_allclose(v, rv, rtol=0, atol=1e-15)
    assert sim.step == 1


@pytest.mark.parametrize("noise", [0.0, 0.1])
@pytest.mark.parametrize("prec,tol", [("Float64", 1e-14), ("Float32", 2e-6)])
def test_cpu_backend_matches_golden_model(noise, prec, tol):
    sim = _sim(L=18, prec=prec, noise=noise, seed=4)
    sim.iterate(12)
    u, v = sim.get_fields()
    ru, rv = ref.run(18, 12, noise_amp=noise, seed=4)
    assert np.abs(u - ru).max() < tol and np.abs(v - rv).max() < tol


def test_outer_boundary_alternates():
    """outer u ghosts read 1 at even steps and 0 at odd steps (buffer swap)."""
    sim = _sim(L=10)
    assert sim.full_state(0)[0, 0, sim.geom.xo, 0].item() == 1.0
    assert float(sim.full_state(1).abs().max()) == 0.0
    # one step reads u ghosts = 1; the corner cell (1.0 initially) sees 3 neighbours of 1
    sim.iterate(1)
    u, _ = sim.get_fields()
    ru, _ = ref.run(10, 1)
    assert u[0, 0, 0] == ru[0, 0, 0]
    # without the alternation (ghost u = 1 every step) the 2nd step would differ
    sim.iterate(1)
    u2, _ = sim.get_fields()
    uu, vv = ref.init_fields((10, 10, 10))
    for t in range(2):
        uu, vv = ref.step(uu, vv, 0, 0.02, 0.048, 1.0, 0.2, 0.1, 0.0, 0)  # always-even ghosts
    assert np.abs(u2 - uu).max() > 1e-6
    ru2, _ = ref.run(10, 2)
    np.testing.assert_allclose(u2, ru2, atol=1e-15)


@pytest.mark.parametrize("fuse", [2, 3])
def test_multistep_passes_match_single_steps(fuse):
    a = _sim(L=14, noise=0.1, seed=8)
    b = _sim(L=14, noise=0.1, seed=8, fuse=fuse)
    a.iterate(10)
    b.iterate(10)
    np.testing.assert_array_equal(a.get_fields()[0], b.get_fields()[0])


def test_periodic_extension_matches_golden():
    sim = _sim(L=12, noise=0.1, seed=2, periodic=True, fuse=2)
    sim.iterate(6)
    u, v = sim.get_fields()
    ru, rv = ref.run(12, 6, noise_amp=0.1, seed=2, periodic=True)
    np.testing.assert_allclose(u, ru, atol=1e-14)
    np.testing.assert_allclose(v, rv, atol=1e-14)


def test_set_fields_and_stats():
    sim = _sim(L=8)
    rng = np.random.default_rng(1)
    u = rng.random((8, 8, 8))
    v = rng.random((8, 8, 8))
    sim.set_fields(u, v)
    gu, gv = sim.get_fields()
    np.testing.assert_array_equal(gu, u)
    s = sim.stats()
    assert s[0] == pytest.approx(u.sum()) and s[1] == u.min() and s[5] == v.max()
    g = sim.global_stats()
    assert g["mean_v"] == pytest.approx(v.mean())
    with pytest.raises(ValueError):
        sim.set_fields(u[:4], v)


def test_hip_backend_fails_loudly_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(RuntimeError, match="no GPU"):
        _sim(L=8, backend="AMDGPU")


@pytest.mark.parametrize("lo,hi,prec", [(-0.3, 0.7, "Float64"), (0.1, 0.35, "Float64"),
                                        (-1.0, 2.5, "Float32")])
def test_random_init_any_range_matches_numpy_oracle(lo, hi, prec):
    """gs::random_init_cell evaluates (hi - lo) * frac + lo unfused, like the numpy oracle
    (ops/reference.py random_fields), so any range gives the same bits (not just [0, 1))."""
    L = 14
    sim = _sim(L=L, prec=prec)
    sim.randomize_fields(seed=11, lo=lo, hi=hi)
    u, v = sim.get_fields()
    dt = np.float64 if prec == "Float64" else np.float32
    ru, rv = ref.random_fields((L, L, L), seed=11, lo=lo, hi=hi, dtype=dt)
    assert np.array_equal(u, ru) and np.array_equal(v, rv)
    assert u.min() >= lo and u.max() < hi
