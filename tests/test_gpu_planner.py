"""The pass-depth planner on the MI355X with the outer-ghost refresh priced (engine.h
plan_depths / Engine::plan_passes, Engine::fill_ms): prepare() times one ensure_bc refresh, the
plan groups its passes by depth parity (at most one refresh inside a window, none at its start
when the first group matches the other buffer's ghosts), and the planned run still matches the
CPU golden model.  Reference step loop being scheduled: src/GrayScott.jl:81-96."""
import numpy as np
import pytest
import torch

from grayscott_amd.models.grayscott import GrayScott
from grayscott_amd.parallel.decomp import init_domain
from grayscott_amd.utils.config import Settings

pytestmark = pytest.mark.gpu

PHYS = dict(F=0.02, k=0.048, dt=1.0, Du=0.2, Dv=0.1)


@pytest.fixture(autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from grayscott_amd.ops import native
    native.load("hip")
    native.fused_unpin()
    yield
    native.fused_unpin()


def _switches(plan):
    return sum(1 for a, b in zip(plan, plan[1:]) if (a & 1) != (b & 1))


def _cpu(L, steps):
    s = Settings(L=L, precision="Float32", noise=0.1, backend="CPU", seed=2024, **PHYS)
    sim = GrayScott(s, init_domain(L, 1, 0), fuse=1)
    try:
        sim.init_fields()
        sim.iterate(steps)
        return sim.get_fields()
    finally:
        sim.close()


@pytest.mark.parametrize("L", [192, 256])
def test_refresh_priced_plans_match_golden(L, debug_knob):
    """From the reference's seed-cube state (its boundary ghosts switch with the time parity):
    windows of 5, 20 and 23 steps as planned, then the CPU golden model over the same 48."""
    s = Settings(L=L, precision="Float32", noise=0.1, backend="AMDGPU", seed=2024, **PHYS)
    sim = GrayScott(s, init_domain(L, 1, 0))
    try:
        sim.init_fields()
        fill = sim.engine.fill_ms()
        assert 0.0 < fill < 0.5, fill  # six ghost faces: microseconds, not a pass
        plans = []
        for n in (5, 20, 23):
            p = sim.engine.plan_passes(n)
            assert sum(p) == n and _switches(p) <= 1, p
            plans.append(p)
            sim.iterate(n)
        debug_knob("plan_fill", 0)
        plain = sim.engine.plan_passes(20)
        assert sum(plain) == 20
        u, v = sim.get_fields()
    finally:
        sim.close()
    gu, gv = _cpu(L, 48)
    err = max(float(np.abs(u - gu).max()), float(np.abs(v - gv).max()))
    print(f"L={L} refresh {fill * 1e3:.1f} us plans {plans} (unpriced: {plain}) max|d| {err:.2e}")
    assert err < 2e-5, err
