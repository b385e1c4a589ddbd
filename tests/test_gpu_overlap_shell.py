"""Cell-granular comm/compute overlap on ONE MI355X: the inner launch (all tiles, outputs
clipped to >= k from the flagged faces) plus the face-slab shell (k_slab, slab.hpp) must write
every interior cell exactly once and equal the plain fused pass bit for bit -- the condition
for an overlapped multi-rank pass to equal the one-rank run.

Each case randomises the state, runs the full k-step pass into the spare buffer, poisons that
buffer's interior with NaN, then runs inner + shell into it and compares.  Single-rank
sub-domains (no transport): the flagged faces stand in for faces with neighbours, so the
global-boundary resets of intermediate levels, the noise counters at global offsets and the
periodic wrap are all exercised.
"""
import numpy as np
import pytest
import torch

from grayscott_amd.models.grayscott import GrayScott
from grayscott_amd.ops import native
from grayscott_amd.parallel.decomp import CartDomain, init_domain
from grayscott_amd.utils.config import Settings

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.set_device(0)


def _block(L, sizes, offsets):
    return CartDomain(nprocs=1, rank=0, L=tuple(L), dims=[1, 1, 1], coords=(0, 0, 0),
                      proc_sizes=list(sizes), proc_offsets=list(offsets), periodic=False,
                      nbr27=[-1] * 27)


def _interior(sim, which):
    g = sim.geom
    nx, ny, nz = sim.domain.proc_sizes
    return sim.full_state(which)[g.H:g.H + nz, g.H:g.H + ny, g.xo:g.xo + nx]


@pytest.mark.parametrize("variant", [0, 1])
@pytest.mark.parametrize("dom,k,prec,sides,step", [
    (init_domain((48, 40, 36), 1, 0), 3, "Float32", 63, 4),
    (init_domain((48, 40, 36), 1, 0), 2, "Float32", 63, 7),
    (init_domain((40, 36, 32), 1, 0), 3, "Float64", 63, 3),
    (init_domain((37, 29, 31), 1, 0), 3, "Float32", 63, 0),
    (init_domain((64, 48, 40), 1, 0), 3, "Float32", 2 | 8 | 32, 2),     # one-sided (config 3)
    (init_domain((64, 48, 40), 1, 0), 3, "Float32", 16 | 32, 5),        # z slabs only
    (init_domain((64, 48, 40), 1, 0), 3, "Float32", 1 | 4, 1),          # x / y faces only
    (init_domain(32, 1, 0, periodic=True), 3, "Float32", 63, 9),
    (init_domain(32, 1, 0, periodic=True), 2, "Float64", 63, 2),
    (_block((96, 80, 72), (40, 36, 28), (24, 20, 16)), 3, "Float32", 63, 6),  # interior block
    (_block((96, 80, 72), (40, 36, 28), (56, 44, 44)), 3, "Float32", 63, 6),  # at the + corner
    (_block((130, 64, 64), (130, 24, 20), (0, 17, 11)), 3, "Float32", 12 | 48, 3),  # odd oy
])
def test_inner_plus_shell_equals_full_pass(dom, k, prec, sides, step, variant):
    s = Settings(L=dom.L[0], precision=prec, F=0.02, k=0.048, dt=1.0, Du=0.2, Dv=0.1,
                 noise=0.1, backend="AMDGPU", seed=99)
    sim = GrayScott(s, dom, fuse=k)
    try:
        sim.init_fields()
        sim.randomize_fields(seed=11)
        sim.set_step(step)
        lib, h = sim.engine.lib, sim.engine.h
        cur = sim.engine.current
        nz = dom.proc_sizes[2]
        native.check(lib, lib.gs_fused_runs_raw(h, k, 0, nz, 0, 0, 0, 0), "full")
        torch.cuda.synchronize()
        ref = _interior(sim, 1 - cur).clone()
        _interior(sim, 1 - cur).fill_(float("nan"))
        torch.cuda.synchronize()
        z0 = k if sides & 16 else 0
        z1 = nz - k if sides & 32 else nz
        native.check(lib, lib.gs_fused_runs_raw(h, k, z0, z1 - z0, 0, 0, sides & 15, 1), "inner")
        native.check(lib, lib.gs_shell_raw(h, k, sides, variant), "shell")
        torch.cuda.synchronize()
        out = _interior(sim, 1 - cur).clone()
        assert torch.isfinite(ref).all()
        bad = ~torch.isfinite(out)
        assert not bad.any(), f"{int(bad.sum())} interior cells never written"
        np.testing.assert_array_equal(out.cpu().numpy(), ref.cpu().numpy())
    finally:
        sim.close()
