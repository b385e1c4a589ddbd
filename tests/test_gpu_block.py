"""The small-grid block kernel (csrc/hip/block.hpp, k_block) vs the z-marching fused kernel.

k_block is one more candidate of the fused kernel's autotuner, so it must reproduce k_fused bit
for bit: same neighbour-sum order, Philox stream, boundary resets.  Checked from the benchmarks'
random init (rough data, every cell's noise draw matters) on grids where the x rows fill the
wave exactly (L = 64, the +x ghost added on lane 63), partly (L = 36, 42: the ghost is a lane)
and with rows that are not a multiple of the 4-row noise quads (L = 42), at both fuse depths; and
against the CPU golden backend (the reference's update, Simulation_CPU.jl:92-112).
"""
import numpy as np
import pytest
import torch

from grayscott_amd.models.grayscott import GrayScott
from grayscott_amd.parallel.decomp import init_domain
from grayscott_amd.utils.config import Settings

pytestmark = pytest.mark.gpu

BLOCKS = ["blk8x2w8", "blk4x4w8", "blk8x2w16", "blk4x4w16", "blk8x4w16", "blk8x2w16l", "blk4x4w16l"]


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from grayscott_amd.ops import native
    native.load("hip")
    yield
    native.fused_unpin()


def _run(L, fuse, steps, cfg=None, backend="AMDGPU", random=True):
    from grayscott_amd.ops import native
    if backend == "AMDGPU":
        if cfg is None:
            native.fused_unpin()
        else:
            native.fused_select(cfg)
    s = Settings(L=L, precision="Float32", F=0.02, k=0.048, dt=1.0, Du=0.2, Dv=0.1, noise=0.1,
                 backend=backend, seed=19)
    sim = GrayScott(s, init_domain(L, 1, 0), fuse=fuse)
    try:
        sim.init_fields()
        if random:
            sim.randomize_fields(seed=3)
        sim.iterate(steps)
        return sim.get_fields()
    finally:
        sim.close()


@pytest.mark.parametrize("L", [64, 42, 36])
@pytest.mark.parametrize("fuse", [2, 3])
def test_block_kernel_bitwise_vs_fused(L, fuse):
    steps = 4 * fuse + 1  # whole passes plus a remainder step
    ref = _run(L, fuse, steps, cfg="4x8:1s")
    for name in BLOCKS:
        u, v = _run(L, fuse, steps, cfg=name)
        np.testing.assert_array_equal(u, ref[0], err_msg=f"{name} u")
        np.testing.assert_array_equal(v, ref[1], err_msg=f"{name} v")


@pytest.mark.parametrize("fuse", [2, 3])
def test_block_kernel_vs_cpu_golden(fuse):
    g = _run(64, fuse, 30, cfg="blk8x2w8")
    c = _run(64, 1, 30, backend="CPU")
    assert np.abs(g[0] - c[0]).max() < 2e-5
    assert np.abs(g[1] - c[1]).max() < 2e-5


def test_block_kernel_from_seed_state():
    # the reference's own initial state (u = 1, v = 0, 13^3 seed cube): smooth data, boundary
    # values switching with the time parity
    ref = _run(64, 3, 20, cfg="4x8:1s", random=False)
    u, v = _run(64, 3, 20, cfg="blk4x4w8", random=False)
    np.testing.assert_array_equal(u, ref[0])
    np.testing.assert_array_equal(v, ref[1])


def test_autotuner_times_block_kernel_at_l64():
    """At L = 64 the tuner's candidate list includes the block kernels; whatever it picks must
    reproduce the pinned k_fused result."""
    from grayscott_amd.ops import native
    native.fused_unpin()
    s = Settings(L=64, precision="Float32", F=0.02, k=0.048, dt=1.0, Du=0.2, Dv=0.1, noise=0.1,
                 backend="AMDGPU", seed=19)
    sim = GrayScott(s, init_domain(64, 1, 0), fuse=2)
    try:
        sim.init_fields()
        sim.randomize_fields(seed=3)
        choice = sim.fused_choice()
        sim.iterate(9)
        got = sim.get_fields()
    finally:
        sim.close()
    print("L=64 tuned choice:", choice)
    ref = _run(64, 2, 9, cfg="4x8:1s")
    np.testing.assert_array_equal(got[0], ref[0])
    np.testing.assert_array_equal(got[1], ref[1])


def test_auto_depth_is_measured_single_rank():
    """fuse left to the engine (single rank): H = 3 ghosts, prepare() runs the depth with the
    lower tuned time per step (engine.h depth()); the result stays within the golden tolerance.
    (fp32: H = 4 since round 6, the LDS-ring kernel's T = 4 entry.)"""
    from grayscott_amd.ops import native
    native.fused_unpin()
    s = Settings(L=64, precision="Float32", F=0.02, k=0.048, dt=1.0, Du=0.2, Dv=0.1, noise=0.1,
                 backend="AMDGPU", seed=19)
    sim = GrayScott(s, init_domain(64, 1, 0))
    try:
        sim.init_fields()
        assert sim.fuse == 4 and sim.depth in (2, 3, 4)
        choice = sim.fused_choice()
        print("L=64 auto depth:", sim.depth, choice)
        per_step = {n: c[2] / n for n, c in choice.items()}
        assert sim.depth == min(per_step, key=per_step.get)
        sim.iterate(24)
        g = sim.get_fields()
    finally:
        sim.close()
    c = _run(64, 1, 24, backend="CPU", random=False)
    assert np.abs(g[0] - c[0]).max() < 2e-5
    assert np.abs(g[1] - c[1]).max() < 2e-5


@pytest.mark.parametrize("L,depth", [((64, 64, 32), 2), ((192, 160, 12), 3)])
def test_auto_depth_without_tuning_uses_plane_rule(L, depth, monkeypatch):
    """GS_AUTOTUNE=0: nothing is timed, so the engine falls back to the plane-size rule (T=2
    below 160^2 x-y planes, else the full depth up to T=3) instead of always running T=3."""
    from grayscott_amd.ops import native
    native.fused_unpin()
    monkeypatch.setenv("GS_AUTOTUNE", "0")
    s = Settings(L=L[0], precision="Float32", F=0.02, k=0.048, dt=1.0, Du=0.2, Dv=0.1,
                 noise=0.1, backend="AMDGPU", seed=19)
    sim = GrayScott(s, init_domain(L, 1, 0))
    try:
        sim.init_fields()
        assert sim.fuse == 4 and sim.depth == depth
        assert all(c[2] == 0.0 for c in sim.fused_choice().values())
    finally:
        sim.close()


@pytest.mark.parametrize("L,k,step", [((48, 40, 36), 2, 7), ((64, 40, 36), 3, 5), ((36, 36, 36), 2, 0)])
def test_block_kernel_raw_pass_reads_stored_ghosts(L, k, step):
    """A raw fused pass (the timing / overlap-test primitive gs_fused_runs_raw) runs without the
    engine's ensure_bc, so the stored x ghosts need not be the boundary value of the pass's time
    (here: the init's u = 1 ghosts at an odd step).  k_fused reads them from the buffer; k_block
    takes them to be the boundary value (it costs 5-10 % at L=64 to read them,
    profiles/r3_block.txt), so only Backend::fused() -- always after ensure_bc -- may launch it:
    a raw pass with a block shape pinned runs k_fused and matches it bit for bit."""
    from grayscott_amd.ops import native
    outs = []
    try:
        for cfg in ("4x8:1s", "blk8x2w8", "blk4x4w16"):
            native.fused_select(cfg)
            s = Settings(L=L[0], precision="Float32", F=0.02, k=0.048, dt=1.0, Du=0.2, Dv=0.1,
                         noise=0.1, backend="AMDGPU", seed=99)
            sim = GrayScott(s, init_domain(L, 1, 0), fuse=k)
            try:
                sim.init_fields()
                sim.randomize_fields(seed=11)
                sim.set_step(step)
                lib, h = sim.engine.lib, sim.engine.h
                nz = sim.domain.proc_sizes[2]
                native.check(lib, lib.gs_fused_runs_raw(h, k, 0, nz, 0, 0, 0, 0), "full")
                torch.cuda.synchronize()
                outs.append(sim.full_state(1 - sim.engine.current).cpu().numpy().copy())
            finally:
                sim.close()
    finally:
        native.fused_unpin()
    g = sim.geom
    nx, ny, nz = init_domain(L, 1, 0).proc_sizes
    inner = (slice(g.H, g.H + nz), slice(g.H, g.H + ny), slice(g.xo, g.xo + nx))
    for o in outs[1:]:
        np.testing.assert_array_equal(o[inner], outs[0][inner])
