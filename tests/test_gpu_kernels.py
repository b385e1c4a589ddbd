"""gfx950 kernels vs the CPU golden backend and the plain-PyTorch reference.

Mirrors the reference's backend-parity test (test/unit/simulation/unit-Simulation_CUDA.jl:10-32,
CPU vs CUDA init for L = 8..128) and extends it to the time step, fused multi-step passes,
fp64 and the periodic extension.  Every test here needs an MI355X.
"""
import numpy as np
import pytest
import torch

from grayscott_amd.models.grayscott import GrayScott
from grayscott_amd.ops import reference as ref
from grayscott_amd.parallel.decomp import init_domain
from grayscott_amd.utils.config import Settings

pytestmark = pytest.mark.gpu


def _sim(backend, L, prec="Float32", noise=0.1, fuse=None, periodic=False, use_fused=True,
         steps=0, seed=11):
    s = Settings(L=L, precision=prec, F=0.02, k=0.048, dt=1.0, Du=0.2, Dv=0.1, noise=noise,
                 backend=backend, periodic=periodic, seed=seed)
    sim = GrayScott(s, init_domain(L, 1, 0, periodic=periodic), fuse=fuse, use_fused=use_fused)
    sim.init_fields()
    if steps:
        sim.iterate(steps)
    return sim


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from grayscott_amd.ops import native
    native.load("hip")  # fail loudly if the gfx950 library is missing


@pytest.mark.parametrize("L", [8, 16, 32, 64, 128])
def test_init_parity(L):
    g = _sim("AMDGPU", L)
    c = _sim("CPU", L)
    gu, gv = g.get_fields()
    cu, cv = c.get_fields()
    np.testing.assert_array_equal(gu, cu)
    np.testing.assert_array_equal(gv, cv)
    # ghosts follow the reference init too (u = 1 incl. ghosts, u_temp = 0)
    full = g.full_state(0).cpu().numpy()
    assert full[0, 0, g.geom.xo - 1, 0] == 1.0
    assert float(g.full_state(1).abs().max()) == 0.0


@pytest.mark.parametrize("prec,tol", [("Float32", 2e-5), ("Float64", 1e-12)])
@pytest.mark.parametrize("noise", [0.0, 0.1])
def test_step_matches_cpu(prec, tol, noise):
    g = _sim("AMDGPU", 24, prec, noise, fuse=1, steps=25)
    c = _sim("CPU", 24, prec, noise, fuse=1, steps=25)
    gu, gv = g.get_fields()
    cu, cv = c.get_fields()
    assert np.abs(gu - cu).max() < tol
    assert np.abs(gv - cv).max() < tol


def test_step_matches_torch_reference():
    L, n = 20, 9
    g = _sim("AMDGPU", L, "Float32", 0.1, fuse=1, steps=n, seed=3)
    u, v = ref.init_fields((L, L, L), dtype=np.float32)
    for t in range(n):
        u, v = ref.step(u, v, t, 0.02, 0.048, 1.0, 0.2, 0.1, 0.1, 3, backend="torch")
    gu, gv = g.get_fields()
    assert np.abs(gu - u).max() < 2e-5
    assert np.abs(gv - v).max() < 2e-5


@pytest.mark.parametrize("fuse", [2, 3, 4])
@pytest.mark.parametrize("prec", ["Float32", "Float64"])
def test_fused_passes_match_single_steps(fuse, prec):
    a = _sim("AMDGPU", 40, prec, 0.1, fuse=1, steps=23)
    b = _sim("AMDGPU", 40, prec, 0.1, fuse=fuse, steps=23)
    au, av = a.get_fields()
    bu, bv = b.get_fields()
    tol = 2e-5 if prec == "Float32" else 1e-12
    assert np.abs(au - bu).max() < tol
    assert np.abs(av - bv).max() < tol
    assert b.step == 23


def test_fused_kernel_vs_stepwise_bitwise_close():
    # temporally blocked kernel vs the same passes done as single steps (same fuse depth)
    a = _sim("AMDGPU", 64, "Float32", 0.1, fuse=2, use_fused=False, steps=16)
    b = _sim("AMDGPU", 64, "Float32", 0.1, fuse=2, use_fused=True, steps=16)
    au, av = a.get_fields()
    bu, bv = b.get_fields()
    assert np.abs(au - bu).max() < 1e-5
    assert np.abs(av - bv).max() < 1e-5


def test_periodic_matches_reference():
    L, n = 16, 6
    g = _sim("AMDGPU", L, "Float64", 0.1, fuse=2, periodic=True, steps=n, seed=5)
    u, v = ref.run(L, n, noise_amp=0.1, seed=5, periodic=True)
    gu, gv = g.get_fields()
    assert np.abs(gu - u).max() < 1e-12
    assert np.abs(gv - v).max() < 1e-12


def test_odd_and_non_multiple_of_4_sizes():
    for L in (13, 30, 66):
        g = _sim("AMDGPU", L, "Float64", 0.1, fuse=2, steps=7)
        c = _sim("CPU", L, "Float64", 0.1, fuse=1, steps=7)
        assert np.abs(g.get_fields()[0] - c.get_fields()[0]).max() < 1e-12


def test_stats_and_determinism():
    a = _sim("AMDGPU", 48, steps=30)
    b = _sim("AMDGPU", 48, steps=30)
    np.testing.assert_array_equal(a.get_fields()[0], b.get_fields()[0])
    s = a.stats()
    u, v = a.get_fields()
    assert abs(s[0] - u.astype(np.float64).sum()) < 1e-3 * u.size
    assert s[1] == pytest.approx(float(u.min()))
    assert s[5] == pytest.approx(float(v.max()))


def test_gpu_cli_run(tmp_path):
    """The reference CUDA job configuration (scripts/job_*: 1 rank, 1 GPU) on the HIP backend."""
    import os
    import subprocess
    import sys

    from grayscott_amd.io.bp4 import BP4Reader
    from grayscott_amd.utils.config import get_settings, write_settings_toml

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    s = get_settings([os.path.join(root, "tests", "functional", "config_amdgpu.toml")])
    s.steps, s.plotgap, s.checkpoint, s.checkpoint_freq = 200, 50, True, 100
    s.output, s.checkpoint_output = str(tmp_path / "gs.bp"), str(tmp_path / "ck.bp")
    cfg = str(tmp_path / "c.toml")
    write_settings_toml(s, cfg)
    r = subprocess.run([sys.executable, os.path.join(root, "gray-scott.py"), cfg],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    with BP4Reader(s.output) as rd:
        assert rd.steps == 4 and rd.read("step", 3) == 200
        u = rd.read("U", -1)
    c = _sim("CPU", 64, "Float32", 0.1, fuse=1, steps=200, seed=s.seed)
    assert np.abs(u - c.get_fields()[0]).max() < 1e-3
    with BP4Reader(s.checkpoint_output) as ck:
        assert ck.read("step") == 200


_CFG_SNIPPET = r"""
import sys, numpy as np
sys.path.insert(0, sys.argv[1])
from grayscott_amd.models.grayscott import GrayScott
from grayscott_amd.parallel.decomp import init_domain
from grayscott_amd.utils.config import Settings
out = []
for fused in (False, True):
    s = Settings(L=70, precision="Float32", F=0.02, k=0.048, dt=1.0, Du=0.2, Dv=0.1, noise=0.1,
                 backend="AMDGPU", seed=21)
    sim = GrayScott(s, init_domain(70, 1, 0), fuse=int(sys.argv[2]), use_fused=fused)
    sim.init_fields(); sim.iterate(17)
    out.append(sim.get_fields())
print(max(np.abs(out[0][0] - out[1][0]).max(), np.abs(out[0][1] - out[1][1]).max()))
"""


@pytest.mark.parametrize("cfg,sched", [
    ("4x8:1", 0), ("8x4:1", 0), ("4x12:2", 0), ("8x4:1s", 0), ("8x4:4s", 0), ("4x8:1s", 0),
    ("4x8:4s", 0), ("", 1), ("8x4:2", 1), ("4x8:4s", 1), ("", 2), ("4x8:1", 2), ("4x8:2", 0),
    ("4x12:3", 2), ("4x12:1s", 2), ("4x12:2s", 1), ("4x12:1", 0), ("4x16:1s", 2)])
@pytest.mark.parametrize("fuse", [2, 3])
def test_fused_tuning_configs_agree(cfg, sched, fuse):
    """Every selectable fused-kernel configuration / schedule reproduces the single-step path."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, GS_FUSED_CFG=cfg, GS_FUSED_SCHED=str(sched))
    r = subprocess.run([sys.executable, "-c", _CFG_SNIPPET, root, str(fuse)], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert float(r.stdout.strip().splitlines()[-1]) < 1e-5


@pytest.mark.parametrize("prec", ["Float32", "Float64"])
def test_autotuner_choice_is_valid_and_state_unchanged(prec):
    """prepare() (run by init_fields) times candidates on the live buffers: the initial state
    must still match the CPU init, and the chosen kernel must reproduce single steps."""
    g = _sim("AMDGPU", 72, prec, 0.1, fuse=3)
    c = _sim("CPU", 72, prec, 0.1, fuse=1)
    np.testing.assert_array_equal(g.get_fields()[0], c.get_fields()[0])
    choice = g.fused_choice()
    assert set(choice) == {2, 3}
    for name, sched, ms in choice.values():
        assert isinstance(name, str) and sched in (0, 1, 2) and ms > 0
    g.iterate(11)
    c.iterate(11)
    tol = 2e-5 if prec == "Float32" else 1e-12
    assert np.abs(g.get_fields()[0] - c.get_fields()[0]).max() < tol
    assert np.abs(g.get_fields()[1] - c.get_fields()[1]).max() < tol



@pytest.mark.parametrize("prec,L", [("Float32", 40), ("Float64", 40), ("Float32", 300)])
def test_snapshot_minmax_equals_host_scan(prec, L):
    """The output snapshot's min / max (k_extract_mm partials, reduced on the host) equal a scan
    of the snapshot itself, and the snapshot equals get_fields (nx = 300: two x chunks)."""
    g = _sim("AMDGPU", L, prec, 0.1, fuse=2)
    g.randomize_fields(seed=3, lo=-0.5, hi=1.5)
    g.iterate(5)
    u, v, wait, mm = g.snapshot_fields("t", minmax=True)
    wait()
    (a, b), (c, d) = mm()
    assert (a, b, c, d) == (u.min(), u.max(), v.min(), v.max())
    gu, gv = g.get_fields()
    np.testing.assert_array_equal(u, gu)
    np.testing.assert_array_equal(v, gv)
    g.close()


@pytest.mark.parametrize("L,fuse,sched", [(200, 3, 2), (256, 3, 1), (200, 2, 0), (96, 3, 2),
                                          (256, 2, 2)])
def test_fp64_lds_ring_bitwise_vs_register_ring(L, fuse, sched):
    """The fp64 LDS-ring shape (csrc/hip/fused.hpp "4x8:1sl": FCfg::LR + LRC -- level-0 planes by
    LDS-DMA into a PF + 1 ring, the centre plane from registers, Philox keys / step words in
    VGPRs) equals the register-ring production shape 4x8:1s bit for bit: edge tiles in x and y
    (L = 200), a z extent that leaves short chunks (L = 96), every schedule."""
    from grayscott_amd.models.grayscott import GrayScott
    from grayscott_amd.ops import native
    from grayscott_amd.parallel.decomp import init_domain
    from grayscott_amd.utils.config import Settings
    out = []
    try:
        for cfg in ("4x8:1s", "4x8:1sl"):
            native.fused_select(cfg)
            native.fused_sched(sched)
            s = Settings(L=L, precision="Float64", F=0.02, k=0.048, dt=1.0, Du=0.2, Dv=0.1,
                         noise=0.1, backend="AMDGPU", seed=31)
            sim = GrayScott(s, init_domain(L, 1, 0), fuse=fuse)
            try:
                sim.init_fields()
                sim.randomize_fields(seed=3)
                sim.iterate(4 * fuse + 1)
                out.append(sim.get_fields())
            finally:
                sim.close()
    finally:
        native.fused_unpin()
    assert np.isfinite(out[1][0]).all()
    np.testing.assert_array_equal(out[1][0], out[0][0])
    np.testing.assert_array_equal(out[1][1], out[0][1])


@pytest.mark.parametrize("prec,fuse,cfg,sched,steps", [
    ("Float32", 4, "4x12:1sl", 1, 240),    # T=4 LDS ring, unfolded (edge tiles at L=200)
    ("Float32", 2, "4x12:2sfl", 0, 240),   # T=2 LDS ring, 2-plane prefetch, folded, schedule 0
    ("Float64", 3, "4x8:1sl", 0, 120)])    # fp64 LDS ring (centre plane in registers)
def test_lds_ring_soak_bitwise_vs_register_ring(prec, fuse, cfg, sched, steps):
    """Soak of the LDS ring's hand-counted DMA waits (csrc/hip/fused.hpp lr_wait / pad_store): a
    long run through an LDS-ring shape equals the register-ring T=3 run bit for bit (every fused
    depth is bit-identical; the step counts avoid a single-step remainder, whose k_step1 kernel
    rounds differently).  A wait that lets a DMA piece land late shows up as a mismatch at a
    segment start (profiles/r6_f64_lr.txt, r6_lr_soak.txt)."""
    from grayscott_amd.models.grayscott import GrayScott
    from grayscott_amd.ops import native
    from grayscott_amd.parallel.decomp import init_domain
    from grayscott_amd.utils.config import Settings
    out = []
    try:
        for f, c, sc in ((3, "4x12:1s" if prec == "Float32" else "4x8:1s", 2), (fuse, cfg, sched)):
            native.fused_select(c)
            native.fused_sched(sc)
            s = Settings(L=200, precision=prec, F=0.02, k=0.048, dt=1.0, Du=0.2, Dv=0.1,
                         noise=0.1, backend="AMDGPU", seed=11)
            sim = GrayScott(s, init_domain(200, 1, 0), fuse=f)
            try:
                sim.init_fields()
                sim.randomize_fields(seed=5)
                sim.iterate(steps)
                out.append(sim.get_fields())
            finally:
                sim.close()
    finally:
        native.fused_unpin()
    np.testing.assert_array_equal(out[1][0], out[0][0])
    np.testing.assert_array_equal(out[1][1], out[0][1])
