"""Correctness at the headline configuration (BASELINE.json: L=512 fp32, random-init u/v, noise
0.1) and at L=256: the production fused kernels against the native OpenMP golden model with the
same Philox stream, the pattern of the reference's backend-parity test
(test/unit/simulation/unit-Simulation_CUDA.jl:10-32, CPU vs GPU).

Each case runs in its own process: pinned tile/schedule choices are process-wide settings
(GS_FUSED_CFG / GS_FUSED_SCHED), and the autotuned case must see a fresh autotuner.
"""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_SNIPPET = r"""
import sys, numpy as np, torch
sys.path.insert(0, sys.argv[1])
from grayscott_amd.models.grayscott import GrayScott
from grayscott_amd.parallel.decomp import init_domain
from grayscott_amd.utils.config import Settings
L, prec, fuse, steps = int(sys.argv[2]), sys.argv[3], int(sys.argv[4]), int(sys.argv[5])
if len(sys.argv) > 6 and sys.argv[6] == "philox_generic":
    from grayscott_amd.ops import native
    native.debug_set("philox_generic", 1)
sims = {}
for backend in ("AMDGPU", "CPU"):
    s = Settings(L=L, precision=prec, F=0.02, k=0.048, dt=1.0, Du=0.2, Dv=0.1, noise=0.1,
                 backend=backend, seed=2024)
    sims[backend] = GrayScott(s, init_domain(L, 1, 0), fuse=fuse if backend == "AMDGPU" else 1)
    sims[backend].init_fields()
g, c = sims["AMDGPU"], sims["CPU"]
g.randomize_fields(seed=7)
u0, v0 = g.get_fields()
c.set_fields(u0, v0)
g.iterate(steps)
c.iterate(steps)
gu, gv = g.get_fields()
cu, cv = c.get_fields()
assert np.isfinite(gu).all() and np.isfinite(gv).all()
err = max(float(np.abs(gu - cu).max()), float(np.abs(gv - cv).max()))
import hashlib
ch = g.fused_choice()
print("digest", hashlib.sha1(gu.tobytes() + gv.tobytes()).hexdigest())
print("choice", {k: (v[0], v[1]) for k, v in ch.items()})
print(err)
"""


def _run(L, prec, fuse, steps, env=None, timeout=600, extra=()):
    e = dict(os.environ)
    e.update(env or {})
    r = subprocess.run([sys.executable, "-c", _SNIPPET, ROOT, str(L), prec, str(fuse), str(steps),
                        *extra],
                       env=e, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = r.stdout.strip().splitlines()
    return float(lines[-1]), lines[-2] + " " + lines[-3]


@pytest.mark.parametrize("L", [256, 512])
def test_headline_autotuned_t3_matches_golden(L):
    """The autotuned T=3 choice (the bench path) on random data, 9 steps = 3 fused passes."""
    err, choice = _run(L, "Float32", 3, 9)
    assert err < 2e-5, (err, choice)


@pytest.mark.parametrize("cfg,sched,L", [("4x12:2s", 2, 512), ("4x12:1s", 1, 512),
                                         ("4x12:2s", 1, 256), ("4x8:1s", 2, 256)])
def test_headline_pinned_tiles_match_golden(cfg, sched, L):
    """Pinned production tiles / schedules at T=3 (the ones the autotuner picks at L >= 256)."""
    err, choice = _run(L, "Float32", 3, 6, env={"GS_FUSED_CFG": cfg, "GS_FUSED_SCHED": str(sched)})
    assert err < 2e-5, (err, choice)


@pytest.mark.parametrize("L,fuse,sched", [(256, 3, 1), (256, 3, 2), (128, 3, 2), (128, 2, 1),
                                           (192, 3, 0)])
def test_folded_strip_matches_golden_and_plain_tile(L, fuse, sched):
    """4x12:1sf (fused.hpp FCfg::FOLD): the last x strip's narrow tiles run two per wave (lanes
    0-31 one y-tile, 32-63 the next).  Against the golden model, and bit for bit against the
    same tile without folding (every tile choice computes the same bits).  The last strip
    holds 24 outputs at L=256 T=3, 12 at L=128 T=3, 8 at L=128 T=2 and 18 at L=192 T=3 (<= 32 - 2T:
    all fold); schedules 0, 1 and 2."""
    env = {"GS_FUSED_CFG": "4x12:1sf", "GS_FUSED_SCHED": str(sched)}
    err, choice = _run(L, "Float32", fuse, 2 * fuse, env=env)
    assert err < 2e-5, (err, choice)
    err2, choice2 = _run(L, "Float32", fuse, 2 * fuse,
                         env={"GS_FUSED_CFG": "4x12:1s", "GS_FUSED_SCHED": str(sched)})
    d1 = [w for w in choice.split() if len(w) == 40][0]
    d2 = [w for w in choice2.split() if len(w) == 40][0]
    assert d1 == d2, (choice, choice2)


def test_headline_fp64_t2_matches_golden():
    """fp64 at T=2 (its default depth), L=256, autotuned tile."""
    err, choice = _run(256, "Float64", 2, 6)
    assert err < 1e-12, (err, choice)


def test_philox_q32_path_matches_generic():
    """The 32-bit-counter Philox path (rounds 1-3 on the SALU) and the generic 64-bit one give
    bit-identical results: same stream, same kernel otherwise."""
    a, da = _run(96, "Float32", 3, 6)
    b, db = _run(96, "Float32", 3, 6, extra=("philox_generic",))
    assert a < 2e-5 and b < 2e-5
    digest = lambda info: info.split("digest ")[1].split()[0]  # noqa: E731
    assert digest(da) == digest(db)


def test_production_library_rejects_ablation_variants():
    """Wrong-by-design ablation kernels exist only in the `make ablation` build."""
    from grayscott_amd.ops import native
    assert native.fused_cfg_lookup("4x12:2s-abl1") == -1
    assert native.fused_cfg_lookup("4x12:2s-abl2") == -1
    assert native.fused_cfg_lookup("4x12:2s") > 0
    with pytest.raises(ValueError):
        native.fused_select("4x12:2s-abl1")

