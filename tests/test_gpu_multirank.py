"""Multi-rank GPU runs on ONE MI355X (several processes share the device).

RCCL refuses two ranks on one GPU, so these use the host-staged gloo transport: they verify
the gfx950 pack/unpack kernels, the 26-direction halo plan and the fused kernel's ghost
handling across real process boundaries.  The RCCL transport itself runs in bench.py on the
8-GPU node.
"""
import numpy as np
import pytest
import torch

from .mp_utils import run_ranks

pytestmark = pytest.mark.gpu


def _cfg(L, steps, fuse, periodic=False, prec="Float32", transport="host"):
    return {"settings": dict(L=L, precision=prec, F=0.02, k=0.048, dt=1.0, Du=0.2, Dv=0.1,
                             noise=0.1, backend="AMDGPU", periodic=periodic, seed=1234),
            "steps": steps, "fuse": fuse, "transport": transport}


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


@pytest.mark.parametrize("world,L,fuse,periodic,prec", [
    (2, 48, 2, False, "Float32"),
    (4, 40, 2, False, "Float64"),
    (8, 36, 2, False, "Float32"),
    (4, 32, 3, True, "Float32"),
    (2, 30, 1, False, "Float64"),
])
def test_gpu_decomposed_matches_single_rank(world, L, fuse, periodic, prec):
    steps = 9
    u1, v1, _ = run_ranks(1, _cfg(L, steps, fuse, periodic, prec))
    un, vn, meta = run_ranks(world, _cfg(L, steps, fuse, periodic, prec))
    assert all(m["transport"] == "host" for m in meta)
    tol = 0 if prec == "Float64" else 0
    np.testing.assert_allclose(un, u1, rtol=0, atol=tol)
    np.testing.assert_allclose(vn, v1, rtol=0, atol=tol)


@pytest.mark.parametrize("world,L,fuse,prec,overlap", [
    (2, 48, 2, "Float32", "on"),
    (4, 64, 3, "Float32", "on"),
    (3, 40, 2, "Float64", "on"),
    (2, 48, 3, "Float32", "off"),
])
def test_gpu_z_slabs_overlap_matches_single_rank(world, L, fuse, prec, overlap):
    """z-slab decomposition: the inner planes run while the halo exchange is in flight on the
    comm stream, the boundary slabs after it lands -- bit-identical to one rank."""
    steps = 11
    u1, v1, _ = run_ranks(1, _cfg(L, steps, fuse, False, prec))
    cfg = _cfg(L, steps, fuse, False, prec)
    cfg["settings"].update(decomposition="z", overlap=overlap)
    un, vn, meta = run_ranks(world, cfg)
    assert all(m["zplanes"] for m in meta)
    assert all(m["overlapped"] == (overlap == "on") for m in meta)
    np.testing.assert_array_equal(un, u1)
    np.testing.assert_array_equal(vn, v1)


@pytest.mark.parametrize("world,L,fuse,prec,overlap", [
    (2, 48, 2, "Float32", "on"),
    (4, 64, 3, "Float32", "on"),
    (8, 64, 3, "Float32", "on"),
    (4, 40, 2, "Float64", "on"),
    (8, 48, 2, "Float32", "off"),
])
def test_gpu_balanced_overlap_matches_single_rank(world, L, fuse, prec, overlap):
    """Balanced (Dims_create) grid with packed halos: the inner tiles x inner planes run while
    pack / transport / unpack are in flight on the comm stream, then the z end slabs and the
    ring tiles -- bit-identical to one rank."""
    steps = 11
    u1, v1, _ = run_ranks(1, _cfg(L, steps, fuse, False, prec))
    cfg = _cfg(L, steps, fuse, False, prec)
    cfg["settings"].update(decomposition="balanced", overlap=overlap)
    un, vn, meta = run_ranks(world, cfg)
    assert not any(m["zplanes"] for m in meta)
    assert all(m["overlapped"] == (overlap == "on") for m in meta)
    np.testing.assert_array_equal(un, u1)
    np.testing.assert_array_equal(vn, v1)


@pytest.mark.parametrize("world,dims,L,fuse", [(4, [1, 2, 2], 64, 3), (8, [1, 2, 4], 64, 2)])
def test_gpu_hybrid_slabs_overlap_matches_single_rank(world, dims, L, fuse):
    """z slabs split along y (packed halos, one tile ring): overlapped passes with the ring
    tiles on the comm stream next to the z end slabs -- bit-identical to one rank."""
    steps = 11
    u1, v1, _ = run_ranks(1, _cfg(L, steps, fuse))
    cfg = _cfg(L, steps, fuse)
    cfg["settings"].update(overlap="on")
    cfg["dims"] = dims
    un, vn, meta = run_ranks(world, cfg)
    assert all(m["overlapped"] for m in meta)
    np.testing.assert_array_equal(un, u1)
    np.testing.assert_array_equal(vn, v1)


@pytest.mark.parametrize("world,L,fuse,decomp,overlap", [
    (1, 40, 3, "balanced", "auto"),
    (4, 40, 2, "balanced", "auto"),
    (2, 48, 2, "z", "on"),
])
def test_gpu_halo_poisoning(world, L, fuse, decomp, overlap):
    """NaN in every ghost / padding cell (incl. the fused kernel's masked lanes) never
    reaches the interior, with the fused kernel, the z-slab overlap and packed halos."""
    steps = 9
    u1, v1, _ = run_ranks(1, _cfg(L, steps, fuse))
    cfg = _cfg(L, steps, fuse)
    cfg["settings"].update(decomposition=decomp, overlap=overlap)
    cfg["poison"] = True
    un, vn, _ = run_ranks(world, cfg)
    assert np.isfinite(un).all() and np.isfinite(vn).all()
    np.testing.assert_array_equal(un, u1)
    np.testing.assert_array_equal(vn, v1)


def test_gpu_bench_two_ranks_tunes_data_path():
    """bench.py under torchrun with 2 ranks on the one GPU (host transport: RCCL refuses two
    ranks on one device): every candidate data path is self-checked and timed, the JSON line
    reports the table, and the timed run uses the winner."""
    import json
    import os
    import subprocess
    import sys

    from .mp_utils import ROOT, free_port
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), "bench.py",
           "--gpus", "2", "--L", "96", "--steps", "24", "--warmup", "6", "--transport", "host"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    tab = d["data_path_tuning"]
    # every row is timed, or left out by the link-probe model (parallel/autotune.py: modelled
    # more than 20 % slower than the best row; the reference grid never is)
    timed = [row for row in tab if not row.get("skipped")]
    assert len(timed) >= 3 and all(row["ok"] for row in timed)
    assert all(row["skipped"] == "model" and row["dims"] != [2, 1, 1]
               for row in tab if row.get("skipped")), tab
    assert d["link_probe"] is not None and d["link_probe"]["ipc"] == "ok"
    best = min(timed, key=lambda row: row["ms_per_step"])
    assert d["config"]["dims"] == best["dims"] and d["config"]["fuse_steps"] == best["fuse"]
    assert d["n_gpus"] == 2 and d["value"] > 0 and d["check"]["finite"]


def test_gpu_bench_eight_ranks_self_launch_small():
    """The driver's SCALE command shape at N=8, rehearsed on the one GPU at a small L with the
    default transport (auto + the IPC candidates): `python bench.py --gpus 8` starts the ranks
    itself, tunes the data path, and checks the TIMED configuration against the golden model
    on every rank's block afterwards (check.golden_ok)."""
    import json
    import os
    import subprocess
    import sys

    from .mp_utils import ROOT
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, "bench.py", "--gpus", "8", "--L", "64", "--steps", "6", "--warmup", "3",
           "--check-steps", "6", "--timeout", "420"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=480, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 8 and d["world"]["ranks"] == 8 and d["value"] > 0
    assert d["check"]["golden_ok"] and d["check"]["max_abs_err"] < 2e-5
    tab = d["data_path_tuning"]
    assert all(row.get("ok") or row.get("check_errors") or row.get("skipped") for row in tab)
