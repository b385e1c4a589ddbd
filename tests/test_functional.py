"""Functional CLI runs (reference test/functional/functional-GrayScott.jl: `mpirun -n 4` of the
CPU configs, exit code 0) plus checkpoint/restart and fault-injection scenarios.  Ranks are
launched with torchrun on 127.0.0.1 (gloo control plane)."""
import os
import subprocess
import sys

import numpy as np
import pytest

from grayscott_amd.io.bp4 import BP4Reader
from grayscott_amd.utils.config import get_settings, write_settings_toml

from .mp_utils import ROOT, free_port

FUNC = os.path.join(ROOT, "tests", "functional")


def launch(cfg_path, nprocs, cwd, env=None, timeout=600):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node",
           str(nprocs), "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
           os.path.join(ROOT, "gray-scott.py"), cfg_path]
    e = dict(os.environ)
    e["OMP_NUM_THREADS"] = "1"
    e.update(env or {})
    return subprocess.run(cmd, cwd=cwd, env=e, capture_output=True, text=True, timeout=timeout)


def _cfg(tmp_path, name, **kw):
    s = get_settings([os.path.join(FUNC, "config_cpu_plain.toml")])
    for k, v in kw.items():
        setattr(s, k, v)
    p = str(tmp_path / name)
    write_settings_toml(s, p)
    return p


@pytest.mark.parametrize("cfg", ["config_cpu_plain.toml", "config_cpu_ka.toml"])
def test_functional_4_ranks(cfg, tmp_path):
    r = launch(os.path.join(FUNC, cfg), 4, str(tmp_path))
    assert r.returncode == 0, r.stderr[-3000:]
    with BP4Reader(str(tmp_path / "gs-4ranks-64L-F32.bp")) as rd:
        assert rd.steps == 100
        assert [rd.read("step", i) for i in (0, 1, 99)] == [10, 20, 1000]
        assert len(rd.variables(0)["U"].blocks) == 4
        u = rd.read("U", -1)
        assert np.isfinite(u).all() and u.shape == (64, 64, 64)


def test_decomposition_invariant_output(tmp_path):
    out = {}
    for n in (1, 3):
        d = tmp_path / f"r{n}"
        d.mkdir()
        cfg = _cfg(d, "c.toml", steps=30, plotgap=15, L=24, output="o.bp")
        r = launch(cfg, n, str(d))
        assert r.returncode == 0, r.stderr[-3000:]
        with BP4Reader(str(d / "o.bp")) as rd:
            out[n] = (rd.read("U", -1), rd.read("V", -1))
    np.testing.assert_array_equal(out[1][0], out[3][0])
    np.testing.assert_array_equal(out[1][1], out[3][1])


def _mpiexec():
    import shutil
    for c in (shutil.which("mpiexec"), "/opt/conda/bin/mpiexec"):
        if c and os.path.exists(c):
            return c
    return None


@pytest.mark.skipif(_mpiexec() is None, reason="no mpiexec on this machine")
def test_mpiexec_launch_4_ranks(tmp_path):
    """The reference's own launch form (`mpirun -n 4 ...`, functional-GrayScott.jl:9): ranks
    come from the MPI launcher's environment (PMI_RANK / OMPI_COMM_WORLD_RANK), same output as
    one rank."""
    out = {}
    for n in (1, 4):
        d = tmp_path / f"r{n}"
        d.mkdir()
        cfg = _cfg(d, "c.toml", steps=12, plotgap=6, L=24, output="o.bp")
        e = dict(os.environ, OMP_NUM_THREADS="1", MASTER_ADDR="127.0.0.1",
                 MASTER_PORT=str(free_port()))
        for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
            e.pop(k, None)
        r = subprocess.run([_mpiexec(), "-n", str(n), sys.executable,
                            os.path.join(ROOT, "gray-scott.py"), cfg], cwd=str(d), env=e,
                           capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-3000:]
        with BP4Reader(str(d / "o.bp")) as rd:
            assert rd.steps == 2
            assert len(rd.variables(0)["U"].blocks) == n
            out[n] = rd.read("U", -1)
    np.testing.assert_array_equal(out[1], out[4])


def test_launcher_env_mapping():
    from grayscott_amd.parallel.dist import launcher_env
    assert launcher_env({}) == (0, 1, 0)
    assert launcher_env({"PMI_RANK": "3", "PMI_SIZE": "4", "MPI_LOCALRANKID": "1"}) == (3, 4, 1)
    assert launcher_env({"OMPI_COMM_WORLD_RANK": "2", "OMPI_COMM_WORLD_SIZE": "8"}) == (2, 8, 2)
    assert launcher_env({"SLURM_PROCID": "5", "SLURM_NTASKS": "8", "SLURM_LOCALID": "5",
                         "RANK": "1", "WORLD_SIZE": "2"}) == (1, 2, 1)


def test_tuned_decomposition_run(tmp_path):
    """decomposition = "tune": the data path is self-checked and timed before the run, and the
    output equals a one-rank run."""
    out = {}
    for n, dec in ((1, "auto"), (2, "tune")):
        d = tmp_path / f"r{n}"
        d.mkdir()
        r = launch(_cfg(d, "c.toml", steps=12, plotgap=12, L=24, output="o.bp",
                        decomposition=dec), n, str(d))
        assert r.returncode == 0, r.stderr[-3000:]
        with BP4Reader(str(d / "o.bp")) as rd:
            out[n] = rd.read("U", -1)
    np.testing.assert_array_equal(out[1], out[2])


def test_checkpoint_restart_bitwise(tmp_path):
    """Run 40 steps straight vs 20 steps + restart (with a different rank count) to 40."""
    full = tmp_path / "full"
    full.mkdir()
    r = launch(_cfg(full, "c.toml", L=24, steps=40, plotgap=20, output="o.bp"), 2, str(full))
    assert r.returncode == 0, r.stderr[-3000:]
    part = tmp_path / "part"
    part.mkdir()
    r = launch(_cfg(part, "a.toml", L=24, steps=20, plotgap=20, output="a.bp", checkpoint=True,
                    checkpoint_freq=20, checkpoint_output="ck.bp"), 2, str(part))
    assert r.returncode == 0, r.stderr[-3000:]
    with BP4Reader(str(part / "ck.bp")) as ck:
        assert ck.read("step") == 20
        assert ck.process_groups(0)[0]["io"] == "SimulationCheckpoint"
    r = launch(_cfg(part, "b.toml", L=24, steps=40, plotgap=20, output="b.bp", restart=True,
                    restart_input="ck.bp"), 3, str(part))
    assert r.returncode == 0, r.stderr[-3000:]
    with BP4Reader(str(full / "o.bp")) as a, BP4Reader(str(part / "b.bp")) as b:
        # a new output file starts with the restart step (the restored state, bit for bit)
        assert [b.read("step", i) for i in range(b.steps)] == [20, 40]
        for i in range(2):
            np.testing.assert_array_equal(a.read("U", i), b.read("U", i))
            np.testing.assert_array_equal(a.read("V", i), b.read("V", i))


def test_fault_injection_and_recovery(tmp_path):
    """A run killed after step 30 resumes from its last checkpoint (step 30) and ends with the
    same output history as an uninterrupted run: the same step list (the restart keeps the
    steps written before the failure, cuts off nothing it needs, and rewrites the step the dead
    run had not committed) and bitwise the same U/V at every step."""
    ref = tmp_path / "ref"
    ref.mkdir()
    r = launch(_cfg(ref, "c.toml", L=20, steps=50, plotgap=10, output="o.bp"), 2, str(ref))
    assert r.returncode == 0, r.stderr[-3000:]
    run = tmp_path / "run"
    run.mkdir()
    cfg = _cfg(run, "c.toml", L=20, steps=50, plotgap=10, output="o.bp", checkpoint=True,
               checkpoint_freq=10, checkpoint_output="ck.bp")
    r = launch(cfg, 2, str(run), env={"GS_FAIL_AT_STEP": "30"})
    assert r.returncode != 0
    with BP4Reader(str(run / "ck.bp")) as ck:
        assert ck.read("step") == 30
    with BP4Reader(str(run / "o.bp")) as b:
        assert [b.read("step", i) for i in range(b.steps)] in ([10, 20], [10, 20, 30])
    # restart with another rank count: the subfiles of the dead run's ranks stay referenced
    cfg2 = _cfg(run, "c2.toml", L=20, steps=50, plotgap=10, output="o.bp", checkpoint=True,
                checkpoint_freq=10, checkpoint_output="ck.bp", restart=True, restart_input="ck.bp")
    r = launch(cfg2, 3, str(run))
    assert r.returncode == 0, r.stderr[-3000:]
    with BP4Reader(str(ref / "o.bp")) as a, BP4Reader(str(run / "o.bp")) as b:
        steps_a = [a.read("step", i) for i in range(a.steps)]
        steps_b = [b.read("step", i) for i in range(b.steps)]
        assert steps_a == steps_b == [10, 20, 30, 40, 50]
        for i in range(a.steps):
            np.testing.assert_array_equal(a.read("U", i), b.read("U", i))
            np.testing.assert_array_equal(a.read("V", i), b.read("V", i))
        assert b.attributes["F"] == a.attributes["F"]


def test_restart_cuts_off_later_output_steps(tmp_path):
    """Restarting from an older checkpoint drops the output steps written after it and
    continues the file from there (no duplicate or stale steps)."""
    run = tmp_path / "run"
    run.mkdir()
    # checkpoints every 10 steps into separate files: keep the step-20 one aside
    cfg = _cfg(run, "c.toml", L=16, steps=20, plotgap=5, output="o.bp", checkpoint=True,
               checkpoint_freq=20, checkpoint_output="ck20.bp")
    assert launch(cfg, 1, str(run)).returncode == 0
    cfg = _cfg(run, "c1.toml", L=16, steps=35, plotgap=5, output="o.bp", restart=True,
               restart_input="ck20.bp")
    assert launch(cfg, 2, str(run)).returncode == 0
    with BP4Reader(str(run / "o.bp")) as b:
        assert [b.read("step", i) for i in range(b.steps)] == [5, 10, 15, 20, 25, 30, 35]
    # now go back to step 20 again: 25..35 are cut off and rewritten
    cfg = _cfg(run, "c2.toml", L=16, steps=30, plotgap=5, output="o.bp", restart=True,
               restart_input="ck20.bp")
    assert launch(cfg, 1, str(run)).returncode == 0
    ref = tmp_path / "ref"
    ref.mkdir()
    assert launch(_cfg(ref, "c.toml", L=16, steps=30, plotgap=5, output="o.bp"), 1,
                  str(ref)).returncode == 0
    with BP4Reader(str(ref / "o.bp")) as a, BP4Reader(str(run / "o.bp")) as b:
        assert [b.read("step", i) for i in range(b.steps)] == [5, 10, 15, 20, 25, 30]
        for i in range(a.steps):
            np.testing.assert_array_equal(a.read("U", i), b.read("U", i))


def test_one_failing_rank_ends_the_job(tmp_path):
    """Job-wide failure handling: rank 1 of 4 raises at step 20; every rank exits
    non-zero on its own (no launcher kills them), well within GS_COMM_TIMEOUT."""
    import time

    from grayscott_amd.parallel.launch import free_port as fp
    from grayscott_amd.parallel.launch import worker_env
    cfg = _cfg(tmp_path, "c.toml", steps=60, plotgap=10, L=24, output=str(tmp_path / "o.bp"))
    port = fp()
    extra = {"OMP_NUM_THREADS": "1", "GS_RAISE_AT_STEP": "20", "GS_FAIL_RANK": "1",
             "GS_COMM_TIMEOUT": "120"}
    t0 = time.monotonic()
    procs = [subprocess.Popen([sys.executable, os.path.join(ROOT, "gray-scott.py"), cfg],
                              cwd=str(tmp_path), env=worker_env(r, 4, port, extra=extra),
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
             for r in range(4)]
    outs = []
    try:
        for p in procs:
            outs.append(p.communicate(timeout=100))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    codes = [p.returncode for p in procs]
    assert all(c != 0 for c in codes), (codes, [o[1][-800:] for o in outs])
    assert "injected failure on rank 1" in outs[1][1]
    assert time.monotonic() - t0 < 100
