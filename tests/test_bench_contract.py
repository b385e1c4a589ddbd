"""bench.py contract (the driver's interface): one JSON line from rank 0 with the required keys,
for one process and for a torchrun multi-rank launch (gloo/CPU here; the GPU variant runs the
same code over RCCL on the driver's 8-GPU node).  The multi-rank run must pass its built-in
self-check of the data path against the golden model (parallel/autotune.py)."""
import json
import os
import subprocess
import sys

import pytest

from .mp_utils import free_port

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
        "scaling", "vs_baseline", "dtype", "data", "config"}


def _last_json(out: str) -> dict:
    lines = [l for l in out.strip().splitlines() if l.startswith("{")]
    assert len(lines) == 1, out[-2000:]
    return json.loads(lines[0])


def test_bench_single_process():
    r = subprocess.run([sys.executable, "bench.py", "--backend", "CPU", "--L", "32", "--steps", "6",
                        "--warmup", "2"], cwd=ROOT, capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, OMP_NUM_THREADS="2"))
    assert r.returncode == 0, r.stderr[-2000:]
    d = _last_json(r.stdout)
    assert KEYS <= set(d)
    assert d["steps"] == 6 and d["warmup"] == 2 and d["value"] > 0
    assert d["config"]["L"] == 32 and d["check"]["finite"]
    # the per-phase timing window after the timed region
    ph = d["phases"]["chosen"]["summary"]
    assert ph["passes"] == 10 and ph["pass_us"] > 0 and "step" in ph["phase_us"]


@pytest.mark.parametrize("decomp", ["z", "balanced"])
def test_bench_torchrun_two_ranks(decomp):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), "bench.py",
           "--gpus", "2", "--backend", "CPU", "--L", "32", "--steps", "6", "--warmup", "2",
           "--decomposition", decomp, "--check", "golden", "--check-steps", "4"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=600,
                       env=dict(os.environ, OMP_NUM_THREADS="1"))
    assert r.returncode == 0, r.stderr[-3000:]
    d = _last_json(r.stdout)
    assert len(r.stdout.strip().splitlines()) == 1, r.stdout[-2000:]
    assert KEYS <= set(d)
    tab = d["data_path_tuning"]
    assert len(tab) == 1 and tab[0]["ok"] and tab[0]["ms_per_step"] > 0
    assert d["config"]["dims"] == ([1, 1, 2] if decomp == "z" else [2, 1, 1])
    # the timed multi-rank path against the golden model on each rank's grown block: the CPU
    # backend runs the golden model's own kernel, so the blocks agree bit for bit
    assert d["check"]["golden_ok"] and d["check"]["max_abs_err"] == 0.0
    assert d["check"]["golden_steps"] == 4
    ph = d["phases"]["chosen"]
    assert len(ph["per_rank"]) == 2
    assert {"pack", "transport", "unpack"} <= set(ph["summary"]["phase_us"])
    assert ph["summary"]["bytes_per_neighbour_max"] > 0
    assert ph["summary"]["accounted"] is not None


def test_bench_self_launch_two_ranks():
    """`python bench.py --gpus 2` with no launcher starts both ranks itself (parallel/launch.py)
    and prints exactly one JSON line (rank 0's)."""
    env = dict(os.environ, OMP_NUM_THREADS="1")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--backend", "CPU", "--L", "32",
                        "--steps", "6", "--warmup", "2", "--decomposition", "balanced"],
                       cwd=ROOT, capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _last_json(r.stdout)
    # stdout is that one line and nothing else (the gloo rendezvous report goes to stderr)
    assert len(r.stdout.strip().splitlines()) == 1, r.stdout[-2000:]
    assert KEYS <= set(d)
    assert d["world"]["ranks"] == 2 and len(d["world"]["per_rank"]) == 2
    assert d["tuning_s"] >= 0 and d["wall_s"] > 0
    assert d["reference_grid"]["dims"] == [2, 1, 1]
    assert d["reference_grid"]["ms_per_step"] > 0


def test_bench_self_launch_propagates_failure():
    """A rank that fails makes the whole self-launched job fail (non-zero status, no hang)."""
    env = dict(os.environ, OMP_NUM_THREADS="1", GS_COMM_TIMEOUT="60", GS_RAISE_AT_STEP="0",
               GS_FAIL_RANK="1")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--backend", "CPU", "--L", "16",
                        "--steps", "2", "--warmup", "1", "--decomposition", "balanced"],
                       cwd=ROOT, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode != 0
    assert "injected failure on rank 1" in r.stderr
    # one parseable line all the same: no value, the status and the failing rank
    d = _last_json(r.stdout)
    assert KEYS <= set(d)
    assert d["value"] is None and d["status"] == "rank_failed" and d["failed_rank"] == 1


def _no_launcher_env(**extra):
    env = dict(os.environ, OMP_NUM_THREADS="1", **extra)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    return env


@pytest.mark.parametrize("launch", ["self", "torchrun"])
def test_bench_deadline_stalled_rank(launch):
    """A rank that stops answering (GS_STALL_AT_STEP on rank 1) while rank 0 waits in a
    collective: every rank gives up at the job's deadline, well before the control plane's
    own timeout, and stdout still carries exactly one parseable line (status "timeout", the
    phase rank 0 was in)."""
    import time
    env = _no_launcher_env(GS_COMM_TIMEOUT="300", GS_STALL_AT_STEP="0", GS_FAIL_RANK="1")
    args = ["bench.py", "--gpus", "2", "--backend", "CPU", "--L", "16", "--steps", "2",
            "--warmup", "1", "--decomposition", "balanced", "--deadline", "45"]
    if launch == "torchrun":
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node",
               "2", "--master-addr", "127.0.0.1", "--master-port", str(free_port())] + args
    else:
        cmd = [sys.executable] + args
    t0 = time.monotonic()
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=240, env=env)
    took = time.monotonic() - t0
    assert r.returncode != 0
    assert took < 150, took
    d = _last_json(r.stdout)
    assert KEYS <= set(d)
    assert d["value"] is None and d["status"] == "timeout" and d["deadline_s"] == 45
    assert d["phase"] == "warm-up"  # rank 0 waits for rank 1 in the barrier after it
    # the tuning rows finished before the stall are in the record
    assert len(d["data_path_tuning"]) == 1 and d["data_path_tuning"][0]["ok"]


def test_spawn_local_fail_fast(tmp_path):
    """spawn_local: one worker exits 3 at once, the other would sleep for minutes: the job ends
    within the grace period with the failing worker's status."""
    import time

    from grayscott_amd.parallel.launch import spawn_local
    prog = ("import os, sys, time\n"
            "r = int(os.environ['RANK'])\n"
            "assert os.environ['WORLD_SIZE'] == '2' and os.environ['MASTER_ADDR'] == '127.0.0.1'\n"
            "sys.exit(3) if r == 1 else time.sleep(300)\n")
    t0 = time.monotonic()
    rc = spawn_local(2, [sys.executable, "-c", prog], grace=2.0)
    assert rc == 3
    assert time.monotonic() - t0 < 60


def test_parallelism_label():
    """The JSON line's config.parallelism names the grid, and with neighbours the halo kind
    (in-place planes for z slabs, packed otherwise), the transport and the overlap."""
    import bench
    assert bench.parallelism_label([1, 1, 1], "none", False) == "spatial-3d 1x1x1"
    assert bench.parallelism_label([1, 1, 8], "ipc", True) == \
        "spatial-z-slabs 1x1x8 (ipc plane halos, overlapped)"
    assert bench.parallelism_label([2, 2, 2], "rccl", False) == "spatial-3d 2x2x2 (rccl packed halos)"
    assert bench.parallelism_label([2, 2, 1], "ipc", True) == \
        "spatial-3d 2x2x1 (ipc packed halos, overlapped)"
    assert bench.parallelism_label([2, 2, 2], "ipc", True, True) == \
        "spatial-3d 2x2x2 (ipc packed halos, gated)"
