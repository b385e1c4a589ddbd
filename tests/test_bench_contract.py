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


@pytest.mark.parametrize("decomp", ["z", "balanced"])
def test_bench_torchrun_two_ranks(decomp):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), "bench.py",
           "--gpus", "2", "--backend", "CPU", "--L", "32", "--steps", "6", "--warmup", "2",
           "--decomposition", decomp]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=600,
                       env=dict(os.environ, OMP_NUM_THREADS="1"))
    assert r.returncode == 0, r.stderr[-3000:]
    d = _last_json(r.stdout)
    assert KEYS <= set(d)
    tab = d["data_path_tuning"]
    assert len(tab) == 1 and tab[0]["ok"] and tab[0]["ms_per_step"] > 0
    assert d["config"]["dims"] == ([1, 1, 2] if decomp == "z" else [2, 1, 1])
