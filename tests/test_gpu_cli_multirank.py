"""The user CLI (gray-scott.py) with several ranks on the MI355X: the reference's functional test
(test/functional/functional-GrayScott.jl: `mpirun -n 4` of a config, exit code 0, output read
back) on the HIP backend, launched with torchrun on 127.0.0.1.  The ranks share the one card of
the box (IPC peer stores between processes on one device; RCCL refuses several ranks per device,
so "auto" takes the host path), and the aggregated BP4 output must equal the one-rank run's bit
for bit -- the decomposition, the halo transport, the per-rank output blocks and the reader all
in one check."""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from grayscott_amd.io.bp4 import BP4Reader
from grayscott_amd.utils.config import get_settings, write_settings_toml

from .mp_utils import ROOT, free_port

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _run(d, nprocs, transport):
    s = get_settings([os.path.join(ROOT, "tests", "functional", "config_amdgpu.toml")])
    s.L, s.steps, s.plotgap, s.output = 48, 24, 12, "o.bp"
    s.transport = transport
    cfg = str(d / "c.toml")
    write_settings_toml(s, cfg)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node",
           str(nprocs), "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
           os.path.join(ROOT, "gray-scott.py"), cfg]
    e = dict(os.environ)
    e["OMP_NUM_THREADS"] = "1"
    e.setdefault("GS_COMM_TIMEOUT", "60")
    r = subprocess.run(cmd, cwd=str(d), env=e, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    with BP4Reader(str(d / "o.bp")) as rd:
        assert rd.steps == 2 and rd.read("step", 1) == 24
        assert len(rd.variables(0)["U"].blocks) == nprocs
        return rd.read("U", -1), rd.read("V", -1)


@pytest.mark.parametrize("transport", ["ipc", "auto"])
def test_cli_four_ranks_match_one_rank(tmp_path, transport):
    out = {}
    for n in (1, 4):
        d = tmp_path / f"r{n}"
        d.mkdir()
        out[n] = _run(d, n, transport)
    np.testing.assert_array_equal(out[1][0], out[4][0])
    np.testing.assert_array_equal(out[1][1], out[4][1])
    assert np.isfinite(out[4][0]).all() and out[4][0].shape == (48, 48, 48)
