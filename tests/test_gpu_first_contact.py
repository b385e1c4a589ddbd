"""First contact of a multi-GPU job is bounded.

The RCCL communicator is created non-blocking (``ncclCommInitRankConfig`` with
``blocking = 0``, csrc/hip/backend_hip.hip ``init_comm``) and its set-up is polled under
GS_COMM_TIMEOUT: a communicator of two ranks of which only one ever calls init must fail within
the timeout instead of blocking the process for good.  The reference simply hangs there
(``MPI.Init`` / ``Cart_create``, src/simulation/communication.jl:15-33).

The child process runs on the one GPU of the box; the test bounds it with its own timeout, so
a regression shows as a failed test, not a hung session.
"""
import os
import subprocess
import sys
import textwrap
import time

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = textwrap.dedent("""
    import os, sys, time
    sys.path.insert(0, {root!r})
    os.environ["GS_COMM_TIMEOUT"] = "6"
    import torch
    torch.cuda.set_device(0)
    from grayscott_amd.models.grayscott import GrayScott
    from grayscott_amd.ops import native
    from grayscott_amd.parallel.decomp import init_domain
    from grayscott_amd.utils.config import Settings
    s = Settings(L=16, precision="Float32", backend="AMDGPU", noise=0.1)
    sim = GrayScott(s, init_domain(16, 1, 0))
    uid = native.rccl_unique_id()
    t0 = time.monotonic()
    try:
        sim.engine.rccl_init(uid, 2, 0)   # rank 1 never joins
    except RuntimeError as ex:
        print("FAILED_IN", round(time.monotonic() - t0, 2), str(ex)[:300], flush=True)
    else:
        print("JOINED", flush=True)
    sim.close()
""")


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def test_rccl_init_without_peer_fails_within_timeout():
    t0 = time.monotonic()
    r = subprocess.run([sys.executable, "-c", CHILD.format(root=ROOT)], capture_output=True,
                       text=True, timeout=150)
    took = time.monotonic() - t0
    out = r.stdout
    assert "FAILED_IN" in out, (out[-2000:], r.stderr[-3000:])
    el = float(out.split("FAILED_IN", 1)[1].split()[0])
    # the set-up gave up after GS_COMM_TIMEOUT (6 s), not later
    assert 5.5 <= el < 30.0, out
    assert "GS_COMM_TIMEOUT" in out or "RCCL" in out, out
    assert took < 150
