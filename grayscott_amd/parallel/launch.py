"""Single-node process launcher: one worker process per GPU, no external launcher needed.

The reference is started as ``mpirun -n N julia ... gray-scott.jl`` (test/functional/
functional-GrayScott.jl:9, scripts/job_*.sh).  Here ``torchrun`` / ``mpiexec`` / ``srun`` keep
working (``parallel/dist.py`` reads their environment), and a script can also launch itself:
``spawn_local`` starts N copies of a command with the torch.distributed rendezvous variables of
a one-node job (RANK, WORLD_SIZE, LOCAL_RANK, MASTER_ADDR=127.0.0.1, MASTER_PORT), waits for
all of them, and fails fast: when one worker exits non-zero, the others get ``grace`` seconds
and are then killed, so a dead rank never leaves its peers blocked in a collective.

This module imports nothing that touches the GPU (no torch): the parent of the workers must
never initialise HIP -- each worker owns its device, and a parent holding a HIP context would
also forbid replacing itself with another program on this platform.
"""
from __future__ import annotations

import os
import signal
import socket
import subprocess
import sys
import time
from typing import Dict, List, Optional, Sequence, Tuple

# Launcher environments: torchrun, then the MPI / batch launchers the reference is run with
# (`mpirun -n N`, test/functional/functional-GrayScott.jl:9; srun / jsrun in scripts/job_*.sh).
LAUNCHERS = (
    ("RANK", "WORLD_SIZE", "LOCAL_RANK"),                                  # torchrun / spawn_local
    ("PMI_RANK", "PMI_SIZE", "MPI_LOCALRANKID"),                           # MPICH / hydra
    ("OMPI_COMM_WORLD_RANK", "OMPI_COMM_WORLD_SIZE", "OMPI_COMM_WORLD_LOCAL_RANK"),  # Open MPI
    ("SLURM_PROCID", "SLURM_NTASKS", "SLURM_LOCALID"),                     # srun
)


def launcher_env(env=None) -> Tuple[int, int, int]:
    """(rank, world_size, local_rank) from the first launcher whose variables are set."""
    env = os.environ if env is None else env
    for rk, sz, lc in LAUNCHERS:
        if rk in env and sz in env:
            rank = int(env[rk])
            return rank, int(env[sz]), int(env.get(lc, rank))
    return 0, 1, 0


def under_launcher(env=None) -> bool:
    """Whether this process is one rank of a launched multi-process job."""
    return launcher_env(env)[1] > 1


def free_port(host: str = "127.0.0.1") -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind((host, 0))
        return s.getsockname()[1]


def worker_env(rank: int, nprocs: int, port: int, base: Optional[Dict[str, str]] = None,
               extra: Optional[Dict[str, str]] = None) -> Dict[str, str]:
    env = dict(os.environ if base is None else base)
    # a stale launcher context of another kind must not shadow ours (launcher_env order)
    for rk, sz, lc in LAUNCHERS[1:]:
        for k in (rk, sz, lc):
            env.pop(k, None)
    env.update({"RANK": str(rank), "WORLD_SIZE": str(nprocs), "LOCAL_RANK": str(rank),
                "LOCAL_WORLD_SIZE": str(nprocs), "GROUP_RANK": "0",
                "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port),
                "GS_SPAWNED": "1"})
    if extra:
        env.update(extra)
    return env


def spawn_local(nprocs: int, cmd: Sequence[str], *, port: Optional[int] = None,
                extra_env: Optional[Dict[str, str]] = None, timeout: Optional[float] = None,
                grace: float = 30.0, cwd: Optional[str] = None,
                rank0_stdout=None, others_stdout=None, poll: float = 0.05,
                info: Optional[dict] = None) -> int:
    """Run ``cmd`` as ``nprocs`` local ranks and return the job's exit status.

    Rank 0's stdout goes to ``rank0_stdout`` (default: this process's stdout); the other ranks'
    stdout goes to ``others_stdout`` (default: this process's stderr), so only rank 0 can print
    a result line.  stderr is inherited.  The status is 0 only if every rank exited 0; otherwise
    it is the first failure's code (negative signal numbers mapped to 128 + signal).  A rank
    still running ``grace`` seconds after another failed, or when ``timeout`` expires, is
    terminated (SIGTERM, then SIGKILL 10 s later) -- each by the PID this call started.
    ``info`` (a dict, filled in): ``failed_rank`` (the first rank seen failing, or None),
    ``timed_out`` (the ``timeout`` ended the job) and ``codes`` (every rank's exit status)."""
    port = port or free_port()
    out0 = rank0_stdout if rank0_stdout is not None else sys.stdout
    outn = others_stdout if others_stdout is not None else sys.stderr
    try:
        out0.flush()
        outn.flush()
    except Exception:
        pass
    procs: List[subprocess.Popen] = []
    try:
        for r in range(nprocs):
            procs.append(subprocess.Popen(list(cmd), cwd=cwd,
                                          env=worker_env(r, nprocs, port, extra=extra_env),
                                          stdout=out0 if r == 0 else outn))
        t0 = time.monotonic()
        first_fail: Optional[int] = None
        failed_rank: Optional[int] = None
        timed_out = False
        fail_time = None
        while True:
            codes = [p.poll() for p in procs]
            if all(c is not None for c in codes):
                break
            for r, c in enumerate(codes):
                if c not in (None, 0) and first_fail is None:
                    first_fail = _status(c)
                    failed_rank = r
                    fail_time = time.monotonic()
            now = time.monotonic()
            if ((fail_time is not None and now - fail_time > grace) or
                    (timeout is not None and now - t0 > timeout)):
                if first_fail is None:
                    first_fail = 124  # timeout(1)'s status
                    timed_out = True
                _terminate(procs)
                break
            time.sleep(poll)
        codes = [p.wait() for p in procs]
        if first_fail is None:
            bad = [(r, _status(c)) for r, c in enumerate(codes) if c != 0]
            if bad:
                failed_rank, first_fail = bad[0]
            else:
                first_fail = 0
        if info is not None:
            info.update(failed_rank=failed_rank, timed_out=timed_out,
                        codes=[_status(c) for c in codes])
        return first_fail
    except BaseException:
        _terminate(procs)
        raise


def _status(code: int) -> int:
    return 128 - code if code < 0 else code


def _terminate(procs: Sequence[subprocess.Popen], wait: float = 10.0) -> None:
    alive = [p for p in procs if p.poll() is None]
    for p in alive:
        try:
            p.send_signal(signal.SIGTERM)
        except ProcessLookupError:
            pass
    t0 = time.monotonic()
    while any(p.poll() is None for p in alive) and time.monotonic() - t0 < wait:
        time.sleep(0.05)
    for p in alive:
        if p.poll() is None:
            try:
                p.kill()
            except ProcessLookupError:
                pass
    for p in alive:
        try:
            p.wait(timeout=wait)
        except subprocess.TimeoutExpired:
            pass
