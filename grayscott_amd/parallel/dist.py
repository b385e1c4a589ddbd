"""Process-group bootstrap: one process per MI355X, torch.distributed control plane.

The reference bootstraps with ``MPI.Init`` (communication.jl:20) and uses MPI for everything.
Here the *control plane* (rendezvous, barriers, timing reductions, RCCL unique-id broadcast,
BP metadata gathers) is a torch.distributed **gloo** group created from the torchrun
environment (RANK / WORLD_SIZE / LOCAL_RANK / MASTER_ADDR / MASTER_PORT); the *data plane*
(halo exchange) is RCCL over xGMI, driven natively by ``libgs_hip.so``.
"""
from __future__ import annotations

import contextlib
import os
import sys
from dataclasses import dataclass
from datetime import timedelta
from typing import Any, List, Optional

import torch
import torch.distributed as dist

from .launch import launcher_env  # noqa: F401  (re-exported: the launcher table lives there)


@dataclass
class DistContext:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    initialized_here: bool = False
    _nccl_group: Any = None

    @property
    def is_distributed(self) -> bool:
        return self.world_size > 1 and dist.is_available() and dist.is_initialized()

    # -- control-plane collectives (cheap, CPU tensors over gloo) -------------------------
    def barrier(self) -> None:
        if self.is_distributed:
            dist.barrier()

    def allreduce(self, value: float, op: str = "max") -> float:
        if not self.is_distributed:
            return float(value)
        t = torch.tensor([float(value)], dtype=torch.float64)
        dist.all_reduce(t, op={"max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN,
                               "sum": dist.ReduceOp.SUM}[op])
        return float(t.item())

    def allreduce_array(self, values, op: str = "sum"):
        if not self.is_distributed:
            return [float(v) for v in values]
        t = torch.tensor([float(v) for v in values], dtype=torch.float64)
        dist.all_reduce(t, op={"max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN,
                               "sum": dist.ReduceOp.SUM}[op])
        return t.tolist()

    def gather_object(self, obj: Any, dst: int = 0) -> Optional[List[Any]]:
        if not self.is_distributed:
            return [obj]
        out = [None] * self.world_size if self.rank == dst else None
        dist.gather_object(obj, out, dst=dst)
        return out

    def allgather_object(self, obj: Any) -> List[Any]:
        if not self.is_distributed:
            return [obj]
        out = [None] * self.world_size
        dist.all_gather_object(out, obj)
        return out

    def broadcast_object(self, obj: Any, src: int = 0) -> Any:
        if not self.is_distributed:
            return obj
        lst = [obj]
        dist.broadcast_object_list(lst, src=src)
        return lst[0]

    def nccl_group(self):
        """Lazily created NCCL(RCCL) process group, for the torch halo transport on GPU."""
        if self._nccl_group is None:
            self._nccl_group = dist.new_group(backend="nccl")
        return self._nccl_group

    def finalize(self) -> None:
        if self.initialized_here and dist.is_initialized():
            dist.destroy_process_group()
            self.initialized_here = False


_CTX: Optional[DistContext] = None


def comm_timeout_s() -> float:
    """Seconds a control-plane collective or a device halo wait may block before the job is
    declared dead (GS_COMM_TIMEOUT, default 900; the RCCL watchdog reads the same variable)."""
    try:
        return max(1.0, float(os.environ.get("GS_COMM_TIMEOUT", "900")))
    except ValueError:
        return 900.0


def init_from_env(device: str = "cpu") -> DistContext:
    """Initialise (once) from the launcher's environment (torchrun, mpiexec, srun, or
    ``parallel.launch.spawn_local``).  Without torchrun, the gloo rendezvous uses MASTER_ADDR
    (default 127.0.0.1: one node) and MASTER_PORT (default 29531).  Every gloo collective is
    bounded by GS_COMM_TIMEOUT seconds, so a dead peer turns into an error, not a hang."""
    global _CTX
    if _CTX is not None:
        return _CTX
    rank, world, local = launcher_env()
    ctx = DistContext(rank=rank, world_size=world, local_rank=local)
    if device == "hip":
        torch.cuda.set_device(local % max(1, torch.cuda.device_count()))
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29531")
        with _stdout_to_stderr():  # gloo prints its connection report on fd 1
            dist.init_process_group(backend="gloo", rank=rank, world_size=world,
                                    timeout=timedelta(seconds=comm_timeout_s()))
        ctx.initialized_here = True
    _CTX = ctx
    return ctx


@contextlib.contextmanager
def _stdout_to_stderr():
    """Send what native code writes to fd 1 to fd 2 for the duration (stdout carries the
    benchmark's one JSON line; the gloo rendezvous prints "[Gloo] Rank 0 is connected to ..."
    there)."""
    sys.stdout.flush()
    try:
        saved = os.dup(1)
    except OSError:  # no usable fd 1
        yield
        return
    try:
        os.dup2(2, 1)
        yield
    finally:
        sys.stdout.flush()
        os.dup2(saved, 1)
        os.close(saved)


def reset() -> None:
    """Forget the cached context (tests)."""
    global _CTX
    if _CTX is not None:
        _CTX.finalize()
    _CTX = None
