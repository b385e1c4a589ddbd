"""Process-group bootstrap: one process per MI355X, torch.distributed control plane.

The reference bootstraps with ``MPI.Init`` (communication.jl:20) and uses MPI for everything.
Here the *control plane* (rendezvous, barriers, timing reductions, RCCL unique-id broadcast,
BP metadata gathers) is a torch.distributed **gloo** group created from the torchrun
environment (RANK / WORLD_SIZE / LOCAL_RANK / MASTER_ADDR / MASTER_PORT); the *data plane*
(halo exchange) is RCCL over xGMI, driven natively by ``libgs_hip.so``.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Any, List, Optional

import torch
import torch.distributed as dist


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


# Launcher environments: torchrun, then the MPI / batch launchers the reference is run with
# (`mpirun -n N`, test/functional/functional-GrayScott.jl:9; srun / jsrun in scripts/job_*.sh).
_LAUNCHERS = (
    ("RANK", "WORLD_SIZE", "LOCAL_RANK"),                                  # torchrun
    ("PMI_RANK", "PMI_SIZE", "MPI_LOCALRANKID"),                           # MPICH / hydra
    ("OMPI_COMM_WORLD_RANK", "OMPI_COMM_WORLD_SIZE", "OMPI_COMM_WORLD_LOCAL_RANK"),  # Open MPI
    ("SLURM_PROCID", "SLURM_NTASKS", "SLURM_LOCALID"),                     # srun
)


def launcher_env(env=None):
    """(rank, world_size, local_rank) from the first launcher whose variables are set."""
    env = os.environ if env is None else env
    for rk, sz, lc in _LAUNCHERS:
        if rk in env and sz in env:
            rank = int(env[rk])
            return rank, int(env[sz]), int(env.get(lc, rank))
    return 0, 1, 0


def init_from_env(device: str = "cpu") -> DistContext:
    """Initialise (once) from the launcher's environment (torchrun, mpiexec, srun).  Without
    torchrun, the gloo rendezvous uses MASTER_ADDR (default 127.0.0.1: one node) and
    MASTER_PORT (default 29531)."""
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
        dist.init_process_group(backend="gloo", rank=rank, world_size=world)
        ctx.initialized_here = True
    _CTX = ctx
    return ctx


def reset() -> None:
    """Forget the cached context (tests)."""
    global _CTX
    if _CTX is not None:
        _CTX.finalize()
    _CTX = None
