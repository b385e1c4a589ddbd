"""Halo-exchange transports.

The reference exchanges six faces per field with 12 blocking, host-staged ``MPI.Sendrecv!``
calls (communication.jl:138-199, vector datatypes :109-126) -- and on GPUs never copies the
result back (defect D1).  Here the native scheduler packs every outgoing slab (faces, and
edges/corners when several steps are fused per exchange) of BOTH fields into one contiguous
buffer, so a neighbour pair exchanges exactly one message per direction.  The buffers are
moved by one of:

* ``rccl``  -- native ``ncclSend``/``ncclRecv`` in one ``ncclGroupStart/End`` on the compute
               stream, issued from C++ (libgs_hip.so) -- the production path on MI355X/xGMI.
* ``torch`` -- ``torch.distributed.batch_isend_irecv`` called back from the native scheduler
               on the buffers' device (gloo for the CPU backend, NCCL/RCCL for GPU buffers).
* ``host``  -- the same over gloo with the GPU buffers staged through pinned host memory.
               Slow, but it lets several ranks share one GPU (RCCL refuses duplicate GPUs),
               which is how the multi-rank GPU path is tested on a single MI355X.
"""
from __future__ import annotations

from typing import List, Optional

import torch
import torch.distributed as dist


class TorchTransport:
    """Callback transport over torch.distributed point-to-point ops.

    Tags encode the direction so that gloo matches messages unambiguously: the send towards
    direction ``d`` carries tag ``d`` and lands in the peer's ghost ``26 - d``.
    """

    def __init__(self, plan: dict, send: torch.Tensor, recv: torch.Tensor, rank: int,
                 group=None, stage_host: bool = False):
        self.rank = rank
        self.group = group
        self.stage_host = stage_host and send.is_cuda
        self.send_dev, self.recv_dev = send, recv
        if self.stage_host:
            self.send = torch.empty(send.shape, dtype=send.dtype, pin_memory=True)
            self.recv = torch.empty(recv.shape, dtype=recv.dtype, pin_memory=True)
        else:
            self.send, self.recv = send, recv
        self.send_views = []
        self.recv_views = []
        # `send`/`recv` are flat tensors of scalars: 2 scalars (u, v) per cell
        for m in plan["send"]:
            if m["peer"] == rank:
                continue
            self.send_views.append((m["peer"], m["dir"],
                                    self.send[2 * m["offset"]: 2 * (m["offset"] + m["cells"])]))
        self.recv_pairs = []
        for m in plan["recv"]:
            if m["peer"] == rank:
                continue
            sl = slice(2 * m["offset"], 2 * (m["offset"] + m["cells"]))
            self.recv_views.append((m["peer"], 26 - m["dir"], self.recv[sl]))
            self.recv_pairs.append((recv[sl], self.recv[sl]))

    def __call__(self) -> None:
        if self.stage_host:
            self.send.copy_(self.send_dev)
        ops: List[dist.P2POp] = []
        for peer, tag, view in self.recv_views:
            ops.append(dist.P2POp(dist.irecv, view, peer, group=self.group, tag=tag))
        for peer, tag, view in self.send_views:
            ops.append(dist.P2POp(dist.isend, view, peer, group=self.group, tag=tag))
        if ops:
            for w in dist.batch_isend_irecv(ops):
                w.wait()
        if self.stage_host:
            # only the remote segments: self-messages were written natively on the device
            for dev_view, host_view in self.recv_pairs:
                dev_view.copy_(host_view, non_blocking=True)
