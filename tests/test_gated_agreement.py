"""Gated passes are agreed per depth across ranks: every depth 2..fuse can
run gated (prepare() tunes each; a planned or remainder pass of any depth takes the gated path),
and whether a rank can (gated_supported(k): gate_fits, per-depth occupancy, shared landing slots)
is per-rank state.  models/grayscott.py _agree_gated_depths reduces the per-depth mask over the
ranks and switches the failing depths off everywhere.  2-rank gloo test with engines whose
support differs per depth (the native engine's side is engine.h set_gated_depth / gated(k)).
"""
import os

import pytest
import torch.multiprocessing as mp


class _FakeEngine:
    def __init__(self, support):
        self.support = dict(support)
        self.off = set()

    def gated(self, k):
        return self.support.get(k, False) and k not in self.off

    def set_gated_depth(self, k, on):
        if not on:
            self.off.add(k)


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK="0", OMP_NUM_THREADS="1")
    from grayscott_amd.models.grayscott import _agree_gated_depths
    from grayscott_amd.parallel import dist as gdist
    ctx = gdist.init_from_env("cpu")
    # rank 0 cannot run depth 2 gated (e.g. its sub-domain fails gate_fits(2)); rank 1 can
    support = {2: rank == 1, 3: True, 4: False}
    eng = _FakeEngine(support)
    out = _agree_gated_depths(eng, ctx, 4)
    q.put((rank, out, sorted(eng.off), [eng.gated(k) for k in (2, 3, 4)]))
    ctx.finalize()


def test_ranks_agree_per_depth():
    from tests.mp_utils import free_port
    world = 2
    q = mp.get_context("spawn").Queue()
    port = free_port()
    procs = [mp.get_context("spawn").Process(target=_worker, args=(r, world, port, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, out, off, now in res:
        assert out == {2: False, 3: True, 4: False}, (rank, out)
        assert now == [False, True, False], (rank, now)
        assert 2 in off
