"""Multi-rank data-path tuning (parallel/autotune.py) across 2 gloo ranks on the CPU: every
candidate is self-checked against the golden model and timed, and all ranks agree."""
import json
import os
import sys
import tempfile

import torch.multiprocessing as mp

from .mp_utils import ROOT, free_port


def _worker(rank, world, port, out):
    sys.path.insert(0, ROOT)
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": "0",
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port),
                       "OMP_NUM_THREADS": "1"})
    from grayscott_amd.parallel import autotune
    from grayscott_amd.parallel import dist as gdist
    from grayscott_amd.parallel.autotune import candidates, tune_data_path
    from grayscott_amd.utils.config import Settings

    # count the self-checks per transport (fail fast: a failed pinned transport is tried once)
    calls = []
    real = autotune.selfcheck

    def counting(ctx, backend, dims, fuse, transport, overlap, **kw):
        calls.append(transport)
        return real(ctx, backend, dims, fuse, transport, overlap, **kw)

    autotune.selfcheck = counting

    ctx = gdist.init_from_env("cpu")
    s = Settings(L=24, precision="Float32", F=0.02, k=0.048, dt=1.0, Du=0.2, Dv=0.1, noise=0.1,
                 backend="CPU", transport="auto")
    assert candidates(24, 2, "cpu") == [([2, 1, 1], 0, "auto")]
    # the third candidate pins the IPC transport, which the CPU backend cannot run: it must be
    # reported as failed without disturbing the others (no fallback chain for pinned transports)
    r = tune_data_path(s, ctx, 24, "cpu", cands=[([1, 1, 2], 1), ([2, 1, 1], 0),
                                                  ([1, 1, 2], 1, "auto", {}, "ipc"),
                                                  ([2, 1, 1], 0, "auto", {}, "ipc"),
                                                  ([2, 1, 1], 0, "off", {}, "ipc")],
                       steps=4, warmup=1)
    r["selfcheck_calls"] = calls
    with open(os.path.join(out, f"r{rank}.json"), "w") as fh:
        json.dump(r, fh)
    ctx.finalize()


def test_tune_data_path_two_ranks():
    with tempfile.TemporaryDirectory() as out:
        mp.start_processes(_worker, args=(2, free_port(), out), nprocs=2, join=True,
                           start_method="spawn")
        r0, r1 = (json.load(open(os.path.join(out, f"r{i}.json"))) for i in range(2))
    assert r0["dims"] == r1["dims"] and r0["dims"] in ([1, 1, 2], [2, 1, 1])
    assert [row["dims"] for row in r0["table"]] == [[1, 1, 2], [2, 1, 1], [1, 1, 2], [2, 1, 1],
                                                   [2, 1, 1]]
    assert all(row["ok"] and row["ms_per_step"] > 0 for row in r0["table"][:2])
    assert r0["table"][2]["transport_req"] == "ipc" and r0["table"][2]["ok"] is False
    assert "ipc" in r0["table"][2]["check_errors"][0]
    # fail fast: the later IPC rows are skipped with the first failure's reason, and IPC was
    # self-checked once on each rank
    for row in r0["table"][3:]:
        assert row["ok"] is False and row["skipped"].startswith("ipc failed: ")
        assert "check_errors" not in row
    assert r0["selfcheck_calls"].count("ipc") == 1 and r1["selfcheck_calls"].count("ipc") == 1
    assert r0["transport"] == "torch" and r0["fuse"] == 1


def test_candidates_for_mi355x():
    from grayscott_amd.parallel.autotune import candidates
    # the reference's Dims_create grid first (always timed, reported as reference_grid), then
    # z slabs with and without overlap
    assert candidates(512, 8, "hip") == [([2, 2, 2], 0, "auto"), ([1, 1, 8], 0, "auto"),
                                        ([1, 1, 8], 0, "off"), ([2, 2, 2], 0, "off"),
                                        ([2, 2, 2], 2, "auto"),
                                        ([1, 2, 4], 0, "auto"), ([1, 2, 4], 0, "off"),
                                        ([1, 1, 8], 0, "auto", {}, "ipc"),
                                        ([1, 1, 8], 0, "off", {}, "ipc"),
                                        ([2, 2, 2], 0, "auto", {}, "ipc"),
                                        ([2, 2, 2], 0, "off", {}, "ipc"),
                                        ([2, 2, 2], 2, "auto", {}, "ipc")]
    assert candidates(512, 1, "hip") == [([1, 1, 1], 0, "auto")]


def test_candidates_without_ipc(monkeypatch):
    from grayscott_amd.parallel.autotune import candidates
    monkeypatch.setenv("GS_TUNE_IPC", "0")
    assert all(len(c) < 5 for c in candidates(512, 8, "hip"))
