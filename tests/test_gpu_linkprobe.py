"""The link probe (csrc/hip/probe.hpp, parallel/linkprobe.py) on ONE MI355X: ranks sharing the
device still map each other's buffers through IPC and time their puts (the xGMI hop is what an
8-GPU node adds); RCCL refuses two ranks on one device, which the probe must report -- agreed by
every rank, within seconds -- instead of hanging.  The 8-GPU numbers come from the driver's
bench runs (bench.py link_probe)."""
import json
import os
import sys
import tempfile
import traceback

import pytest
import torch
import torch.multiprocessing as mp

from .mp_utils import ROOT, free_port

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _worker(rank, world, port, outdir):
    try:
        sys.path.insert(0, ROOT)
        os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": "0",
                           "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port),
                           "GS_COMM_TIMEOUT": "60"})
        from grayscott_amd.parallel import dist as gdist
        from grayscott_amd.parallel.linkprobe import probe_links
        ctx = gdist.init_from_env("hip")
        out = probe_links(ctx, reps=3)
        with open(os.path.join(outdir, f"rank{rank}.json"), "w") as f:
            json.dump(out, f)
        ctx.barrier()
        ctx.finalize()
    except Exception:
        with open(os.path.join(outdir, f"error{rank}.txt"), "w") as fh:
            fh.write(traceback.format_exc())
        raise


@pytest.mark.parametrize("world", [2, 3])
def test_link_probe_on_one_gpu(world):
    port = free_port()
    with tempfile.TemporaryDirectory() as outdir:
        pc = mp.start_processes(_worker, args=(world, port, outdir), nprocs=world, join=False,
                                start_method="spawn")
        while not pc.join(120):
            pass
        errs = [f for f in os.listdir(outdir) if f.startswith("error")]
        assert not errs, open(os.path.join(outdir, errs[0])).read()
        outs = [json.load(open(os.path.join(outdir, f"rank{r}.json"))) for r in range(world)]
    assert all(o == outs[0] for o in outs), "every rank returns the same probe"
    o = outs[0]
    print(json.dumps(o["summary"]), o["rccl"], o["probe_s"])
    assert o["ipc"] == "ok"
    assert len(o["pairs"]) == world * (world - 1) // 2
    for p in o["pairs"]:
        assert p["pci"][0] and p["pci"][0] == p["pci"][1]  # one device
        assert set(p["ipc_us"]) == {str(s) for s in o["sizes"]}
        big = p["ipc_GBps"][str(max(o["sizes"]))]
        assert big is not None and 5.0 < big < 10000.0, p
    # RCCL with several ranks on one device: reported, agreed, and no rate invented
    assert o["rccl_failed"] and o["rccl"] != "ok"
    assert "rccl_us_max" not in o["summary"]
    assert o["probe_s"] < 60
