"""Link probe bookkeeping and the tuner's exchange model (CPU only: no device is touched).

The probe itself (csrc/hip/probe.hpp) runs in tests/test_gpu_linkprobe.py; here: the pair
schedule, the pair table / summary, the transfer-time interpolation, the per-neighbour message
sizes and the pruning rule (parallel/autotune.py model_step_ms / prune_by_model)."""
import itertools

import pytest

from grayscott_amd.parallel import autotune
from grayscott_amd.parallel.decomp import dims_create, init_domain
from grayscott_amd.parallel.linkprobe import PROBE_SIZES, round_robin, summarize, transfer_us


@pytest.mark.parametrize("n", range(2, 10))
def test_round_robin_covers_every_pair_once(n):
    rounds = round_robin(n)
    assert len(rounds) == (n - 1 if n % 2 == 0 else n)
    seen = []
    for pairs in rounds:
        ranks = [r for p in pairs for r in p]
        assert len(ranks) == len(set(ranks)), "a rank twice in one round"
        seen += pairs
    assert sorted(seen) == sorted(itertools.combinations(range(n), 2))


def _link(us_by_size, tr="rccl"):
    """A probe result whose slowest pair takes us_by_size[s] microseconds at size s."""
    return {"summary": {f"{tr}_us_max": {str(s): t for s, t in us_by_size.items()}}}


def test_summary_takes_the_slower_direction_and_pair():
    sizes = [4096, 1 << 20]
    rounds = round_robin(4)
    allm = []
    for r in range(4):
        d = {"ipc": {}, "rccl": {}}
        for pairs in rounds:
            for a, b in pairs:
                if r in (a, b):
                    peer = b if r == a else a
                    for s in sizes:
                        # pair (0, 3) is the slow link; rank 3 -> 0 the slow direction
                        slow = 4.0 if {a, b} == {0, 3} and r == 3 else 1.0
                        d["ipc"][f"{peer}:{s}"] = slow * (5.0 + s / 50e3)
        allm.append(d)
    out = summarize(allm, [f"pci{r}" for r in range(4)], sizes, rounds)
    assert len(out["pairs"]) == 6
    p03 = [p for p in out["pairs"] if p["ranks"] == [0, 3]][0]
    assert p03["ipc_us"][str(1 << 20)] == pytest.approx(4.0 * (5.0 + (1 << 20) / 50e3), rel=1e-3)
    assert p03["pci"] == ["pci0", "pci3"]
    s = out["summary"]
    assert s["ipc_us_max"][str(1 << 20)] == p03["ipc_us"][str(1 << 20)]
    assert s["ipc_GBps_min"][str(1 << 20)] < s["ipc_GBps_median"][str(1 << 20)]
    assert "rccl_us_max" not in s  # nothing probed on RCCL


def test_transfer_interpolates_and_extrapolates():
    link = _link({4096: 10.0, 1 << 20: 30.0, 4 << 20: 90.0})
    assert transfer_us(link, "rccl", 4096) == 10.0
    assert transfer_us(link, "rccl", 100) == 10.0  # below the smallest: its time
    assert transfer_us(link, "rccl", (1 << 20) + (3 << 19)) == pytest.approx(60.0)
    assert transfer_us(link, "rccl", 8 << 20) == pytest.approx(180.0)  # the largest's rate
    assert transfer_us(link, "ipc", 4096) is None
    assert transfer_us(None, "rccl", 4096) is None


def test_pass_messages_of_the_reference_grid_and_z_slabs():
    H = 3
    dom = init_domain(512, 8, 0, periodic=False, dims=[2, 2, 2])
    msgs = sorted(autotune.pass_messages(dom, H))
    assert msgs == sorted([H * 256 * 256] * 3 + [H * H * 256] * 3 + [H ** 3])
    mid = init_domain(512, 8, 3, periodic=False, dims=[1, 1, 8])
    assert autotune.pass_messages(mid, H) == [H * 518 * 518] * 2
    end = init_domain(512, 8, 0, periodic=False, dims=[1, 1, 8])
    assert autotune.pass_messages(end, H) == [H * 518 * 518]
    # the probe's largest size is the z-slab message at T=3 without the ghost frame
    assert PROBE_SIZES[-1] == 512 * 512 * 3 * 8


def test_model_prefers_the_grid_on_slow_links_and_slabs_never_win_more_than_overlap():
    comp = 0.16  # ms per step of the update (a 512^3 / 8 rank at ~800k MLUPS per GPU)
    slow = _link({4096: 10.0, 1 << 20: 1e6 * (1 << 20) / 20e9, 8 << 20: 1e6 * (8 << 20) / 20e9})
    grid = autotune.model_step_ms(512, 8, [2, 2, 2], 3, "off", "rccl", slow, comp)
    zs = autotune.model_step_ms(512, 8, [1, 1, 8], 3, "off", "rccl", slow, comp)
    zs_ov = autotune.model_step_ms(512, 8, [1, 1, 8], 3, "auto", "rccl", slow, comp)
    # 20 GB/s: a 6.4 MB slab message is ~320 us per pass against 79 us for a 1.6 MB face; in
    # sequence the grid wins, overlapped the slab's exchange hides under its 480 us pass
    assert grid < zs and zs_ov < zs
    assert zs_ov == pytest.approx(comp * (1 + autotune.overlap_cost([1, 1, 8], "rccl")))
    assert grid == pytest.approx(comp + 1e3 * (3 * 256 * 256 * 8) / 20e9 / 3, rel=0.02)
    # fast links: the exchange hides under the update when overlapped
    fast = _link({4096: 5.0, 8 << 20: 1e6 * (8 << 20) / 400e9})
    zs_fast = autotune.model_step_ms(512, 8, [1, 1, 8], 3, "auto", "rccl", fast, comp)
    assert zs_fast == pytest.approx(comp * (1 + autotune.overlap_cost([1, 1, 8], "rccl")))
    # a 2x2x2 rank's stream-overlapped pass costs a third more than its update (RCCL), so on
    # fast links the pass in sequence is the better model row
    g_ov = autotune.model_step_ms(512, 8, [2, 2, 2], 3, "auto", "rccl", fast, comp)
    g_off = autotune.model_step_ms(512, 8, [2, 2, 2], 3, "off", "rccl", fast, comp)
    assert g_off < g_ov == pytest.approx(comp * 1.34)


def test_prune_rule_protects_the_reference_grid():
    pred = {0: 1.30, 1: 1.0, 2: 1.19, 3: 1.21, 4: 2.0}
    out = autotune.prune_by_model(pred, protected=[0])
    assert set(out) == {3, 4}
    assert out[4] == pytest.approx(2.0)
    assert autotune.prune_by_model({}, protected=[]) == {}


def test_candidate_table_is_pruned_by_the_model_on_slow_links():
    """The whole decision for an 8-rank L=512 job: with 8 GB/s links (a z-slab message then
    takes 800 us, more than the 480 us pass it could hide under) every z-slab candidate is
    modelled > 20 % slower than the best grid row and would be skipped; the reference grid rows
    are protected.  With 400 GB/s links no z slab is pruned; the only rows ruled out are the
    stream-overlapped packed grids on RCCL, whose split pass costs a third more than the update
    (overlap_cost) while the exchange they would hide is short."""
    comp = 0.16
    bal = dims_create(8)
    cands = autotune.candidates(512, 8, "hip")
    for rate, expect_pruned in ((8e9, True), (400e9, False)):
        link = _link({4096: 10.0, 8 << 20: 1e6 * (8 << 20) / rate})
        pred = {}
        for i, c in enumerate(cands):
            f = c[1] if c[1] > 0 else 3
            tr = c[4] if len(c) > 4 else "rccl"
            link2 = {"summary": {**link["summary"], "ipc_us_max": link["summary"]["rccl_us_max"]}}
            pred[i] = autotune.model_step_ms(512, 8, c[0], f, c[2], tr, link2, comp)
        protected = [i for i, c in enumerate(cands) if list(c[0]) == list(bal)]
        out = autotune.prune_by_model(pred, protected)
        zslab = [i for i, c in enumerate(cands) if list(c[0]) == [1, 1, 8]]
        assert not set(out) & set(protected)
        if expect_pruned:
            assert set(zslab) <= set(out), (pred, out)
        else:
            assert not set(out) & set(zslab), (pred, out)
            for i in out:
                c = cands[i]
                assert c[2] != "off" and not (len(c) > 4 and c[4] == "ipc"), c
                assert list(c[0]) not in ([1, 1, 8], list(bal)), c


class _OneRankView:
    """Rank 0's view of an 8-rank job whose collectives are identities (every rank agrees)."""
    world_size, rank, is_distributed = 8, 0, False

    def allreduce(self, v, op="max"):
        return float(v)

    def broadcast_object(self, obj, src=0):
        return obj

    def allgather_object(self, obj):
        return [obj]


@pytest.mark.parametrize("rate,rccl_failed", [(8e9, False), (400e9, False), (400e9, True)])
def test_tuner_skips_what_the_model_rules_out(monkeypatch, rate, rccl_failed):
    """tune_data_path with a probe result: nothing is checked or timed for the rows the model
    rules out (slow links: the z slabs), the reference grid rows always are, the recorded
    predictions sit next to the timings, and with RCCL unusable the IPC rows go first and the
    host fallbacks are not timed."""
    from grayscott_amd.utils.config import Settings
    timed = []

    def fake_check(ctx, backend, dims, f, tr, ov, **kw):
        return True, 0.0, tr if tr != "auto" else ("host" if rccl_failed else "rccl"), None

    def fake_time(s, ctx, L, dims, f, steps=0, warmup=0, skip_rccl=False, info=None):
        timed.append((list(dims), f, s.overlap, s.transport))
        if info is not None:
            info["comp_ms_per_step"] = 0.16
        slow = rate < 1e10 and list(dims) == [1, 1, 8]
        return (0.30 if slow else 0.17) * steps * 1e-3, s.overlap != "off"

    monkeypatch.setattr(autotune, "selfcheck", fake_check)
    monkeypatch.setattr(autotune, "time_data_path", fake_time)
    link = {"summary": {k: {"4096": 10.0, str(8 << 20): 1e6 * (8 << 20) / rate}
                        for k in ("rccl_us_max", "ipc_us_max")},
            "rccl_failed": rccl_failed, "ipc": "ok"}
    if rccl_failed:
        del link["summary"]["rccl_us_max"]
    s = Settings(L=512, precision="Float32", backend="AMDGPU")
    out = autotune.tune_data_path(s, _OneRankView(), 512, "hip", steps=10, warmup=1, link=link)
    tab = out["table"]
    bal = dims_create(8)
    assert any(r.get("ok") for r in tab if r["dims"] == bal)  # BASELINE config 3: always timed
    assert not any(r.get("skipped") == "model" for r in tab if r["dims"] == bal)
    assert all("model_ms_per_step" in r for r in tab if r.get("ok") and r is not tab[0])
    if rate < 1e10:
        zs = [r for r in tab if r["dims"] == [1, 1, 8]]
        assert zs and all(r.get("skipped") == "model" for r in zs), zs
        assert not any(d == [1, 1, 8] for d, *_ in timed)
    elif rccl_failed:
        assert tab[0].get("transport_req") == "ipc"
        host = [r for r in tab if r.get("skipped", "").startswith("rccl unavailable")]
        assert host and not any(t == "auto" for *_, t in timed)
    else:
        # fast links: only the RCCL stream-overlapped packed grids (1.34x passes) may be ruled out
        for r in tab:
            if r.get("skipped"):
                assert r["skipped"] == "model" and r["dims"] not in ([1, 1, 8], bal), r
                assert r["overlap_req"] != "off" and r.get("transport_req") != "ipc", r


def test_explicit_transport_rows_are_timed_even_without_rccl(monkeypatch):
    """--transport host (or torch / ipc): the rows the user pinned the run's transport for are
    timed although the probe found RCCL unusable (only "auto" / "rccl" runs skip their host
    fallbacks)."""
    from grayscott_amd.utils.config import Settings
    timed = []

    def fake_check(ctx, backend, dims, f, tr, ov, **kw):
        return True, 0.0, tr, None

    def fake_time(s, ctx, L, dims, f, steps=0, warmup=0, skip_rccl=False, info=None):
        timed.append(s.transport)
        if info is not None:
            info["comp_ms_per_step"] = 0.16
        return 0.2 * steps * 1e-3, False

    monkeypatch.setattr(autotune, "selfcheck", fake_check)
    monkeypatch.setattr(autotune, "time_data_path", fake_time)
    link = {"summary": {"ipc_us_max": {"4096": 10.0, str(8 << 20): 30.0}},
            "rccl_failed": True, "ipc": "ok"}
    s = Settings(L=512, precision="Float32", backend="AMDGPU", transport="host")
    out = autotune.tune_data_path(s, _OneRankView(), 512, "hip", steps=10, warmup=1, link=link)
    assert not any(str(r.get("skipped", "")).startswith("rccl unavailable") for r in out["table"])
    assert "host" in timed


def _probe_worker(rank, world, port, outdir):
    import json
    import os
    import sys

    from .mp_utils import ROOT
    sys.path.insert(0, ROOT)
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": "0",
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    from grayscott_amd.parallel import dist as gdist
    from grayscott_amd.parallel.linkprobe import probe_links
    ctx = gdist.init_from_env("cpu")
    out = probe_links(ctx, reps=1)
    with open(os.path.join(outdir, f"rank{rank}.json"), "w") as f:
        json.dump(out, f)
    ctx.barrier()
    ctx.finalize()


def test_probe_without_a_device_is_agreed_and_does_not_hang(tmp_path):
    """Ranks that cannot create the probe's device buffers (no GPU here) still make the same
    collectives: every rank returns the same record, with the IPC failure and no rates, within
    seconds -- the failure path a node with a broken device takes before the tuner runs."""
    import json

    import torch.multiprocessing as mp

    from .mp_utils import free_port
    pc = mp.start_processes(_probe_worker, args=(2, free_port(), str(tmp_path)), nprocs=2,
                            join=False, start_method="spawn")
    import time
    t0 = time.monotonic()
    while not pc.join(60):
        assert time.monotonic() - t0 < 120, "probe ranks hung"
    outs = [json.load(open(tmp_path / f"rank{r}.json")) for r in range(2)]
    assert outs[0]["ipc"] == outs[1]["ipc"] and outs[0]["ipc"] != "ok"
    assert outs[0]["rccl"] == "not probed" and not outs[0]["rccl_failed"]
    assert outs[0]["summary"] == {} and len(outs[0]["pairs"]) == 1
