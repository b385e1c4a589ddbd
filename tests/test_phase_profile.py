"""Per-phase timing of the scheduler's passes (csrc/include/gs/phase.h).

The reference only times the whole run (gray-scott.jl:12, ``@time``).  Here every phase of a
pass -- pack, transport, unpack, inner, shell, fused, step, bc -- is bracketed by timestamps in
stream order (hipEvents on the GPU, the host clock on the synchronous CPU backend) inside an
explicit profiling window.  These CPU tests check the bookkeeping: which phases appear for which
data path, that the window reports its passes and steps, that the parts account for the pass,
and that profiling does not change the results.
"""
import numpy as np
import pytest

from grayscott_amd.models.grayscott import GrayScott
from grayscott_amd.parallel.decomp import init_domain
from grayscott_amd.utils.config import Settings
from tests.mp_utils import run_ranks


def _sim(L=24, periodic=False, fuse=None):
    s = Settings(L=L, precision="Float32", noise=0.1, backend="CPU")
    sim = GrayScott(s, init_domain(L, 1, 0, periodic=periodic), fuse=fuse)
    sim.init_fields()
    return sim


def test_single_rank_profile_phases():
    sim = _sim()
    try:
        r = sim.phase_profile(5)
    finally:
        sim.close()
    assert r["passes"] == 5 and r["steps"] == 5 and not r["truncated"]
    assert set(r["phase_us"]) <= {"step", "bc"} and "step" in r["phase_us"]
    assert r["per_pass"]["step"] == 1.0
    assert r["pass_us"] > 0 and r["window_us"] >= r["phase_us"]["step"]
    # one rank, no neighbours: no exchange at all
    assert r["exchange_us"] == 0 and r["bytes_per_neighbour"] == {}
    assert 0 < r["accounted"] <= 1.5  # host clock, medians vs the mean pass: not exact


def test_profile_does_not_change_results():
    a, b = _sim(periodic=True), _sim(periodic=True)
    try:
        a.iterate(7)
        b.phase_profile(4)
        b.iterate(3)
        ua, va = a.get_fields()
        ub, vb = b.get_fields()
    finally:
        a.close()
        b.close()
    assert np.array_equal(ua, ub) and np.array_equal(va, vb)


def test_profile_truncation_is_reported():
    sim = _sim()
    try:
        sim.engine.prof_start(6)
        sim.engine.advance(4)
        r = sim.engine.prof_stop()
    finally:
        sim.close()
    assert r["truncated"]


def test_periodic_self_exchange_phases():
    # periodic single rank: the wraps are self copies inside the pack phase, then the unpack
    sim = _sim(periodic=True)
    try:
        r = sim.phase_profile(3)
    finally:
        sim.close()
    assert {"pack", "unpack", "step"} <= set(r["phase_us"])
    assert "transport" not in r["phase_us"]
    assert r["exchange_us"] >= r["phase_us"]["pack"]


@pytest.mark.timeout(300)
def test_two_rank_profile_reports_exchange():
    cfg = {"settings": dict(L=24, steps=4, precision="Float32", noise=0.1, backend="CPU"),
           "steps": 4, "profile_steps": 6}
    _, _, meta = run_ranks(2, cfg)
    for m in meta:
        p = m["profile"]
        assert p["passes"] == 6 and p["steps"] == 6
        assert {"pack", "transport", "unpack", "step"} <= set(p["phase_us"])
        assert p["per_pass"]["transport"] == 1.0
        # one neighbour (2 x 1 x 1 grid): one face of 12 x 24 x 24 ... of (u, v) fp32 pairs
        (peer, nbytes), = p["bytes_per_neighbour"].items()
        assert int(peer) == 1 - meta.index(m)
        assert nbytes == 24 * 24 * 8
        assert p["exchange_us"] >= p["phase_us"]["transport"]
        assert p["link_GBps"] is not None and p["link_GBps"] > 0
        assert 0 < p["accounted"] <= 1.5  # medians vs the mean pass: not exact


def test_driver_perf_log_uses_stream_ordered_compute_timer(tmp_path):
    """The driver's perf log: one record per output interval with the compute time taken from
    the stream-ordered timer (no synchronisation around compute), plus the run summary."""
    import json

    from grayscott_amd.driver import run

    log = tmp_path / "perf.jsonl"
    s = Settings(L=16, steps=12, plotgap=4, precision="Float32", noise=0.1, backend="CPU",
                 output=str(tmp_path / "o.bp"), perf_log=str(log))
    res = run(s)
    recs = [json.loads(l) for l in log.read_text().splitlines()]
    steps = [r for r in recs if "step" in r]
    assert [r["step"] for r in steps] == [4, 8, 12]
    assert all(r["steps"] == 4 and r["compute_s"] > 0 and r["io_s"] > 0 for r in steps)
    summ = recs[-1]["summary"]
    assert summ["timers"]["compute"]["calls"] == 3
    assert summ["timers"]["compute"]["clock"] == "host"
    assert abs(summ["compute_s"] - sum(r["compute_s"] for r in steps)) < 1e-9
    assert res["steps"] == 12


def test_critical_path_models():
    """The three pass schedules' critical paths (models/grayscott.py critical_path): sequential
    parts add up; one overlapped pass hides the exchange behind the inner part and then runs the
    shell; chained passes (engine.h advance_chained) run shell_p beside inner_p, so the period is
    max(inner, exchange + shell) -- the recurrence c_p = max(c_{p-1}, e_{p-1}) + I,
    e_p = max(e_{p-1} + X, c_{p-1}) + S, simulated here."""
    from grayscott_amd.models.grayscott import critical_path
    seq = {"pack": 5.0, "transport": 20.0, "unpack": 4.0, "fused": 100.0, "bc": 10.0}
    assert critical_path(seq, 29.0, {"bc": 0.5}, False) == pytest.approx(29 + 100 + 5)
    ov = {"inner": 80.0, "shell": 25.0}
    assert critical_path(ov, 50.0, {}, False) == pytest.approx(105.0)
    assert critical_path(ov, 90.0, {}, False) == pytest.approx(115.0)
    for inner, xch, shell in ((80.0, 50.0, 25.0), (80.0, 70.0, 25.0), (40.0, 10.0, 5.0)):
        c = e = 0.0
        ends = []
        for _ in range(200):
            c, e = max(c, e) + inner, max(e + xch, c) + shell
            ends.append(e)
        period = (ends[-1] - ends[-101]) / 100
        assert critical_path({"inner": inner, "shell": shell}, xch, {}, True) == \
            pytest.approx(period)
