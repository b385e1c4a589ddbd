"""The pass-depth planner (csrc/include/gs/engine.h plan_depths / Engine::plan_passes): the
partition of an iterate(n) into fused passes of depth 2..kmax with the lowest summed measured
pass time.  CPU-only: gs::plan_depths through libgs_core (the GPU path feeds it the autotuner's
per-depth pass times; tests/test_gpu_oracle.py runs the planned passes against the oracle).
Reference step loop being scheduled: src/GrayScott.jl:81-96 (one exchange + calculate per step).
"""
import functools
import random

import pytest

from grayscott_amd.ops import native


def _brute(cost, n):
    """Exact minimum over all partitions of n into depths 2..kmax (memoised recursion)."""
    ks = sorted(cost)

    @functools.lru_cache(maxsize=None)
    def best(m):
        if m == 0:
            return 0.0
        vals = [best(m - k) + cost[k] for k in ks if k <= m and best(m - k) < 1e300]
        return min(vals) if vals else 1e300

    return best(n)


def _cost(plan, cost):
    return sum(cost[k] for k in plan)


def test_driver_window_drops_the_remainder_pass():
    # round-5 kernels (T=2 0.479 ms, T=3 0.559 ms per pass, no T=4): 6 x 3 + 2 (the greedy plan)
    assert native.plan_depths({2: 0.479, 3: 0.559}, 20) == [3, 3, 3, 3, 3, 3, 2]
    # round-6 tuned times (profiles/r6_t4.txt): two T=4 passes replace the remainder pass
    c = {2: 0.4625, 3: 0.5137, 4: 0.6905}
    p = native.plan_depths(c, 20)
    assert sorted(p, reverse=True) == p and sum(p) == 20
    assert p == [4, 4, 3, 3, 3, 3]
    assert _cost(p, c) < _cost([3] * 6 + [2], c)


def test_plans_are_optimal_and_exact():
    rng = random.Random(7)
    for _ in range(60):
        kmax = rng.choice([3, 4, 5])
        cost = {k: rng.uniform(0.3, 1.0) * k ** rng.uniform(0.6, 1.1) for k in range(2, kmax + 1)}
        for n in [2, 3, 5, 7, 10, 11, 20, 23, 57, 100]:
            p = native.plan_depths(cost, n)
            assert sum(p) == n and all(2 <= k <= kmax for k in p)
            assert p == sorted(p, reverse=True)
            assert _cost(p, cost) == pytest.approx(_brute(cost, n), rel=1e-12)


def test_long_runs_use_the_cheapest_depth_per_step():
    cost = {2: 0.46, 3: 0.51, 4: 0.70}  # T=3 cheapest per step (0.170 vs 0.175 vs 0.23)
    n = 100000
    p = native.plan_depths(cost, n)
    assert sum(p) == n and len(p) >= n // 3
    assert p.count(3) >= len(p) - 3  # only the short tail may mix depths
    # and within one pass of the optimum over the whole run
    assert _cost(p, cost) <= (n / 3) * cost[3] + max(cost.values())


def test_degenerate_inputs():
    assert native.plan_depths({2: 0.4, 3: 0.5}, 1) == [1]  # a lone single step
    assert native.plan_depths({2: 0.4, 3: 0.5}, 0) == []
    assert native.plan_depths({2: 0.4, 3: 0.0}, 20) == []  # an untimed depth: greedy schedule
    with pytest.raises(ValueError):
        native.plan_depths({2: 0.4, 3: 0.5, 8: 1.0}, 20)


def test_engine_without_timed_depths_keeps_the_greedy_schedule():
    """The CPU backend times no fused depth: Engine::plan_passes is empty (greedy by depth)."""
    from grayscott_amd.models.grayscott import GrayScott
    from grayscott_amd.parallel.decomp import init_domain
    from grayscott_amd.utils.config import Settings

    s = Settings(L=24, precision="Float32", noise=0.1, backend="CPU")
    sim = GrayScott(s, init_domain(24, 1, 0), fuse=3)
    try:
        sim.init_fields()
        assert sim.engine.plan_passes(20) == []
    finally:
        sim.close()


def _refreshes(plan, pp):
    """Outer-ghost refreshes a plan needs: one per depth-parity switch between consecutive
    passes, plus one if the first pass's parity is not ``pp`` (engine.h ensure_bc)."""
    n = sum(1 for a, b in zip(plan, plan[1:]) if (a & 1) != (b & 1))
    if plan and pp >= 0 and (plan[0] & 1) != pp:
        n += 1
    return n


def test_parity_switches_are_priced():
    c = {2: 0.4625, 3: 0.5137, 4: 0.6905}  # 4,4,3,3,3,3 = 3.4358 vs 5 x 4 = 3.4525
    # no refresh cost: the plain optimum, deepest first
    assert native.plan_depths(c, 20, 0.0, -1) == [4, 4, 3, 3, 3, 3]
    # after an even pass (pp = 0) the mixed plan needs one refresh; at 16 us it still wins
    assert native.plan_depths(c, 20, 0.016, 0) == [4, 4, 3, 3, 3, 3]
    # after an odd pass the odd group goes first (one refresh, not two)
    assert native.plan_depths(c, 20, 0.016, 1) == [3, 3, 3, 3, 4, 4]
    # a dearer refresh: the all-even plan needs none after an even pass
    assert native.plan_depths(c, 20, 0.030, 0) == [4, 4, 4, 4, 4]


def test_parity_aware_plans_are_optimal():
    rng = random.Random(11)
    for _ in range(40):
        kmax = rng.choice([3, 4, 5])
        cost = {k: rng.uniform(0.3, 1.0) * k ** rng.uniform(0.6, 1.1) for k in range(2, kmax + 1)}
        fill = rng.uniform(0.0, 0.3)
        for pp in (-1, 0, 1):
            for n in [2, 3, 5, 7, 10, 20, 23]:
                p = native.plan_depths(cost, n, fill, pp)
                assert sum(p) == n and all(2 <= k <= kmax for k in p)
                got = _cost(p, cost) + fill * _refreshes(p, pp)
                # brute force over every multiset, arranged with the fewest refreshes
                best = 1e300

                def walk(m, kmin, acc):
                    nonlocal best
                    if m == 0:
                        ev = any(k % 2 == 0 for k in acc)
                        od = any(k % 2 for k in acc)
                        r = 1 if ev and od else (1 if pp >= 0 and (1 if od else 0) != pp else 0)
                        best = min(best, _cost(acc, cost) + fill * r)
                        return
                    for k in range(kmin, kmax + 1):
                        if k <= m:
                            walk(m - k, k, acc + [k])

                walk(n, 2, [])
                assert got == pytest.approx(best, rel=1e-9, abs=1e-12)
