"""bench.py's C5 peak: the highest paced rate one run keeps
at achieved/offered >= 0.99, bisected between half and all of the unpaced
median.  CPU only: a fake run with a known capacity."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402


def test_sustained_rate_finds_the_capacity():
    cap = 4.2e6
    calls = []

    def run_at(rate):   # a path that keeps up to cap, then saturates at it
        calls.append(rate)
        return min(rate, cap) * (1.0 if rate <= cap else 0.97)

    rate, trail = bench.sustained_rate(run_at, 5.6e6)
    assert len(calls) == 5 and len(trail) == 5
    assert cap * (1 - 0.5 * 5.6 / 4.2 / 32) - 1 <= rate <= cap          # within one bisection step below
    assert all(t[1] >= 0.99 for t in trail if t[0] <= rate)


def test_sustained_rate_never_exceeds_the_unpaced_median():
    rate, trail = bench.sustained_rate(lambda r: r, 3.0e6)
    assert rate < 3.0e6 and rate >= 3.0e6 * (1 - 1 / 32) - 1


def test_sustained_rate_stays_at_the_floor_when_nothing_holds():
    rate, trail = bench.sustained_rate(lambda r: 0.5 * r, 3.0e6)
    assert rate == 1.5e6 and all(t[1] < 0.99 for t in trail)


def test_keep_off_moves_every_thread_and_restores():
    """bench.keep_off: inside the block every thread of this process (one
    started before it too) runs off the spinning cores and their SMT
    siblings, children get the same mask, and the old masks come back."""
    import threading
    from firedancer_amd import tile
    node = sorted(os.sched_getaffinity(0))
    if len(tile.physical_cores(node)) < 2:
        import pytest
        pytest.skip("one physical core")
    spin = tile.physical_cores(node)[:1]
    busy = tile.core_siblings(spin[0])
    stop = threading.Event()
    th = threading.Thread(target=stop.wait)
    th.start()
    before = {int(t): os.sched_getaffinity(int(t)) for t in os.listdir("/proc/self/task")}
    try:
        with bench.keep_off(spin, node, True) as iso:
            assert iso.child_mask(node) == sorted(set(node) - busy)
            for t in os.listdir("/proc/self/task"):
                assert not (os.sched_getaffinity(int(t)) & busy), t
        for t, m in before.items():
            assert os.sched_getaffinity(t) == m
        with bench.keep_off(spin, node, False) as iso:   # --no-isolate-cores
            assert iso.child_mask(node) == node
            assert os.sched_getaffinity(0) == before[os.getpid()]
    finally:
        stop.set()
        th.join()


def test_core_siblings_parses_the_topology():
    from firedancer_amd import tile
    for c in sorted(os.sched_getaffinity(0))[:4]:
        sib = tile.core_siblings(c)
        assert c in sib and all(tile.core_siblings(x) == sib for x in sib if os.path.exists(
            f"/sys/devices/system/cpu/cpu{x}/topology/thread_siblings_list"))
