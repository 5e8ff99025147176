"""CPU: the thread -> device assignment of one shared coder.

``ClassifierProcessor`` shares ONE coder among its ThreadPoolExecutor workers
(``/root/reference/wicca/classifying_tools.py:144, 414-419``, call ``:317``)
and builds a new pool per depth (``:546-551``).  ``HaarCoder(device="auto")``
binds each worker thread, on its first call, to the least-loaded device and
frees the slot when the thread ends.  Device ids are injected, so no GPU is
needed.
"""
import gc
import threading
from concurrent.futures import ThreadPoolExecutor

import pytest

from wicca_amd import HaarCoder
from wicca_amd.coder import DeviceBinder


def _pool_bind(binder, workers, tasks=None):
    """Every worker thread of a pool asks for its device (all alive at once)."""
    tasks = tasks or workers
    gate = threading.Barrier(workers)
    got = {}

    def task(_):
        d = binder.device()
        slot = [s for t, s, _ in binder.history if t == threading.get_ident()][-1]
        got[threading.get_ident()] = (slot, d)
        try:
            gate.wait(timeout=10)
        except threading.BrokenBarrierError:
            pass
        assert binder.device() == d  # sticky for the thread's life
        return slot

    with ThreadPoolExecutor(max_workers=workers) as ex:
        slots = list(ex.map(task, range(tasks)))
    return slots, got


def test_32_threads_spread_over_8_slots():
    b = DeviceBinder([0] * 8)
    slots, got = _pool_bind(b, 32)
    per = [list(s for s, _ in got.values()).count(k) for k in range(8)]
    assert per == [4] * 8, per
    assert all(d == 0 for _, d in got.values())


def test_uneven_pool_balanced_within_one():
    b = DeviceBinder([3, 5, 7])
    _, got = _pool_bind(b, 10)
    per = [list(s for s, _ in got.values()).count(k) for k in range(3)]
    assert max(per) - min(per) <= 1 and sum(per) == 10
    assert {d for _, d in got.values()} == {3, 5, 7}


def test_slots_released_when_threads_end():
    b = DeviceBinder([0, 1, 2, 3])
    _pool_bind(b, 8)
    gc.collect()
    assert b.live_counts() == [0, 0, 0, 0]
    # the next depth's pool (a new executor) spreads over every slot again
    _, got = _pool_bind(b, 4)
    assert sorted(s for s, _ in got.values()) == [0, 1, 2, 3]


def test_single_thread_keeps_its_device():
    b = DeviceBinder([0, 1])
    first = b.device()
    assert all(b.device() == first for _ in range(10))
    assert len(b.history) == 1


def test_coder_device_modes():
    c = HaarCoder(device="auto", devices=[0] * 4)
    assert c.binder is not None and c._dev() == 0
    assert HaarCoder(device=2)._dev() == 2 and HaarCoder(device=2).binder is None
    assert HaarCoder(device=None)._dev() == -1
    with pytest.raises(ValueError):
        HaarCoder(device="gpu")
    with pytest.raises(ValueError):
        HaarCoder(device=0, devices=[0, 1])
    with pytest.raises(ValueError):
        DeviceBinder([])


def test_multi_process_rank_follows_current_device(monkeypatch):
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "8")
    assert DeviceBinder().devices == [-1]
