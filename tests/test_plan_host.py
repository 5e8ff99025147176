"""StagePlan's host logic (wicca_amd/plan.py) with a stand-in for the native
matrix call: one computation per batch under the reference's thread layout
(a pool of classifier tasks per depth, classifying_tools.py:414-419 / :546-551),
retirement once every expected (shape, depth) request was served, background
computation of the next batch, the byte cap, shared failures, and unplanned
pairs falling back to the per-call stage."""
import concurrent.futures
import threading
import time

import numpy as np
import pytest

from wicca_amd import plan as P


class FakeMatrix:
    def __init__(self, delay=0.0, fail_on=None, fail_times=None):
        self.calls = []
        self.delay = delay
        self.fail_on = fail_on
        self.fail_times = fail_times  # None: always
        self.lock = threading.Lock()

    def __call__(self, paths, shapes, depths, interp, border, k, device, errors):
        with self.lock:
            self.calls.append((tuple(paths), device, tuple(depths)))
            fail = self.fail_on is not None and self.fail_on in paths and (
                self.fail_times is None or sum(self.fail_on in c[0] for c in self.calls) <= self.fail_times)
        time.sleep(self.delay)
        if fail:
            raise ValueError("image 0: corrupt")
        n = len(paths)
        out = {}
        for (w, h) in shapes:
            res = np.full((n, h, w, 3), hash(tuple(paths)) % 251, np.uint8)
            for d in depths:
                out[((w, h), d)] = (res, np.full((n, h, w, 3), d, np.uint8))
        return out


def _plan(classifiers, depths, **kw):
    fake = kw.pop("fake", None) or FakeMatrix()
    plan = P.StagePlan(classifiers, depths, **kw)
    plan._matrix = fake
    return plan, fake


CLASSIFIERS = [(224, 224)] * 9 + [(331, 331)] + [(299, 299)] * 3 + [(240, 240)]


@pytest.mark.parametrize("prefetch", [False, True])
def test_each_batch_computed_once_and_retired(prefetch):
    batches = [[f"/x/{i}.jpg", f"/x/{i}b.jpg"] for i in range(5)]
    plan, fake = _plan(CLASSIFIERS, range(2, 7), batches=batches if prefetch else None,
                       fake=FakeMatrix(delay=0.01))
    for d in range(2, 7):
        def classify(shape):
            for b in batches:
                imgs, icons = plan.get_img_batch(b, shape, d)
                assert imgs.shape == (2, shape[1], shape[0], 3)
                assert (icons == d).all()
        with concurrent.futures.ThreadPoolExecutor(max_workers=len(CLASSIFIERS)) as ex:
            list(ex.map(classify, CLASSIFIERS))
    plan.close()
    assert sorted(c[0] for c in fake.calls) == sorted(tuple(b) for b in batches)
    assert plan.cached_batches() == 0 and plan.cached_bytes() == 0
    assert plan.stats["retired"] == len(batches)
    if prefetch:
        assert plan.stats["prefetched"] >= 1


def test_shared_outputs_are_read_only():
    plan, _ = _plan([(224, 224)] * 2, (3,), copy=False)
    a, _ = plan.get_img_batch(["/a.jpg"], (224, 224), 3)
    b, _ = plan.get_img_batch(["/a.jpg"], (224, 224), 3)
    assert a is b and not a.flags.writeable
    with pytest.raises(ValueError):
        a[:] = 0


def test_requests_get_private_copies():
    plan, _ = _plan([(224, 224)] * 2, (3,))
    a, _ = plan.get_img_batch(["/a.jpg"], (224, 224), 3)
    a[:] = 0
    b, _ = plan.get_img_batch(["/a.jpg"], (224, 224), 3)
    assert b.any()


def test_byte_cap_evicts_and_recomputes():
    plan, fake = _plan([(224, 224), (240, 240)], (2, 3), cache_bytes=1)
    plan.get_img_batch(["/a.jpg"], (224, 224), 2)
    plan.get_img_batch(["/b.jpg"], (224, 224), 2)  # /a is dropped (over the cap)
    plan.get_img_batch(["/a.jpg"], (240, 240), 3)  # recomputed
    assert [c[0] for c in fake.calls] == [("/a.jpg",), ("/b.jpg",), ("/a.jpg",)]
    assert plan.stats["evicted"] >= 1


def test_failure_is_shared_by_waiting_requesters():
    """The requesters waiting on a batch when its computation fails all see
    that failure (one computation); the failure is not cached."""
    plan, fake = _plan([(224, 224)] * 3, (2, 3), fake=FakeMatrix(delay=0.3, fail_on="/bad.jpg"))
    errs = []
    go = threading.Barrier(6)

    def req():
        go.wait()
        try:
            plan.get_img_batch(["/ok.jpg", "/bad.jpg"], (224, 224), 2)
        except ValueError as e:
            errs.append(str(e))
    ts = [threading.Thread(target=req) for _ in range(6)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert len(errs) == 6 and len(fake.calls) == 1
    assert plan.cached_batches() == 0


def test_transient_failure_is_retried():
    """a transient failure (e.g. a device OOM in the background
    batch) is shared only with the requesters already waiting; the next
    request computes the batch again and succeeds -- including a failure in
    the prefetch thread, which the foreground then recomputes."""
    plan, fake = _plan([(224, 224)] * 2, (2,), fake=FakeMatrix(fail_on="/t.jpg", fail_times=1))
    with pytest.raises(ValueError):
        plan.get_img_batch(["/t.jpg"], (224, 224), 2)
    imgs, _ = plan.get_img_batch(["/t.jpg"], (224, 224), 2)
    assert imgs.shape == (1, 224, 224, 3) and len(fake.calls) == 2
    batches = [["/a.jpg"], ["/t.jpg"]]
    plan, fake = _plan([(224, 224)], (2,), batches=batches, fake=FakeMatrix(fail_on="/t.jpg", fail_times=1))
    plan.get_img_batch(batches[0], (224, 224), 2)  # starts /t.jpg in the background: it fails
    for t in plan._prefetch:
        t.join()
    imgs, _ = plan.get_img_batch(batches[1], (224, 224), 2)
    assert imgs.shape == (1, 224, 224, 3)
    assert sorted(c[0] for c in fake.calls) == [("/a.jpg",), ("/t.jpg",), ("/t.jpg",)]
    assert plan.stats["failed"] == 1


def _run_reference_loop(plan, classifiers, depths, batches):
    """process_classifiers: depths outermost, a pool of classifier tasks per
    depth, each walking the folder's batches (classifying_tools.py:546-551,
    :414-419, :339-346)."""
    for d in depths:
        def classify(shape):
            for b in batches:
                imgs, icons = plan.get_img_batch(b, shape, d)
                assert imgs.shape == (len(b), shape[1], shape[0], 3) and (icons == d).all()
        with concurrent.futures.ThreadPoolExecutor(max_workers=len(classifiers)) as ex:
            list(ex.map(classify, classifiers))


@pytest.mark.parametrize("known", [True, False])
def test_folder_larger_than_the_cache_runs_per_depth(known):
    """a folder whose outputs for all depths exceed cache_bytes.
    Keeping every depth of every batch until the last depth (the cyclic access
    of the depth loop) would evict exactly the batch the next depth starts with
    and recompute every batch at every depth for all depths.  The plan computes
    per (batch, depth) instead: each batch once per depth -- one decode for all
    14 classifiers -- with no more host memory than a few batches of one depth."""
    depths = (2, 3, 4, 5, 6)
    batches = [[f"/f/{i}_{j}.jpg" for j in range(3)] for i in range(12)]
    per_batch_all = 3 * sum(w * h * 3 for (w, h) in set(CLASSIFIERS)) * (1 + len(depths))
    cap = 4 * per_batch_all  # a third of the folder
    plan, fake = _plan(CLASSIFIERS, depths, batches=batches if known else None, cache_bytes=cap)
    assert plan.per_depth == known
    _run_reference_loop(plan, CLASSIFIERS, depths, batches)
    plan.close()
    n = len(batches) * len(depths)
    if known:
        assert len(fake.calls) == n and all(len(c[2]) == 1 for c in fake.calls)
        assert plan.stats["evicted"] == 0
    else:  # found out at the first eviction: at most the batches computed before it were wasted
        assert plan.per_depth
        assert len(fake.calls) <= n + len(batches)
    assert plan.cached_batches() == 0


def test_folder_that_fits_computes_every_depth_at_once():
    depths = (2, 3)
    batches = [[f"/g/{i}.jpg"] for i in range(4)]
    plan, fake = _plan(CLASSIFIERS, depths, batches=batches, cache_bytes=1 << 40)
    assert not plan.per_depth
    _run_reference_loop(plan, CLASSIFIERS, depths, batches)
    plan.close()
    assert len(fake.calls) == len(batches) and all(c[2] == depths for c in fake.calls)


def test_unplanned_pair_uses_the_per_call_stage(monkeypatch):
    import wicca_amd.jpeg as WJ
    seen = []
    monkeypatch.setattr(WJ, "get_img_batch", lambda *a, **k: seen.append(a) or ("imgs", "icons"))
    plan, fake = _plan([(224, 224)], (2, 3))
    assert plan.get_img_batch(["/a.jpg"], (299, 299), 2) == ("imgs", "icons")
    assert plan.get_img_batch(["/a.jpg"], (224, 224), 5) == ("imgs", "icons")
    assert len(seen) == 2 and not fake.calls and plan.stats["unplanned"] == 2


def test_next_batch_overlaps_the_requested_one():
    """With batches known, the next batch starts computing when a batch is
    first requested (not when it is done): two computations overlap."""
    batches = [[f"/o/{i}.jpg"] for i in range(4)]
    live, peak = [0], [0]
    lock = threading.Lock()

    class Probe(FakeMatrix):
        def __call__(self, *a):
            with lock:
                live[0] += 1
                peak[0] = max(peak[0], live[0])
            try:
                return super().__call__(*a)
            finally:
                with lock:
                    live[0] -= 1
    plan, fake = _plan([(224, 224)], (2,), batches=batches, fake=Probe(delay=0.1))
    for b in batches:
        plan.get_img_batch(b, (224, 224), 2)
    plan.close()
    assert peak[0] >= 2 and len(fake.calls) == len(batches)


def test_devices_round_robin_over_batches():
    batches = [[f"/{i}.jpg"] for i in range(4)]
    plan, fake = _plan([(224, 224)], (2,), batches=batches, devices=[0, 1])
    for b in batches:
        plan.get_img_batch(b, (224, 224), 2)
    plan.close()
    assert {c[0][0]: c[1] for c in fake.calls} == {"/0.jpg": 0, "/1.jpg": 1, "/2.jpg": 0, "/3.jpg": 1}


def test_default_cache_is_bounded():
    assert 0 < P._default_cache_bytes() <= 32 << 30


def test_depth_forms_and_validation():
    assert P._norm_depths(range(2, 7)) == (2, 3, 4, 5, 6)
    assert P._norm_depths([3, 3, 2]) == (3, 2)
    assert P._norm_depths(4) == (4,)
    with pytest.raises(TypeError):
        P._norm_depths(2.5)
    with pytest.raises(ValueError):
        P.StagePlan([], (2,))


def test_folder_batches_follow_classify(tmp_path):
    import os
    for i in range(7):
        (tmp_path / f"{i}.jpg").write_bytes(b"x")
    b = P.folder_batches(tmp_path, 3)
    names = os.listdir(tmp_path)
    assert [len(x) for x in b] == [3, 3, 1]
    assert [os.path.basename(p) for x in b for p in x] == names
