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
    def __init__(self, delay=0.0, fail_on=None):
        self.calls = []
        self.delay = delay
        self.fail_on = fail_on
        self.lock = threading.Lock()

    def __call__(self, paths, shapes, depths, interp, border, k, device, errors):
        with self.lock:
            self.calls.append((tuple(paths), device))
        time.sleep(self.delay)
        if self.fail_on is not None and self.fail_on in paths:
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


def test_failure_is_shared_by_every_requester():
    plan, fake = _plan([(224, 224)] * 3, (2, 3), fake=FakeMatrix(delay=0.02, fail_on="/bad.jpg"))
    errs = []

    def req():
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


def test_unplanned_pair_uses_the_per_call_stage(monkeypatch):
    import wicca_amd.jpeg as WJ
    seen = []
    monkeypatch.setattr(WJ, "get_img_batch", lambda *a, **k: seen.append(a) or ("imgs", "icons"))
    plan, fake = _plan([(224, 224)], (2, 3))
    assert plan.get_img_batch(["/a.jpg"], (299, 299), 2) == ("imgs", "icons")
    assert plan.get_img_batch(["/a.jpg"], (224, 224), 5) == ("imgs", "icons")
    assert len(seen) == 2 and not fake.calls and plan.stats["unplanned"] == 2


def test_devices_round_robin_over_batches():
    batches = [[f"/{i}.jpg"] for i in range(4)]
    plan, fake = _plan([(224, 224)], (2,), batches=batches, devices=[0, 1])
    for b in batches:
        plan.get_img_batch(b, (224, 224), 2)
    plan.close()
    assert {c[0][0]: c[1] for c in fake.calls} == {"/0.jpg": 0, "/1.jpg": 1, "/2.jpg": 0, "/3.jpg": 1}


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
