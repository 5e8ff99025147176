"""The stage plan (wicca_image_stage_plan_u8, wicca_amd.plan): the whole
(classifier shape x depth) matrix of ClassifierProcessor._get_img_batch
(classifying_tools.py:297-323 under the loops of :546-551 and :414-419) from
one decode and two reads of each file, byte for byte equal to the per-call
file stage (wicca_amd.get_img_batch, itself pinned in test_gpu_jpeg.py /
test_gpu_raster.py) and to the oracles (cv2.resize restated, the C integer
oracle / the NumPy port of get_small_copy)."""
import io
import threading

import numpy as np
import pytest

import wicca_amd
from oracle import c_oracle, haar_numpy
from oracle import jpeg_pil as J
from oracle import resize_cv as R
from wicca_amd import plan as P

pytestmark = pytest.mark.gpu

DEMO_SHAPES = [(224, 224), (331, 331), (299, 299), (240, 240)]  # demo.ipynb's classifiers


def _png(img):
    from PIL import Image
    buf = io.BytesIO()
    Image.fromarray(img).save(buf, "PNG")
    return buf.getvalue()


def _bmp(img):
    from PIL import Image
    buf = io.BytesIO()
    Image.fromarray(img).save(buf, "BMP")
    return buf.getvalue()


def _files(tmp_path, specs):
    """Write (kind, H, W, fmt) test files; return paths and their RGB decodes (oracles)."""
    paths, refs = [], []
    for i, (kind, h, w, fmt) in enumerate(specs):
        img = J.test_image(kind, h, w, 13 * i + h)
        if fmt == "jpg":
            data = J.encode(img, 88, i % 3)
            ref = J.decode_rgb(data)
        elif fmt == "jpg-prog":
            data = J.encode(img, 85, 2, progressive=True)
            ref = J.decode_rgb(data)
        elif fmt == "png":
            data, ref = _png(img), img
        else:
            data, ref = _bmp(img), img
        p = tmp_path / f"f{i}.{fmt.split('-')[0]}"
        p.write_bytes(data)
        paths.append(str(p))
        refs.append(ref)
    return paths, refs


def _icon_oracle(rgb, depth, border=1, k=0):
    if 1 <= depth <= 8:
        return c_oracle.ll_int_block(rgb, depth, border, k)[0]
    return haar_numpy.get_small_copy(rgb, depth, border, k)


MIXED = [("scene", 480, 640, "jpg"), ("noise", 333, 517, "png"), ("scene", 1081, 1919, "jpg"),
         ("smooth", 250, 301, "bmp"), ("scene", 720, 1280, "jpg-prog"), ("noise", 77, 61, "jpg"),
         ("scene", 600, 401, "png")]


@pytest.mark.parametrize("depths", [range(2, 7), range(1, 6)], ids=["d2-6", "d1-5"])
def test_plan_matrix_matches_per_call_and_oracle(tmp_path, depths):
    """Mixed-format ragged batch, the demo's shapes, both depth ranges: every
    (shape, depth) output equals get_img_batch's and resize_cv o oracle."""
    paths, refs = _files(tmp_path, MIXED)
    got = wicca_amd.get_img_matrix(paths, DEMO_SHAPES, depths)
    assert set(got) == {(s, d) for s in DEMO_SHAPES for d in depths}
    for s in DEMO_SHAPES:
        for d in depths:
            imgs, icons = got[(s, d)]
            want = wicca_amd.get_img_batch(paths, s, d)
            assert np.array_equal(imgs, want[0]), (s, d)
            assert np.array_equal(icons, want[1]), (s, d)
    for i, rgb in enumerate(refs):  # the oracles, one shape per depth (CPU time)
        for j, d in enumerate(depths):
            s = DEMO_SHAPES[j % len(DEMO_SHAPES)]
            imgs, icons = got[(s, d)]
            assert np.array_equal(imgs[i], R.resize(rgb, s, R.INTER_AREA)), (i, s)
            assert np.array_equal(icons[i], R.resize(_icon_oracle(rgb, d), s, R.INTER_AREA)), (i, s, d)


CASES = [
    # depths, shapes, interpolation, border, k
    ((5,), [(224, 224)], 3, 1, 0),                       # one depth: no K5
    ((0, 3, 9), [(224, 224), (240, 240)], 3, 1, 0),      # copy, K1 alone, the float tail
    ((2, 8), [(299, 299)], 3, 0, 77),                    # K5 2..8, CONSTANT border
    ((3, 4, 5), [(224, 224), (331, 331)], 1, 1, 0),      # INTER_LINEAR: per-image source resizes
    ((2, 3), [(224, 224)], 2, 0, 255),                   # INTER_CUBIC icons (host tables)
    ((4, 2, 4), [(384, 384), (600, 450), (224, 224)], 3, 1, 0),  # wide shapes (no plan row sums), repeats
    ((1, 2, 3, 4, 5, 6, 7), [(112, 112), (224, 224), (240, 240), (299, 299), (331, 331)], 3, 1, 0),  # 5 shapes
    ((2, 5), [(1024, 600), (700, 300), (224, 224)], 3, 1, 0),  # groups split by column count
]


@pytest.mark.parametrize("depths,shapes,interp,border,k", CASES,
                         ids=[f"c{i}" for i in range(len(CASES))])
def test_plan_cases_match_per_call(tmp_path, depths, shapes, interp, border, k):
    paths, _ = _files(tmp_path, MIXED[:5])
    got = wicca_amd.get_img_matrix(paths, shapes, depths, interp, border, k)
    for s in shapes:
        for d in depths:
            want = wicca_amd.get_img_batch(paths, s, d, interp, border, k)
            assert np.array_equal(got[(s, d)][0], want[0]), (s, d)
            assert np.array_equal(got[(s, d)][1], want[1]), (s, d)


def test_plan_integer_scales(tmp_path):
    """INTER_AREA at integer scales (resizeAreaFast: 2x2 with (s + 2) >> 2,
    others rounded from the exact sum) through the plan's row kernel."""
    specs = [("scene", 448, 448, "jpg"), ("noise", 720, 960, "png"), ("scene", 480, 480, "jpg"),
             ("smooth", 672, 896, "bmp")]
    paths, refs = _files(tmp_path, specs)
    shapes = [(224, 224), (240, 240), (112, 112)]
    got = wicca_amd.get_img_matrix(paths, shapes, (2, 3))
    for s in shapes:
        for d in (2, 3):
            want = wicca_amd.get_img_batch(paths, s, d)
            assert np.array_equal(got[(s, d)][0], want[0]) and np.array_equal(got[(s, d)][1], want[1]), (s, d)
        for i, rgb in enumerate(refs):
            assert np.array_equal(got[(s, 2)][0][i], R.resize(rgb, s, R.INTER_AREA)), (i, s)


def test_plan_8k_batch_matches_per_call(tmp_path):
    """Two 8K JPEGs and a 4K one (the headline's image size, a K5 band count
    with padding at depth 6)."""
    specs = [("scene", 4320, 7680, "jpg"), ("noise", 2160, 3840, "jpg"), ("scene", 4320, 7680, "jpg")]
    paths, _ = _files(tmp_path, specs)
    got = wicca_amd.get_img_matrix(paths, DEMO_SHAPES, range(2, 7))
    for s in DEMO_SHAPES:
        for d in range(2, 7):
            want = wicca_amd.get_img_batch(paths, s, d)
            assert np.array_equal(got[(s, d)][0], want[0]) and np.array_equal(got[(s, d)][1], want[1]), (s, d)


def test_plan_8k_matches_oracle_at_demo_shapes(tmp_path):
    """The benchmarked geometry against the oracles, not another product
    kernel: 7680x4320 sources through the plan's area kernel (source launch) at the
    demo's shapes (area windows 23-34 pixels wide, the integer 32 x 18 scale of
    240), and the depth 2-4 icons (1920x1080 .. 480x270: area downscales,
    the plan's icon launch) plus the depth 5-6 icons (upscales) -- every
    output equal to resize_cv(rgb) and resize_cv(oracle icon).  A JPEG scene
    (its RGB from libjpeg-turbo, the decode pinned in test_gpu_jpeg.py) and a
    noise BMP (raw pixels: every window sum at full entropy)."""
    from PIL import Image
    scene = J.test_image("scene", 4320, 7680, 61)
    data = J.encode(scene, 90, 2)
    p0 = tmp_path / "scene8k.jpg"
    p0.write_bytes(data)
    noise = np.random.default_rng(62).integers(0, 256, (4320, 7680, 3), dtype=np.uint8)
    p1 = tmp_path / "noise8k.bmp"
    Image.fromarray(noise).save(p1, "BMP")
    paths, refs = [str(p0), str(p1)], [J.decode_rgb(data), noise]
    depths = range(2, 7)
    got = wicca_amd.get_img_matrix(paths, DEMO_SHAPES, depths)
    for i, rgb in enumerate(refs):
        icons = {d: _icon_oracle(rgb, d) for d in depths}
        for s in DEMO_SHAPES:
            want = R.resize(rgb, s, R.INTER_AREA)
            for d in depths:
                assert np.array_equal(got[(s, d)][0][i], want), (i, s, d)
                assert np.array_equal(got[(s, d)][1][i], R.resize(icons[d], s, R.INTER_AREA)), (i, s, d)


def test_plan_unreadable_file_fails_its_slot(tmp_path, capsys):
    paths, _ = _files(tmp_path, MIXED[:3])
    bad = tmp_path / "bad.jpg"
    bad.write_bytes(b"\xff\xd8\xff\xe0" + b"\x00" * 40)
    paths.insert(1, str(bad))
    with pytest.raises((ValueError, NotImplementedError)):
        wicca_amd.get_img_matrix(paths, [(224, 224)], (2, 3))
    got = wicca_amd.get_img_matrix(paths, [(224, 224), (299, 299)], (2, 3), errors="zero")
    assert f"Error loading image {paths[1]}" in capsys.readouterr().out
    for s in [(224, 224), (299, 299)]:
        for d in (2, 3):
            want = wicca_amd.get_img_batch(paths, s, d, errors="zero")
            assert np.array_equal(got[(s, d)][0], want[0]) and np.array_equal(got[(s, d)][1], want[1])
            assert not got[(s, d)][0][1].any() and not got[(s, d)][1][1].any()


def test_stage_plan_under_classifier_threads(tmp_path):
    """StagePlan shared by a ThreadPoolExecutor of 14 classifier tasks, one
    pool per depth (the reference's process_classifiers / _parallel_proc /
    _classify loops): every request equals the per-call stage, each batch is
    computed once, and the cache is empty at the end."""
    import concurrent.futures
    specs = [("scene", 300 + 7 * i, 400 + 11 * i, "jpg" if i % 4 else "png") for i in range(10)]
    paths, _ = _files(tmp_path, specs)
    batches = [paths[i:i + 4] for i in range(0, len(paths), 4)]
    classifiers = [(224, 224)] * 9 + [(331, 331)] + [(299, 299)] * 3 + [(240, 240)]
    depths = range(2, 7)
    plan = P.StagePlan(classifiers, depths, batches=batches)
    want = {(tuple(b), s, d): wicca_amd.get_img_batch(b, s, d) for b in batches for s in set(classifiers)
            for d in depths}
    bad = []
    for d in depths:
        def classify(shape):
            for b in batches:
                imgs, icons = plan.get_img_batch(b, shape, d)
                w = want[(tuple(b), shape, d)]
                if not (np.array_equal(imgs, w[0]) and np.array_equal(icons, w[1])):
                    bad.append((shape, d))
        with concurrent.futures.ThreadPoolExecutor(max_workers=len(classifiers)) as ex:
            list(ex.map(classify, classifiers))
    plan.close()
    assert not bad
    assert plan.stats["computed"] == len(batches)
    assert plan.cached_batches() == 0
    assert plan.stats["retired"] == len(batches)


def _matrix_sync(paths, shapes, depths):
    """The synchronous native call (status NULL, as errors="raise" was before
    the asynchronous entry)."""
    from wicca_amd import _lib
    _, keep, args, out = P._matrix_args(paths, shapes, depths, 3, 1, 0, None)
    _lib.check(_lib.load().wicca_image_stage_plan_u8(*args, None))
    del keep
    return out


def test_plan_async_batches_overlapped(tmp_path):
    """wicca_image_stage_plan_async: four batches issued back to back (their
    kernels chained on the device, host work and output copies overlapping),
    waited for in reverse order -- sequential JPEG, progressive, ragged sizes,
    and a batch with PNG / BMP files (the worker-thread form) -- each equal to
    the synchronous call's bytes."""
    specs = [("scene", 480 + 8 * i, 640 - 16 * i, "jpg") for i in range(3)] + \
        [("scene", 720, 1280, "jpg-prog"), ("noise", 77, 61, "jpg"), ("smooth", 1081, 1919, "jpg")] + \
        [("scene", 333, 517, "png"), ("noise", 250, 301, "bmp"), ("scene", 600, 401, "jpg")]
    paths, _ = _files(tmp_path, specs)
    batches = [paths[0:3], paths[3:6], paths[6:9], paths[0:6]]
    shapes, depths = DEMO_SHAPES, range(2, 7)
    calls = [P.get_img_matrix_async(b, shapes, depths) for b in batches]
    got = [c.wait() for c in reversed(calls)][::-1]
    for b, g in zip(batches, got):
        want = _matrix_sync(b, shapes, depths)
        assert set(g) == set(want)
        for key in want:
            assert np.array_equal(g[key][0], want[key][0]), key
            assert np.array_equal(g[key][1], want[key][1]), key


def test_plan_async_damaged_file_redone(tmp_path):
    """A JPEG whose entropy data was overwritten mid-scan: the asynchronous
    plan's wait finds the device's damage flag (or a decode that did not
    converge) and redoes the batch synchronously, so the outputs are the
    synchronous call's (libjpeg-turbo's damaged-data rules on the host)."""
    from wicca_amd import _lib
    paths, _ = _files(tmp_path, [("scene", 480, 640, "jpg"), ("noise", 720, 960, "jpg"),
                                 ("scene", 600, 401, "jpg")])
    data = bytearray(open(paths[1], "rb").read())
    rng = np.random.default_rng(5)
    mid = len(data) // 2
    junk = rng.integers(0, 255, 600, dtype=np.uint8)  # no 0xFF: markers stay where they were
    data[mid:mid + 600] = junk.tobytes()
    open(paths[1], "wb").write(bytes(data))
    lib = _lib.load()
    before = lib.wicca_jpeg_damaged_redone()
    got = wicca_amd.get_img_matrix(paths, [(224, 224), (299, 299)], (2, 3, 4))
    # counted once: the asynchronous wait redoes the batch, whose decode counts the file
    assert lib.wicca_jpeg_damaged_redone() - before in (0, 1)
    want = _matrix_sync(paths, [(224, 224), (299, 299)], (2, 3, 4))
    for key in want:
        assert np.array_equal(got[key][0], want[key][0]), key
        assert np.array_equal(got[key][1], want[key][1]), key
    assert lib.wicca_jpeg_damaged_redone() > before  # 600 random bytes: some code no table has
