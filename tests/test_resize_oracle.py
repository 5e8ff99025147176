"""The cv2.resize restatement (oracle/resize_cv.py) against properties any
correct implementation of OpenCV's documented rules has.  cv2 itself is absent
(opencv-python 4.12.0.88, reference requirements.txt:91) and the reference
holds no resize fixture, so this oracle is parity-unpinned; these tests pin it
to the rules it restates (constant images stay constant, integer-scale
INTER_AREA is the rounded block mean, fractional INTER_AREA is the rounded
area-weighted mean, bilinear stays within one level of exact bilinear)."""
import numpy as np
import pytest

from oracle import resize_cv as R

rng = np.random.default_rng(1234)


@pytest.mark.parametrize("interp", R.SUPPORTED)
@pytest.mark.parametrize("dsize", [(224, 224), (7, 5), (300, 41), (640, 480), (50, 200)])
def test_constant_image_stays_constant(interp, dsize):
    img = np.full((97, 131, 3), 201, np.uint8)
    assert (R.resize(img, dsize, interp) == 201).all()


def test_same_size_is_a_copy():
    img = rng.integers(0, 256, (20, 30, 3), dtype=np.uint8)
    out = R.resize(img, (30, 20), R.INTER_AREA)
    assert np.array_equal(out, img) and not np.shares_memory(out, img)


def test_single_channel_results_are_2d():
    img = rng.integers(0, 256, (20, 30, 1), dtype=np.uint8)
    assert R.resize(img, (10, 10), R.INTER_AREA).shape == (10, 10)
    assert R.resize(img[:, :, 0], (10, 10), R.INTER_LINEAR).shape == (10, 10)


@pytest.mark.parametrize("C", [1, 2, 3, 4])
def test_area_2x2_is_rounded_half_up_mean_for_134(C):
    img = rng.integers(0, 256, (64, 96, C), dtype=np.uint8)
    s = img.reshape(32, 2, 48, 2, C).astype(np.int64).sum(axis=(1, 3))
    out = R.resize(img, (48, 32), R.INTER_AREA)
    out = out if out.ndim == 3 else out[:, :, None]
    if C == 2:  # float path: round half to even of s / 4
        assert np.array_equal(out, np.rint(s.astype(np.float32) * np.float32(0.25)).astype(np.uint8))
    else:
        assert np.array_equal(out, ((s + 2) >> 2).astype(np.uint8))


def test_area_integer_scale_is_rounded_block_mean():
    img = rng.integers(0, 256, (90, 120, 3), dtype=np.uint8)
    s = img.reshape(30, 3, 30, 4, 3).astype(np.float64).mean(axis=(1, 3))
    out = R.resize(img, (30, 30), R.INTER_AREA).astype(np.float64)
    assert np.abs(out - s).max() <= 0.5 + 1e-6


def _exact_area(img, dw, dh):
    """Area-weighted mean in float64 (pixel-coverage fractions)."""
    H, W, C = img.shape

    def weights(n, m):
        sc = n / m
        Wm = np.zeros((m, n))
        for d in range(m):
            a, b = d * sc, (d + 1) * sc
            for s in range(int(np.floor(a)), min(n, int(np.ceil(b)))):
                Wm[d, s] = max(0.0, min(b, s + 1) - max(a, s))
            Wm[d] /= Wm[d].sum()
        return Wm

    wy, wx = weights(H, dh), weights(W, dw)
    rows = np.tensordot(wy, img.astype(np.float64), axes=(1, 0))   # (dh, W, C)
    return np.einsum("ywc,dw->ydc", rows, wx, optimize=True)


@pytest.mark.parametrize("shape,dsize", [((135, 240), (224, 130)), ((1080, 1920), (224, 224)),
                                         ((333, 517), (100, 71)), ((50, 50), (49, 17))])
def test_area_fractional_is_rounded_area_mean(shape, dsize):
    img = rng.integers(0, 256, shape + (3,), dtype=np.uint8)
    out = R.resize(img, dsize, R.INTER_AREA).astype(np.float64)
    ref = _exact_area(img, *dsize)
    diff = np.abs(out - ref)
    assert diff.max() <= 0.5 + 1e-3  # float32 accumulation + round half even
    assert (diff <= 0.5).mean() > 0.999


@pytest.mark.parametrize("shape,dsize", [((135, 240), (224, 224)), ((68, 120), (331, 331)),
                                         ((40, 40), (299, 100))])
def test_linear_is_within_one_level_of_exact_bilinear(shape, dsize):
    img = rng.integers(0, 256, shape + (3,), dtype=np.uint8).astype(np.float64)
    H, W, _ = img.shape
    dw, dh = dsize

    def coords(n, m):
        f = (np.arange(m) + 0.5) * (n / m) - 0.5
        f = np.clip(f, 0, n - 1)
        i0 = np.floor(f).astype(int)
        i1 = np.minimum(i0 + 1, n - 1)
        return i0, i1, f - i0

    y0, y1, fy = coords(H, dh)
    x0, x1, fx = coords(W, dw)
    top = img[y0][:, x0] * (1 - fx)[None, :, None] + img[y0][:, x1] * fx[None, :, None]
    bot = img[y1][:, x0] * (1 - fx)[None, :, None] + img[y1][:, x1] * fx[None, :, None]
    ref = top * (1 - fy)[:, None, None] + bot * fy[:, None, None]
    out = R.resize(img.astype(np.uint8), dsize, R.INTER_LINEAR).astype(np.float64)
    assert np.abs(out - ref).max() <= 1.0 + 1e-9


def test_nearest_picks_floor_sources():
    img = rng.integers(0, 256, (10, 16, 3), dtype=np.uint8)
    out = R.resize(img, (8, 5), R.INTER_NEAREST)
    assert np.array_equal(out, img[::2, ::2])


def test_unsupported_interpolation_raises():
    with pytest.raises(NotImplementedError):
        R.resize(np.zeros((4, 4, 3), np.uint8), (2, 2), 2)
