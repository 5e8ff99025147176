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
    # cv2.INTER_MAX (7) and the WARP_* flags are not interpolations of cv2.resize
    with pytest.raises(NotImplementedError):
        R.resize(np.zeros((4, 4, 3), np.uint8), (2, 2), 7)


# ---- INTER_CUBIC / INTER_LANCZOS4 / INTER_LINEAR_EXACT / INTER_NEAREST_EXACT ----
# (the interpolations ClassifierProcessor accepts beyond the demo's,
# /root/reference/wicca/classifying_tools.py:168-176; parity-unpinned like the rest)

def _ref_separable(img, dw, dh, kern, K):
    """float64 separable filter with half-pixel centres and replicated borders."""
    H, W, C = img.shape
    src = img.astype(np.float64)

    def axis_w(n, m):
        sc = n / m
        Wm = np.zeros((m, n))
        for d in range(m):
            f = (d + 0.5) * sc - 0.5
            s = int(np.floor(f))
            t = f - s
            w = np.array([kern(t + (K // 2 - 1) - j) for j in range(K)])
            w /= w.sum()
            for j in range(K):
                Wm[d, min(max(s - (K // 2 - 1) + j, 0), n - 1)] += w[j]
        return Wm

    Wx, Wy = axis_w(W, dw), axis_w(H, dh)
    tmp = np.einsum("hwc,xw->hxc", src, Wx, optimize=True)
    return np.einsum("yh,hxc->yxc", Wy, tmp, optimize=True)


def _cubic_k(t, A=-0.75):
    t = abs(t)
    if t <= 1:
        return (A + 2) * t ** 3 - (A + 3) * t ** 2 + 1
    if t < 2:
        return A * t ** 3 - 5 * A * t ** 2 + 8 * A * t - 4 * A
    return 0.0


def _lanczos_k(t, a=4):
    return 1.0 if t == 0 else (a * np.sin(np.pi * t) * np.sin(np.pi * t / a) / (np.pi * t) ** 2 if abs(t) < a else 0.0)


@pytest.mark.parametrize("dsize", [(224, 224), (53, 37), (300, 410)])
def test_cubic_close_to_float_bicubic(dsize):
    img = rng.integers(0, 256, (120, 170, 3), dtype=np.uint8)
    ref = np.clip(_ref_separable(img, dsize[0], dsize[1], _cubic_k, 4), 0, 255)
    out = R.resize(img, dsize, R.INTER_CUBIC).astype(np.float64)
    assert np.abs(out - ref).max() <= 1.5


@pytest.mark.parametrize("dsize", [(224, 224), (53, 37), (300, 410)])
def test_lanczos4_close_to_float_lanczos(dsize):
    img = rng.integers(0, 256, (120, 170, 3), dtype=np.uint8)
    ref = np.clip(_ref_separable(img, dsize[0], dsize[1], _lanczos_k, 8), 0, 255)
    out = R.resize(img, dsize, R.INTER_LANCZOS4).astype(np.float64)
    assert np.abs(out - ref).max() <= 2.0


def test_cubic_coefficients_partition_unity():
    for x in np.linspace(0, 0.999, 37, dtype=np.float32):
        c = R.cubic_coeffs(x)
        assert abs(float(sum(np.float64(v) for v in c)) - 1.0) < 1e-6
        l = R.lanczos4_coeffs(x)
        assert abs(float(sum(np.float64(v) for v in l)) - 1.0) < 1e-5
    assert R.lanczos4_coeffs(0.0)[3] == np.float32(1.0)


def test_cubic_simd_and_scalar_paths_agree_closely():
    """OpenCV's float (SIMD) and integer (tail) vertical cubic paths may differ
    in the last bit only: a 1-channel 13-wide output has 8 SIMD + 5 tail bytes."""
    img = rng.integers(0, 256, (40, 29), dtype=np.uint8)
    a = R.resize(img, (13, 50), R.INTER_CUBIC).astype(int)
    b = R.resize(img.T.copy(), (50, 13), R.INTER_CUBIC).T.astype(int)
    assert np.abs(a - b).max() <= 1


@pytest.mark.parametrize("dsize", [(224, 224), (53, 37), (300, 410), (131, 97)])
def test_linear_exact_close_to_float_bilinear(dsize):
    img = rng.integers(0, 256, (97, 131, 3), dtype=np.uint8)
    ref = _ref_separable(img, dsize[0], dsize[1], lambda t: max(0.0, 1 - abs(t)), 2)
    out = R.resize(img, dsize, R.INTER_LINEAR_EXACT).astype(np.float64)
    # 8-bit weights (1/512 each way) plus the final rounding
    assert np.abs(out - ref).max() <= 1.25


def test_linear_exact_half_size_is_area():
    img = rng.integers(0, 256, (64, 96, 3), dtype=np.uint8)
    assert np.array_equal(R.resize(img, (48, 32), R.INTER_LINEAR_EXACT), R.resize(img, (48, 32), R.INTER_AREA))


@pytest.mark.parametrize("src,dst", [(100, 50), (99, 33), (224, 224 * 3), (480, 224), (7, 300)])
def test_nearest_exact_picks_pixel_centres(src, dst):
    """resizeNN_bitexact: the source pixel under each destination pixel centre
    (floor((d + 0.5) * src / dst)), within the 16-bit fixed point's reach."""
    idx = R.nearest_exact_index(src, dst)
    exact = np.minimum(np.floor((np.arange(dst) + 0.5) * src / dst).astype(int), src - 1)
    assert np.abs(idx - exact).max() <= 1 and (idx == exact).mean() > 0.98


@pytest.mark.parametrize("interp,K", [(R.INTER_CUBIC, 4), (R.INTER_LANCZOS4, 8)])
@pytest.mark.parametrize("src,dst", [((135, 240), (224, 224)), ((4320, 7680), (331, 331)), ((7, 5), (299, 240)),
                                     ((224, 224), (448, 112)), ((1, 1), (3, 2)), ((68, 120), (240, 240))])
def test_engine_coefficient_tables_match_oracle(interp, K, src, dst):
    """The C++ host tables the GPU kernel reads (wicca_resize_kernel_tables,
    no device needed) equal the oracle's restatement of OpenCV's
    interpolateCubic / interpolateLanczos4 entry for entry."""
    import ctypes
    from wicca_amd import _lib
    lib = _lib.load()
    (H, W), (dh, dw) = src, dst
    need = ctypes.c_int64()
    assert lib.wicca_resize_kernel_tables(H, W, dw, dh, interp, None, 0, ctypes.byref(need)) == 0
    tab = (ctypes.c_int32 * need.value)()
    assert lib.wicca_resize_kernel_tables(H, W, dw, dh, interp, tab, need.value, ctypes.byref(need)) == 0
    t = np.frombuffer(tab, np.int32).astype(np.int64)
    xo, xa = R.kernel_tables(W, dw, W / dw if False else 1.0 / (dw / W), K)
    yo, yb = R.kernel_tables(H, dh, 1.0 / (dh / H), K)
    ref = np.concatenate([xo, xa.ravel(), yo, yb.ravel()])
    assert t.shape == ref.shape and np.array_equal(t, ref)


@pytest.mark.parametrize("shape", [(300, 517, 3), (1081, 1919, 3), (448, 448, 3), (77, 61, 1), (240, 480, 4),
                                   (135, 240, 3)])
@pytest.mark.parametrize("dsize", [(224, 224), (331, 331), (299, 299), (240, 240), (112, 112), (30, 20)])
def test_compiled_area_matches_numpy_restatement(shape, dsize):
    """oracle/area_cpu.c (the plan bench's compiled CPU baseline) gives the
    NumPy restatement's bytes for every INTER_AREA downscale and copy, and
    declines the upscales (OpenCV's bilinear path)."""
    from oracle import c_oracle
    img = rng.integers(0, 256, shape, dtype=np.uint8)
    got = c_oracle.area_resize(img, dsize)
    if dsize[0] > shape[1] or dsize[1] > shape[0]:
        assert got is None
        return
    want = R.resize(img, dsize, R.INTER_AREA)
    assert np.array_equal(got, want)
    view = np.zeros((shape[0], shape[1] + 5, shape[2]), np.uint8)[:, 2:2 + shape[1]]  # a strided view
    view[...] = img
    assert np.array_equal(c_oracle.area_resize(view, dsize), want)
