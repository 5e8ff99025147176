"""GPU cv2.resize (wicca_resize_u8 / wicca_icon_stage_u8) against the CPU
restatement oracle/resize_cv.py, bit for bit.  Shapes follow the reference's
caller (classifying_tools.py:315, :318): 8K / 4K sources and the icons of
depths 1-6 resized to the demo's classifier inputs (224, 240, 299, 331),
plus OpenCV's special cases (integer scales, copies, upscales, C = 1..4).
Parity against an OpenCV binary is unpinned (cv2 absent)."""
import ctypes

import numpy as np
import pytest

import wicca_amd
from oracle import c_oracle
from oracle import resize_cv as R
from wicca_amd import _lib

pytestmark = pytest.mark.gpu

CASES = [
    ((135, 240), (224, 224)), ((68, 120), (224, 224)), ((270, 480), (224, 224)),
    ((540, 960), (240, 240)), ((1080, 1920), (299, 299)), ((2160, 3840), (331, 331)),
    ((448, 448), (224, 224)), ((672, 896), (224, 224)), ((100, 150), (50, 75)),
    ((101, 99), (331, 331)), ((30, 40), (40, 30)), ((33, 47), (47, 33)), ((64, 64), (64, 64)),
    ((17, 3), (5, 9)), ((5, 700), (224, 1)), ((1, 1), (3, 2)),
]


@pytest.mark.parametrize("interp", R.SUPPORTED)
@pytest.mark.parametrize("shape,dsize", CASES, ids=[f"{s[0]}x{s[1]}-{d[0]}x{d[1]}" for s, d in CASES])
def test_resize_rgb_matches_oracle(shape, dsize, interp):
    rng = np.random.default_rng(hash((shape, dsize, interp)) % 2**32)
    img = rng.integers(0, 256, shape + (3,), dtype=np.uint8)
    assert np.array_equal(wicca_amd.resize(img, dsize, interp), R.resize(img, dsize, interp))


@pytest.mark.parametrize("C", [1, 2, 4])
@pytest.mark.parametrize("interp", R.SUPPORTED)
def test_resize_channels(C, interp):
    rng = np.random.default_rng(C * 10 + interp)
    for shape, dsize in (((135, 240), (224, 224)), ((96, 64), (48, 32)), ((77, 91), (300, 20))):
        img = rng.integers(0, 256, shape + (C,), dtype=np.uint8)
        got = wicca_amd.resize(img, dsize, interp)
        assert np.array_equal(got, R.resize(img, dsize, interp)), (shape, dsize)
    assert wicca_amd.resize(img[:, :, 0], (10, 10), interp).shape == (10, 10)


def test_resize_8k_source_to_224():
    """The caller's source resize at BASELINE configs[2] size (one 8K RGB image)."""
    from wicca_amd.synth import synth_image
    img = synth_image(5, 0, 4320, 7680, 3)
    assert np.array_equal(wicca_amd.resize(img, (224, 224), R.INTER_AREA),
                          R.resize(img, (224, 224), R.INTER_AREA))


def test_resize_strided_view():
    rng = np.random.default_rng(2)
    big = rng.integers(0, 256, (300, 500, 3), dtype=np.uint8)
    view = big[10:250, 7:400]
    assert np.array_equal(wicca_amd.resize(view, (224, 224)), R.resize(view, (224, 224)))


def test_resize_rejects_unimplemented_interpolation():
    with pytest.raises(ValueError, match="interpolation 7"):
        wicca_amd.resize(np.zeros((8, 8, 3), np.uint8), (4, 4), 7)


def test_resize_uniform_device_batch():
    torch = pytest.importorskip("torch")
    n, H, W, C, dw, dh = 6, 135, 240, 3, 224, 224
    rng = np.random.default_rng(9)
    host = rng.integers(0, 256, (n, H, W, C), dtype=np.uint8)
    src = torch.from_numpy(host).cuda()
    dst = torch.empty((n, dh, dw, C), dtype=torch.uint8, device="cuda")
    _lib.check(_lib.load().wicca_resize_u8_uniform(
        ctypes.c_void_p(src.data_ptr()), n, H, W, C, W * C, H * W * C,
        ctypes.c_void_p(dst.data_ptr()), dw, dh, dw * C, dh * dw * C, R.INTER_AREA, -1, None))
    got = dst.cpu().numpy()
    for i in range(n):
        assert np.array_equal(got[i], R.resize(host[i], (dw, dh), R.INTER_AREA))


@pytest.mark.parametrize("depth,shape,interp", [(5, (224, 224), 3), (2, (299, 299), 3),
                                                (6, (331, 331), 1), (3, (240, 240), 0),
                                                (0, (224, 224), 3), (9, (224, 224), 3)])
def test_icon_stage_equals_caller_composition(coder, depth, shape, interp):
    """_get_img_batch (classifying_tools.py:312-323) on decoded images: resized
    source + resized icon, stacked — vs the oracle composition."""
    rng = np.random.default_rng(depth)
    sizes = [(431, 645), (1080, 1920), (97, 1201), (600, 600), (1023, 777)]
    imgs = [rng.integers(0, 256, s + (3,), dtype=np.uint8) for s in sizes]
    got_img, got_icon = coder.icon_stage(imgs, depth, shape, interp)
    assert got_img.shape == (len(imgs), shape[1], shape[0], 3) == got_icon.shape
    for i, im in enumerate(imgs):
        assert np.array_equal(got_img[i], R.resize(im, shape, interp)), i
        icon = c_oracle.ll_f32_levels(im, depth)[0] if depth > 0 else im
        assert np.array_equal(got_icon[i], R.resize(icon, shape, interp)), i


def test_icon_stage_constant_border(coder):
    rng = np.random.default_rng(4)
    imgs = [rng.integers(0, 256, s + (3,), dtype=np.uint8) for s in ((100, 130), (64, 64))]
    got_img, got_icon = coder.icon_stage(imgs, 3, (224, 224), 3, border_type=0, border_constant=77)
    for i, im in enumerate(imgs):
        icon = c_oracle.ll_int_block(im, 3, 0, 77)[0]
        assert np.array_equal(got_icon[i], R.resize(icon, (224, 224), 3)), i


def test_resize_uniform_device_batch_area_two_pass():
    """INTER_AREA downscales of a device batch take the two-pass path (row sums
    in workspace scratch, several images per launch); rows wider than the LDS
    stage (W * C > 24 KiB) take the one-pass kernel."""
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(12)
    for (n, H, W, dw, dh) in ((5, 540, 960, 224, 224), (2, 41, 8500, 100, 20)):
        C = 3
        host = rng.integers(0, 256, (n, H, W, C), dtype=np.uint8)
        pitch = (W * C + 15) // 16 * 16
        src = torch.zeros((n, H, pitch), dtype=torch.uint8, device="cuda")
        src[:, :, :W * C] = torch.from_numpy(host.reshape(n, H, W * C)).cuda()
        dst = torch.empty((n, dh, dw, C), dtype=torch.uint8, device="cuda")
        _lib.check(_lib.load().wicca_resize_u8_uniform(
            ctypes.c_void_p(src.data_ptr()), n, H, W, C, pitch, H * pitch,
            ctypes.c_void_p(dst.data_ptr()), dw, dh, dw * C, dh * dw * C, R.INTER_AREA, -1, None))
        got = dst.cpu().numpy()
        for i in range(n):
            assert np.array_equal(got[i], R.resize(host[i], (dw, dh), R.INTER_AREA)), (H, W, i)
