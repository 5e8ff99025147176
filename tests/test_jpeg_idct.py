"""The IDCT the reference's decoder runs on damaged data: libjpeg-turbo's
x86-64 SIMD ISLOW (oracle/jpeg_idct.py) pinned against Pillow's decode of
one-component files built around extreme coefficients and quantisers (CPU),
and the device's restatement of it (wicca_amd/csrc/jpeg.hip idct8_lane_v)
decoding the same files on the GPU."""
import io

import numpy as np
import pytest

from jpeg_scans import coef_file, gray_file
from oracle import jpeg_idct as I

W = H = 64


def _cases():
    """(coefficients (64 blocks x 64), quantisation table) probes: sparse
    full-range blocks, row-0-only blocks (pass 1's shortcut), DC-only blocks,
    small dense blocks; 8-bit and 16-bit quantisers; DC values accumulating
    up to the int16 range."""
    rng = np.random.default_rng(0)
    out = []
    for trial in range(24):
        mode = trial % 4
        qt = rng.integers(1, 256, 64) if trial % 3 else rng.integers(1, 65536, 64)
        co = np.zeros((64, 64), np.int64)
        if mode == 0:
            co[:] = rng.integers(-1023, 1024, (64, 64)) * (rng.random((64, 64)) < 0.3)
        elif mode == 1:
            co[:, :8] = rng.integers(-1023, 1024, (64, 8))
        elif mode == 3:
            co[:] = rng.integers(-50, 51, (64, 64)) * (rng.random((64, 64)) < 0.5)
        co[:, 0] = np.cumsum(rng.integers(-2047, 2048, 64)).clip(-32768, 32767)
        if np.abs(np.diff(np.concatenate([[0], co[:, 0]]))).max() > 2047:
            co[:, 0] = rng.integers(-2000, 2000, 64).cumsum().clip(-30000, 30000) // 2
        out.append((co.astype(np.int16), qt))
    return out


CASES = _cases()


def _image(px):
    """(64 blocks, 8, 8) in raster block order -> the 64 x 64 image."""
    return px.reshape(8, 8, 8, 8).transpose(0, 2, 1, 3).reshape(H, W)


def _pillow(data):
    from PIL import Image
    return np.asarray(Image.open(io.BytesIO(data)).convert("L"))


@pytest.mark.parametrize("i", range(len(CASES)))
def test_simd_idct_oracle_matches_pillow(i):
    co, qt = CASES[i]
    got = _pillow(gray_file(co, qt, W, H))
    assert np.array_equal(_image(I.idct_islow_simd(co, qt)), got)


def test_three_component_probe_decodes():
    """coef_file's 4:4:4 files decode (Pillow) with luma = the oracle's IDCT."""
    from PIL import Image
    n = len(CASES)
    data = coef_file([CASES[0], CASES[1 % n], CASES[2 % n]], W, H)
    im = Image.open(io.BytesIO(data))
    im.draft(None, None)
    assert im.size == (W, H) and im.mode == "RGB"
    ycc = np.asarray(Image.open(io.BytesIO(data)).convert("RGB"))
    assert ycc.shape == (H, W, 3)


def test_probes_separate_the_two_idcts():
    """The probes are ones where jidctint.c and the SIMD code disagree."""
    diff = sum(int((_image(I.idct_islow_c(co, qt)) != _image(I.idct_islow_simd(co, qt))).sum()) for co, qt in CASES)
    assert diff > 10_000


def test_valid_range_identical():
    """Coefficients of real encodes (|dequantised| within DCT range): both IDCTs agree."""
    rng = np.random.default_rng(9)
    co = (rng.normal(0, 30, (4000, 64)) * (rng.random((4000, 64)) < 0.4)).astype(np.int64)
    co[:, 0] = rng.integers(-127, 128, 4000)
    qt = rng.integers(1, 9, 64)
    assert np.array_equal(I.idct_islow_c(co, qt), I.idct_islow_simd(co, qt))


@pytest.mark.gpu
def test_device_idct_matches_pillow_on_extreme_files():
    """The whole GPU decode of the probe files (the one-component path: luma
    IDCT in the fused kernel) and of three-component variants (chroma IDCT
    kernel + colour) against Pillow."""
    from oracle import jpeg_pil as J
    from wicca_amd import jpeg as WJ
    files = [gray_file(co, qt, W, H) for co, qt in CASES]
    got = WJ.decode_batch(files)
    for i, data in enumerate(files):
        assert np.array_equal(got[i][..., 0], _pillow(data)), i
    n = len(CASES)
    files3 = [coef_file([CASES[i], CASES[(i + 1) % n], CASES[(i + 2) % n]], W, H) for i in range(n)]
    got3 = WJ.decode_batch(files3)
    for i, data in enumerate(files3):
        assert np.array_equal(got3[i], J.decode_rgb(data)), i
