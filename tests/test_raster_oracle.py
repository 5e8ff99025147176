"""CPU: pin the PNG / BMP / TIFF restatement (oracle/raster_ref.py) to Pillow 12.2.0.

Every case the GPU test (tests/test_gpu_raster.py) compares against the
restatement is checked here against Pillow's own decoders first, except the
two parity-unpinned cases named in the oracle's header (16-bit gray PNG,
16-bit BMP), which are checked against hand-computed values instead.
"""
from __future__ import annotations

import io

import numpy as np
import pytest

from oracle import raster_ref as rr

PNG_CASES = [  # (colour type, bits)
    (0, 1), (0, 2), (0, 4), (0, 8), (2, 8), (2, 16), (3, 1), (3, 2), (3, 4), (3, 8), (4, 8), (4, 16),
    (6, 8), (6, 16),
]


def png_samples(ct: int, bits: int, h: int, w: int, seed: int):
    rng = np.random.default_rng(seed)
    ch = rr.CHANNELS[ct]
    hi = (1 << bits) if ct != 3 else min(1 << bits, 200)
    s = rng.integers(0, hi, (h, w, ch), dtype=np.int64)
    # smooth regions so the filters see non-trivial predictions
    s[: h // 2, : w // 2] = (np.arange(w // 2)[None, :, None] * 7 + np.arange(h // 2)[:, None, None] * 3) % hi
    pal = rng.integers(0, 256, (hi, 3), dtype=np.int64).astype(np.uint8) if ct == 3 else None
    return s, pal


@pytest.mark.parametrize("interlace", [False, True])
@pytest.mark.parametrize("ct,bits", PNG_CASES)
def test_png_oracle_vs_pillow(ct, bits, interlace):
    s, pal = png_samples(ct, bits, 37, 29, seed=ct * 100 + bits)
    data = rr.encode_png(s, ct, bits, interlace=interlace, palette=pal)
    got = rr.decode_png(data)
    assert got.shape == (37, 29, 3) and got.dtype == np.uint8
    if ct == 0 and bits == 16:
        return  # unpinned: checked in test_png16_gray_high_byte
    np.testing.assert_array_equal(got, rr.pillow_rgb(data))


@pytest.mark.parametrize("f", range(5))
def test_png_each_filter(f):
    s, _ = png_samples(2, 8, 16, 21, seed=f)
    data = rr.encode_png(s, 2, 8, filters=f)
    np.testing.assert_array_equal(rr.decode_png(data), rr.pillow_rgb(data))
    np.testing.assert_array_equal(rr.decode_png(data), s.astype(np.uint8))


def test_png16_gray_high_byte():
    s = np.array([[0, 255, 256, 65535, 0x1234]], np.int64)
    got = rr.decode_png(rr.encode_png(s, 0, 16))
    np.testing.assert_array_equal(got[0, :, 0], [0, 0, 1, 255, 0x12])


def test_png_tiny_interlaced_empty_passes():
    for h, w in [(1, 1), (1, 5), (3, 1), (2, 2), (5, 3)]:
        s, _ = png_samples(2, 8, h, w, seed=h * 10 + w)
        data = rr.encode_png(s, 2, 8, interlace=True)
        np.testing.assert_array_equal(rr.decode_png(data), rr.pillow_rgb(data))


def test_pillow_written_png():
    from PIL import Image
    rng = np.random.default_rng(3)
    img = rng.integers(0, 256, (40, 33, 3), dtype=np.uint8)
    for mode in ["RGB", "RGBA", "L", "LA", "P", "1"]:
        im = Image.fromarray(img).convert(mode)
        b = io.BytesIO()
        im.save(b, "PNG")
        np.testing.assert_array_equal(rr.decode_png(b.getvalue()), rr.pillow_rgb(b.getvalue()))


@pytest.mark.parametrize("bpp", [1, 4, 8, 24, 32])
@pytest.mark.parametrize("top_down", [False, True])
def test_bmp_oracle_vs_pillow(bpp, top_down):
    rng = np.random.default_rng(bpp)
    h, w = 19, 23
    if bpp <= 8:
        img = rng.integers(0, 1 << bpp, (h, w), dtype=np.uint8)
        pal = rng.integers(0, 256, (1 << bpp, 3), dtype=np.uint8)
    else:
        img = rng.integers(0, 256, (h, w, 3), dtype=np.uint8)
        pal = None
    data = rr.encode_bmp(img, bpp, palette=pal, top_down=top_down)
    want = pal[img] if bpp <= 8 else img
    np.testing.assert_array_equal(rr.decode_bmp(data), want)
    np.testing.assert_array_equal(rr.decode_bmp(data), rr.pillow_rgb(data))


def test_bmp_core_header_vs_pillow():
    rng = np.random.default_rng(7)
    img = rng.integers(0, 16, (9, 14), dtype=np.uint8)
    pal = rng.integers(0, 256, (16, 3), dtype=np.uint8)
    data = rr.encode_bmp(img, 4, palette=pal, core_header=True)
    np.testing.assert_array_equal(rr.decode_bmp(data), pal[img])
    np.testing.assert_array_equal(rr.decode_bmp(data), rr.pillow_rgb(data))


def test_pillow_written_bmp():
    from PIL import Image
    rng = np.random.default_rng(5)
    img = rng.integers(0, 256, (21, 30, 3), dtype=np.uint8)
    for mode in ["RGB", "L", "P", "1"]:
        b = io.BytesIO()
        Image.fromarray(img).convert(mode).save(b, "BMP")
        np.testing.assert_array_equal(rr.decode_bmp(b.getvalue()), rr.pillow_rgb(b.getvalue()))


@pytest.mark.parametrize("fields565", [None, False, True])
def test_bmp16_opencv_shifts(fields565):
    # unpinned (Pillow rescales by 255/31): OpenCV's icvCvt_BGR5552BGR / 5652BGR shifts
    img = np.array([[[255, 255, 255], [8, 4, 0], [0, 0, 255], [100, 50, 25]]], np.uint8)
    got = rr.decode_bmp(rr.encode_bmp(img, 16, fields565=fields565))
    if fields565:
        want = np.stack([img[..., 0] & 0xF8, img[..., 1] & 0xFC, img[..., 2] & 0xF8], axis=2)
    else:
        want = img & 0xF8
    np.testing.assert_array_equal(got, want)


# ----------------------------------------------------------------------------- TIFF
def tiff_case(kind: str, h: int, w: int, seed: int):
    """(samples, photometric, bits, colormap, extra) for a TIFF test image."""
    rng = np.random.default_rng(seed)
    if kind == "rgb":
        return rng.integers(0, 256, (h, w, 3), dtype=np.uint8), 2, 8, None, None
    if kind == "gray":
        return rng.integers(0, 256, (h, w), dtype=np.uint8), 1, 8, None, None
    if kind == "white":
        return rng.integers(0, 256, (h, w), dtype=np.uint8), 0, 8, None, None
    if kind in ("gray1", "gray4"):
        b = 1 if kind == "gray1" else 4
        return rng.integers(0, 1 << b, (h, w), dtype=np.uint8), 1, b, None, None
    if kind in ("pal8", "pal4"):
        b = 8 if kind == "pal8" else 4
        cm = rng.integers(0, 256, (1 << b, 3), dtype=np.int64) * 257
        return rng.integers(0, 1 << b, (h, w), dtype=np.uint8), 3, b, cm, None
    if kind == "rgba_assoc":
        return rng.integers(0, 256, (h, w, 4), dtype=np.uint8), 2, 8, None, 1
    raise ValueError(kind)


TIFF_KINDS = ["rgb", "gray", "white", "gray1", "gray4", "pal8", "pal4", "rgba_assoc"]


@pytest.mark.parametrize("kind", TIFF_KINDS)
@pytest.mark.parametrize("comp,pred,tile,be", [(1, 1, None, False), (8, 2, None, True), (32773, 1, (16, 32), False),
                                              (8, 1, (32, 16), True)])
def test_tiff_oracle_vs_pillow(kind, comp, pred, tile, be):
    s, photo, bits, cm, extra = tiff_case(kind, 37, 45, seed=len(kind))
    if bits != 8:
        pred = 1
    data = rr.encode_tiff(s, photo, bits, comp, pred, tile=tile, big_endian=be, colormap=cm, extra_samples=extra)
    if kind == "rgba_assoc":  # Pillow un-premultiplies; libtiff (cv2) keeps the stored colours
        with pytest.raises(NotImplementedError):
            rr.decode_tiff(data)
        return
    got = rr.decode_tiff(data)
    np.testing.assert_array_equal(got, rr.pillow_rgb(data))
    if kind == "rgb":
        np.testing.assert_array_equal(got, s)
    if kind == "white":
        np.testing.assert_array_equal(got[..., 0], 255 - s)


def test_tiff_unassociated_alpha_premultiplied():
    # unpinned (Pillow drops alpha): libtiff's RGBA interface premultiplies
    px = np.array([[[200, 100, 50, 128], [255, 255, 255, 0], [10, 20, 30, 255]]], np.uint8)
    got = rr.decode_tiff(rr.encode_tiff(px, 2, extra_samples=2))
    np.testing.assert_array_equal(got[0], [[100, 50, 25], [0, 0, 0], [10, 20, 30]])


# ----------------------------------------------------------------------------- GIF
@pytest.mark.parametrize("interlace", [False, True])
@pytest.mark.parametrize("h,w,npal", [(1, 1, 2), (7, 5, 4), (20, 30, 256), (64, 100, 16)])
def test_gif_writer_and_expected_vs_pillow(h, w, npal, interlace):
    rng = np.random.default_rng(h * w + npal)
    idx = rng.integers(0, npal, (h, w), dtype=np.uint8)
    pal = rng.integers(0, 256, (npal, 3), dtype=np.uint8)
    data = rr.encode_gif(idx, pal, interlace=interlace)
    np.testing.assert_array_equal(rr.gif_expected(idx, pal), rr.pillow_rgb(data))


@pytest.mark.parametrize("rle4", [False, True])
@pytest.mark.parametrize("absolute,skips", [(False, False), (True, False), (True, True)])
def test_rle_bmp_writer_matches_pillow(rle4, absolute, skips):
    """oracle encode_bmp_rle's files and expected indices against Pillow's
    decode (encoded and absolute runs, end of line, delta escapes)."""
    rng = np.random.default_rng(11 + 2 * rle4 + skips)
    pal = rng.integers(0, 256, (16 if rle4 else 256, 3)).astype(np.uint8)
    for shape in ((37, 53), (1, 1), (2, 255), (64, 300)):
        idx = rng.integers(0, len(pal), shape).astype(np.uint8)
        idx[:, : shape[1] // 3] = idx[:, :1]  # long runs too
        data, want = rr.encode_bmp_rle(idx, pal, rle4, absolute, skips)
        assert np.array_equal(rr.pillow_rgb(data), pal[want]), shape


def test_pnm_writer_matches_pillow():
    rng = np.random.default_rng(3)
    for img in (rng.integers(0, 256, (17, 29), dtype=np.uint8), rng.integers(0, 256, (8, 5, 3), dtype=np.uint8)):
        got = rr.pillow_rgb(rr.encode_pnm(img))
        want = np.repeat(img[..., None], 3, axis=2) if img.ndim == 2 else img
        assert np.array_equal(got, want)
