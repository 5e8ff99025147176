"""CPU: the PNG / BMP / TIFF / GIF host half of the any-format decode (raster_host.cpp
through wicca_image_info, no device): format sniffing, header validation
with libpng / OpenCV BmpDecoder error behaviour, the committed golden files'
sizes, and the ASan + UBSan mutation fuzz (tests/native/raster_fuzz.cpp)."""
import json
import os
import struct
import zlib

import numpy as np
import pytest

from oracle import raster_ref as rr
from wicca_amd import jpeg as WJ

GOLD = os.path.join(os.path.dirname(__file__), "golden", "raster")
CASES = json.load(open(os.path.join(GOLD, "cases.json")))["cases"]


@pytest.mark.parametrize("case", CASES, ids=[c["file"] for c in CASES])
def test_golden_info(case):
    data = open(os.path.join(GOLD, case["file"]), "rb").read()
    h, w, kind = WJ.image_info(data)
    assert (h, w) == (case["height"], case["width"])
    ext = case["file"].rsplit(".", 1)[1]
    assert kind == {"tif": "tiff", "pgm": "pnm", "ppm": "pnm"}.get(ext, ext)


def _ihdr_png(w=4, h=3, bits=8, ct=2, il=0, crc_ok=True, idat=True, iend=True):
    ihdr = struct.pack(">IIBBBBB", w, h, bits, ct, 0, 0, il)
    chunk = struct.pack(">I", 13) + b"IHDR" + ihdr + struct.pack(">I", zlib.crc32(b"IHDR" + ihdr) ^ (0 if crc_ok else 1))
    out = rr.SIG + chunk
    if idat:
        out += rr._chunk(b"IDAT", zlib.compress(b"\0" * 16))
    if iend:
        out += rr._chunk(b"IEND", b"")
    return out


def test_png_header_errors():
    assert WJ.image_info(_ihdr_png())[:2] == (3, 4)
    for bad in [_ihdr_png(crc_ok=False), _ihdr_png(bits=3), _ihdr_png(ct=3, bits=16), _ihdr_png(ct=5),
                _ihdr_png(il=2), _ihdr_png(w=0), _ihdr_png(idat=False), _ihdr_png(iend=False),
                _ihdr_png(ct=3),  # palette image without PLTE
                rr.SIG + b"\x00\x00", rr.SIG]:
        with pytest.raises(ValueError):
            WJ.image_info(bad)
    with pytest.raises(NotImplementedError):
        WJ.image_info(_ihdr_png(w=70000))


def test_bmp_header_errors():
    img = np.zeros((5, 6, 3), np.uint8)
    good = rr.encode_bmp(img, 24)
    assert WJ.image_info(good)[:3] == (5, 6, "bmp")
    rle = good[:30] + struct.pack("<I", 1) + good[34:]
    bpp2 = good[:28] + struct.pack("<H", 2) + good[30:]
    bad565 = rr.encode_bmp(img, 16, fields565=True)
    k = bad565.index(struct.pack("<III", 0xF800, 0x7E0, 0x1F))
    bad_masks = bad565[:k] + struct.pack("<III", 0xFF00, 0xF0, 0xF) + bad565[k + 12:]
    for unsup in (bpp2, bad_masks):
        with pytest.raises(NotImplementedError):
            WJ.image_info(unsup)
    rle_ok, _ = rr.encode_bmp_rle(np.zeros((5, 6), np.uint8), np.zeros((4, 3), np.uint8))
    assert WJ.image_info(rle_ok)[:3] == (5, 6, "bmp")
    neg_w = good[:18] + struct.pack("<i", -6) + good[22:]
    # rle: BI_RLE8 on a 24-bit header is no valid BMP
    for bad in (good[:-1], good[:20], neg_w, good[:14] + struct.pack("<I", 20) + good[18:], rle):
        with pytest.raises(ValueError):
            WJ.image_info(bad)


def test_tiff_header_errors():
    img = np.zeros((6, 5, 3), np.uint8)
    good = rr.encode_tiff(img, 2, compression=8)
    assert WJ.image_info(good) == (6, 5, "tiff")
    for bad in (good[:7], b"II*\x00" + b"\0" * 20, good[:4] + b"\xff\xff\xff\x7f" + good[8:]):
        with pytest.raises(ValueError):
            WJ.image_info(bad)
    for unsup in (rr.encode_tiff(img.astype(np.uint16) * 257, 2, bits=16),          # 16-bit samples
                  rr.encode_tiff(np.zeros((6, 5, 4), np.uint8), 5),                 # CMYK
                  rr.encode_tiff(img, 2, compression=7)):                           # JPEG-in-TIFF
        with pytest.raises(NotImplementedError):
            WJ.image_info(unsup)


def test_gif_header_errors():
    idx = np.zeros((4, 6), np.uint8)
    good = rr.encode_gif(idx, np.array([[0, 0, 0], [255, 255, 255]], np.uint8), screen=(10, 8), pos=(2, 1))
    assert WJ.image_info(good) == (8, 10, "gif")
    for bad in (good[:12], b"GIF89a" + b"\0" * 20, good[:13] + b"\x3b", good[:6] + b"\0\0" + good[8:]):
        with pytest.raises(ValueError):
            WJ.image_info(bad)


def test_unrecognised_formats():
    for data in (b"GIF90a" + b"\0" * 20, b"", b"B", b"\x00\x00\x01\x00"):
        with pytest.raises(ValueError):
            WJ.image_info(data)


def test_raster_fuzz_sanitized():
    """ASan + UBSan build of raster_host.cpp under the chunk / header mutation
    fuzz, with the device conversion's read bounds checked for every accepted
    mutant (tests/native/raster_fuzz.cpp; seeds: tests/golden/raster/)."""
    import shutil
    import subprocess
    if shutil.which("g++") is None or not os.path.isdir("/opt/rocm/include"):
        pytest.skip("g++ or ROCm headers missing")
    csrc = os.path.join(os.path.dirname(__file__), "..", "wicca_amd", "csrc")
    r = subprocess.run(["make", "-s", "-C", csrc, "sanitize_raster", "FUZZ_ITERS=40000"], capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "iterations=40000" in r.stdout and "unpacked=" in r.stdout
