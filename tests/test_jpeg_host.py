"""JPEG host side without a GPU: the checker (Pillow / libjpeg-turbo) still
produces the committed golden decodes, and the C-ABI parser reads the files'
geometry, EXIF orientation and rejects what the GPU decoder does not handle."""
import ctypes
import hashlib
import json
import os

import numpy as np
import pytest

from oracle import jpeg_pil as J
from wicca_amd import _lib

GOLD = os.path.join(os.path.dirname(__file__), "golden", "jpeg")
META = json.load(open(os.path.join(GOLD, "cases.json")))
CASES = META["cases"]


def _read(name):
    return open(os.path.join(GOLD, name), "rb").read()


def _info(data, orient=1):
    arr = np.frombuffer(data, np.uint8)
    h, w = ctypes.c_int64(), ctypes.c_int64()
    c, o = ctypes.c_int(), ctypes.c_int()
    rc = _lib.load().wicca_jpeg_info(arr.ctypes.data, arr.size, orient, ctypes.byref(h), ctypes.byref(w),
                                     ctypes.byref(c), ctypes.byref(o))
    return rc, h.value, w.value, c.value, o.value


def test_checker_version_matches_fixtures():
    assert J.libjpeg_version() == META["libjpeg_turbo"]


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_checker_reproduces_golden(case):
    rgb = J.decode_rgb(_read(case["file"]))
    assert rgb.shape == (case["height"], case["width"], 3)
    assert hashlib.sha256(rgb.tobytes()).hexdigest() == case["sha256_rgb"]


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_parser_geometry_and_orientation(case):
    rc, h, w, c, o = _info(_read(case["file"]))
    assert rc == 0, _lib.last_error()
    assert (h, w) == (case["height"], case["width"])
    assert o == case["orientation"]
    assert c == (1 if case["name"].startswith("gray") else 3)


def test_parser_rejects_unsupported_and_corrupt():
    img = J.test_image("scene", 32, 32, 1)
    rc, *_ = _info(J.encode(img, progressive=True))
    assert rc == _lib.WICCA_ERR_UNSUPPORTED
    assert "progressive" in _lib.last_error()
    rc, *_ = _info(b"\x89PNG\r\n\x1a\n" + b"\x00" * 40)
    assert rc == _lib.WICCA_ERR_DECODE
    good = J.encode(img)
    rc, *_ = _info(good[:40])
    assert rc == _lib.WICCA_ERR_DECODE


def test_destuff_avx2_matches_scalar(tmp_path):
    """The 32-byte de-stuffer and the memchr one agree on 20,000 random scans."""
    import shutil
    import subprocess
    gxx = shutil.which("g++")
    if gxx is None or not os.path.isdir("/opt/rocm/include"):
        pytest.skip("g++ or ROCm headers missing")
    src = os.path.join(os.path.dirname(__file__), "native", "destuff_fuzz.cpp")
    exe = str(tmp_path / "destuff_fuzz")
    subprocess.run([gxx, "-O2", "-std=c++17", "-I/opt/rocm/include", "-D__HIP_PLATFORM_AMD__", src, "-o", exe],
                   check=True, capture_output=True, timeout=120)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and "bad=0" in r.stdout, r.stdout
