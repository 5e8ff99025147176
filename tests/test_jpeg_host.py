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
    assert c == (1 if "gray" in case["name"] else 3)


def test_parser_rejects_unsupported_and_corrupt():
    img = J.test_image("scene", 32, 32, 1)
    good = J.encode(img)
    sof = good.index(b"\xff\xc0")
    lossless = good[:sof + 1] + b"\xc3" + good[sof + 2:]  # SOF3: lossless
    rc, *_ = _info(lossless)
    assert rc == _lib.WICCA_ERR_UNSUPPORTED and "lossless" in _lib.last_error()
    arith = good[:sof + 1] + b"\xc9" + good[sof + 2:]  # SOF9: arithmetic coding
    rc, *_ = _info(arith)
    assert rc == _lib.WICCA_ERR_UNSUPPORTED
    rc, *_ = _info(b"\x89PNG\r\n\x1a\n" + b"\x00" * 40)
    assert rc == _lib.WICCA_ERR_DECODE
    rc, *_ = _info(good[:40])
    assert rc == _lib.WICCA_ERR_DECODE


def test_progressive_parses():
    data = J.encode(J.test_image("scene", 37, 53, 1), 80, 2, progressive=True)
    rc, h, w, c, o = _info(data)
    assert rc == 0 and (h, w, c) == (37, 53, 3)


def _host_coefs(data, force):
    from jpeg_scans import coefficients
    return coefficients(data, force)


PROG = [("scene", 64, 80, 2, 75, 0), ("noise", 135, 241, 0, 70, 0), ("smooth", 333, 517, 1, 50, 0),
        ("gray", 50, 77, 0, 80, 0), ("scene", 480, 640, 2, 85, 3), ("noise", 200, 300, 2, 60, 1),
        ("scene", 17, 9, 1, 95, 0), ("smooth", 256, 256, 2, 30, 7)]


@pytest.mark.parametrize("kind,H,W,sub,q,rb", PROG, ids=[f"{k}-{h}x{w}-s{s}-q{q}-r{r}" for k, h, w, s, q, r in PROG])
def test_progressive_coefficients_equal_baseline(kind, H, W, sub, q, rb):
    """libjpeg-turbo codes the same quantised DCT coefficients progressively
    (DC / AC first and refinement scans, EOB runs) or in one sequential scan;
    the host progressive decoder (jdphuff.c semantics) must recover exactly the
    coefficients the sequential decoder reads from the baseline file.  No GPU."""
    img = J.test_image(kind, H, W, H + W + sub)
    base = J.encode(img, q, sub, rb)
    prog = J.encode(img, q, sub, rb, progressive=True)
    assert np.array_equal(_host_coefs(base, 1), _host_coefs(prog, 0))


SPLIT = [("scene", 64, 80, 2, 75, (0, 1, 2), 0), ("noise", 135, 241, 0, 70, (2, 0, 1), 0),
         ("smooth", 333, 517, 1, 50, (1, 2, 0), 0), ("gray", 50, 77, 0, 80, (0,), 0),
         ("scene", 17, 9, 2, 95, (0, 1, 2), 0), ("noise", 201, 299, 2, 60, (0, 2, 1), 0),
         ("scene", 120, 200, 2, 80, (0, 1, 2), 7), ("gray", 64, 64, 0, 90, (0,), 1),
         ("smooth", 99, 161, 1, 60, (2, 1, 0), 40)]


def _real_blocks(data, coefs):
    """Mask of the coded blocks: a non-interleaved scan covers only the
    component's ceil(dw/8) x ceil(dh/8) blocks, not the MCU padding."""
    from jpeg_scans import _segments
    sof = next(p for m, p in _segments(data) if m in (0xC0, 0xC1))
    H, W, nc = (sof[1] << 8) | sof[2], (sof[3] << 8) | sof[4], sof[5]
    hv = [(sof[7 + 3 * c] >> 4, sof[7 + 3 * c] & 15) if nc > 1 else (1, 1) for c in range(nc)]
    hmax, vmax = max(h for h, _ in hv), max(v for _, v in hv)
    mask = []
    for h, v in hv:
        bw, bh = -(-W // (8 * hmax)) * h, -(-H // (8 * vmax)) * v
        wb, hb = -(-(-(-W * h // hmax)) // 8), -(-(-(-H * v // vmax)) // 8)
        m = np.zeros((bh, bw), bool)
        m[:hb, :wb] = True
        mask.append(m.ravel())
    mask = np.concatenate(mask)
    assert mask.size * 64 == coefs.size
    return mask


@pytest.mark.parametrize("kind,H,W,sub,q,order,ri", SPLIT,
                         ids=[f"{k}-{h}x{w}-s{s}-o{''.join(map(str, o))}-r{r}" for k, h, w, s, q, o, r in SPLIT])
def test_multiscan_sequential_coefficients(kind, H, W, sub, q, order, ri):
    """A baseline file re-coded as one non-interleaved scan per component (in
    any component order, own Huffman tables): Pillow decodes it to the same
    pixels as the original (the writer is right), and the host sequential
    multi-scan decoder recovers the original's coefficients, with and without
    restart intervals.  No GPU."""
    from jpeg_scans import split_scans
    img = J.test_image(kind, H, W, H * W + sub)
    base = J.encode(img, q, sub)
    ref = _host_coefs(base, 1)
    split = split_scans(base, ref, order, ri)
    assert split.count(b"\xff\xda") == len(order)
    assert np.array_equal(J.decode_rgb(split), J.decode_rgb(base))
    got = _host_coefs(split, int(len(order) == 1))  # one gray scan is a single-scan (device) file
    mask = np.repeat(_real_blocks(base, ref), 64)
    assert np.array_equal(got[mask], ref[mask])
    assert not got[~mask].any()


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


def _segments(data):
    """(offset, length incl. marker, marker) of the segments before the scan."""
    out, p = [], 2
    while p + 4 <= len(data) and data[p] == 0xFF:
        m = data[p + 1]
        ln = (data[p + 2] << 8) | data[p + 3]
        out.append((p, 2 + ln, m))
        if m == 0xDA:
            break
        p += 2 + ln
    return out


def _seed():
    return bytearray(_read("scene_420_q75.jpg"))


def test_parser_rejects_oversubscribed_huffman_table():
    """bits[1] = 3: libjpeg-turbo's 'Bogus Huffman table
    definition'; used to write past the 512-entry lookup."""
    for counts in ({1: 3}, {1: 2}, {1: 1, 2: 2}, {2: 4}, {9: 255}):
        d = _seed()
        at, _, _ = [s for s in _segments(d) if s[2] == 0xC4][0]
        body = at + 4
        for l in range(1, 17):
            d[body + l] = 0
        total = 0
        for l, n in counts.items():
            d[body + l] = n
            total += n
        # keep the segment consistent: the first table's values are reused as
        # they are (the length field still covers them when total is small)
        rc, *_ = _info(bytes(d))
        assert rc in (_lib.WICCA_ERR_DECODE,), (counts, rc, _lib.last_error())


def test_parser_rejects_dc_symbol_above_15():
    d = _seed()
    for at, ln, m in _segments(d):
        if m == 0xC4 and (d[at + 4] >> 4) == 0:  # a DC table
            d[at + 4 + 17] = 16
            break
    rc, *_ = _info(bytes(d))
    assert rc == _lib.WICCA_ERR_DECODE and "Huffman" in _lib.last_error()


def test_parser_rejects_subsampled_luma_and_duplicate_ids():
    d = _seed()
    at, _, _ = [s for s in _segments(d) if s[2] in (0xC0, 0xC1)][0]
    y = at + 4 + 6
    sub = bytearray(d)
    sub[y + 1] = 0x11   # Y 1x1
    sub[y + 4] = 0x22   # Cb 2x2
    rc, *_ = _info(bytes(sub))
    assert rc == _lib.WICCA_ERR_UNSUPPORTED and "luma" in _lib.last_error()
    dup = bytearray(d)
    dup[y + 3] = dup[y]  # Cb id = Y id
    rc, *_ = _info(bytes(dup))
    assert rc == _lib.WICCA_ERR_DECODE and "duplicate" in _lib.last_error()
    dsos = bytearray(d)
    at, _, _ = [s for s in _segments(d) if s[2] == 0xDA][0]
    dsos[at + 7] = dsos[at + 5]  # second scan component = first
    rc, *_ = _info(bytes(dsos))
    assert rc == _lib.WICCA_ERR_DECODE and "duplicate" in _lib.last_error()


def test_parser_short_sos_at_end_of_buffer():
    d = _seed()
    at, _, _ = [s for s in _segments(d) if s[2] == 0xDA][0]
    cut = bytes(d[:at]) + b"\xff\xda\x00\x02"  # SOS with an empty payload, nothing after it
    arr = np.frombuffer(cut, np.uint8).copy()
    rc, *_ = _info(arr.tobytes())
    assert rc == _lib.WICCA_ERR_DECODE


def test_parser_fuzz_sanitized():
    """ASan + UBSan build of jpeg_host.cpp under the marker-segment mutation
    fuzz (tests/native/parser_fuzz.cpp; seeds: the golden JPEGs)."""
    import shutil
    import subprocess
    if shutil.which("g++") is None or not os.path.isdir("/opt/rocm/include"):
        pytest.skip("g++ or ROCm headers missing")
    csrc = os.path.join(os.path.dirname(__file__), "..", "wicca_amd", "csrc")
    r = subprocess.run(["make", "-s", "-C", csrc, "sanitize", "FUZZ_ITERS=60000"], capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "iterations=60000" in r.stdout and "accepted=" in r.stdout


def test_all_slots_unreadable_needs_no_device(tmp_path, capsys):
    """Per-slot failure without a GPU: when no file of a batch parses, every
    slot fails on its own (None / zero outputs) and nothing reaches the device."""
    from wicca_amd import jpeg as WJ
    import wicca_amd
    bad = [b"\x89PNG\r\n\x1a\n" + b"\x00" * 64, b"\xff\xd8\xff\xdb\x00", b""]
    bad[2] = b"not a jpeg at all"
    assert WJ.decode_batch(bad, errors="none") == [None, None, None]
    paths = []
    for i, b in enumerate(bad):
        p = tmp_path / f"b{i}.jpg"
        p.write_bytes(b)
        paths.append(str(p))
    imgs, icons = wicca_amd.get_img_batch(paths, (32, 32), 3, errors="zero")
    assert imgs.shape == (3, 32, 32, 3) and not imgs.any() and not icons.any()
    out = capsys.readouterr().out
    assert all(f"Error loading image {p}" in out for p in paths)
    with pytest.raises(ValueError):
        WJ.decode_batch(bad)


def test_load_image_prints_the_reference_message(tmp_path, capsys, monkeypatch):
    """An unreadable file: load_image prints what the reference prints for any
    file cv2.imread cannot read (validate_image's message for None,
    validation.py:94-95) and returns None; WICCA_LOAD_DETAIL=1 prints the
    decoder's reason instead.  No device is needed (the file fails to parse)."""
    import wicca_amd
    p = tmp_path / "notes.txt"
    p.write_bytes(b"not an image at all")
    assert wicca_amd.load_image(str(p)) is None
    assert capsys.readouterr().out.strip() == \
        f"Error loading image {p}: Image didn't found. Please check your input."
    monkeypatch.setenv("WICCA_LOAD_DETAIL", "1")
    assert wicca_amd.load_image(str(p)) is None
    assert "unrecognised image format" in capsys.readouterr().out


def host_coefs_as_libjpeg_pixels(data: bytes, img, quality: int, sub: int):
    """libjpeg-turbo's pixels for the host entropy decoder's coefficients of
    `data`: the coefficients re-encoded as a sequential file (tests/jpeg_scans.py;
    same quantisation tables: a baseline encode of the same image and quality)
    and decoded by Pillow."""
    from jpeg_scans import coefficients, split_scans
    base = J.encode(img, quality, sub)
    return J.decode_rgb(split_scans(base, coefficients(data, 1)))


DAMAGED = [("scene", 2, 0), ("scene", 2, 8), ("noise", 0, 0), ("scene", 1, 3), ("gray", 0, 0), ("smooth", 2, 16)]


@pytest.mark.parametrize("kind,sub,rb", DAMAGED, ids=[f"{k}-s{s}-r{r}" for k, s, r in DAMAGED])
@pytest.mark.parametrize("cut", [0.2, 0.3, 0.5, 0.7, 0.95, 0.999])
def test_host_decoder_on_truncated_files_matches_libjpeg(kind, sub, rb, cut):
    """The host entropy decoder (which redoes every file the device marks
    damaged) on a truncated file: its coefficients give libjpeg-turbo's pixels
    for the file (Pillow with LOAD_TRUNCATED_IMAGES: the fake EOI cv2.imread's
    source manager also inserts; the running MCU decoded on from zero bits,
    the rest grey)."""
    img = J.test_image(kind, 200, 344, 17 + sub + rb)
    if kind == "gray":
        img = img[..., 0] if img.ndim == 3 else img
    data = J.encode(img, 88, sub, rb)
    short = data[:int(len(data) * cut)]
    assert np.array_equal(host_coefs_as_libjpeg_pixels(short, img, 88, sub), J.decode_rgb(short, truncated=True))


@pytest.mark.parametrize("seed", range(10))
def test_host_decoder_on_corrupted_files_matches_libjpeg(seed):
    """Flipped bytes inside the entropy-coded data (markers intact): codes no
    table has (17 bits, symbol 0), runs past coefficient 63 (written to 63),
    segments whose data runs out; the host decoder's coefficients give
    libjpeg-turbo's pixels."""
    rng = np.random.default_rng(100 + seed)
    kind = ("scene", "noise", "smooth")[seed % 3]
    sub = seed % 3
    img = J.test_image(kind, 160, 232, seed)
    data = bytearray(J.encode(img, 80, sub, 8 if seed % 2 else 0))
    sos = bytes(data).index(b"\xff\xda")
    start = sos + 2 + int.from_bytes(data[sos + 2:sos + 4], "big")
    for pos in rng.integers(start + 4, len(data) - 4, 3 + seed):
        if data[pos] != 0xFF and data[pos - 1] != 0xFF:
            nv = data[pos] ^ int(rng.integers(1, 255))
            if nv != 0xFF:
                data[pos] = nv
    try:
        got = host_coefs_as_libjpeg_pixels(bytes(data), img, 80, sub)
    except KeyError:  # a coefficient the re-encoder's tables cannot code (size > 10)
        pytest.skip("coefficients outside the baseline tables")
    assert np.array_equal(got, J.decode_rgb(bytes(data), truncated=True))


RST_DAMAGE = ["next1", "next2", "prior1", "far", "dropped", "garbage-ff00", "not-rst"]


@pytest.mark.parametrize("how", RST_DAMAGE)
def test_host_decoder_resyncs_restart_markers_like_libjpeg(how):
    """Damaged restart markers: libjpeg's read_restart_marker /
    jpeg_resync_to_restart (an RSTn one or two ahead leaves the segment empty,
    one or two behind is skipped, one further off is taken; stray bytes with
    FF00 pairs before a marker are skipped) -- the host decoder's coefficients
    give libjpeg-turbo's pixels."""
    img = J.test_image("scene", 160, 232, 5)
    data = bytearray(J.encode(img, 85, 2, 4))
    sos = bytes(data).index(b"\xff\xda")
    start = sos + 2 + int.from_bytes(data[sos + 2:sos + 4], "big")
    rst = [i for i in range(start, len(data) - 1) if data[i] == 0xFF and 0xD0 <= data[i + 1] <= 0xD7]
    at = rst[len(rst) // 3]
    num = data[at + 1] - 0xD0
    if how in ("next1", "next2", "prior1", "far"):
        data[at + 1] = 0xD0 + (num + {"next1": 1, "next2": 2, "prior1": -1, "far": 4}[how]) % 8
    elif how == "dropped":
        del data[at:at + 2]
    elif how == "garbage-ff00":
        data[at:at] = b"\x12\xff\x00\x34\xff\xff\x00\x56"
    else:
        data[at + 1] = 0x01  # TEM: a code below SOF0, skipped by the resync
    got = host_coefs_as_libjpeg_pixels(bytes(data), img, 85, 2)
    assert np.array_equal(got, J.decode_rgb(bytes(data), truncated=True))
