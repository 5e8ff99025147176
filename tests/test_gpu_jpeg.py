"""GPU JPEG decode (load_image, data_loader.py:31-63) against libjpeg-turbo
3.1.4.1 through Pillow (oracle/jpeg_pil.py), bit for bit: the committed golden
files, then a generated corpus over content, sizes (MCU-aligned and ragged),
qualities, 4:4:4 / 4:2:2 / 4:2:0 / grayscale, restart intervals, optimised
Huffman tables and EXIF orientations; batched decode; the file-based caller
stage (_get_img_batch, classifying_tools.py:297-323)."""
import hashlib
import json
import os

import numpy as np
import pytest

import wicca_amd
from oracle import c_oracle
from oracle import jpeg_pil as J
from oracle import resize_cv as R
from wicca_amd import _lib
from wicca_amd import jpeg as WJ

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden", "jpeg")
CASES = json.load(open(os.path.join(GOLD, "cases.json")))["cases"]


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_golden_files(case):
    data = open(os.path.join(GOLD, case["file"]), "rb").read()
    rgb = WJ.decode(data)
    assert rgb.shape == (case["height"], case["width"], 3)
    assert hashlib.sha256(rgb.tobytes()).hexdigest() == case["sha256_rgb"]


GEN = []
for kind in ("scene", "noise", "smooth"):
    for (H, W) in ((16, 16), (17, 33), (64, 80), (135, 241), (333, 517)):
        for sub in (0, 1, 2):
            for q in (50, 95):
                GEN.append((kind, H, W, sub, q, 0, False))
GEN += [("scene", 480, 640, 2, 75, rb, opt) for rb in (1, 5, 64) for opt in (False, True)]
GEN += [("scene", 1080, 1920, sub, 85, 0, False) for sub in (0, 1, 2)]
GEN += [("noise", 2160, 3840, 2, 100, 0, False), ("scene", 4320, 7680, 2, 90, 0, False)]


@pytest.mark.parametrize("kind,H,W,sub,q,rb,opt", GEN,
                         ids=[f"{k}-{h}x{w}-s{s}-q{q}-r{r}-o{int(o)}" for k, h, w, s, q, r, o in GEN])
def test_generated_corpus(kind, H, W, sub, q, rb, opt):
    img = J.test_image(kind, H, W, H * 7 + W + sub)
    data = J.encode(img, q, sub, rb, 0, opt)
    assert np.array_equal(WJ.decode(data), J.decode_rgb(data))


@pytest.mark.parametrize("H,W", [(9, 13), (64, 64), (250, 333)])
@pytest.mark.parametrize("q", [40, 90, 100])
def test_grayscale(H, W, q):
    img = J.test_image("gray", H, W, q)
    data = J.encode(img, q, restart_rows=1 if q == 90 else 0)
    got = WJ.decode(data)
    assert np.array_equal(got, J.decode_rgb(data))
    assert np.array_equal(got[:, :, 0], got[:, :, 2])


@pytest.mark.parametrize("orient", range(1, 9))
def test_exif_orientation(orient):
    img = J.test_image("scene", 37, 58, orient)
    data = J.encode(img, 85, 2, orientation=orient)
    assert np.array_equal(WJ.decode(data), J.decode_rgb(data, apply_orientation=True))
    assert np.array_equal(WJ.decode(data, apply_orientation=False),
                          J.decode_rgb(data, apply_orientation=False))


def test_batch_decode_mixed():
    blobs = [J.encode(J.test_image(k, h, w, i), q, s, rb)
             for i, (k, h, w, q, s, rb) in enumerate([("scene", 100, 120, 75, 2, 0),
                                                      ("noise", 31, 77, 90, 0, 3),
                                                      ("gray", 50, 50, 60, 0, 0),
                                                      ("smooth", 240, 320, 95, 1, 0)])]
    got = WJ.decode_batch(blobs)
    for b, g in zip(blobs, got):
        assert np.array_equal(g, J.decode_rgb(b))


PROG = [(k, h, w, s, q, rb) for k, (h, w) in (("scene", (333, 517)), ("smooth", (64, 80)), ("gray", (97, 55)))
        for s in (0, 1, 2) for q, rb in ((50, 0), (90, 0), (85, 4))]
PROG += [("scene", 1080, 1920, 2, 90, 0), ("noise", 200, 300, 2, 60, 1), ("scene", 4320, 7680, 2, 85, 0)]


@pytest.mark.parametrize("kind,H,W,sub,q,rb", PROG, ids=[f"{k}-{h}x{w}-s{s}-q{q}-r{r}" for k, h, w, s, q, r in PROG])
def test_progressive_matches_libjpeg(kind, H, W, sub, q, rb):
    """Progressive JPEG (SOF2, libjpeg's default progression: DC / AC first
    and refinement scans): host entropy decode + the device back end, bit for
    bit against libjpeg-turbo."""
    img = J.test_image(kind, H, W, H * 3 + W + sub)
    data = J.encode(img, q, sub, rb, progressive=True)
    assert np.array_equal(WJ.decode(data), J.decode_rgb(data))


SPLIT = [("scene", 333, 517, 2, 85, (0, 1, 2), 0), ("noise", 135, 241, 0, 70, (2, 0, 1), 0),
         ("smooth", 64, 80, 1, 50, (1, 2, 0), 3), ("scene", 1080, 1920, 2, 90, (0, 2, 1), 0),
         ("scene", 17, 9, 2, 95, (2, 1, 0), 1), ("noise", 240, 320, 2, 75, (0, 1, 2), 100)]


@pytest.mark.parametrize("kind,H,W,sub,q,order,ri", SPLIT,
                         ids=[f"{k}-{h}x{w}-s{s}-o{''.join(map(str, o))}-r{r}" for k, h, w, s, q, o, r in SPLIT])
def test_multiscan_sequential_matches_libjpeg(kind, H, W, sub, q, order, ri):
    """A sequential file with one non-interleaved scan per component (T.81
    A.2.2; re-coded from a baseline file by tests/jpeg_scans.py): host entropy
    decode + the device back end, bit for bit against libjpeg-turbo, and in a
    batch with the device-decoded original."""
    from jpeg_scans import coefficients, split_scans
    img = J.test_image(kind, H, W, H * 5 + W + sub)
    base = J.encode(img, q, sub)
    split = split_scans(base, coefficients(base, 1), order, ri)
    ref = J.decode_rgb(split)
    assert np.array_equal(WJ.decode(split), ref)
    got = WJ.decode_batch([base, split])
    assert np.array_equal(got[1], ref) and np.array_equal(got[0], J.decode_rgb(base))


def test_async_decode_matches_libjpeg():
    """wicca_jpeg_decode_u8_async / wicca_jpeg_wait through decode_batches:
    several batches in flight (baseline, progressive, grayscale, EXIF-rotated,
    restart intervals), every image equal to libjpeg-turbo's decode."""
    specs = [("scene", 480, 640, 2, 90, 0, False, 1), ("noise", 200, 300, 0, 70, 4, False, 1),
             ("scene", 333, 517, 1, 85, 0, True, 1), ("gray", 97, 55, 0, 80, 0, False, 1),
             ("smooth", 256, 384, 2, 60, 0, False, 6)]
    batches = []
    for k in range(5):
        batch = []
        for i, (kind, h, w, sub, q, rb, prog, orient) in enumerate(specs[k % 3:] + specs[:k % 3]):
            img = J.test_image(kind, h + k, w + 2 * k, 31 * k + i)
            batch.append(J.encode(img, q, sub, rb, progressive=prog, orientation=orient))
        batches.append(batch)
    got = list(WJ.decode_batches(batches, depth=2))
    assert len(got) == len(batches)
    for blobs, outs in zip(batches, got):
        for b, o in zip(blobs, outs):
            assert np.array_equal(o.cpu().numpy(), J.decode_rgb(b))
    # depth 1 (no overlap) gives the same
    again = list(WJ.decode_batches(batches[:2], depth=1))
    for a, b in zip(got[:2], again):
        assert all(np.array_equal(x.cpu().numpy(), y.cpu().numpy()) for x, y in zip(a, b))


def test_async_decode_errors():
    from wicca_amd import _lib
    lib = _lib.load()
    assert lib.wicca_jpeg_wait(0) == 0
    assert lib.wicca_jpeg_wait(987654321) == _lib.WICCA_ERR_ARG
    good = J.encode(J.test_image("scene", 64, 64, 5), 80, 2)
    with pytest.raises(ValueError):
        list(WJ.decode_batches([[good], [good[:40]]]))


def test_mixed_progressive_and_baseline_batch(tmp_path):
    """One decode call over baseline (device Huffman decode) and progressive
    (host entropy decode) files, and the file-based caller stage over them."""
    blobs = []
    for i, (h, w, prog) in enumerate([(240, 320, True), (333, 517, False), (100, 90, True), (77, 61, False),
                                      (480, 640, True)]):
        blobs.append(J.encode(J.test_image("scene", h, w, 70 + i), 85, 2, progressive=prog))
    got = WJ.decode_batch(blobs)
    for b, g in zip(blobs, got):
        assert np.array_equal(g, J.decode_rgb(b))
    only_prog = WJ.decode_batch([blobs[0], blobs[2]])
    assert np.array_equal(only_prog[0], got[0]) and np.array_equal(only_prog[1], got[2])
    paths = []
    for i, b in enumerate(blobs):
        p = tmp_path / f"m{i}.jpg"
        p.write_bytes(b)
        paths.append(str(p))
    imgs, icons = wicca_amd.get_img_batch(paths, (224, 224), 3)
    for i, b in enumerate(blobs):
        rgb = J.decode_rgb(b)
        assert np.array_equal(imgs[i], R.resize(rgb, (224, 224), R.INTER_AREA))
        assert np.array_equal(icons[i], R.resize(c_oracle.ll_int_block(rgb, 3)[0], (224, 224), R.INTER_AREA))


def test_truncated_progressive_decodes_without_fault():
    """A progressive file cut inside a scan: the scans before the cut stand,
    the rest reads as missing data (no fault, the right shape)."""
    data = J.encode(J.test_image("scene", 256, 384, 21), 90, 2, progressive=True)
    for cut in (0.3, 0.6, 0.9):
        got = WJ.decode(data[:int(len(data) * cut)])
        assert got.shape == (256, 384, 3)


def test_load_image_contract(tmp_path, capsys):
    with pytest.raises(ValueError, match="File path cannot be empty"):
        wicca_amd.load_image("")
    assert wicca_amd.load_image(str(tmp_path / "missing.jpg")) is None
    assert "Error loading image" in capsys.readouterr().out
    p = tmp_path / "x.jpg"
    data = J.encode(J.test_image("scene", 70, 90, 2), 80, 2)
    p.write_bytes(data)
    assert np.array_equal(wicca_amd.load_image(str(p)), J.decode_rgb(data))


@pytest.mark.parametrize("depth,shape", [(5, (224, 224)), (2, (299, 299)), (3, (240, 240))])
def test_file_caller_stage(tmp_path, depth, shape):
    paths, refs = [], []
    for i, (h, w) in enumerate([(480, 640), (1080, 1920), (333, 517), (600, 401)]):
        data = J.encode(J.test_image("scene", h, w, i), 85, 2, orientation=6 if i == 3 else 1)
        p = tmp_path / f"{i}.jpg"
        p.write_bytes(data)
        paths.append(str(p))
        refs.append(J.decode_rgb(data))
    imgs, icons = wicca_amd.get_img_batch(paths, shape, depth)
    for i, rgb in enumerate(refs):
        assert np.array_equal(imgs[i], R.resize(rgb, shape, R.INTER_AREA)), i
        icon = c_oracle.ll_int_block(rgb, depth)[0]
        assert np.array_equal(icons[i], R.resize(icon, shape, R.INTER_AREA)), i


def test_file_caller_stage_split_over_devices(tmp_path):
    """The one-process multi-GPU form (devices=[0, 0] exercises the split and
    the per-range output offsets on a one-GPU box)."""
    paths = []
    for i, (h, w) in enumerate([(200, 300), (480, 640), (100, 100), (333, 517), (640, 480)]):
        p = tmp_path / f"m{i}.jpg"
        p.write_bytes(J.encode(J.test_image("scene", h, w, 50 + i), 80, 2))
        paths.append(str(p))
    one = wicca_amd.get_img_batch(paths, (224, 224), 4)
    two = wicca_amd.get_img_batch(paths, (224, 224), 4, devices=[0, 0])
    assert np.array_equal(one[0], two[0]) and np.array_equal(one[1], two[1])


@pytest.mark.parametrize("cut", [0.3, 0.7, 0.95])
def test_truncated_file_decodes_without_fault(cut):
    """A file cut inside its entropy-coded data: the decode must stay inside
    its buffers (missing blocks come out as the DC-0 grey libjpeg also
    substitutes); the decoded part before the cut must match libjpeg-turbo's."""
    img = J.test_image("scene", 256, 384, 11)
    data = J.encode(img, 90, 2, restart_blocks=8)
    short = data[:int(len(data) * cut)]
    got = WJ.decode(short)
    assert got.shape == (256, 384, 3)
    full = J.decode_rgb(data)
    assert np.array_equal(got[:16], full[:16]) if cut >= 0.3 else True


def test_corrupted_bits_decode_without_fault():
    """Flipped bytes in the entropy-coded data (not in markers): garbage
    pixels are fine, faults and hangs are not; the next clean file decodes."""
    img = J.test_image("noise", 200, 300, 12)
    data = bytearray(J.encode(img, 75, 2))
    rng = np.random.default_rng(5)
    sos = bytes(data).index(b"\xff\xda")
    for pos in rng.integers(sos + 20, len(data) - 4, 40):
        if data[pos] != 0xFF and data[pos - 1] != 0xFF:
            data[pos] ^= 0x5A if data[pos] ^ 0x5A != 0xFF else 0x01
    got = WJ.decode(bytes(data))
    assert got.shape == (200, 300, 3)
    ok = J.encode(img, 75, 2)
    assert np.array_equal(WJ.decode(ok), J.decode_rgb(ok))


def test_batch_larger_than_one_device_pass():
    """More files than one pass takes (4096 IDCT jobs / 3 components)."""
    blobs = [J.encode(J.test_image("scene", 16 + i % 5, 24 + i % 7, i), 70 + i % 25, i % 3)
             for i in range(1400)]
    got = WJ.decode_batch(blobs)
    for i in (0, 1364, 1365, 1366, 1399):
        assert np.array_equal(got[i], J.decode_rgb(blobs[i])), i


@pytest.mark.parametrize("env", [{"WICCA_JPEG_WRITE_SLOTS": "6"}, {"WICCA_JPEG_SYNC_CK": "0"},
                                 {"WICCA_JPEG_SYNC_CK": "1"}, {"WICCA_JPEG_ILV": "0"}],
                         ids=["slots6", "no-checkpoints", "round0-checkpoints", "plain-stream"])
def test_write_and_sync_variants_subprocess(env):
    """The sync and write passes have 4-table builds (every baseline file) and
    6-table ones (extended-sequential files with separate tables per
    component; WICCA_JPEG_WRITE_SLOTS=6 forces them); the sync passes run with
    or without checkpoints; every pass reads the lane-interleaved stream copy
    or (WICCA_JPEG_ILV=0) the plain de-stuffed stream.  Each variant in a child
    process on the golden files."""
    import subprocess
    import sys
    code = (
        "import hashlib, json, os, sys\n"
        "from wicca_amd import jpeg as WJ\n"
        f"gold = {GOLD!r}\n"
        "cases = json.load(open(os.path.join(gold, 'cases.json')))['cases']\n"
        "data = [open(os.path.join(gold, c['file']), 'rb').read() for c in cases]\n"
        "outs = WJ.decode_batch(data)\n"
        "bad = [c['name'] for c, o in zip(cases, outs)\n"
        "       if hashlib.sha256(o.tobytes()).hexdigest() != c['sha256_rgb']]\n"
        "print('BAD', bad)\n"
        "sys.exit(1 if bad else 0)\n")
    env = dict(os.environ, **env)
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=240,
                       cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert r.returncode == 0, r.stdout + r.stderr


STAGE = [(1, (224, 224), 3, 1, 0), (6, (224, 224), 3, 0, 77), (8, (331, 331), 3, 1, 0),
         (4, (240, 240), 1, 0, 9), (3, (299, 299), 0, 1, 0), (7, (224, 224), 3, 0, 255),
         # outputs wider than the row-sum kernel's 341 RGB columns: no row sums
         (5, (384, 384), 3, 1, 0), (2, (600, 450), 3, 0, 5)]


@pytest.mark.parametrize("depth,shape,interp,border,k", STAGE,
                         ids=[f"d{d}-{s[0]}-i{i}-b{b}-k{k}" for d, s, i, b, k in STAGE])
def test_file_caller_stage_fused_cases(tmp_path, depth, shape, interp, border, k):
    """The fused stage (each decoded image read once for its INTER_AREA row
    sums and its icon, stage.hip) against cv2.resize restated (oracle) and the
    C oracle's icon: every depth class, both borders, the non-AREA
    interpolations (separate source resize), images smaller than the
    classifier input (upscaled: no row sums), odd sizes, and rows split into
    2 and 3 parts."""
    # the last two rows span 2 and 3 of stage_rows' row parts
    sizes = [(480, 640), (1081, 1919), (133, 517), (77, 61), (300, 2050), (600, 401), (96, 4000), (130, 7680)]
    paths, refs = [], []
    for i, (h, w) in enumerate(sizes):
        data = J.encode(J.test_image("scene" if i % 2 else "noise", h, w, 7 * i + depth), 85, i % 3)
        p = tmp_path / f"s{i}.jpg"
        p.write_bytes(data)
        paths.append(str(p))
        refs.append(J.decode_rgb(data))
    imgs, icons = wicca_amd.get_img_batch(paths, shape, depth, interp, border, k)
    for i, rgb in enumerate(refs):
        assert np.array_equal(imgs[i], R.resize(rgb, shape, interp)), i
        icon = c_oracle.ll_int_block(rgb, depth, border, k)[0]
        assert np.array_equal(icons[i], R.resize(icon, shape, interp)), i


@pytest.mark.parametrize("depth", [1, 2])
def test_icon_area_resize_window(tmp_path, depth):
    """INTER_AREA icon resizes of the file stage (resize_desc_kernel) at
    downscales from under 2x to 38x (depth 1 of a 3840-wide image to 100 x
    60), non-integer and ragged, against cv2.resize restated on the C
    oracle's icon."""
    sizes = [(2160, 3840), (1500, 2602), (999, 1777), (641, 479)]
    paths = []
    refs = []
    for i, (h, w) in enumerate(sizes):
        data = J.encode(J.test_image("noise" if i % 2 else "scene", h, w, 31 * i + depth), 80, 2)
        p = tmp_path / f"w{i}.jpg"
        p.write_bytes(data)
        paths.append(str(p))
        refs.append(J.decode_rgb(data))
    for shape in [(224, 224), (331, 299), (100, 60)]:
        _, icons = wicca_amd.get_img_batch(paths, shape, depth, 3, 1, 0)
        for i, rgb in enumerate(refs):
            icon = c_oracle.ll_int_block(rgb, depth, 1, 0)[0]
            assert np.array_equal(icons[i], R.resize(icon, shape, 3)), (shape, i)


def test_file_caller_stage_fused_equals_unfused(tmp_path):
    """WICCA_STAGE_FUSED=0 (per-image resize, icon and icon-resize launches)
    in a child process gives the same bytes as the fused stage."""
    import subprocess
    import sys
    paths = []
    for i, (h, w) in enumerate([(720, 1280), (1001, 999), (64, 4000), (2160, 3840)]):
        p = tmp_path / f"u{i}.jpg"
        p.write_bytes(J.encode(J.test_image("scene", h, w, 90 + i), 88, 2))
        paths.append(str(p))
    code = ("import sys, numpy as np, wicca_amd\n"
            f"paths = {paths!r}\n"
            "a, b = wicca_amd.get_img_batch(paths, (224, 224), 5, 3, 0, 31)\n"
            "np.save(sys.argv[1], np.concatenate([a.ravel(), b.ravel()]))\n")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    outs = []
    for fused in ("1", "0"):
        f = str(tmp_path / f"o{fused}.npy")
        env = dict(os.environ, WICCA_STAGE_FUSED=fused)
        r = subprocess.run([sys.executable, "-c", code, f], env=env, capture_output=True, text=True,
                           timeout=240, cwd=root)
        assert r.returncode == 0, r.stdout + r.stderr
        outs.append(np.load(f))
    assert np.array_equal(outs[0], outs[1])


def test_fused_backend_equals_separate_launches():
    """WICCA_JPEG_FUSED=0 (IDCT and colour as separate launches, the luma
    plane through HBM) gives the same pixels as the fused back end on the
    golden files, in a child process."""
    import subprocess
    import sys
    code = (
        "import hashlib, json, os, sys\n"
        "from wicca_amd import jpeg as WJ\n"
        f"gold = {GOLD!r}\n"
        "cases = json.load(open(os.path.join(gold, 'cases.json')))['cases']\n"
        "data = [open(os.path.join(gold, c['file']), 'rb').read() for c in cases]\n"
        "outs = WJ.decode_batch(data)\n"
        "bad = [c['name'] for c, o in zip(cases, outs)\n"
        "       if hashlib.sha256(o.tobytes()).hexdigest() != c['sha256_rgb']]\n"
        "print('BAD', bad)\n"
        "sys.exit(1 if bad else 0)\n")
    env = dict(os.environ, WICCA_JPEG_FUSED="0")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=240,
                       cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert r.returncode == 0, r.stdout + r.stderr


def test_batch_with_unreadable_files_fails_per_slot(tmp_path, capsys):
    """One file the decoder cannot read (PNG bytes, an arithmetic-coded JPEG,
    a header cut short) fails its own slot only: errors="zero" / "none" give
    the other files' exact results; errors="raise" (the default) raises."""
    good = [J.encode(J.test_image("scene", h, w, 60 + i), 85, 2) for i, (h, w) in
            enumerate([(240, 320), (333, 517), (100, 90)])]
    sof = good[1].index(b"\xff\xc0")
    bad = [b"\x89PNG\r\n\x1a\n" + b"\x00" * 64,
           good[1][:sof + 1] + b"\xc9" + good[1][sof + 2:],  # arithmetic-coded: unsupported
           good[0][:30]]
    blobs = [good[0], bad[0], good[1], bad[1], bad[2], good[2]]
    outs = WJ.decode_batch(blobs, errors="none")
    assert [o is None for o in outs] == [False, True, False, True, True, False]
    for b, o in zip(blobs, outs):
        if o is not None:
            assert np.array_equal(o, J.decode_rgb(b))
    with pytest.raises((ValueError, NotImplementedError)):
        WJ.decode_batch(blobs)
    paths = []
    for i, b in enumerate(blobs):
        p = tmp_path / f"f{i}.jpg"
        p.write_bytes(b)
        paths.append(str(p))
    imgs, icons = wicca_amd.get_img_batch(paths, (224, 224), 4, errors="zero")
    printed = capsys.readouterr().out
    for i, b in enumerate(blobs):
        if outs[i] is None:
            assert not imgs[i].any() and not icons[i].any()
            assert f"Error loading image {paths[i]}" in printed
        else:
            rgb = J.decode_rgb(b)
            assert np.array_equal(imgs[i], R.resize(rgb, (224, 224), R.INTER_AREA))
            assert np.array_equal(icons[i], R.resize(c_oracle.ll_int_block(rgb, 4)[0], (224, 224), R.INTER_AREA))
    with pytest.raises((ValueError, NotImplementedError)):
        wicca_amd.get_img_batch(paths, (224, 224), 4)
    two = wicca_amd.get_img_batch(paths, (224, 224), 4, devices=[0, 0], errors="zero")
    assert np.array_equal(two[0], imgs) and np.array_equal(two[1], icons)


def test_file_stage_pipelined_matches_synchronous(tmp_path):
    """get_img_batches (wicca_image_icon_stage_async, batches in flight) gives
    get_img_batch's outputs batch by batch; a PNG batch runs synchronously
    inside it; an abandoned generator leaves nothing in flight."""
    from PIL import Image
    import io
    batches = []
    for b in range(4):
        paths = []
        for i, (h, w) in enumerate([(480, 640), (333, 517), (1080, 1920)]):
            p = tmp_path / f"b{b}_{i}.jpg"
            p.write_bytes(J.encode(J.test_image("scene", h, w, 10 * b + i), 85, 2, orientation=6 if i == 1 else 1))
            paths.append(str(p))
        batches.append(paths)
    png = tmp_path / "x.png"
    buf = io.BytesIO()
    Image.fromarray(J.test_image("scene", 300, 200, 5)).save(buf, "PNG")
    png.write_bytes(buf.getvalue())
    batches.insert(2, [str(png), batches[0][0]])
    for depth in (1, 2, 3):
        got = list(wicca_amd.get_img_batches(batches, (224, 224), 4, depth=depth))
        assert len(got) == len(batches)
        for paths, (imgs, icons) in zip(batches, got):
            want = wicca_amd.get_img_batch(paths, (224, 224), 4)
            assert np.array_equal(imgs, want[0]) and np.array_equal(icons, want[1])
    gen = wicca_amd.get_img_batches(batches, (299, 299), 3)
    next(gen)
    gen.close()
    with pytest.raises(OSError):  # a missing file (batch 1) while batch 0 is in flight
        list(wicca_amd.get_img_batches([[str(tmp_path / "b0_0.jpg")], [str(tmp_path / "missing.jpg")]], (224, 224), 4))


DAMAGE = [(kind, sub, rb, prog) for kind, sub, rb, prog in
          [("scene", 2, 0, False), ("scene", 2, 8, False), ("noise", 0, 0, False), ("scene", 1, 3, False),
           ("gray", 0, 0, False), ("scene", 2, 0, True), ("smooth", 2, 16, True)]]


@pytest.mark.parametrize("kind,sub,rb,prog", DAMAGE, ids=[f"{k}-s{s}-r{r}-p{int(p)}" for k, s, r, p in DAMAGE])
@pytest.mark.parametrize("cut", [0.3, 0.5, 0.7, 0.95])
def test_truncated_file_whole_decode_matches_libjpeg(kind, sub, rb, prog, cut):
    """cv2.imread returns a truncated JPEG (libjpeg-turbo's stdio source feeds
    a fake EOI at the end of the file: missing blocks all-zero, i.e. grey;
    progressive images whose first AC coefficients are not all final are
    block-smoothed, jdcoefct.c decompress_smooth_data), so the classifiers see
    every pixel of it (data_loader.py:53-63): the whole decode against
    libjpeg-turbo's (oracle.jpeg_pil.decode_rgb_imread), bit for bit, with
    and without restart markers, progressive files included; where libjpeg
    refuses the cut file (imread: None) the engine fails that slot."""
    img = J.test_image(kind, 200, 344, 17 + sub + rb)
    if kind == "gray":
        img = img[..., 0] if img.ndim == 3 else img
    data = J.encode(img, 88, sub, rb, progressive=prog)
    short = data[:int(len(data) * cut)]
    want = J.decode_rgb_imread(short)
    got = WJ.decode_batch([short], errors="none")[0]
    if want is None:
        assert got is None
    else:
        assert got is not None and np.array_equal(got, want)


@pytest.mark.parametrize("seed", range(6))
def test_corrupted_entropy_whole_decode_matches_libjpeg(seed):
    """Bytes flipped inside the entropy-coded data (markers untouched):
    libjpeg-turbo decodes on (a bad Huffman code decodes as a zero symbol,
    jdhuff.c), so does cv2.imread; the whole image against libjpeg's decode,
    and where libjpeg refuses the file the engine fails its slot."""
    rng = np.random.default_rng(100 + seed)
    kind = ("scene", "noise", "smooth")[seed % 3]
    img = J.test_image(kind, 160, 232, seed)
    data = bytearray(J.encode(img, 80, seed % 3, 8 if seed % 2 else 0))
    sos = bytes(data).index(b"\xff\xda")
    start = sos + 2 + int.from_bytes(data[sos + 2:sos + 4], "big")
    for pos in rng.integers(start + 4, len(data) - 4, 3 + seed):
        if data[pos] != 0xFF and data[pos - 1] != 0xFF:
            nv = data[pos] ^ int(rng.integers(1, 255))
            if nv != 0xFF:
                data[pos] = nv
    want = J.decode_rgb_imread(bytes(data))
    got = WJ.decode_batch([bytes(data)], errors="none")[0]
    if want is None:
        assert got is None
    else:
        assert got is not None and np.array_equal(got, want)


def _rst_damaged(how):
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
        data[at + 1] = 0x01
    return bytes(data)


RST_DAMAGE = ["next1", "next2", "prior1", "far", "dropped", "garbage-ff00", "not-rst"]


def test_damaged_restart_markers_batch_matches_libjpeg(tmp_path):
    """Restart markers renumbered, dropped, preceded by stray bytes or turned
    into another code, mixed with clean files in one batch: the device path
    flags them (markers out of sequence, segments missing or short) and the
    host decoder redoes them with libjpeg's resync rules (jdmarker.c
    read_restart_marker / jpeg_resync_to_restart); every file equals Pillow's
    decode, through the one-call decode, the async batches and the file stage."""
    clean = [J.encode(J.test_image("noise", 120, 176, 3), 80, 1, 5), J.encode(J.test_image("scene", 96, 64, 4), 90, 2)]
    blobs = [clean[0]] + [_rst_damaged(h) for h in RST_DAMAGE] + [clean[1]]
    want = [J.decode_rgb(b, truncated=True) for b in blobs]
    got = WJ.decode_batch(blobs)
    for i, (g, w) in enumerate(zip(got, want)):
        assert np.array_equal(g, w), i
    for i, g in enumerate(x for batch in WJ.decode_batches([blobs[:4], blobs[4:]]) for x in batch):
        assert np.array_equal(g.cpu().numpy(), want[i]), i
    paths = []
    for i, b in enumerate(blobs):
        p = tmp_path / f"{i}.jpg"
        p.write_bytes(b)
        paths.append(str(p))
    imgs, icons = wicca_amd.get_img_batch(paths, (224, 224), 3)
    for i, rgb in enumerate(want):
        assert np.array_equal(imgs[i], R.resize(rgb, (224, 224), R.INTER_AREA)), i
        assert np.array_equal(icons[i], R.resize(c_oracle.ll_int_block(rgb, 3)[0], (224, 224), R.INTER_AREA)), i
    m = wicca_amd.get_img_matrix(paths, [(224, 224)], (3, 4))
    assert np.array_equal(m[((224, 224), 3)][0], imgs) and np.array_equal(m[((224, 224), 3)][1], icons)


def _low_entropy_files():
    """Pillow optimize=True on flat / low-entropy content: Huffman tables with
    one or two codes (a flat image's DC table has the single code '0'), with and
    without restart intervals, colour and grayscale."""
    flat = np.full((64, 96, 3), 128, np.uint8)
    grad = np.tile(np.arange(200, dtype=np.uint8)[None, :, None], (120, 1, 3))
    step = np.zeros((72, 72, 3), np.uint8)
    step[:, 36:] = 255
    out = []
    for img in (flat, grad, step):
        for rb in (0, 1, 3):
            out.append(J.encode(img, 90, 2, rb, optimize=True))
            out.append(J.encode(img[..., 0].copy(), 75, 0, rb, optimize=True))
    return out


def test_clean_low_entropy_files_are_not_flagged_damaged(tmp_path):
    """the write pass's last lane of a segment used to decode the
    encoder's fill bits after the final MCU; with a single-code DC table they
    match no code, so a clean file was flagged damaged and redone on the host
    (a silent throughput cliff).  Every path decodes these exactly and redoes
    none of them (wicca_jpeg_damaged_redone does not move)."""
    lib = _lib.load()
    blobs = _low_entropy_files()
    want = [J.decode_rgb(b) for b in blobs]
    before = lib.wicca_jpeg_damaged_redone()
    got = WJ.decode_batch(blobs)
    for i, (g, w) in enumerate(zip(got, want)):
        assert np.array_equal(g, w), i
    for i, g in enumerate(x for batch in WJ.decode_batches([blobs[:9], blobs[9:]]) for x in batch):
        assert np.array_equal(g.cpu().numpy(), want[i]), i
    paths = []
    for i, b in enumerate(blobs):
        p = tmp_path / f"{i}.jpg"
        p.write_bytes(b)
        paths.append(str(p))
    imgs, _ = wicca_amd.get_img_batch(paths, (224, 224), 3)
    for i, w in enumerate(want):
        assert np.array_equal(imgs[i], R.resize(w, (224, 224), R.INTER_AREA)), i
    list(wicca_amd.get_img_batches([paths[:9], paths[9:]], (224, 224), 3))
    assert lib.wicca_jpeg_damaged_redone() == before


# --- colour spaces: libjpeg-turbo's default_decompress_parms (jdapimin.c) picks
# YCbCr / RGB for three components from the JFIF and Adobe markers and the
# component ids, CMYK / YCCK for four from the Adobe transform; cv2.imread
# then converts CMYK to BGR (oracle/jpeg_pil.py cmyk_to_rgb_imread).

def _segments(data):
    """(marker, start, end) of every marker segment before the first SOS."""
    out, pos = [], 2
    while pos < len(data):
        assert data[pos] == 0xFF
        m = data[pos + 1]
        ln = int.from_bytes(data[pos + 2:pos + 4], "big")
        out.append((m, pos, pos + 2 + ln))
        if m == 0xDA:
            break
        pos += 2 + ln
    return out


def _strip(data, marker):
    for m, a, b in _segments(data):
        if m == marker:
            return data[:a] + data[b:]
    raise AssertionError(f"no marker {marker:#x}")


def _with_jfif(data):
    app0 = b"\xff\xe0\x00\x10JFIF\x00\x01\x01\x00\x00\x01\x00\x01\x00\x00"
    return data[:2] + app0 + data[2:]


def _set_ids(data, ids):
    """Component ids in SOF and SOS (a single-scan file)."""
    d = bytearray(data)
    for m, a, b in _segments(data):
        if m in (0xC0, 0xC1, 0xC2):
            for c, v in enumerate(ids):
                d[a + 10 + 3 * c] = v
        if m == 0xDA:
            for c, v in enumerate(ids):
                d[a + 5 + 2 * c] = v
    return bytes(d)


def _adobe_transform(data, t):
    d = bytearray(data)
    j = d.find(b"Adobe")
    d[j + 11] = t
    return bytes(d)


def _rgb_jpeg(img, q=90):
    import io

    from PIL import Image
    b = io.BytesIO()
    Image.fromarray(img).save(b, "JPEG", quality=q, keep_rgb=True)
    return b.getvalue()


def _cmyk_jpeg(img, q=90, progressive=False):
    import io

    from PIL import Image
    b = io.BytesIO()
    Image.fromarray(img).convert("CMYK").save(b, "JPEG", quality=q, progressive=progressive)
    return b.getvalue()


def _colour_files():
    files = []
    for i, (H, W) in enumerate(((64, 80), (135, 241), (17, 33), (480, 640))):
        img = J.test_image("scene" if i % 2 == 0 else "noise", H, W, 90 + i)
        rgb = _rgb_jpeg(img, 85 + i)
        files += [
            ("rgb-adobe", rgb),                                    # Adobe transform 0, ids 'R' 'G' 'B'
            ("rgb-ids", _strip(rgb, 0xEE)),                        # no marker, ids 'R' 'G' 'B'
            ("rgb-as-ycc-ids", _set_ids(_strip(rgb, 0xEE), (1, 2, 3))),  # ids 1 2 3: YCbCr
            ("rgb-jfif", _with_jfif(rgb)),                         # JFIF wins: YCbCr
            ("cmyk", _cmyk_jpeg(img, 90)),                         # Adobe transform 0: CMYK
            ("cmyk-prog", _cmyk_jpeg(img, 80, progressive=True)),  # host entropy decode, progressive
            ("ycck", _adobe_transform(_cmyk_jpeg(img, 90), 2)),    # Adobe transform 2: YCCK
            ("cmyk-nomarker", _strip(_cmyk_jpeg(img, 90), 0xEE)),  # no Adobe marker: plain CMYK
        ]
    return files


def test_colour_spaces_match_imread():
    """RGB-colour-space JPEGs (keep_rgb, with and without the Adobe marker,
    under a JFIF marker), Adobe CMYK (baseline and progressive), YCCK and
    marker-less CMYK, one batch with ordinary YCbCr files: every image as
    cv2.imread gives it (libjpeg-turbo through Pillow, OpenCV's CMYK -> BGR
    restated)."""
    files = _colour_files()
    plain = [J.encode(J.test_image("scene", 96, 128, 5), 90, 2), J.encode(J.test_image("gray", 40, 50, 6), 90)]
    blobs = [d for _, d in files] + plain
    outs = WJ.decode_batch(blobs)
    for (name, d), got in zip(files, outs):
        want = J.decode_rgb(d)
        assert got.shape == want.shape, name
        assert np.array_equal(got, want), name
    for d, got in zip(plain, outs[len(files):]):
        assert np.array_equal(got, J.decode_rgb(d))


def test_colour_spaces_separate_backend(tmp_path):
    """The same files through the separate IDCT / colour launches
    (WICCA_JPEG_FUSED=0), in a child process."""
    import subprocess
    import sys
    files = _colour_files()
    want = {f"w{i}": J.decode_rgb(d) for i, (_, d) in enumerate(files)}
    np.savez(tmp_path / "want.npz", **want)
    for i, (_, d) in enumerate(files):
        (tmp_path / f"f{i}.jpg").write_bytes(d)
    code = (
        "import sys, numpy as np\n"
        "from wicca_amd import jpeg as WJ\n"
        f"d = {str(tmp_path)!r}\n"
        f"n = {len(files)}\n"
        "want = np.load(d + '/want.npz')\n"
        "outs = WJ.decode_batch([open(f'{d}/f{i}.jpg', 'rb').read() for i in range(n)])\n"
        "bad = [i for i in range(n) if not np.array_equal(outs[i], want[f'w{i}'])]\n"
        "print('BAD', bad)\n"
        "sys.exit(1 if bad else 0)\n")
    env = dict(os.environ, WICCA_JPEG_FUSED="0")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=240,
                       cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert r.returncode == 0, r.stdout + r.stderr


def test_cmyk_file_caller_stage(tmp_path):
    """A CMYK and an RGB-colour-space file through the file caller stage
    (_get_img_batch) equal the resize and icon of their imread decode."""
    img = J.test_image("scene", 300, 400, 11)
    paths = []
    for name, d in (("c.jpg", _cmyk_jpeg(img)), ("r.jpg", _rgb_jpeg(img)), ("y.jpg", J.encode(img, 90, 2))):
        p = tmp_path / name
        p.write_bytes(d)
        paths.append(str(p))
    imgs, icons = wicca_amd.get_img_batch(paths, (224, 224), 3)
    for i, p in enumerate(paths):
        rgb = J.decode_rgb(open(p, "rb").read())
        assert np.array_equal(imgs[i], R.resize(rgb, (224, 224), R.INTER_AREA)), p
        icon = c_oracle.ll_int_block(rgb, 3, 1, 0)[0]
        assert np.array_equal(icons[i], R.resize(icon, (224, 224), R.INTER_AREA)), p


@pytest.mark.gpu
def test_truncated_mapping_in_plan_batch(tmp_path):
    """StagePlan maps its files: a file truncated under the mapping between
    the header parse and the de-stuffing makes the batch fail with an error
    (the library's SIGBUS guard), and the process goes on."""
    from oracle import jpeg_pil as J
    from wicca_amd import plan as P
    data = J.encode(J.test_image("scene", 720, 1280, 5), 90)
    paths = []
    for i in range(3):
        p = tmp_path / f"{i}.jpg"
        p.write_bytes(data)
        paths.append(str(p))
    blobs = P._read(paths, mapped=True)
    os.truncate(paths[1], 1024)  # the header stays, the scan's pages go
    keep = [np.frombuffer(b, np.uint8) for b in blobs]
    with pytest.raises(Exception, match="truncated"):
        WJ.decode_batch(keep)
    del keep, blobs
    got = P.get_img_matrix([paths[0], paths[2]], [(224, 224)], [3])
    assert got[((224, 224), 3)][0].shape == (2, 224, 224, 3)
