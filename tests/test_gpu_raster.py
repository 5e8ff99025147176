"""GPU PNG / BMP decode (load_image's cv2.imread for the .png / .bmp inputs
ClassifierProcessor counts, classifying_tools.py:162; data_loader.py:53-58)
against the restatement in oracle/raster_ref.py (itself pinned to Pillow
12.2.0 in tests/test_raster_oracle.py) and, at sizes the pure-Python
restatement is slow for, against Pillow directly; mixed-format batches; the
file-based caller stage; corrupt files failing their own slot."""
import hashlib
import io
import json
import os
import struct
import zlib

import numpy as np
import pytest

import wicca_amd
from oracle import c_oracle
from oracle import jpeg_pil as J
from oracle import raster_ref as rr
from oracle import resize_cv as R
from wicca_amd import jpeg as WJ

pytestmark = pytest.mark.gpu

from test_raster_oracle import PNG_CASES, png_samples  # noqa: E402


@pytest.mark.parametrize("interlace", [False, True])
@pytest.mark.parametrize("ct,bits", PNG_CASES)
def test_png_types_vs_oracle(ct, bits, interlace):
    blobs = []
    for i, (h, w) in enumerate([(1, 1), (3, 5), (37, 29), (64, 131)]):
        s, pal = png_samples(ct, bits, h, w, seed=ct * 1000 + bits * 10 + i)
        blobs.append(rr.encode_png(s, ct, bits, interlace=interlace, palette=pal))
    outs = WJ.decode_batch(blobs)
    for b, o in zip(blobs, outs):
        assert np.array_equal(o, rr.decode_png(b))
    assert WJ.image_info(blobs[2])[:3] == (37, 29, "png")


@pytest.mark.parametrize("f", range(5))
@pytest.mark.parametrize("ct,bits", [(2, 8), (6, 16), (0, 4), (3, 8)])
def test_png_each_filter(ct, bits, f):
    s, pal = png_samples(ct, bits, 23, 41, seed=f)
    data = rr.encode_png(s, ct, bits, palette=pal, filters=f)
    assert np.array_equal(WJ.decode(data), rr.decode_png(data))


def test_png_split_idat_and_ancillary_chunks():
    s, _ = png_samples(2, 8, 50, 70, seed=9)
    anc = [(b"gAMA", struct.pack(">I", 45455)), (b"tEXt", b"Comment\x00hello"), (b"sRGB", b"\x00")]
    data = rr.encode_png(s, 2, 8, idat_split=97, extra_chunks=anc)
    assert np.array_equal(WJ.decode(data), rr.pillow_rgb(data))
    # an ancillary chunk with a bad CRC is ignored (libpng: a warning)
    k = data.index(b"tEXt")
    bad = data[:k + 4] + b"X" + data[k + 5:]
    assert np.array_equal(WJ.decode(bad), rr.pillow_rgb(data))


@pytest.mark.parametrize("mode", ["RGB", "RGBA", "L", "LA", "P", "1"])
@pytest.mark.parametrize("H,W", [(480, 640), (1080, 1920)])
def test_pillow_written_png(mode, H, W):
    from PIL import Image
    img = J.test_image("scene", H, W, H + len(mode))
    b = io.BytesIO()
    Image.fromarray(img).convert(mode).save(b, "PNG", compress_level=1)
    data = b.getvalue()
    assert np.array_equal(WJ.decode(data), rr.pillow_rgb(data))


def test_png_8k_rgb_vs_pillow():
    from PIL import Image
    img = J.test_image("scene", 4320, 7680, 11)
    b = io.BytesIO()
    Image.fromarray(img).save(b, "PNG", compress_level=1)
    assert np.array_equal(WJ.decode(b.getvalue()), img)


@pytest.mark.parametrize("bpp", [1, 4, 8, 24, 32])
@pytest.mark.parametrize("top_down", [False, True])
def test_bmp_vs_oracle(bpp, top_down):
    rng = np.random.default_rng(bpp + 10 * top_down)
    blobs = []
    for (h, w) in [(1, 1), (7, 3), (19, 23), (100, 257)]:
        if bpp <= 8:
            idx = rng.integers(0, 1 << bpp, (h, w), dtype=np.uint8)
            pal = rng.integers(0, 256, (1 << bpp, 3), dtype=np.uint8)
            blobs.append(rr.encode_bmp(idx, bpp, palette=pal, top_down=top_down))
        else:
            blobs.append(rr.encode_bmp(rng.integers(0, 256, (h, w, 3), dtype=np.uint8), bpp, top_down=top_down))
    for b, o in zip(blobs, WJ.decode_batch(blobs)):
        assert np.array_equal(o, rr.decode_bmp(b))
        assert np.array_equal(o, rr.pillow_rgb(b))


@pytest.mark.parametrize("fields565", [None, False, True])
def test_bmp16(fields565):
    img = np.random.default_rng(3).integers(0, 256, (31, 45, 3), dtype=np.uint8)
    data = rr.encode_bmp(img, 16, fields565=fields565)
    assert np.array_equal(WJ.decode(data), rr.decode_bmp(data))  # OpenCV's shifts (unpinned)


def test_bmp_core_header_and_pillow_written():
    from PIL import Image
    rng = np.random.default_rng(8)
    idx = rng.integers(0, 256, (33, 47), dtype=np.uint8)
    pal = rng.integers(0, 256, (256, 3), dtype=np.uint8)
    data = rr.encode_bmp(idx, 8, palette=pal, core_header=True)
    assert np.array_equal(WJ.decode(data), pal[idx])
    img = J.test_image("scene", 300, 401, 4)
    for mode in ["RGB", "L", "P", "1"]:
        b = io.BytesIO()
        Image.fromarray(img).convert(mode).save(b, "BMP")
        assert np.array_equal(WJ.decode(b.getvalue()), rr.pillow_rgb(b.getvalue())), mode


def _mixed_files(tmp_path):
    from PIL import Image
    paths, refs = [], []
    specs = [("jpg", 480, 640), ("png", 333, 517), ("bmp", 600, 401), ("png", 1080, 1920), ("jpg", 250, 333),
             ("bmp", 91, 123)]
    for i, (fmt, h, w) in enumerate(specs):
        img = J.test_image("scene", h, w, 70 + i)
        if fmt == "jpg":
            data = J.encode(img, 85, 2)
            ref = J.decode_rgb(data)
        else:
            b = io.BytesIO()
            Image.fromarray(img).save(b, "PNG" if fmt == "png" else "BMP")
            data = b.getvalue()
            ref = img
        p = tmp_path / f"{i}.{fmt}"
        p.write_bytes(data)
        paths.append(str(p))
        refs.append(ref)
    return paths, refs


def test_mixed_format_batch_decode(tmp_path):
    paths, refs = _mixed_files(tmp_path)
    outs = WJ.decode_batch([open(p, "rb").read() for p in paths])
    for o, r in zip(outs, refs):
        assert np.array_equal(o, r)
    for p, r in zip(paths, refs):
        assert np.array_equal(wicca_amd.load_image(p), r)


@pytest.mark.parametrize("depth,shape", [(5, (224, 224)), (3, (299, 299))])
def test_mixed_format_file_caller_stage(tmp_path, depth, shape):
    paths, refs = _mixed_files(tmp_path)
    imgs, icons = wicca_amd.get_img_batch(paths, shape, depth)
    for i, rgb in enumerate(refs):
        assert np.array_equal(imgs[i], R.resize(rgb, shape, R.INTER_AREA)), i
        icon = c_oracle.ll_int_block(rgb, depth)[0]
        assert np.array_equal(icons[i], R.resize(icon, shape, R.INTER_AREA)), i
    two = wicca_amd.get_img_batch(paths, shape, depth, devices=[0, 0])
    assert np.array_equal(two[0], imgs) and np.array_equal(two[1], icons)


def _recrc(data: bytes, at: int) -> bytes:
    """Fix the CRC of the chunk whose type starts at `at`."""
    n = struct.unpack(">I", data[at - 4:at])[0]
    crc = struct.pack(">I", zlib.crc32(data[at:at + 4 + n]) & 0xFFFFFFFF)
    return data[:at + 4 + n] + crc + data[at + 8 + n:]


def test_corrupt_png_and_bmp_fail_their_slot(tmp_path, capsys):
    s, _ = png_samples(2, 8, 40, 60, seed=1)
    good_png = rr.encode_png(s, 2, 8, filters=4)
    k = good_png.index(b"IDAT")
    idat_crc = good_png[:k + 10] + bytes([good_png[k + 10] ^ 0xFF]) + good_png[k + 11:]  # CRC mismatch
    raw = zlib.decompress(good_png[k + 4:k + 4 + struct.unpack(">I", good_png[k - 4:k])[0]])
    bad_filter_raw = bytes([7]) + raw[1:]
    comp = zlib.compress(bad_filter_raw)
    bad_filter = good_png[:k - 4] + struct.pack(">I", len(comp)) + b"IDAT" + comp + b"\0\0\0\0" + \
        good_png[k + 8 + struct.unpack(">I", good_png[k - 4:k])[0]:]
    bad_filter = _recrc(bad_filter, k)
    short_comp = zlib.compress(raw[: len(raw) // 2])
    short = good_png[:k - 4] + struct.pack(">I", len(short_comp)) + b"IDAT" + short_comp + b"\0\0\0\0" + \
        good_png[k + 8 + struct.unpack(">I", good_png[k - 4:k])[0]:]
    short = _recrc(short, k)
    no_iend = good_png[:-12]
    img = np.random.default_rng(2).integers(0, 256, (20, 30, 3), dtype=np.uint8)
    good_bmp = rr.encode_bmp(img, 24)
    trunc_bmp = good_bmp[:-50]
    rle_bmp = good_bmp[:30] + struct.pack("<I", 1) + good_bmp[34:]
    blobs = [good_png, idat_crc, good_bmp, bad_filter, short, no_iend, trunc_bmp, rle_bmp, b"GIF89a" + b"\0" * 30]
    outs = WJ.decode_batch(blobs, errors="none")
    assert [o is None for o in outs] == [False, True, False, True, True, True, True, True, True]
    assert np.array_equal(outs[0], s.astype(np.uint8)) and np.array_equal(outs[2], img)
    with pytest.raises((ValueError, NotImplementedError)):
        WJ.decode_batch(blobs)
    with pytest.raises(ValueError):  # BI_RLE8 on a 24-bit header: no valid BMP
        WJ.decode(rle_bmp)
    paths = []
    for i, b in enumerate(blobs):
        p = tmp_path / f"c{i}.png"
        p.write_bytes(b)
        paths.append(str(p))
    imgs, icons = wicca_amd.get_img_batch(paths, (224, 224), 3, errors="zero")
    printed = capsys.readouterr().out
    for i, o in enumerate(outs):
        if o is None:
            assert not imgs[i].any() and not icons[i].any(), i
            assert f"Error loading image {paths[i]}" in printed
        else:
            assert np.array_equal(imgs[i], R.resize(o, (224, 224), R.INTER_AREA))
            assert np.array_equal(icons[i], R.resize(c_oracle.ll_int_block(o, 3)[0], (224, 224), R.INTER_AREA))
    for p, o in zip(paths, outs):
        got = wicca_amd.load_image(p)
        assert (got is None) == (o is None)


GOLD_CASES = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "raster", "cases.json")))["cases"]


@pytest.mark.parametrize("case", GOLD_CASES, ids=[c["file"] for c in GOLD_CASES])
def test_golden_files(case):
    """The committed files (tests/golden/make_raster_seeds.py), expected RGB
    SHA-256 from Pillow 12.2.0 (from the restatement for the two unpinned kinds)."""
    data = open(os.path.join(os.path.dirname(__file__), "golden", "raster", case["file"]), "rb").read()
    rgb = WJ.decode(data)
    assert rgb.shape == (case["height"], case["width"], 3)
    assert hashlib.sha256(rgb.tobytes()).hexdigest() == case["sha256_rgb"]


from test_raster_oracle import TIFF_KINDS, tiff_case  # noqa: E402


@pytest.mark.parametrize("kind", TIFF_KINDS)
@pytest.mark.parametrize("comp,pred,tile,be", [(1, 1, None, False), (8, 2, None, True), (32773, 1, (16, 32), False),
                                              (8, 1, (32, 16), True), (8, 2, (16, 16), False)])
def test_tiff_vs_oracle(kind, comp, pred, tile, be):
    blobs, wants = [], []
    for i, (h, w) in enumerate([(1, 1), (5, 3), (37, 45), (130, 257)]):
        s, photo, bits, cm, extra = tiff_case(kind, h, w, seed=i + len(kind))
        p = pred if bits == 8 else 1
        data = rr.encode_tiff(s, photo, bits, comp, p, tile=tile, big_endian=be, colormap=cm, extra_samples=extra,
                              rows_per_strip=7)
        blobs.append(data)
        wants.append(s[..., :3] if kind == "rgba_assoc" else rr.decode_tiff(data))
    for o, want in zip(WJ.decode_batch(blobs), wants):
        assert np.array_equal(o, want)


def test_tiff_unassociated_alpha():
    s = np.random.default_rng(4).integers(0, 256, (33, 50, 4), dtype=np.uint8)
    data = rr.encode_tiff(s, 2, extra_samples=2, compression=8)
    want = ((s[..., :3].astype(np.uint32) * s[..., 3:4] + 127) // 255).astype(np.uint8)
    assert np.array_equal(WJ.decode(data), want)
    assert np.array_equal(rr.decode_tiff(data), want)


@pytest.mark.parametrize("mode", ["RGB", "L", "P", "1", "LA"])
@pytest.mark.parametrize("comp", [None, "tiff_lzw", "tiff_deflate", "packbits"])
def test_pillow_written_tiff(mode, comp):
    from PIL import Image
    img = J.test_image("scene", 300, 401, 7)
    b = io.BytesIO()
    Image.fromarray(img).convert(mode).save(b, "TIFF", compression=comp)
    data = b.getvalue()
    assert np.array_equal(WJ.decode(data), rr.pillow_rgb(data))
    assert WJ.image_info(data) == (300, 401, "tiff")


def test_tiff_lzw_8k_vs_pillow():
    from PIL import Image
    img = J.test_image("scene", 4320, 7680, 12)
    b = io.BytesIO()
    Image.fromarray(img).save(b, "TIFF", compression="tiff_lzw")
    assert np.array_equal(WJ.decode(b.getvalue()), img)


def test_tiff_unsupported_and_corrupt():
    from PIL import Image
    img = J.test_image("scene", 40, 60, 3)
    b = io.BytesIO()
    Image.fromarray(img).save(b, "TIFF", compression="jpeg")
    with pytest.raises(NotImplementedError):
        WJ.decode(b.getvalue())
    b = io.BytesIO()
    Image.fromarray(img).save(b, "TIFF", compression="tiff_lzw")
    good = b.getvalue()
    s = np.frombuffer(good, np.uint8)
    cut = good[:200]  # strips outside the file
    outs = WJ.decode_batch([good, cut, good[:7]], errors="none")
    assert np.array_equal(outs[0], img) and outs[1] is None and outs[2] is None
    assert s.size > 200


def test_pipelined_stage_with_png_batches(tmp_path):
    """get_img_batches over PNG / BMP / mixed batches (their stage runs on a
    host thread of its own): the same outputs as get_img_batch, batch by
    batch; a corrupt PNG (found during the inflate) fails at its wait."""
    paths, refs = _mixed_files(tmp_path)
    batches = [paths[:3], paths[3:], [paths[1], paths[3]], paths]
    for depth in (1, 2):
        got = list(wicca_amd.get_img_batches(batches, (224, 224), 3, depth=depth))
        for b, (imgs, icons) in zip(batches, got):
            want = wicca_amd.get_img_batch(b, (224, 224), 3)
            assert np.array_equal(imgs, want[0]) and np.array_equal(icons, want[1])
    s, _ = png_samples(2, 8, 40, 60, seed=1)
    good = rr.encode_png(s, 2, 8)
    k = good.index(b"IDAT")
    bad = tmp_path / "bad.png"
    bad.write_bytes(good[:k + 10] + bytes([good[k + 10] ^ 0xFF]) + good[k + 11:])  # IDAT CRC error
    with pytest.raises(ValueError):
        list(wicca_amd.get_img_batches([paths[:2], [str(bad)], paths[2:4]], (224, 224), 3))


@pytest.mark.parametrize("interlace", [False, True])
@pytest.mark.parametrize("local", [False, True])
def test_gif_vs_expected(interlace, local):
    """GIF first frame: full-screen images against Pillow; partial frames and
    transparency against the restatement (black canvas, parity unpinned)."""
    rng = np.random.default_rng(int(interlace) * 2 + int(local))
    blobs, wants = [], []
    for (h, w, npal, screen, pos, tr) in [(1, 1, 2, None, (0, 0), None), (7, 5, 4, None, (0, 0), None),
                                          (40, 60, 256, None, (0, 0), None), (33, 17, 16, (50, 40), (9, 11), None),
                                          (20, 30, 8, None, (0, 0), 3), (25, 25, 32, (30, 26), (5, 1), 0),
                                          (300, 401, 256, None, (0, 0), None)]:
        idx = rng.integers(0, npal, (h, w), dtype=np.uint8)
        idx[: h // 2] = (np.arange(w) % npal)[None, :]
        pal = rng.integers(0, 256, (npal, 3), dtype=np.uint8)
        data = rr.encode_gif(idx, pal, screen=screen, pos=pos, transparent=tr, interlace=interlace,
                             local_palette=local)
        blobs.append(data)
        want = rr.gif_expected(idx, pal, screen=screen, pos=pos, transparent=tr)
        if screen is None and tr is None:
            assert np.array_equal(want, rr.pillow_rgb(data))
        wants.append(want)
    for o, want in zip(WJ.decode_batch(blobs), wants):
        assert np.array_equal(o, want)


def test_pillow_written_gif_and_mixed_stage(tmp_path):
    from PIL import Image
    img = J.test_image("scene", 1080, 1920, 21)
    b = io.BytesIO()
    Image.fromarray(img).convert("P").save(b, "GIF")
    data = b.getvalue()
    assert np.array_equal(WJ.decode(data), rr.pillow_rgb(data))
    p = tmp_path / "x.gif"
    p.write_bytes(data)
    paths, refs = _mixed_files(tmp_path)
    paths.append(str(p))
    refs.append(rr.pillow_rgb(data))
    imgs, icons = wicca_amd.get_img_batch(paths, (224, 224), 4)
    for i, rgb in enumerate(refs):
        assert np.array_equal(imgs[i], R.resize(rgb, (224, 224), R.INTER_AREA)), i
        assert np.array_equal(icons[i], R.resize(c_oracle.ll_int_block(rgb, 4)[0], (224, 224), R.INTER_AREA)), i


def test_decode_batches_mixed_formats(tmp_path):
    """jpeg.decode_batches over all-JPEG and mixed batches: device tensors
    equal to the synchronous decode of the same files."""
    paths, refs = _mixed_files(tmp_path)
    blobs = [open(p, "rb").read() for p in paths]
    batches = [[blobs[0], blobs[4]], blobs[:3], [blobs[4]], blobs]
    got = list(WJ.decode_batches(batches, device=0))
    assert len(got) == len(batches)
    for batch, outs in zip(batches, got):
        for b, t in zip(batch, outs):
            assert np.array_equal(t.cpu().numpy(), WJ.decode(b))


def test_gif_oversized_frame_descriptor_is_cheap():
    """A 1x1 canvas whose image descriptor claims a 65535 x 65535 frame (ADVICE
    r03): the host decode holds one stream row at a time, so the file decodes
    in well under a second to the canvas pixel the stream reaches."""
    import time
    idx = np.array([[1, 0, 1]], np.uint8)
    pal = np.array([[10, 20, 30], [200, 100, 50]], np.uint8)
    data = bytearray(rr.encode_gif(idx, pal, screen=(1, 1)))
    k = data.index(b"\x2c")
    data[k + 5:k + 9] = struct.pack("<HH", 65535, 65535)  # frame width / height
    t0 = time.perf_counter()
    got = WJ.decode(bytes(data))
    assert time.perf_counter() - t0 < 5.0
    assert got.shape == (1, 1, 3) and got[0, 0].tolist() == [200, 100, 50]


@pytest.mark.parametrize("rle4", [False, True], ids=["rle8", "rle4"])
def test_rle_bmp_vs_pillow(rle4):
    """BI_RLE8 / BI_RLE4 BMPs (encoded and absolute runs, end of line, delta
    escapes; skipped pixels take palette entry 0) against Pillow, batched with
    an uncompressed BMP."""
    rng = np.random.default_rng(21 + rle4)
    pal = rng.integers(0, 256, (16 if rle4 else 256, 3)).astype(np.uint8)
    blobs, wants = [], []
    for absolute, skips, shape in [(False, False, (37, 53)), (True, False, (64, 300)), (True, True, (120, 257)),
                                   (True, True, (1, 1))]:
        idx = rng.integers(0, len(pal), shape).astype(np.uint8)
        idx[:, : shape[1] // 3] = idx[:, :1]
        data, want = rr.encode_bmp_rle(idx, pal, rle4, absolute, skips)
        blobs.append(data)
        wants.append(pal[want])
    plain = rr.encode_bmp(rng.integers(0, 256, (30, 41, 3), dtype=np.uint8), 24)
    got = WJ.decode_batch(blobs + [plain])
    for i, data in enumerate(blobs):
        assert np.array_equal(got[i], wants[i]), i
        assert np.array_equal(got[i], rr.pillow_rgb(data)), i
    assert np.array_equal(got[-1], rr.decode_bmp(plain))


def test_rle_bmp_corrupt_rules():
    """Corrupt or unusual RLE data, PARITY UNPINNED (cv2 absent; restated from
    OpenCV's BmpDecoder, where Pillow refuses or clips): end of bitmap before
    the last row (the rest takes palette entry 0), a run past a row's end
    (fails the file's slot; Pillow clips it), and a delta past the bottom row
    (ends the bitmap: the rows it skips take palette entry 0).  Pinned here so
    that a change of these rules is deliberate."""
    rng = np.random.default_rng(5)
    pal = rng.integers(0, 256, (256, 3)).astype(np.uint8)
    idx = rng.integers(0, 256, (20, 33)).astype(np.uint8)
    early, want = rr.encode_bmp_rle(idx, pal, False, True, False, end_early=True)
    assert np.array_equal(WJ.decode(early), pal[want])
    good, _ = rr.encode_bmp_rle(idx, pal)
    hdr = 14 + 40 + 4 * 256
    over = good[:hdr] + bytes([200, 9]) + good[hdr:]  # a 200-pixel run in a 33-pixel row
    got = WJ.decode_batch([over, good], errors="none")
    assert got[0] is None and np.array_equal(got[1], pal[idx])
    # a delta escape of 50 rows after the first stored row (the bottom one)
    runs, _ = rr.encode_bmp_rle(idx, pal, False, False)  # encoded runs only: the first 00 00 is an end of line
    first_eol = next(i for i in range(hdr, len(runs) - 1, 2) if runs[i] == 0 and runs[i + 1] == 0)
    deep = runs[:first_eol + 2] + bytes([0, 2, 0, 50]) + runs[first_eol + 2:]
    want = np.zeros_like(idx)
    want[-1] = idx[-1]
    assert np.array_equal(WJ.decode(deep), pal[want])


def _plain_pnm(img: np.ndarray, rng) -> bytes:
    """A plain (ASCII) P2 / P3 file of `img`: tokens split over lines of
    random length, runs of whitespace, comments between samples."""
    gray = img.ndim == 2
    h, w = img.shape[:2]
    out = [b"P2\n" if gray else b"P3\n", b"# plain\n", b"%d %d\n255\n" % (w, h)]
    line = []
    for v in img.reshape(-1).tolist():
        line.append(b"%d" % v)
        if rng.random() < 0.05:
            out.append(b" ".join(line) + (b"  # note 12 34\n" if rng.random() < 0.3 else b"\n\t"))
            line = []
    out.append(b" ".join(line) + b"\n")
    return b"".join(out)


def test_pnm_vs_pillow(tmp_path, capsys):
    """PGM / PPM at maxval 255, binary (P5 / P6) and plain (P2 / P3: tokens,
    whitespace and comments), and P4 bitmaps (load_image, file stage), pinned
    to Pillow; plain P1 bitmaps and other maxvals fail their slot as
    unsupported."""
    from PIL import Image
    rng = np.random.default_rng(8)
    gray = rng.integers(0, 256, (61, 93), dtype=np.uint8)
    rgb = rng.integers(0, 256, (480, 640, 3), dtype=np.uint8)
    bits = rng.integers(0, 2, (37, 75), dtype=np.uint8)
    buf = io.BytesIO()
    Image.fromarray((bits * 255).astype(np.uint8)).convert("1").save(buf, format="PPM")
    pbm = buf.getvalue()
    assert pbm[:2] == b"P4"
    blobs = [rr.encode_pnm(gray), rr.encode_pnm(rgb, comment=False), _plain_pnm(gray, rng),
             _plain_pnm(rgb[:97, :133], rng), pbm]
    got = WJ.decode_batch(blobs)
    assert np.array_equal(got[0], np.repeat(gray[..., None], 3, axis=2))
    assert np.array_equal(got[1], rgb)
    assert np.array_equal(got[2], got[0])
    assert np.array_equal(got[3], rgb[:97, :133])
    assert np.array_equal(got[4], np.repeat((bits * 255)[..., None], 3, axis=2))
    for i, data in enumerate(blobs):
        assert np.array_equal(got[i], rr.pillow_rgb(data)), i
    plain_pbm = b"P1\n2 2\n0 1 1 0\n"
    wide = b"P5\n2 2\n65535\n" + bytes(8)
    short = b"P2\n2 2\n255\n0 1 2\n"
    bad_token = b"P3\n1 1\n255\n1 x 3\n"
    assert WJ.decode_batch([plain_pbm, wide, short, bad_token, blobs[0]], errors="none")[:4] == [None] * 4
    p = tmp_path / "x.ppm"
    p.write_bytes(blobs[1])
    imgs, icons = wicca_amd.get_img_batch([str(p)], (224, 224), 3)
    assert np.array_equal(imgs[0], R.resize(rgb, (224, 224), R.INTER_AREA))
    assert np.array_equal(icons[0], R.resize(c_oracle.ll_int_block(rgb, 3)[0], (224, 224), R.INTER_AREA))


@pytest.mark.parametrize("spp,photometric,extra", [(3, 2, None), (4, 2, 2), (2, 1, 2)])
@pytest.mark.parametrize("layout", ["strips", "tiles", "deflate_pred"])
def test_tiff_separate_planes_vs_pillow(spp, photometric, extra, layout):
    """PlanarConfiguration 2 (8-bit RGB, RGBA unassociated, gray + alpha):
    each plane's strips / tiles, interleaved on the host; pinned to Pillow
    (libtiff 4.7.1; with libtiff's unassociated-alpha rule, rr.decode_tiff)
    and equal to the same image stored chunky."""
    rng = np.random.default_rng(spp * 7 + len(layout))
    img = rng.integers(0, 256, (45, 70, spp), dtype=np.uint8)
    kw = dict(tile=(32, 16)) if layout == "tiles" else dict(rows_per_strip=7)
    if layout == "deflate_pred":
        kw.update(compression=8, predictor=2)
    sep = rr.encode_tiff(img, photometric, extra_samples=extra, planar=2, **kw)
    chunky = rr.encode_tiff(img, photometric, extra_samples=extra, **kw)
    got = WJ.decode_batch([sep, chunky])
    assert np.array_equal(got[0], got[1])
    if spp != 2:  # Pillow has no raw mode for separate gray + alpha planes: the chunky file is the check
        assert np.array_equal(got[0], rr.decode_tiff(sep))
    assert np.array_equal(got[1], rr.decode_tiff(chunky))
