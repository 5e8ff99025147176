"""PNG / BMP / TIFF decode checker and test-file writer — TEST INFRASTRUCTURE.

The reference's ``load_image`` is ``cv2.imread(path)`` (IMREAD_COLOR) +
``cvtColor(BGR2RGB)`` (``/root/reference/wicca/data_loader.py:53-58``);
``ClassifierProcessor`` counts ``.png`` and ``.bmp`` inputs
(``classifying_tools.py:162``).  cv2 (opencv-python 4.12.0.88) is absent
here, so this module restates what IMREAD_COLOR does with those files, in
NumPy + zlib, from the formats' specifications and OpenCV's decoders:

* PNG (ISO/IEC 15948; OpenCV ``PngDecoder`` over libpng): inflate the
  concatenated IDAT data, reconstruct rows (filters 0-4), de-interlace Adam7,
  then ``png_set_expand_gray_1_2_4_to_8`` (x255 / x85 / x17),
  ``png_set_palette_to_rgb``, ``png_set_gray_to_rgb``, ``png_set_strip_alpha``,
  ``png_set_strip_16`` (high byte).
* BMP (OpenCV ``BmpDecoder``): palette entries BGRx, 16-bit 5-5-5 / 5-6-5
  with ``component << 3`` (``<< 2`` for 6-bit green), 24-bit BGR, 32-bit BGRx,
  rows bottom-up unless the height is negative, row stride padded to 4 B.

Pinning: for every 8-bit PNG colour type, sub-byte gray / palette, Adam7, and
the 1/4/8/24/32-bit BMPs, ``tests/test_raster_oracle.py`` checks this
restatement against Pillow 12.2.0's decoders (``Image.convert("RGB")`` drops
alpha and expands palettes / gray the same way).  16-bit PNG RGB(A) is pinned
the same way (Pillow keeps the high byte).  16-bit gray PNG (Pillow clips
instead of taking the high byte) and 16-bit BMP (Pillow rescales 5-bit values
by 255/31; OpenCV shifts) are **parity unpinned**: the restatement follows
OpenCV's code as described above.

* TIFF (OpenCV ``TiffDecoder``: 8-bit output goes through libtiff's RGBA
  interface): checked against Pillow 12.2.0 (libtiff 4.7.1 for the
  compressed strips) for gray / WhiteIsZero / RGB / palette / bilevel files,
  none / LZW / Deflate / PackBits, predictor 2, strips and tiles, both byte
  orders; RGBA with unassociated alpha follows libtiff's premultiplication
  (``decode_tiff``, parity unpinned).
* GIF (OpenCV ``GifDecoder``, first frame): a full-screen image without
  transparency is checked against Pillow's decode; transparent and
  uncovered pixels are black in the restatement (``gif_expected``: OpenCV
  draws onto a zeroed BGRA canvas and drops alpha; Pillow fills with the
  palette / background colour instead), parity unpinned.  Only ``tests/``
  uses this module.
"""
from __future__ import annotations

import struct
import zlib

import numpy as np

SIG = b"\x89PNG\r\n\x1a\n"
CHANNELS = {0: 1, 2: 3, 3: 1, 4: 2, 6: 4}
# Adam7: (x0, y0, dx, dy) per pass
ADAM7 = [(0, 0, 8, 8), (4, 0, 8, 8), (0, 4, 4, 8), (2, 0, 4, 4), (0, 2, 2, 4), (1, 0, 2, 2), (0, 1, 1, 2)]


# ----------------------------------------------------------------------------- PNG
def _chunks(data: bytes):
    pos = 8
    while pos + 8 <= len(data):
        n, t = struct.unpack(">I4s", data[pos:pos + 8])
        yield t, data[pos + 8:pos + 8 + n]
        pos += 12 + n
        if t == b"IEND":
            break


def _paeth(a: int, b: int, c: int) -> int:
    p = a + b - c
    pa, pb, pc = abs(p - a), abs(p - b), abs(p - c)
    if pa <= pb and pa <= pc:
        return a
    return b if pb <= pc else c


def _unfilter(raw: bytes, w: int, h: int, bits_pp: int, pos: int):
    """Reconstructed rows (h, row_bytes) of one (sub-)image starting at raw[pos]."""
    rb = (w * bits_pp + 7) // 8
    bpp = max(1, bits_pp // 8)
    out = np.zeros((h, rb), np.uint8)
    prev = np.zeros(rb, np.int64)
    for y in range(h):
        f = raw[pos]
        x = np.frombuffer(raw, np.uint8, rb, pos + 1).astype(np.int64)
        pos += 1 + rb
        if f == 0:
            r = x
        elif f == 1:
            r = x.copy()
            for i in range(bpp, rb):
                r[i] = (r[i] + r[i - bpp]) & 255
        elif f == 2:
            r = (x + prev) & 255
        elif f == 3:
            r = x.copy()
            for i in range(rb):
                a = r[i - bpp] if i >= bpp else 0
                r[i] = (r[i] + ((a + prev[i]) >> 1)) & 255
        elif f == 4:
            r = x.copy()
            for i in range(rb):
                a = r[i - bpp] if i >= bpp else 0
                c = prev[i - bpp] if i >= bpp else 0
                r[i] = (r[i] + _paeth(int(a), int(prev[i]), int(c))) & 255
        else:
            raise ValueError("bad adaptive filter value")
        out[y] = r
        prev = r
    return out, pos


def _samples(rows: np.ndarray, w: int, ch: int, bits: int) -> np.ndarray:
    """(h, w, ch) integer samples of reconstructed rows (16-bit: high byte)."""
    h = rows.shape[0]
    if bits == 16:
        return rows[:, : w * ch * 2].reshape(h, w, ch, 2)[..., 0]
    if bits == 8:
        return rows[:, : w * ch].reshape(h, w, ch)
    bitsarr = np.unpackbits(rows, axis=1)[:, : w * bits].reshape(h, w, bits)
    weights = (1 << np.arange(bits - 1, -1, -1)).astype(np.uint8)
    return (bitsarr * weights).sum(axis=2).astype(np.uint8)[..., None]


def decode_png(data: bytes) -> np.ndarray:
    """RGB (H, W, 3) uint8 of a PNG file as cv2.imread(IMREAD_COLOR) + BGR2RGB."""
    if data[:8] != SIG:
        raise ValueError("not a PNG")
    ihdr = None
    pal = np.zeros((256, 3), np.uint8)
    idat = b""
    for t, body in _chunks(data):
        if t == b"IHDR":
            ihdr = struct.unpack(">IIBBBBB", body)
        elif t == b"PLTE":
            p = np.frombuffer(body, np.uint8).reshape(-1, 3)
            pal[: len(p)] = p
        elif t == b"IDAT":
            idat += body
    w, h, bits, ct, _, _, il = ihdr
    ch = CHANNELS[ct]
    raw = zlib.decompressobj().decompress(idat)
    if il == 0:
        rows, _ = _unfilter(raw, w, h, ch * bits, 0)
        s = _samples(rows, w, ch, bits)
    else:
        s = np.zeros((h, w, ch), np.uint8)
        pos = 0
        for x0, y0, dx, dy in ADAM7:
            pw = (w - x0 + dx - 1) // dx if w > x0 else 0
            ph = (h - y0 + dy - 1) // dy if h > y0 else 0
            if pw == 0 or ph == 0:
                continue
            rows, pos = _unfilter(raw, pw, ph, ch * bits, pos)
            s[y0::dy, x0::dx] = _samples(rows, pw, ch, bits)
    if ct == 3:
        return pal[s[..., 0]]
    if ct in (0, 4):
        g = s[..., 0].astype(np.uint32)
        if bits < 8:
            g = g * (255 // ((1 << bits) - 1))
        return np.repeat(g.astype(np.uint8)[..., None], 3, axis=2)
    return np.ascontiguousarray(s[..., :3])


def _filter_row(cur: np.ndarray, prev: np.ndarray, bpp: int, f: int) -> bytes:
    cur = cur.astype(np.int64)
    prev = prev.astype(np.int64)
    a = np.concatenate([np.zeros(bpp, np.int64), cur[:-bpp]]) if len(cur) > bpp else np.zeros_like(cur)
    if len(cur) > bpp:
        c = np.concatenate([np.zeros(bpp, np.int64), prev[:-bpp]])
    else:
        c = np.zeros_like(cur)
    if f == 0:
        o = cur
    elif f == 1:
        o = cur - a
    elif f == 2:
        o = cur - prev
    elif f == 3:
        o = cur - ((a + prev) >> 1)
    else:
        pred = np.array([_paeth(int(x), int(y), int(z)) for x, y, z in zip(a, prev, c)], np.int64)
        o = cur - pred
    return bytes([f]) + (o & 255).astype(np.uint8).tobytes()


def _pack(samples: np.ndarray, bits: int) -> np.ndarray:
    """Rows of (h, w*ch) samples packed to bytes (16-bit big-endian)."""
    h = samples.shape[0]
    if bits == 16:
        return samples.astype(">u2").view(np.uint8).reshape(h, -1)
    if bits == 8:
        return samples.astype(np.uint8)
    bitsarr = ((samples[..., None].astype(np.uint8) >> np.arange(bits - 1, -1, -1).astype(np.uint8)) & 1)
    return np.packbits(bitsarr.reshape(h, -1), axis=1)


def _chunk(t: bytes, body: bytes) -> bytes:
    return struct.pack(">I", len(body)) + t + body + struct.pack(">I", zlib.crc32(t + body) & 0xFFFFFFFF)


def encode_png(samples: np.ndarray, color_type: int, bits: int = 8, interlace: bool = False,
               palette: np.ndarray | None = None, filters=None, level: int = 6, idat_split: int = 0,
               extra_chunks=()) -> bytes:
    """A PNG file of (H, W, ch) integer samples (ch per colour type; values
    < 2**bits).  filters: None (cycle 0..4 per row), an int, or a callable
    (row index) -> filter type.  idat_split: IDAT chunk size (0: one chunk).
    extra_chunks: (type, body) pairs written before IDAT."""
    samples = np.asarray(samples)
    if samples.ndim == 2:
        samples = samples[..., None]
    h, w, ch = samples.shape
    assert ch == CHANNELS[color_type]
    bits_pp = ch * bits
    bpp = max(1, bits_pp // 8)
    pick = (lambda y: y % 5) if filters is None else (filters if callable(filters) else (lambda y: filters))
    raw = bytearray()
    subs = []
    if interlace:
        for x0, y0, dx, dy in ADAM7:
            sub = samples[y0::dy, x0::dx]
            if sub.size:
                subs.append(sub)
    else:
        subs.append(samples)
    k = 0
    for sub in subs:
        sh, sw, _ = sub.shape
        rows = _pack(sub.reshape(sh, sw * ch), bits)
        prev = np.zeros(rows.shape[1], np.uint8)
        for y in range(sh):
            raw += _filter_row(rows[y], prev, bpp, pick(k))
            prev = rows[y]
            k += 1
    comp = zlib.compress(bytes(raw), level)
    out = SIG + _chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, bits, color_type, 0, 0, 1 if interlace else 0))
    if palette is not None:
        out += _chunk(b"PLTE", np.asarray(palette, np.uint8).tobytes())
    for t, body in extra_chunks:
        out += _chunk(t, body)
    step = idat_split or len(comp) or 1
    for i in range(0, max(len(comp), 1), step):
        out += _chunk(b"IDAT", comp[i:i + step])
    return out + _chunk(b"IEND", b"")


# ----------------------------------------------------------------------------- BMP
def decode_bmp(data: bytes) -> np.ndarray:
    """RGB (H, W, 3) uint8 of an uncompressed BMP as cv2.imread + BGR2RGB."""
    off, size = struct.unpack("<I", data[10:14])[0], struct.unpack("<I", data[14:18])[0]
    if size == 12:
        w, h, _, bpp = struct.unpack("<hhHH", data[18:26])
        comp, clrused, pal_pos, ent = 0, 0, 26, 3
    else:
        w, h, _, bpp, comp = struct.unpack("<iiHHI", data[18:34])
        clrused = struct.unpack("<i", data[46:50])[0]
        pal_pos, ent = 14 + size, 4
    bottom_up = h > 0
    h = abs(h)
    stride = (w * bpp + 31) // 32 * 4
    px = np.frombuffer(data, np.uint8, stride * h, off).reshape(h, stride)
    if bottom_up:
        px = px[::-1]
    if bpp <= 8:
        cnt = clrused or (1 << bpp)
        pal = np.zeros((256, 3), np.uint8)
        p = np.frombuffer(data, np.uint8, cnt * ent, pal_pos).reshape(cnt, ent)
        pal[:cnt] = p[:, 2::-1]
        idx = _samples(px, w, 1, bpp)[..., 0] if bpp < 8 else px[:, :w]
        return pal[idx]
    if bpp == 24:
        return np.ascontiguousarray(px[:, : 3 * w].reshape(h, w, 3)[..., ::-1])
    if bpp == 32:
        return np.ascontiguousarray(px[:, : 4 * w].reshape(h, w, 4)[..., 2::-1])
    v = px[:, : 2 * w].reshape(h, w, 2).astype(np.uint32)
    v = v[..., 0] | (v[..., 1] << 8)
    six = False
    if comp == 3:
        mpos = 54 if size >= 52 else 14 + size
        rm, gm, bm = struct.unpack("<III", data[mpos:mpos + 12])
        six = gm == 0x7E0
    b = (v & 31) << 3
    if six:
        g, r = ((v >> 5) & 63) << 2, ((v >> 11) & 31) << 3
    else:
        g, r = ((v >> 5) & 31) << 3, ((v >> 10) & 31) << 3
    return np.stack([r, g, b], axis=2).astype(np.uint8)


def encode_bmp(img: np.ndarray, bpp: int = 24, palette: np.ndarray | None = None, top_down: bool = False,
               fields565: bool | None = None, core_header: bool = False) -> bytes:
    """A BMP file: bpp 24 / 32 of an (H, W, 3) RGB array, 1/4/8 of an (H, W)
    index array with an (n, 3) RGB palette, 16 of (H, W, 3) RGB (5-5-5 as
    BI_RGB; fields565 True/False -> BI_BITFIELDS 5-6-5 / 5-5-5)."""
    img = np.asarray(img)
    h, w = img.shape[:2]
    stride = (w * bpp + 31) // 32 * 4
    if bpp == 24:
        rows = img[..., ::-1].reshape(h, w * 3)
    elif bpp == 32:
        rows = np.concatenate([img[..., ::-1], np.full((h, w, 1), 0x7F, np.uint8)], axis=2).reshape(h, w * 4)
    elif bpp == 16:
        r, g, b = (img[..., i].astype(np.uint32) for i in range(3))
        v = ((r >> 3) << 11 | (g >> 2) << 5 | (b >> 3)) if fields565 else ((r >> 3) << 10 | (g >> 3) << 5 | (b >> 3))
        rows = np.stack([v & 255, v >> 8], axis=2).astype(np.uint8).reshape(h, w * 2)
    else:
        rows = _pack(img.astype(np.uint8), bpp)
    px = np.zeros((h, stride), np.uint8)
    px[:, : rows.shape[1]] = rows
    if not top_down:
        px = px[::-1]
    pal = b""
    comp = 0
    if bpp <= 8:
        p = np.asarray(palette, np.uint8)
        ent = 3 if core_header else 4
        q = np.zeros((len(p), ent), np.uint8)
        q[:, :3] = p[:, ::-1]
        pal = q.tobytes()
    elif bpp == 16 and fields565 is not None:
        comp = 3
        pal = struct.pack("<III", 0xF800, 0x7E0, 0x1F) if fields565 else struct.pack("<III", 0x7C00, 0x3E0, 0x1F)
    if core_header:
        hdr = struct.pack("<IhhHH", 12, w, -h if top_down else h, 1, bpp)
    else:
        clr = len(palette) if bpp <= 8 else 0
        hdr = struct.pack("<IiiHHIIiiII", 40, w, -h if top_down else h, 1, bpp, comp, stride * h, 2835, 2835,
                          clr, 0)
    off = 14 + len(hdr) + len(pal)
    total = off + px.size
    return b"BM" + struct.pack("<IHHI", total, 0, 0, off) + hdr + pal + px.tobytes()


def encode_bmp_rle(idx: np.ndarray, palette: np.ndarray, rle4: bool = False, absolute: bool = True,
                   skips: bool = False, end_early: bool = False):
    """A BI_RLE8 / BI_RLE4 BMP of an (H, W) index array (bottom-up) and the
    indices a decoder must produce: rows as encoded runs (a repeated index, or
    for RLE4 an alternating pair) and, with `absolute`, absolute runs of 3..64
    indices (padded to 16 bits; even counts for RLE4); end of line after every row; `skips` ends
    some rows early (end of line) and opens others with a delta escape over
    their first two pixels -- skipped pixels decode as index 0; `end_early`
    stops with end of bitmap halfway (OpenCV fills the rest with palette
    entry 0, Pillow refuses such a file).  Returns (file bytes, indices)."""
    idx = np.asarray(idx, np.uint8)
    h, w = idx.shape
    want = idx.copy()
    out = bytearray()
    stop = max(1, h // 2) if end_early else h
    for ys, r in enumerate(range(h - 1, -1, -1)):  # stored bottom-up
        if ys >= stop:
            want[r, :] = 0
            continue
        row = [int(v) for v in idx[r]]
        end, x = w, 0
        if skips and ys % 5 == 3:  # end of line before the row's end
            end = w // 2
            want[r, end:] = 0
        if skips and ys % 7 == 2 and w > 4:  # a delta escape over the first two pixels
            out += bytes([0, 2, 2, 0])
            want[r, :2] = 0
            x = 2
        while x < end:
            if rle4:
                a = row[x]
                bb = row[x + 1] if x + 1 < end else 0
                n = 1
                while x + n < end and n < 255 and row[x + n] == (a if n % 2 == 0 else bb):
                    n += 1
                if absolute and n < 3 and end - x >= 4:
                    m = min(end - x, 64) & ~1  # even: Pillow reads odd RLE4 absolute runs one pixel short
                    vals = row[x:x + m] + [0]
                    packed = bytes((vals[i] << 4) | vals[i + 1] for i in range(0, m, 2))
                    out += bytes([0, m]) + packed + (b"\0" if len(packed) % 2 else b"")
                    x += m
                    continue
                out += bytes([n, (a << 4) | (bb if n > 1 else 0)])
                x += n
            else:
                v = row[x]
                n = 1
                while x + n < end and n < 255 and row[x + n] == v:
                    n += 1
                if absolute and n < 3 and end - x >= 3:
                    m = min(end - x, 64)
                    out += bytes([0, m]) + bytes(row[x:x + m]) + (b"\0" if m % 2 else b"")
                    x += m
                    continue
                out += bytes([n, v])
                x += n
        out += bytes([0, 0])  # end of line
    out += bytes([0, 1])  # end of bitmap
    p = np.asarray(palette, np.uint8)
    q = np.zeros((len(p), 4), np.uint8)
    q[:, :3] = p[:, ::-1]
    pal = q.tobytes()
    hdr = struct.pack("<IiiHHIIiiII", 40, w, h, 1, 4 if rle4 else 8, 2 if rle4 else 1, len(out), 2835, 2835, len(p), 0)
    off = 14 + len(hdr) + len(pal)
    return b"BM" + struct.pack("<IHHI", off + len(out), 0, 0, off) + hdr + pal + bytes(out), want


def encode_pnm(img: np.ndarray, comment: bool = True) -> bytes:
    """Binary PGM (P5, an (H, W) array) or PPM (P6, (H, W, 3)) at maxval 255."""
    img = np.asarray(img, np.uint8)
    magic = b"P5" if img.ndim == 2 else b"P6"
    h, w = img.shape[:2]
    head = magic + b"\n" + (b"# written by the test suite\n" if comment else b"") + f"{w} {h}\n255\n".encode()
    return head + img.tobytes()


# ----------------------------------------------------------------------------- TIFF
def _packbits(b: bytes) -> bytes:
    out = bytearray()
    i = 0
    while i < len(b):
        j = i
        while j < len(b) and j - i < 128 and b[j] == b[i]:
            j += 1
        if j - i >= 3:
            out += bytes([(257 - (j - i)) & 255, b[i]])
            i = j
            continue
        j = i
        while j < len(b) and j - i < 128 and not (j + 2 < len(b) and b[j] == b[j + 1] == b[j + 2]):
            j += 1
        out += bytes([j - i - 1]) + b[i:j]
        i = j
    return bytes(out)


def _tiff_rows(samples: np.ndarray, bits: int) -> np.ndarray:
    h = samples.shape[0]
    return _pack(samples.reshape(h, -1), bits)


def encode_tiff(samples: np.ndarray, photometric: int, bits: int = 8, compression: int = 1, predictor: int = 1,
                tile=None, rows_per_strip: int = 8, big_endian: bool = False, colormap=None,
                extra_samples=None, planar: int = 1) -> bytes:
    """A TIFF file of (H, W[, spp]) samples: compression 1 none / 8 Deflate /
    32773 PackBits, predictor 2 (8-bit), strips of rows_per_strip rows or
    tiles (tw, th), either byte order; colormap (2**bits, 3) 16-bit values;
    planar 2: each sample's plane stored on its own (PlanarConfiguration 2,
    plane 0's strips / tiles first)."""
    samples = np.asarray(samples)
    if samples.ndim == 2:
        samples = samples[..., None]
    h, w, spp = samples.shape
    e = ">" if big_endian else "<"
    planes = [samples[..., c:c + 1] for c in range(spp)] if planar == 2 else [samples]

    def code(seg_samples):
        rows = _tiff_rows(seg_samples, bits).astype(np.uint8)
        if predictor == 2:
            r = rows.astype(np.int64).reshape(rows.shape[0], -1, seg_samples.shape[2])
            d = r.copy()
            d[:, 1:] = r[:, 1:] - r[:, :-1]
            rows = (d & 255).astype(np.uint8).reshape(rows.shape[0], -1)
        raw = rows.tobytes()
        if compression == 8:
            return zlib.compress(raw)
        if compression == 32773:
            return b"".join(_packbits(rows[i].tobytes()) for i in range(rows.shape[0]))
        return raw

    segs = []
    for pl in planes:
        if tile:
            tw, th = tile
            for ty in range(0, h, th):
                for tx in range(0, w, tw):
                    t = np.zeros((th, tw, pl.shape[2]), samples.dtype)
                    blk = pl[ty:ty + th, tx:tx + tw]
                    t[:blk.shape[0], :blk.shape[1]] = blk
                    segs.append(code(t))
        else:
            for y in range(0, h, rows_per_strip):
                segs.append(code(pl[y:y + rows_per_strip]))
    body = bytearray(b"MM\x00*" if big_endian else b"II*\x00") + b"\0\0\0\0"
    offs = []
    for sgm in segs:
        offs.append(len(body))
        body += sgm
        if len(body) % 2:
            body += b"\0"
    entries = []  # (tag, type, values)

    def arr(vals, typ):
        fmt = {3: "H", 4: "I"}[typ]
        nonlocal body
        if len(vals) * (2 if typ == 3 else 4) <= 4:
            return None
        at = len(body)
        body += struct.pack(e + fmt * len(vals), *vals)
        return at

    entries.append((256, 4, [w]))
    entries.append((257, 4, [h]))
    entries.append((258, 3, [bits] * spp))
    entries.append((259, 3, [compression]))
    entries.append((262, 3, [photometric]))
    if not tile:
        entries.append((273, 4, offs))
    entries.append((277, 3, [spp]))
    if not tile:
        entries.append((278, 4, [rows_per_strip]))
        entries.append((279, 4, [len(x) for x in segs]))
    entries.append((284, 3, [planar]))
    if predictor != 1:
        entries.append((317, 3, [predictor]))
    if colormap is not None:
        cm = np.asarray(colormap, np.int64)
        entries.append((320, 3, list(cm[:, 0]) + list(cm[:, 1]) + list(cm[:, 2])))
    if tile:
        entries.append((322, 3, [tile[0]]))
        entries.append((323, 3, [tile[1]]))
        entries.append((324, 4, offs))
        entries.append((325, 4, [len(x) for x in segs]))
    if extra_samples is not None:
        entries.append((338, 3, [extra_samples]))
    laid = []
    for tag, typ, vals in sorted(entries):
        at = arr([int(v) for v in vals], typ)
        laid.append((tag, typ, [int(v) for v in vals], at))
    if len(body) % 2:
        body += b"\0"
    ifd = len(body)
    body[4:8] = struct.pack(e + "I", ifd)
    body += struct.pack(e + "H", len(laid))
    for tag, typ, vals, at in laid:
        if at is None:
            fmt = {3: "H", 4: "I"}[typ]
            v = struct.pack(e + fmt * len(vals), *vals).ljust(4, b"\0")
        else:
            v = struct.pack(e + "I", at)
        body += struct.pack(e + "HHI", tag, typ, len(vals)) + v
    body += b"\0\0\0\0"
    return bytes(body)


def decode_tiff(data: bytes) -> np.ndarray:
    """RGB of a TIFF as cv2.imread's 8-bit path sees it (libtiff's RGBA
    interface): Pillow's decode (libtiff 4.7.1 underneath for the compressed
    files), with libtiff's unassociated-alpha premultiplication
    ((v * a + 127) // 255, tif_getimage.c) applied to RGBA files whose
    ExtraSamples is 2 — that rule is parity unpinned."""
    import io
    from PIL import Image
    im = Image.open(io.BytesIO(data))
    im.load()
    extra = im.tag_v2.get(338)
    if im.mode == "RGBA" and (extra == 1 or extra == (1,)):
        # associated alpha: libtiff hands the stored (premultiplied) colours
        # through; Pillow un-premultiplies them, so it cannot be the checker
        raise NotImplementedError("associated-alpha TIFF: compare against the stored samples")
    if im.mode == "RGBA" and (extra == 2 or extra == (2,)):
        a = np.asarray(im).astype(np.uint32)
        return ((a[..., :3] * a[..., 3:4] + 127) // 255).astype(np.uint8)
    return np.asarray(im.convert("RGB")).copy()


# ----------------------------------------------------------------------------- GIF
def _gif_lzw_encode(idx: np.ndarray, min_size: int) -> bytes:
    """GIF LZW (LSB-first codes, a clear code first, width growing at 2^width)."""
    clear, eoi = 1 << min_size, (1 << min_size) + 1
    out, acc, nb = bytearray(), 0, 0
    width = min_size + 1

    def put(code):
        nonlocal acc, nb
        acc |= code << nb
        nb += width
        while nb >= 8:
            out.append(acc & 255)
            acc >>= 8
            nb -= 8

    table = {(i,): i for i in range(clear)}
    nxt = eoi + 1
    put(clear)
    w = ()
    for k in idx.reshape(-1).tolist():
        wk = w + (k,)
        if wk in table:
            w = wk
            continue
        put(table[w])
        if nxt < 4096:
            table[wk] = nxt
            nxt += 1
            if nxt > (1 << width) and width < 12:
                width += 1
        else:  # table full: start over
            put(clear)
            table = {(i,): i for i in range(clear)}
            nxt = eoi + 1
            width = min_size + 1
        w = (k,)
    if w:
        put(table[w])
    put(eoi)
    if nb:
        out.append(acc & 255)
    return bytes(out)


def encode_gif(idx: np.ndarray, palette: np.ndarray, screen=None, pos=(0, 0), transparent=None,
               interlace: bool = False, local_palette: bool = False) -> bytes:
    """A one-image GIF89a: (h, w) indices into `palette` ((2^k, 3) RGB), drawn
    at pos (x, y) on a screen (W, H) (default: the image's size)."""
    idx = np.asarray(idx, np.uint8)
    h, w = idx.shape
    W, H = screen or (w, h)
    pal = np.asarray(palette, np.uint8)
    k = max(1, int(np.ceil(np.log2(len(pal)))))
    table = np.zeros((1 << k, 3), np.uint8)
    table[:len(pal)] = pal
    min_size = max(2, k)
    rows = idx
    if interlace:
        order = list(range(0, h, 8)) + list(range(4, h, 8)) + list(range(2, h, 4)) + list(range(1, h, 2))
        rows = idx[order]
    out = bytearray(b"GIF89a" + struct.pack("<HH", W, H))
    if local_palette:
        out += bytes([0x00, 0, 0])
    else:
        out += bytes([0x80 | (k - 1), 0, 0]) + table.tobytes()
    if transparent is not None:
        out += bytes([0x21, 0xF9, 4, 1, 0, 0, transparent, 0])
    out += b"\x2c" + struct.pack("<HHHH", pos[0], pos[1], w, h)
    out += bytes([(0x80 | (k - 1) if local_palette else 0) | (0x40 if interlace else 0)])
    if local_palette:
        out += table.tobytes()
    data = _gif_lzw_encode(rows, min_size)
    out += bytes([min_size])
    for i in range(0, len(data), 255):
        blk = data[i:i + 255]
        out += bytes([len(blk)]) + blk
    out += b"\x00\x3b"
    return bytes(out)


def gif_expected(idx: np.ndarray, palette: np.ndarray, screen=None, pos=(0, 0), transparent=None) -> np.ndarray:
    """cv2.imread's first frame as restated (parity unpinned for transparency
    and partial frames): a black canvas, the image's palette colours drawn at
    pos, transparent pixels left black."""
    idx = np.asarray(idx, np.uint8)
    h, w = idx.shape
    W, H = screen or (w, h)
    pal = np.zeros((256, 3), np.uint8)
    pal[:len(palette)] = palette
    canvas = np.zeros((H, W, 3), np.uint8)
    x0, y0 = pos
    sub = idx[: max(0, min(h, H - y0)), : max(0, min(w, W - x0))]
    rgb = pal[sub]
    if transparent is not None:
        keep = sub != transparent
        region = canvas[y0:y0 + sub.shape[0], x0:x0 + sub.shape[1]]
        region[keep] = rgb[keep]
    else:
        canvas[y0:y0 + sub.shape[0], x0:x0 + sub.shape[1]] = rgb
    return canvas


def decode_rgb(data: bytes) -> np.ndarray:
    """The restatement for any of the formats."""
    if data[:8] == SIG:
        return decode_png(data)
    if data[:2] == b"BM":
        return decode_bmp(data)
    if data[:4] in (b"II*\x00", b"MM\x00*"):
        return decode_tiff(data)
    raise ValueError("not a PNG, BMP or TIFF file")


def pillow_rgb(data: bytes) -> np.ndarray:
    """Pillow 12.2.0's decode, alpha dropped / palette and gray expanded (the pin)."""
    import io
    from PIL import Image
    im = Image.open(io.BytesIO(data))
    im.load()
    return np.asarray(im.convert("RGB")).copy()
