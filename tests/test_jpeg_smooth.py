"""Damaged progressive JPEGs the way cv2.imread returns them, without a GPU.

The reference reads every file with ``cv2.imread`` (``/root/reference/wicca/
data_loader.py:53``): libjpeg-turbo at its defaults, through the stdio source
manager.  Two behaviours of that decoder matter for files cut short:

* interblock smoothing (``do_block_smoothing``, on by default; jdcoefct.c
  ``smoothing_ok`` / ``decompress_smooth_data``) of a progressive image whose
  first nine AC coefficients are not all final -- the host entropy decoder
  restates it (``jpeg_host.cpp`` ``block_smooth``);
* the fake EOI the stdio source manager feeds at the end of the file, so a cut
  inside a marker segment is read on from FF D9 FF D9 ... (mostly an error:
  imread returns None).

The checker is libjpeg-turbo 3.1.4.1 itself (Pillow) fed the same bytes
(``oracle.jpeg_pil.decode_rgb_imread``); the engine's coefficients are re-coded
as a sequential file and decoded by the same library, so the pixels compare
the coefficients (smoothed ones included) exactly.  No GPU."""
import numpy as np
import pytest

from oracle import jpeg_pil as J
from test_jpeg_host import host_coefs_as_libjpeg_pixels

# kind, subsampling (0 4:4:4, 1 4:2:2, 2 4:2:0), restart blocks, H, W
PROG = [("scene", 2, 0, 200, 344), ("smooth", 2, 16, 77, 131), ("scene", 1, 0, 45, 40),
        ("noise", 0, 0, 77, 131), ("gray", 0, 0, 200, 344), ("scene", 0, 3, 77, 131),
        ("smooth", 1, 0, 200, 344), ("scene", 2, 5, 45, 40), ("scene", 2, 0, 333, 517)]
CUTS = np.linspace(0.03, 0.999, 17)


def _engine(short, img, q, sub):
    try:
        return host_coefs_as_libjpeg_pixels(short, img, q, sub)
    except AssertionError:  # the engine refuses the file (wicca_jpeg_host_coefficients != 0)
        return None


@pytest.mark.parametrize("kind,sub,rb,H,W", PROG, ids=[f"{k}-s{s}-r{r}-{h}x{w}" for k, s, r, h, w in PROG])
def test_truncated_progressive_matches_imread(kind, sub, rb, H, W):
    """17 cuts through a progressive file (libjpeg-turbo's default script: DC
    first, AC first, refinements): the smoothed coefficients give libjpeg's
    pixels exactly; where libjpeg refuses the cut file, so does the engine."""
    img = J.test_image(kind, H, W, 17 + sub + rb)
    data = J.encode(img, 88, sub, rb, progressive=True)
    compared = 0
    for cut in CUTS:
        short = data[:int(len(data) * cut)]
        want = J.decode_rgb_imread(short)
        got = _engine(short, img, 88, sub)
        if want is None:
            assert got is None, cut
            continue
        assert got is not None, cut
        assert np.array_equal(got, want), cut
        compared += 1
    assert compared >= len(CUTS) // 2


def test_smoothing_changes_pixels_where_libjpeg_smooths():
    """The cases above are not vacuous: a progressive file cut after its DC
    scan is smoothed by libjpeg (the DC-only Gaussian kernel and the nine AC
    estimates), and the engine's answer differs from the plain coefficients'."""
    from jpeg_scans import coefficients, split_scans
    img = J.test_image("scene", 200, 344, 19)
    data = J.encode(img, 88, 2, progressive=True)
    sos = data.index(b"\xff\xda")
    start = sos + 2 + ((data[sos + 2] << 8) | data[sos + 3])
    end = next(i for i in range(start, len(data) - 1)
               if data[i] == 0xFF and data[i + 1] != 0 and not 0xD0 <= data[i + 1] <= 0xD7)
    short = data[:end - 10]  # inside the first (DC) scan's tail
    want = J.decode_rgb_imread(short)
    assert want is not None
    assert np.array_equal(host_coefs_as_libjpeg_pixels(short, img, 88, 2), want)
    # the same coefficients unsmoothed: re-code the first scan's DC values only
    base = J.encode(img, 88, 2)
    plain = coefficients(short, 0).reshape(-1, 64).copy()
    dc_only = np.zeros_like(plain)
    dc_only[:, 0] = plain[:, 0]
    assert not np.array_equal(J.decode_rgb(split_scans(base, dc_only.ravel())), want)


def _insert_before_second_sos(data: bytes, seg: bytes) -> bytes:
    sos = [i for i in range(len(data) - 1) if data[i] == 0xFF and data[i + 1] == 0xDA]
    return data[:sos[1]] + seg + data[sos[1]:]


def test_dqt_between_scans_is_not_latched():
    """libjpeg latches each component's quantisation table at its first scan
    (jdinput.c latch_quant_tables): a DQT redefining table 0 between scans
    changes nothing; the engine latches too."""
    img = J.test_image("smooth", 96, 128, 3)
    data = J.encode(img, 70, 2, progressive=True)
    dqt = b"\xff\xdb\x00\x43\x00" + bytes([1] * 64)
    odd = _insert_before_second_sos(data, dqt)
    want = J.decode_rgb_imread(odd)
    assert np.array_equal(want, J.decode_rgb(data))
    assert np.array_equal(host_coefs_as_libjpeg_pixels(odd, img, 70, 2), want)


@pytest.mark.parametrize("where", ["marker", "length", "index", "counts", "values-mid", "values-end", "sos-len",
                                   "sos-comps", "sos-params", "sos-complete"])
def test_cut_inside_a_segment_between_scans(where):
    """A progressive file cut inside the DHT or SOS segment that opens a later
    scan: libjpeg reads the rest of the segment from the fake EOIs (a table
    index 0xFF or 0xD9, counts past 256, an SOS of 255 components: error -- or
    a table whose last values are FF / D9, which no scan uses: the image); the
    engine gives None where libjpeg refuses, else the same pixels."""
    img = J.test_image("scene", 120, 160, 8)
    data = J.encode(img, 85, 2, progressive=True)
    sos = [i for i in range(len(data) - 1) if data[i] == 0xFF and data[i + 1] == 0xDA]
    dht = [i for i in range(sos[0], len(data) - 1) if data[i] == 0xFF and data[i + 1] == 0xC4]
    assert dht, "libjpeg-turbo's progressive files define tables between scans"
    d0 = dht[0]
    dlen = (data[d0 + 2] << 8) | data[d0 + 3]
    s1 = next(i for i in sos if i > d0)
    slen = (data[s1 + 2] << 8) | data[s1 + 3]
    cut = {"marker": d0 + 1, "length": d0 + 3, "index": d0 + 4, "counts": d0 + 10,
           "values-mid": d0 + 2 + dlen // 2 + 9, "values-end": d0 + 2 + dlen - 1,
           "sos-len": s1 + 3, "sos-comps": s1 + 5, "sos-params": s1 + 2 + slen - 2,
           "sos-complete": s1 + 2 + slen}[where]
    short = data[:cut]
    want = J.decode_rgb_imread(short)
    got = _engine(short, img, 85, 2)
    if want is None:
        assert got is None
    else:
        assert got is not None and np.array_equal(got, want)
