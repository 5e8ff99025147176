"""JPEG decode checker — TEST INFRASTRUCTURE.

The reference decodes with ``cv2.imread`` (opencv-python 4.12.0.88,
``requirements.txt:91``), i.e. libjpeg-turbo at its defaults (ISLOW integer
IDCT, fancy upsampling, integer YCbCr -> RGB), followed by ``cvtColor(BGR2RGB)``
(``/root/reference/wicca/data_loader.py:53-58``).  cv2 is absent here; Pillow
12.2.0 is present and bundles libjpeg-turbo 3.1.4.1 with the same defaults
(``dct_method`` ISLOW unless draft mode, ``do_fancy_upsampling`` on,
``JCS_RGB`` output), so its decode is the checker for the GPU decoder
(``wicca_amd/csrc/jpeg.hip``): parity is pinned to libjpeg-turbo 3.1.4.1 via
Pillow, not to an OpenCV binary.  EXIF orientation is applied with
``ImageOps.exif_transpose`` (cv2.imread's IMREAD_COLOR applies it too).
Only ``tests/`` and the golden-fixture script use this module.
"""
from __future__ import annotations

import io

import numpy as np


def libjpeg_version() -> str:
    from PIL import features
    return str(features.version("libjpeg_turbo"))


def decode_rgb(data: bytes, apply_orientation: bool = True, truncated: bool = False) -> np.ndarray:
    """RGB (H, W, 3) uint8 decode of a JPEG file's bytes.

    truncated=True: Pillow's ``ImageFile.LOAD_TRUNCATED_IMAGES`` — at the end
    of the data libjpeg-turbo gets a fake EOI marker and finishes the image
    with its "insufficient data" rule (missing blocks are all-zero, i.e. grey),
    the same source-manager behaviour ``cv2.imread`` has on a damaged file
    (libjpeg warns and returns the image)."""
    from PIL import Image, ImageFile, ImageOps
    prev = ImageFile.LOAD_TRUNCATED_IMAGES
    ImageFile.LOAD_TRUNCATED_IMAGES = truncated
    try:
        im = Image.open(io.BytesIO(data))
        im.load()
    finally:
        ImageFile.LOAD_TRUNCATED_IMAGES = prev
    if apply_orientation:
        im = ImageOps.exif_transpose(im)
    if im.mode == "CMYK":
        return cmyk_to_rgb_imread(np.asarray(im))
    return np.asarray(im.convert("RGB")).copy()


def cmyk_to_rgb_imread(cmyk: np.ndarray) -> np.ndarray:
    """What ``cv2.imread`` + ``cvtColor(BGR2RGB)`` makes of a four-component
    JPEG whose libjpeg-turbo CMYK output Pillow returned as ``cmyk``.

    Pillow reads every CMYK JPEG as rawmode ``CMYK;I`` ("assume adobe
    conventions", JpegImagePlugin.py), so libjpeg's own output is ``255 -
    cmyk``.  OpenCV's JpegDecoder asks libjpeg for JCS_CMYK and converts each
    pixel with ``icvCvt_CMYK2BGR_8u_C4C3R``: c = k - ((255 - c) * k >> 8),
    likewise m and y, BGR = (y, m, c), i.e. RGB = (c, m, y).  Restated from
    OpenCV's published source (cv2 is absent here): this last step is parity
    unpinned; libjpeg's CMYK / YCCK decode before it is pinned through
    Pillow."""
    raw = 255 - cmyk.astype(np.int32)
    k = raw[..., 3:4]
    return (k - (((255 - raw[..., :3]) * k) >> 8)).astype(np.uint8)


_FAKE_EOI_TAIL = b"\xff\xd9" * 32769  # covers a 65535-byte marker segment read from the tail


def decode_rgb_imread(data: bytes) -> np.ndarray | None:
    """What ``cv2.imread`` returns for a file's bytes, damaged ones included:
    OpenCV reads files through libjpeg's stdio source manager, whose
    ``fill_input_buffer`` (jdatasrc.c) hands the decoder a fake EOI (FF D9)
    every time the file has no more bytes -- so a file cut inside a marker
    segment is read on from FF D9 FF D9 ... (mostly a libjpeg error: imread
    gives None), and a file cut inside entropy-coded data ends at an EOI.
    Restated by feeding Pillow's libjpeg-turbo the bytes followed by that
    tail (Pillow's own LOAD_TRUNCATED_IMAGES appends ONE EOI, and a decoder
    that suspends inside a segment leaves a black image instead).  None where
    libjpeg refuses the file."""
    try:
        return decode_rgb(bytes(data) + _FAKE_EOI_TAIL)
    except Exception:  # noqa: BLE001 -- libjpeg error_exit: imread returns an empty Mat
        return None


def encode(img: np.ndarray, quality: int = 75, subsampling: int = 2, restart_blocks: int = 0,
           restart_rows: int = 0, optimize: bool = False, progressive: bool = False,
           orientation: int = 1) -> bytes:
    """JPEG bytes of an (H, W, 3) RGB or (H, W) gray uint8 array (libjpeg-turbo encoder)."""
    from PIL import Image
    im = Image.fromarray(img)
    kw = dict(quality=quality, optimize=optimize, progressive=progressive)
    if img.ndim == 3:
        kw["subsampling"] = subsampling
    if restart_blocks:
        kw["restart_marker_blocks"] = restart_blocks
    if restart_rows:
        kw["restart_marker_rows"] = restart_rows
    if orientation != 1:
        ex = Image.Exif()
        ex[0x0112] = orientation
        kw["exif"] = ex.tobytes()
    b = io.BytesIO()
    im.save(b, "JPEG", **kw)
    return b.getvalue()


def test_image(kind: str, H: int, W: int, seed: int) -> np.ndarray:
    """Deterministic content: 'noise' (long Huffman codes), 'smooth' (many EOBs),
    'scene' (blobs + edges + noise), 'gray' (2-D)."""
    rng = np.random.default_rng(seed)
    if kind == "noise":
        return rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
    y, x = np.mgrid[0:H, 0:W].astype(np.float64)
    if kind == "smooth":
        r = 127 + 120 * np.sin(x / max(W, 1) * 3.1 + 0.3)
        g = 127 + 120 * np.cos(y / max(H, 1) * 2.3)
        b = 127 + 100 * np.sin((x + y) / max(H + W, 1) * 5.0)
        return np.clip(np.stack([r, g, b], -1), 0, 255).astype(np.uint8)
    base = np.zeros((H, W, 3))
    for _ in range(6):
        cx, cy = rng.uniform(0, W), rng.uniform(0, H)
        rad = rng.uniform(0.05, 0.4) * max(H, W)
        col = rng.uniform(0, 255, 3)
        m = ((x - cx) ** 2 + (y - cy) ** 2) < rad ** 2
        base[m] = 0.5 * base[m] + 0.5 * col
    base += rng.normal(0, 12, base.shape)
    img = np.clip(base, 0, 255).astype(np.uint8)
    return img[:, :, 0] if kind == "gray" else img
