"""Writes tests/golden/raster/: small PNG / BMP / TIFF files (every PNG
colour type family, Adam7, each filter, BMP palette / 16 / 24 / 32-bit,
top-down, RLE8 / RLE4, TIFF LZW / Deflate + predictor + tiles + big-endian /
PackBits / WhiteIsZero / unassociated alpha, binary PGM / PPM) and
cases.json with each file's expected RGB SHA-256 from Pillow 12.2.0 (the pin;
the parity-unpinned kinds, 16-bit gray PNG, 16-bit BMP and unassociated-alpha
TIFF, from the restatement oracle/raster_ref.py).  They seed the ASan/UBSan mutation fuzz
(tests/native/raster_fuzz.cpp) and are decoded on the GPU by
tests/test_gpu_raster.py::test_golden_files.

    python tests/golden/make_raster_seeds.py
"""
import hashlib
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from oracle import raster_ref as rr  # noqa: E402

OUT = os.path.join(os.path.dirname(__file__), "raster")


def samples(ct, bits, h, w, seed):
    rng = np.random.default_rng(seed)
    ch = rr.CHANNELS[ct]
    hi = 1 << bits
    s = rng.integers(0, hi, (h, w, ch), dtype=np.int64)
    s[: h // 2] = (np.arange(w)[None, :, None] * 5 + np.arange(h // 2)[:, None, None] * 3) % hi
    return s


def main():
    os.makedirs(OUT, exist_ok=True)
    files = {}
    files["rgb8_adam7.png"] = rr.encode_png(samples(2, 8, 23, 31, 1), 2, 8, interlace=True)
    files["rgb8_filters.png"] = rr.encode_png(samples(2, 8, 20, 17, 2), 2, 8, idat_split=64)
    pal = np.random.default_rng(3).integers(0, 256, (16, 3), dtype=np.uint8)
    files["pal4.png"] = rr.encode_png(samples(3, 4, 19, 27, 4), 3, 4, palette=pal)
    files["gray2_adam7.png"] = rr.encode_png(samples(0, 2, 13, 11, 5), 0, 2, interlace=True)
    files["gray16.png"] = rr.encode_png(samples(0, 16, 9, 14, 6), 0, 16)
    files["graya8.png"] = rr.encode_png(samples(4, 8, 12, 10, 7), 4, 8)
    files["rgba16_adam7.png"] = rr.encode_png(samples(6, 16, 11, 9, 8), 6, 16, interlace=True)
    rng = np.random.default_rng(9)
    img = rng.integers(0, 256, (15, 21, 3), dtype=np.uint8)
    files["bgr24.bmp"] = rr.encode_bmp(img, 24)
    files["bgrx32_topdown.bmp"] = rr.encode_bmp(img, 32, top_down=True)
    files["bgr565.bmp"] = rr.encode_bmp(img, 16, fields565=True)
    idx = rng.integers(0, 256, (14, 19), dtype=np.uint8)
    files["pal8.bmp"] = rr.encode_bmp(idx, 8, palette=rng.integers(0, 256, (256, 3), dtype=np.uint8))
    files["pal1_topdown.bmp"] = rr.encode_bmp(idx & 1, 1, palette=np.array([[10, 20, 30], [200, 100, 50]], np.uint8),
                                              top_down=True)
    from PIL import Image
    import io
    b = io.BytesIO()
    Image.fromarray(img).save(b, "TIFF", compression="tiff_lzw")
    files["rgb_lzw.tif"] = b.getvalue()
    gray = rng.integers(0, 256, (35, 33), dtype=np.uint8)
    files["gray_deflate_pred_tiled_be.tif"] = rr.encode_tiff(gray, 1, 8, 8, 2, tile=(16, 16), big_endian=True)
    cm = rng.integers(0, 256, (16, 3), dtype=np.int64) * 257
    files["pal4_packbits.tif"] = rr.encode_tiff(idx & 15, 3, 4, 32773, colormap=cm, rows_per_strip=5)
    files["white1.tif"] = rr.encode_tiff(idx & 1, 0, 1, 1)
    rgba = rng.integers(0, 256, (9, 11, 4), dtype=np.uint8)
    files["rgba_unassoc.tif"] = rr.encode_tiff(rgba, 2, 8, 8, extra_samples=2)
    gidx = rng.integers(0, 16, (13, 17), dtype=np.uint8)
    gpal = rng.integers(0, 256, (16, 3), dtype=np.uint8)
    files["full.gif"] = rr.encode_gif(gidx, gpal)
    files["partial_transparent_interlaced.gif"] = rr.encode_gif(gidx, gpal, screen=(25, 20), pos=(3, 4),
                                                                transparent=5, interlace=True)
    ridx = rng.integers(0, 256, (17, 23), dtype=np.uint8)
    ridx[:, :9] = ridx[:, :1]
    files["pal8_rle8.bmp"], _ = rr.encode_bmp_rle(ridx, rng.integers(0, 256, (256, 3), dtype=np.uint8))
    files["pal4_rle4_skips.bmp"], _ = rr.encode_bmp_rle(ridx & 15, rng.integers(0, 256, (16, 3), dtype=np.uint8),
                                                         rle4=True, skips=True)
    files["gray.pgm"] = rr.encode_pnm(rng.integers(0, 256, (9, 13), dtype=np.uint8))
    files["rgb.ppm"] = rr.encode_pnm(img, comment=False)
    cases = []
    for name, data in sorted(files.items()):
        with open(os.path.join(OUT, name), "wb") as f:
            f.write(data)
        unpinned = name in ("gray16.png", "bgr565.bmp", "rgba_unassoc.tif", "partial_transparent_interlaced.gif")
        if name.endswith(".gif"):
            rgb = (rr.gif_expected(gidx, gpal) if name == "full.gif" else
                   rr.gif_expected(gidx, gpal, screen=(25, 20), pos=(3, 4), transparent=5))
        elif name.endswith((".pgm", ".ppm")) or "_rle" in name:
            rgb = rr.pillow_rgb(data)
        else:
            rgb = rr.decode_rgb(data)
        if not unpinned:
            assert np.array_equal(rgb, rr.pillow_rgb(data)), name
        cases.append({"file": name, "height": int(rgb.shape[0]), "width": int(rgb.shape[1]),
                      "sha256_rgb": hashlib.sha256(rgb.tobytes()).hexdigest(),
                      "expected_from": "restatement (parity unpinned)" if unpinned else "Pillow 12.2.0"})
    with open(os.path.join(OUT, "cases.json"), "w") as f:
        json.dump({"cases": cases}, f, indent=1)


if __name__ == "__main__":
    main()
