"""Writes tests/golden/jpeg/: small JPEG files from Pillow's libjpeg-turbo
encoder and the SHA-256 of Pillow's RGB decode of each (the checker of the GPU
decoder, oracle/jpeg_pil.py).  Run from the repo root:
    python tests/golden/make_jpeg_golden.py
"""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from oracle import jpeg_pil as J  # noqa: E402

CASES = [
    # name, kind, H, W, quality, subsampling, restart_blocks, restart_rows, optimize, orientation
    ("scene_420_q75", "scene", 96, 128, 75, 2, 0, 0, False, 1),
    ("scene_422_q90", "scene", 61, 83, 90, 1, 0, 0, False, 1),
    ("scene_444_q95", "scene", 33, 47, 95, 0, 0, 0, True, 1),
    ("noise_420_q100", "noise", 40, 56, 100, 2, 0, 0, False, 1),
    ("smooth_420_q30", "smooth", 120, 90, 30, 2, 0, 0, True, 1),
    ("scene_420_rst3", "scene", 100, 150, 80, 2, 3, 0, False, 1),
    ("scene_444_rstrow", "scene", 70, 70, 85, 0, 0, 1, False, 1),
    ("gray_q80", "gray", 77, 101, 80, 0, 0, 0, False, 1),
    ("gray_rst1", "gray", 24, 40, 60, 0, 1, 0, False, 1),
    ("scene_420_orient6", "scene", 48, 80, 75, 2, 0, 0, False, 6),
    ("scene_420_orient3", "scene", 50, 66, 75, 2, 0, 0, False, 3),
    ("tiny_3x5", "scene", 3, 5, 90, 2, 0, 0, False, 1),
]
# progressive (SOF2: libjpeg's default progression, DC and AC first and
# refinement scans) - decoded by the host entropy decoder + device back end
PROGRESSIVE = [
    ("prog_scene_420_q80", "scene", 90, 122, 80, 2, 0, 0, False, 1),
    ("prog_scene_444_rst2", "scene", 57, 75, 90, 0, 2, 0, False, 1),
    ("prog_gray_q70", "gray", 41, 66, 70, 0, 0, 0, False, 1),
    ("prog_smooth_422_orient8", "smooth", 64, 40, 85, 1, 0, 0, True, 8),
]


def main():
    out = os.path.join(HERE, "jpeg")
    os.makedirs(out, exist_ok=True)
    meta = {"libjpeg_turbo": J.libjpeg_version(), "cases": []}
    for i, (name, kind, H, W, q, sub, rb, rr, opt, orient) in enumerate(CASES + PROGRESSIVE):
        img = J.test_image(kind, H, W, 1000 + i)
        data = J.encode(img, q, sub, rb, rr, opt, orientation=orient, progressive=i >= len(CASES))
        with open(os.path.join(out, name + ".jpg"), "wb") as f:
            f.write(data)
        rgb = J.decode_rgb(data)
        meta["cases"].append({"name": name, "file": name + ".jpg", "height": rgb.shape[0],
                              "width": rgb.shape[1], "orientation": orient,
                              "sha256_rgb": hashlib.sha256(rgb.tobytes()).hexdigest()})
    with open(os.path.join(out, "cases.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print(f"{len(CASES) + len(PROGRESSIVE)} cases, libjpeg-turbo {meta['libjpeg_turbo']}")


if __name__ == "__main__":
    main()
