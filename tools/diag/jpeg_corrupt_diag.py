"""GPU decode of the corrupted-entropy test files (tests/test_gpu_jpeg.py
test_corrupted_entropy_whole_decode_matches_libjpeg) against libjpeg-turbo's
(Pillow) and against the host entropy decoder's coefficients; set
WICCA_JPEG_TIMING=1 to see whether the device flagged the file damaged."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests"))
import numpy as np
from oracle import jpeg_pil as J
from wicca_amd import jpeg as WJ
from test_jpeg_host import host_coefs_as_libjpeg_pixels


def corrupted(seed):
    rng = np.random.default_rng(100 + seed)
    kind = ("scene", "noise", "smooth")[seed % 3]
    img = J.test_image(kind, 160, 232, seed)
    data = bytearray(J.encode(img, 80, seed % 3, 8 if seed % 2 else 0))
    sos = bytes(data).index(b"\xff\xda")
    start = sos + 2 + int.from_bytes(data[sos + 2:sos + 4], "big")
    flips = []
    for pos in rng.integers(start + 4, len(data) - 4, 3 + seed):
        if data[pos] != 0xFF and data[pos - 1] != 0xFF:
            nv = data[pos] ^ int(rng.integers(1, 255))
            if nv != 0xFF:
                flips.append((int(pos), data[pos], nv))
                data[pos] = nv
    return bytes(data), img, seed % 3, flips


for seed in [int(a) for a in sys.argv[1:]] or range(6):
    data, img, sub, flips = corrupted(seed)
    want = J.decode_rgb(data, truncated=True)
    got = WJ.decode(data)
    hc = host_coefs_as_libjpeg_pixels(data, img, 80, sub)
    d = np.any(got != want, axis=2)
    print(f"seed {seed} sub {sub} flips {flips} host==pillow {np.array_equal(hc, want)} device==pillow "
          f"{not d.any()} device==host {np.array_equal(got, hc)}", flush=True)
    if d.any():
        ys, xs = np.nonzero(d)
        print("   diff px", int(d.sum()), "rows", ys.min(), ys.max(), "cols", xs.min(), xs.max(),
              "first", (int(ys[0]), int(xs[0])), got[ys[0], xs[0]].tolist(), want[ys[0], xs[0]].tolist())
