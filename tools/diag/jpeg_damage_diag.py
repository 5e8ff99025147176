"""GPU decode of damaged JPEG files vs libjpeg-turbo's (Pillow, LOAD_TRUNCATED_IMAGES):
where they differ (diagnostic for tests/test_gpu_jpeg.py's damage cases)."""
import sys
import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
from oracle import jpeg_pil as J
from wicca_amd import jpeg as WJ


def report(tag, got, want):
    d = np.any(got != want, axis=2)
    if not d.any():
        print(tag, "EQUAL")
        return
    ys, xs = np.nonzero(d)
    print(tag, "diff px", int(d.sum()), "rows", ys.min(), ys.max(), "cols", xs.min(), xs.max())
    y, x = ys[0], xs[0]
    print("   first diff at", (y, x), "got", got[y, x:x + 4].tolist(), "want", want[y, x:x + 4].tolist())
    # rows entirely grey in each
    gg = [r for r in range(got.shape[0]) if (got[r] == 128).all()]
    wg = [r for r in range(want.shape[0]) if (want[r] == 128).all()]
    print("   grey rows got from", gg[0] if gg else None, "want from", wg[0] if wg else None)


for kind, sub, rb, prog in [("scene", 2, 0, False), ("scene", 1, 3, False), ("gray", 0, 0, False),
                            ("scene", 2, 8, False)]:
    img = J.test_image(kind, 200, 344, 17 + sub + rb)
    if kind == "gray":
        img = img[..., 0] if img.ndim == 3 else img
    data = J.encode(img, 88, sub, rb, progressive=prog)
    for cut in (0.3, 0.5):
        short = data[:int(len(data) * cut)]
        report(f"{kind} s{sub} r{rb} p{int(prog)} cut{cut}", WJ.decode(short), J.decode_rgb(short, truncated=True))
