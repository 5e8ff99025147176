"""The JPEG data-loader loop alone (wicca_jpeg_decode_u8_async, one batch in
flight ahead), for a rocprofv3 --kernel-trace --memory-copy-trace timeline:

    rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d OUT -- \
        python3 tools/jpeg_pipeline_trace.py [batches]

then `python3 tools/jpeg_pipeline_trace.py --summarize OUT` prints, per batch,
the span of its kernels and copies and the device idle time between batches."""
import ctypes
import glob
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def run(batches: int):
    import torch
    from oracle import jpeg_pil
    from wicca_amd import _lib
    lib = _lib.load()
    B, H, W = 25, 4320, 7680
    distinct = [jpeg_pil.encode(jpeg_pil.test_image("scene", H, W, 40 + k), 90, 2) for k in range(4)]
    blobs = [distinct[i % 4] for i in range(B)]
    keep = [np.frombuffer(b, np.uint8) for b in blobs]
    ptrs = (ctypes.c_void_p * B)(*[k.ctypes.data for k in keep])
    sizes = (ctypes.c_int64 * B)(*[k.size for k in keep])
    pitch = (W * 3 + 127) // 128 * 128
    devs = [torch.empty(B * H * pitch, dtype=torch.uint8, device="cuda") for _ in range(2)]
    sets = [(ctypes.c_void_p * B)(*[d.data_ptr() + i * H * pitch for i in range(B)]) for d in devs]
    pitches = (ctypes.c_int64 * B)(*([pitch] * B))

    def issue(k):
        t = ctypes.c_int64(0)
        _lib.check(lib.wicca_jpeg_decode_u8_async(ptrs, sizes, B, sets[k % 2], pitches, 1, -1, ctypes.byref(t)))
        return t.value

    prev = issue(0)
    t0 = time.perf_counter()
    for k in range(1, batches):
        cur = issue(k)
        _lib.check(lib.wicca_jpeg_wait(prev))
        prev = cur
    _lib.check(lib.wicca_jpeg_wait(prev))
    print(f"{(time.perf_counter() - t0) / (batches - 1) * 1e3:.2f} ms per batch (wall, after the first)")


def summarize(root: str):
    import csv
    ev = []
    for pat, kind in (("*kernel_trace.csv", "K"), ("*memory_copy_trace.csv", "C")):
        for path in glob.glob(os.path.join(root, "**", pat), recursive=True):
            for r in csv.DictReader(open(path)):
                name = r.get("Kernel_Name") or r.get("Direction") or "copy"
                ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), kind, name[:40],
                           int(r.get("Bytes", 0) or 0)))
    ev.sort()
    t0 = ev[0][0]
    # kernel busy intervals merged; idle gaps longer than 50 us listed
    busy = []
    for s, e, k, n, b in ev:
        if k != "K":
            continue
        if busy and s <= busy[-1][1]:
            busy[-1][1] = max(busy[-1][1], e)
        else:
            busy.append([s, e])
    span = (busy[-1][1] - busy[0][0]) / 1e6
    kern = sum(e - s for s, e in busy) / 1e6
    print(f"kernel span {span:.2f} ms, kernels busy {kern:.2f} ms ({kern / span:.0%})")
    gaps = [(busy[i][0] - busy[i - 1][1]) / 1e3 for i in range(1, len(busy))]
    big = [(round((busy[i - 1][1] - t0) / 1e6, 2), round(g, 1)) for i, g in enumerate(gaps, 1) if g > 50]
    print("device idle gaps > 50 us (at ms, us):", big[:40])
    copies = [(s, e, b) for s, e, k, n, b in ev if k == "C" and b > 1 << 20]
    tot = sum(b for _, _, b in copies)
    cbusy = sum(e - s for s, e, _ in copies) / 1e6
    print(f"H2D/D2H copies > 1 MiB: {len(copies)}, {tot / 1e9:.2f} GB, busy {cbusy:.2f} ms")


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--summarize":
        summarize(sys.argv[2])
    else:
        run(int(sys.argv[1]) if len(sys.argv) > 1 else 8)
