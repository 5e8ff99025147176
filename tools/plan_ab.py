#!/usr/bin/env python3
"""One stage-plan variant on the bench's 25 x 8K JPEG batch (A/B helper).

    python tools/plan_ab.py --lib tools/variants/lib_x.so [--reps 4] [--ref /tmp/ref.json]

Encodes (once per box, cached under /tmp/wicca_plan_ab) the plan bench's 25
distinct 8K JPEG files, runs wicca_image_stage_plan_u8 (the demo's 4 shapes,
depths 2..6) `reps` times through the given library and prints the wall time
per call.  --ref: the SHA-256 of every output array is written there by the
first variant and compared by every later one (byte-identical outputs or exit
1), so kernel variants are checked against the in-tree product path.  Run it
under rocprofv3 --kernel-trace for the per-kernel times (tools/kstats.py).
"""
from __future__ import annotations

import argparse
import ctypes
import glob
import hashlib
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

SHAPES = [(224, 224), (331, 331), (299, 299), (240, 240)]


def blobs(n, H, W, quality=90):
    d = f"/tmp/wicca_plan_ab/{n}_{W}x{H}_q{quality}"
    paths = sorted(glob.glob(os.path.join(d, "*.jpg")))
    if len(paths) != n:
        os.makedirs(d, exist_ok=True)
        import bench

        class A:
            pass
        a = A()
        a.quality = quality
        for i, b in enumerate(bench.distinct_jpegs(a, n, H, W)):
            with open(os.path.join(d, f"{i:03d}.jpg"), "wb") as f:
                f.write(b)
        paths = sorted(glob.glob(os.path.join(d, "*.jpg")))
    return [open(p, "rb").read() for p in paths]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=os.path.join(REPO, "wicca_amd", "libwicca_hip.so"))
    ap.add_argument("--reps", type=int, default=4)
    ap.add_argument("--images", type=int, default=25)
    ap.add_argument("--height", type=int, default=4320)
    ap.add_argument("--width", type=int, default=7680)
    ap.add_argument("--depths", default="2,3,4,5,6")
    ap.add_argument("--ref", default=None)
    args = ap.parse_args()
    os.environ["WICCA_HIP_LIB"] = os.path.abspath(args.lib)
    from wicca_amd import _lib
    lib = _lib.load()
    B, H, W = args.images, args.height, args.width
    depths = [int(x) for x in args.depths.split(",")]
    data = blobs(B, H, W)
    keep = [np.frombuffer(b, np.uint8) for b in data]
    ptrs = (ctypes.c_void_p * B)(*[k.ctypes.data for k in keep])
    sizes = (ctypes.c_int64 * B)(*[k.size for k in keep])
    res = [_lib.pinned_empty((B, h, w, 3)) for (w, h) in SHAPES]
    ico = [[_lib.pinned_empty((B, h, w, 3)) for _ in depths] for (w, h) in SHAPES]
    c_shapes = (ctypes.c_int64 * 8)(*[v for sh in SHAPES for v in sh])
    c_depths = (ctypes.c_int * len(depths))(*depths)
    c_res = (ctypes.c_void_p * 4)(*[r.ctypes.data for r in res])
    c_ico = (ctypes.c_void_p * (4 * len(depths)))(*[a.ctypes.data for row in ico for a in row])

    def plan():
        _lib.check(lib.wicca_image_stage_plan_u8(ptrs, sizes, B, c_shapes, 4, c_depths, len(depths), 1, 0, 3,
                                                 c_res, c_ico, -1, None))
    plan()
    t = []
    for _ in range(args.reps):
        t0 = time.perf_counter()
        plan()
        t.append((time.perf_counter() - t0) * 1e3)
    h = {}
    for si, sh in enumerate(SHAPES):
        h[f"src{sh}"] = hashlib.sha256(res[si].tobytes()).hexdigest()
        for di, d in enumerate(depths):
            h[f"icon{sh}d{d}"] = hashlib.sha256(ico[si][di].tobytes()).hexdigest()
    same = None
    if args.ref:
        if os.path.exists(args.ref):
            ref = json.load(open(args.ref))
            bad = [k for k in ref if ref[k] != h.get(k)]
            same = not bad
        else:
            json.dump(h, open(args.ref, "w"))
            same, bad = True, []
    print(json.dumps({"lib": os.path.basename(args.lib), "ms": [round(x, 3) for x in t],
                      "median_ms": round(sorted(t)[len(t) // 2], 3), "identical_to_ref": same,
                      **({"differs": bad[:8]} if same is False else {})}), flush=True)
    if same is False:
        sys.exit(1)


if __name__ == "__main__":
    main()
