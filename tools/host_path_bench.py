#!/usr/bin/env python3
"""Host-array (PCIe-inclusive) throughput of the drop-in path.

Times HaarCoder.get_small_copy / get_small_copies on numpy images that live
in host memory — exactly what ClassifierProcessor._get_img_batch passes
(classifying_tools.py:317) — single-threaded, from a thread pool, and as a
ragged batch.  Prints one JSON line per measurement.
"""
from __future__ import annotations

import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    import numpy as np

    from wicca_amd import HaarCoder
    from wicca_amd.synth import synth_image

    D = int(os.environ.get("DEPTH", "5"))
    H, W, C = 4320, 7680, 3
    imgs = [synth_image(7, i, H, W, C) for i in range(16)]
    coder = HaarCoder()
    coder.get_small_copy(imgs[0], D)  # warm (workspace allocation)
    mb = H * W * C / 1e6

    def rec(name, n, secs):
        print(json.dumps({"case": name, "images": n, "ms_per_image": round(secs / n * 1e3, 3),
                          "MP_per_s": round(n * H * W / 1e6 / secs, 1),
                          "GB_per_s_h2d": round(n * mb / 1e3 / secs, 2),
                          "mode": os.environ.get("WICCA_H2D", "default")}), flush=True)

    t0 = time.perf_counter()
    for im in imgs:
        coder.get_small_copy(im, D)
    rec("single_thread", len(imgs), time.perf_counter() - t0)

    for threads in (4, 8, 16):
        with ThreadPoolExecutor(threads) as ex:
            list(ex.map(lambda im: coder.get_small_copy(im, D), imgs[:threads]))
            t0 = time.perf_counter()
            list(ex.map(lambda im: coder.get_small_copy(im, D), imgs * 2))
            rec(f"threads_{threads}", 2 * len(imgs), time.perf_counter() - t0)

    coder.get_small_copies(imgs[:4], D)
    t0 = time.perf_counter()
    coder.get_small_copies(imgs, D)
    rec("ragged_batch_call", len(imgs), time.perf_counter() - t0)

    # raw PCIe reference: torch pageable and pinned copies of the same bytes
    try:
        import torch
        x = torch.from_numpy(imgs[0])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(8):
            x.cuda()
        torch.cuda.synchronize()
        rec("torch_pageable_h2d", 8, time.perf_counter() - t0)
        xp = x.pin_memory()
        t0 = time.perf_counter()
        for _ in range(8):
            xp.cuda(non_blocking=True)
        torch.cuda.synchronize()
        rec("torch_pinned_h2d", 8, time.perf_counter() - t0)
    except Exception as e:  # pragma: no cover
        print(json.dumps({"case": "torch_reference", "error": repr(e)}))
    ok = all(np.array_equal(coder.get_small_copy(im, D), coder.get_small_copies([im], D)[0])
             for im in imgs[:2])
    print(json.dumps({"case": "consistency", "ok": ok}))


if __name__ == "__main__":
    main()
