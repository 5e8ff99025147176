"""Where the StagePlan loop's time goes (diagnostic, GPU box): the bench's
folder of distinct 8K JPEG batches, then
  1. get_img_matrix per batch back to back (no StagePlan),
  2. the ClassifierProcessor-shaped StagePlan loop with ahead = 0 and 2,
     each native computation timed (start, end) relative to the loop start.
Usage: python tools/plan_loop_probe.py [batches]"""
import argparse
import os
import shutil
import sys
import tempfile
import threading
import time
from concurrent.futures import ThreadPoolExecutor

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    import bench
    from wicca_amd import plan as P
    nb = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    args = argparse.Namespace(quality=90)
    B, H, W = 25, 4320, 7680
    depths = [2, 3, 4, 5, 6]
    blobs = bench.distinct_jpegs(args, nb * B, H, W)
    tmp = tempfile.mkdtemp(prefix="wicca_probe_", dir="/tmp")
    try:
        batches = []
        for b in range(nb):
            paths = []
            for i in range(B):
                p = os.path.join(tmp, f"{b:03d}_{i:03d}.jpg")
                with open(p, "wb") as f:
                    f.write(blobs[b * B + i])
                paths.append(p)
            batches.append(paths)
        shapes = list(dict.fromkeys(bench.DEMO_CLASSIFIERS))
        P.get_img_matrix(batches[0], shapes, depths)  # warm
        for rep in range(2):
            t = time.perf_counter()
            for paths in batches:
                t1 = time.perf_counter()
                P.get_img_matrix(paths, shapes, depths)
                print(f"  matrix {1e3 * (time.perf_counter() - t1):.1f} ms")
            print(f"back to back: {1e3 * (time.perf_counter() - t) / nb:.1f} ms per batch")
        for ahead in (0, 2, 0, 2):
            log = []
            lock = threading.Lock()
            sp = P.StagePlan(bench.DEMO_CLASSIFIERS, depths, batches=batches, ahead=ahead, copy=False)
            inner = sp._matrix

            def timed(*a, _inner=inner):
                t1 = time.perf_counter()
                r = _inner(*a)
                with lock:
                    log.append((t1 - t0, time.perf_counter() - t0))
                return r
            sp._matrix = timed
            t0 = time.perf_counter()
            for d in depths:
                def classify(shape):
                    for paths in batches:
                        sp.get_img_batch(paths, shape, d)
                with ThreadPoolExecutor(len(bench.DEMO_CLASSIFIERS)) as ex:
                    list(ex.map(classify, bench.DEMO_CLASSIFIERS))
                print(f"  ahead {ahead}: depth {d} done at {1e3 * (time.perf_counter() - t0):.1f} ms")
            wall = time.perf_counter() - t0
            sp.close()
            print(f"ahead {ahead}: {1e3 * wall / nb:.1f} ms per batch; computations (start, end) ms: " +
                  " ".join(f"({1e3 * a:.0f},{1e3 * b:.0f})" for a, b in sorted(log)))
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
