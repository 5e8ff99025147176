"""The asynchronous stage plan's timeline (diagnostic, GPU box): the bench's
distinct 8K JPEG batches through get_img_matrix_async with one batch in
flight ahead (issue k+1, then wait k), each issue and wait timed; run under
rocprofv3 --kernel-trace --memory-copy-trace for the device side.
Usage: python tools/plan_async_probe.py [batches] [reps]"""
import argparse
import os
import shutil
import sys
import tempfile
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    import bench
    from wicca_amd import plan as P
    nb = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    args = argparse.Namespace(quality=90)
    B, H, W = 25, 4320, 7680
    depths = [2, 3, 4, 5, 6]
    shapes = list(dict.fromkeys(bench.DEMO_CLASSIFIERS))
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
        for paths in batches[:2]:
            P.get_img_matrix(paths, shapes, depths)  # warm: workspaces, pinned pool
        for ahead in (1, 2, 0):
            for rep in range(reps):
                log = []
                keep = []
                inflight = []
                t0 = time.perf_counter()
                for paths in batches:
                    t1 = time.perf_counter()
                    inflight.append(P.get_img_matrix_async(paths, shapes, depths))
                    t2 = time.perf_counter()
                    log.append(f"issue {1e3 * (t1 - t0):.1f}+{1e3 * (t2 - t1):.1f}")
                    while len(inflight) > ahead:
                        t3 = time.perf_counter()
                        keep.append(inflight.pop(0).wait())
                        log.append(f"wait {1e3 * (t3 - t0):.1f}+{1e3 * (time.perf_counter() - t3):.1f}")
                while inflight:
                    t3 = time.perf_counter()
                    keep.append(inflight.pop(0).wait())
                    log.append(f"wait {1e3 * (t3 - t0):.1f}+{1e3 * (time.perf_counter() - t3):.1f}")
                wall = time.perf_counter() - t0
                print(f"ahead {ahead} rep {rep}: {1e3 * wall / nb:.1f} ms per batch | " + " ".join(log), flush=True)
                del keep
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
