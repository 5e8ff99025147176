"""Per-kernel summary of a rocprofv3 --kernel-trace directory: launches,
average / median / min duration per (kernel, grid), sorted by total time.
Usage: python tools/kstats.py <rocprofv3 output dir> [--seq SUBSTRING]
(--seq: also the durations of the kernels whose name contains SUBSTRING, in
dispatch order, e.g. the JPEG sync passes of each call.)"""
import collections
import csv
import glob
import os
import statistics
import sys


def main(root, seq=None):
    groups = collections.defaultdict(list)
    order = []
    for path in glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True):
        with open(path) as f:
            for r in csv.DictReader(f):
                grid = "x".join(r[c] for c in sorted(r) if c.startswith("Grid_Size") and r[c])
                d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
                groups[(r["Kernel_Name"], grid)].append(d)
                if seq and seq in r["Kernel_Name"]:
                    order.append((int(r["Start_Timestamp"]), d))
    rows = sorted(groups.items(), key=lambda kv: -sum(kv[1]))
    print(f"{'total_ms':>9} {'n':>5} {'avg_us':>9} {'med_us':>9} {'min_us':>9}  kernel [grid]")
    for (name, grid), d in rows:
        print(f"{sum(d) / 1e6:9.3f} {len(d):5d} {statistics.mean(d) / 1e3:9.1f} {statistics.median(d) / 1e3:9.1f} "
              f"{min(d) / 1e3:9.1f}  {name[:90]} [{grid}]")
    if seq:
        print(f"\n{seq} in dispatch order (us):")
        print(" ".join(f"{d / 1e3:.0f}" for _, d in sorted(order)))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[3] if len(sys.argv) > 3 and sys.argv[2] == "--seq" else None)
