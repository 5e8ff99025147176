"""Average PMC counter value per dispatch, per kernel, of a rocprofv3 --pmc
run (counter_collection.csv).  Usage: python tools/pmc_kernels.py <dir>"""
import collections
import csv
import glob
import os
import sys


def main(root):
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for path in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for r in csv.DictReader(f):
                k = r["Kernel_Name"][:70]
                acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
                disp[k].add(r["Dispatch_Id"])
    for k, cs in sorted(acc.items(), key=lambda kv: -max(kv[1].values())):
        n = len(disp[k])
        print(f"{k}  ({n} dispatches)")
        for c, v in sorted(cs.items()):
            print(f"    {c:24s} {v / n:16.4g}")


if __name__ == "__main__":
    main(sys.argv[1])
