#!/bin/bash
# HBM traffic of the PNG / BMP / TIFF conversion kernel: two rocprofv3 PMC
# passes (FETCH_SIZE, WRITE_SIZE: separate runs) over `bench.py --config bmp`,
# per-dispatch bytes with bench.py's gfx950 correction (pmc_hbm_bytes).
# Usage (GPU box): bash tools/pmc_raster.sh <tag>
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d "$OUT/$C" -- \
        python3 "$R/bench.py" --config bmp --steps 2 --warmup 0 --no-verify --no-cpu-baseline > "$OUT/bench_$C.log" 2>&1
done
python3 - "$OUT" "$R" <<'PY'
import sys
sys.path.insert(0, sys.argv[2])
import bench
import csv, glob, os
out = sys.argv[1]
vals = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    acc, n = 0.0, set()
    for path in glob.glob(os.path.join(out, c, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            if "raster_convert_kernel" in r["Kernel_Name"] and r["Counter_Name"] == c:
                acc += float(r["Counter_Value"])
                n.add(r["Dispatch_Id"])
    vals[c] = acc / max(1, len(n))
    print(f"{c}: {vals[c]:.1f} KiB per dispatch ({len(n)} dispatches)")
b = bench.pmc_hbm_bytes(vals["FETCH_SIZE"], vals["WRITE_SIZE"])
alg = 25 * 7680 * 4320 * 3 * 2
print(f"HBM bytes per dispatch {b}; algorithmic {alg} (rows in + RGB out); "
      f"ratio {b['hbm_bytes_per_launch'] / alg:.4f}")
PY
echo "pmc $TAG done"
