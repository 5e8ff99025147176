#!/bin/bash
# One rocprofv3 PMC pass over any bench.py leg (per-kernel counter sums by
# tools/pmc_kernels.py).  Usage (GPU box): bash tools/pmc_bench.sh <tag> "<counters>" <bench args...>
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1
CNT=$2
shift 2
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc $CNT --output-format csv -d "$OUT/raw" -- \
    python3 "$R/bench.py" "$@" > "$OUT/bench.log" 2>&1
python3 "$R/tools/pmc_kernels.py" "$OUT/raw" > "$OUT/summary.txt"
echo "pmc $TAG done"
