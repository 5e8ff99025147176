#!/bin/bash
# rocprofv3 kernel trace + stats of any bench.py leg, summarised per kernel by
# tools/kstats.py.  Usage (GPU box): bash tools/profile_bench.sh <tag> <bench args...>
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1
shift
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -- \
    python3 "$R/bench.py" "$@" > "$OUT/bench.log" 2>&1
python3 "$R/tools/kstats.py" "$OUT/kt" > "$OUT/kstats.txt"
echo "profile $TAG done"
