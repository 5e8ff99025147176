#!/bin/bash
# rocprofv3 evidence for bench.py's dominant kernel (run on the GPU box):
#   1. kernel trace + stats (durations),
#   2. PMC pass FETCH_SIZE, 3. PMC pass WRITE_SIZE (separate passes; gfx950
#      TCC slots cannot hold both), then tools/pmc_summary.py -> profiles/.
# Usage: bash tools/profile_gpu.sh <tag> [bench args...]
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=${1:-r01}
shift || true
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
ARGS="--no-cpu-baseline --no-live-pmc $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -- \
    python3 "$R/bench.py" --steps 20 --warmup 3 $ARGS > "$OUT/bench_kt.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -- \
    python3 "$R/bench.py" --steps 5 --warmup 1 --no-verify $ARGS > "$OUT/bench_fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -- \
    python3 "$R/bench.py" --steps 5 --warmup 1 --no-verify $ARGS > "$OUT/bench_write.log" 2>&1
python3 "$R/tools/pmc_summary.py" "$OUT" > "$OUT/summary.json"
echo "profile $TAG done"
