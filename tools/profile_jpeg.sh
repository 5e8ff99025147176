#!/bin/bash
# rocprofv3 kernel trace + stats of bench.py --config jpeg (GPU JPEG decode and
# the file-based caller stage), summarised per kernel by tools/kstats.py.
# Usage (on the GPU box): bash tools/profile_jpeg.sh <tag> [bench args...]
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=${1:-jpeg}
shift || true
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -- \
    python3 "$R/bench.py" --config jpeg --steps 5 --warmup 1 "$@" > "$OUT/bench.log" 2>&1
python3 "$R/tools/kstats.py" "$OUT/kt" --seq jpeg_sync > "$OUT/kstats.txt"
echo "profile $TAG done"
