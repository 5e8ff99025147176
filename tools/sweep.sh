#!/bin/bash
# Depth sweep of BASELINE configs[2] (128 x 8K RGB, D=1..6) and configs[1]
# (32 x 4K RGB, D=3) on one GPU.  Output: gpurun_out/sweep_<tag>.jsonl
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=${1:-r01}
OUT=$R/gpurun_out/sweep_$TAG.jsonl
: > "$OUT"
for D in 1 2 3 4 5 6; do
  timeout -k 10 200 python3 "$R/bench.py" --depth $D --steps 20 --warmup 3 --no-cpu-baseline >> "$OUT"
done
timeout -k 10 200 python3 "$R/bench.py" --depth 3 --images 32 --height 2160 --width 3840 \
    --steps 50 --warmup 5 --no-cpu-baseline >> "$OUT"
echo "sweep $TAG done"
