#!/bin/bash
# On the GPU box: --config multi (K5) for each tools/variants/lib_*.so, interleaved rounds.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
DEPTHS=${DEPTHS:-"2,3,4,5,6"}
ROUNDS=${ROUNDS:-2}
OUT=$R/gpurun_out/ab_multi${TAG:+_$TAG}.jsonl
: > "$OUT"
for round in $(seq $ROUNDS); do
  for lib in "$@"; do
    line=$(WICCA_HIP_LIB=$lib timeout -k 10 120 python3 "$R/bench.py" --config multi --depths "$DEPTHS" --steps 10 --warmup 3 --no-cpu-baseline --no-verify)
    echo "{\"lib\": \"$(basename "$lib")\", \"round\": $round, \"bench\": $line}" >> "$OUT"
  done
done
echo "ab_multi done"
