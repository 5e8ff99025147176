#!/bin/bash
# On the GPU box: bench every tools/variants/lib_*.so at the given depths,
# interleaved rounds in separate processes.  Output gpurun_out/variants_<tag>.jsonl
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1; shift
DEPTHS=${DEPTHS:-"1 3 5"}
ROUNDS=${ROUNDS:-2}
OUT=$R/gpurun_out/variants_$TAG.jsonl
: > "$OUT"
for round in $(seq $ROUNDS); do
  for lib in "$R"/tools/variants/lib_*.so; do
    for D in $DEPTHS; do
      name=$(basename "$lib" .so)
      line=$(WICCA_HIP_LIB=$lib timeout -k 10 120 python3 "$R/bench.py" --depth $D --steps 20 --warmup 3 --no-cpu-baseline --no-verify "$@")
      echo "{\"variant\": \"$name\", \"round\": $round, \"bench\": $line}" >> "$OUT"
    done
  done
done
echo "variants $TAG done"
