#!/bin/bash
# A/B of JPEG decode variants on the GPU box: for each spec NAME[:ENV=VAL,...]
# (NAME = a tools/variants/lib_NAME.so or "cur" for the in-tree library) one
# stats run (WICCA_JPEG_TIMING) and one rocprofv3 kernel trace of the jpeg bench.
# AB_ARGS: extra bench.py arguments (e.g. --no-verify for timing-only ablations).
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
for spec in "$@"; do
  name=${spec%%:*}; envs=""
  [ "$name" != "$spec" ] && envs=${spec#*:}
  lib=$R/wicca_amd/libwicca_hip.so
  [ "$name" != "cur" ] && lib=$R/tools/variants/lib_${name%%+*}.so
  tag=$(echo "$spec" | tr ':,=/' '____')
  (
    export WICCA_HIP_LIB=$lib
    for kv in ${envs//,/ }; do export "$kv"; done
    WICCA_JPEG_TIMING=1 timeout -k 10 200 python3 "$R/bench.py" --config jpeg --steps 2 --warmup 1 ${AB_ARGS:-} \
      > "$R/gpurun_out/ab_$tag.out" 2> "$R/gpurun_out/ab_$tag.err"
    bash "$R/tools/profile_jpeg.sh" "ab_$tag" ${AB_ARGS:-} > /dev/null 2>&1
  )
  echo "$spec done"
done
