#!/bin/bash
# Build tuning variants of libwicca_hip.so into tools/variants/ (run here, not
# on the box): each spec NAME[:FLAGS] is the in-tree Makefile's library built
# with extra compiler FLAGS (e.g. -DWICCA_JPEG_WRITE_S4=0) into lib_NAME.so.
# ONLY="stage jpeg": rebuild just those objects with FLAGS, the others are
# copied from the in-tree build (which must be current).
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
V=$R/tools/variants
mkdir -p "$V"
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  [ "$name" = "$spec" ] && flags=""
  if [ -n "${ONLY:-}" ]; then
    mkdir -p "$V/build_$name"
    cp -p "$R/wicca_amd/csrc/build/"*.o "$V/build_$name/"
    for o in $ONLY; do rm -f "$V/build_$name/$o.o"; done
  fi
  make -s -C "$R/wicca_amd/csrc" -j8 OBJ="$V/build_$name" OUT="$V/lib_$name.so" EXTRA="$flags"
  rm -rf "$V/build_$name"
done
ls -la "$V"
