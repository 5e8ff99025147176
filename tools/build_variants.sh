#!/bin/bash
# Build tuning variants of libwicca_hip.so into tools/variants/ (run here, not on the box).
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
V=$R/tools/variants
mkdir -p "$V"
build() {  # name, extra flags
  local name=$1; shift
  local B=$V/build_$name
  mkdir -p "$B"
  local F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off"
  /opt/rocm/bin/hipcc $F "$@" -c "$R/wicca_amd/csrc/haar_ll.hip" -o "$B/haar_ll.o" &
  for m in haar_multi haar_multi_d12 haar_multi_d34 haar_multi_d57; do
    /opt/rocm/bin/hipcc $F "$@" -c "$R/wicca_amd/csrc/$m.hip" -o "$B/$m.o" &
  done
  /opt/rocm/bin/hipcc $F "$@" -c "$R/wicca_amd/csrc/resize.hip" -o "$B/resize.o" &
  /opt/rocm/bin/hipcc $F "$@" -c "$R/wicca_amd/csrc/stage.hip" -o "$B/stage.o" &
  /opt/rocm/bin/hipcc $F "$@" -c "$R/wicca_amd/csrc/jpeg.hip" -o "$B/jpeg.o" &
  /opt/rocm/bin/hipcc $F "$@" -x hip -c "$R/wicca_amd/csrc/jpeg_host.cpp" -o "$B/jpeg_host.o" &
  /opt/rocm/bin/hipcc $F "$@" -c "$R/wicca_amd/csrc/raster.hip" -o "$B/raster.o" &
  /opt/rocm/bin/hipcc $F "$@" -x hip -c "$R/wicca_amd/csrc/raster_host.cpp" -o "$B/raster_host.o" &
  g++ -O3 -std=c++17 -fPIC -c "$R/wicca_amd/csrc/inflate.cpp" -o "$B/inflate.o" &
  for c in capi capi_resize capi_jpeg capi_raster; do
    /opt/rocm/bin/hipcc $F "$@" -x hip -c "$R/wicca_amd/csrc/$c.cpp" -o "$B/$c.o" &
  done
  wait
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$V/lib_$name.so" "$B"/haar_ll.o "$B"/haar_multi*.o "$B/resize.o" "$B/stage.o" "$B/jpeg.o" "$B/jpeg_host.o" "$B/raster.o" "$B/raster_host.o" "$B/inflate.o" "$B"/capi*.o -lz
  rm -rf "$B"
}
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  [ "$name" = "$spec" ] && flags=""
  build "$name" $flags &
done
wait
ls -la "$V"
