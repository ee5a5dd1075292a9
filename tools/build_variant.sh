#!/bin/bash
# Build an alternate libnldsc_amd.so with extra compile flags for tools/band_ab.py A/B runs:
#   tools/build_variant.sh ab_libs/vpm6.so -DNLDSC_F4_VPM=6
set -e
OUT=$1; shift
HERE=$(cd "$(dirname "$0")/.." && pwd)
TMP=$(mktemp -d)
mkdir -p "$(dirname "$OUT")"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 "$@" -c $HERE/nldsc_amd/csrc/ld_kernels.hip -o $TMP/k.o
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 "$@" -c $HERE/nldsc_amd/csrc/ld_engine.cpp -o $TMP/e.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $TMP/k.o $TMP/e.o -o "$OUT" -Wl,-rpath,/opt/rocm/lib -Wl,-soname,libnldsc_amd.so
rm -rf $TMP
