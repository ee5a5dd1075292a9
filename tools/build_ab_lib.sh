#!/bin/bash
# Build libnldsc_amd.so of another git revision (the engine sources and the C ABI header as committed there), or of
# the working tree (REV = WORKTREE) with extra compiler flags (e.g. -DNLDSC_SOME_VARIANT=1), into ab_libs/<name>.so,
# for same-box interleaved A/B timing against the working tree's library (tools/ab_libs.py).
#   bash tools/build_ab_lib.sh <git-rev | WORKTREE> <name> [extra hipcc flags...]
set -e
REV=$1; NAME=$2; shift 2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
W=$(mktemp -d /tmp/ablib.XXXXXX)
mkdir -p "$W/nldsc_amd/csrc" "$W/include" "$ROOT/ab_libs"
for f in ld_kernels.hip ld_kernels.h ld_engine.cpp band_plan.cpp band_plan.h tsv_format.cpp; do
  if [ "$REV" = WORKTREE ]; then cp "$ROOT/nldsc_amd/csrc/$f" "$W/nldsc_amd/csrc/$f"
  else git -C "$ROOT" show "$REV:nldsc_amd/csrc/$f" > "$W/nldsc_amd/csrc/$f"; fi
done
if [ "$REV" = WORKTREE ]; then cp "$ROOT/include/nldsc_ld.h" "$W/include/nldsc_ld.h"
else git -C "$ROOT" show "$REV:include/nldsc_ld.h" > "$W/include/nldsc_ld.h"; fi
cd "$W/nldsc_amd/csrc"
HIPCC=/opt/rocm/bin/hipcc
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-result $*"
$HIPCC $F -c ld_kernels.hip -o k.o &
$HIPCC $F -c ld_engine.cpp -o e.o &
g++ -O2 -std=c++17 -fPIC -c tsv_format.cpp -o t.o
g++ -O2 -std=c++17 -fPIC -c band_plan.cpp -o p.o
wait
$HIPCC --offload-arch=gfx950 -shared -fPIC k.o e.o t.o p.o -o "$ROOT/ab_libs/$NAME.so" -Wl,-rpath,/opt/rocm/lib
rm -rf "$W"
echo "built ab_libs/$NAME.so from $REV $*"
