#!/bin/bash
# Same-box A/B of study builds (tools/build_ab_lib.sh WORKTREE <name> -D...): gpurun --timeout 900 -- bash tools/gpu_r6_ab.sh <tag> "<wl>:<lib>,<lib>" ...
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=$1; shift
O=gpurun_out/$T; mkdir -p $O
for spec in "$@"; do
  wl=${spec%%:*}; libs=${spec#*:}
  L=""
  for n in ${libs//,/ }; do
    if [ "$n" = tree ]; then L="$L tree=nldsc_amd/libnldsc_amd.so"; else L="$L $n=ab_libs/$n.so"; fi
  done
  echo "[$(date +%H:%M:%S)] $wl:$L"
  timeout -k 10 400 python tools/ab_libs.py --libs $L --workload $wl --runs 10 > $O/ab_$wl.json 2> $O/ab_$wl.err || { tail $O/ab_$wl.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/ab_$wl.json').read())['ab']['$wl']
for k,v in d.items(): print('  ', k, round(v['band_ms_median'],4), round(v['total_ms_median'],4), v['band_kernel'])"
done
echo "[$(date +%H:%M:%S)] done"
