#!/bin/bash
# round 3: super-item tile shape of the quad plan (NLDSC_Q_TILE) on the C5 slice, one process, interleaved
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r3x; mkdir -p $O
timeout -k 10 600 python tools/ab_libs.py --libs t16x16=nldsc_amd/libnldsc_amd.so t4x8=nldsc_amd/libnldsc_amd.so,NLDSC_Q_TILE=4x8 t8x8=nldsc_amd/libnldsc_amd.so,NLDSC_Q_TILE=8x8 t2x16=nldsc_amd/libnldsc_amd.so,NLDSC_Q_TILE=2x16 --workload c5 --runs 6 \
  > $O/ab_qtile.json 2> $O/ab_qtile.err || { tail $O/ab_qtile.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/ab_qtile.json'))['ab']
for w,v in d.items(): print(w, {k:(round(x['band_ms_median'],2), round(x['band_ms_min'],2)) for k,x in v.items()})"
timeout -k 10 400 python tools/ab_libs.py --libs base=nldsc_amd/libnldsc_amd.so serial=nldsc_amd/libnldsc_amd.so,NLDSC_PLAN_SERIAL=1 --workload c2 c3 --runs 10 \
  > $O/ab_serial.json 2> $O/ab_serial.err || { tail $O/ab_serial.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/ab_serial.json'))['ab']
for w,v in d.items(): print(w, {k:(round(x['total_ms_median'],3), round(x['band_ms_median'],3)) for k,x in v.items()})"
