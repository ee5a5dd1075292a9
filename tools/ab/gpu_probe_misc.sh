#!/bin/bash
# (1) does ab_libs.py's second engine in a process pay extra host time? the same library three times, C2;
# (2) kernel timeline of the 1/8 shard on the current build
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-misc}; mkdir -p $O
timeout -k 10 300 python tools/ab_libs.py --libs a=ab_libs/r4_cur.so b=ab_libs/r4_cur.so c=ab_libs/r4_cur.so --workload c2 --runs 6 > $O/ab.json 2> $O/ab.err || { tail $O/ab.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1])['ab']
for w,v in d.items():
  for n,x in v.items(): print(w,n,round(x['total_ms_median'],3),round(x['band_ms_median'],3), x['stages_ms_median'])"
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d $O/p0 -o k --output-format csv -- python3 bench.py --no-cpu --no-file --steps 5 --rehearse 0/8 > $O/r0.json 2> $O/r0.err || { tail $O/r0.err; exit 1; }
find $O/p0 -name "*kernel_trace.csv" -exec cp {} $O/trace_r0.csv \;
find $O/p0 -name "*memory_copy_trace.csv" -exec cp {} $O/copy_r0.csv \;
