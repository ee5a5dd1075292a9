#!/bin/bash
# schedule tests + the 1/8 shard's step time and kernel timeline on the current build
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-shc}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -k "schedule or plan or ksplit or split_halo" --timeout 300 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for i in 1 2; do
timeout -k 10 200 python bench.py --no-cpu --no-file --steps 20 --rehearse 0/8 > $O/r0_$i.json 2> $O/r0_$i.err || { tail $O/r0_$i.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/r0_$i.json').read().strip().splitlines()[-1]); print('shard', round(d['ms_per_step'],3), d['stages_ms'])"
done
timeout -k 10 200 rocprofv3 --kernel-trace -d $O/p0 -o k --output-format csv -- python3 bench.py --no-cpu --no-file --steps 5 --rehearse 0/8 > $O/r0.json 2> $O/r0.err || { tail $O/r0.err; exit 1; }
find $O/p0 -name "*kernel_trace.csv" -exec cp {} $O/trace_r0.csv \;
