#!/bin/bash
# round 3 study: strong-scaling shards (bench --rehearse R/N) with round launches from 1 round of items on
# (NLDSC_ROUND_MIN=1: round launches + a K-split last round) vs the default (4 rounds; smaller bands K-split whole)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r3rm; mkdir -p $O
run() {  # <label> <rehearse> <round_min>
  NLDSC_ROUND_MIN=$3 NLDSC_DEBUG_TIMING=1 timeout -k 10 200 python bench.py --no-cpu --no-file --steps 20 --rehearse $2 > $O/$1.json 2> $O/$1.err || { tail $O/$1.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); s=d['stages_ms']
print('$1', round(d['ms_per_step'],3), s['band_ms'], s['count_ms'], d['roofline'].get('work_items'))"
}
for k in 1 2; do
for r in 0/8 3/8 1/4 1/2; do
  l=${r/\//of}
  run ${l}_def_$k $r 4 || exit 1
  run ${l}_rm1_$k $r 1 || exit 1
done
done
