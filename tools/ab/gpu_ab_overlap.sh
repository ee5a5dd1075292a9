#!/bin/bash
# count-free pipeline check: its bitwise tests + the round-launch / K-split / rare-variant tests around it, then
# a same-box A/B of the C3 bench (count pass vs count-free) and the 1/8 rehearsal
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-cfree}
mkdir -p $O
step() { echo "[$(date +%H:%M:%S)] $*"; }
step tests
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
  -k "count_overlap or round_launch or ksplit or deferred or rare or full_size" > $O/tests.log 2>&1 || { echo tests failed; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
step ab
for k in 1 2; do
  NLDSC_COUNT_OVERLAP=0 timeout -k 10 200 python bench.py --no-cpu --no-file --steps 10 > $O/c3_count_$k.json 2> $O/ab.err || { tail $O/ab.err; exit 1; }
  timeout -k 10 200 python bench.py --no-cpu --no-file --steps 10 > $O/c3_ovl_$k.json 2> $O/ab.err || { tail $O/ab.err; exit 1; }
done
for r in 0 3; do
  NLDSC_COUNT_OVERLAP=0 timeout -k 10 200 python bench.py --no-cpu --no-file --steps 10 --rehearse $r/8 > $O/r${r}of8_count.json 2> $O/ab.err || { tail $O/ab.err; exit 1; }
  timeout -k 10 200 python bench.py --no-cpu --no-file --steps 10 --rehearse $r/8 > $O/r${r}of8_ovl.json 2> $O/ab.err || { tail $O/ab.err; exit 1; }
done
for f in $O/*.json; do python3 -c "
import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); s=d['stages_ms']
print('$f'.split('/')[-1], round(d['ms_per_step'],3), s)"; done
step done
