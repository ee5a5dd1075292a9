#!/bin/bash
# strong-scaling bench over RCCL (a process group of one on the one-GPU box: --force-dist): the score-table gather on a
# side stream beside the next step (default) against gathering before the next step (--no-gather-overlap); the same
# table digest; then the torchrun GPU tests
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-go}; mkdir -p $O
for i in 1 2; do
timeout -k 10 200 python bench.py --force-dist --no-cpu --no-file --steps 20 > $O/ovl$i.json 2> $O/ovl$i.err || { tail $O/ovl$i.err; exit 1; }
timeout -k 10 200 python bench.py --force-dist --no-cpu --no-file --steps 20 --no-gather-overlap > $O/seq$i.json 2> $O/seq$i.err || { tail $O/seq$i.err; exit 1; }
done
timeout -k 10 200 python bench.py --no-cpu --no-file --steps 5 > $O/one.json 2> $O/one.err || { tail $O/one.err; exit 1; }
for f in ovl1 seq1 ovl2 seq2 one; do python3 -c "
import json; d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]); print('$f', round(d['ms_per_step'],3), d['stages_ms'].get('total_ms'), d['stages_ms'].get('gather_ms'), d['table_digest'])"; done
timeout -k 10 600 python -u -m pytest tests/test_gpu_torchrun.py -x -v --timeout 300 --timeout-method thread > $O/torchrun.log 2>&1 || { tail -30 $O/torchrun.log; exit 1; }
tail -2 $O/torchrun.log
