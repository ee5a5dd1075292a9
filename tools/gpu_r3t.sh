#!/bin/bash
# round 3: the 2 x 2 LDS-shared workgroups for every C3 block pair (NLDSC_T2=2) on the block-interleaved layout,
# against the default (single-block round launches)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r3t; mkdir -p $O
timeout -k 10 400 python tools/ab_libs.py --libs base=nldsc_amd/libnldsc_amd.so t2all=nldsc_amd/libnldsc_amd.so,NLDSC_T2=2 --workload c3 c2 --runs 8 \
  > $O/ab_t2all.json 2> $O/ab_t2all.err || { tail $O/ab_t2all.err; exit 1; }
cat $O/ab_t2all.json
