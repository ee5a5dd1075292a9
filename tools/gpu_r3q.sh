#!/bin/bash
# round 3: quad super-items in round launches (one workgroup per CU per launch) vs one launch, C5 slice and C3m0
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r3q; mkdir -p $O
timeout -k 10 600 python tools/ab_libs.py --libs base=nldsc_amd/libnldsc_amd.so qrounds=nldsc_amd/libnldsc_amd.so,NLDSC_Q_ROUNDS=1 --workload c5 c3m0 --runs 6 \
  > $O/ab_qrounds.json 2> $O/ab_qrounds.err || { tail $O/ab_qrounds.err; exit 1; }
cat $O/ab_qrounds.json
