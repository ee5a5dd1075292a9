#!/bin/bash
# round end: PMC passes of the committed kernels (C3, C2, C5 slice) and the default bench line that reads them
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-r3g}
bash tools/gpu_round.sh $T skip-tests pmc || exit 1
