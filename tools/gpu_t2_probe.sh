#!/bin/bash
# 2x2-workgroup study: the bitwise parity tests, then same-box A/B of $NLDSC_T2 (0 single-block, 1 routed, 2 all 2x2)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-t2a}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k 2x2 > $O/t2_tests.log 2>&1 || { echo "t2 tests failed"; tail -60 $O/t2_tests.log; exit 1; }
tail -3 $O/t2_tests.log
S="--steps 10"
bash tools/gpu_ab_env.sh ${1:-t2a} "c3r:NLDSC_T2=1:$S" "c3s:NLDSC_T2=0:$S" "m0r:NLDSC_T2=1:$S --missing 0" "m0s:NLDSC_T2=0:$S --missing 0" "m0a:NLDSC_T2=2:$S --missing 0" "c2r:NLDSC_T2=1:$S --n-org 50000 --additive-only" "c2s:NLDSC_T2=0:$S --n-org 50000 --additive-only"
