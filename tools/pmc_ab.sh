#!/bin/bash
# SQ/GRBM counters of the band kernel for two builds (ab_libs/head.so vs ab_libs/vb.so), one pass each
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for L in head vb; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU --kernel-trace \
    -d gpurun_out/pmcab/$L -o s --output-format csv -- python3 tools/run_lib.py ab_libs/$L.so --runs 2 > gpurun_out/pmcab_$L.log 2>&1 \
    || { echo "pmc $L failed"; tail gpurun_out/pmcab_$L.log; exit 1; }
  cat gpurun_out/pmcab_$L.log | grep band
done
find gpurun_out/pmcab -name "*.db" -delete 2>/dev/null; true
