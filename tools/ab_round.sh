#!/bin/bash
# A/B of launch rounding and VALU interleave variants of the fp4 band kernel (C3 geometry)
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python tools/band_ab.py --rounds 5 --n-snp 80000 --length-cm 280 \
  --variants "base=f4:xcd,r-1=f4:xcd:round-1,r1024=f4:xcd:round1024,r4096=f4:xcd:round4096,noxcd_r-1=f4:round-1,vpm4=ab_libs/vpm4.so:f4:xcd,vpm6=ab_libs/vpm6.so:f4:xcd,vpm6r=ab_libs/vpm6.so:f4:xcd:round-1" \
  --out gpurun_out/ab1.json > gpurun_out/ab1.log 2>&1
rc=$?
tail -80 gpurun_out/ab1.log
exit $rc
