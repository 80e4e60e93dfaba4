#!/bin/bash
# C4 A/B of existing switches on the new step: stride-2 dgrad kernel, masked C = 1 dgrad on MFMA.
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
O=gpurun_out/c4ab_r05x.txt
for i in 1 2; do
  for E in "X=0" "SPECENH_CONV_NO_S2=1" "SPECENH_C1_MASK_MFMA=1"; do
    echo -n "$E " >> $O
    env $E timeout -k 10 120 python tools/c4_prof.py --steps 100 2>/dev/null | grep c4 >> $O || exit 1
  done
done
cat $O
