#!/bin/bash
# masked C = 1 conv (C4 input gradient of the last conv): MFMA vs VALU at batch 128 / 2048,
# and the C4 train step with each.
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
O=gpurun_out/c1mask_r05r.txt
for B in 128 2048; do
  echo "batch $B" >> $O
  SPECENH_C1_MASK_MFMA=1 timeout -k 10 120 python tools/c1_bench.py --batch $B >> $O 2>&1 || exit 1
done
for i in 1 2 3; do
  for V in 0 1; do
    echo -n "C1_MASK_MFMA=$V " >> $O
    SPECENH_C1_MASK_MFMA=$V timeout -k 10 120 python tools/c4_prof.py --steps 100 2>/dev/null | grep c4 >> $O || exit 1
  done
done
cat $O
