#!/bin/bash
# SQ instruction/stall counters and HBM bytes of one autoencoder layer
# (tools/conv_one.py LAYER), one rocprofv3 --pmc pass per counter group.
# Usage: tools/pmc_sq.sh LAYER TAG   (from the repo root on the GPU box; writes
# gpurun_out/pmc_sq/<TAG>_*)
R=$(pwd)
L=$1; TAG=$2
OUT=$R/gpurun_out/pmc_sq
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for G in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
         "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
         "SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS" \
         "FETCH_SIZE" "WRITE_SIZE"; do
  timeout -s KILL 60 rocprofv3 --pmc $G --output-format csv -d $OUT/${TAG}_$i -o p -- python3 $R/tools/conv_one.py $L --reps 3 > $OUT/${TAG}_$i.log 2>&1 || exit 1
  i=$((i+1))
done
