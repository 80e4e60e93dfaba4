#!/bin/bash
# SQ instruction/stall counters and HBM bytes of whatever `python3 CMD...` launches, one
# rocprofv3 --pmc pass per counter group (each within the gfx950 per-pass slot limits).
# Usage (repo root, GPU box): tools/pmc_cmd.sh TAG script.py [args...]
#   -> gpurun_out/pmc_cmd/<TAG>_<i>/ ; summarise with tools/pmc_summary.py
R=$(pwd)
TAG=$1; shift
OUT=$R/gpurun_out/pmc_cmd
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for G in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
         "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
         "SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_MFMA" \
         "FETCH_SIZE" "WRITE_SIZE"; do
  timeout -s KILL 90 rocprofv3 --pmc $G --output-format csv -d $OUT/${TAG}_$i -o p -- python3 "$@" > $OUT/${TAG}_$i.log 2>&1 || exit 1
  i=$((i+1))
done
