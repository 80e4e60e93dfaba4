#!/bin/bash
# rocprofv3 --pmc passes of every shipped kernel at the bench's launch shapes
# (tools/pmc_workload.py targets), one counter group per run, each under its own time limit.
# Run from the repo root on the GPU box:
#   bash tools/pmc_refresh.sh [targets...]      (default: c5 c2 csd c3 c4)
# then fold here: python tools/pmc_fold.py gpurun_out/pmc profiles/pmc_r05.json
R=$(pwd)
OUT=$R/gpurun_out/pmc
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
TARGETS=${*:-c5 c2 csd c3 c4}
P0="FETCH_SIZE"
P1="WRITE_SIZE"
P2="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE"
P3="SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM"
for T in $TARGETS; do
  i=0
  for G in "$P0" "$P1" "$P2" "$P3"; do
    D=$OUT/${T}_p$i
    echo "[pmc_refresh] $T pass $i: $G"
    timeout -s KILL 150 rocprofv3 --pmc $G --output-format csv -d $D -o p -- \
      python3 $R/tools/pmc_workload.py $T $D > $D.log 2>&1 || { echo "[pmc_refresh] FAILED $T pass $i"; tail -5 $D.log; exit 1; }
    i=$((i+1))
  done
done
echo "[pmc_refresh] done"
