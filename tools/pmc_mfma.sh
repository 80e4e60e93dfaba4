#!/bin/bash
# MFMA / LDS / VALU counters of the autoencoder's forward layers (tools/conv_one.py), one
# rocprofv3 --pmc pass (8 SQ + 1 GRBM counters) per layer. Run from the repo root on the GPU
# box; writes gpurun_out/pmc_mfma/<layer>/; summarise with tools/pmc_mfma_summary.py.
R=$(pwd)
OUT=$R/gpurun_out/pmc_mfma
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for L in ${LAYERS:-l1 l2 l3 ct1 ct2 tail}; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --output-format csv -d $OUT/$L -o p -- python3 $R/tools/conv_one.py $L --reps 3 > $OUT/$L.log 2>&1 || exit 1
done
