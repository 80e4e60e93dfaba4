#!/bin/bash
# PMC passes over the autoencoder's forward layers (tools/conv_one.py). Run from the repo root
# on the GPU box; writes gpurun_out/pmc_conv/*.
set -e
R=$(pwd)
OUT=$R/gpurun_out/pmc_conv
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --output-format csv -d $OUT/p1 -o p1 -- python3 $R/tools/conv_one.py all --reps 3 > $OUT/p1.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d $OUT/p2 -o p2 -- python3 $R/tools/conv_one.py all --reps 3 > $OUT/p2.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/p3 -o p3 -- python3 $R/tools/conv_one.py all --reps 3 > $OUT/p3.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/p4 -o p4 -- python3 $R/tools/conv_one.py all --reps 3 > $OUT/p4.log 2>&1
