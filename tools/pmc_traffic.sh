#!/bin/bash
# HBM traffic (rocprofv3 FETCH_SIZE / WRITE_SIZE, one counter per pass) of the bench's
# kernels at the bench shapes: the autoencoder layers that run without a fused pool
# (tools/conv_one.py LAYER: that layer's launch only) and the C2 STFT (tools/stft_one.py).
# Run from the repo root on the GPU box; writes gpurun_out/pmc_traffic/*.
R=$(pwd)
OUT=$R/gpurun_out/pmc_traffic
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for L in l1 l2 l3 ct1 ct2 ct3 last tail; do
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $OUT/${L}_$C -o p -- python3 $R/tools/conv_one.py $L --reps 3 > $OUT/${L}_$C.log 2>&1 || exit 1
  done
done
for C in FETCH_SIZE WRITE_SIZE; do
  REPS=3 timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $OUT/stft_c2_$C -o p -- python3 $R/tools/stft_one.py > $OUT/stft_c2_$C.log 2>&1 || exit 1
done
