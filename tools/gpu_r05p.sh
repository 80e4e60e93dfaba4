#!/bin/bash
# variant models: Conv2DTranspose launch options (default / CONVT_PAIR=1 / PATCH_WSPLIT=0)
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
for rnd in 1 2; do
for M in manual_scan hyper_k5 hyper_k3; do
  echo "== $M default" >> gpurun_out/ae_layers_r05p.txt
  timeout -k 10 200 python tools/ae_layers.py --model $M >> gpurun_out/ae_layers_r05p.txt 2>&1 || exit 1
  echo "== $M CONVT_PAIR=1" >> gpurun_out/ae_layers_r05p.txt
  SPECENH_CONVT_PAIR=1 timeout -k 10 200 python tools/ae_layers.py --model $M >> gpurun_out/ae_layers_r05p.txt 2>&1 || exit 1
  echo "== $M PATCH_WSPLIT=0" >> gpurun_out/ae_layers_r05p.txt
  SPECENH_PATCH_WSPLIT=0 timeout -k 10 200 python tools/ae_layers.py --model $M >> gpurun_out/ae_layers_r05p.txt 2>&1 || exit 1
done
done
