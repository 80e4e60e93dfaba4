#!/bin/bash
# Per-call GPU script (overwritten per experiment).
set -o pipefail
mkdir -p gpurun_out
ROUNDS=3 timeout -k 10 900 bash tools/lib_ab.sh tools/layer_ab.py --reps 20 -- main crold dtold > gpurun_out/s18_layer_ab.txt 2>&1 || exit 1
ROUNDS=2 timeout -k 10 600 bash tools/lib_ab.sh tools/ae_layers.py --model hyper_k3 --batch 1024 -- main crold > gpurun_out/s18_hyper_ab.txt 2>&1
