#!/bin/bash
# Per-call GPU script (overwritten per experiment).
set -o pipefail
mkdir -p gpurun_out
ROUNDS=4 timeout -k 10 900 bash tools/lib_ab.sh bench.py --steps 60 --warmup 10 --no-stages --no-cpu-baseline -- main noswz > gpurun_out/s15_bench_ab.txt 2>&1
