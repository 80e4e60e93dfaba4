#!/bin/bash
# Per-call GPU script (overwritten per experiment).
set -o pipefail
mkdir -p gpurun_out
for r in 1 2 3; do
  for cfg in "" "SPECENH_ENC2_WPE2=1" "SPECENH_ROWS_SHORT_LEAD=1"; do
    echo "== [$cfg] round $r"; env $cfg timeout -k 10 120 python tools/layer_ab.py --reps 20 2>&1 | grep -v "amdgpu.ids\|variant" || exit 1
  done
done > gpurun_out/s36_layer_env_ab.txt 2>&1
cat gpurun_out/s36_layer_env_ab.txt
