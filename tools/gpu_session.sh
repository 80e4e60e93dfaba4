#!/bin/bash
# Per-call GPU script (overwritten per experiment).
set -o pipefail
mkdir -p gpurun_out
bash tools/gpu.sh r06e tests || exit 1
for r in 1 2; do timeout -k 10 120 python tools/c4_prof.py --steps 40 2>&1 | grep -v amdgpu.ids; done
