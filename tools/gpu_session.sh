#!/bin/bash
# Per-call GPU script (overwritten per experiment).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python tools/c4_routed_probe.py > gpurun_out/s32_routed.txt 2>&1 || { tail gpurun_out/s32_routed.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/s32_routed.txt
