#!/bin/bash
# Per-call GPU script (overwritten per experiment).
set -o pipefail
mkdir -p gpurun_out
R=$(pwd)
bash tools/pmc_refresh.sh > gpurun_out/s25_pmc.log 2>&1 || { tail -20 gpurun_out/s25_pmc.log; exit 1; }
tail -2 gpurun_out/s25_pmc.log
cd $R
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/c4st -o run -- python3 $R/tools/c4_prof.py --steps 30) > gpurun_out/s25_c4stats.log 2>&1 || exit 1
mkdir -p gpurun_out/c4stats_s25 && find /tmp/c4st -name '*stats.csv' -exec cp {} gpurun_out/c4stats_s25/ \; && find /tmp/c4st -name '*kernel_trace.csv' -exec cp {} gpurun_out/c4stats_s25/run_kernel_trace.csv \;
tail -2 gpurun_out/s25_c4stats.log
