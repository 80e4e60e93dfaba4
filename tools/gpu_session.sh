#!/bin/bash
# Per-call GPU script (overwritten per experiment).
set -o pipefail
mkdir -p gpurun_out
R=$(pwd)
timeout -k 10 700 python -u -m pytest tests/test_ae_gpu.py tests/test_c4_fit_gpu.py tests/test_ops_gpu.py tests/test_conv_s2_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/s24_pytest.txt 2>&1 || { tail -30 gpurun_out/s24_pytest.txt; exit 1; }
tail -1 gpurun_out/s24_pytest.txt
for r in 1 2 3; do
  for cfg in "1 1 1" "2 0 0" "2 0 1"; do
    set -- $cfg
    echo "== streams $1 accum $2 no_routed $3 round $r"; SPECENH_WGRAD_STREAMS=$1 SPECENH_WGRAD_ACCUM=$2 SPECENH_NO_POOL_ROUTED=$3 timeout -k 10 120 python tools/c4_prof.py --steps 40 || exit 1
  done
done > gpurun_out/s24_c4_ab.txt 2>&1
grep -v amdgpu.ids gpurun_out/s24_c4_ab.txt
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/c4tr -o run -- python3 $R/tools/c4_prof.py --steps 10) > gpurun_out/s24_c4trace.log 2>&1 || exit 1
mkdir -p gpurun_out/c4trace_s24 && find /tmp/c4tr -name '*kernel_trace.csv' -exec cp {} gpurun_out/c4trace_s24/run_kernel_trace.csv \;
python tools/c4_timeline.py gpurun_out/c4trace_s24/run_kernel_trace.csv > gpurun_out/s24_timeline.txt
cat gpurun_out/s24_timeline.txt
