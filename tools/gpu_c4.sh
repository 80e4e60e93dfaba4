#!/bin/bash
# C4 training check on the gpurun box: the training-path GPU tests, the 3-layer train step,
# the rocprof kernel stats of 30 steps.   bash tools/gpu_c4.sh TAG
TAG=${1:-c4}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_wgrad_gpu.py tests/test_c4_fit_gpu.py tests/test_ae_gpu.py tests/test_dp_gpu.py tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.txt 2>&1 || { tail -30 gpurun_out/pytest_$TAG.txt; exit 1; }
tail -1 gpurun_out/pytest_$TAG.txt
for M in 3layer hyper_k3; do
  timeout -k 10 120 python tools/ae_bench.py --model $M --dtype bf16 >> gpurun_out/ae_bench_$TAG.txt 2>&1 || exit 1
done
grep '^{' gpurun_out/ae_bench_$TAG.txt | cut -c1-200
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/profc4_$TAG -o prof -- python3 $R/tools/c4_prof.py --steps 30 > $R/gpurun_out/c4prof_$TAG.log 2>&1 || exit 1
mkdir -p $R/gpurun_out/profc4_$TAG && find /tmp/profc4_$TAG -name '*kernel_stats.csv' -exec cp {} $R/gpurun_out/profc4_$TAG/ \;
echo done
