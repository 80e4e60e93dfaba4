#!/bin/bash
# 7 x 7 convolutions on the patch kernel (+ fused pool): AE / conv tests, variant timings.
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_ae_gpu.py tests/test_conv_s2_gpu.py tests/test_narrow_gpu.py tests/test_c4_fit_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r05o.txt 2>&1 && tail -2 gpurun_out/pytest_r05o.txt && \
for M in hyper_k7 hyper_k5; do
  timeout -k 10 200 python tools/ae_layers.py --model $M >> gpurun_out/ae_layers_r05o.txt 2>&1 || exit 1
  timeout -k 10 200 python tools/ae_bench.py --model $M --dtype bf16 >> gpurun_out/ae_bench_r05o.txt 2>&1 || exit 1
done
