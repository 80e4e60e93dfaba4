#!/bin/bash
# one-output-channel MFMA conv: narrow-kernel tests, AE tests, variant models per layer + ae_bench.
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_narrow_gpu.py tests/test_ae_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r05n.txt 2>&1 && tail -2 gpurun_out/pytest_r05n.txt && \
for M in manual_scan hyper_k3 hyper_k5 hyper_k7; do
  timeout -k 10 200 python tools/ae_layers.py --model $M >> gpurun_out/ae_layers_r05n.txt 2>&1 || exit 1
  timeout -k 10 200 python tools/ae_bench.py --model $M --dtype bf16 >> gpurun_out/ae_bench_r05n.txt 2>&1 || exit 1
done
