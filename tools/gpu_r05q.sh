#!/bin/bash
# k = 7 first layer fused with its pool: AE tests, k7 model timings.
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_ae_gpu.py tests/test_narrow_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r05q.txt 2>&1 && tail -2 gpurun_out/pytest_r05q.txt && \
timeout -k 10 200 python tools/ae_layers.py --model hyper_k7 > gpurun_out/ae_layers_r05q.txt 2>&1 && \
timeout -k 10 200 python tools/ae_bench.py --model hyper_k7 --dtype bf16 > gpurun_out/ae_bench_r05q.txt 2>&1
