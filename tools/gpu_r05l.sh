#!/bin/bash
# conv_rows_pool_kernel: scalar step counters (main) vs per-step divisions (divs); tests, layer A/B

R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_conv_rows_gpu.py tests/test_c5_chain_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r05l.txt 2>&1 && tail -2 gpurun_out/pytest_r05l.txt && \
bash tools/lib_ab.sh tools/layer_ab.py --reps 20 -- main divs > gpurun_out/layer_ab_r05l.txt 2>&1
