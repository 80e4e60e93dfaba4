#!/bin/bash
# 7 x 7 weight gradients on the MFMA kernel (tap groups): tests + hyper_k7 / 3layer train
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_wgrad_gpu.py tests/test_ae_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r05ac.txt 2>&1 || { grep -v "^$" gpurun_out/pytest_r05ac.txt | tail -30; exit 1; }
tail -1 gpurun_out/pytest_r05ac.txt
for M in hyper_k7 hyper_k5 3layer; do timeout -k 10 120 python tools/ae_bench.py --model $M --dtype bf16 2>/dev/null | grep '^{' | cut -c1-330; done
timeout -k 10 120 python tools/c4_prof.py --steps 100 2>/dev/null | grep c4
