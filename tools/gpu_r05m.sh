#!/bin/bash
# merged fp64 fallback launch: SVD tests; C5 SVD stage timing with EIG_SPLIT=0/1 (3 rounds).
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_svd_gpu.py tests/test_svd_top1_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r05m.txt 2>&1 && tail -2 gpurun_out/pytest_r05m.txt && \
for rnd in 1 2 3; do
  SPECENH_EIG_SPLIT=1 timeout -k 10 120 python tools/svd_c5.py >> gpurun_out/svd_c5_ab_r05m.txt 2>&1 || exit 1
  SPECENH_EIG_SPLIT=0 timeout -k 10 120 python tools/svd_c5.py >> gpurun_out/svd_c5_ab_r05m.txt 2>&1 || exit 1
done
