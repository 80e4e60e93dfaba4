#!/bin/bash
# weight gradients on a side stream: tests, C4 train-step A/B (serial vs overlap, 3 rounds),
# new SVD G Z path test.
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_ae_gpu.py tests/test_dp_gpu.py tests/test_svd_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r05j.txt 2>&1 && tail -2 gpurun_out/pytest_r05j.txt && \
for rnd in 1 2 3; do
  SPECENH_WGRAD_SERIAL=1 timeout -k 10 120 python tools/ae_bench.py --steps 50 >> gpurun_out/c4_overlap_ab_r05j.txt 2>&1 || exit 1
  timeout -k 10 120 python tools/ae_bench.py --steps 50 >> gpurun_out/c4_overlap_ab_r05j.txt 2>&1 || exit 1
done
