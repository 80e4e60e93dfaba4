#!/bin/bash
# subspace_kernel G Z with four rows per thread (main) vs one (noquad); P = 8 at 4 waves per
# SIMD (wpe8x4); per-phase clocks (ssstats build); SVD tests.
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_svd_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r05i.txt 2>&1 && tail -2 gpurun_out/pytest_r05i.txt && \
bash tools/lib_ab.sh tools/svd_bench.py -- noquad main wpe8x4 > gpurun_out/svd_ab_r05i.txt 2>&1 && \
SPECENH_LIB=$R/tools/variants/libspecenh_ssstats.so timeout -k 10 120 python tools/ss_stats.py > gpurun_out/ss_stats_r05i.txt 2>&1
