#!/bin/bash
# P = 8 Grams on fp64 MFMA split over the waves (main) vs VALU butterflies (p8valu); YtY unrolled
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_svd_gpu.py tests/test_svd_top1_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r05k.txt 2>&1 ; rc=$?; tail -2 gpurun_out/pytest_r05k.txt
[ $rc = 0 ] || exit $rc
bash tools/lib_ab.sh tools/svd_bench.py -- p8valu main > gpurun_out/svd_ab_r05k.txt 2>&1 && \
SPECENH_LIB=$R/tools/variants/libspecenh_ssstats.so timeout -k 10 120 python tools/ss_stats.py > gpurun_out/ss_stats_r05k.txt 2>&1
