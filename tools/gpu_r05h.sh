#!/bin/bash
# enc2 stagger A/B (layer times, two library builds interleaved) and the row-kernel tests.
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_conv_rows_gpu.py tests/test_c5_chain_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r05h.txt 2>&1 || { tail -30 gpurun_out/pytest_r05h.txt; exit 1; }
tail -1 gpurun_out/pytest_r05h.txt
bash tools/lib_ab.sh tools/layer_ab.py --reps 20 -- main nostag > gpurun_out/layer_ab_r05h.txt 2>&1 || { tail -20 gpurun_out/layer_ab_r05h.txt; exit 1; }
grep -v amdgpu gpurun_out/layer_ab_r05h.txt
