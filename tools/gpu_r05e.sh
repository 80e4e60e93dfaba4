#!/bin/bash
# decoder3 read-ahead A/B (layer times, two library builds interleaved), then the C4 check.
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
bash tools/lib_ab.sh tools/layer_ab.py --reps 20 -- main nora > gpurun_out/layer_ab_r05e.txt 2>&1 || { tail -20 gpurun_out/layer_ab_r05e.txt; exit 1; }
grep -v amdgpu gpurun_out/layer_ab_r05e.txt | tail -40
timeout -k 10 300 python -u -m pytest tests/test_decoder_tail_gpu.py tests/test_c5_chain_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r05e.txt 2>&1 || { tail -30 gpurun_out/pytest_r05e.txt; exit 1; }
tail -1 gpurun_out/pytest_r05e.txt
bash tools/gpu_c4.sh c4b
