#!/bin/bash
# STFT 16-byte emit A/B (two builds), convT1 phase-split vs per-wave (variant switch), their tests.
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_stft_gpu.py tests/test_stft_team_gpu.py tests/test_conv_rows_gpu.py tests/test_c5_chain_gpu.py tests/test_reference_shapes_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r05f.txt 2>&1 || { tail -30 gpurun_out/pytest_r05f.txt; exit 1; }
tail -1 gpurun_out/pytest_r05f.txt
bash tools/lib_ab.sh tools/stft_c2_bench.py -- main narrow > gpurun_out/stft_ab_r05f.txt 2>&1 || { tail -20 gpurun_out/stft_ab_r05f.txt; exit 1; }
grep -v amdgpu gpurun_out/stft_ab_r05f.txt
timeout -k 10 300 python tools/layer_ab.py --reps 20 "" "SPECENH_CONVT_PW=1" > gpurun_out/layer_ab_r05f.txt 2>&1 || { tail -20 gpurun_out/layer_ab_r05f.txt; exit 1; }
grep -v amdgpu gpurun_out/layer_ab_r05f.txt
timeout -k 10 200 python tools/stft_c2_flags.py > gpurun_out/stft_flags_r05f.txt 2>&1 || exit 1
grep -v amdgpu gpurun_out/stft_flags_r05f.txt
