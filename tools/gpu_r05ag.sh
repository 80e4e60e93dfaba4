#!/bin/bash
# C4 step: patch-kernel workgroup target (SPECENH_PATCH_MIN_WG) with the S2 default of 2 N tiles;
# then the conv / S2 GPU tests on the new defaults
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
for i in 1 2; do for V in 512 256 128 1024; do echo -n "PATCH_MIN_WG=$V "; SPECENH_PATCH_MIN_WG=$V timeout -k 10 120 python tools/c4_prof.py --steps 200 2>/dev/null | grep c4 || exit 1; done; done
echo -n "S2_MIN_NT=1 (old) "; SPECENH_S2_MIN_NT=1 timeout -k 10 120 python tools/c4_prof.py --steps 200 2>/dev/null | grep c4 || exit 1
timeout -k 10 500 python -u -m pytest tests/test_ae_gpu.py tests/test_conv_rows_gpu.py tests/test_c4_fit_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r05ag.txt 2>&1 || { grep -v "^$" gpurun_out/pytest_r05ag.txt | tail -30; exit 1; }
tail -1 gpurun_out/pytest_r05ag.txt
