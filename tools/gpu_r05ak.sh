#!/bin/bash
# pooled first-layer wgrad overwrites its slice (no zeroing launch): tests + C4 step
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_ae_gpu.py tests/test_ops_gpu.py tests/test_wgrad_gpu.py tests/test_dp_gpu.py tests/test_c4_fit_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r05ak.txt 2>&1 || { grep -v "^$" gpurun_out/pytest_r05ak.txt | tail -30; exit 1; }
tail -1 gpurun_out/pytest_r05ak.txt
for i in 1 2 3; do timeout -k 10 120 python tools/c4_prof.py --steps 200 2>/dev/null | grep c4 || exit 1; done
