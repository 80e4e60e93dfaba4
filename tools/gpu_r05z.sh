#!/bin/bash
# first conv's weight gradient on the current stream: tests + C4 step
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_ae_gpu.py tests/test_dp_gpu.py tests/test_c4_fit_gpu.py tests/test_wgrad_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r05z.txt 2>&1 || { grep -v "^$" gpurun_out/pytest_r05z.txt | tail -30; exit 1; }
tail -1 gpurun_out/pytest_r05z.txt
for i in 1 2 3; do timeout -k 10 120 python tools/c4_prof.py --steps 100 2>/dev/null | grep c4; done
