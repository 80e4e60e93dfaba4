#!/bin/bash
# BCE inside the fused training tail: tests + C4 step A/B
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_ae_gpu.py tests/test_ops_gpu.py tests/test_dp_gpu.py tests/test_c4_fit_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r05ae.txt 2>&1 || { grep -v "^$" gpurun_out/pytest_r05ae.txt | tail -30; exit 1; }
tail -1 gpurun_out/pytest_r05ae.txt
for i in 1 2 3; do for V in 1 0; do echo -n "NO_BCE_FUSION=$V "; SPECENH_NO_BCE_FUSION=$V timeout -k 10 120 python tools/c4_prof.py --steps 200 2>/dev/null | grep c4; done; done
