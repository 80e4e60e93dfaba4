#!/bin/bash
# C4 fork/join events: torch events vs library events (system / device-scope release).
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
O=gpurun_out/c4fork_r05u.txt
for i in 1 2 3; do
  for M in torch system device; do
    echo -n "FORK=$M " >> $O
    SPECENH_FORK=$M timeout -k 10 120 python tools/c4_prof.py --steps 100 2>/dev/null | grep c4 >> $O || exit 1
  done
done
cat $O
timeout -k 10 300 python -u -m pytest tests/test_ae_gpu.py tests/test_dp_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r05u.txt 2>&1; tail -2 gpurun_out/pytest_r05u.txt
