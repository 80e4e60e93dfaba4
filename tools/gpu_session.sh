#!/bin/bash
# Per-call GPU script (overwritten per experiment).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_ae_gpu.py tests/test_c4_fit_gpu.py tests/test_dp_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/s21_pytest.txt 2>&1 || { tail -30 gpurun_out/s21_pytest.txt; exit 1; }
tail -1 gpurun_out/s21_pytest.txt
for r in 1 2 3; do
  for b in 1 0; do
    echo "== no_pool_routed $b round $r"; SPECENH_NO_POOL_ROUTED=$b timeout -k 10 120 python tools/c4_prof.py --steps 40 || exit 1
  done
done > gpurun_out/s21_c4_routed_ab.txt 2>&1
grep -v amdgpu.ids gpurun_out/s21_c4_routed_ab.txt
