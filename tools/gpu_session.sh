#!/bin/bash
# Per-call GPU script (overwritten per experiment).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_narrow_gpu.py tests/test_ae_gpu.py tests/test_c4_fit_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/s27_pytest.txt 2>&1 || { tail -30 gpurun_out/s27_pytest.txt; exit 1; }
tail -1 gpurun_out/s27_pytest.txt
for r in 1 2 3; do
  for cfg in "SPECENH_C1_MASK_MFMA=0" "SPECENH_C1_MASK_MFMA=1"; do
    echo "== [$cfg] round $r"; env $cfg timeout -k 10 120 python tools/c4_prof.py --steps 40 || exit 1
  done
done > gpurun_out/s27_c4_ab.txt 2>&1
grep -v amdgpu.ids gpurun_out/s27_c4_ab.txt
