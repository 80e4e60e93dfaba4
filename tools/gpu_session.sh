#!/bin/bash
# Per-call GPU script (overwritten per experiment).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_conv_rows_gpu.py tests/test_c4_fit_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/s19_pytest.txt 2>&1 || { tail -30 gpurun_out/s19_pytest.txt; exit 1; }
tail -1 gpurun_out/s19_pytest.txt
for r in 1 2 3; do
  for b in 0 -1; do
    echo "== bands $b round $r"; SPECENH_ROWS_BANDS=$b timeout -k 10 120 python tools/c4_prof.py --steps 40 || exit 1
  done
done > gpurun_out/s19_c4_bands_ab.txt 2>&1
cat gpurun_out/s19_c4_bands_ab.txt | grep -v amdgpu.ids
