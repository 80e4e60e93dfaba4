#!/bin/bash
# Per-call GPU script (overwritten per experiment).
set -o pipefail
mkdir -p gpurun_out
python -c "import torch; print('prio range', torch.cuda.Stream.priority_range())"
for r in 1 2 3; do
  for cfg in "SPECENH_CHAIN_PRIO=0" "SPECENH_CHAIN_PRIO=1"; do
    echo "== [$cfg] round $r"; env $cfg timeout -k 10 120 python tools/c4_prof.py --steps 40 || exit 1
  done
done > gpurun_out/s38_c4_prio_ab.txt 2>&1
grep -v amdgpu.ids gpurun_out/s38_c4_prio_ab.txt
SPECENH_CHAIN_PRIO=1 timeout -k 10 300 python -u -m pytest tests/test_ae_gpu.py -k "side_stream or pool_routed or engine" -x -q --timeout 120 --timeout-method thread 2>&1 | tail -1
