#!/bin/bash
# Per-call GPU script (overwritten per experiment).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_decoder_tail_gpu.py tests/test_c5_chain_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/s33_pytest.txt 2>&1 || { tail -30 gpurun_out/s33_pytest.txt; exit 1; }
tail -1 gpurun_out/s33_pytest.txt
ROUNDS=4 timeout -k 10 700 bash tools/lib_ab.sh tools/layer_ab.py --reps 20 -- main d3prev > gpurun_out/s33_layer_ab.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/s33_layer_ab.txt | grep -v variant
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" 2>&1 | tail -2
