#!/bin/bash
# Per-call GPU script (overwritten per experiment).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_decoder_tail_gpu.py tests/test_c5_chain_gpu.py tests/test_decoder3_mapping.py -x -q --timeout 120 --timeout-method thread > gpurun_out/s35_pytest.txt 2>&1 || { tail -30 gpurun_out/s35_pytest.txt; exit 1; }
tail -1 gpurun_out/s35_pytest.txt
bash tools/gpu.sh r06d bench prof
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" 2>&1 | tail -1
