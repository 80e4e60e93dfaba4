#!/bin/bash
# fused training tail (convT3 + conv_out with map / logits / output stores): tests, C4 A/B.
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_ae_gpu.py tests/test_ops_gpu.py tests/test_c4_fit_gpu.py -x -q -s --timeout 120 --timeout-method thread -k "training_tail or side_stream or bf16_relative or fp16_relative or fused_conv_pool or opcheck or c4" > gpurun_out/pytest_r05v.txt 2>&1 || { grep -v "^$" gpurun_out/pytest_r05v.txt | tail -30; exit 1; }
grep "map \|passed\|failed" gpurun_out/pytest_r05v.txt
O=gpurun_out/c4tail_r05v.txt
for i in 1 2 3; do
  for V in 1 0; do
    echo -n "NO_TAIL_TRAIN=$V " >> $O
    SPECENH_NO_TAIL_TRAIN=$V timeout -k 10 120 python tools/c4_prof.py --steps 100 2>/dev/null | grep c4 >> $O || exit 1
  done
done
cat $O
