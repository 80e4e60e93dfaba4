# round-6 GPU session: row-sweep pooled conv for K = 3 / 32 -> 32 (tests + variant layers)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/gpu.sh s8 tests:tests/test_conv_rows_gpu.py,tests/test_ae_gpu.py || exit 1
for M in hyper_k3 hyper_k5 hyper_k7 manual_scan 3layer; do
  timeout -k 10 200 python tools/ae_layers.py --model $M > gpurun_out/s8_layers_$M.txt 2>&1 || { tail -5 gpurun_out/s8_layers_$M.txt; exit 1; }
  grep -v amdgpu.ids gpurun_out/s8_layers_$M.txt | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['model'], d['total_ms'], [(l['kernel'][:40], l['ms']) for l in d['launches']])"
done
