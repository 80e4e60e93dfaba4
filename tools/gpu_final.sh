#!/bin/bash
# Round-end measurement pass on the gpurun box: full GPU tests, the default bench, rocprof kernel
# stats of the C5 chain (one stream), of the C4 train step and of the C3 SVD, the AE model
# variants, and the PMC refresh of every target. Steps chained; the first failure ends the run.
#   bash tools/gpu_final.sh TAG        (FINAL_PMC=0: skip the PMC passes, run them as a second
#                                      call: bash tools/pmc_refresh.sh c5 c2 csd c3 c4)
TAG=${1:-final}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
echo "[final] pytest"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.txt 2>&1 || { tail -30 gpurun_out/pytest_$TAG.txt; exit 1; }
tail -1 gpurun_out/pytest_$TAG.txt
echo "[final] bench"
timeout -k 10 420 python bench.py --steps 20 --warmup 3 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_$TAG.json'));print(d['value'],d['ms_per_step'],d['roofline']['frac'],d['accuracy']['pass'],d['accuracy']['out_rel_max'])"
echo "[final] ae variants"
for M in 3layer manual_scan hyper_k3 hyper_k5 hyper_k7; do
  timeout -k 10 120 python tools/ae_bench.py --model $M --dtype bf16 >> gpurun_out/ae_bench_$TAG.txt 2>&1 || exit 1
done
echo "[final] rocprof c5"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$TAG -o prof -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-stages --streams 1 > $R/gpurun_out/bench_prof_$TAG.json 2> $R/gpurun_out/bench_prof_$TAG.err || exit 1
mkdir -p $R/gpurun_out/prof_$TAG && find /tmp/prof_$TAG -name '*kernel_stats.csv' -exec cp {} $R/gpurun_out/prof_$TAG/ \;
echo "[final] rocprof c4"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/profc4_$TAG -o prof -- python3 $R/tools/c4_prof.py --steps 30 > $R/gpurun_out/c4prof_$TAG.log 2>&1 || exit 1
mkdir -p $R/gpurun_out/profc4_$TAG && find /tmp/profc4_$TAG -name '*kernel_stats.csv' -exec cp {} $R/gpurun_out/profc4_$TAG/ \;
echo "[final] rocprof c3"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/profc3_$TAG -o prof -- python3 $R/tools/svd_bench.py > $R/gpurun_out/c3prof_$TAG.log 2>&1 || exit 1
mkdir -p $R/gpurun_out/profc3_$TAG && find /tmp/profc3_$TAG -name '*kernel_stats.csv' -exec cp {} $R/gpurun_out/profc3_$TAG/ \;
cd $R
if [ "${FINAL_PMC:-1}" != 0 ]; then
  echo "[final] pmc"
  rm -rf gpurun_out/pmc
  bash tools/pmc_refresh.sh c5 c2 csd c3 c4 || exit 1
fi
echo "[final] done"
