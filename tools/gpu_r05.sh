#!/bin/bash
# Round-5 GPU check on the gpurun box (repo root): GPU tests, the default bench, the rocprof
# kernel stats of the C5 chain (one stream) and of the C4 train step, the AE model variants,
# optionally the PMC refresh of given targets. Every GPU step has its own time limit and the
# steps are chained: the first failure ends the run.
#   bash tools/gpu_r05.sh TAG [pmc TARGETS...]
TAG=${1:-run}; shift
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
step() { echo "[gpu_r05] $1"; }
step pytest
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.txt 2>&1 || { tail -30 gpurun_out/pytest_$TAG.txt; exit 1; }
tail -1 gpurun_out/pytest_$TAG.txt
step bench
timeout -k 10 420 python bench.py --steps 20 --warmup 3 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_$TAG.json'));print(d['value'],d['ms_per_step'],d['roofline']['frac'],d['accuracy']['pass'],d['accuracy']['out_rel_max'])"
step "ae variants"
for M in 3layer manual_scan hyper_k3 hyper_k5 hyper_k7; do
  timeout -k 10 120 python tools/ae_bench.py --model $M --dtype bf16 >> gpurun_out/ae_bench_$TAG.txt 2>&1 || exit 1
done
for M in 3layer hyper_k3; do
  timeout -k 10 120 python tools/ae_bench.py --model $M --dtype float16 >> gpurun_out/ae_bench_$TAG.txt 2>&1 || exit 1
done
step "stft flags"
timeout -k 10 200 python tools/stft_c2_flags.py > gpurun_out/stft_flags_$TAG.txt 2>&1 || exit 1
step "rocprof c5"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$TAG -o prof -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-stages --streams 1 > $R/gpurun_out/bench_prof_$TAG.json 2> $R/gpurun_out/bench_prof_$TAG.err || exit 1
mkdir -p $R/gpurun_out/prof_$TAG && find /tmp/prof_$TAG -name '*stats.csv' -exec cp {} $R/gpurun_out/prof_$TAG/ \;
step "rocprof c4"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/profc4_$TAG -o prof -- python3 $R/tools/c4_prof.py --steps 30 > $R/gpurun_out/c4prof_$TAG.log 2>&1 || exit 1
mkdir -p $R/gpurun_out/profc4_$TAG && find /tmp/profc4_$TAG -name '*kernel_stats.csv' -exec cp {} $R/gpurun_out/profc4_$TAG/ \;
cd $R
if [ "$1" = "pmc" ]; then
  shift
  step "pmc $*"
  bash tools/pmc_refresh.sh "$@" || exit 1
fi
step done
