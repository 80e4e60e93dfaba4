#!/bin/bash
# GPU check on the gpurun box (repo root): GPU tests, the default bench, the
# rocprofv3 kernel stats of the timed chain (one stream), optionally the PMC refresh.
#   bash tools/gpu_run.sh TAG [pmc] [pytest args...]
TAG=${1:-run}; shift
PMC=0
if [ "$1" = "pmc" ]; then PMC=1; shift; fi
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
echo "[gpu_run] pytest"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread "$@" > gpurun_out/pytest_$TAG.txt 2>&1 || { tail -30 gpurun_out/pytest_$TAG.txt; exit 1; }
tail -2 gpurun_out/pytest_$TAG.txt
echo "[gpu_run] bench"
timeout -k 10 420 python bench.py --steps 20 --warmup 3 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_$TAG.json'));print(d['value'],d['ms_per_step'],d['roofline']['frac'],d['accuracy']['pass'])"
echo "[gpu_run] rocprof stats"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$TAG -o prof -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-stages --streams 1 > $R/gpurun_out/bench_prof_$TAG.json 2> $R/gpurun_out/bench_prof_$TAG.err || exit 1
mkdir -p $R/gpurun_out/prof_$TAG && find /tmp/prof_$TAG -name '*stats.csv' -exec cp {} $R/gpurun_out/prof_$TAG/ \;
cd $R
if [ $PMC = 1 ]; then
  echo "[gpu_run] pmc"
  bash tools/pmc_refresh.sh || exit 1
fi
echo "[gpu_run] done"
