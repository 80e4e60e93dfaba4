#!/bin/bash
# GPU check on the gpurun box: gpu tests, bench, rocprof kernel stats. Usage: bash tools/gpu_check.sh TAG [pytest-args]
# Only the rocprof *_stats.csv summaries are kept (the kernel traces exceed gpurun's copy-back cap).
TAG=${1:-run}; shift
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out && \
timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread "$@" > gpurun_out/pytest_$TAG.txt 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$TAG -o prof -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-stages --streams 1 > $R/gpurun_out/bench_prof_$TAG.json 2> $R/gpurun_out/bench_prof_$TAG.err && \
mkdir -p $R/gpurun_out/prof_$TAG && find /tmp/prof_$TAG -name '*stats.csv' -exec cp {} $R/gpurun_out/prof_$TAG/ \;
