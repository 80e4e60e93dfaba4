#!/bin/bash
# GPU check on the gpurun box: gpu tests, bench, rocprof kernel stats. Usage: bash tools/gpu_check.sh TAG [pytest-args]
TAG=${1:-run}; shift
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread "$@" > gpurun_out/pytest_$TAG.txt 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -o prof -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/bench_prof_$TAG.json 2> $GRAFT_REPO_ROOT/gpurun_out/bench_prof_$TAG.err
