#!/bin/bash
# One parametrised launcher for gpurun calls (repo root on the box). Steps run in order,
# each under its own time limit; the first failing step ends the call (no GPU work after a
# fault, abort or time-out).
#   bash tools/gpu.sh TAG STEP [STEP ...]
# STEP:
#   tests                   every -m gpu test
#   tests:FILE[,FILE...]    those test files (paths under tests/, -k via tests:FILE::name)
#   bench                   the default bench.py line          -> gpurun_out/bench_TAG.json
#   prof                    rocprofv3 --kernel-trace --stats of the one-stream C5 chain
#                                                              -> gpurun_out/prof_TAG/
#   pmc                     tools/pmc_refresh.sh (PMC passes of the bench kernels)
#   py:SCRIPT[:ARGS]        python SCRIPT ARGS (ARGS: commas become spaces) -> gpurun_out/TAG_<name>.txt
TAG=${1:?tag}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
for STEP in "$@"; do
  echo "[gpu.sh] $STEP"
  case "$STEP" in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
        > gpurun_out/pytest_$TAG.txt 2>&1 || { grep -v '^$' gpurun_out/pytest_$TAG.txt | tail -30; exit 1; }
      tail -1 gpurun_out/pytest_$TAG.txt ;;
    tests:*)
      FILES=$(echo "${STEP#tests:}" | tr ',' ' ')
      timeout -k 10 600 python -u -m pytest $FILES -x -q -s --timeout 120 --timeout-method thread \
        > gpurun_out/pytest_$TAG.txt 2>&1 || { grep -v '^$' gpurun_out/pytest_$TAG.txt | tail -30; exit 1; }
      tail -1 gpurun_out/pytest_$TAG.txt ;;
    bench)
      timeout -k 10 420 python bench.py --steps 20 --warmup 3 > gpurun_out/bench_$TAG.json \
        2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
      python -c "import json;d=json.load(open('gpurun_out/bench_$TAG.json'));print(d['value'],d['ms_per_step'],d['roofline']['frac'],d['accuracy']['pass'])" ;;
    prof)
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats \
        --output-format csv -d /tmp/prof_$TAG -o prof -- python3 "$R/bench.py" --steps 10 --warmup 2 \
        --no-cpu-baseline --no-stages --streams 1 > "$R/gpurun_out/bench_prof_$TAG.json" \
        2> "$R/gpurun_out/bench_prof_$TAG.err") || exit 1
      mkdir -p gpurun_out/prof_$TAG && find /tmp/prof_$TAG -name '*stats.csv' -exec cp {} gpurun_out/prof_$TAG/ \; ;;
    pmc)
      bash tools/pmc_refresh.sh || exit 1 ;;
    py:*)
      SPEC=${STEP#py:}
      SCRIPT=${SPEC%%:*}
      ARGS=""
      [ "$SPEC" != "$SCRIPT" ] && ARGS=$(echo "${SPEC#*:}" | tr ',' ' ')
      NAME=$(basename "$SCRIPT" .py)
      timeout -k 10 600 python -u $SCRIPT $ARGS > gpurun_out/${TAG}_$NAME.txt 2>&1 \
        || { tail -30 gpurun_out/${TAG}_$NAME.txt; exit 1; }
      tail -15 gpurun_out/${TAG}_$NAME.txt ;;
    *)
      echo "unknown step $STEP"; exit 2 ;;
  esac
done
echo "[gpu.sh] done"
