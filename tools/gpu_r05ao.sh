#!/bin/bash
# C5 headline: stream count A/B (slices per 4096-shot step)
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
for i in 1 2; do for S in 2 3 4 1; do echo -n "streams=$S "; timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-stages --streams $S 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(round(d['value']), round(d['ms_per_step'],4))" || exit 1; done; done
