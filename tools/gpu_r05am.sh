#!/bin/bash
# weight-gradient LDS swizzle (SPECENH_WGRAD_SWZ): per-layer wgrad and C4 step, same box
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
bash tools/lib_ab.sh tools/wgrad_bench.py -- main noswz 2>&1 | grep "==\|total\|conv"
bash tools/lib_ab.sh tools/c4_prof.py --steps 200 -- main noswz main noswz 2>&1 | grep "==\|c4"
