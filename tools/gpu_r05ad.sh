#!/bin/bash
# C4 step: 7x7-wgrad library vs the previous revision's (the 22x22 patch rows, tap groups)
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
export SPECENH_NO_BCE_FUSION=1
bash tools/lib_ab.sh tools/c4_prof.py --steps 200 -- main pre_k7 main pre_k7 2>&1 | grep "==\|c4"
