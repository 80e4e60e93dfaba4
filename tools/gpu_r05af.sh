#!/bin/bash
# C4 step: stride-2 input gradients with more output channels per workgroup (SPECENH_S2_MIN_NT)
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
for i in 1 2; do for V in 0 2 4; do echo -n "S2_MIN_NT=$V "; SPECENH_S2_MIN_NT=$V timeout -k 10 120 python tools/c4_prof.py --steps 200 2>/dev/null | grep c4 || exit 1; done; done
