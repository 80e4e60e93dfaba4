#!/bin/bash
# one-input-channel weight gradient: tiles per workgroup (SPECENH_WGRAD_C1_TILES), C4 step
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
for i in 1 2; do for V in 4 8 16 2; do echo -n "WGRAD_C1_TILES=$V "; SPECENH_WGRAD_C1_TILES=$V timeout -k 10 120 python tools/c4_prof.py --steps 200 2>/dev/null | grep c4 || exit 1; done; done
