#!/bin/bash
# C4 step: weight-gradient workgroup target (SPECENH_WGRAD_WG)
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
for i in 1 2; do for V in 4096 2048 1024 8192; do echo -n "WGRAD_WG=$V "; SPECENH_WGRAD_WG=$V timeout -k 10 120 python tools/c4_prof.py --steps 200 2>/dev/null | grep c4 || exit 1; done; done
