#!/bin/bash
# C4 launch-bound probe: eager vs captured graph.
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
O=gpurun_out/c4graph_r05s.txt
for B in 128 256; do
  echo "batch $B" >> $O
  timeout -k 10 180 python tools/c4_graph.py --batch $B >> $O 2>&1 || { cat $O; exit 1; }
done
SPECENH_WGRAD_SERIAL=1 timeout -k 10 180 python tools/c4_graph.py --batch 128 >> $O 2>&1 || { cat $O; exit 1; }
cat $O
