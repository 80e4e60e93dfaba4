#!/bin/bash
# C4 kernel timeline (kernel trace of 10 steps, csv)
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/c4trace_${TAG:-r05t}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/c4t_${TAG:-r05t} -o run -- python3 $R/tools/c4_prof.py --steps 10 > $R/gpurun_out/c4trace_${TAG:-r05t}/log.txt 2>&1 || exit 1
find /tmp/c4t_${TAG:-r05t} -name '*kernel_trace.csv' -exec cp {} $R/gpurun_out/c4trace_${TAG:-r05t}/ \;
ls $R/gpurun_out/c4trace_${TAG:-r05t}
