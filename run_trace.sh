#!/bin/bash
# kernel trace of tools/ab.py "$@" + the timeline of one step
cd "$GRAFT_REPO_ROOT"; R=$GRAFT_REPO_ROOT; cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/tr -o run -- python3 $R/tools/ab.py "$@" --rounds 2 > $R/gpurun_out/tr.log 2>&1 || { tail -5 $R/gpurun_out/tr.log; exit 1; }
cd $R && python3 tools/timeline.py gpurun_out/tr/run_kernel_trace.csv 12 26
