#!/bin/bash
# A/B of tools/ab.py variants, then the kernel-trace timeline of the FIRST variant
cd "$GRAFT_REPO_ROOT"; R=$GRAFT_REPO_ROOT
timeout -k 10 600 python3 tools/ab.py "$@" || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/tr -o run -- python3 $R/tools/ab.py $1 --rounds 2 > $R/gpurun_out/tr.log 2>&1 || { tail -5 $R/gpurun_out/tr.log; exit 1; }
cd $R && python3 tools/timeline.py gpurun_out/tr/run_kernel_trace.csv 12 26
