#!/bin/bash
# kernel trace of a short bench run (2 streams) + per-(kernel, grid) stats
cd "$GRAFT_REPO_ROOT"; R=$GRAFT_REPO_ROOT; cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/tb -o run -- python3 $R/bench.py --steps 10 --warmup 5 --no-cpu-baseline "$@" > $R/gpurun_out/tb.log 2>&1 || { tail -5 $R/gpurun_out/tb.log; exit 1; }
cd $R && python3 tools/trace_stats.py gpurun_out/tb/run_kernel_trace.csv gpurun_out/tb/stats.csv && tail -1 gpurun_out/tb.log | cut -c1-200
