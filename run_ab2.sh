#!/bin/bash
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python tools/ab.py "$@" --rounds 10 2>&1 | tail -6
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/ab_prof -o run -- python3 $GRAFT_REPO_ROOT/tools/ab.py "$@" --rounds 2 > /dev/null 2>&1
cut -c1-120 $GRAFT_REPO_ROOT/gpurun_out/ab_prof/run_kernel_stats.csv
