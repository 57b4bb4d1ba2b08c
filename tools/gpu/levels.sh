#!/bin/bash
# per-level kernel durations (one stream) for each lib given
cd "$GRAFT_REPO_ROOT"; R=$GRAFT_REPO_ROOT; cd /tmp && export TMPDIR=/tmp
k=0
for v in "$@"; do
  k=$((k+1))
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/lv$k -o run -- python3 $R/tools/ab.py $v --rounds 2 > $R/gpurun_out/lv$k.log 2>&1 || { tail -5 $R/gpurun_out/lv$k.log; exit 1; }
  echo "== $v"; (cd $R && python3 tools/trace_stats.py gpurun_out/lv$k/run_kernel_trace.csv gpurun_out/lv$k/stats.csv | grep -v copyBuffer)
done
