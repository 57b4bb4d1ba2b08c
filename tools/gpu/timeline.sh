#!/bin/bash
# kernel timeline of one step for each tools/ab.py variant given (kernel trace)
cd "$GRAFT_REPO_ROOT"; R=$GRAFT_REPO_ROOT; cd /tmp && export TMPDIR=/tmp
k=0
for v in "$@"; do
  k=$((k+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/tl$k -o run -- python3 $R/tools/ab.py $v --rounds 2 > $R/gpurun_out/tl$k.log 2>&1 || { tail -5 $R/gpurun_out/tl$k.log; exit 1; }
  echo "== $v"; grep pairs/s $R/gpurun_out/tl$k.log | cut -c1-160
  (cd $R && python3 tools/timeline.py gpurun_out/tl$k/run_kernel_trace.csv ${STEP:-12} ${N:-30})
done
