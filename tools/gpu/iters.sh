#!/bin/bash
# finest-level search launch duration vs iteration count (one stream)
cd "$GRAFT_REPO_ROOT"; R=$GRAFT_REPO_ROOT; cd /tmp && export TMPDIR=/tmp
LIB=${LIB:-optical-flow-using-dense-inverse-search_amd/disflow/libdis_hip.so}
for it in ${ITERS:-0 1 12 25 50}; do
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/it$it -o run -- python3 $R/tools/ab.py $LIB:streams=1,iters=$it --rounds 2 > $R/gpurun_out/it$it.log 2>&1 || { tail -5 $R/gpurun_out/it$it.log; exit 1; }
  echo "iters=$it"; (cd $R && python3 tools/trace_stats.py gpurun_out/it$it/run_kernel_trace.csv gpurun_out/it$it/stats.csv | grep search8 | head -3)
done
