#!/bin/bash
# pyramid kernel duration for presets (F=0 writes level 0)
cd "$GRAFT_REPO_ROOT"; R=$GRAFT_REPO_ROOT; cd /tmp && export TMPDIR=/tmp
for pr in medium slow; do
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/py_$pr -o run -- python3 $R/tools/ab.py optical-flow-using-dense-inverse-search_amd/disflow/libdis_hip.so:streams=1,iters=1 --preset $pr --rounds 2 --steps 3 > $R/gpurun_out/py_$pr.log 2>&1 || { tail -5 $R/gpurun_out/py_$pr.log; exit 1; }
  echo "== $pr"; (cd $R && python3 tools/trace_stats.py gpurun_out/py_$pr/run_kernel_trace.csv /tmp/x.csv | grep -E "pyramid|output|upsample|densify")
done
