#!/bin/bash
# r03 session 15: per-call timeline of the sub-batch streams, no profiler
# (diagnostic build with in-kernel clocks)
cd "$GRAFT_REPO_ROOT"; R=$GRAFT_REPO_ROOT
L=$R/optical-flow-using-dense-inverse-search_amd/disflow/libdis_hip_stamp.so
for args in "" "--streams 1" "--no-graphs" "--streams 1 --no-graphs"; do
  echo "=== $args"
  DIS_STAMP=1 DISFLOW_LIB=$L timeout -k 10 200 python3 tools/stamp_probe.py --steps 40 $args > gpurun_out/stamp.log 2>&1; rc=$?
  cat gpurun_out/stamp.log | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
done
