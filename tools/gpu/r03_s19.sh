#!/bin/bash
# r03 session 19: per-call timeline with sub-batch 0 on the caller's stream
cd "$GRAFT_REPO_ROOT"; R=$GRAFT_REPO_ROOT
D=$R/optical-flow-using-dense-inverse-search_amd/disflow
for L in libdis_hip_stamp.so libdis_hip_stampc.so; do
for args in "" "--no-graphs"; do
  echo "=== $L $args"
  DIS_STAMP=1 DISFLOW_LIB=$D/$L timeout -k 10 200 python3 tools/stamp_probe.py --steps 40 $args > gpurun_out/stamp.log 2>&1; rc=$?
  grep median gpurun_out/stamp.log; [ $rc -eq 0 ] || { tail -5 gpurun_out/stamp.log; exit $rc; }
done; done
