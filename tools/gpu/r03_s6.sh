#!/bin/bash
# r03 session 6: strip pyramid (levels 1..6 in one kernel) parity + A/B
cd "$GRAFT_REPO_ROOT"
D=optical-flow-using-dense-inverse-search_amd/disflow
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/t_pyr.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -4 gpurun_out/t_pyr.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu/ab_search.sh $D/libdis_hip_pyr1.so $D/libdis_hip_p12.so $D/libdis_hip.so || exit $?
echo "=== one stream"
timeout -k 10 600 bash tools/gpu/levels.sh $D/libdis_hip_pyr1.so:streams=1 $D/libdis_hip.so:streams=1
