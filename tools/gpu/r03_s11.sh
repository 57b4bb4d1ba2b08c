#!/bin/bash
# r03 session 11: LPP-2 split iteration (per-patch work shared by the two
# lanes) -- full GPU parity of the default build, parity of the unfenced
# variant, step A/B against the unsplit build, one-stream search durations
cd "$GRAFT_REPO_ROOT"; R=$GRAFT_REPO_ROOT
D=optical-flow-using-dense-inverse-search_amd/disflow
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/t_split.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 gpurun_out/t_split.log; [ $rc -eq 0 ] || exit $rc
DISFLOW_LIB=$R/$D/libdis_hip_nofence.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -rf --timeout 200 --timeout-method thread > gpurun_out/t_nofence.log 2>&1; rc=$?
echo "tests nofence rc=$rc"; tail -2 gpurun_out/t_nofence.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu/ab_search.sh $D/libdis_hip_nosplit.so $D/libdis_hip.so $D/libdis_hip_nofence.so || exit $?
echo "=== one stream"
timeout -k 10 400 bash tools/gpu/levels.sh $D/libdis_hip_nosplit.so:streams=1 $D/libdis_hip.so:streams=1 $D/libdis_hip_nofence.so:streams=1
