#!/bin/bash
# r03 session 21: k_pyr_tail with several level-2 tiles per wave
cd "$GRAFT_REPO_ROOT"; R=$GRAFT_REPO_ROOT
D=optical-flow-using-dense-inverse-search_amd/disflow
for v in "" _tpw1 _tpw2 _tpw5; do
  DISFLOW_LIB=$R/$D/libdis_hip$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -rf --timeout 200 --timeout-method thread > gpurun_out/t$v.log 2>&1; rc=$?
  echo "tests $v rc=$rc"; tail -1 gpurun_out/t$v.log; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 500 python3 tools/ab.py $D/libdis_hip_tpw1.so $D/libdis_hip_tpw2.so $D/libdis_hip.so $D/libdis_hip_tpw5.so --rounds 8 --steps 10 > gpurun_out/ab_t.log 2>&1; echo "ab rc=$?"; grep median gpurun_out/ab_t.log
echo "=== one stream"
timeout -k 10 500 bash tools/gpu/levels.sh $D/libdis_hip_tpw1.so:streams=1 $D/libdis_hip_tpw2.so:streams=1 $D/libdis_hip.so:streams=1 $D/libdis_hip_tpw5.so:streams=1 2>&1 | grep "==\|pyr"
