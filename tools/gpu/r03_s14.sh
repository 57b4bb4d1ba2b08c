#!/bin/bash
# r03 session 14: k_pyr12 waves in chunked XCD order (halo rows shared in one
# L2 while the waves in flight keep the plain order's DRAM locality)
cd "$GRAFT_REPO_ROOT"; R=$GRAFT_REPO_ROOT
D=optical-flow-using-dense-inverse-search_amd/disflow
for v in c4 c8 c32; do
  DISFLOW_LIB=$R/$D/libdis_hip_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -rf --timeout 200 --timeout-method thread > gpurun_out/t_$v.log 2>&1; rc=$?
  echo "tests $v rc=$rc"; tail -1 gpurun_out/t_$v.log; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 500 python3 tools/ab.py $D/libdis_hip.so $D/libdis_hip_c4.so $D/libdis_hip_c8.so $D/libdis_hip_c32.so --rounds 8 --steps 10 > gpurun_out/ab_c.log 2>&1; echo "ab rc=$?"; grep median gpurun_out/ab_c.log
echo "=== one stream"
timeout -k 10 500 bash tools/gpu/levels.sh $D/libdis_hip.so:streams=1 $D/libdis_hip_c4.so:streams=1 $D/libdis_hip_c8.so:streams=1 $D/libdis_hip_c32.so:streams=1 2>&1 | grep -v "k_search\|fill" || exit $?
cd /tmp && export TMPDIR=/tmp
k=0
for v in $D/libdis_hip.so:streams=1 $D/libdis_hip_c8.so:streams=1 $D/libdis_hip_c32.so:streams=1; do
  k=$((k+1))
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d $R/gpurun_out/pm${k}_$c -o run -- python3 $R/tools/ab.py $R/$v --rounds 1 > $R/gpurun_out/pm${k}_$c.log 2>&1 || { echo "pmc $k $c failed"; tail -5 $R/gpurun_out/pm${k}_$c.log; exit 1; }
  done
  echo "== pmc $v"
  (cd $R && python3 tools/pmc_traffic.py gpurun_out/pm${k}_FETCH_SIZE/run_counter_collection.csv gpurun_out/pm${k}_WRITE_SIZE/run_counter_collection.csv --out gpurun_out/pm$k.json | grep -i "pyr")
done
