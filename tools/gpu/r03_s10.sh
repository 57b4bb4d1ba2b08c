#!/bin/bash
# r03 session 10: k_pyr12 with RW level-2 rows per wave (halo rows read once
# per RW rows) -- parity of each variant, step A/B, one-stream durations, PMC bytes
cd "$GRAFT_REPO_ROOT"; R=$GRAFT_REPO_ROOT
D=optical-flow-using-dense-inverse-search_amd/disflow
for v in r2w3 r2w4 r4w3; do
  DISFLOW_LIB=$R/$D/libdis_hip_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -rf --timeout 200 --timeout-method thread > gpurun_out/t_$v.log 2>&1; rc=$?
  echo "tests $v rc=$rc"; tail -2 gpurun_out/t_$v.log; [ $rc -eq 0 ] || exit $rc
done
bash tools/gpu/ab_search.sh $D/libdis_hip.so $D/libdis_hip_r2w3.so $D/libdis_hip_r2w4.so $D/libdis_hip_r4w3.so || exit $?
echo "=== one stream"
timeout -k 10 500 bash tools/gpu/levels.sh $D/libdis_hip.so:streams=1 $D/libdis_hip_r2w3.so:streams=1 $D/libdis_hip_r2w4.so:streams=1 $D/libdis_hip_r4w3.so:streams=1 2>&1 | grep -v "k_search\|fill" || exit $?
cd /tmp && export TMPDIR=/tmp
k=0
for v in $D/libdis_hip.so:streams=1 $D/libdis_hip_r2w3.so:streams=1 $D/libdis_hip_r4w3.so:streams=1; do
  k=$((k+1))
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d $R/gpurun_out/pm${k}_$c -o run -- python3 $R/tools/ab.py $R/$v --rounds 1 > $R/gpurun_out/pm${k}_$c.log 2>&1 || { echo "pmc $k $c failed"; tail -5 $R/gpurun_out/pm${k}_$c.log; exit 1; }
  done
  echo "== pmc $v"
  (cd $R && python3 tools/pmc_traffic.py gpurun_out/pm${k}_FETCH_SIZE/run_counter_collection.csv gpurun_out/pm${k}_WRITE_SIZE/run_counter_collection.csv --out gpurun_out/pm$k.json | grep -i "pyr")
done
