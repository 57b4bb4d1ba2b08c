#!/bin/bash
# r03 session 8: k_pyr12 in XCD order -- parity, step A/B, one-stream
# durations and HBM bytes (FETCH_SIZE / WRITE_SIZE) with and without the remap
cd "$GRAFT_REPO_ROOT"; R=$GRAFT_REPO_ROOT
D=optical-flow-using-dense-inverse-search_amd/disflow
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/t_pyr.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 gpurun_out/t_pyr.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu/ab_search.sh $D/libdis_hip_noxcd.so $D/libdis_hip.so || exit $?
echo "=== one stream"
timeout -k 10 400 bash tools/gpu/levels.sh $D/libdis_hip_noxcd.so:streams=1 $D/libdis_hip.so:streams=1 || exit $?
cd /tmp && export TMPDIR=/tmp
k=0
for v in $D/libdis_hip_noxcd.so:streams=1 $D/libdis_hip.so:streams=1; do
  k=$((k+1))
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d $R/gpurun_out/pm${k}_$c -o run -- python3 $R/tools/ab.py $R/$v --rounds 1 > $R/gpurun_out/pm${k}_$c.log 2>&1 || { echo "pmc $k $c failed"; tail -5 $R/gpurun_out/pm${k}_$c.log; exit 1; }
  done
  echo "== pmc $v"
  (cd $R && python3 tools/pmc_traffic.py gpurun_out/pm${k}_FETCH_SIZE/run_counter_collection.csv gpurun_out/pm${k}_WRITE_SIZE/run_counter_collection.csv --out gpurun_out/pm$k.json | grep -i "pyr\|output")
done
