#!/bin/bash
# HBM bytes per launch (PMC FETCH_SIZE / WRITE_SIZE passes) of the finest-level
# search and the other kernels, one stream, for each tools/ab.py variant given
cd "$GRAFT_REPO_ROOT"; R=$GRAFT_REPO_ROOT; mkdir -p gpurun_out; cd /tmp && export TMPDIR=/tmp
k=0
for v in "$@"; do
  k=$((k+1))
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $R/gpurun_out/fa${k}_$c -o run -- python3 $R/tools/ab.py $v:streams=1 --rounds 1 --steps 3 > $R/gpurun_out/fa${k}_$c.log 2>&1 || { tail -5 $R/gpurun_out/fa${k}_$c.log; exit 1; }
  done
  echo "== $v"
  (cd $R && python3 tools/pmc_traffic.py gpurun_out/fa${k}_FETCH_SIZE/run_counter_collection.csv gpurun_out/fa${k}_WRITE_SIZE/run_counter_collection.csv --out gpurun_out/fa${k}_traffic.json | grep -E "k_search8<2|pyr|output")
done
