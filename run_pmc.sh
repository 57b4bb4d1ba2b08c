#!/bin/bash
# PMC counter passes (each its own rocprofv3 run; no tracing domains combined).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-pmc}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > "$GRAFT_REPO_ROOT/gpurun_out/counters_list.txt" 2>&1
echo "list rc=$?"
i=0
for set in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_$i" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_$i.log" 2>&1
  rc=$?
  echo "pass $i ($set) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_$i.log"; exit $rc; fi
done
