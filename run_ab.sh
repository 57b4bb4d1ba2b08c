#!/bin/bash
# A/B: run bench.py against alternative library builds (DISFLOW_LIB).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for spec in "$@"; do
  lib=${spec%%:*}; extra=""
  [ "$spec" != "$lib" ] && extra=${spec#*:}
  for rep in 1 2; do
    DISFLOW_LIB="$GRAFT_REPO_ROOT/$lib" timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline $extra > gpurun_out/ab.log 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "rc=$rc for $lib"; tail -5 gpurun_out/ab.log; exit $rc; fi
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); print('$spec', 'rep$rep', 'pairs/s %.0f'%d['value'], 'search avg ms %.4f'%d['roofline']['avg_launch_ms'], 'ms/step %.3f'%d['ms_per_step'])"
  done
done
