#!/bin/bash
# r03 session 17: bench line with the unlinked, graph-replayed pipelined leg
cd "$GRAFT_REPO_ROOT"
for i in 1 2; do
timeout -k 10 400 python3 bench.py --no-cpu-baseline > gpurun_out/bench_pipe$i.log 2>&1; rc=$?
echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_pipe$i.log; exit $rc; }
grep '^{' gpurun_out/bench_pipe$i.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
print('value', round(d['value']), 'pipelined', round(d['pipelined']['value']), d['pipelined']['outputs_identical'], 'tol', round(d['tolerance_mode']['value']), 'frac', round(d['roofline']['frac'],3))"
done
