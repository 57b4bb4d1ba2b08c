#!/bin/bash
# r03 session 18: bench on a dedicated stream vs the default stream (A/B, alternating)
cd "$GRAFT_REPO_ROOT"
for i in 1 2 3; do
for m in "" "--default-stream"; do
timeout -k 10 400 python3 bench.py --no-cpu-baseline --no-tolerance-mode $m > gpurun_out/bench_s$i.log 2>&1; rc=$?
[ $rc -eq 0 ] || { echo "bench rc=$rc"; tail -5 gpurun_out/bench_s$i.log; exit $rc; }
grep '^{' gpurun_out/bench_s$i.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
print('$m'.ljust(18), 'value', round(d['value']), 'pipelined', round(d['pipelined']['value']), 'frac', round(d['roofline']['frac'],3))"
done; done
