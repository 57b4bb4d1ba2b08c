#!/bin/bash
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
P=optical-flow-using-dense-inverse-search_amd/disflow
timeout -k 10 300 python tools/ab.py $P/libdis_hip.so --rounds 4 2>&1 | tail -1
for args in "--steps 10 --warmup 2" "--steps 10 --warmup 2 --no-kernel-timing" "--steps 40 --warmup 5"; do
  timeout -k 10 300 python bench.py $args --no-cpu-baseline > gpurun_out/cmp.log 2>&1 || { tail -3 gpurun_out/cmp.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/cmp.log').read().strip().splitlines()[-1]); print('$args', 'pairs/s %.0f'%d['value'], 'ms/step %.3f'%d['ms_per_step'])"
done
