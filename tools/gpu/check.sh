#!/bin/bash
# GPU suite + per-config throughput; every GPU step time-limited, stop on failure
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gt.log 2>&1; rc=$?
tail -3 gpurun_out/gt.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/bench_configs.py --steps 30 --warmup 10 > gpurun_out/cfgs.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/cfgs.log | python -c "import json,sys; [print((d:=json.loads(l))['config'], round(d.get('pairs_per_s', d.get('fields_per_s')))) for l in sys.stdin]"; exit $rc
