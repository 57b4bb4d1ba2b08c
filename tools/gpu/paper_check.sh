#!/bin/bash
# GPU suite, then per-kernel durations and throughput of paper mode (1080p MEDIUM)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gt.log 2>&1; rc=$?
tail -3 gpurun_out/gt.log; [ $rc -eq 0 ] || exit $rc
L=optical-flow-using-dense-inverse-search_amd/disflow
bash tools/gpu/levels.sh $L/libdis_hip.so:streams=1,paper=1 | head -12
timeout -k 10 300 python tools/bench_configs.py --configs 2,2p --steps 30 --warmup 10 > gpurun_out/c.log 2>&1 || { tail -3 gpurun_out/c.log; exit 1; }
grep -v amdgpu gpurun_out/c.log | python -c "import json,sys; [print((d:=json.loads(l))['config'], round(d['pairs_per_s'])) for l in sys.stdin]"
