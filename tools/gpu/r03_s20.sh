#!/bin/bash
# r03 session 20: bench's N > 1 path rehearsed (2 ranks, gloo, one card) with
# the dedicated-stream / two-context bench, then per-config throughput
cd "$GRAFT_REPO_ROOT"
bash tools/gpu/rehearse_multi.sh || exit $?
timeout -k 10 600 python -u tools/bench_configs.py --steps 30 --warmup 10 > gpurun_out/cfgs.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/cfgs.log > gpurun_out/r03_bench_configs.jsonl
python -c "import json,sys; [print((d:=json.loads(l))['config'], round(d.get('pairs_per_s', d.get('fields_per_s')))) for l in open('gpurun_out/r03_bench_configs.jsonl')]"; exit $rc
