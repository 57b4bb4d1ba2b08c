#!/bin/bash
# pyramid / end-to-end parity tests, then per-kernel durations (one stream)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gt.log 2>&1; rc=$?
tail -3 gpurun_out/gt.log; [ $rc -eq 0 ] || exit $rc
L=optical-flow-using-dense-inverse-search_amd/disflow
bash tools/gpu/levels.sh $L/libdis_hip.so:streams=1 | grep -E "==|pyramid|output"
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/b.log 2>&1 || { tail -3 gpurun_out/b.log; exit 1; }
tail -1 gpurun_out/b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', round(d['value']), d['ms_per_step'])"
