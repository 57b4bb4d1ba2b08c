#!/bin/bash
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/bench_a.log 2>&1 || exit $?
tail -1 gpurun_out/bench_a.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
timeout -k 10 400 python bench.py --no-cpu-baseline --streams 1 > gpurun_out/bench_b.log 2>&1 || exit $?
tail -1 gpurun_out/bench_b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
