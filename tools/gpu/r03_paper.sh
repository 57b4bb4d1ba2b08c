#!/bin/bash
# r03 session: paper-mode densify interior fast path -- paper parity, then the
# config-2p kernel trace and throughput.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests -k "paper" > gpurun_out/paper_tests.log 2>&1
rc=$?; tail -2 gpurun_out/paper_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu/cfg_trace.sh 2p | head -4
timeout -k 10 300 python3 tools/bench_configs.py --configs 2p,2 --steps 20 --warmup 5 > gpurun_out/cfg_2p.log 2>&1; grep '^{' gpurun_out/cfg_2p.log | cut -c1-160
