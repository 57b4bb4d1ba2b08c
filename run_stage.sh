#!/bin/bash
cd "$GRAFT_REPO_ROOT"; R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python3 -m pytest tests -x -q -m gpu > gpurun_out/gt.log 2>&1 || { tail -30 gpurun_out/gt.log; exit 1; }
tail -2 gpurun_out/gt.log
timeout -k 10 300 python3 tools/bench_configs.py --configs 1,2,3,5,colour > gpurun_out/cfg.log 2>&1 || { tail -5 gpurun_out/cfg.log; exit 1; }
cut -c1-220 gpurun_out/cfg.log
timeout -k 10 200 python3 bench.py > gpurun_out/bench.log 2>&1 || { tail -5 gpurun_out/bench.log; exit 1; }
cut -c1-300 gpurun_out/bench.log
./run_cfg_trace.sh 5
