#!/bin/bash
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu -k "cli" --timeout 120 --timeout-method thread > gpurun_out/gt_cli.log 2>&1; rc=$?
tail -3 gpurun_out/gt_cli.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/bench_configs.py > gpurun_out/cfgs.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/cfgs.log; exit $rc
