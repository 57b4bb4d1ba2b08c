#!/bin/bash
# DIS_PRECISION_FMA: tolerance tests, then configs 2/3 exact vs FMA throughput
# with the finest search launch's roofline
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_tolerance.py > gpurun_out/tol.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|FMA mode|passed|failed|assert" gpurun_out/tol.log | tail -20; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/bench_configs.py --configs ${CFGS:-2,2f,3,3f} --steps 20 --warmup 5 > gpurun_out/cfgs.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/cfgs.log; exit $rc
