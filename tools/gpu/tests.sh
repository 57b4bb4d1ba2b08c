#!/bin/bash
# GPU test suite (optionally a subset: tools/gpu/tests.sh <pytest args>), one
# process, per-test timeout; stops at the first failure
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu "${@:-tests}" > gpurun_out/gt.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/gt.log | tail -80; exit $rc
