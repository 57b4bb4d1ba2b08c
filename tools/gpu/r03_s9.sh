#!/bin/bash
# r03 session 9: maximum-size frames (2^28 pixels: square batch, tallest,
# widest) bit-exact vs the oracle, then the whole GPU suite with the
# row-parallel oracle
cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests/test_limits.py -m gpu -x -v -rf --timeout 600 --timeout-method thread > gpurun_out/t_limits.log 2>&1; rc=$?
echo "limits rc=$rc"; tail -8 gpurun_out/t_limits.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/t_all.log 2>&1; rc=$?
echo "all rc=$rc"; tail -4 gpurun_out/t_all.log; exit $rc
