#!/bin/bash
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -k "paper" --timeout 120 --timeout-method thread > gpurun_out/gt_paper.log 2>&1; rc=$?
tail -30 gpurun_out/gt_paper.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gt.log 2>&1; rc=$?
tail -3 gpurun_out/gt.log; exit $rc
