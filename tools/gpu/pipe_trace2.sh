#!/bin/bash
# linked two-in-flight pattern: rates, a trace, and the linked-contexts GPU test
cd "$GRAFT_REPO_ROOT"; R=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "linked or ping_pong or two_threads or graph_replay" --timeout 200 --timeout-method thread > gpurun_out/t_link.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/t_link.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
run() { local name=$1; shift; timeout -k 10 300 "$@" > $R/gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -5 $R/gpurun_out/$name.log; exit $rc; }; }
run probe python3 $R/tools/pipe_probe.py
cat $R/gpurun_out/probe.log
run tr_link rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/tr_link -o run -- python3 $R/tools/pipe_trace.py --mode two --nsub 1 --link 1 --steps 16
cd $R
echo "== tr_link"; python3 tools/timeline.py gpurun_out/tr_link/run_kernel_trace.csv 8 60
