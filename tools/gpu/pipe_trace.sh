#!/bin/bash
# kernel traces of the serving pattern (two engines, two streams) vs the headline loop
cd "$GRAFT_REPO_ROOT"; R=$GRAFT_REPO_ROOT; mkdir -p gpurun_out; cd /tmp && export TMPDIR=/tmp
run() { local name=$1; shift; timeout -k 10 300 "$@" > $R/gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -5 $R/gpurun_out/$name.log; exit $rc; }; }
run probe python3 $R/tools/pipe_probe.py
cat $R/gpurun_out/probe.log
run tr_two rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/tr_two -o run -- python3 $R/tools/pipe_trace.py --mode two --nsub 1
run tr_two2 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/tr_two2 -o run -- python3 $R/tools/pipe_trace.py --mode two --nsub 2
run tr_one rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/tr_one -o run -- python3 $R/tools/pipe_trace.py --mode one --nsub 2
cd $R
for t in tr_two tr_two2 tr_one; do echo "== $t"; python3 tools/timeline.py gpurun_out/$t/run_kernel_trace.csv 8 40; done
