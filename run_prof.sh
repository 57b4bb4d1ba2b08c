#!/bin/bash
# rocprofv3 kernel trace + stats of a short bench run (no PMC counters here).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-r01}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 2 --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log" 2>&1
rc=$?
echo "rocprof rc=$rc"; tail -2 "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log"
find "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG" -name "*stats*" | head
for f in $(find "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG" -name "*kernel_stats.csv"); do cat "$f" | cut -c1-250; done
exit $rc
