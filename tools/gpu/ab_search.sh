#!/bin/bash
# A/B of search-kernel builds: whole-step time (interleaved, one process) and
# per-level kernel durations (one stream) for each library given
cd "$GRAFT_REPO_ROOT"; R=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
D=optical-flow-using-dense-inverse-search_amd/disflow
timeout -k 10 400 python3 tools/ab.py "$@" --rounds 8 --steps 10 > gpurun_out/ab_search.log 2>&1; rc=$?
echo "ab rc=$rc"; cat gpurun_out/ab_search.log | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 bash tools/gpu/levels.sh "$@"
