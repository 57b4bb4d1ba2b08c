#!/bin/bash
# r03 session 16: serving patterns with graphs (two engines unlinked) vs the bench's one-engine call
cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python3 tools/pipe_probe2.py --rounds 4 > gpurun_out/probe2.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/probe2.log; exit $rc
