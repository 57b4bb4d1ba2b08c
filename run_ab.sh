#!/bin/bash
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 200 python tools/ctx_probe.py 4 > gpurun_out/c.log 2>&1 || { tail gpurun_out/c.log; exit 1; }
grep -v amdgpu gpurun_out/c.log
