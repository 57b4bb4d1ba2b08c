#!/bin/bash
# Interleaved A/B of library builds, then each build's pyramid / output kernel
# durations (one stream): tools/gpu/ab_pyr.sh lib1 lib2 ...
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python3 tools/ab.py --spawn ${SPAWN:-3} --rounds 3 --steps 10 "$@" > gpurun_out/ab.log 2>&1 || { tail gpurun_out/ab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/ab.log
args=(); for v in "$@"; do args+=("$v:streams=1"); done
bash tools/gpu/levels.sh "${args[@]}" | grep -E "==|k_pyramid|k_output|3768320"
