#!/bin/bash
# LDS-conflict experiment: per-kernel durations (one stream) + SQ counters
# for each library given (tools/gpu/levels.sh + tools/gpu/pmc_sq.sh)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
args=(); for v in "$@"; do args+=("$v:streams=1"); done
bash tools/gpu/levels.sh "${args[@]}" | grep -E "==|k_search8<2, false" || exit 1
TOPK=1 bash tools/gpu/pmc_sq.sh "${args[@]}"
