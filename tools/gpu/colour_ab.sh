#!/bin/bash
# colour-coding throughput per library build (tools/bench_configs.py colour),
# interleaved twice: bash tools/gpu/colour_ab.sh libdis_hip.so libdis_hip_x.so ...
cd "$GRAFT_REPO_ROOT"; D=optical-flow-using-dense-inverse-search_amd/disflow
for r in 1 2; do
  for v in "$@"; do
    DISFLOW_LIB=$D/$v timeout -k 10 120 python3 tools/bench_configs.py --configs colour > gpurun_out/colour_ab.log 2>&1 || { tail -5 gpurun_out/colour_ab.log; exit 1; }
    echo "$v $(grep '^{' gpurun_out/colour_ab.log)"
  done
done
