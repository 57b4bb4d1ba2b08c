#!/bin/bash
# r03 session: v_sqrt_f32 error direction on the pyramid's domain, then the
# one-sided sqrt corrections A/B'd against the default (pyramid durations).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 60 tools/sqrt_dir || exit 1
D=optical-flow-using-dense-inverse-search_amd/disflow
SPAWN=3 bash tools/gpu/ab_pyr.sh $D/libdis_hip.so $D/libdis_hip_sq1.so $D/libdis_hip_sq2.so
