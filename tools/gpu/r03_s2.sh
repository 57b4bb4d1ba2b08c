#!/bin/bash
# r03 session 2: linked two-in-flight probe + search-kernel A/B
cd "$GRAFT_REPO_ROOT"
D=optical-flow-using-dense-inverse-search_amd/disflow
bash tools/gpu/pipe_trace2.sh || exit $?
bash tools/gpu/ab_search.sh $D/libdis_hip_ts0.so $D/libdis_hip.so $D/libdis_hip_sel.so
