#!/bin/bash
# r03 session 22: sub-batch stream count A/B (graphs on)
cd "$GRAFT_REPO_ROOT"
D=optical-flow-using-dense-inverse-search_amd/disflow
timeout -k 10 500 python3 tools/ab.py $D/libdis_hip.so:streams=2 $D/libdis_hip.so:streams=3 $D/libdis_hip.so:streams=4 $D/libdis_hip.so:streams=1 --rounds 6 --steps 10 > gpurun_out/ab_s.log 2>&1; echo "ab rc=$?"; grep median gpurun_out/ab_s.log
