#!/bin/bash
# r03 session 7: profile round (trace, FETCH/WRITE, SQ, bench line), then an
# A/B of the coarse-level lane-layout thresholds
cd "$GRAFT_REPO_ROOT"
D=optical-flow-using-dense-inverse-search_amd/disflow
bash tools/gpu/profile_round.sh || exit $?
cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python3 tools/ab.py $D/libdis_hip.so $D/libdis_hip_lpp4.so $D/libdis_hip_lpp8.so --rounds 8 --steps 10 > gpurun_out/ab_lpp.log 2>&1; echo "ab rc=$?"; grep median gpurun_out/ab_lpp.log
timeout -k 10 400 python3 tools/ab.py $D/libdis_hip.so:streams=1 $D/libdis_hip_lpp4.so:streams=1 $D/libdis_hip_lpp8.so:streams=1 --rounds 6 --steps 10 > gpurun_out/ab_lpp1.log 2>&1; echo "ab1 rc=$?"; grep median gpurun_out/ab_lpp1.log
