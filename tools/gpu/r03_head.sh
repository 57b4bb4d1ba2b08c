#!/bin/bash
# r03 session: upper bound of collapsing the coarse head -- knock-out builds
# (wrong values) without the level >= 4 / >= 3 searches (u = 0 there) and
# without the k_search8_fb launches, A/B'd against the default in the
# two-sub-batch step (graphs on, as bench.py). Build the variants first (CPU):
#   tools/build_variants.sh head4:"-DDIS_EXP_SKIP_HEAD=4" head3:"-DDIS_EXP_SKIP_HEAD=3" nofb:"-DDIS_EXP_NO_FB=1"
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
D=optical-flow-using-dense-inverse-search_amd/disflow
timeout -k 10 900 python3 tools/ab.py --spawn 4 --rounds 3 --steps 10 $D/libdis_hip.so $D/libdis_hip_head4.so $D/libdis_hip_head3.so $D/libdis_hip_nofb.so > gpurun_out/ab_head.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/ab_head.log | tail -8; exit $rc
