#!/bin/bash
# r03 session: 17/15 and 15/17 sub-batch splits of 32 pairs against 16/16.
# Variants: tools/build_variants.sh sp1:"-DDIS_EXP_SPLIT0=1" spm1:"-DDIS_EXP_SPLIT0=-1"
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
D=optical-flow-using-dense-inverse-search_amd/disflow
timeout -k 10 600 python3 tools/ab.py --spawn 8 --rounds 3 --steps 10 $D/libdis_hip.so $D/libdis_hip_sp1.so $D/libdis_hip_spm1.so > gpurun_out/ab_split.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/ab_split.log | tail -4; exit $rc
