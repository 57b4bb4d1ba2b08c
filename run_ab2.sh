#!/bin/bash
cd "$GRAFT_REPO_ROOT"
L=optical-flow-using-dense-inverse-search_amd/disflow
timeout -k 10 400 python3 tools/ab.py --spawn 3 --rounds 4 $L/libdis_hip.so $L/libdis_hip_sm.so > gpurun_out/ab_c2.log 2>&1 || { tail gpurun_out/ab_c2.log; exit 1; }
cat gpurun_out/ab_c2.log | grep -v amdgpu.ids
timeout -k 10 400 python3 tools/ab.py --spawn 2 --rounds 3 --steps 3 --batch 2 --preset slow --width 3840 --height 2160 $L/libdis_hip.so $L/libdis_hip_sm.so > gpurun_out/ab_c5.log 2>&1 || { tail gpurun_out/ab_c5.log; exit 1; }
cat gpurun_out/ab_c5.log | grep -v amdgpu.ids
