#!/bin/bash
cd "$GRAFT_REPO_ROOT"
L=optical-flow-using-dense-inverse-search_amd/disflow/libdis_hip.so
timeout -k 10 600 python3 tools/ab.py --spawn 2 --rounds 3 --steps 3 --batch 2 --preset slow --width 3840 --height 2160 $L $L:streams=1 $L:vr=0 $L:vr=0,streams=1 $L:vr=1 > gpurun_out/ab_c5.log 2>&1 || { tail gpurun_out/ab_c5.log; exit 1; }
cat gpurun_out/ab_c5.log | grep -v amdgpu.ids
