#!/bin/bash
cd "$GRAFT_REPO_ROOT"; R=$GRAFT_REPO_ROOT
L=optical-flow-using-dense-inverse-search_amd/disflow
timeout -k 10 300 python3 -m pytest tests -x -q -m gpu -k "var_refine or slow_preset or refinement" > gpurun_out/gt.log 2>&1 || { tail -30 gpurun_out/gt.log; exit 1; }
tail -2 gpurun_out/gt.log
timeout -k 10 600 python3 tools/ab.py --spawn 2 --rounds 3 --steps 3 --batch 2 --preset slow --width 3840 --height 2160 $L/libdis_hip.so $L/libdis_hip_ng.so $L/libdis_hip.so:vr=0 > gpurun_out/ab_c5.log 2>&1 || { tail gpurun_out/ab_c5.log; exit 1; }
grep -v amdgpu.ids gpurun_out/ab_c5.log
timeout -k 10 500 python3 -m pytest tests -x -q -m gpu > gpurun_out/gt.log 2>&1 || { tail -30 gpurun_out/gt.log; exit 1; }
tail -2 gpurun_out/gt.log
