#!/bin/bash
# r03 session 3: in-kernel spread-block search tests + search / pyramid A/B
cd "$GRAFT_REPO_ROOT"
D=optical-flow-using-dense-inverse-search_amd/disflow
DISFLOW_LIB=$PWD/$D/libdis_hip_fbc.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q \
  -k "fallback or uncorrelated or large_shift or compat or lanes_per_patch" --timeout 200 --timeout-method thread \
  > gpurun_out/t_fbc.log 2>&1; rc=$?; echo "fbc tests rc=$rc"; tail -3 gpurun_out/t_fbc.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu/ab_search.sh $D/libdis_hip_ts0.so $D/libdis_hip_pyr1.so $D/libdis_hip.so $D/libdis_hip_sel.so $D/libdis_hip_fbc.so $D/libdis_hip_fbcsel.so
